#!/bin/bash
# Builds a variant of the HIP library with extra compile definitions into
# variants/lib_<name>.so for same-box A/B runs (tools/ab_variants.sh).
# usage: tools/build_variant.sh <name> [-DKNOB=value ...]
set -e
name=$1; shift
cd "$(dirname "$0")/.."
mkdir -p variants
S=orb_slam3_vio_fixes_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-result "$@" \
    $S/extractor.hip $S/matcher.hip $S/stereo.hip $S/kfdb.hip $S/vocab.cpp -o variants/lib_$name.so
echo variants/lib_$name.so
