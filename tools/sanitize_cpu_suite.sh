#!/bin/bash
# The CPU test suite with the checker built under ASan + UBSan:
# the oracle is rebuilt with -fsanitize=address,undefined into oracle/_san/,
# preloaded runtimes, leak checking off (CPython's arenas), and every
# `pytest -m "not gpu"` test that calls it runs against that build; then the
# native sanitizer drivers (tests/native: ASan/UBSan and TSan builds of the
# oracle, vocab.cpp and the batch gather).  Any sanitizer report fails.
# usage: tools/sanitize_cpu_suite.sh [pytest args...]
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p oracle/_san
g++ -O1 -g -std=c++17 -fPIC -shared -ffp-contract=off -fno-omit-frame-pointer -fsanitize=address,undefined \
    -fno-sanitize-recover=all -Iinclude oracle/orb_oracle.cpp -o oracle/_san/liborb_oracle.so -lpthread
export ORB_ORACLE_LIB=$PWD/oracle/_san/liborb_oracle.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
LD_PRELOAD="$(g++ -print-file-name=libasan.so) $(g++ -print-file-name=libubsan.so)" \
    python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
make -s -C tests/native san
python -m pytest tests/test_sanitizers.py -q -p no:cacheprovider
