#!/bin/bash
# Kernel-trace stats (and the first two PMC groups) of library variants on one
# box, matching not overlapped (bench.py --no-pipeline): per-kernel times that
# no other kernel shares.  usage: tools/prof_variants.sh OUTDIR "v1 v2 ..."
set -o pipefail
out=$1; vars=$2
mkdir -p "$out"
export TMPDIR=/tmp
cp orb_slam3_vio_fixes_amd/liborb_mi355x.so "$out/.default.so"
ARGS="--no-pipeline --steps 10 --warmup 2 --cpu-sample 0 --no-host-api"
for v in $vars; do
  cp "variants/lib_$v.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
  mkdir -p "$out/$v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$v/trace" -o run -- python3 bench.py $ARGS > "$out/$v/bench.json" 2> "$out/$v/rocprof.err" || { echo "$v trace failed"; tail -5 "$out/$v/rocprof.err"; cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so; exit 1; }
  python tools/kstats.py "$out/$v/trace/run_kernel_trace.csv" --csv "$out/$v/kernel_stats_by_grid.csv" > "$out/$v/kstats.txt"
  if [ -n "$NOPMC" ]; then echo "== $v"; head -4 "$out/$v/kstats.txt"; continue; fi
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/$v/pmc/p$i" -o run -- python3 bench.py $ARGS > "$out/$v/pmc_p$i.log" 2>&1 || { echo "$v pmc $i failed"; cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so; exit 1; }
  done
  python tools/pmc_summary.py "$out/$v/pmc" --csv "$out/$v/pmc_summary.csv" > "$out/$v/pmc_summary.txt"
  echo "== $v"; head -8 "$out/$v/kstats.txt"; grep -E "k_pyr_stream|k_fast_cells|k_sfi_resolve" "$out/$v/pmc_summary.txt" | cut -c1-400
done
cp "$out/.default.so" orb_slam3_vio_fixes_amd/liborb_mi355x.so
python tools/plan_info.py
