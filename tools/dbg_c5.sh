set -o pipefail
out=gpurun_out/dbg1; mkdir -p $out
for v in vgpr agpr; do
  cp variants/lib_$v.so orb_slam3_vio_fixes_amd/liborb_mi355x.so
  for big in 1 0; do
    ORBM_BOWK_BIG=$big timeout -k 10 200 python -u -m pytest tests/test_gpu_c5.py -m gpu -q --timeout 100 --timeout-method thread -k "map_wide or adversarial" > $out/t_${v}_$big.log 2>&1; echo "$v big=$big rc=$? $(tail -1 $out/t_${v}_$big.log)"
  done
done
