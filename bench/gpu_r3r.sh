#!/bin/bash
# r3r: band forward XFill on conv2 waves: tests (DIRECT=1) + kernel/bench A/B
set -o pipefail
O=gpurun_out/r3r; mkdir -p $O
MNISTX_BAND_XF2=1 timeout -k 10 200 python -u -m pytest tests/test_lenet_band_gpu.py -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
for v in 0 1 0 1; do
  MNISTX_BAND_XF2=$v timeout -k 10 120 python bench/micro_band.py one 1 65536 > $O/micro_$v.log 2>&1 || exit 1
  echo "xf2=$v $(tail -1 $O/micro_$v.log)"
done
for v in 0 1 0 1; do
  MNISTX_BAND_XF2=$v timeout -k 10 120 python bench.py --steps 30 --warmup 5 --comm_probe 0 > $O/bench_$v.log 2>&1 || exit 1
  echo "xf2=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log)"
done
