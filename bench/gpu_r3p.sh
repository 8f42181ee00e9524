#!/bin/bash
# r3p: band forward wave-priority A/B (kernel alone + full bench)
set -o pipefail
O=gpurun_out/r3p; mkdir -p $O
for v in 0 1 2 0 1 2; do
  MNISTX_BAND_PRIO=$v timeout -k 10 120 python bench/micro_band.py one 1 65536 > $O/micro_$v.log 2>&1 || exit 1
  echo "prio=$v $(tail -1 $O/micro_$v.log)"
done
for v in 0 1 0 1; do
  MNISTX_BAND_PRIO=$v timeout -k 10 120 python bench.py --steps 30 --warmup 5 --comm_probe 0 > $O/bench_$v.log 2>&1 || exit 1
  echo "prio=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log)"
done
