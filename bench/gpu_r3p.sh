#!/bin/bash
# band forward wave priority after the in-lane rework: MNISTX_BAND_PRIO 1 (conv1 waves) / 0 / 2 (conv2 waves)
set -o pipefail
O=gpurun_out/r3p; mkdir -p $O
bash bench/gpu_env_ab.sh 3 "MNISTX_BAND_PRIO=1" "MNISTX_BAND_PRIO=0" "MNISTX_BAND_PRIO=2" -- --steps 30 --warmup 5 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 200 python bench/micro_band.py > $O/micro_band.txt 2>&1; cat $O/micro_band.txt
