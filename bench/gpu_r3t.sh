#!/bin/bash
# r3t: reference CNN, halo kernels MFMA-phase s_setprio A/B
set -o pipefail
O=gpurun_out/r3t; mkdir -p $O
run() { local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 --steps 20 --warmup 5 --comm_probe 0 > $O/bench_$tag.log 2>&1 || exit 1
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.log) $(grep -o '"forward": [0-9.]*' $O/bench_$tag.log) $(grep -o '"backward": [0-9.]*' $O/bench_$tag.log)"; }
for rep in 1 2; do run base MNISTX_NOOP=1; run halo MNISTX_HALO_PRIO=1; done
