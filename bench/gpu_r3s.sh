#!/bin/bash
# r3s: MFMA-phase s_setprio A/B in the LeNet backward kernels (dgrad / wgrads)
set -o pipefail
O=gpurun_out/r3s; mkdir -p $O
run() { local tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 30 --warmup 5 --comm_probe 0 > $O/bench_$tag.log 2>&1 || exit 1
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$tag.log) $(grep -o '"backward": [0-9.]*' $O/bench_$tag.log)"; }
for rep in 1 2; do
  run base MNISTX_NOOP=1; run dg MNISTX_DGRAD_PRIO=1; run wg MNISTX_WGRAD_PRIO=1; run both MNISTX_DGRAD_PRIO=1 MNISTX_WGRAD_PRIO=1
done
