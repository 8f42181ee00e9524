#!/bin/bash
# split-K workgroup target of the grouped head weight gradients (MNISTX_WGRAD_BLOCKS), same box, interleaved
set -o pipefail
O=gpurun_out/r3wgb; mkdir -p $O
for rep in 1 2 3; do
  for v in 512 256 128 384; do
    MNISTX_WGRAD_BLOCKS=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --phases 0 --comm_probe 0 > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || exit 1
    echo "$v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $O/b_${v}_$rep.json)"
  done
done
