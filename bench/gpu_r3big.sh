#!/bin/bash
# split-K workgroup target of the 128x128-tile dense weight gradient (reference local3), same box, interleaved
set -o pipefail
O=gpurun_out/r3big; mkdir -p $O
for rep in 1 2; do
  for v in 400 256 600 800; do
    MNISTX_WGRAD_BLOCKS_BIG=$v timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 --steps 20 --warmup 5 --comm_probe 0 > $O/r_${v}_$rep.json 2> $O/r_${v}_$rep.err || exit 1
    echo "$v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $O/r_${v}_$rep.json)"
  done
done
