#!/bin/bash
# LeNet backward knobs re-checked at HEAD (same box, interleaved): conv1 wgrad images per group, dgrad variant
set -o pipefail
O=gpurun_out/r3knobs2; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 "$@" > $O/$tag.json 2> $O/$tag.err || exit 1; echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.json)"; }
for rep in 1 2; do
  run base_$rep python bench.py --steps 30 --comm_probe 0
  run c1wimgs2_$rep env MNISTX_C1_WG_IMGS=2 python bench.py --steps 30 --comm_probe 0
  run dgvar2_$rep env MNISTX_DGRAD_VAR=2 python bench.py --steps 30 --comm_probe 0
done
