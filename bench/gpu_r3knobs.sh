#!/bin/bash
# driver-default LeNet bench: prewarm length and the head threads-per-window knob, same box, interleaved
set -o pipefail
O=gpurun_out/r3knobs; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 "$@" > $O/$tag.json 2> $O/$tag.err || exit 1; echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.json)"; }
for rep in 1 2; do
  run pw300_$rep python bench.py
  run pw1000_$rep python bench.py --prewarm_ms 1000
  run tpw2_$rep env MNISTX_HEAD_TPW=2 python bench.py
done
