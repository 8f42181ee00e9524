#!/bin/bash
# Same-box A/B of the LeNet-5 input paths (bench.py --input prep|bf16|u8), interleaved.
# Usage: bash bench/gpu_input_ab.sh TAG [rounds] [extra bench args...]
TAG=${1:-input_ab}; R=${2:-2}; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for m in prep bf16 u8; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --phases 0 --input $m "$@" > $OUT/$m.$r.log 2>&1 || { echo "$m rc=$?"; exit 1; }
    echo "$m.$r $(grep -o '"ms_per_step": [0-9.]*' $OUT/$m.$r.log)"
  done
done
