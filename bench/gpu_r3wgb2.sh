#!/bin/bash
# MNISTX_WGRAD_BLOCKS default 256: GPU tests + LeNet / reference-CNN benches, and the old 512 for the reference CNN
set -o pipefail
O=gpurun_out/r3wgb2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py > $O/lenet_$i.json 2> $O/lenet_$i.err || exit 1; echo "lenet $(grep -o '"ms_per_step": [0-9.]*' $O/lenet_$i.json)"; done
for v in 256 512 256 512; do MNISTX_WGRAD_BLOCKS=$v timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 --steps 20 --warmup 5 --comm_probe 0 > $O/ref_$v.json 2> $O/ref_$v.err || exit 1; echo "ref $v $(grep -o '"ms_per_step": [0-9.]*' $O/ref_$v.json)"; done
