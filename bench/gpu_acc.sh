#!/bin/bash
# steps-to-99%-train-accuracy on one GPU: HIP kernels vs the PyTorch-ROCm baseline.  Usage: bash bench/gpu_acc.sh TAG
TAG=${1:-acc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python bench/steps_to_acc.py --impl hip > $OUT/hip_b128.log 2>&1 && \
timeout -k 10 600 python bench/steps_to_acc.py --impl torch > $OUT/torch_b128.log 2>&1 && \
timeout -k 10 600 python bench/steps_to_acc.py --impl hip --batch 1024 --lr 0.05 > $OUT/hip_b1024.log 2>&1
RC=$?
tail -n1 $OUT/*.log
exit $RC
