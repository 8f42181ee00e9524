#!/bin/bash
# Rehearse the multi-rank bench/main paths on ONE GPU (ranks share the card).
#  1. bench.py, 2 ranks, gloo (host-staged all-reduce of the same gradient buckets)
#  2. main.py DP training (2 ranks, gloo) on LeNet-5 with checkpoints
# RCCL itself cannot be rehearsed here: it refuses two ranks on one device
# ("Duplicate GPU detected", profiles/r1s3/dp_rehearsal/bench_rccl2_refused.log).
# Usage: bash bench/gpu_dp_rehearsal.sh TAG
TAG=${1:-dp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1
step() { local name=$1; shift; local t=$1; shift; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step bench_gloo2 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --dist_backend gloo && \
step main_dp2 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29612 main.py --model=lenet5 --in_channels=1 --config=configs/lenet5_synth.yaml \
    --train_dir=$OUT/train_dp2 --max_steps=40 --dp_backend=gloo
grep -h metric $OUT/bench_*.log
