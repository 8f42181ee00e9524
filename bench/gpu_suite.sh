#!/bin/bash
# One gpurun call: GPU tests, smoke, CLI end-to-end (HIP), PS mode on one GPU
# (gloo-staged transport), benches.  Every GPU step has its own time limit and
# the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/suite
mkdir -p $OUT
step() { local name=$1; shift; local t=$1; shift; echo "== $name" ; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc" >> $OUT/$name.log; echo "$name rc=$rc"; return $rc; }
step tests 600 python -m pytest tests -x -q -m gpu && \
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" && \
step cli_ref 300 python main.py --model=reference_cnn --in_channels=3 --max_steps=300 --test_interval=100 --batch_size=128 --train_dir=/tmp/gs/ref --train_data=synthetic://20000 --test_data=synthetic://2000?seed=1 --base_lr=0.05 --optimizer=momentum --log_device_placement && \
step cli_lenet_resume 300 python main.py --model=lenet5 --in_channels=1 --max_steps=400 --test_interval=200 --batch_size=256 --train_dir=/tmp/gs/ref --train_dir=/tmp/gs/lenet --train_data=synthetic://20000 --test_data=synthetic://2000?seed=1 --base_lr=0.05 --optimizer=momentum && \
step cli_lenet_resume2 300 python main.py --model=lenet5 --in_channels=1 --max_steps=600 --test_interval=200 --batch_size=256 --train_dir=/tmp/gs/lenet --train_data=synthetic://20000 --test_data=synthetic://2000?seed=1 --base_lr=0.05 --optimizer=momentum && \
step infer 300 python inference.py --model=/tmp/gs/lenet --validate --val_data=synthetic://3000?seed=2 --output_dir=/tmp/gs/inf --output_file=val.json --impl=hip && \
step bench_lenet 300 python bench.py --steps 20 --warmup 5 && \
step bench_ref 300 python bench.py --model reference_cnn --batch 8192 --steps 10 --warmup 3 && \
step bench_ref_torch 300 python bench.py --model reference_cnn --batch 8192 --steps 10 --warmup 3 --impl torch
CHAIN=$?
PSC="--model=lenet5 --in_channels=1 --max_steps=200 --test_interval=100 --batch_size=256 --train_dir=/tmp/gs/ps --train_data=synthetic://20000 --test_data=synthetic://2000?seed=1 --ps_hosts=localhost:29700 --worker_hosts=localhost:29701,localhost:29702 --ps_backend=gloo --log_step_count_steps=50"
if [ $CHAIN -eq 0 ]; then
  echo "== ps_mode"
  (timeout -k 10 240 python main.py $PSC --job_name=ps --task_id=0 > $OUT/ps0.log 2>&1; echo "rc=$?" >> $OUT/ps0.log) &
  (timeout -k 10 240 python main.py $PSC --job_name=worker --task_id=1 > $OUT/w1.log 2>&1; echo "rc=$?" >> $OUT/w1.log) &
  timeout -k 10 240 python main.py $PSC --job_name=worker --task_id=0 > $OUT/w0.log 2>&1; echo "rc=$?" >> $OUT/w0.log
  wait
  tail -n 2 $OUT/ps0.log $OUT/w0.log $OUT/w1.log
fi
