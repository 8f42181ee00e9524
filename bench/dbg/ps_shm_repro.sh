#!/bin/bash
# 1 PS + 2 HIP workers on the shm data plane with the logs under gpurun_out (a hang shows
# where each process stopped).   bash bench/dbg/ps_shm_repro.sh OUT [backend] [model] [cin] [batch]
OUT=gpurun_out/$1; BK=${2:-shm}; MODEL=${3:-lenet5}; CIN=${4:-1}; BS=${5:-256}
mkdir -p $OUT; rm -rf /tmp/shm_repro_train
P=$((29000 + RANDOM % 1000))
common="--model=$MODEL --in_channels=$CIN --batch_size=$BS --max_steps=60 --test_interval=30 --log_step_count_steps=0
 --train_data=synthetic://8000 --test_data=synthetic://512?seed=1 --eval_examples=512 --train_dir=/tmp/shm_repro_train
 --ps_hosts=localhost:$P --worker_hosts=localhost:$((P+100)),localhost:$((P+101)) --ps_backend=$BK --optimizer=momentum --base_lr=0.02"
export PYTHONUNBUFFERED=1 OMP_NUM_THREADS=2
python main.py $common --job_name=ps --task_id=0 > $OUT/ps0.log 2>&1 & p0=$!
python main.py $common --job_name=worker --task_id=0 > $OUT/w0.log 2>&1 & p1=$!
python main.py $common --job_name=worker --task_id=1 > $OUT/w1.log 2>&1 & p2=$!
for i in $(seq 1 100); do
  sleep 1
  if ! kill -0 $p0 2>/dev/null && ! kill -0 $p1 2>/dev/null && ! kill -0 $p2 2>/dev/null; then break; fi
done
rc=0
for p in $p0 $p1 $p2; do if kill -0 $p 2>/dev/null; then echo "pid $p still running: killing"; kill -9 $p; rc=1; fi; done
wait
for f in ps0 w0 w1; do echo "== $f"; tail -6 $OUT/$f.log; done
exit $rc
