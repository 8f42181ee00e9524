#!/bin/bash
# r3o: PS bench 1 PS + 1 worker (no GPU sharing between workers) and 1 PS + 3 workers, B=128
set -o pipefail
O=gpurun_out/r3o; mkdir -p $O
for n in 2 4 2 4; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --mode ps --batch 128 --steps 300 --warmup 30 > $O/ps_n$n.log 2>&1 || exit 1
  python bench/ps_summary.py "n=$n" $O/ps_n$n.log
done
