#!/bin/bash
# PS mode, 1 PS + (N-1) workers on this box's GPU(s): the shm data plane (CPU PS) against
# ipc (GPU PS), interleaved.   bash bench/ps_ab.sh OUT [N] [ROUNDS] [extra bench args]
set -o pipefail
OUT=gpurun_out/$1; N=${2:-4}; R=${3:-2}; shift 3
mkdir -p $OUT
port=29617
for i in $(seq 1 $R); do
  for t in shm ipc; do
    port=$((port + 1))
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $port bench.py --mode ps --batch 128 --steps 300 --warmup 30 --ps_transport $t "$@" \
      > $OUT/${t}_$i.json 2> $OUT/${t}_$i.err || { tail -20 $OUT/${t}_$i.err; exit 1; }
    python3 - $OUT/${t}_$i.json $t $i <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], sys.argv[3], "ms/update", d["ms_per_update"], "ps_us_per_msg", d["ps_us_per_msg"],
      "workers", [(c["push_us"], c["reply_wait_us"], c["pull_us"], c["compute_us"]) for c in d["ps_comm"]])
PY
  done
done
