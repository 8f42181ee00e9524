#!/bin/bash
# Same-box A/B of two kernel-extension builds, N interleaved rounds (A = in-tree .so,
# B = abso/base.so): whole-step ms of each run and the per-build medians.
# Usage: bash bench/gpu_so_ab_n.sh TAG N [bench args]
TAG=$1; N=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
SO=$(ls distributed_tensorflow_ibm_mnist_amd/_kernels*.so)
cp $SO abso/new.so
use() { cp abso/$1.so $SO; }
for r in $(seq 1 $N); do
  for t in A B; do
    if [ $t = A ]; then use new; else use base; fi
    timeout -k 10 200 python bench.py --steps 40 --warmup 5 --phases 0 "$@" > $OUT/$t$r.log 2>&1 || { use new; exit 1; }
  done
done
use new
python3 - "$OUT" "$N" <<'PY'
import json, statistics, sys
out, n = sys.argv[1], int(sys.argv[2])
v = {t: [json.loads([l for l in open(f"{out}/{t}{r}.log") if '"metric"' in l][0])["ms_per_step"] for r in range(1, n + 1)] for t in "AB"}
for t in "AB":
    print(t, " ".join(f"{x:.4f}" for x in v[t]), "median", f"{statistics.median(v[t]):.4f}")
PY
