#!/bin/bash
# Interleaved whole-step A/B of env settings: bash bench/gpu_env_ab.sh ROUNDS "ENV=a" "ENV=b" ... -- <bench args>
R=$1; shift
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
shift
for r in $(seq 1 $R); do
  for v in "${VARS[@]}"; do
    out=$(env $v timeout -k 10 120 python bench.py --phases 0 --eager_steps 0 "$@" 2>/dev/null | tail -1) || { echo "failed: $v"; exit 1; }
    echo "[$v] $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("ms/step %.4f" % d["ms_per_step"])')"
  done
done
