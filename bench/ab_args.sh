#!/bin/bash
# Same-box A/B of two bench argument sets on THIS tree, interleaved N rounds:
#   ARGS_A="..." ARGS_B="..." [ENV_A="K=V ..."] [ENV_B="K=V ..."] bash bench/ab_args.sh OUT [N]
set -o pipefail
OUT=gpurun_out/$1; N=${2:-3}
mkdir -p $OUT
for i in $(seq 1 $N); do
  for side in A B; do
    var="ARGS_$side"; evar="ENV_$side"
    timeout -k 10 300 env ${!evar} python bench.py ${!var} > $OUT/${side}_$i.json 2> $OUT/${side}_$i.err || { tail -5 $OUT/${side}_$i.err; exit 1; }
    echo "$side $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/${side}_$i.json) $(grep -o '"phase_ms_eager": {[^}]*}' $OUT/${side}_$i.json)"
  done
done
