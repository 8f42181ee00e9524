#!/bin/bash
# Same-box A/B of the default bench: this tree vs the tree at $AB_OLD (a git worktree of an
# earlier commit with its own in-tree build), interleaved N rounds.
#   bash bench/ab_bench.sh OUT [N] [bench args...]
set -o pipefail
OUT=gpurun_out/$1; N=${2:-3}; shift 2
mkdir -p $OUT
OLD=${AB_OLD:-ab_old}
for i in $(seq 1 $N); do
  for side in new old; do
    if [ $side = new ]; then dir=.; else dir=$OLD; fi
    (cd $dir && timeout -k 10 300 python bench.py "$@") > $OUT/${side}_$i.json 2> $OUT/${side}_$i.err || { tail -5 $OUT/${side}_$i.err; exit 1; }
    echo "$side $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/${side}_$i.json) $(grep -o '"phase_ms_eager": {[^}]*}' $OUT/${side}_$i.json)"
  done
done
