#!/bin/bash
# Same-box A/B: this tree vs $AB_OLD (default ab_old: a git worktree of an earlier commit
# with its own in-tree build), N interleaved rounds of a python command run in each tree.
#   bash bench/ab_micro.sh OUT N <python args...>
set -o pipefail
OUT=gpurun_out/$1; N=$2; shift 2
mkdir -p $OUT
OLD=${AB_OLD:-ab_old}
for i in $(seq 1 $N); do
  for side in new old; do
    if [ $side = new ]; then dir=.; else dir=$OLD; fi
    (cd $dir && timeout -k 10 300 python "$@") > $OUT/${side}_$i.txt 2> $OUT/${side}_$i.err || { tail -5 $OUT/${side}_$i.err; exit 1; }
    echo "$side $i $(grep -o '"us": [0-9.]*\|"ms_per_step": [0-9.]*' $OUT/${side}_$i.txt | tr '\n' ' ')"
  done
done
