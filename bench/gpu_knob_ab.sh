#!/bin/bash
# Same-box A/B of env knobs on the kernel table: bash bench/gpu_knob_ab.sh TAG "ENV=a ENV2=b" "ENV=c" ... -- <bench args>
# Each variant: one rocprofv3 --kernel-trace --stats run (eager, 5 + 2 steps); prints the top kernels.
TAG=$1; shift
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
k=0
for v in "${VARS[@]}"; do
  OUT=gpurun_out/$TAG/v$k; mkdir -p $OUT
  env $v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --graph 0 --phases 0 --eager_steps 0 "$@" > $OUT/prof.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/prof.log; exit 1; }
  python3 bench/prof_summary.py $OUT/prof 7 $OUT/kernels.md > /dev/null
  echo "== [$v]"; head -9 $OUT/kernels.md | tail -7; grep "total GPU" $OUT/kernels.md
  k=$((k+1))
done
