#!/bin/bash
# Kernel-trace profile of one bench configuration (eager, 20 steps after 5 warmup steps and
# the default 300 ms clock prewarm, whose GEMMs fall before the first step boundary):
#   bash bench/gpu_prof.sh TAG [ENV=VAL ...] -- <bench args>
# Writes gpurun_out/TAG/kernels.md (per-kernel us per step over the 20 timed steps, and the
# traced wall span per step to reconcile the kernel sum with) and TAG/bench.json (the traced
# run's own bench line: ms_per_step under the tracer).
TAG=$1; shift
ENVS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done
shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for e in "${ENVS[@]}"; do export "$e"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py "$@" --steps 20 --warmup 5 --graph 0 --phases 0 --eager_steps 0 --comm_probe 0 > $OUT/prof.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof.log; exit 1; }
grep '^{' $OUT/prof.log | tail -1 > $OUT/bench.json
python3 bench/prof_summary.py $OUT/prof 25 $OUT/kernels.md 5 > /dev/null && head -14 $OUT/kernels.md && tail -2 $OUT/kernels.md
