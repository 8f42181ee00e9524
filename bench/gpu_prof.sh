#!/bin/bash
# Kernel-trace profile of one bench configuration (eager, 5 steps + 2 warmup):
#   bash bench/gpu_prof.sh TAG [ENV=VAL ...] -- <bench args>
# Writes gpurun_out/TAG/kernels.md (per-kernel us per step).  No GEMM clock prewarm
# (--prewarm_ms 0): its hipBLASLt launches would otherwise land in the per-step table.
TAG=$1; shift
ENVS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done
shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for e in "${ENVS[@]}"; do export "$e"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py "$@" --steps 5 --warmup 2 --prewarm_ms 0 --graph 0 --phases 0 --eager_steps 0 > $OUT/prof.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof.log; exit 1; }
python3 bench/prof_summary.py $OUT/prof 7 $OUT/kernels.md > /dev/null && head -14 $OUT/kernels.md
