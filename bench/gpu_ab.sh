#!/bin/bash
# Same-box A/B: bench (twice each, interleaved) + one kernel trace per arm.
# Usage: bash bench/gpu_ab.sh TAG "ENV=val|-" "extra bench args for B|-" [common bench args...]
TAG=$1; shift; ENVB=$1; shift; ARGB=$1; shift
[ "$ENVB" = "-" ] && ENVB="MNISTX_AB_NOOP=1"
[ "$ARGB" = "-" ] && ARGB=""
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { local name=$1; shift; local t=$1; shift; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step benchA1 300 python bench.py --steps 30 --warmup 5 --phases 0 "$@" && \
step benchB1 300 env $ENVB python bench.py --steps 30 --warmup 5 --phases 0 $ARGB "$@" && \
step benchA2 300 python bench.py --steps 30 --warmup 5 --phases 0 "$@" && \
step benchB2 300 env $ENVB python bench.py --steps 30 --warmup 5 --phases 0 $ARGB "$@" && \
step profA 300 rocprofv3 --kernel-trace --stats -d $OUT/profA -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --graph 0 --phases 0 "$@" && \
export $ENVB && \
step profB 300 rocprofv3 --kernel-trace --stats -d $OUT/profB -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --graph 0 --phases 0 $ARGB "$@"
for f in benchA1 benchB1 benchA2 benchB2; do echo "$f $(grep -h metric $OUT/$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"; done
