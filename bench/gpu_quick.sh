#!/bin/bash
# Targeted GPU check: selected tests (-k expr), then a bench + kernel trace of one model.
# Usage: bash bench/gpu_quick.sh TAG "pytest -k expr" [bench args...]
TAG=$1; shift; KEXPR=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { local name=$1; shift; local t=$1; shift; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 300 python -u -m pytest tests -x -q -m gpu -k "$KEXPR" --timeout 120 --timeout-method thread && \
step bench 300 python bench.py --steps 20 --warmup 5 "$@" && \
step prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --graph 0 --phases 0 "$@"
tail -1 $OUT/tests.log; grep -h metric $OUT/bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['config']['model'], d['value'], d['ms_per_step'])"
