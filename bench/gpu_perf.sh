#!/bin/bash
# GPU tests + benches + kernel-trace profiles (one gpurun call).  Usage: bash bench/gpu_perf.sh TAG
TAG=${1:-perf}
OUT=gpurun_out/$TAG
mkdir -p $OUT
step() { local name=$1; shift; local t=$1; shift; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 600 python -m pytest tests -x -q -m gpu && \
step bench_lenet 300 python bench.py --steps 20 --warmup 5 && \
step bench_ref 300 python bench.py --model reference_cnn --batch 16384 --steps 10 --warmup 3 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
step prof_lenet 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_lenet -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --graph 0 && \
step prof_ref 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_ref -o run --output-format csv -- python3 bench.py --model reference_cnn --batch 16384 --steps 5 --warmup 2 --graph 0
grep -h metric $OUT/bench_*.log | python3 -c "import sys,json; [print(json.loads(l)['config']['model'], json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
