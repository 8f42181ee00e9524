OUT=gpurun_out/${1:-xcd1}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { local name=$1; shift; local t=$1; shift; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread && \
step micro 200 python bench/micro_wgrad.py && \
step bench_lenet 200 python bench.py --steps 30 --warmup 5 && \
step bench_ref 200 python bench.py --model reference_cnn --batch 16384 --steps 10 --warmup 3 && \
step prof_lenet 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_lenet -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --graph 0 --phases 0 && \
step prof_ref 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_ref -o run --output-format csv -- python3 bench.py --model reference_cnn --batch 16384 --steps 5 --warmup 2 --graph 0 --phases 0
grep -h metric $OUT/bench_*.log | python3 -c "import sys,json; [print(json.loads(l)['config']['model'], json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
