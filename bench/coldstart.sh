#!/bin/bash
# Cold-start diagnosis on one box (VERDICT r5 ask 5): the driver's bench line, then the
# per-step curve after each kind of prewarm, then a kernel trace of a cold run split by
# step window.   bash bench/coldstart.sh OUT
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 200 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $OUT/bench.json
for pre in none copy gemm steps; do
  sleep 5
  timeout -k 10 200 python bench/step_trace.py --pre $pre --json $OUT/trace_$pre.json > $OUT/trace_$pre.txt 2>&1 \
    || { tail -5 $OUT/trace_$pre.txt; exit 1; }
  head -1 $OUT/trace_$pre.txt | cut -c1-400; tail -1 $OUT/trace_$pre.txt
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
sleep 5
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 bench/step_trace.py \
  --pre none --steps 250 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
python3 bench/coldstart_kernels.py $OUT/prof 250 $OUT/kernels_by_window.md
echo coldstart done
