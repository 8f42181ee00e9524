#!/bin/bash
# r3n: conv2+LRN+pool fused forward (reference CNN): tests, bench A/B, kernel table
set -o pipefail
O=gpurun_out/r3n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lrnpool or lrn_pool or halo or lrn" tests/test_executor_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
for v in 1 0 1 0; do for nw in 16 8; do [ $v = 0 ] && [ $nw = 8 ] && continue;
  MNISTX_LRNPOOL_NW=$nw MNISTX_FOLD_LRNPOOL=$v timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 --steps 20 --warmup 5 --comm_probe 0 > $O/bench_${v}_$nw.log 2>&1 || exit 1
  echo "fold=$v nw=$nw $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$nw.log)"; done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --model reference_cnn --batch 16384 --steps 5 --warmup 2 --prewarm_ms 0 --graph 0 --phases 0 --comm_probe 0 > $O/prof.log 2>&1 && python3 bench/prof_summary.py $O/prof 7 $O/kernels.md > /dev/null && head -16 $O/kernels.md
