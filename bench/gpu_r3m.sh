#!/bin/bash
# r3m: fp32 halo conv2 tests + fp32 reference-CNN bench (halo on / off)
set -o pipefail
O=gpurun_out/r3m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_f32_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit 1
for v in 1 0; do
  MNISTX_F32_HALO=$v timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 --precision fp32 --steps 5 --warmup 2 --comm_probe 0 > $O/bench_$v.log 2>&1 || exit 1
  echo "halo=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --model reference_cnn --batch 16384 --precision fp32 --steps 3 --warmup 1 --prewarm_ms 0 --graph 0 --phases 0 --comm_probe 0 > $O/prof.log 2>&1 && python3 bench/prof_summary.py $O/prof 4 $O/kernels.md > /dev/null && head -14 $O/kernels.md
