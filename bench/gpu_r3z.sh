#!/bin/bash
# pooled-K conv1 weight gradient: tests, env A/B against the unpool kernel, kernel table
set -o pipefail
O=gpurun_out/r3z; mkdir -p $O
timeout -k 10 200 python bench/dbg/c1w_dbg.py 2>&1 | grep "==" ; timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "convpool or lenet_conv1" > $O/k1.log 2>&1; rc=$?
tail -3 $O/k1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_executor_gpu.py tests/test_lenet_band_gpu.py tests/test_kernels_gpu.py tests/test_dp_hip_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/gpu_env_ab.sh 3 "MNISTX_C1W_POOLK=1" "MNISTX_C1W_POOLK=0" -- --steps 30 --warmup 5 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
bash bench/gpu_prof.sh r3z/prof -- --comm_probe 0 > /dev/null && head -8 $O/prof/kernels.md
