#!/bin/bash
# grouped head weight gradients: 64x128 vs 64x64 tiles (env A/B, same build) + tests
set -o pipefail
O=gpurun_out/r3x; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_executor_gpu.py tests/test_mlp_head_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/gpu_env_ab.sh 3 "MNISTX_WG_GROUP_BN=128" "MNISTX_WG_GROUP_BN=64" -- --steps 30 --warmup 5 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
bash bench/gpu_prof.sh r3x/prof128 -- --comm_probe 0 > /dev/null && grep -E "gemm_wg|total" $O/prof128/kernels.md
bash bench/gpu_prof.sh r3x/prof64 MNISTX_WG_GROUP_BN=64 -- --comm_probe 0 > /dev/null && grep -E "gemm_wg|total" $O/prof64/kernels.md
