#!/bin/bash
# finalize_k prefetch/overlap: tests + kernel table; split-K target A/B (MNISTX_WGRAD_BLOCKS 512 vs 256)
set -o pipefail
O=gpurun_out/r3y; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_executor_gpu.py tests/test_mlp_head_gpu.py tests/test_kernels_gpu.py tests/test_cli_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/gpu_env_ab.sh 3 "MNISTX_WGRAD_BLOCKS=512" "MNISTX_WGRAD_BLOCKS=256" -- --steps 30 --warmup 5 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
bash bench/gpu_prof.sh r3y/prof -- --comm_probe 0 > /dev/null && cat $O/prof/kernels.md
bash bench/gpu_prof.sh r3y/prof256 MNISTX_WGRAD_BLOCKS=256 -- --comm_probe 0 > /dev/null && grep -E "splitk|gemm_wg|total" $O/prof256/kernels.md
