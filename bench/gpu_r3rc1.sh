#!/bin/bash
# reference CNN conv1 banded forward: tests + env A/B + kernel table
set -o pipefail
O=gpurun_out/r3rc1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_cli_gpu.py tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/gpu_env_ab.sh 2 "MNISTX_REFC1_BAND=1" "MNISTX_REFC1_BAND=0" -- --model reference_cnn --batch 16384 --steps 20 --warmup 5 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
bash bench/gpu_prof.sh r3rc1/prof -- --model reference_cnn --batch 16384 --comm_probe 0 > /dev/null && grep -E "refc1|convpool_fwd|total" $O/prof/kernels.md
