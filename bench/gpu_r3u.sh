#!/bin/bash
# r3 session 2: in-lane conv1 pooling in the band forward -- band tests, same-box A/B, kernel table
set -o pipefail
O=gpurun_out/r3u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lenet_band_gpu.py tests/test_executor_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/gpu_env_ab.sh 3 "MNISTX_BAND_INLANE=1" "MNISTX_BAND_INLANE=0" -- --steps 20 --warmup 5 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
bash bench/gpu_prof.sh r3u/prof -- --comm_probe 0 > /dev/null && head -8 $O/prof/kernels.md
