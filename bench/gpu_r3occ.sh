#!/bin/bash
# reference conv1 wgrad (LRN fold) at 3 waves per SIMD: tests + .so A/B on the reference CNN
set -o pipefail
O=gpurun_out/r3occ; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_cli_gpu.py tests/test_ops_autograd_gpu.py tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/gpu_so_ab.sh r3occ/ab --model reference_cnn --batch 16384 --comm_probe 0 && python3 bench/prof_summary.py $O/ab/profA 7 $O/ab/kernelsA.md > /dev/null && python3 bench/prof_summary.py $O/ab/profB 7 $O/ab/kernelsB.md > /dev/null && grep -h -E "convpool_wgrad|total" $O/ab/kernelsA.md $O/ab/kernelsB.md
