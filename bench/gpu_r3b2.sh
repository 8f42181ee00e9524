#!/bin/bash
# band conv2 column remap: band tests + .so A/B vs abso/base.so
set -o pipefail
O=gpurun_out/r3b3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lenet_band_gpu.py tests/test_executor_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/gpu_so_ab.sh r3b3/ab --comm_probe 0 && python3 bench/prof_summary.py $O/ab/profA 7 $O/ab/kernelsA.md > /dev/null && python3 bench/prof_summary.py $O/ab/profB 7 $O/ab/kernelsB.md > /dev/null && grep band $O/ab/kernelsA.md $O/ab/kernelsB.md
