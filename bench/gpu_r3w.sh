#!/bin/bash
# band (in-lane conv1 + conv2) / executor / kernel / PS (incl. in-place session recovery over ipc)
# GPU tests, then a same-box A/B against abso/base.so and the new build's kernel table
set -o pipefail
O=gpurun_out/r3w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_lenet_band_gpu.py tests/test_executor_gpu.py tests/test_kernels_gpu.py tests/test_mlp_head_gpu.py -x -q --timeout 120 --timeout-method thread > $O/k_tests.log 2>&1; rc=$?
tail -3 $O/k_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_ps_gpu.py -x -v --timeout 200 --timeout-method thread --basetemp=/tmp/r3w_tmp > $O/ps_tests.log 2>&1; rc=$?
tail -10 $O/ps_tests.log; [ $rc -eq 0 ] || { cp -r /tmp/r3w_tmp/*recovery* $O/ 2>/dev/null; exit $rc; }
bash bench/gpu_so_ab.sh r3w/ab --comm_probe 0 && python3 bench/prof_summary.py $O/ab/profA 7 $O/ab/kernelsA.md > /dev/null && python3 bench/prof_summary.py $O/ab/profB 7 $O/ab/kernelsB.md > /dev/null && cat $O/ab/kernelsA.md && head -4 $O/ab/kernelsB.md
