#!/bin/bash
# band forward: tests, role busy/wait split, same-box A/B vs the previous build (abso/base.so)
set -o pipefail
O=gpurun_out/r3v; mkdir -p $O
#timeout -k 10 300 python -u -m pytest tests/test_lenet_band_gpu.py tests/test_executor_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
#tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
#timeout -k 10 200 python bench/micro_band.py > $O/micro_band.txt 2>&1 || { cat $O/micro_band.txt; exit 1; }
#cat $O/micro_band.txt
bash bench/gpu_so_ab.sh r3v/ab --comm_probe 0 && python3 bench/prof_summary.py $O/ab/profA 7 $O/ab/kernelsA.md > /dev/null && python3 bench/prof_summary.py $O/ab/profB 7 $O/ab/kernelsB.md > /dev/null && head -5 $O/ab/kernelsA.md $O/ab/kernelsB.md
