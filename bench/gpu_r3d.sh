#!/bin/bash
set -o pipefail
O=gpurun_out/r3d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lenet_band_gpu.py -x -q --timeout 120 --timeout-method thread > $O/band_tests.log 2>&1 || { tail -30 $O/band_tests.log; exit 1; }
tail -1 $O/band_tests.log
timeout -k 10 600 python bench/micro_band.py > $O/micro.txt 2>&1; cat $O/micro.txt
