#!/bin/bash
# round 3: banded LeNet forward -- its tests, then the suite, the bench and a kernel table
set -o pipefail
O=gpurun_out/r3a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lenet_band_gpu.py -x -v --timeout 120 --timeout-method thread > $O/band_tests.log 2>&1 || { tail -30 $O/band_tests.log; exit 1; }
tail -3 $O/band_tests.log
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
MNISTX_BAND_FWD=0 timeout -k 10 200 python bench.py > $O/bench_noband.json 2>> $O/bench.err || exit 1
cat $O/bench_noband.json
bash bench/gpu_prof.sh r3a/prof_lenet -- --steps 5 || exit 1
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1; echo "suite rc=$?"; tail -3 $O/tests.log
