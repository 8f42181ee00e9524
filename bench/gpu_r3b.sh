#!/bin/bash
# band forward: tests, bench A/B, kernel table
set -o pipefail
O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lenet_band_gpu.py -x -v --timeout 120 --timeout-method thread > $O/band_tests.log 2>&1 || { tail -30 $O/band_tests.log; exit 1; }
tail -2 $O/band_tests.log
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
MNISTX_BAND_FWD=0 timeout -k 10 200 python bench.py > $O/bench_noband.json 2>> $O/bench.err || exit 1
timeout -k 10 200 python bench.py > $O/bench2.json 2>> $O/bench.err || exit 1
python3 -c "
import json
for f in ['bench','bench_noband','bench2']:
    d=json.load(open('$O/'+f+'.json')); print(f, d['ms_per_step'], d.get('phase_ms_eager'))"
bash bench/gpu_prof.sh r3b/prof_lenet -- --steps 5 || exit 1
