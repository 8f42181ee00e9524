#!/bin/bash
# PS / comm-probe tests first (new code), then the rest of the suite, smoke, bench
set -o pipefail
O=gpurun_out/r3h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ps_gpu.py tests/test_bench_multirank_gpu.py -x -v --timeout 280 --timeout-method thread > $O/new_tests.log 2>&1; rc=$?
tail -15 $O/new_tests.log; echo "new rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 280 --timeout-method thread --deselect tests/test_ps_gpu.py --deselect tests/test_bench_multirank_gpu.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; echo "suite rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
