#!/bin/bash
# full GPU suite + smoke + driver-default bench (one call)
set -o pipefail
O=gpurun_out/${1:-suite_r3}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --durations=15 --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
