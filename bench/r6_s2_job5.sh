# lenet_bwd: pool1-record code words prefetched one tile ahead; tests + same-box A/B vs ab_old
set -o pipefail
O=gpurun_out/r6s2/bwd_aw; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_lenet_bwd_gpu.py tests/test_executor_gpu.py -k "lenet" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/ab_micro.sh r6s2/bwd_aw/ab 3 bench.py || exit 1
timeout -k 10 120 python bench/micro_lenet_bwd_quick.py > $O/micro_new.txt 2>&1; tail -2 $O/micro_new.txt
(cd ab_old && timeout -k 10 120 python bench/micro_lenet_bwd_quick.py) > $O/micro_old.txt 2>&1; tail -2 $O/micro_old.txt
