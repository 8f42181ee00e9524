# lenet_bwd: conv2 wgrad k-steps through one runtime-group code path (no switch)
set -o pipefail
O=gpurun_out/r6s2/c2rt; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_lenet_bwd_gpu.py tests/test_executor_gpu.py -k "lenet" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 120 python bench/micro_lenet_bwd_quick.py > $O/micro_new_$i.txt 2>&1; echo "new $(tail -1 $O/micro_new_$i.txt)"
(cd ab_old && timeout -k 10 120 python bench/micro_lenet_bwd_quick.py) > $O/micro_old_$i.txt 2>&1; echo "old $(tail -1 $O/micro_old_$i.txt)"
done
