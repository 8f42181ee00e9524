# band forward: pool1 record copy-out on conv2 wave 7 only
set -o pipefail
O=gpurun_out/r6s2/copyw7; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_lenet_band_gpu.py tests/test_lenet_bwd_gpu.py tests/test_executor_gpu.py -k "band or lenet or u8" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 120 python bench/micro_band.py one 2 65536 > $O/m_new_$i.txt 2>&1; echo "new $(tail -1 $O/m_new_$i.txt)"
(cd ab_old && timeout -k 10 120 python bench/micro_band.py one 2 65536) > $O/m_old_$i.txt 2>&1; echo "old $(tail -1 $O/m_old_$i.txt)"
done
bash bench/ab_micro.sh r6s2/copyw7/ab 4 bench.py || exit 1
