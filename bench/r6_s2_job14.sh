# non-temporal loads for the LeNet step's last-use streams (band input rows; bwd records, dp2, codes, input)
set -o pipefail
O=gpurun_out/r6s2/nt; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_lenet_band_gpu.py tests/test_lenet_bwd_gpu.py -k "band or bwd" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/ab_micro.sh r6s2/nt/ab 4 bench.py || exit 1
bash bench/gpu_prof.sh r6s2/nt/prof -- --batch 65536 || exit 1
