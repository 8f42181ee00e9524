set -o pipefail
O=gpurun_out/r6/job4; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_executor_gpu.py -k "u8_input_path or reference_cnn" tests/test_refc1_wgrad_gpu.py > $O/tests.log 2>&1; rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_ps_gpu.py > $O/ps_tests.log 2>&1; rc=$?; tail -4 $O/ps_tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/ab_micro.sh r6/job4/ref3_ab 2 bench.py --model reference_cnn --in_channels 3 --batch 16384 || exit 1
echo job4 done
