# refc1_wgrad: input fragments one (plane, row tile) ahead of their MFMA pair
set -o pipefail
O=gpurun_out/r6s2/rwpipe; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_refc1_wgrad_gpu.py tests/test_executor_gpu.py -k "refc1 or refcnn or reference" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/ab_micro.sh r6s2/rwpipe/ab3 3 bench.py --model reference_cnn --in_channels 3 --batch 16384 || exit 1
bash bench/ab_micro.sh r6s2/rwpipe/ab1 2 bench.py --model reference_cnn --batch 16384 || exit 1
bash bench/gpu_prof.sh r6s2/rwpipe/prof -- --model reference_cnn --in_channels 3 --batch 16384 || exit 1
