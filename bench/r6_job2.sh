set -o pipefail
O=gpurun_out/r6/job2; mkdir -p $O
timeout -k 10 120 bash bench/dbg/ps_shm_repro.sh r6/job2/shm || exit 1
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_lenet_band_gpu.py > $O/band_tests.log 2>&1; rc=$?; tail -3 $O/band_tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/ab_micro.sh r6/job2/band_ab 3 bench/micro_band.py one 2 65536 || exit 1
bash bench/ab_micro.sh r6/job2/bench_ab 2 bench.py || exit 1
echo job2 done
