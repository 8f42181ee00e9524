set -o pipefail
O=gpurun_out/r6/job3; mkdir -p $O
timeout -k 10 100 python bench/dbg/band_p0.py > $O/p0_new.txt 2>&1; cat $O/p0_new.txt | grep -v amdgpu.ids
(cd ab_old && timeout -k 10 100 python bench/dbg/band_p0.py) > $O/p0_old.txt 2>&1; grep -v amdgpu.ids $O/p0_old.txt
timeout -k 10 200 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_lenet_band_gpu.py -k "not dataset_gather" > $O/band_tests.log 2>&1; tail -3 $O/band_tests.log
bash bench/ab_micro.sh r6/job3/band_ab 3 bench/micro_band.py one 2 65536 || exit 1
bash bench/ab_micro.sh r6/job3/bench_ab 2 bench.py || exit 1
echo job3 done
