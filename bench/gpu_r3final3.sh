#!/bin/bash
# HEAD evidence after the band conv2 bank fix: band/executor/kernel tests, smoke, driver-default benches,
# no-prewarm, kernel table, PMC
set -o pipefail
O=gpurun_out/r3final3; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_lenet_band_gpu.py tests/test_executor_gpu.py tests/test_kernels_gpu.py tests/test_cli_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
for i in 1 2 3; do timeout -k 10 200 python bench.py > $O/bench_default_$i.json 2> $O/bench_$i.err || exit 1; done
timeout -k 10 200 python bench.py --prewarm_ms 0 > $O/bench_noprewarm.json 2> $O/bench_np.err || exit 1
for f in bench_default_1 bench_default_2 bench_default_3 bench_noprewarm; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $O/$f.json)"; done
bash bench/gpu_prof.sh r3final3/prof_lenet -- --comm_probe 0 > /dev/null && head -16 gpurun_out/r3final3/prof_lenet/kernels.md
bash bench/pmc.sh r3final3/pmc_lenet -- --comm_probe 0 --prewarm_ms 0 && python3 bench/pmc_summary.py gpurun_out/r3final3/pmc_lenet gpurun_out/r3final3/pmc_lenet/pmc.md > /dev/null && grep -E "band|dgrad_pair|wgrad" gpurun_out/r3final3/pmc_lenet/pmc.md
echo done
