#!/bin/bash
# r3 session-3 final (after the conv1 / conv2 wgrad base changes): full GPU suite + smoke + driver-default bench x2 + no-prewarm bench + LeNet kernel table
# + reference CNN kernel table + reference CNN bf16 / fp32 benches
set -o pipefail
O=gpurun_out/r3final6; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --durations=10 --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
for i in 1 2; do timeout -k 10 200 python bench.py > $O/bench_default_$i.json 2> $O/bench_$i.err || exit 1; done
timeout -k 10 200 python bench.py --prewarm_ms 0 > $O/bench_noprewarm.json 2> $O/bench_np.err || exit 1
timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 --steps 20 --warmup 5 > $O/bench_refcnn.json 2> $O/bench_ref.err || exit 1
timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 --precision fp32 --steps 5 --warmup 2 > $O/bench_refcnn_fp32.json 2> $O/bench_f32.err || exit 1
for f in bench_default_1 bench_default_2 bench_noprewarm bench_refcnn bench_refcnn_fp32; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $O/$f.json)"; done
bash bench/gpu_prof.sh r3final6/prof_lenet -- --comm_probe 0 > /dev/null && head -16 gpurun_out/r3final6/prof_lenet/kernels.md
bash bench/gpu_prof.sh r3final6/prof_ref -- --model reference_cnn --batch 16384 --comm_probe 0 > /dev/null && head -30 gpurun_out/r3final6/prof_ref/kernels.md
echo done
