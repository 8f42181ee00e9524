# reference CNN conv1 argmax codes 4 bits each (refc1n forward -> refc1_wgrad): tests, then
# same-box interleaved A/B (cin 1 x3, cin 3 x2) and kernel tables
set -o pipefail
O=gpurun_out/r6s2/codes4; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_refc1_fwd_gpu.py tests/test_refc1_wgrad_gpu.py tests/test_executor_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do for t in 0 1; do
  MNISTX_REFC1_CODES4=$t timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/c${t}_$i.json 2>/dev/null || exit 1
  echo "codes4 $t $(grep -o '"ms_per_step": [0-9.]*' $O/c${t}_$i.json)"
done; done
for i in 1 2; do for t in 0 1; do
  MNISTX_REFC1_CODES4=$t timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 --in_channels 3 > $O/c3_${t}_$i.json 2>/dev/null || exit 1
  echo "cin3 codes4 $t $(grep -o '"ms_per_step": [0-9.]*' $O/c3_${t}_$i.json)"
done; done
bash bench/gpu_prof.sh r6s2/codes4/p0 MNISTX_REFC1_CODES4=0 -- --model reference_cnn --batch 16384 > /dev/null && \
bash bench/gpu_prof.sh r6s2/codes4/p1 MNISTX_REFC1_CODES4=1 -- --model reference_cnn --batch 16384 > /dev/null && \
grep "refc1\|total" $O/p*/kernels.md
