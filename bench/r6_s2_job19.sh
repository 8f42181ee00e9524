# reference CNN softmax tail fusion (ce_tail_k): tests, then same-box interleaved A/B, then the
# split-K target sweep of job18 (one pass)
set -o pipefail
O=gpurun_out/r6s2/cetail; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ce_tail_gpu.py tests/test_mlp_head_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2 3; do for t in 0 1; do
  MNISTX_CE_TAIL=$t timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/t${t}_$i.json 2>/dev/null || exit 1
  echo "ce_tail $t $(grep -o '"ms_per_step": [0-9.]*' $O/t${t}_$i.json)"
done; done
for t in 256 1024 2048; do
  MNISTX_WGRAD_BLOCKS=$t timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/wgb${t}.json 2>/dev/null || exit 1
  echo "wgrad target $t $(grep -o '"ms_per_step": [0-9.]*' $O/wgb${t}.json)"
done
