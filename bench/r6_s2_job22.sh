# packed norm2 -> pool2 kernels (lrn_pool14_*): full GPU suite (the window-sum contraction
# change touches every LRN kernel), then same-box interleaved A/B and kernel tables
set -o pipefail
O=gpurun_out/r6s2/lrnpk; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do for t in 0 1; do
  MNISTX_LRN_PK=$t timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/pk${t}_$i.json 2>/dev/null || exit 1
  echo "lrn_pk $t $(grep -o '"ms_per_step": [0-9.]*' $O/pk${t}_$i.json)"
done; done
bash bench/gpu_prof.sh r6s2/lrnpk/p0 MNISTX_LRN_PK=0 -- --model reference_cnn --batch 16384 > /dev/null && \
bash bench/gpu_prof.sh r6s2/lrnpk/p1 MNISTX_LRN_PK=1 -- --model reference_cnn --batch 16384 > /dev/null && \
grep "lrn_pool\|total" $O/p*/kernels.md
