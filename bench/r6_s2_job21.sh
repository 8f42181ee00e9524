# ce_tail_k waves per block (32 rows each): 1 (512 blocks at B=16384), 2, 4 -- tests at the new
# default, then same-box interleaved step A/B
set -o pipefail
O=gpurun_out/r6s2/cetail_nw; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ce_tail_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for t in 1 2 4; do
  MNISTX_CE_TAIL_NW=$t timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/nw${t}_$i.json 2>/dev/null || exit 1
  echo "nw $t $(grep -o '"ms_per_step": [0-9.]*' $O/nw${t}_$i.json)"
done; done
bash bench/gpu_prof.sh r6s2/cetail_nw/p1 MNISTX_CE_TAIL_NW=1 -- --model reference_cnn --batch 16384 > /dev/null && \
bash bench/gpu_prof.sh r6s2/cetail_nw/p2 MNISTX_CE_TAIL_NW=2 -- --model reference_cnn --batch 16384 > /dev/null && \
grep ce_tail $O/p*/kernels.md
