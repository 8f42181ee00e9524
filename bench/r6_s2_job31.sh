# LeNet grouped head weight gradient: K rows per step 32 (default) / 64 (PF 2, 3) / 96
set -o pipefail
O=gpurun_out/r6s2/wgbk; mkdir -p $O
MNISTX_WG_GROUP_BK=64 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_head_gpu.py tests/test_executor_gpu.py -k "lenet or head" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for t in 32 64 642 96; do
  MNISTX_WG_GROUP_BK=$t timeout -k 10 200 python bench.py > $O/k${t}_$i.json 2>/dev/null || exit 1
  echo "bk $t $(grep -o '"ms_per_step": [0-9.]*' $O/k${t}_$i.json)"
done; done
