# split target 192: executor / head tests, and the reference CNN (local4 wgrad 4 vs 5 splits)
set -o pipefail
O=gpurun_out/r6s2/wgb_ref; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_executor_gpu.py tests/test_mlp_head_gpu.py tests/test_ce_tail_gpu.py tests/test_fused_launch_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for t in 256 192; do
  MNISTX_WGRAD_BLOCKS=$t timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/t${t}_$i.json 2>/dev/null || exit 1
  echo "ref target $t $(grep -o '"ms_per_step": [0-9.]*' $O/t${t}_$i.json)"
done; done
