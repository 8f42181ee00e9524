# grouped head weight gradient: one split count for fc3 / fc4 / fc5 (balanced K per block)
set -o pipefail
O=gpurun_out/r6s2/wgbal; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_executor_gpu.py tests/test_mlp_head_gpu.py -k "lenet or head or group" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
ENV_A="MNISTX_WGRAD_GROUP_BLOCKS=0" ENV_B="MNISTX_WGRAD_GROUP_BLOCKS=768" bash bench/ab_args.sh r6s2/wgbal/ab 4 || exit 1
for t in 512 1024 1536; do
  MNISTX_WGRAD_GROUP_BLOCKS=$t timeout -k 10 200 python bench.py > $O/t$t.json 2>/dev/null || exit 1
  echo "target $t $(grep -o '"ms_per_step": [0-9.]*' $O/t$t.json) $(grep -o '"backward": [0-9.]*' $O/t$t.json)"
done
bash bench/gpu_prof.sh r6s2/wgbal/prof -- --batch 65536 || exit 1
