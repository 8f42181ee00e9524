# LeNet head weight-gradient split target 256 vs 192: kernel tables + 4 more interleaved pairs
set -o pipefail
O=gpurun_out/r6s2/lenet_wgb3; mkdir -p $O
bash bench/gpu_prof.sh r6s2/lenet_wgb3/p256 MNISTX_WGRAD_BLOCKS=256 -- > /dev/null && \
bash bench/gpu_prof.sh r6s2/lenet_wgb3/p192 MNISTX_WGRAD_BLOCKS=192 -- > /dev/null && \
grep "wg_group\|splitk\|lenet_bwd\|total" $O/p256/kernels.md $O/p192/kernels.md || exit 1
for i in 1 2 3 4; do for t in 256 192; do
  MNISTX_WGRAD_BLOCKS=$t timeout -k 10 200 python bench.py > $O/t${t}_$i.json 2>/dev/null || exit 1
  echo "target $t $(grep -o '"ms_per_step": [0-9.]*' $O/t${t}_$i.json)"
done; done
