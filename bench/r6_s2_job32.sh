# LeNet grouped head weight gradient: split-K block target 256 (default) / 384 / 512 / 192
set -o pipefail
O=gpurun_out/r6s2/lenet_wgb2; mkdir -p $O
for i in 1 2 3 4; do for t in 256 192 128 224; do
  MNISTX_WGRAD_BLOCKS=$t timeout -k 10 200 python bench.py > $O/t${t}_$i.json 2>/dev/null || exit 1
  echo "target $t $(grep -o '"ms_per_step": [0-9.]*' $O/t${t}_$i.json)"
done; done
