# reference CNN: split-K target of the few-tile dense weight gradients (local4: 51 tiles)
set -o pipefail
O=gpurun_out/r6s2/refwgb; mkdir -p $O
for i in 1 2; do for t in 256 512 1024 2048; do
  MNISTX_WGRAD_BLOCKS=$t timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/t${t}_$i.json 2>/dev/null || exit 1
  echo "target $t $(grep -o '"ms_per_step": [0-9.]*' $O/t${t}_$i.json) $(grep -o '"backward": [0-9.]*' $O/t${t}_$i.json)"
done; done
