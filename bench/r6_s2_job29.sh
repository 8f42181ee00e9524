# refc1n3 spill fix (scalar LRN epilogue for 3 channels): tests, cin 1 / cin 3 step, cin 3 kernel table
set -o pipefail
O=gpurun_out/r6s2/cin3fix; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_refc1_fwd_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do for c in 1 3; do
  timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 --in_channels $c > $O/c${c}_$i.json 2>/dev/null || exit 1
  echo "cin $c $(grep -o '"ms_per_step": [0-9.]*' $O/c${c}_$i.json)"
done; done
bash bench/gpu_prof.sh r6s2/cin3fix/p3 -- --model reference_cnn --batch 16384 --in_channels 3 > /dev/null && \
grep "refc1\|total" $O/p3/kernels.md
