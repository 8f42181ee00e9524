# eager split-K reduce of the big slabs (local3 60 MB+, conv2 52 MB) vs one flush at the end
set -o pipefail
O=gpurun_out/r6s2/eager; mkdir -p $O
MNISTX_EAGER_REDUCE_MB=16 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_executor_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for t in 0 60 16; do
  MNISTX_EAGER_REDUCE_MB=$t timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/e${t}_$i.json 2>/dev/null || exit 1
  echo "eager $t $(grep -o '"ms_per_step": [0-9.]*' $O/e${t}_$i.json)"
done; done
