# refc1n_fwd_k (conv1 + pool1 + norm1 in one launch): tests, same-box A/B, kernel table
set -o pipefail
O=gpurun_out/r6s2/refc1n; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_refc1_fwd_gpu.py tests/test_executor_gpu.py -k "refc1 or refcnn or lrn" > $O/tests.log 2>&1; rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for f in 0 1; do
  MNISTX_FOLD_LRN_FWD1=$f timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/b${f}_$i.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "fold=$f $(grep -o '"ms_per_step": [0-9.]*' $O/b${f}_$i.json) $(grep -o '"forward": [0-9.]*' $O/b${f}_$i.json)"
done; done
bash bench/gpu_prof.sh r6s2/refc1n/prof -- --model reference_cnn --batch 16384 || exit 1
