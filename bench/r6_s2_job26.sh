# refc1_wgrad with the LRN backward of two rounds packed (v_pk): tests, micro old vs new,
# whole reference-CNN step old vs new (same box, interleaved)
set -o pipefail
O=gpurun_out/r6s2/refc1pk; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_refc1_wgrad_gpu.py tests/test_refc1_fwd_gpu.py tests/test_kernels_gpu.py -k "refc1 or lrn or refcnn" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 120 python bench/micro_refc1.py > $O/micro_new_$i.json 2>/dev/null || exit 1
  (cd ab_old && timeout -k 10 120 python bench/micro_refc1.py) > $O/micro_old_$i.json 2>/dev/null || exit 1
done
cat $O/micro_*.json | cut -c1-300
bash bench/ab_bench.sh r6s2/refc1pk/ab 3 --model reference_cnn --batch 16384 | cut -c1-60
