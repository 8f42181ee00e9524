# refc1n3_fwd_k (3-channel conv1 + pool1 + norm1): tests, same-box A/B vs the convpool path, kernel table
set -o pipefail
O=gpurun_out/r6s2/refc1n3; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_refc1_fwd_gpu.py tests/test_executor_gpu.py -k "refc1 or refcnn or lrn or reference_cnn3" > $O/tests.log 2>&1; rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for f in 1 2; do
  MNISTX_REFC1_FWD=$f timeout -k 10 200 python bench.py --model reference_cnn --in_channels 3 --batch 16384 > $O/b${f}_$i.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "variant=$f $(grep -o '"ms_per_step": [0-9.]*' $O/b${f}_$i.json) $(grep -o '"forward": [0-9.]*' $O/b${f}_$i.json)"
done; done
timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/b_cin1.json 2>$O/b.err || exit 1
echo "cin1 $(grep -o '"ms_per_step": [0-9.]*' $O/b_cin1.json)"
bash bench/gpu_prof.sh r6s2/refc1n3/prof -- --model reference_cnn --in_channels 3 --batch 16384 || exit 1
ENV_A="MNISTX_BWD_REVERSE=0" ENV_B="MNISTX_BWD_REVERSE=1" bash bench/ab_args.sh r6s2/bwd_rev 3 || exit 1
