# refc1_wgrad 3 channels: 16-byte image pad (conflict-free A reads): tests, micro and step vs ab_old
set -o pipefail
O=gpurun_out/r6s2/wg3pad; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_refc1_wgrad_gpu.py tests/test_refc1_fwd_gpu.py tests/test_executor_gpu.py -k "refc1 or refcnn or cin3 or reference" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 120 python bench/micro_refc1.py --cin 3 > $O/micro_new_$i.json 2>/dev/null || exit 1
  (cd ab_old && timeout -k 10 120 python bench/micro_refc1.py --cin 3) > $O/micro_old_$i.json 2>/dev/null || exit 1
  echo "new $(grep -o '"refc1_us": [0-9.]*' $O/micro_new_$i.json) old $(grep -o '"refc1_us": [0-9.]*' $O/micro_old_$i.json)"
done
bash bench/ab_bench.sh r6s2/wg3pad/ab 3 --model reference_cnn --batch 16384 --in_channels 3 | cut -c1-40
