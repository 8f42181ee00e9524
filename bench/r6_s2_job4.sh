# refc1n3: A-fragment ring (next group's 9 reads in flight under this group's MFMAs)
set -o pipefail
O=gpurun_out/r6s2/refc1n3b; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_refc1_fwd_gpu.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --model reference_cnn --in_channels 3 --batch 16384 > $O/b3_$i.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "cin3 $(grep -o '"ms_per_step": [0-9.]*' $O/b3_$i.json) $(grep -o '"forward": [0-9.]*' $O/b3_$i.json)"
  timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/b1_$i.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "cin1 $(grep -o '"ms_per_step": [0-9.]*' $O/b1_$i.json) $(grep -o '"forward": [0-9.]*' $O/b1_$i.json)"
done
bash bench/gpu_prof.sh r6s2/refc1n3b/prof -- --model reference_cnn --in_channels 3 --batch 16384 || exit 1
