# round-6 tree: full GPU suite, smoke, benches (LeNet driver default x2, reference CNN 1 / 3 channels)
set -o pipefail
O=gpurun_out/r6s2/suite; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $O/tests_gpu.log 2>&1; rc=$?; tail -3 $O/tests_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py > $O/lenet_$i.json 2>/dev/null || exit 1
  echo "lenet $(grep -o '"ms_per_step": [0-9.]*' $O/lenet_$i.json)"
done
timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 > $O/ref1.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --model reference_cnn --in_channels 3 --batch 16384 > $O/ref3.json 2>/dev/null || exit 1
echo "ref1 $(grep -o '"ms_per_step": [0-9.]*' $O/ref1.json) ref3 $(grep -o '"ms_per_step": [0-9.]*' $O/ref3.json)"
