# round-6 end-of-round evidence: full GPU suite, smoke, LeNet driver-default bench x3,
# reference CNN 1 / 3 channels x2, kernel tables of all three
set -o pipefail
O=gpurun_out/r6final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $O/tests_gpu.log 2>&1; rc=$?; tail -3 $O/tests_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/lenet_$i.json 2>/dev/null || exit 1
  echo "lenet $(grep -o '"ms_per_step": [0-9.]*' $O/lenet_$i.json)"
done
for i in 1 2; do for c in 1 3; do
  timeout -k 10 200 python bench.py --model reference_cnn --batch 16384 --in_channels $c > $O/ref${c}_$i.json 2>/dev/null || exit 1
  echo "ref cin $c $(grep -o '"ms_per_step": [0-9.]*' $O/ref${c}_$i.json)"
done; done
bash bench/gpu_prof.sh r6final/prof_lenet -- > /dev/null && \
bash bench/gpu_prof.sh r6final/prof_ref1 -- --model reference_cnn --batch 16384 > /dev/null && \
bash bench/gpu_prof.sh r6final/prof_ref3 -- --model reference_cnn --batch 16384 --in_channels 3 > /dev/null && \
for f in $O/prof_*/kernels.md; do tail -n 2 $f; done
