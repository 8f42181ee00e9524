set -o pipefail
O=gpurun_out/r6s2/base; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench1.json 2> $O/bench1.err || { tail -5 $O/bench1.err; exit 1; }
cat $O/bench1.json
bash bench/gpu_prof.sh r6s2/base/prof -- --batch 65536 || exit 1
timeout -k 10 300 python bench.py > $O/bench2.json 2> $O/bench2.err || exit 1
cat $O/bench2.json
