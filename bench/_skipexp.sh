cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for sk in 0 1 2 3; do
  MNISTX_EXP_SKIP=$sk timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/skip$sk -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --graph 0 --phases 0 --eager_steps 0 > gpurun_out/skip$sk.log 2>&1 || exit 1
  python3 bench/prof_summary.py gpurun_out/skip$sk 7 gpurun_out/skip$sk.md > /dev/null; echo "skip=$sk"; grep quad gpurun_out/skip$sk.md
done
