#!/bin/bash
# conv1 wgrad variants: correctness (pooled-K SPLIT 1), step A/B and per-kernel time of each
set -o pipefail
O=gpurun_out/r3z2; mkdir -p $O
MNISTX_C1W_POOLK=1 MNISTX_C1W_SPLIT=1 timeout -k 10 200 python bench/dbg/c1w_dbg.py 2>&1 | grep "=="
MNISTX_C1W_POOLK=1 MNISTX_C1W_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "convpool or lenet_conv1" > $O/k1.log 2>&1; rc=$?
tail -1 $O/k1.log; [ $rc -eq 0 ] || exit $rc
bash bench/gpu_env_ab.sh 2 "MNISTX_C1W_POOLK=0" "MNISTX_C1W_POOLK=1 MNISTX_C1W_SPLIT=0" "MNISTX_C1W_POOLK=1 MNISTX_C1W_SPLIT=1" -- --steps 30 --warmup 5 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
bash bench/gpu_prof.sh r3z2/prof_old MNISTX_C1W_POOLK=0 -- --comm_probe 0 > /dev/null && echo "old: $(grep -E 'c1w|wgrad_pair' $O/prof_old/kernels.md)"
bash bench/gpu_prof.sh r3z2/prof_s0 MNISTX_C1W_POOLK=1 MNISTX_C1W_SPLIT=0 -- --comm_probe 0 > /dev/null && echo "s0: $(grep -E 'c1w|wgrad_pair' $O/prof_s0/kernels.md)"
bash bench/gpu_prof.sh r3z2/prof_s1 MNISTX_C1W_POOLK=1 MNISTX_C1W_SPLIT=1 -- --comm_probe 0 > /dev/null && echo "s1: $(grep -E 'c1w|wgrad_pair' $O/prof_s1/kernels.md)"
