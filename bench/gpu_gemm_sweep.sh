#!/bin/bash
# Large dense GEMM sweep (reference CNN local3 / local4 shapes): tile x prefetch
# depth for the forward / data-gradient launches.  Usage: bash bench/gpu_gemm_sweep.sh TAG
OUT=gpurun_out/${1:-gemm_sweep}; mkdir -p $OUT
for cfg in "-1 1" "4 2" "4 3" "3 1" "3 2" "8 1" "8 2"; do
  set -- $cfg
  MNISTX_GEMM_TILE=$1 MNISTX_GEMM_PF=$2 timeout -k 10 120 python bench/micro_local3.py 16384 3136 1024 fwd \
    > $OUT/t$1_pf$2.log 2>&1 || exit $?
  echo "tile=$1 pf=$2"; grep -E "^(fwd|dgrad) +mnistx" $OUT/t$1_pf$2.log
done
