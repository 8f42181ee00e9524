#!/bin/bash
# Backward-overlap budget sweep (same box): baseline vs --overlap all with
# co-residency budgets MNISTX_OVERLAP_WGS="dgrad,side_wgrad[,conv1_wgrad]" per CU.
OUT=gpurun_out/${1:-ovl}; mkdir -p $OUT
run() {  # run TAG ENV_ASSIGNMENT [bench args...]
  local tag=$1 envs=$2; shift 2
  timeout -k 10 200 env $envs python bench.py --steps 30 --warmup 5 --phases 0 "$@" > $OUT/$tag.log 2>&1 || return 1
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log)"
}
run base MNISTX_NOOP=1 && run all MNISTX_NOOP=1 --overlap all && \
run w21 MNISTX_OVERLAP_WGS=2,1 --overlap all && run w214 MNISTX_OVERLAP_WGS=2,1,4 --overlap all && \
run w12 MNISTX_OVERLAP_WGS=1,2 --overlap all && run w22 MNISTX_OVERLAP_WGS=2,2 --overlap all && \
run w114 MNISTX_OVERLAP_WGS=1,1,4 --overlap all && run base2 MNISTX_NOOP=1
