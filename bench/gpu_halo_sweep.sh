#!/bin/bash
# conv_halo.hip variant sweep on the reference CNN (same box); prints ms/step per variant.
# Usage: bash bench/gpu_halo_sweep.sh TAG "FWD=a DGRAD=b" ...   (default: every variant)
OUT=gpurun_out/${1:-halo}; shift; mkdir -p $OUT
r() { local f=$1 d=$2; timeout -k 10 200 env MNISTX_HALO_FWD=$f MNISTX_HALO_DGRAD=$d python bench.py --model reference_cnn --batch 16384 --steps 10 --warmup 3 --phases 0 --eager_steps 0 > $OUT/f${f}_d${d}.log 2>&1 || return 1; echo "fwd=$f dgrad=$d $(grep -o '"ms_per_step": [0-9.]*' $OUT/f${f}_d${d}.log)"; }
PAIRS=${@:-"0:0 1:1 2:2 3:3 4:0 0:0"}
for p in $PAIRS; do r ${p%%:*} ${p##*:} || exit 1; done
