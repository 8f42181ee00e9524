#!/bin/bash
# conv_halo.hip variant sweep on the reference CNN (same box); prints ms/step per variant
OUT=gpurun_out/${1:-halo}; mkdir -p $OUT
r() { timeout -k 10 200 env "$@" python bench.py --model reference_cnn --batch 16384 --steps 10 --warmup 3 --phases 0 > $OUT/$(echo "$@" | tr ' =' '__').log 2>&1 || return 1; echo "$@ $(grep -o '"ms_per_step": [0-9.]*' $OUT/$(echo "$@" | tr ' =' '__').log)"; }
r MNISTX_HALO_FWD=0 MNISTX_HALO_DGRAD=0 && r MNISTX_HALO_FWD=3 MNISTX_HALO_DGRAD=0 && r MNISTX_HALO_FWD=1 MNISTX_HALO_DGRAD=1 && \
r MNISTX_HALO_FWD=0 MNISTX_HALO_DGRAD=0 && r MNISTX_CONV_HALO=0
