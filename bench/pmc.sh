#!/bin/bash
# PMC counter passes (kernel-trace only, no sys/runtime trace).  Usage: bash bench/pmc.sh TAG -- <bench args>
TAG=$1; shift; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace -d $OUT/pmc1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --graph 0 "$@" > $OUT/pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --graph 0 "$@" > $OUT/pmc2.log 2>&1
echo "pmc rc=$?"
# HBM bytes per kernel (FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2: one pass each)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc3 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --graph 0 "$@" > $OUT/pmc3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc4 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --graph 0 "$@" > $OUT/pmc4.log 2>&1
echo "bytes rc=$?"
