#!/bin/bash
set -o pipefail
O=gpurun_out/r3c; mkdir -p $O
timeout -k 10 600 python bench/micro_band.py > $O/micro.txt 2>&1; cat $O/micro.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace -d $O/pmc1 -o run --output-format csv -- python3 bench/micro_band.py one 0 65536 > $O/pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc2 -o run --output-format csv -- python3 bench/micro_band.py one 0 65536 > $O/pmc2.log 2>&1
echo pmc rc=$?
python3 bench/pmc_summary.py $O $O/pmc.md | head -5
