#!/bin/bash
set -o pipefail
O=gpurun_out/r3e; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for dbg in 0 2; do
MNISTX_BAND_DBG=$dbg timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace -d $O/d$dbg/pmc1 -o run --output-format csv -- python3 bench/micro_band.py one 0 65536 > $O/pmc1_$dbg.log 2>&1 && \
MNISTX_BAND_DBG=$dbg timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d $O/d$dbg/pmc2 -o run --output-format csv -- python3 bench/micro_band.py one 0 65536 > $O/pmc2_$dbg.log 2>&1 || exit 1
python3 bench/pmc_summary.py $O/d$dbg $O/pmc_d$dbg.md | grep band
done
python3 - <<'PY'
import csv,glob
for d in ("0","2"):
    for f in glob.glob(f"gpurun_out/r3e/d{d}/pmc*/*counter_collection.csv"):
        acc={}
        for r in csv.DictReader(open(f)):
            if "band" in r["Kernel_Name"]: acc[r["Counter_Name"]]=float(r["Counter_Value"])
        print(d, {k: f"{v:.3g}" for k,v in acc.items()})
PY
