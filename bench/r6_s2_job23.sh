# packed vs generic norm2 -> pool2 kernels in isolation + one PMC pass over both
set -o pipefail
O=gpurun_out/r6s2/lrnpk_micro; mkdir -p $O
timeout -k 10 120 python bench/micro_lrnpool.py > $O/micro.json 2> $O/micro.err || { tail $O/micro.err; exit 1; }
cat $O/micro.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc -o run --output-format csv -- python3 bench/micro_lrnpool.py --rounds 1 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
ls $O/pmc
