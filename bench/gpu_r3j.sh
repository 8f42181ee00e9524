#!/bin/bash
# r3j: MFMA/VALU co-issue microbench; PS bench at B=128 (1 PS + 3 workers); reference-CNN
# DP overlap trace at the BASELINE batch with one-rank RCCL collectives; LeNet bench w/o prewarm.
set -o pipefail
O=gpurun_out/r3j; mkdir -p $O
export TMPDIR=/tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 bench/micro/mfma_valu_overlap.hip -o /tmp/mvo 2>/dev/null && timeout -k 10 60 /tmp/mvo > $O/overlap.txt 2>&1 && cat $O/overlap.txt && \
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --mode ps --batch 128 --steps 300 --warmup 30 > $O/ps_b128.log 2>&1 && tail -1 $O/ps_b128.log && \
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --prewarm_ms 0 > $O/lenet_noprewarm.log 2>&1 && tail -1 $O/lenet_noprewarm.log && \
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/lenet_default.log 2>&1 && tail -1 $O/lenet_default.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/dp_trace -o dp -- python3 bench.py --model reference_cnn \
  --batch 16384 --steps 4 --warmup 2 --force_collectives 1 --graph 0 --prewarm_ms 0 --comm_probe 0 > $O/dp_trace.log 2>&1 && tail -1 $O/dp_trace.log
echo "rc=$?"
