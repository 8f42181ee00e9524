#!/bin/bash
# r3k: PS bench A/B (PS stream priority on/off) at B=128, 1 PS + 3 workers; small-batch graphed DP step.
set -o pipefail
O=gpurun_out/r3k; mkdir -p $O
ps() {  # tag env...
  local tag=$1; shift
  timeout -k 10 240 env "$@" python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --mode ps --batch 128 --steps 300 --warmup 30 > $O/ps_$tag.log 2>&1 && \
  python bench/ps_summary.py $tag $O/ps_$tag.log
}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 bench/micro/mfma_valu_overlap2.hip -o /tmp/mvo2 2>/dev/null && timeout -k 10 60 /tmp/mvo2 && \
ps def MNISTX_NOOP=1 && ps hq4 MNISTX_PS_HW_QUEUES=4 && ps def2 MNISTX_NOOP=1 && ps hq2 MNISTX_PS_HW_QUEUES=2 && ps def3 MNISTX_NOOP=1 && \
timeout -k 10 120 python bench.py --batch 128 --steps 500 --warmup 50 --graph 1 --prewarm_ms 0 --comm_probe 0 --phases 0 > $O/dp_b128.log 2>&1 && tail -1 $O/dp_b128.log | cut -c1-400
echo "rc=$?"
