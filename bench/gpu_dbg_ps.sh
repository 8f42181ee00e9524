#!/bin/bash
O=gpurun_out/dbgps; mkdir -p $O
MNIST_FI_CORRUPT_PUSH=0:4 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=3 --master-addr=127.0.0.1 --master-port=29533 bench.py --mode ps --ps_transport ipc --batch 256 --steps 20 --warmup 2 > $O/out.txt 2>&1; echo "rc=$?" >> $O/out.txt
grep -v "amdgpu.ids\|hostname of the client" $O/out.txt | tail -40
