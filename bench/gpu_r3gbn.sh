#!/bin/bash
# head weight-gradient column tile 64 vs 128 with the 256-workgroup split-K target, same box, interleaved
set -o pipefail
O=gpurun_out/r3gbn; mkdir -p $O
for rep in 1 2 3; do
  for v in 128 64; do
    MNISTX_WG_GROUP_BN=$v timeout -k 10 200 python bench.py --steps 30 --comm_probe 0 > $O/g_${v}_$rep.json 2> $O/g_${v}_$rep.err || exit 1
    echo "$v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $O/g_${v}_$rep.json)"
  done
done
