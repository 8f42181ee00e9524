#!/bin/bash
# PMC of the reference CNN step (B = 16384)
set -o pipefail
bash bench/pmc.sh r3refpmc -- --model reference_cnn --batch 16384 --comm_probe 0 --prewarm_ms 0 && python3 bench/pmc_summary.py gpurun_out/r3refpmc gpurun_out/r3refpmc/pmc.md > /dev/null && cat gpurun_out/r3refpmc/pmc.md | cut -c1-400
