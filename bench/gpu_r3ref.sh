#!/bin/bash
# reference CNN B=16384: kernel table + PMC
set -o pipefail
bash bench/gpu_prof.sh r3ref/prof -- --model reference_cnn --batch 16384 --comm_probe 0 > /dev/null && cat gpurun_out/r3ref/prof/kernels.md
bash bench/pmc.sh r3ref/pmc -- --model reference_cnn --batch 16384 --comm_probe 0 --prewarm_ms 0 && python3 bench/pmc_summary.py gpurun_out/r3ref/pmc gpurun_out/r3ref/pmc/pmc.md > /dev/null && grep -vE "at::native|^\|---" gpurun_out/r3ref/pmc/pmc.md | head -20
