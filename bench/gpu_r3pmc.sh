#!/bin/bash
# PMC of the LeNet step with the pooled-K conv1 wgrad (and the unpool kernel for comparison)
set -o pipefail
bash bench/pmc.sh r3pmc/pk -- --comm_probe 0 --prewarm_ms 0 && python3 bench/pmc_summary.py gpurun_out/r3pmc/pk gpurun_out/r3pmc/pk/pmc.md > /dev/null && grep -E "c1w|wgrad_pair|kernel \|" gpurun_out/r3pmc/pk/pmc.md
export MNISTX_C1W_POOLK=0
bash bench/pmc.sh r3pmc/old -- --comm_probe 0 --prewarm_ms 0 && python3 bench/pmc_summary.py gpurun_out/r3pmc/old gpurun_out/r3pmc/old/pmc.md > /dev/null && grep -E "c1w|wgrad_pair" gpurun_out/r3pmc/old/pmc.md
