# round-end PMC passes (instruction mix, MFMA busy, LDS conflicts, HBM bytes): LeNet, reference CNN
set -o pipefail
bash bench/pmc.sh r6final/pmc_lenet -- && \
python3 bench/pmc_summary.py gpurun_out/r6final/pmc_lenet gpurun_out/r6final/pmc_lenet/pmc.md > /dev/null && \
bash bench/pmc.sh r6final/pmc_ref1 -- --model reference_cnn --batch 16384 && \
python3 bench/pmc_summary.py gpurun_out/r6final/pmc_ref1 gpurun_out/r6final/pmc_ref1/pmc.md > /dev/null && \
head -12 gpurun_out/r6final/pmc_lenet/pmc.md
