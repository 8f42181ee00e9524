# reference CNN PMC passes (instruction mix, MFMA busy, HBM bytes per kernel)
set -o pipefail
bash bench/pmc.sh r6s2/refpmc -- --model reference_cnn --batch 16384 && \
python3 bench/pmc_summary.py gpurun_out/r6s2/refpmc gpurun_out/r6s2/refpmc/pmc.md > /dev/null && head -30 gpurun_out/r6s2/refpmc/pmc.md
