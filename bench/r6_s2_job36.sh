# PMC passes, reference CNN with 3 input channels (the refc1n3 / refc1_wgrad<3> rows)
set -o pipefail
bash bench/pmc.sh r6final/pmc_ref3 -- --model reference_cnn --batch 16384 --in_channels 3 && \
python3 bench/pmc_summary.py gpurun_out/r6final/pmc_ref3 gpurun_out/r6final/pmc_ref3/pmc.md > /dev/null && \
grep "refc1" gpurun_out/r6final/pmc_ref3/pmc.md
