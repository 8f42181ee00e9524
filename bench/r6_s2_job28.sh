# kernel tables: reference CNN cin 1 vs cin 3 (the 3-channel gap)
set -o pipefail
bash bench/gpu_prof.sh r6s2/cin3/p1 -- --model reference_cnn --batch 16384 > /dev/null && \
bash bench/gpu_prof.sh r6s2/cin3/p3 -- --model reference_cnn --batch 16384 --in_channels 3 > /dev/null && \
cat gpurun_out/r6s2/cin3/p1/kernels.md gpurun_out/r6s2/cin3/p3/kernels.md | grep -v Cijk
