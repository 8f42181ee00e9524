# kernel tables of the reference CNN step with / without the fused softmax tail
set -o pipefail
bash bench/gpu_prof.sh r6s2/cetail_prof/t0 MNISTX_CE_TAIL=0 -- --model reference_cnn --batch 16384 && \
bash bench/gpu_prof.sh r6s2/cetail_prof/t1 MNISTX_CE_TAIL=1 -- --model reference_cnn --batch 16384
