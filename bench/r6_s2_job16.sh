# reference CNN: dense weight gradients on a side stream beside the data-gradient chain
set -o pipefail
ARGS_A="--model reference_cnn --batch 16384 --overlap none" ARGS_B="--model reference_cnn --batch 16384 --overlap dense" bash bench/ab_args.sh r6s2/refov 3 || exit 1
