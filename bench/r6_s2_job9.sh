set -o pipefail
bash bench/ab_micro.sh r6s2/xidx2/ab 4 bench.py || exit 1
bash bench/ab_micro.sh r6s2/xidx2/ab_ref 2 bench.py --model reference_cnn --batch 16384 || exit 1
