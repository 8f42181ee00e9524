# 3-channel conv1 weight gradient: where the time goes (skip bits), scalar vs packed-pair LRN
set -o pipefail
O=gpurun_out/r6s2/wg3; mkdir -p $O
timeout -k 10 120 python bench/micro_refc1.py --cin 1 > $O/cin1.json 2>/dev/null || exit 1
timeout -k 10 120 python bench/micro_refc1.py --cin 3 > $O/cin3.json 2>/dev/null || exit 1
MNISTX_REFC1_PK3=1 timeout -k 10 120 python bench/micro_refc1.py --cin 3 > $O/cin3_pk.json 2>/dev/null || exit 1
cat $O/cin1.json $O/cin3.json $O/cin3_pk.json
