set -o pipefail
O=gpurun_out/r6s2/bwd_aw2; mkdir -p $O
for i in 1 2; do
timeout -k 10 120 python bench/micro_lenet_bwd_quick.py > $O/micro_new_$i.txt 2>&1; echo "new $(tail -1 $O/micro_new_$i.txt)"
(cd ab_old && timeout -k 10 120 python bench/micro_lenet_bwd_quick.py) > $O/micro_old_$i.txt 2>&1; echo "old $(tail -1 $O/micro_old_$i.txt)"
done
