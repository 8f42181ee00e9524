#!/bin/bash
# steps-to-99% over several data/init seeds (the threshold crossing is order-sensitive)
OUT=gpurun_out/${1:-accs}; mkdir -p $OUT
for s in 0 1 2 3 4; do
  timeout -k 10 300 python bench/steps_to_acc.py --impl hip --seed $s > $OUT/hip_b128_s$s.log 2>&1 || exit 1
  timeout -k 10 300 python bench/steps_to_acc.py --impl hip --batch 1024 --lr 0.05 --seed $s > $OUT/hip_b1024_s$s.log 2>&1 || exit 1
done
for s in 0 1 2; do
  timeout -k 10 300 python bench/steps_to_acc.py --impl torch --seed $s > $OUT/torch_b128_s$s.log 2>&1 || exit 1
done
for f in $OUT/*.log; do python3 -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$(basename $f)', d['value'], d['seconds'])"; done
