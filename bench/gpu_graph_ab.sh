#!/bin/bash
# hipGraph replay vs eager stream launches, interleaved same-box A/B:
#   bash bench/gpu_graph_ab.sh TAG [bench args...]
# Prints ms/step of each run (graph=1 / graph=0 alternating, 3 rounds).
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in 1 2 3; do
  for gr in 1 0; do
    timeout -k 10 120 python bench.py --steps 50 --warmup 10 --phases 0 --eager_steps 0 --graph $gr "$@" \
      > $OUT/g${gr}_r$r.log 2>&1 || { echo "run failed (graph=$gr)"; tail -5 $OUT/g${gr}_r$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('graph=%s ms/step %.4f' % (sys.argv[2], d['ms_per_step']))" $OUT/g${gr}_r$r.log $gr
  done
done
