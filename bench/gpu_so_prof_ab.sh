#!/bin/bash
# Same-box interleaved kernel-trace A/B of two builds: A = the in-tree .so, B = abso/base.so,
# profiled A B A B (eager, 5 + 2 steps each).  Usage: bash bench/gpu_so_prof_ab.sh TAG [bench args]
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
SO=$(ls distributed_tensorflow_ibm_mnist_amd/_kernels*.so)
cp $SO abso/new.so
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
use() { cp abso/$1.so $SO; }
p() { timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --graph 0 --phases 0 --eager_steps 0 "$@" > $OUT/prof$tag.log 2>&1 && python3 bench/prof_summary.py $OUT/prof$tag 7 $OUT/k$tag.md > /dev/null; }
use new && tag=A1 p "$@" && use base && tag=B1 p "$@" && use new && tag=A2 p "$@" && use base && tag=B2 p "$@"
rc=$?; use new
python3 - "$OUT" <<'PY'
import re, sys, collections
out = sys.argv[1]
tab = collections.defaultdict(dict)
for tag in ("A1", "B1", "A2", "B2"):
    for l in open(f"{out}/k{tag}.md"):
        m = re.match(r"\| `([^`]*)` \| \d+ \| [0-9.]+ \| ([0-9.]+) \|", l)
        if m: tab[m.group(1)][tag] = float(m.group(2))
        if "total GPU" in l: tab["TOTAL"][tag] = float(re.findall(r"\*\*([0-9.]+)\*\*", l)[0])
rows = sorted(tab.items(), key=lambda kv: -max(kv[1].values()))[:10]
print("| kernel | A1 | B1 | A2 | B2 |")
for k, v in rows:
    print(f"| {k[:70]} | " + " | ".join(f"{v.get(t, 0):.1f}" for t in ("A1", "B1", "A2", "B2")) + " |")
PY
exit $rc
