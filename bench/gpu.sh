#!/bin/bash
# One parametrised GPU runner for gpurun (replaces the per-experiment gpu_*.sh scripts).
#
#   bash bench/gpu.sh OUT STEP [STEP ...]
#
# OUT   directory under gpurun_out/ for every artefact of the call
# STEP  one of
#   tests[:EXPR]        pytest -m gpu (optionally -k EXPR), 900 s limit
#   smoke               __graft_entry__.smoke()
#   bench[:NAME]        python bench.py ARGS (NAME.json; ARGS from $ARGS_<NAME> or none)
#   prof[:NAME]         rocprofv3 kernel trace of a bench config -> NAME/kernels.md
#   pmc[:NAME]          PMC passes (bench/pmc.sh) of a bench config -> NAME/pmc.md
#   py:SCRIPT           python bench/SCRIPT.py (args from $ARGS_SCRIPT) -> SCRIPT.txt, 300 s limit
# Every step runs under its own timeout; the first failure ends the call (no retries).
# Per-step bench arguments: export ARGS_<NAME>="--model reference_cnn --batch 16384" before
# the call (NAME defaults to the step kind).
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for step in "$@"; do
  kind=${step%%:*}; name=${step#*:}; [ "$name" = "$step" ] && name=$kind
  tag=$(printf '%s' "$name" | tr -c 'A-Za-z0-9_' '_')
  args=""
  if [[ "$name" =~ ^[A-Za-z_][A-Za-z0-9_]*$ ]]; then var="ARGS_${name}"; args=${!var}; fi
  case $kind in
    tests)
      sel=(); [ "$name" != "tests" ] && sel=(-k "$name")
      timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu "${sel[@]}" --durations=12 --timeout 240 \
        --timeout-method thread > "$OUT/tests_$tag.log" 2>&1; rc=$?
      tail -n 4 "$OUT/tests_$tag.log"; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 \
        || { cat $OUT/smoke.txt; exit 1; }
      cat $OUT/smoke.txt ;;
    bench)
      timeout -k 10 300 python bench.py $args > $OUT/$name.json 2> $OUT/$name.err \
        || { tail -8 $OUT/$name.err; exit 1; }
      echo "$name $(grep -o '"ms_per_step": [0-9.]*' $OUT/$name.json) $(grep -o '"value": [0-9.]*' $OUT/$name.json)" ;;
    prof)
      bash bench/gpu_prof.sh ${OUT#gpurun_out/}/$name -- --comm_probe 0 $args > /dev/null \
        || { echo "prof $name failed"; exit 1; }
      head -20 $OUT/$name/kernels.md ;;
    pmc)
      bash bench/pmc.sh ${OUT#gpurun_out/}/$name -- $args || exit 1
      python3 bench/pmc_summary.py $OUT/$name $OUT/$name/pmc.md > /dev/null 2>&1; head -30 $OUT/$name/pmc.md ;;
    py)
      timeout -k 10 300 python -u bench/$name.py $args > $OUT/$name.txt 2>&1 || { tail -8 $OUT/$name.txt; exit 1; }
      tail -n 5 $OUT/$name.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu.sh done"
