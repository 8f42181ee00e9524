# round-end evidence (two calls): A = full GPU suite, smoke, default bench; B = rocprof / PMC /
# reference CNN and fp32 benches and micro timings
export ARGS_ref="--model reference_cnn --batch 16384 --steps 30 --warmup 5"
export ARGS_f32="--model reference_cnn --batch 16384 --precision fp32 --steps 8 --warmup 3"
export SKIPS=0
case ${2:-A} in
  A) bash bench/gpu.sh ${1:-r4final} tests smoke bench ;;
  B) bash bench/gpu.sh ${1:-r4final} prof pmc bench:ref prof:ref bench:f32 prof:f32 py:micro_refc1 py:micro_lenet_bwd ;;
esac
