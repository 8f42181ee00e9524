# round-end evidence (two calls): A = full GPU suite, smoke, default bench; B = rocprof / PMC /
# reference CNN (1 and 3 channels) and fp32 benches and micro timings
export ARGS_ref="--model reference_cnn --batch 16384 --steps 30 --warmup 5"
export ARGS_ref3="--model reference_cnn --in_channels 3 --batch 16384 --steps 30 --warmup 5"
export ARGS_f32="--model reference_cnn --batch 16384 --precision fp32 --steps 8 --warmup 3"
export SKIPS=0
case ${2:-A} in
  A) bash bench/gpu.sh ${1:-r5final} tests smoke bench ;;
  B) bash bench/gpu.sh ${1:-r5final} prof pmc bench:ref prof:ref bench:ref3 bench:f32 prof:f32 py:micro_gemm256 py:micro_lenet_bwd ;;
esac
