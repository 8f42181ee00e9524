# round-end evidence in one call: full GPU suite, smoke, default bench + rocprof + PMC,
# reference CNN bf16 bench + rocprof, fp32 bench + rocprof, micro timings
export ARGS_ref="--model reference_cnn --batch 16384 --steps 30 --warmup 5"
export ARGS_f32="--model reference_cnn --batch 16384 --precision fp32 --steps 8 --warmup 3"
bash bench/gpu.sh ${1:-r4final} tests smoke bench prof pmc bench:ref prof:ref bench:f32 prof:f32 py:micro_refc1 py:micro_lenet_bwd
