set -o pipefail
O=gpurun_out/r6/job5; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_executor_gpu.py -k "head_wgrad_late" tests/test_ps_gpu.py > $O/tests.log 2>&1; rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash bench/ab_micro.sh r6/job5/ref3_ab 2 bench.py --model reference_cnn --in_channels 3 --batch 16384 || exit 1
ENV_A="MNISTX_HEAD_WGRAD_LATE=0" ENV_B="MNISTX_HEAD_WGRAD_LATE=1" bash bench/ab_args.sh r6/job5/order 3 || exit 1
timeout -k 10 500 python -u bench/ps_capacity.py --model reference_cnn --workers 3,7 --transports ipc,shm --updates 1000 > $O/cap_ref.txt 2>&1; rc=$?; grep '^{' $O/cap_ref.txt; [ $rc -eq 0 ] || { tail -5 $O/cap_ref.txt; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --mode ps --model reference_cnn --in_channels 3 --batch 128 --steps 50 --warmup 5 > $O/bench_ref_ps_w3.json 2> $O/bench_ref_ps_w3.err; rc=$?; cat $O/bench_ref_ps_w3.json; [ $rc -eq 0 ] || { tail -5 $O/bench_ref_ps_w3.err; exit $rc; }
echo job5 done
