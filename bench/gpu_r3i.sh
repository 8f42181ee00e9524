#!/bin/bash
set -o pipefail
O=gpurun_out/r3i; mkdir -p $O
timeout -k 10 90 python bench/ipc_event_probe.py > $O/probe.txt 2>&1; echo "probe rc=$?"; tail -3 $O/probe.txt
timeout -k 10 250 python -u -m pytest "tests/test_ps_gpu.py::test_ps_mode_hip_workers_one_gpu" -x -v --timeout 230 --timeout-method thread > $O/ps1.log 2>&1; rc=$?
tail -5 $O/ps1.log; echo "ps rc=$rc"
