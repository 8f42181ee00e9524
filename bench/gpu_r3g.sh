#!/bin/bash
set -o pipefail
O=gpurun_out/r3g; mkdir -p $O
timeout -k 10 600 python bench/micro_band.py > $O/micro.txt 2>&1; cat $O/micro.txt
