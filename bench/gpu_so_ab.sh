#!/bin/bash
# Same-box A/B of two builds of the kernel extension: A = the in-tree .so, B = abso/base.so
# (interleaved A B A B), plus a kernel trace of each.  Usage: bash bench/gpu_so_ab.sh TAG [bench args]
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
SO=$(ls distributed_tensorflow_ibm_mnist_amd/_kernels*.so)
cp $SO abso/new.so
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
use() { cp abso/$1.so $SO; }
b() { timeout -k 10 200 python bench.py --steps 30 --warmup 5 --phases 0 "$@" > $OUT/$tag.log 2>&1 && echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log)"; }
use new && tag=A1 b "$@" && use base && tag=B1 b "$@" && use new && tag=A2 b "$@" && use base && tag=B2 b "$@" && \
use new && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/profA -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --graph 0 --phases 0 "$@" > $OUT/profA.log 2>&1 && \
use base && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/profB -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --graph 0 --phases 0 "$@" > $OUT/profB.log 2>&1
rc=$?; use new; exit $rc
