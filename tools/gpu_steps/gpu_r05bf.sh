#!/bin/bash
# round-5 GPU step bf: pattern SpMV fast 64-row blocks (AFEM_SPMV_FAST=1), first form (row loop per lane) -- 0.733 vs 0.498 ms per C2 iteration
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/cg_probe.py AFEM_SPMV_FAST 0 1 0 1 --n 215 --iters 100 --reps 3 > gpurun_out/r05bf_cg215.log 2>&1 || exit $?
