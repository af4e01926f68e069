#!/bin/bash
# round-5 GPU step aq: the 64-row pattern SpMV held to 6 / 8 waves per SIMD (VGPR caps, spills) vs 5
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/cg_probe.py AFEM_SPMV_WAVES 0 6 8 0 6 8 --n 215 --iters 100 --reps 3 > gpurun_out/r05aq_cg215.log 2>&1 || exit $?
