#!/bin/bash
# round-5 GPU step bp: pattern SpMV with the value stream non-temporal (AFEM_SPMV_NTV=1) -- CG A/B at C2 and C4
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/cg_probe.py AFEM_SPMV_NTV 0 1 0 1 --n 215 --iters 100 --reps 3 > gpurun_out/r05bp_cg215.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/cg_probe.py AFEM_SPMV_NTV 0 1 0 1 --n 463 --iters 30 --reps 2 > gpurun_out/r05bp_cg463.log 2>&1 || exit $?
