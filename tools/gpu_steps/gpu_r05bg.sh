#!/bin/bash
# round-5 GPU step bg: pattern SpMV fast blocks, the other blocks with batched row loads -- parity, CG A/B at C2 and C4
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "pattern_spmv" > gpurun_out/r05bg_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cg_probe.py AFEM_SPMV_FAST 0 1 0 1 --n 215 --iters 100 --reps 3 > gpurun_out/r05bg_cg215.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/cg_probe.py AFEM_SPMV_FAST 0 1 0 1 --n 463 --iters 30 --reps 2 > gpurun_out/r05bg_cg463.log 2>&1 || exit $?
