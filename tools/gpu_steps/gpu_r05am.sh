#!/bin/bash
# round-5 GPU step am: pattern SpMV with 128- and 64-row blocks (AFEM_SPMV_BS: less LDS per block) vs 256
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/cg_probe.py AFEM_SPMV_BS 256 128 64 256 128 64 --n 215 --iters 100 --reps 3 > gpurun_out/r05am_cg215.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/cg_probe.py AFEM_SPMV_BS 256 128 64 --n 463 --iters 20 --reps 2 > gpurun_out/r05am_cg463.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "pattern or pcg" > gpurun_out/r05am_tests.log 2>&1 || exit $?
