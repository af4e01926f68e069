#!/bin/bash
# round-5 GPU step p: pattern SpMV with the value stream loaded before the column-image barrier
# (AFEM_SPMV_HOIST, default 1), stream SpMV row ranges loaded early; unit kernel 64-row instance
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_distributed.py -k "pcg or solve or spmv or pattern or cg or distributed" > gpurun_out/r05p_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cg_probe.py AFEM_SPMV_HOIST 0 1 0 1 --n 215 --iters 100 --reps 3 > gpurun_out/r05p_cg215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cg_probe.py AFEM_SPMV_HOIST 0 1 --n 463 --iters 20 --reps 2 > gpurun_out/r05p_cg463.log 2>&1 || exit $?
