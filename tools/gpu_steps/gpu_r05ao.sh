#!/bin/bash
# round-5 GPU step ao: the CSR-stream SpMV in 64-row blocks -- C2 with the stream kernel (AFEM_SPMV=nopat),
# the unstructured system's Jacobi / AMG solves, and the SpMV / CG / distributed / AMG tests
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_distributed.py tests/test_gpu_amg.py tests/test_gpu_multigrid.py -k "pcg or solve or spmv or pattern or cg or distributed or amg or multigrid or rccl" > gpurun_out/r05ao_tests.log 2>&1 || exit $?
AFEM_SPMV=nopat timeout -k 10 300 python3 -u tools/cg_probe.py AFEM_SPMV_BS 256 64 256 64 --n 215 --iters 100 --reps 3 > gpurun_out/r05ao_cg215_stream.log 2>&1 || exit $?
timeout -k 10 900 python3 -u tools/amg_probe.py 6 1e-8 - AFEM_SPMV_BS=256 > gpurun_out/r05ao_amg.log 2>&1 || exit $?
