#!/bin/bash
# round-5 GPU step k: canonical-path 16-B row stores (V bit 512), CG vector kernels with two 16-B accesses
# per thread (AFEM_CG_VEC2=2) and the two-stage SpMV-partial reduce, C3 SQ / LDS counters
export TMPDIR=/tmp
mkdir -p gpurun_out
AFEM_CUBES_V=880 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "random_numbering or canonical or natural" > gpurun_out/r05k_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py -k "pcg or solve or spmv or pattern or cg" > gpurun_out/r05k_tests_cg.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 215 --rounds 3 --mesh arrays 'default:' 'st16: AFEM_CUBES_V=880' > gpurun_out/r05k_ab_arrays.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cg_probe.py AFEM_CG_VEC2 1 2 --n 215 --iters 100 --reps 3 > gpurun_out/r05k_cg215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cg_probe.py AFEM_CG_VEC2 1 2 --n 463 --iters 20 --reps 2 > gpurun_out/r05k_cg463.log 2>&1 || exit $?
PASSES="sq lds" bash tools/profile_legs.sh gpurun_out/r05k_prof c3 || exit $?
