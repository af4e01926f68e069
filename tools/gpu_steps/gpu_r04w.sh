#!/bin/bash
# round-4 GPU step w: cube kernel, 15 accumulator planes, loads after the cubes,
# 3 waves/SIMD by registers: parity (both strides) + A/B of the strides
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube" > gpurun_out/r04w_tests.log 2>&1 || exit $?
AFEM_CUBES_STRIDE=49 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube" > gpurun_out/r04w_tests49.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/cubes_ab.py 215 20 8 16 > gpurun_out/r04w_ab215.log 2>&1 || exit $?
AFEM_CUBES_STRIDE=49 timeout -k 10 200 python3 -u tools/cubes_ab.py 215 20 8 16 32 > gpurun_out/r04w_ab215_s49.log 2>&1 || exit $?
AFEM_CUBES_STRIDE=49 timeout -k 10 300 python3 -u tools/cubes_ab.py 463 6 16 32 > gpurun_out/r04w_ab463_s49.log 2>&1 || exit $?
