#!/bin/bash
# round-4 GPU step y: cube kernel with the top face carried in registers: parity + A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
AFEM_CUBES_CARRY=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube" > gpurun_out/r04y_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 215 40 12 > gpurun_out/r04y_ab_c0s49.log 2>&1 || exit $?
AFEM_CUBES_CARRY=1 timeout -k 10 300 python3 -u tools/cubes_ab.py 215 40 12 > gpurun_out/r04y_ab_c1s49.log 2>&1 || exit $?
AFEM_CUBES_CARRY=1 AFEM_CUBES_STRIDE=64 timeout -k 10 300 python3 -u tools/cubes_ab.py 215 40 12 > gpurun_out/r04y_ab_c1s64.log 2>&1 || exit $?
