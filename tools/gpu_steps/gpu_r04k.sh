#!/bin/bash
# round-4 GPU step k: cube kernel after the staging/prefetch changes
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube or slab or bitwise_repro or structured" > gpurun_out/r04k_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/cubes_ab.py 215 20 8 16 > gpurun_out/r04k_ab215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 463 5 16 32 > gpurun_out/r04k_ab463.log 2>&1 || exit $?
