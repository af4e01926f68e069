#!/bin/bash
# round-4 GPU step ak: cube kernel with wave-scope LDS ordering instead of __syncthreads: parity + A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube" > gpurun_out/r04ak_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 215 40 12 > gpurun_out/r04ak_ab215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 463 12 29 > gpurun_out/r04ak_ab463.log 2>&1 || exit $?
