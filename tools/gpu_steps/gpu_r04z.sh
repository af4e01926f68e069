#!/bin/bash
# round-4 GPU step z: cube kernel with the carry at 64-row planes (new default): parity, C2 / C4 zs A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube" > gpurun_out/r04z_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 215 40 8 12 16 > gpurun_out/r04z_ab215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 463 12 16 29 48 > gpurun_out/r04z_ab463.log 2>&1 || exit $?
