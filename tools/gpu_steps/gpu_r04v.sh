#!/bin/bash
# round-4 GPU step v: cube kernel without waits on in-flight loads (branch-free
# adds and stores, staging at the end of the iteration): parity + A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube" > gpurun_out/r04v_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/cubes_ab.py 215 20 8 16 32 > gpurun_out/r04v_ab215.log 2>&1 || exit $?
AFEM_CUBES_STRIDE=49 timeout -k 10 200 python3 -u tools/cubes_ab.py 215 20 8 16 > gpurun_out/r04v_ab215_s49.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 463 6 16 32 > gpurun_out/r04v_ab463.log 2>&1 || exit $?
