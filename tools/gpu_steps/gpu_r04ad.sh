#!/bin/bash
# round-4 GPU step ad: cube kernel with the y-face exchange: parity + A/B against x only
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube" > gpurun_out/r04ad_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 215 40 12 > gpurun_out/r04ad_ab215.log 2>&1 || exit $?
AFEM_CUBES_YEX=0 timeout -k 10 300 python3 -u tools/cubes_ab.py 215 40 12 > gpurun_out/r04ad_ab215_y0.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 463 12 29 > gpurun_out/r04ad_ab463.log 2>&1 || exit $?
