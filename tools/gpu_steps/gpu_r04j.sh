#!/bin/bash
# round-4 GPU step j: the cube kernel (parity tests, C2 / C4 A/B against the strip kernels)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r04j_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r04j_tests.log
timeout -k 10 200 python3 -u tools/cubes_ab.py 215 20 8 16 32 > gpurun_out/r04j_ab215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 463 5 16 32 > gpurun_out/r04j_ab463.log 2>&1 || exit $?
