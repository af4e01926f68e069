#!/bin/bash
# round-4 GPU step ar: cube kernel with wave-uniform readlanes instead of LDS permutes in the flush: parity + A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube" > gpurun_out/r04ar_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 215 40 13 > gpurun_out/r04ar_ab215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/zs_sweep.py 215 10 4 12 13 > gpurun_out/r04ar_zs215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/cubes_ab.py 463 12 29 > gpurun_out/r04ar_ab463.log 2>&1 || exit $?
