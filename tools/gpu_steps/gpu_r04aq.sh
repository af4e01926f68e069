#!/bin/bash
# round-4 GPU step aq: z-segment sweep of the cube kernel at settled clocks
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/zs_sweep.py 215 10 4 8 10 12 13 14 16 20 > gpurun_out/r04aq_zs215.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/zs_sweep.py 463 4 3 16 24 29 36 48 64 > gpurun_out/r04aq_zs463.log 2>&1 || exit $?
