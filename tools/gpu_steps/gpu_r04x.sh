#!/bin/bash
# round-4 GPU step x: cube kernel (49-row planes) steady state: 60 interleaved reps, zs 4/8/12
export TMPDIR=/tmp
mkdir -p gpurun_out
AFEM_CUBES_STRIDE=49 timeout -k 10 300 python3 -u tools/cubes_ab.py 215 60 4 8 12 > gpurun_out/r04x_ab215_s49.log 2>&1 || exit $?
AFEM_CUBES_STRIDE=49 timeout -k 10 300 python3 -u tools/cubes_ab.py 463 12 24 32 48 > gpurun_out/r04x_ab463_s49.log 2>&1 || exit $?
