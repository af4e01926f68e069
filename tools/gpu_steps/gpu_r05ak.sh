#!/bin/bash
# round-5 GPU step ak: C4 CG with the two-stage reduce of the SpMV partials on / off (one process)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/cg_probe.py AFEM_REDUCE_2STAGE 1 0 --n 463 --iters 20 --reps 3 > gpurun_out/r05ak_cg463.log 2>&1 || exit $?
