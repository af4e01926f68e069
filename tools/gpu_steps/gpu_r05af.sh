#!/bin/bash
# round-5 GPU step af: cube kernel z-segment length at the current default (C2, C4), settled clocks
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_knobs.py --n 215 --rounds 4 'zs8: AFEM_CUBES_ZS=8' 'zs6: AFEM_CUBES_ZS=6' 'zs10: AFEM_CUBES_ZS=10' 'zs12: AFEM_CUBES_ZS=12' 'zs16: AFEM_CUBES_ZS=16' > gpurun_out/r05af_zs215.log 2>&1 || exit $?
timeout -k 10 500 python3 -u tools/ab_knobs.py --n 463 --rounds 3 --reps 8 'zs8: AFEM_CUBES_ZS=8' 'zs12: AFEM_CUBES_ZS=12' 'zs16: AFEM_CUBES_ZS=16' 'zs24: AFEM_CUBES_ZS=24' > gpurun_out/r05af_zs463.log 2>&1 || exit $?
