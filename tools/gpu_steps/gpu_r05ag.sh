#!/bin/bash
# round-5 GPU step ag: cube kernel z-segment length, second sweep with more rounds (C2, C4)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_knobs.py --n 215 --rounds 8 'zs8: AFEM_CUBES_ZS=8' 'zs12: AFEM_CUBES_ZS=12' 'zs14: AFEM_CUBES_ZS=14' 'zs10: AFEM_CUBES_ZS=10' > gpurun_out/r05ag_zs215.log 2>&1 || exit $?
timeout -k 10 500 python3 -u tools/ab_knobs.py --n 463 --rounds 5 --reps 8 'zs8: AFEM_CUBES_ZS=8' 'zs16: AFEM_CUBES_ZS=16' 'zs20: AFEM_CUBES_ZS=20' 'zs14: AFEM_CUBES_ZS=14' > gpurun_out/r05ag_zs463.log 2>&1 || exit $?
