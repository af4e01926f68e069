#!/bin/bash
# round-5 GPU step ah: cube kernel z-segment length against the default formula (n/16: C2 13, C4 29)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/ab_knobs.py --n 463 --rounds 5 --reps 8 'default:' 'zs16: AFEM_CUBES_ZS=16' 'zs29: AFEM_CUBES_ZS=29' 'zs36: AFEM_CUBES_ZS=36' > gpurun_out/r05ah_zs463.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/ab_knobs.py --n 215 --rounds 8 'default:' 'zs12: AFEM_CUBES_ZS=12' 'zs16: AFEM_CUBES_ZS=16' > gpurun_out/r05ah_zs215.log 2>&1 || exit $?
