#!/bin/bash
# round-5 GPU step d: cube kernel store / load-placement variants (values must stay bitwise equal)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_knobs.py --n 215 --rounds 4 'base:' 'early: AFEM_CUBES_DIAG=16' 'nt: AFEM_CUBES_DIAG=32' \
  'st16: AFEM_CUBES_DIAG=64' 'early+st16: AFEM_CUBES_DIAG=80' 'early+nt: AFEM_CUBES_DIAG=48' 'early+nostore: AFEM_CUBES_DIAG=17' > gpurun_out/r05d_ab215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 463 --rounds 2 --reps 8 'base:' 'early: AFEM_CUBES_DIAG=16' 'st16: AFEM_CUBES_DIAG=64' 'early+st16: AFEM_CUBES_DIAG=80' > gpurun_out/r05d_ab463.log 2>&1 || exit $?
