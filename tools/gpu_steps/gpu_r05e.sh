#!/bin/bash
# round-5 GPU step e: cube kernel store variants combined (non-temporal 8-B / 16-B stores, early coordinate loads)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_knobs.py --n 215 --rounds 4 'base:' 'early+nt: AFEM_CUBES_DIAG=48' 'early+nt+st16: AFEM_CUBES_DIAG=112' \
  'nt+st16: AFEM_CUBES_DIAG=96' 'early+st16: AFEM_CUBES_DIAG=80' > gpurun_out/r05e_ab215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 463 --rounds 3 --reps 8 'base:' 'early+nt: AFEM_CUBES_DIAG=48' 'early+nt+st16: AFEM_CUBES_DIAG=112' 'early+st16: AFEM_CUBES_DIAG=80' > gpurun_out/r05e_ab463.log 2>&1 || exit $?
