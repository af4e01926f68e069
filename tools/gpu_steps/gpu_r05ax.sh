#!/bin/bash
# round-5 GPU step ax: complete-layer flush with plain (not non-temporal) 16-B value stores
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_knobs.py --rounds 4 'nt16: AFEM_CUBES_V=1904' 'plain16: AFEM_CUBES_V=1872' \
  > gpurun_out/r05ax_ab.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/ab_knobs.py --n 463 --rounds 3 --reps 8 'nt16: AFEM_CUBES_V=1904' \
  'plain16: AFEM_CUBES_V=1872' > gpurun_out/r05ax_ab463.log 2>&1 || exit $?
