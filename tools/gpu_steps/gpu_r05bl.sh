#!/bin/bash
# round-5 GPU step bl: k_cube_unstage with non-temporal line loads (1) / value stores (2) / both (3)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_knobs.py --mesh arrays --rounds 4 'plain: AFEM_UNSTAGE_V=0' 'ntload: AFEM_UNSTAGE_V=1' \
  'ntstore: AFEM_UNSTAGE_V=2' 'both: AFEM_UNSTAGE_V=3' > gpurun_out/r05bl_ab.log 2>&1 || exit $?
