#!/bin/bash
# round-5 GPU step aw: the complete-layer flush storing rows from registers (V bit 2048) -- parity, A/B
# against the LDS image; no-store diagnostics of both
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "direct_row_stores or face_sharing or matches_oracle" > gpurun_out/r05aw_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/ab_knobs.py --rounds 4 'image: AFEM_CUBES_V=1904' 'direct: AFEM_CUBES_V=3952' \
  'image_nostore: AFEM_CUBES_V=1905' 'direct_nostore: AFEM_CUBES_V=3953' > gpurun_out/r05aw_ab.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/ab_knobs.py --n 463 --rounds 3 --reps 8 'image: AFEM_CUBES_V=1904' \
  'direct: AFEM_CUBES_V=3952' > gpurun_out/r05aw_ab463.log 2>&1 || exit $?
