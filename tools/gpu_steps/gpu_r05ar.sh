#!/bin/bash
# round-5 GPU step ar: the staged canonical cube path (V bit 1024) -- parity, A/B on the
# random-numbered C2 arrays, kernel trace of both passes
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "random_numbering or staged_canonical" > gpurun_out/r05ar_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/ab_knobs.py --mesh arrays --rounds 4 'single: AFEM_CUBES_V=880' \
  'staged: AFEM_CUBES_V=1904' > gpurun_out/r05ar_ab.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05ar_prof -o prof -- \
  python3 -u $GRAFT_REPO_ROOT/tools/ab_knobs.py --mesh arrays --rounds 1 'staged: AFEM_CUBES_V=1904' \
  > $GRAFT_REPO_ROOT/gpurun_out/r05ar_prof.log 2>&1 || exit $?
