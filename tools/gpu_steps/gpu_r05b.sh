#!/bin/bash
# round-5 GPU step b: cube kernel fast flush for complete layers: parity, A/B at C2 and C4; C2 trace retry
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube or natural" > gpurun_out/r05b_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 215 'full:' 'general: AFEM_CUBES_FULL=0' > gpurun_out/r05b_ab215.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 463 --rounds 3 --reps 8 'full:' 'general: AFEM_CUBES_FULL=0' > gpurun_out/r05b_ab463.log 2>&1 || exit $?
PASSES=trace bash tools/profile_legs.sh gpurun_out/r05b_prof c2 || exit $?
