#!/bin/bash
# round-5 GPU step bm: non-temporal unstage by default -- staged / canonical parity tests, the c2_arrays leg + trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "staged_canonical or random_numbering or canonical" > gpurun_out/r05bm_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --no-headline --legs c2_arrays > gpurun_out/r05bm_bench.log 2>&1 || exit $?
PASSES="trace fetch write" bash tools/profile_legs.sh gpurun_out/r05bm_legs c2_arrays || exit $?
