#!/bin/bash
# round-5 GPU step be: staged canonical path test with a matrix-only (no RHS) assembly
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "staged_canonical or random_numbering" > gpurun_out/r05be_tests.log 2>&1 || exit $?
