#!/bin/bash
# round-5 GPU step at: the staged canonical path as the default -- cube / canonical parity tests,
# the c2_arrays bench leg, its trace + FETCH / WRITE passes (both kernels)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "cube or canonical or random or lattice or natural" > gpurun_out/r05at_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --no-headline --legs c2_arrays > gpurun_out/r05at_bench.log 2>&1 || exit $?
PASSES="trace fetch write sq" bash tools/profile_legs.sh gpurun_out/r05at_legs c2_arrays || exit $?
