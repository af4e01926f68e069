#!/bin/bash
# round-5 GPU step bo: C3 non-temporal x-run stores by default -- block-3 tests, the c3 leg, its trace + PMC
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_elasticity3d.py \
  tests/test_gpu_passmo.py > gpurun_out/r05bo_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --no-headline --legs c3 > gpurun_out/r05bo_bench.log 2>&1 || exit $?
PASSES="trace fetch write" bash tools/profile_legs.sh gpurun_out/r05bo_legs c3 || exit $?
