#!/bin/bash
# round-5 GPU step ba: AMG fine level fused (entry, residual into the restriction, exit) -- tests, probe
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_amg.py \
  > gpurun_out/r05ba_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/amg_probe.py 6 1e-8 - AFEM_AMG_SWEEPS=2 AFEM_AMG_GRAPH=1 - > gpurun_out/r05ba_amg.log 2>&1 || exit $?
