#!/bin/bash
# round-5 GPU step ay: AMG with the K-cycle on levels 1..k (AFEM_AMG_KCYCLE), unstructured leg's system
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_amg.py \
  > gpurun_out/r05ay_tests.log 2>&1 || exit $?
timeout -k 10 500 python3 -u tools/amg_probe.py 6 1e-8 - AFEM_AMG_KCYCLE=1 AFEM_AMG_KCYCLE=2 AFEM_AMG_KCYCLE=16 \
  AFEM_AMG_KCYCLE=2,AFEM_AMG_GRAPH=1 AFEM_AMG_KCYCLE=16,AFEM_AMG_GRAPH=1 > gpurun_out/r05ay_amg.log 2>&1 || exit $?
