#!/bin/bash
# round-5 GPU step aa: AMG with the strength mask, 8-lane propagation and the V-cycle as a HIP graph
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_amg.py > gpurun_out/r05aa_amg_tests.log 2>&1 || exit $?
timeout -k 10 900 python3 -u tools/amg_probe.py 6 1e-8 - AFEM_AMG_GRAPH=0 AFEM_AMG_HOPS0=2,AFEM_AMG_SCALE=1.7 AFEM_AMG_HOPS0=2,AFEM_AMG_SCALE=1.7,AFEM_AMG_GRAPH=0 AFEM_AMG_SCALE=1.7 > gpurun_out/r05aa_amg.log 2>&1 || exit $?
