#!/bin/bash
# round-5 GPU step x: AMG aggregation distance per level, coarse-correction scale, sweeps (unstructured leg system)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/amg_probe.py 6 1e-8 - AFEM_AMG_HOPS0=2 AFEM_AMG_SCALE=1.5 AFEM_AMG_SCALE=1.8 AFEM_AMG_SWEEPS=2 AFEM_AMG_HOPS0=2,AFEM_AMG_SCALE=1.8 AFEM_AMG_THETA=0.0 AFEM_AMG_THETA=0.02 > gpurun_out/r05x_amg.log 2>&1 || exit $?
