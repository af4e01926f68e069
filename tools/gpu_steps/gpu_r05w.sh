#!/bin/bash
# round-5 GPU step w: AMG level sizes and variants on the unstructured leg's system (6x refined L-shape)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/amg_probe.py 6 1e-8 - AFEM_AMG_THETA=0.0 AFEM_AMG_THETA=0.25 AFEM_AMG_HOPS=2 > gpurun_out/r05w_amg.log 2>&1 || exit $?
