#!/bin/bash
# round-5 GPU step z: kernel trace of the AMG-PCG on the unstructured leg's system
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r05z_prof -o run -- python3 -u tools/amg_probe.py 6 1e-8 AFEM_AMG_HOPS0=2,AFEM_AMG_SCALE=1.7 > gpurun_out/r05z.log 2>&1 || exit $?
