#!/bin/bash
# round-4 GPU step t: C4 alone, 20 timed assemblies, kernel trace (the stencil
# kernel's mean against the same run's HIP-event median)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04t_c4_stats -o run -- python3 tools/c4_probe.py 463 50 20 > gpurun_out/r04t_c4_stats.log 2>&1 || exit $?
