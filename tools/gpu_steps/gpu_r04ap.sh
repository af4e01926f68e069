#!/bin/bash
# round-4 GPU step ap: kernel traces of the settled bench (C2) and of C4 alone, for the stats mean
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04ap_trace -o run -- python3 bench.py --steps 20 --warmup 5 --cg-iters 20 --no-cpu-baseline --no-extras > gpurun_out/r04ap_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04ap_trace_c4 -o run -- python3 tools/c4_probe.py 463 2 8 > gpurun_out/r04ap_trace_c4.log 2>&1 || exit $?
