#!/bin/bash
# round-5 GPU step bc: side-leg clock settle -- unstructured / c3 / c2_generic legs at 150 vs 1500 ms settle
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench.py --no-headline --legs unstructured,c3,c2_generic > gpurun_out/r05bc_s150.json 2> gpurun_out/r05bc_s150.err || exit $?
timeout -k 10 400 python3 -u bench.py --no-headline --legs unstructured,c3,c2_generic --settle-ms 1500 > gpurun_out/r05bc_s1500.json 2> gpurun_out/r05bc_s1500.err || exit $?
