#!/bin/bash
# round-5 GPU step v: the unstructured leg (L-shape-3D refined 6x, 11.5 M DoF) with its system solved by
# the Jacobi-PCG and the AMG-PCG (setup, iterations, times)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py --no-headline --legs unstructured_solve > gpurun_out/r05v_unstructured_solve.json 2> gpurun_out/r05v.err || exit $?
