#!/bin/bash
# round-4 GPU step am: back-to-back vs synchronised vs bench-step timing of the cube kernel
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/b2b_probe.py 215 30 > gpurun_out/r04am_b2b.log 2>&1 || exit $?
