#!/bin/bash
# round-4 GPU step an: the cube kernel's slow first launches (warm_probe)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/warm_probe.py 215 > gpurun_out/r04an_warm.log 2>&1 || exit $?
