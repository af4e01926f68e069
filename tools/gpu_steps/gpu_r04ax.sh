#!/bin/bash
# round-4 GPU step ax: c2_arrays cube path against the canonical stencil path, knob held during the assemblies
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/arrays_ab.py AFEM_ASSEMBLY_CUBES 1 0 215 10 > gpurun_out/r04ax_ab.log 2>&1 || exit $?
