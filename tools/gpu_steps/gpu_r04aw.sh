#!/bin/bash
# round-4 GPU step aw: c2_arrays through the cube kernel (canonical maps) against the canonical stencil
# path: A/B, kernel trace and PMC of the cube dispatches
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/arrays_ab.py AFEM_ASSEMBLY_CUBES 1 0 215 10 > gpurun_out/r04aw_ab.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04aw_stats -o run -- python3 tools/arrays_ab.py AFEM_ASSEMBLY_CUBES 1 0 215 10 > gpurun_out/r04aw_stats.log 2>&1 || exit $?
PMC_CMD="tools/arrays_ab.py AFEM_ASSEMBLY_CUBES 1 0 215 3" PMC_PASSES="inst wait fetch write" bash tools/profile_pmc.sh gpurun_out/r04aw_pmc "k_assemble_cubes"
