#!/bin/bash
# round-4 GPU step l: PMC of the cube kernel vs the stencil kernel on C2
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_CMD="tools/cubes_ab.py 215 3 16" PMC_PASSES="inst lds wait wlds fetch write" bash tools/profile_pmc.sh gpurun_out/r04l_pmc "k_assemble_cubes|k_assemble_stencil"
