#!/bin/bash
# round-4 final state, step r: kernel stats + PMC of the generic cell-unit kernel
# (c2_generic's kernel, four functor evaluations in flight per lane)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04r_gen_stats -o run -- python3 tools/generic_probe.py 4 215 10 > gpurun_out/r04r_gen_stats.log 2>&1 || exit $?
PMC_CMD="tools/generic_probe.py 4 215 3" bash tools/profile_pmc.sh gpurun_out/r04r_gen_pmc k_assemble_units
