#!/bin/bash
# round-4 GPU step b: full bench (all legs), kernel stats + PMC of the generic
# cell-unit kernel (c2_generic's kernel, via tools/generic_probe.py)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04b_gen_stats -o run -- python3 tools/generic_probe.py 4 215 10 > gpurun_out/r04b_gen_stats.log 2>&1 || exit $?
PMC_CMD="tools/generic_probe.py 4 215 3" bash tools/profile_pmc.sh gpurun_out/r04b_gen_pmc k_assemble_units
