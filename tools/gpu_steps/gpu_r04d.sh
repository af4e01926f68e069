#!/bin/bash
# round-4 GPU step d: multi-rank rehearsals on one GPU over the host transport
# (C5 at 4 ranks, C4 strong at 8 ranks), a C4-only kernel trace, PMC of the C4 CG SpMV
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/c5_dist.py 1 64 5 gpurun_out/r04d_c5_w1.json > gpurun_out/r04d_c5_w1.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/c5_dist.py 4 64 5 gpurun_out/r04d_c5_w4.json > gpurun_out/r04d_c5_w4.log 2>&1 || exit $?
timeout -k 10 500 python3 -u bench.py --gpus 8 --comm host --scaling strong --n 463 --steps 5 --warmup 2 --cg-iters 20 > gpurun_out/r04d_c4_strong8.json 2> gpurun_out/r04d_c4_strong8.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04d_c4_stats -o run -- python3 tools/c4_probe.py > gpurun_out/r04d_c4_stats.log 2>&1 || exit $?
PMC_CMD="tools/c4_probe.py 463 10" PMC_PASSES="wait fetch write" bash tools/profile_pmc.sh gpurun_out/r04d_c4cg_pmc k_spmv_pat
