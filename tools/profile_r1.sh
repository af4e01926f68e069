#!/bin/bash
# rocprofv3 collection for the assembly kernel (run on the GPU box).
# 1) kernel trace + stats of a normal bench run; 2..5) separate --pmc passes
# (SQ timing, FETCH_SIZE, WRITE_SIZE, LDS) restricted to the assembly kernel.
# Counters are never combined with any other trace; every pass has its own
# time limit and the script stops at the first failure.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
K=${2:-k_assemble_st}
B=${B:-"bench.py --steps 10 --warmup 2 --cg-iters 20 --no-cpu-baseline --no-extras"}
mkdir -p $OUT
timeout -k 5 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
timeout -k 5 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex $K -f csv -d $OUT/pmc_sq -o run -- python3 $B > $OUT/pmc_sq.log 2>&1
timeout -k 5 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K -f csv -d $OUT/pmc_fetch -o run -- python3 $B > $OUT/pmc_fetch.log 2>&1
timeout -k 5 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $K -f csv -d $OUT/pmc_write -o run -- python3 $B > $OUT/pmc_write.log 2>&1
timeout -k 5 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex $K -f csv -d $OUT/pmc_lds -o run -- python3 $B > $OUT/pmc_lds.log 2>&1
echo profile-done
