#!/bin/bash
# round-5 GPU step bs: the CG's pattern SpMV (k_spmv_pat) traced + FETCH / WRITE / SQ at C2 and C4
export TMPDIR=/tmp
mkdir -p gpurun_out
PASSES="trace fetch write sq" bash tools/profile_legs.sh gpurun_out/r05bs_legs c2_spmv c4_spmv || exit $?
