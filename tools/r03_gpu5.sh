#!/bin/bash
# non-temporal value streams (SpMV loads / stencil stores) A/B + SpMV PMC
export TMPDIR=/tmp
B="bench.py --no-extras --no-cpu-baseline"
P="--kernel-include-regex k_spmv_pat -f csv"
tools/gpu_steps.sh \
  "200:base:python $B > gpurun_out/r03_v6_base.json" \
  "200:nt:AFEM_SPMV_NT=1 AFEM_ASSEMBLY_NT=1 python $B > gpurun_out/r03_v6_nt.json" \
  "200:base2:python $B > gpurun_out/r03_v6_base2.json" \
  "200:nt2:AFEM_SPMV_NT=1 AFEM_ASSEMBLY_NT=1 python $B > gpurun_out/r03_v6_nt2.json" \
  "120:pmcsq:timeout -s KILL 110 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS $P -d gpurun_out/r03_spmv/sq -o run -- python3 $B --steps 3" \
  "120:pmcf:timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE $P -d gpurun_out/r03_spmv/fetch -o run -- python3 $B --steps 3" \
  "120:pmcw:timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE $P -d gpurun_out/r03_spmv/write -o run -- python3 $B --steps 3"
