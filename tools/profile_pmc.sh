#!/bin/bash
# PMC passes of one kernel of bench.py (separate rocprofv3 runs, each with its
# own time limit; progress in $OUT/progress.log).  Usage:
#   tools/profile_pmc.sh [out_dir] [kernel_regex]
# Summarise with: python tools/pmc_summary.py <out_dir> <kernel_regex>
OUT=${1:-gpurun_out/pmc}
K=${2:-k_assemble_p1}
# PMC_CMD: the python program + arguments to profile (default: a short bench run)
B=${PMC_CMD:-"bench.py --steps 6 --warmup 1 --cg-iters 2 --no-cpu-baseline --no-extras"}
export TMPDIR=/tmp
mkdir -p $OUT
# PMC_PASSES: the pass names to run (default: all)
pass() {  # name, counters...
  local name=$1; shift
  if [ -n "$PMC_PASSES" ] && [[ " $PMC_PASSES " != *" $name "* ]]; then return 0; fi
  echo "pass $name" >> $OUT/progress.log
  timeout -k 5 150 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -f csv -d $OUT/$name -o run -- python3 $B > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc" >> $OUT/progress.log
  [ $rc -eq 0 ] || exit $rc
}
pass inst SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU
pass wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES
pass wlds SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
pass ta TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum
pass fetch FETCH_SIZE
pass write WRITE_SIZE
echo done >> $OUT/progress.log
