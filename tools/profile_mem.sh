#!/bin/bash
# Memory-side counters of the assembly kernel for ablation modes 0 and 1.
OUT=${1:-gpurun_out/pmem}
B="bench.py --steps 6 --warmup 1 --cg-iters 2 --no-cpu-baseline --no-extras"
K='k_assemble_p1'
mkdir -p $OUT
pass() {  # name, counters...
  local name=$1; shift
  echo "pass $name" >> $OUT/progress.log
  timeout -k 5 150 rocprofv3 --pmc "$@" --kernel-include-regex $K -f csv -d $OUT/$name -o run -- python3 $B > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc" >> $OUT/progress.log
  [ $rc -eq 0 ] || exit $rc
}
for m in ${MODES:-0 1}; do
  export AFEM_ASSEMBLY_ABLATION=$m
  pass m$m.ta TA_TA_BUSY_sum GRBM_GUI_ACTIVE
  pass m$m.tas TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
  pass m$m.tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum
  pass m$m.ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
done
echo done >> $OUT/progress.log
