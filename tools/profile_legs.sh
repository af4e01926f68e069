#!/bin/bash
# rocprofv3 evidence for bench.py's legs, one leg per process (the kernels of
# C2, C4 and c2_arrays_natural share one instance name, so each leg is traced
# alone).  Per leg: a kernel trace + stats of the leg's own bench command, then
# separate --pmc passes (FETCH_SIZE; WRITE_SIZE; optional SQ / LDS groups),
# each under its own time limit; the script stops at the first failure.
#   tools/profile_legs.sh <out_dir> <leg> [<leg> ...]
# legs: c2 (the headline command), c4, c2_spmv / c4_spmv (their CG's pattern SpMV), c3, c2_generic, c2_arrays,
# c2_arrays_natural, unstructured, generic_unstructured.  PASSES (env): pass names to run (default
# "trace fetch write").  Summarise with tools/collect_leg.py.
export TMPDIR=/tmp
OUT=$1
shift
PASSES=${PASSES:-"trace fetch write"}
mkdir -p $OUT
for LEG in "$@"; do
  case $LEG in
    c2) B="bench.py --no-extras --no-cpu-baseline --cg-iters 20"; K="k_assemble_cubes" ;;
    c4) B="bench.py --no-headline --legs c4"; K="k_assemble_cubes" ;;
    c2_spmv) B="bench.py --no-extras --no-cpu-baseline --cg-iters 20"; K="k_spmv_pat" ;;
    c4_spmv) B="bench.py --no-headline --legs c4"; K="k_spmv_pat" ;;
    c3) B="bench.py --no-headline --legs c3"; K="k_assemble_elast" ;;
    c2_generic) B="bench.py --no-headline --legs c2_generic"; K="k_assemble_units" ;;
    c2_arrays) B="bench.py --no-headline --legs c2_arrays"; K="k_assemble_cubes|k_cube_unstage" ;;
    c2_arrays_natural) B="bench.py --no-headline --legs c2_arrays_natural"; K="k_assemble_cubes" ;;
    unstructured) B="bench.py --no-headline --legs unstructured"; K="k_assemble_strip" ;;
    generic_unstructured) B="bench.py --no-headline --legs generic_unstructured"; K="k_assemble_units" ;;
    *) echo "unknown leg $LEG"; exit 2 ;;
  esac
  D=$OUT/$LEG
  mkdir -p $D
  for P in $PASSES; do
    echo "$LEG $P start $(date +%T)" >> $OUT/progress.log
    case $P in
      # the trace runs a 1.5-s settle: its mean over every dispatch of the process (the first ones run at
      # ramping clocks) then matches the bench's settled median (bench.py settle())
      trace) timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/trace -o run -- python3 $B --settle-ms ${TRACE_SETTLE_MS:-1500} > $D/trace.log 2>&1 ;;
      fetch) timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -f csv -d $D/fetch -o run -- python3 $B --settle-ms 0 > $D/fetch.log 2>&1 ;;
      write) timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -f csv -d $D/write -o run -- python3 $B --settle-ms 0 > $D/write.log 2>&1 ;;
      sq) timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-include-regex "$K" -f csv -d $D/sq -o run -- python3 $B --settle-ms 0 > $D/sq.log 2>&1 ;;
      lds) timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex "$K" -f csv -d $D/lds -o run -- python3 $B --settle-ms 0 > $D/lds.log 2>&1 ;;
      *) echo "unknown pass $P"; exit 2 ;;
    esac
    RC=$?
    echo "$LEG $P rc=$RC $(date +%T)" >> $OUT/progress.log
    [ $RC -eq 0 ] || exit $RC
  done
done
echo profile-legs-done >> $OUT/progress.log
