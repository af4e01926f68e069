#!/bin/bash
# round-5 GPU step ae: regression check against the library of commit 14dc85d (libafem_old.so) --
# CG per iteration at C2 / C4 and the c2_arrays leg, alternating processes
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for L in old new; do
    if [ $L = old ]; then export AFEM_LIB=$PWD/arcanefem_amd/libafem_old.so; else unset AFEM_LIB; fi
    timeout -k 10 200 python3 -u tools/cg_probe.py AFEM_CG_VEC2 1 --n 215 --iters 100 --reps 3 > gpurun_out/r05ae_cg215_${L}_$i.log 2>&1 || exit $?
    timeout -k 10 300 python3 -u bench.py --no-headline --legs c2_arrays > gpurun_out/r05ae_arrays_${L}_$i.json 2>/dev/null || exit $?
  done
done
unset AFEM_LIB
