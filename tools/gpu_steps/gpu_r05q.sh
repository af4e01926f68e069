#!/bin/bash
# round-5 GPU step q: the 64-row unit kernel's knobs at C2 -- functor evaluations in flight (UN) and
# the unit count target (AFEM_FUNCTOR_UNITS: z segments per column)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/generic_ab.py 215 10 - - UN=2 UN=3 - AFEM_FUNCTOR_UNITS=8192 AFEM_FUNCTOR_UNITS=32768 AFEM_FUNCTOR_UNITS=24576 - > gpurun_out/r05q_ab.log 2>&1 || exit $?
