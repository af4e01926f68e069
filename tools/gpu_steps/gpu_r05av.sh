#!/bin/bash
# round-5 GPU step av: where the cube kernel's time goes now (diagnostic V bits, values wrong except base)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_knobs.py --rounds 4 'base: AFEM_CUBES_V=1904' 'no_value_stores: AFEM_CUBES_V=1905' \
  'one_add_per_cube: AFEM_CUBES_V=1906' 'no_tet_arith: AFEM_CUBES_V=1908' 'no_full_flush: AFEM_CUBES_V=1912' \
  > gpurun_out/r05av_ab.log 2>&1 || exit $?
