#!/bin/bash
# round-5 GPU step bn: C3 stencil x-run stores non-temporal (a build of libafem with -DAFEM_WG_NT=1) vs the default
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/ab_lib.py arcanefem_amd/libafem.so arcanefem_amd/libafem_wgnt.so 170 20 3 c3 \
  > gpurun_out/r05bn_ab.log 2>&1 || exit $?
