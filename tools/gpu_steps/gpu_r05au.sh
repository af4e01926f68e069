#!/bin/bash
# round-5 GPU step au: unstructured leg, order of the compact / big general lists (AFEM_ASSEMBLY_BIG)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/unstructured_ab.py --levels 6 'side: AFEM_ASSEMBLY_BIG=0' \
  'big_first: AFEM_ASSEMBLY_BIG=1' 'compact_first: AFEM_ASSEMBLY_BIG=2' > gpurun_out/r05au_ab.log 2>&1 || exit $?
