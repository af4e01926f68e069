#!/bin/bash
# round-5 GPU step ap: C3 with one workgroup per CU (3 waves, one per SIMD) against the default two
# (6 waves on 4 SIMDs): does the SIMD sharing set the pace?
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-headline --legs c3 > gpurun_out/r05ap_c3_occ2_$i.json 2>/dev/null || exit $?
  AFEM_ELAST_WG_OCC=1 timeout -k 10 300 python3 -u bench.py --no-headline --legs c3 > gpurun_out/r05ap_c3_occ1_$i.json 2>/dev/null || exit $?
done
