#!/bin/bash
# round-5 GPU step g: non-temporal assembly stores and the strided write-back image of the strip kernels:
# the whole suite, lib A/Bs (unstructured, C3), unstructured LDS-conflict PMC
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05g_tests.log 2>&1
RC=$?
[ $RC -ge 124 ] && exit $RC
timeout -k 10 400 python3 -u tools/ab_lib.py arcanefem_amd/libafem.so arcanefem_amd/libafem_wb0.so 5 20 2 unstructured > gpurun_out/r05g_ab_unstr_wb.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/ab_lib.py arcanefem_amd/libafem.so arcanefem_amd/libafem_nt0.so 5 20 2 unstructured > gpurun_out/r05g_ab_unstr_nt.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_lib.py arcanefem_amd/libafem.so arcanefem_amd/libafem_nt0.so 170 15 2 c3 > gpurun_out/r05g_ab_c3_nt.log 2>&1 || exit $?
PASSES="lds" bash tools/profile_legs.sh gpurun_out/r05g_prof unstructured || exit $?
exit $RC
