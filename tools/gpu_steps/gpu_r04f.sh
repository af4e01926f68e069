#!/bin/bash
# round-4 GPU step f: tiled pattern-SpMV order (bitwise test, C4 CG A/B), canonical
# vs general path on random-numbered C2 (A/B + PMC traffic)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread "tests/test_gpu_parity.py::test_pattern_spmv" > gpurun_out/r04f_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/c4_probe.py 463 50 > gpurun_out/r04f_c4_tile.json 2>&1 || exit $?
AFEM_SPMV_TILE=0 timeout -k 10 200 python3 -u tools/c4_probe.py 463 50 > gpurun_out/r04f_c4_notile.json 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/c4_probe.py 463 50 > gpurun_out/r04f_c4_tile2.json 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/arrays_ab.py AFEM_CANON 1 0 215 10 > gpurun_out/r04f_arrays_ab.log 2>&1 || exit $?
PMC_CMD="tools/arrays_ab.py AFEM_CANON 1 0 215 2" PMC_PASSES="wait fetch write inst" bash tools/profile_pmc.sh gpurun_out/r04f_arrays_pmc k_assemble_st
