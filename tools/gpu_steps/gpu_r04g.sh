#!/bin/bash
# round-4 GPU step g: coalesced CG setup kernels (pattern SpMV + flags tests, C4 CG),
# general-slice bank placement (bitwise test, unstructured A/B + PMC)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread "tests/test_gpu_parity.py::test_pattern_spmv" "tests/test_gpu_parity.py::test_general_slice_variants_bitwise" tests/test_gpu_scale.py tests/test_gpu_multigrid.py > gpurun_out/r04g_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/c4_probe.py 463 50 > gpurun_out/r04g_c4.json 2>&1 || exit $?
AFEM_SPMV_TILE=0 timeout -k 10 200 python3 -u tools/c4_probe.py 463 50 > gpurun_out/r04g_c4_notile.json 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/unstructured_probe.py 6 > gpurun_out/r04g_unstr.log 2>&1 || exit $?
AFEM_BANK_PLACE_GENERAL=0 timeout -k 10 400 python3 -u tools/unstructured_probe.py 6 > gpurun_out/r04g_unstr_nobank.log 2>&1 || exit $?
PMC_CMD="tools/unstructured_probe.py 6" PMC_PASSES="lds wait fetch write" bash tools/profile_pmc.sh gpurun_out/r04g_unstr_pmc k_assemble_strip
