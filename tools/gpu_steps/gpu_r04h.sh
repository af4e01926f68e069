#!/bin/bash
# round-4 GPU step h: local-index-stream general instance (parity + bitwise tests,
# unstructured A/B + PMC), CG setup kernels at C4
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py > gpurun_out/r04h_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/c4_probe.py 463 50 > gpurun_out/r04h_c4.json 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/unstructured_probe.py 6 > gpurun_out/r04h_unstr.log 2>&1 || exit $?
AFEM_ASSEMBLY_LOCAL=0 timeout -k 10 400 python3 -u tools/unstructured_probe.py 6 > gpurun_out/r04h_unstr_nolocal.log 2>&1 || exit $?
PMC_CMD="tools/unstructured_probe.py 6" PMC_PASSES="lds wait inst fetch write" bash tools/profile_pmc.sh gpurun_out/r04h_unstr_pmc k_assemble_strip
