#!/bin/bash
# round-4 GPU step: generic functor path probe + its tests + shim + host-view BC test
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/generic_probe.py 10 215 10 > gpurun_out/r04a_probe.log 2>&1
rc=$?
echo "probe rc=$rc" >> gpurun_out/r04a_probe.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_shim.py "tests/test_gpu_boundary.py::test_host_csr_view_apply_bcs_then_solve" > gpurun_out/r04a_tests.log 2>&1
