#!/bin/bash
# round-4 GPU step c: the failures of r04a (shim on 3 subdomains, 8-slab pattern case), the
# new slice-plan tail test, then bench + generic profiles (gpu_r04b.sh)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_shim.py "tests/test_gpu_generic.py::test_unit_kernel_slice_plan_partial_last_piece" "tests/test_gpu_distributed.py::test_distributed_poisson_solve" > gpurun_out/r04c_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r04c_tests.log
case $rc in 124|137|134|139) exit $rc;; esac
bash tools/gpu_steps/gpu_r04b.sh
