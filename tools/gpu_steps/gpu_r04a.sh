#!/bin/bash
# round-4 GPU step: generic functor path probe + its tests + shim + host-view BC + C3 size + distributed MG / 8 ranks
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max /proc/self/status 2>/dev/null | grep -E "^[0-9]|max|Cpus_allowed_list" > gpurun_out/r04a_cpu.txt; nproc >> gpurun_out/r04a_cpu.txt; echo "OMP=$OMP_NUM_THREADS" >> gpurun_out/r04a_cpu.txt
timeout -k 10 400 python -u tools/generic_probe.py 10 215 10 > gpurun_out/r04a_probe.log 2>&1
rc=$?
echo "probe rc=$rc" >> gpurun_out/r04a_probe.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 900 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_shim.py "tests/test_gpu_boundary.py::test_host_csr_view_apply_bcs_then_solve" "tests/test_gpu_elasticity3d.py::test_c3_full_size_properties" tests/test_gpu_distributed.py "tests/test_gpu_parity.py::test_canonical_lattice_random_numbering" "tests/test_gpu_parity.py::test_random_node_permutation" "tests/test_gpu_parity.py::test_lattice_order_matches_generator_box" > gpurun_out/r04a_tests.log 2>&1
