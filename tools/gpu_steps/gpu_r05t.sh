#!/bin/bash
# round-5 GPU step t: the algebraic multigrid preconditioner (amg.hip) -- parity on the reference's Gmsh
# meshes, a refined unstructured mesh, row elimination, block-3; the multigrid and boundary tests
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_amg.py > gpurun_out/r05t_amg.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multigrid.py tests/test_gpu_boundary.py > gpurun_out/r05t_tests.log 2>&1 || exit $?
