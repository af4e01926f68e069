#!/bin/bash
# round-5 GPU step s: elastodynamics with Rayleigh damping and the generalized-alpha scheme
# (one domain and 3 host-transport slabs) against the oracle's loop; the other time-stepping tests
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_elasticity3d.py tests/test_gpu_passmo.py tests/test_gpu_multigrid.py tests/test_gpu_distributed.py -k "elastodynamics or newmark or passmo" > gpurun_out/r05s_tests.log 2>&1 || exit $?
