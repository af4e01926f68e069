#!/bin/bash
# round-4 GPU step e: the canonical stencil's flat-image store (parity + c2_arrays
# leg), the cell-unit kernel's plan knobs A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread "tests/test_gpu_parity.py::test_canonical_lattice_random_numbering" "tests/test_gpu_parity.py::test_random_node_permutation" > gpurun_out/r04e_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --legs c2_arrays --no-cpu-baseline --steps 10 > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || exit $?
timeout -k 10 400 python3 -u tools/generic_ab.py 215 10 - AFEM_FUNCTOR_FY=4 AFEM_FUNCTOR_UNITS=16384 AFEM_FUNCTOR_FY=4,AFEM_FUNCTOR_UNITS=16384 AFEM_FUNCTOR_FX=4,AFEM_FUNCTOR_FY=4 AFEM_FUNCTOR_ZS=40 > gpurun_out/r04e_ab.log 2>&1
