#!/bin/bash
# round-4 GPU step ah: the cube kernel on random-numbered lattices (canonical maps): parity + c2_arrays leg
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube or canonical or random_node or lattice_order" > gpurun_out/r04ah_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --legs c2_arrays --no-cpu-baseline --steps 10 > gpurun_out/r04ah_bench.json 2> gpurun_out/r04ah_bench.err || exit $?
