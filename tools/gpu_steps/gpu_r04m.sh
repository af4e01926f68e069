#!/bin/bash
# round-4 GPU step m: cube kernel A/B (+ inst / wait PMC)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube or slab or bitwise_repro or structured" > gpurun_out/r04m_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/cubes_ab.py 215 20 8 16 32 > gpurun_out/r04m_ab215.log 2>&1 || exit $?
PMC_CMD="tools/cubes_ab.py 215 3 16" PMC_PASSES="inst wait" bash tools/profile_pmc.sh gpurun_out/r04m_pmc "k_assemble_cubes"
