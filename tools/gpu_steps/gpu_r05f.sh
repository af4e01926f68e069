#!/bin/bash
# round-5 GPU step f: the new cube default (early loads, 16-B non-temporal stores): parity; A/B on the box and the
# random-numbered arrays (canonical path with non-temporal stores)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube or natural or canonical" > gpurun_out/r05f_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 215 --rounds 3 'default:' 'V112: AFEM_CUBES_V=112' 'V0: AFEM_CUBES_V=0' > gpurun_out/r05f_ab_box.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 215 --rounds 3 --mesh arrays 'default:' 'V112: AFEM_CUBES_V=112' 'V0: AFEM_CUBES_V=0' > gpurun_out/r05f_ab_arrays.log 2>&1 || exit $?
