#!/bin/bash
# round-5 GPU step h (f + g, the pool had no box for them): the whole suite with the non-temporal stores, the
# cube default and the strided write-back; cube A/B on the box and the random arrays; lib A/Bs (unstructured:
# strided vs compacted image, nt vs plain; C3: nt vs plain); unstructured LDS-conflict PMC
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05h_tests.log 2>&1
RC=$?
[ $RC -ge 124 ] && exit $RC
AFEM_CUBES_V=496 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube or natural" > gpurun_out/r05h_tests_drows.log 2>&1
RC=$?
[ $RC -ge 124 ] && exit $RC
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 215 --rounds 3 'default:' 'V112: AFEM_CUBES_V=112' 'V0: AFEM_CUBES_V=0' 's49: AFEM_CUBES_STRIDE=49' 'drows: AFEM_CUBES_V=496' > gpurun_out/r05h_ab_box.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 463 --rounds 2 --reps 8 'default:' 's49: AFEM_CUBES_STRIDE=49' 'drows: AFEM_CUBES_V=496' > gpurun_out/r05h_ab_c4.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 215 --rounds 3 --mesh arrays 'default:' 'V112: AFEM_CUBES_V=112' 'V0: AFEM_CUBES_V=0' > gpurun_out/r05h_ab_arrays.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/ab_lib.py arcanefem_amd/libafem.so arcanefem_amd/libafem_wb0.so 5 20 2 unstructured > gpurun_out/r05h_ab_unstr_wb.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/ab_lib.py arcanefem_amd/libafem.so arcanefem_amd/libafem_nt0.so 5 20 2 unstructured > gpurun_out/r05h_ab_unstr_nt.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_lib.py arcanefem_amd/libafem.so arcanefem_amd/libafem_nt0.so 170 15 2 c3 > gpurun_out/r05h_ab_c3_nt.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_lib.py arcanefem_amd/libafem.so arcanefem_amd/libafem_wg0.so 170 15 2 c3 > gpurun_out/r05h_ab_c3_wg.log 2>&1 || exit $?
PASSES="lds" bash tools/profile_legs.sh gpurun_out/r05h_prof unstructured || exit $?
exit $RC
