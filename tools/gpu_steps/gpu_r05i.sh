#!/bin/bash
# round-5 GPU step i: the strip kernels back to the compacted write-back and plain stores; cube default V=112;
# the cube / canonical parity tests; dummy rows on top of V=112 (box, C4); the generic kernel with / without
# non-temporal flush stores (c2_generic leg, alternating processes)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cube or natural or canonical or random or general" > gpurun_out/r05i_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 215 --rounds 4 'default:' 'drows: AFEM_CUBES_V=368' 'V0: AFEM_CUBES_V=0' > gpurun_out/r05i_ab_box.log 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/ab_knobs.py --n 463 --rounds 2 --reps 8 'default:' 'drows: AFEM_CUBES_V=368' > gpurun_out/r05i_ab_c4.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-headline --legs c2_generic > gpurun_out/r05i_gen_nt_$i.json 2>&1 || exit $?
  AFEM_GENERIC_LIB=examples/libafem_generic_example_nt0.so timeout -k 10 200 python3 -u bench.py --no-headline --legs c2_generic > gpurun_out/r05i_gen_nt0_$i.json 2>&1 || exit $?
done
timeout -k 10 300 python3 -u bench.py --no-headline --legs unstructured,c3 > gpurun_out/r05i_unstr_c3.json 2>&1 || exit $?
