#!/bin/bash
# round-5 GPU step o: the unit kernel's 64-row planes compiled in (k_assemble_units<..., SR = 64, ...>:
# no runtime multiply / swizzle per LDS add, 160 VGPRs = 3 waves per SIMD); packed vs 16-B entries
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_shim.py > gpurun_out/r05o_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/generic_ab.py 215 10 - - AFEM_FUNCTOR_PACKED=0 - AFEM_FUNCTOR_PACKED=0 PAD=-1 > gpurun_out/r05o_ab.log 2>&1 || exit $?
