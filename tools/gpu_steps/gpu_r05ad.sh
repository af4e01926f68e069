#!/bin/bash
# round-5 GPU step ad: rocprof evidence for the side legs (c2_generic, c2_arrays, c2_arrays_natural,
# unstructured) -- kernel trace + FETCH_SIZE + WRITE_SIZE; SQ / LDS counters for the unstructured leg
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_legs.sh gpurun_out/r05ad_prof c2_generic c2_arrays c2_arrays_natural unstructured || exit $?
PASSES="sq lds" bash tools/profile_legs.sh gpurun_out/r05ad_prof unstructured || exit $?
