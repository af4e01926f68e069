#!/bin/bash
# thin-box parity of the boundary-aware order
export TMPDIR=/tmp
tools/gpu_steps.sh "300:pytest:python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -k 'thin or edge or stencil or uniform or structured'"
