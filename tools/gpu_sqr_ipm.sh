#!/bin/bash
# The rank-update plugin's tests (incl. its batched solve_socp).
set -e
export TMPDIR=/tmp
O=gpurun_out/sqr
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sqr.py -x -q -rA --tb=short --timeout 200 --timeout-method thread > $O/pytest_sqr_ipm.log 2>&1 || { grep -E "passed|failed|Error|assert|HIP " $O/pytest_sqr_ipm.log | tail -40; exit 1; }
grep -E "HIP |passed|failed" $O/pytest_sqr_ipm.log | tail -5
