#!/bin/bash
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_outcomes.py -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_outcomes.log 2>&1 || { tail -60 gpurun_out/pytest_outcomes.log; exit 1; }
grep -E "PASS|FAIL|reference|structured|hip " gpurun_out/pytest_outcomes.log | tail -20
