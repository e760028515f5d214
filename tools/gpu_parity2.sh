#!/bin/bash
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_outcomes.py tests/test_gpu_large.py tests/test_fixtures.py -m gpu -v -s --timeout 240 --timeout-method thread > gpurun_out/pytest_parity2.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_parity2.log | tail -30; tail -40 gpurun_out/pytest_parity2.log; exit 1; }
grep -E "PASS|FAIL|worst|vs " gpurun_out/pytest_parity2.log | tail -30
