#!/bin/bash
# Dev session: outcome diagnostics, bench (no CPU, no ingest), fine stamps.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_outcomes.py -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_outcomes.log 2>&1 || { grep -E "vs |hip |PASS|FAIL" gpurun_out/pytest_outcomes.log | tail -20; exit 1; }
grep -E "vs |hip |structured |reference_order |PASS|FAIL" gpurun_out/pytest_outcomes.log | tail -12
timeout -k 10 300 python bench.py --no-cpu --no-ingest > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
timeout -k 10 300 python tools/stamps.py C2 > gpurun_out/stamps.log 2>&1 || { tail -30 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
