#!/bin/bash
# Ingest + dense-handle GPU tests, then the default bench line (with the PCIe-inclusive ingest line, no CPU legs).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_dense.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ingest.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_ingest.log | tail -20; tail -60 gpurun_out/pytest_ingest.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/pytest_ingest.log | tail -20
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
