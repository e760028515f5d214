#!/bin/bash
# Quick dev session: GPU tests, C2 bench (no CPU leg), phase stamps.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 python tools/stamps.py C2 > gpurun_out/stamps.log 2>&1 || { tail -30 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
