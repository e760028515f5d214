#!/bin/bash
# Blocked-kernel session: its parity tests, then the rest of the GPU suite,
# then C4 and C2 bench lines (no CPU leg).  The first failure ends the script.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/large_pytest.log 2>&1 || { tail -60 gpurun_out/large_pytest.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/large_pytest.log | tail -20
timeout -k 10 300 python bench.py --config C4 --no-cpu --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || { tail -30 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread --deselect tests/test_gpu_large.py > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_c2.log 2>&1 || { tail -30 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log
