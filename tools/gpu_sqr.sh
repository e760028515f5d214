#!/bin/bash
# Rank-update plugin (socp_sqr_*): its GPU tests, the --mode sqr bench line and
# a rocprofv3 kernel-stats pass of the same command.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sqr.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sqr.log 2>&1 || { tail -60 gpurun_out/pytest_sqr.log; exit 1; }
tail -15 gpurun_out/pytest_sqr.log
timeout -k 10 300 python bench.py --mode sqr --steps 10 --warmup 2 > gpurun_out/bench_sqr.log 2>&1 || { tail -30 gpurun_out/bench_sqr.log; exit 1; }
tail -1 gpurun_out/bench_sqr.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sqr -o sqr -- python3 bench.py --mode sqr --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_sqr.log 2>&1 || { tail -30 gpurun_out/prof_sqr.log; exit 1; }
find gpurun_out/prof_sqr -name "*kernel_stats.csv" | head -3
