#!/bin/bash
# Secondary bench lines: C1 (HBM-bound by the model), C2 under the reference's
# stopping rule (tol=1e-5, maxit=40), each with its rocprofv3 kernel stats.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --config C1 > gpurun_out/bench_c1.log 2>&1 || { tail -20 gpurun_out/bench_c1.log; exit 1; }
tail -1 gpurun_out/bench_c1.log
timeout -k 10 300 python bench.py --mode reference > gpurun_out/bench_ref.log 2>&1 || { tail -20 gpurun_out/bench_ref.log; exit 1; }
tail -1 gpurun_out/bench_ref.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c1 -o c1 -- python bench.py --config C1 --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_c1.log 2>&1 || { tail -20 gpurun_out/prof_c1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ref -o ref -- python bench.py --mode reference --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_ref.log 2>&1 || { tail -20 gpurun_out/prof_ref.log; exit 1; }
find gpurun_out/prof_c1 gpurun_out/prof_ref -name "*kernel_stats.csv"
