#!/bin/bash
# One GPU session: tests, smoke, bench, phase stamps, rocprofv3 kernel trace.
# Every GPU step has its own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
if [ -f socp.jl_amd/lib/libsocp_diag.so ]; then
  timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || { tail -30 gpurun_out/stamps.log; exit 1; }
  cat gpurun_out/stamps.log
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d gpurun_out/prof -o r01 -- python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*stats*"; python tools/rocpd_summary.py $(find gpurun_out/prof -name "*.db" | head -1) gpurun_out/kernel_stats.csv && head -3 gpurun_out/kernel_stats.csv
