#!/bin/bash
# Outcome test (verbose histograms), then the C2 A/B (default vs lib/sweep).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_outcomes.py -s -q --timeout 200 --timeout-method thread > gpurun_out/pytest_outcomes.log 2>&1 || true
grep -A12 "reference rule" gpurun_out/pytest_outcomes.log; tail -3 gpurun_out/pytest_outcomes.log
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=socp.jl_amd/lib/libsocp.so; else L=socp.jl_amd/lib/$v/libsocp.so; fi
    SOCP_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-ingest > gpurun_out/bench_C2_$v.log 2>&1 || { tail -30 gpurun_out/bench_C2_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_C2_$v.log').read().strip().splitlines()[-1]); print('C2 $v rep $rep: value %.4g  kernel_ms %.3f frac %.4f' % (d['value'], d['kernel_ms'], d['roofline']['frac']))"
  done
done
