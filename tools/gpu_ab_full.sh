#!/bin/bash
# Whole GPU suite on the default library, then interleaved benches (config
# $CFG, default C2) of the default library and each variant lib/<v> (args).
set -e
export TMPDIR=/tmp
CFG=${CFG:-C2}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=8 --tb=short --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -40; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=socp.jl_amd/lib/libsocp.so; else L=socp.jl_amd/lib/$v/libsocp.so; fi
    SOCP_AMD_LIB=$L timeout -k 10 200 python bench.py --config $CFG --no-cpu --no-ingest > gpurun_out/bench_${CFG}_$v.log 2>&1 || { tail -30 gpurun_out/bench_${CFG}_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_${CFG}_$v.log').read().strip().splitlines()[-1]); print('$CFG $v rep $rep: value %.4g  kernel_ms %.3f frac %.4f' % (d['value'], d['kernel_ms'], d['roofline']['frac']))"
  done
done
