#!/bin/bash
# A/B of the default library against variant libraries socp.jl_amd/lib/<v>/
# (args): parity subset on the default, then C2 bench lines interleaved twice.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_par.log 2>&1 || { tail -40 gpurun_out/pytest_par.log; exit 1; }
tail -1 gpurun_out/pytest_par.log
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=socp.jl_amd/lib/libsocp.so; else L=socp.jl_amd/lib/$v/libsocp.so; fi
    SOCP_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu > gpurun_out/bench_$v.log 2>&1 || { tail -30 gpurun_out/bench_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_$v.log').read().strip().splitlines()[-1]); print('$v rep $rep: value %.4g  kernel_ms %.3f frac %.4f' % (d['value'], d['kernel_ms'], d['roofline']['frac']))"
  done
done
