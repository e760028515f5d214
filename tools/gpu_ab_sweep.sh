#!/bin/bash
# A/B of sweep variants: default lib vs socp.jl_amd/lib/v0 (per-pivot tile factor)
# vs v1 (LDS transposes): quick parity subset, C2 bench and phase stamps each.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_par.log 2>&1 || { tail -40 gpurun_out/pytest_par.log; exit 1; }
tail -1 gpurun_out/pytest_par.log
for v in "" v0 v1; do
  L=socp.jl_amd/lib/${v:+$v/}
  echo "== variant ${v:-default}"
  SOCP_AMD_LIB=${L}libsocp.so timeout -k 10 200 python bench.py --no-cpu > gpurun_out/bench_$v.log 2>&1 || { tail -30 gpurun_out/bench_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$v.log').read().strip().splitlines()[-1]); print('value %.4g  kernel_ms %.3f frac %.4f' % (d['value'], d['kernel_ms'], d['roofline']['frac']))"
  SOCP_AMD_LIB=${L}libsocp_diag.so timeout -k 10 200 python tools/stamps.py C2 > gpurun_out/stamps_$v.log 2>&1 || { tail -30 gpurun_out/stamps_$v.log; exit 1; }
  cat gpurun_out/stamps_$v.log | grep -v amdgpu.ids
done
