#!/bin/bash
# A/B like gpu_ab.sh, but the parity subset runs on the FIRST variant library
# (a dev build with the C1/C2 shapes) instead of the default one.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
V1=$1
SOCP_AMD_LIB=socp.jl_amd/lib/$V1/libsocp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fixtures.py tests/test_gpu_dense.py -q -x -m gpu -k "C2 or c2 or trajectory or kkt or fixture or outcome or golden or kats" --timeout 120 --timeout-method thread > gpurun_out/pytest_par.log 2>&1 || { tail -40 gpurun_out/pytest_par.log; exit 1; }
tail -1 gpurun_out/pytest_par.log
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=socp.jl_amd/lib/libsocp.so; else L=socp.jl_amd/lib/$v/libsocp.so; fi
    SOCP_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-ingest > gpurun_out/bench_$v.log 2>&1 || { tail -30 gpurun_out/bench_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_$v.log').read().strip().splitlines()[-1]); print('$v rep $rep: value %.4g  kernel_ms %.3f frac %.4f' % (d['value'], d['kernel_ms'], d['roofline']['frac']))"
  done
done
