#!/bin/bash
# A/B of an experimental libsocp build (socp.jl_amd/lib_x) on the blocked kernel:
# its parity tests with the experimental library, then both C4 benches.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
X=$PWD/socp.jl_amd/lib_x/libsocp.so
SOCP_AMD_LIB=$X timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_large.log 2>&1 || { tail -30 gpurun_out/ab_large.log; exit 1; }
tail -2 gpurun_out/ab_large.log
for lib in "" "$X"; do
  SOCP_AMD_LIB=$lib timeout -k 10 200 python bench.py --config C4 --no-cpu --steps 3 --warmup 1 > gpurun_out/ab_bench4.log 2>&1 || { tail -20 gpurun_out/ab_bench4.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab_bench4.log').read().strip().splitlines()[-1]); print('${lib:-base}', d['value'], d['kernel_ms'], d['roofline']['frac'])"
done
