#!/bin/bash
# A/B of an experimental libsocp build (socp.jl_amd/lib_x) against the in-tree one:
# C1/C2 parity subset with the experimental library, then both C2 benches.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
X=$PWD/socp.jl_amd/lib_x/libsocp.so
SOCP_AMD_LIB=$X timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "trajectory or teacher or outcome or backward or batch_vs or full_size" > gpurun_out/ab_parity.log 2>&1 || { tail -30 gpurun_out/ab_parity.log; exit 1; }
tail -2 gpurun_out/ab_parity.log
for lib in "" "$X"; do
  SOCP_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/ab_bench.log 2>&1 || { tail -20 gpurun_out/ab_bench.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1]); print('${lib:-base}', d['value'], d['kernel_ms'], d['roofline']['frac'])"
done
