#!/bin/bash
# C2 bench with the in-tree library and two experimental builds (lib_x, lib_y).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "" "$PWD/socp.jl_amd/lib_x/libsocp.so" "$PWD/socp.jl_amd/lib_y/libsocp.so"; do
  SOCP_AMD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/ab_bench.log 2>&1 || { tail -20 gpurun_out/ab_bench.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1]); print('${lib:-base}', d['value'], d['kernel_ms'])"
done
