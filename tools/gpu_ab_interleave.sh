#!/bin/bash
# Order-unbiased A/B on C4: the in-tree library and socp.jl_amd/lib_y run
# alternately, 3 times each (a fresh process per run; the first run on a box
# tends to be slower, so single back-to-back pairs are biased).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
Y=$PWD/socp.jl_amd/lib_y/libsocp.so
for rep in 1 2 3; do
  for lib in "" "$Y"; do
    SOCP_AMD_LIB=$lib timeout -k 10 200 python bench.py --config C4 --no-cpu --steps 3 --warmup 1 > gpurun_out/abi.log 2>&1 || { tail -20 gpurun_out/abi.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abi.log').read().strip().splitlines()[-1]); print('${lib:+B }${lib:-A}'.split()[0], round(d['kernel_ms'], 2))"
  done
done
