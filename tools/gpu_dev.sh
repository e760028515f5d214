#!/bin/bash
# Tuning loop on the GPU box (dev build with the C1/C2 variants only):
# C1/C2 parity tests, bench (no CPU leg), phase stamps.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "trajectory or teacher or outcome or backward or full_size" > gpurun_out/dev_pytest.log 2>&1 || { tail -40 gpurun_out/dev_pytest.log; exit 1; }
tail -2 gpurun_out/dev_pytest.log
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/dev_bench.log 2>&1 || { tail -30 gpurun_out/dev_bench.log; exit 1; }
python -c "import json;d=json.loads([l for l in open('gpurun_out/dev_bench.log') if l.startswith('{')][0]);print('VALUE',d['value'],'kernel_ms',d['kernel_ms'],'frac',d['roofline']['frac'])"
if [ -f socp.jl_amd/lib/libsocp_diag.so ]; then
  timeout -k 10 200 python tools/stamps.py > gpurun_out/dev_stamps.log 2>&1 || { tail -30 gpurun_out/dev_stamps.log; exit 1; }
  cat gpurun_out/dev_stamps.log
fi
