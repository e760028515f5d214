#!/bin/bash
# Full GPU test suite, then C1 and C2 bench lines without the CPU leg.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for cfg in C1 C2; do
  timeout -k 10 200 python bench.py --config $cfg --no-cpu > gpurun_out/chk_$cfg.log 2>&1 || { tail -20 gpurun_out/chk_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/chk_$cfg.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['kernel_ms'], d['roofline']['frac'])"
done
