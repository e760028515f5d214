#!/bin/bash
# C2 A/B of knob variants lib/<v> (args): parity + fixture tests on each, then
# interleaved C2 benches (3 reps).
set -e
export TMPDIR=/tmp
O=gpurun_out/ab6
mkdir -p $O
for v in "$@"; do
  SOCP_AMD_LIB=socp.jl_amd/lib/$v/libsocp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fixtures.py tests/test_gpu_outcomes.py -m gpu -q -x --tb=short --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_$v.log | head -20; tail -5 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=socp.jl_amd/lib/libsocp.so; else L=socp.jl_amd/lib/$v/libsocp.so; fi
    SOCP_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-ingest > $O/bench_$v.log 2>&1 || { tail -30 $O/bench_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('C2 $v rep $rep: value %.4g  kernel_ms %.3f frac %.4f' % (d['value'], d['kernel_ms'], d['roofline']['frac']))"
  done
done
