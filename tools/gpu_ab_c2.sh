#!/bin/bash
# C2 A/B: the GPU suite on each variant library lib/<v> (args), then interleaved
# C2 benches of the default library and each variant (3 reps).
set -e
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
for v in "$@"; do
  SOCP_AMD_LIB=socp.jl_amd/lib/$v/libsocp.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --tb=short --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_$v.log | head -20; tail -5 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=socp.jl_amd/lib/libsocp.so; else L=socp.jl_amd/lib/$v/libsocp.so; fi
    SOCP_AMD_LIB=$L timeout -k 10 200 python bench.py --config ${CFG:-C2} --no-cpu --no-ingest > $O/bench_$v.log 2>&1 || { tail -30 $O/bench_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('$v rep $rep: value %.4g  kernel_ms %.3f frac %.4f' % (d['value'], d['kernel_ms'], d['roofline']['frac']))"
  done
done
