#!/bin/bash
# GPU suite on the default library (staged C4 SYRK), C4 A/B vs lib/st0 (the
# per-block SYRK), then C2 A/B of scheduler-strategy variants lib/ilp, lib/bias0.
set -e
export TMPDIR=/tmp
O=gpurun_out/ab5
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --tb=short --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
echo "default: $(tail -1 $O/pytest.log)"
for rep in 1 2; do
  for v in default st0; do
    if [ "$v" = default ]; then L=socp.jl_amd/lib/libsocp.so; else L=socp.jl_amd/lib/$v/libsocp.so; fi
    SOCP_AMD_LIB=$L timeout -k 10 200 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu --no-ingest > $O/bench4_$v.log 2>&1 || { tail -30 $O/bench4_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench4_$v.log').read().strip().splitlines()[-1]); print('C4 $v rep $rep: value %.4g  kernel_ms %.3f frac %.4f' % (d['value'], d['kernel_ms'], d['roofline']['frac']))"
  done
done
for v in ilp bias0; do
  SOCP_AMD_LIB=socp.jl_amd/lib/$v/libsocp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fixtures.py -m gpu -q -x --tb=short --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_$v.log | head -20; tail -5 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
  for v in default ilp bias0; do
    if [ "$v" = default ]; then L=socp.jl_amd/lib/libsocp.so; else L=socp.jl_amd/lib/$v/libsocp.so; fi
    SOCP_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-ingest > $O/bench2_$v.log 2>&1 || { tail -30 $O/bench2_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench2_$v.log').read().strip().splitlines()[-1]); print('C2 $v rep $rep: value %.4g  kernel_ms %.3f frac %.4f' % (d['value'], d['kernel_ms'], d['roofline']['frac']))"
  done
done
