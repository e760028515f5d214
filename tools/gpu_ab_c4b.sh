#!/bin/bash
# C4 A/B: GPU suite on the default library, then interleaved C4 benches of the
# default library and each variant lib/<v> (args), 2 reps.
set -e
export TMPDIR=/tmp
O=gpurun_out/ab4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --tb=short --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
echo "default: $(tail -1 $O/pytest.log)"
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=socp.jl_amd/lib/libsocp.so; else L=socp.jl_amd/lib/$v/libsocp.so; fi
    SOCP_AMD_LIB=$L timeout -k 10 200 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu --no-ingest > $O/bench_$v.log 2>&1 || { tail -30 $O/bench_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('C4 $v rep $rep: value %.4g  kernel_ms %.3f frac %.4f' % (d['value'], d['kernel_ms'], d['roofline']['frac']))"
  done
done
SOCP_AMD_LIB=socp.jl_amd/lib/libsocp.so timeout -k 10 200 python bench.py --no-cpu --no-ingest > $O/bench_c2.log 2>&1 || { tail -30 $O/bench_c2.log; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c2.log').read().strip().splitlines()[-1]); print('C2 default: value %.4g  kernel_ms %.3f frac %.4f' % (d['value'], d['kernel_ms'], d['roofline']['frac']))"
