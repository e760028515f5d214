#!/bin/bash
# One GPU session: GPU tests, smoke, the default bench line, the explicit-inverse
# line.  Every GPU step has its own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
O=gpurun_out/${ROUND_TAG:-r05}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|error" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
timeout -k 10 300 python bench.py --explicit-inverse --no-cpu --no-ingest > $O/bench_xi.log 2>&1 || { tail -30 $O/bench_xi.log; exit 1; }
tail -1 $O/bench_xi.log | cut -c1-400
