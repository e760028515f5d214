#!/bin/bash
# Measurement session (round tag $R, default r06): GPU tests, PMC HBM traffic
# (FETCH_SIZE, WRITE_SIZE, one counter per pass) for C2 / C4 / C1, SQ
# issue/stall counters of the C2 kernel, rocprofv3 kernel stats of each
# config's bench command (the explicit-inverse order too), then the bench
# lines against the fresh traffic files (copied to profiles/ by hand).
set -e
export TMPDIR=/tmp
R=${R:-r06}
O=gpurun_out/${R}m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
pmc() {  # name config batch K suffix
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f_$1 -o f -- python3 bench.py --config $2 --steps 1 --warmup 0 --no-cpu --no-ingest > $O/pmc_f_$1.log 2>&1 || { tail -20 $O/pmc_f_$1.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w_$1 -o w -- python3 bench.py --config $2 --steps 1 --warmup 0 --no-cpu --no-ingest > $O/pmc_w_$1.log 2>&1 || { tail -20 $O/pmc_w_$1.log; exit 1; }
  python3 tools/pmc_traffic.py $O/pmc_f_$1 $O/pmc_w_$1 $2 $3 $4 $O/pmc_traffic$5.json
}
pmc c2 C2 65536 8 ""
pmc c4 C4 1024 5 "_c4"
pmc c1 C1 4096 3 "_c1"
echo "pmc done"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/sq1 -o p1 -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ingest > $O/sq1.log 2>&1 || { tail -20 $O/sq1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/sq2 -o p2 -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ingest > $O/sq2.log 2>&1 || { tail -20 $O/sq2.log; exit 1; }
echo "sq done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-ingest > $O/prof_c2.log 2>&1 || { tail -30 $O/prof_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xi -o xi -- python3 bench.py --explicit-inverse --steps 5 --warmup 2 --no-cpu --no-ingest > $O/prof_xi.log 2>&1 || { tail -30 $O/prof_xi.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o c4 -- python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu --no-ingest > $O/prof_c4.log 2>&1 || { tail -30 $O/prof_c4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c1 -o c1 -- python3 bench.py --config C1 --steps 5 --warmup 2 --no-cpu --no-ingest > $O/prof_c1.log 2>&1 || { tail -30 $O/prof_c1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sqr -o sqr -- python3 bench.py --mode sqr --steps 3 --warmup 1 --no-cpu > $O/prof_sqr.log 2>&1 || { tail -30 $O/prof_sqr.log; exit 1; }
echo "prof done"
timeout -k 10 500 python3 bench.py --traffic-json $O/pmc_traffic.json > $O/bench_c2.log 2>&1 || { tail -30 $O/bench_c2.log; exit 1; }
grep '^{' $O/bench_c2.log | cut -c1-300
timeout -k 10 300 python3 bench.py --explicit-inverse --no-cpu --no-ingest > $O/bench_xi.log 2>&1 || { tail -30 $O/bench_xi.log; exit 1; }
timeout -k 10 400 python3 bench.py --config C4 --steps 3 --warmup 1 --no-ingest --traffic-json $O/pmc_traffic_c4.json > $O/bench_c4.log 2>&1 || { tail -30 $O/bench_c4.log; exit 1; }
timeout -k 10 300 python3 bench.py --config C1 --no-ingest --traffic-json $O/pmc_traffic_c1.json > $O/bench_c1.log 2>&1 || { tail -30 $O/bench_c1.log; exit 1; }
timeout -k 10 400 python3 bench.py --mode reference --no-ingest > $O/bench_refrule.log 2>&1 || { tail -30 $O/bench_refrule.log; exit 1; }
timeout -k 10 400 python3 bench.py --mode sqr --steps 10 --warmup 2 > $O/bench_sqr.log 2>&1 || { tail -30 $O/bench_sqr.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
echo "all done"
