set -e
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
pmc() {  # name config batch K suffix
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f_$1 -o f -- python3 bench.py --config $2 --steps 1 --warmup 0 --no-cpu --no-ingest > $O/pmc_f_$1.log 2>&1 || { tail -20 $O/pmc_f_$1.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w_$1 -o w -- python3 bench.py --config $2 --steps 1 --warmup 0 --no-cpu --no-ingest > $O/pmc_w_$1.log 2>&1 || { tail -20 $O/pmc_w_$1.log; exit 1; }
  python3 tools/pmc_traffic.py $O/pmc_f_$1 $O/pmc_w_$1 $2 $3 $4 $O/pmc_traffic$5.json
}
pmc c2 C2 65536 8 ""
pmc c4 C4 1024 5 "_c4"
pmc c1 C1 4096 3 "_c1"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/sq1 -o p1 -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ingest > $O/sq1.log 2>&1 || { tail -20 $O/sq1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/sq2 -o p2 -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ingest > $O/sq2.log 2>&1 || { tail -20 $O/sq2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o c4 -- python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu --no-ingest > $O/prof_c4.log 2>&1 || { tail -30 $O/prof_c4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-ingest > $O/prof_c2.log 2>&1 || { tail -30 $O/prof_c2.log; exit 1; }
echo done
