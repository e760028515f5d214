#!/bin/bash
# Instruction-cache counters of the C2 solver kernel for the default library
# and variant libraries socp.jl_amd/lib/<v>/ (args).  One short pass each.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*" gpurun_out/pmc_list.txt | sort -u | tr '\n' ' ' ; echo
for v in default "$@"; do
  if [ "$v" = default ]; then L=socp.jl_amd/lib/libsocp.so; else L=socp.jl_amd/lib/$v/libsocp.so; fi
  export SOCP_AMD_LIB=$L
  timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/ic1_$v -o s -- python3 bench.py --steps 1 --warmup 0 --no-cpu --batch 16384 > gpurun_out/ic1_$v.log 2>&1 || { tail -20 gpurun_out/ic1_$v.log; exit 1; }
  echo "== $v"; python3 tools/pmc_dump.py gpurun_out/ic1_$v
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d gpurun_out/ic2_$v -o s -- python3 bench.py --steps 1 --warmup 0 --no-cpu --batch 16384 > gpurun_out/ic2_$v.log 2>&1 || { tail -20 gpurun_out/ic2_$v.log; exit 1; }
  python3 tools/pmc_dump.py gpurun_out/ic2_$v
done
