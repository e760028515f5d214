#!/bin/bash
# SQ counter passes on the C2 solver kernel (each pass its own run).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --steps 1 --warmup 0 --no-cpu --no-ingest --batch 16384"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_F64 --output-format csv -d gpurun_out/sq1 -o s -- $B > gpurun_out/sq1.log 2>&1 || { tail -20 gpurun_out/sq1.log; exit 1; }
python tools/pmc_dump.py gpurun_out/sq1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_MUL_F64 SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/sq2 -o s -- $B > gpurun_out/sq2.log 2>&1 || { tail -20 gpurun_out/sq2.log; exit 1; }
python tools/pmc_dump.py gpurun_out/sq2
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d gpurun_out/sq3 -o s -- $B > gpurun_out/sq3.log 2>&1 || { tail -20 gpurun_out/sq3.log; exit 1; }
python tools/pmc_dump.py gpurun_out/sq3
