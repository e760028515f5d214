#!/bin/bash
# SQ counter passes (issue/stall mix) of the C2 solver kernel; one pass per group.
set -e
export TMPDIR=/tmp
O=gpurun_out/sq
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/p1 -o p1 -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ingest > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o p2 -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ingest > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
python3 - <<'PY'
import csv, glob
tot = {}
for f in glob.glob("gpurun_out/sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "socp_small_kernel" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:.6g}")
PY
