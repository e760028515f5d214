#!/bin/bash
# Instruction-cache and issue counters of the rank-update setup/solve kernels (--mode sqr).
set -e
export TMPDIR=/tmp
O=gpurun_out/icsqr
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $O/ic -o s -- python3 bench.py --mode sqr --steps 1 --warmup 0 --no-cpu --batch 16384 > $O/ic.log 2>&1 || { tail -20 $O/ic.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $O/sq -o s -- python3 bench.py --mode sqr --steps 1 --warmup 0 --no-cpu --batch 16384 > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float)
for f in glob.glob("gpurun_out/icsqr/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"]
        if "socp_sqr" not in kn:
            continue
        key = ("setup" if "setup" in kn else "solve", r["Counter_Name"])
        tot[key] += float(r["Counter_Value"])
for k in sorted(tot):
    print(f"{k[0]:6s} {k[1]:28s} {tot[k]:.6g}")
PY
