"""Summarise rocprofv3 --pmc SQ counter CSVs for one kernel into the
profiles/rNN_sq_counters_c2.txt format.

usage: python3 tools/sq_summary.py KERNEL_SUBSTR PROBLEM_ITERS TITLE csv [csv ...]
PROBLEM_ITERS = problems x iterations of the profiled launch (C2: 65536 x 8).
"""
import csv
import sys
from collections import defaultdict

sub, pits, title, files = sys.argv[1], float(sys.argv[2]), sys.argv[3], sys.argv[4:]
v = defaultdict(float)
for f in files:
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            v[r["Counter_Name"]] += float(r["Counter_Value"])
print(f"# {title}")
print("# SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles; "
      "SQ_VALU_MFMA_BUSY_CYCLES in cycles (MI355X_MICROARCH.md)")
for k in sorted(v):
    print(f"{k:28s} {v[k]:.6g}")
wc = v["SQ_WAVE_CYCLES"]
waves = v.get("SQ_WAVES", 0) or 1
per = lambda name: v[name] / pits
print(f"# per problem-iteration: MFMA {per('SQ_INSTS_MFMA'):.0f}, VALU {per('SQ_INSTS_VALU'):.0f}, "
      f"SALU {per('SQ_INSTS_SALU'):.0f}, LDS {per('SQ_INSTS_LDS'):.0f} instructions; "
      f"wave cycles {4 * wc / pits:.0f}")
print(f"# fractions of wave cycles: active {v['SQ_ACTIVE_INST_ANY'] / wc:.3f} "
      f"(VALU {v['SQ_ACTIVE_INST_VALU'] / wc:.3f}), wait_any {v['SQ_WAIT_ANY'] / wc:.3f}, "
      f"wait_inst_any {v['SQ_WAIT_INST_ANY'] / wc:.3f}; "
      f"MFMA busy {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * wc) * waves / waves:.3f}")
