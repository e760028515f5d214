"""Per-variant SQ counters from a rocprofv3 --pmc run of tools/ab_multi.py
(tuning tool): the solver kernel's dispatches are in library order per round,
so dispatch i belongs to library i mod nlibs.  Prints per problem-iteration
values (problem-iterations = batch x K, fixed-K).
  python tools/sq_variants.py <pmc dir> <batch*K> lib1 lib2 ..."""
import csv
import glob
import sys

d, pits, libs = sys.argv[1], float(sys.argv[2]), sys.argv[3:]
rows = []
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "socp_small_kernel<" in r["Kernel_Name"]]
by = {}
for r in rows:
    by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = by.get(int(r["Dispatch_Id"]), {}).get(
        r["Counter_Name"], 0.0) + float(r["Counter_Value"])
ids = sorted(by)
n = len(libs)
names = sorted({c for v in by.values() for c in v})
print("lib".ljust(34) + "".join(f"{c[3:]:>18s}" for c in names))
for i, lib in enumerate(libs):
    ds = [ids[j] for j in range(i, len(ids), n)]
    if not ds:
        continue
    last = by[ds[-1]]
    print(lib[-34:].ljust(34) + "".join(f"{last.get(c, 0) / pits:18.1f}" for c in names))
