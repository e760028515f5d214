"""Print every counter of the solver-kernel dispatches found under a rocprofv3
--pmc output directory: python tools/pmc_dump.py DIR"""
import csv, glob, os, sys
vals = {}
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "socp_small_kernel" in r["Kernel_Name"]:
            k = (r["Dispatch_Id"], r["Counter_Name"])
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
for (d, c), v in sorted(vals.items()):
    print(f"dispatch {d:>4} {c:28s} {v:20.0f}")
