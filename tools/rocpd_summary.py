"""Kernel summary (name, calls, total/avg/min/max ns, resources) from a rocprofv3
rocpd SQLite database: python tools/rocpd_summary.py DB [OUT.csv]."""
import csv, sqlite3, sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute(
    "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
    "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_size), max(scratch_size), "
    "max(grid_x), max(workgroup_x) from kernels group by name order by sum(duration) desc").fetchall()
hdr = ["kernel", "calls", "total_ns", "avg_ns", "min_ns", "max_ns", "vgpr", "agpr", "sgpr", "lds_bytes",
       "scratch_bytes", "grid_x", "workgroup_x"]
out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
w = csv.writer(out)
w.writerow(hdr)
for r in rows:
    w.writerow([r[0][:120]] + list(r[1:]))
