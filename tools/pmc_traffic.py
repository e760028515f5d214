"""HBM traffic per solver launch from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE), corrected as /opt/skills/guides/MI355X_MICROARCH.md prescribes for
gfx950: FETCH_SIZE reports half the bytes of a wide streaming read (x2);
WRITE_SIZE is taken as reported.  Both counters are in KiB.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR CONFIG BATCH FIXED_K OUT.json [KERNEL_SUBSTR]
(KERNEL_SUBSTR: which kernel's dispatches to count; default the solver kernels)
"""
import csv
import glob
import json
import os
import sys


KERNELS = ("socp_small_kernel", "socp_large_kernel")


def per_dispatch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if not any(kn in r["Kernel_Name"] for kn in KERNELS) or r["Counter_Name"] != counter:
                continue
            key = (f, r["Dispatch_Id"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for the solver kernel under {d}")
    return sorted(vals.values())


def main():
    global KERNELS
    fdir, wdir, cfg, batch, fk, out = sys.argv[1:7]
    if len(sys.argv) > 7:
        KERNELS = (sys.argv[7],)
    fetch = per_dispatch(fdir, "FETCH_SIZE")
    write = per_dispatch(wdir, "WRITE_SIZE")
    f_kib = fetch[len(fetch) // 2]
    w_kib = write[len(write) // 2]
    res = {
        "config": cfg, "batch": int(batch), "fixed_k": int(fk), "kernels": list(KERNELS),
        "fetch_size_kib_raw": f_kib, "write_size_kib_raw": w_kib,
        "hbm_read_bytes": 2.0 * f_kib * 1024.0,
        "hbm_write_bytes": w_kib * 1024.0,
        "hbm_bytes_per_launch": 2.0 * f_kib * 1024.0 + w_kib * 1024.0,
        "dispatches": [len(fetch), len(write)],
        "correction": "FETCH_SIZE x2 (gfx950 streaming-read half count), WRITE_SIZE x1; KiB -> bytes",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
