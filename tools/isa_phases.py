"""Static instruction mix per marked region of the register kernel.

Build the marked assembly (never a product build):
  hipcc -DSOCP_MARK -S ... inst_q4_p24_m1.hip -o q4m.s
  python tools/isa_phases.py q4m.s
Regions run from one ';@@BEGIN name' marker to the next."""
import collections
import re
import sys

CATS = [
    ("mfma", r"^v_mfma"), ("accvgpr", r"^v_accvgpr"), ("dpp", r"_dpp|row_|quad_perm"), ("permlane", r"^v_permlane"),
    ("readlane", r"^v_readlane|^v_readfirstlane|^v_writelane"), ("fma64", r"^v_fma_f64"), ("mul64", r"^v_mul_f64"),
    ("add64", r"^v_add_f64"), ("trans64", r"^v_(rcp|rsq|sqrt)_f64|^v_div_"), ("cndmask", r"^v_cndmask"),
    ("vmov", r"^v_mov"), ("valu_other", r"^v_"), ("ds", r"^ds_"), ("vmem", r"^(global|buffer|flat|scratch)_"),
    ("salu", r"^s_(?!waitcnt|nop|cbranch|branch|barrier|setprio|sched|memtime|sleep)"), ("wait", r"^s_waitcnt"),
    ("nop", r"^s_nop"), ("branch", r"^s_c?branch"),
]


def main(path):
    region = "prologue"
    counts = collections.defaultdict(collections.Counter)
    order = []
    for line in open(path):
        t = line.strip()
        m = re.match(r";@@BEGIN (.*)", t)
        if m:
            region = m.group(1)
            if region not in order:
                order.append(region)
            continue
        if not t or t.startswith((";", ".", "/")) or t.endswith(":"):
            continue
        op = t.split()[0]
        for cat, pat in CATS:
            if re.search(pat, op if cat != "dpp" else t):
                counts[region][cat] += 1
                break
        counts[region]["total"] += 1
    cols = ["total"] + [c for c, _ in CATS]
    print(f"{'region':28s}" + "".join(f"{c[:8]:>9s}" for c in cols))
    for r in ["prologue"] + order:
        c = counts[r]
        print(f"{r[:28]:28s}" + "".join(f"{c[k]:9d}" for k in cols))
    tot = collections.Counter()
    for c in counts.values():
        tot.update(c)
    print(f"{'TOTAL':28s}" + "".join(f"{tot[k]:9d}" for k in cols))


if __name__ == "__main__":
    main(sys.argv[1])
