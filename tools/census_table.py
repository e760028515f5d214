"""VALU census of the C2 solver kernel per problem-iteration (tuning tool):
the product build and the SOCP_KO knock-out builds, from the two SQ passes of
tools/sq_variants.py (per-kind VALU counters) and tools/ab_multi.py's times.
Kinds: f64 = FMA + MUL + ADD + TRANS f64 VALU; int = INT32 + INT64 VALU; mfma;
other = VALU - f64 - int - mfma (data movement: v_accvgpr_read/write, DPP /
permlane / readlane moves, v_mov, v_cndmask, ...).  Per phase: the product
minus the knock-out (only knock-outs that keep every problem at maxit, i.e.
the same control flow, are differenced).
  python tools/census_table.py sqa.txt sqb.txt ab.log"""
import re
import sys

KO = {"2": "residuals (solver.jl:109-118)", "16": "  of which G x + s - h", "32": "  of which G'z",
      "128": "  of which A'y, A x", "4": "compute_U", "65536": "H = X'X with X = W^-1 G (SYRK)",
      "8": "factor of S (16 x 16 tile)", "256": "the four triangular solves", "2048": "S^-1 products (solves)",
      "4096": "compute_scaling", "32768": "the corrector's right-hand side", "131072": "Cholesky of H (+ Z, S)",
      "512": "G'v in the solves", "1024": "G v in the solves", "8192": "solve head", "16384": "solve tail"}


def table(path):
    rows = {}
    lines = open(path).read().splitlines()
    cols = [h.strip() for h in re.split(r"(?=INSTS_|ACTIVE_|WAIT_|WAVE_)", lines[0][3:]) if h.strip()]
    for ln in lines[1:]:
        parts = ln.split()
        lib, vals = parts[0], [float(x) for x in parts[1:]]
        m = re.search(r"v_(\w+)/libsocp", lib)
        rows[m.group(1)] = dict(zip(cols, vals))
    return rows


def main(a, b, ab):
    A, B = table(a), table(b)
    times, ok = {}, {}
    for ln in open(ab):
        m = re.search(r"v_(\w+)/libsocp.so: median ([\d.]+) ms.*status \[(\d+), (\d+),", ln)
        if m:
            times[m.group(1)] = float(m.group(2))
            ok[m.group(1)] = int(m.group(4)) == 65536
    def kinds(r, s):
        f64 = r["INSTS_VALU_FMA_F64"] + r["INSTS_VALU_MUL_F64"] + r["INSTS_VALU_ADD_F64"] + r["INSTS_VALU_TRANS_F64"]
        it = r["INSTS_VALU_INT32"] + r["INSTS_VALU_INT64"]
        mf = r["INSTS_MFMA"]
        return dict(valu=r["INSTS_VALU"], mfma=mf, f64=f64, int=it, other=r["INSTS_VALU"] - f64 - it - mf,
                    cyc=4 * s["WAVE_CYCLES"], vcyc=4 * s["ACTIVE_INST_VALU"], wait=4 * s["WAIT_ANY"])
    base = kinds(A["base"], B["base"])
    print("C2 solver kernel, per problem-iteration (65,536 problems x K = 8), product build:")
    print(f"  VALU {base['valu']:.0f} = MFMA {base['mfma']:.0f} + f64 arithmetic {base['f64']:.0f} "
          f"(FMA {A['base']['INSTS_VALU_FMA_F64']:.0f}, MUL {A['base']['INSTS_VALU_MUL_F64']:.0f}, "
          f"ADD {A['base']['INSTS_VALU_ADD_F64']:.0f}, TRANS {A['base']['INSTS_VALU_TRANS_F64']:.0f}) + integer "
          f"{base['int']:.0f} + other (moves, selects) {base['other']:.0f}")
    print(f"  wave cycles {base['cyc']:.0f}, VALU-issue cycles {base['vcyc']:.0f}, waitcnt cycles {base['wait']:.0f}, "
          f"kernel {times['base']:.3f} ms")
    print()
    print(f"{'phase removed (SOCP_KO)':44s}{'ms':>7s}{'K cyc':>8s}{'VALU':>7s}{'MFMA':>6s}{'f64':>6s}{'int':>6s}{'other':>7s}{'wait K':>8s}")
    for b_, name in KO.items():
        key = "ko" + b_
        if key not in A:
            continue
        if not ok.get(key):
            print(f"{name[:43]:44s}  (control flow changed: not differenced)")
            continue
        k = kinds(A[key], B[key])
        d = {x: base[x] - k[x] for x in base}
        print(f"{name[:43]:44s}{times['base'] - times[key]:7.2f}{d['cyc'] / 1e3:8.1f}{d['valu']:7.0f}{d['mfma']:6.0f}"
              f"{d['f64']:6.0f}{d['int']:6.0f}{d['other']:7.0f}{d['wait'] / 1e3:8.1f}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
