#!/usr/bin/env python3
"""Benchmark: IPM problem-iterations/s on the BASELINE.json workload (config C2).

A "step" is one batched solve of this rank's shard: 65,536 independent dense
SOCPs (n=64, m=16, k=96, cones POC32+SOC32+SOC32) generated on the device,
initial point + K=8 interior-point iterations each (fixed-K mode, tol=0,
SURVEY.md §8(d)), plus (N>1) the all-gather of per-problem (status, iters)
over RCCL — the path's only exchange step.  Shards are disjoint global
problem ranges, so scaling is weak.

Output: one JSON line on rank 0 (driver contract), including
  roofline     — FP64 work of the solver kernel (SURVEY.md §8(d) formula,
                 939.3 KFLOP per problem-iteration at C2) over its HIP-event
                 duration on the solver's own stream, against the 78.6 TFLOP/s
                 FP64 peak;
  cpu_baseline — the CPU oracle (reference op order, oracle/) on a bounded
                 sample of the same problems on this host's cores.
Launch: python bench.py [--gpus N --steps K --warmup W]
        N>1 with no launcher: bench.py starts the N ranks itself under
        torch.distributed.run (from a parent that never touches the GPU);
        under a launcher (WORLD_SIZE set) WORLD_SIZE must equal N.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "socp.jl_amd"))

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 (vector = matrix), spec
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, spec


def flops_per_problem_iter(n, m, k, sing=False):
    """SYRK + potrf/potri + A*Li + S + chol(S) + mat-vecs."""
    return (n * (n + 1) * k + n ** 3 + 2 * m * n * n + m * (m + 1) * n + m ** 3 / 3.0
            + 16 * k * n + 12 * m * n + 4 * n * n + 4 * m * m + (n * n if sing else 0))


def flops_executed_per_problem_iter(n, m, k, sing=False, large=False):
    """FP64 work the kernels actually execute per problem-iteration.  Where
    H = L L' is factored and Li is never formed (the register kernel for
    m <= 16, densesolver.jl:47 cholesky! + triangular solves; the blocked
    kernel's default SOCP_LG_CHOL build) potrf is n^3/3 and Z = L^-1 A' is
    m n^2, in place of potrf + potri (n^3) and A*Li (2 m n^2) of the SURVEY.md
    §8(d) formula; where Li is formed (the register kernel for m > 16, and
    --explicit-inverse: potrf + trtri + lauum from the one factor, chol_inv)
    the kernel executes the formula's figure."""
    if not (large or m <= 16):
        return flops_per_problem_iter(n, m, k, sing)
    return (n * (n + 1) * k + n ** 3 / 3.0 + m * n * n + m * (m + 1) * n + m ** 3 / 3.0
            + 16 * k * n + 12 * m * n + 4 * n * n + 4 * m * m + (n * n if sing else 0))


def bytes_per_problem_iter(n, m, k):
    """G, A read once; c, b, h; x, y, z, s read + write."""
    return 8 * (k * n + m * n) + 8 * (n + m + k) + 16 * (n + m + 2 * k)


def cone_str(cones):
    """((kind, offs, dim), ...) -> e.g. 'POC32+SOC32+SOC32' or '8xSOC80'."""
    parts = [("POC" if kind == 0 else "SOC") + str(dim) for kind, _, dim in cones]
    out, i = [], 0
    while i < len(parts):
        j = i
        while j < len(parts) and parts[j] == parts[i]:
            j += 1
        out.append(parts[i] if j - i == 1 else f"{j - i}x{parts[i]}")
        i = j
    return "+".join(out)


BASELINE_METRIC = "IPM iters/sec, 65k-batch n=64 dense SOCP at 1/2/4/8 GPU; achieved HBM GB/s"


def metric_name(cfg, B):
    """BASELINE.json's metric for its C2 workload; the same metric named for
    the other configs' lines (C1, C4 are profile lines, not the headline)."""
    if cfg.name == "C2" and B == cfg.batch:
        return BASELINE_METRIC
    kb = f"{B // 1024}k" if B % 1024 == 0 else str(B)
    return f"IPM iters/sec, {kb}-batch n={cfg.n} dense SOCP ({cfg.name}); achieved HBM GB/s"


def latest_traffic_json(cfg_name):
    """Newest committed PMC traffic summary for the config (profiles/rNN_pmc_traffic[_cfg].json)."""
    import glob
    suffix = "" if cfg_name == "C2" else "_" + cfg_name.lower()
    found = sorted(glob.glob(os.path.join(HERE, "profiles", f"r[0-9][0-9]_pmc_traffic{suffix}.json")))
    return found[-1] if found else os.path.join(HERE, "profiles", f"r01_pmc_traffic{suffix}.json")


def host_cpu_info():
    """nproc, the CPUs this process may run on, and the lscpu model name."""
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    if model is None:
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "model": model}


def baseline_threads():
    """Every core this process may use -- capped by OMP_NUM_THREADS, which the
    GPU box sets to its per-GPU CPU share (16): the machine's other cores
    belong to other jobs."""
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def cpu_baseline(cfg, fixed_k, budget_s=12.0, threads=None, tol=0.0, structured=False, reps=5):
    """Oracle (the reference algorithm restated in C, oracle/) on host cores:
    one warm-up, then the median of `reps` timed batch solves of the same
    sample; the sample size is chosen so the reps take about budget_s."""
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle as O  # test infrastructure: timed as the baseline, never the product
    threads = threads or baseline_threads()
    flags = O.F_STRUCTURED if structured else 0
    P = O.Params(maxit=fixed_k, tol=tol, flags=flags)
    small = flops_per_problem_iter(cfg.n, cfg.m, cfg.k) < 1e7

    def run(chunk, d):
        t0 = time.perf_counter()
        r = O.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, d["c"], d["A"], d["b"], d["G"], d["h"],
                          sing=[0] * chunk, params=P, nthreads=threads)
        return int(r["iters"].sum()), time.perf_counter() - t0

    chunk = 4 * threads if small else threads
    d = O.generate(cfg.cones, chunk, cfg.n, cfg.m, cfg.k, cfg.seed)
    run(chunk, d)  # warm-up (page-in, thread pool)
    _, t_probe = run(chunk, d)
    want = budget_s / reps  # seconds per rep
    if t_probe < want:
        chunk = int(chunk * want / max(t_probe, 1e-4)) // threads * threads or threads
        chunk = min(chunk, 65536)
        d = O.generate(cfg.cones, chunk, cfg.n, cfg.m, cfg.k, cfg.seed)
    rates, total_t = [], 0.0
    for _ in range(reps):
        it, dt = run(chunk, d)
        rates.append(it / dt)
        total_t += dt
    rates.sort()
    med = rates[len(rates) // 2]
    info = host_cpu_info()
    algo = ("oracle/socp_oracle.c structured mode (the kernels' algorithm: X = W^-1 G per cone, H = X'X, "
            "explicit inverse; no dense iWiW)" if structured else
            "oracle/socp_oracle.c (reference op order incl. dense iW*iW' and potrs(I) inverse)")
    return {"value": med, "unit": "problem-iterations/s", "cores": threads, "kind": "port",
            "per_core": med / threads, "nproc": info["nproc"], "affinity_cpus": info["affinity"],
            "cpu_model": info["model"], "reps": [round(x, 1) for x in rates],
            "sample": f"median of {reps} reps x {chunk} {cfg.name} problems (first {chunk} of the seeded workload), "
                      + (f"tol={tol}, maxit={fixed_k}, " if tol else f"fixed-K={fixed_k}, ")
                      + f"{algo}, OpenMP {threads} threads (OMP_NUM_THREADS / affinity), {total_t:.1f}s timed"}


def cpu_allcores(cfg, fixed_k, base, tol=0.0, budget_s=5.0):
    """The reference-order CPU rate on every CPU of the host, extrapolated: the
    GPU box gives one GPU's job a 16-CPU share of its cores (OMP_NUM_THREADS),
    so no run here may use all of them.  The one-thread rate is measured and
    the line reports nproc x that rate (perfect scaling, an upper bound on
    what all cores reach) beside the measured per-core rate of the
    `cpu_baseline` threads -- their ratio is the measured parallel efficiency
    that the extrapolation assumes to hold up to nproc."""
    one = cpu_baseline(cfg, fixed_k, budget_s=budget_s, threads=1, tol=tol, reps=3)
    info = host_cpu_info()
    ncpu = info["affinity"] or info["nproc"]
    return {"value": one["value"] * ncpu, "unit": "problem-iterations/s", "cores": ncpu, "kind": "port",
            "measured": False, "one_thread": one["value"], "per_core_at_threads": base["per_core"],
            "threads": base["cores"], "efficiency_at_threads": base["per_core"] / one["value"],
            "sample": f"extrapolated: {ncpu} CPUs x the 1-thread rate ({one['sample']}); not run on all CPUs "
                      "because the box allots this job OMP_NUM_THREADS of them"}


def ingest_line(S, cfg, B, K, tol, dev_data, steps, ctx):
    """PCIe-inclusive rate (never `value`): the same batch held in host memory
    flows through socp_ingest -- double-buffered pinned staging, batch i+1's
    host-to-device copy on a copy stream under batch i's solve, results back to
    the host.  Two forms: inputs already in the pinned slots (zero-copy
    producer) and inputs in pageable numpy arrays (copied into the slots by
    submit).  Timed region: `steps` batches submitted two deep, every result on
    the host at the end."""
    import numpy as np
    n, m, k = cfg.n, cfg.m, cfg.k
    host = [t.cpu().numpy() for t in dev_data]
    sing = np.zeros(B, np.uint8)
    ing = S.Ingest(cfg.cones, n, m, k, B, ctx=ctx)
    kw = dict(maxit=K, tol=tol)
    views = []
    for _ in range(2):  # fill both slots once (the solve never writes its inputs)
        v = ing.next_inputs()
        for key, arr in zip(("c", "A", "b", "G", "h"), host):
            v[key][:arr.size] = arr
        v["sing"][:B] = 0
        views.append([v[key][:arr.size] for key, arr in zip(("c", "A", "b", "G", "h"), host)] + [v["sing"][:B]])
        views[-1].append(ing.submit(*views[-1][:6], **kw))
    it0 = None
    for v in views:
        it0 = ing.wait(v.pop())["iters"]
    iters_per_batch = int(it0.sum())

    def run(src_of):
        t, outs = [], 0
        t0 = time.perf_counter()
        for i in range(steps):
            if i >= 2:
                ing.wait(t[i - 2])
                outs += 1
            t.append(ing.submit(*src_of(i), **kw))
        for tk in t[outs:]:
            ing.wait(tk)
        return time.perf_counter() - t0

    dt_pin = run(lambda i: views[i % 2])
    dt_page = run(lambda i: host + [sing])
    in_bytes = 8 * B * (n + m * n + m + k * n + k) + B
    out_bytes = 8 * B * (n + m + 2 * k) + 4 * 2 * B + 8 * 3 * B
    ing.close()
    return {
        "value": iters_per_batch * steps / dt_pin,
        "unit": "problem-iterations/s",
        "ms_per_batch": dt_pin / steps * 1e3,
        "h2d_bytes_per_batch": in_bytes,
        "d2h_bytes_per_batch": out_bytes,
        "h2d_GBps": in_bytes * steps / dt_pin / 1e9,
        "pageable": {"value": iters_per_batch * steps / dt_page, "ms_per_batch": dt_page / steps * 1e3,
                     "h2d_GBps": in_bytes * steps / dt_page / 1e9},
        "mode": "socp_ingest: host batch -> pinned slot -> H2D (copy stream) overlapped with the previous "
                "batch's solve -> D2H; `value` = inputs already in pinned slots, `pageable` = inputs in "
                "numpy arrays copied into the slots by submit",
    }


def sqr_model(n, m, k, cones):
    """Algorithmic flops and bytes of one rank-update KKT iteration per problem
    (setup_iter + 2 x solve_kkt of spsolver.jl:60-130): setup = G'DG (one
    triangle) + chol(H) + per SOC cone G'u, G'v and two rank-1 modifications
    + L^-1 A' + S + chol(S); solve = G'v, Gv, two H and one S triangular pair,
    A/A' mat-vecs.  Bytes: setup reads G, A, s, z and writes the record
    (L_H, L_S, lambda, wb); each solve reads G, A, the record and 2(n+m+2k)
    vector entries."""
    soc = [(o, d) for kind, o, d in cones if kind == 1]
    f_setup = (n * (n + 1) * k + n ** 3 / 3.0 + sum(4 * d * n + 4 * n * n for _, d in soc)
               + m * n * n + m * (m + 1) * n + m ** 3 / 3.0 + 20 * k)
    f_solve = 4 * k * n + 4 * n * n + 2 * m * m + 4 * m * n + 30 * k
    rec = n * n + m * m + 2 * k
    b_setup = 8 * (k * n + m * n + 2 * k + rec)
    b_solve = 8 * (k * n + m * n + rec + 2 * (n + m + 2 * k))
    return f_setup, f_solve, b_setup, b_solve


def sqr_bench(args, emit=True):
    """--mode sqr: the rank-update plugin (socp_sqr_*, SparseSolver + SqrScaling,
    spsolver.jl / sqrscalings.jl) at the config's shape.  A step = setup_iter +
    two solve_kkt (one IPM iteration's KKT work) over the whole batch, device
    tensors, at the interior iterate the dense solver reaches after 3
    iterations.  HBM-bound by the algorithmic model (sqr_model)."""
    import torch
    import socp_amd as S
    from socp_amd.configs import CONFIGS
    cfg = CONFIGS[args.config]
    B = args.batch or cfg.batch
    n, m, k = cfg.n, cfg.m, cfg.k
    ctx = S.Context(0)
    c, A, b, G, h = S.generate(cfg.cones, B, n, m, k, cfg.seed, ctx=ctx)
    sing = torch.zeros(B, dtype=torch.uint8, device=G.device)
    it = S.batch_solve(cfg.cones, n, m, k, c, A, b, G, h, sing, maxit=3, tol=0.0, ctx=ctx)
    ctx.sync()
    hd = S.SqrHandle(cfg.cones, n, m, k, A, G, sing, ctx=ctx)
    gen = torch.Generator(device=G.device).manual_seed(5)
    r = [torch.randn(B * q, dtype=torch.float64, device=G.device, generator=gen) for q in (n, m, k, k)]
    out = None
    t_setup, t_solve = [], []

    def step(timed):
        nonlocal out
        hd.setup_iter(it["s"], it["z"])
        if timed:
            t_setup.append(ctx.last_kernel_ms())
        for _ in range(2):
            out = hd.solve_kkt(*r, out=out)
            if timed:
                t_solve.append(ctx.last_kernel_ms())

    for _ in range(args.warmup):
        step(False)
    ctx.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(False)
    ctx.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for _ in range(2):
        step(True)  # per-kernel HIP-event durations, outside the timed region
    ms_setup = sum(t_setup) / len(t_setup)
    ms_solve = sum(t_solve) / len(t_solve)
    st = torch.bincount(out["status"].long(), minlength=5).tolist()
    # the whole IPM on this plugin (socp_sqr_solve_socp, solve_socp with
    # SparseSolver): initial point + fixed-K iterations, the dense headline's mode
    Kf = cfg.fixed_k
    ipm = hd.solve_socp(c, b, h, maxit=Kf, tol=0.0)
    ctx.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        ipm = hd.solve_socp(c, b, h, maxit=Kf, tol=0.0)
    ctx.sync()
    torch.cuda.synchronize()
    dt_ipm = time.perf_counter() - t1
    ipm_iters = int(ipm["iters"].sum().item())
    ipm_st = torch.bincount(ipm["status"].long(), minlength=5).tolist()
    fs, fv, bs, bv = sqr_model(n, m, k, cfg.cones)
    traffic = None
    if args.traffic_json and os.path.exists(args.traffic_json):
        tj = json.load(open(args.traffic_json))
        if tj.get("batch") == B and "socp_sqr_setup_kernel" in tj.get("kernels", []):
            traffic = tj["hbm_bytes_per_launch"]
    setup_gbs = bs * B / (ms_setup * 1e-3) / 1e9
    solve_gbs = bv * B / (ms_solve * 1e-3) / 1e9
    dominant = "setup" if ms_setup >= 2 * ms_solve else "solve"
    ach = setup_gbs if dominant == "setup" else solve_gbs
    line = {
        "metric": "rank-update KKT plugin (SparseSolver + SqrScaling): setup_iter + 2 solve_kkt per problem",
        "value": B * args.steps / dt,
        "unit": "problem-iterations/s (KKT work of one IPM iteration)",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (device generator), iterates after 3 dense IPM iterations",
        "config": {"workload": f"{cfg.name} shape: {B} problems, n={n}, m={m}, k={k}, cones {cone_str(cfg.cones)}; "
                               "socp_sqr_setup_iter + 2 x socp_sqr_solve_kkt on device tensors",
                   "global_batch": B, "parallelism": "dp1"},
        "kernels": {"socp_sqr_setup_kernel_ms": ms_setup, "socp_sqr_solve_kernel_ms": ms_solve},
        "status_counts": st,
        "solve_socp": {"value": ipm_iters * args.steps / dt_ipm, "unit": "problem-iterations/s",
                       "ms_per_solve": dt_ipm / args.steps * 1e3, "status_counts": ipm_st,
                       "mode": f"socp_sqr_solve_socp: initial point + fixed-K={Kf} IPM iterations (tol=0) "
                               "with SqrScaling + the rank-update factor, device tensors"},
        "roofline": {"bound": "hbm", "kernel": f"socp_sqr_{dominant}_kernel", "achieved": ach,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                     "traffic": traffic if dominant == "setup" else None,
                     "hbm_gbs": traffic / (ms_setup * 1e-3) / 1e9 if traffic and dominant == "setup" else None,
                     "setup_GBps": setup_gbs, "solve_GBps": solve_gbs,
                     "setup_TFLOPs": fs * B / (ms_setup * 1e-3) / 1e12,
                     "solve_TFLOPs": fv * B / (ms_solve * 1e-3) / 1e12,
                     "bytes_per_problem": {"setup": bs, "solve": bv}, "flops_per_problem": {"setup": fs, "solve": fv}},
    }
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(HERE, "oracle"))
        import oracle as O  # test infrastructure: the CPU line only
        import numpy as np
        thr = baseline_threads()
        chunk = 64 * thr
        d = O.generate(cfg.cones, chunk, n, m, k, cfg.seed)
        P = O.Params(maxit=cfg.fixed_k, tol=0.0, flags=O.F_SQR)
        rates = []
        for rep in range(4):
            t1 = time.perf_counter()
            rr = O.batch_solve(cfg.cones, n, m, k, d["c"], d["A"], d["b"], d["G"], d["h"],
                               sing=np.zeros(chunk, np.uint8), params=P, nthreads=thr)
            if rep:
                rates.append(int(rr["iters"].sum()) / (time.perf_counter() - t1))
        rates.sort()
        info = host_cpu_info()
        line["cpu_baseline"] = {"value": rates[len(rates) // 2], "unit": "problem-iterations/s (whole IPM iteration)",
                                "cores": thr, "kind": "port", "cpu_model": info["model"], "nproc": info["nproc"],
                                "sample": f"median of 3 reps x {chunk} {cfg.name} problems, fixed-K={cfg.fixed_k}, "
                                          "oracle F_SQR (SqrScaling + rank-update factor restated, whole IPM "
                                          "iteration: a superset of the KKT work timed on the GPU)"}
    if emit:
        print(json.dumps(line), flush=True)
    return line


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`--gpus N` (N > 1) with no launcher around us: start the N ranks here,
    one process per GPU under torch.distributed.run (the driver's own launch
    line), and return its exit code.  This parent never initialises the GPU
    (no HIP call, no torch.cuda query), so the children start clean."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return subprocess.call(cmd, env=env)


def stub_shard_solver(B, K, step_s):
    """--stub-solve (CPU tests of the launcher and the N > 1 accounting only):
    every problem of the shard 'runs' K iterations and converges, after
    `step_s` seconds of wall time.  No GPU, no oracle: bench.py's product line
    is never produced this way on a GPU box (the line names the stub)."""
    import torch

    def solve():
        time.sleep(step_s)
        return {"status": torch.zeros(B, dtype=torch.int32), "iters": torch.full((B,), K, dtype=torch.int32),
                "res": torch.zeros((B, 3), dtype=torch.float64)}
    return solve


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--batch", type=int, default=0, help="problems per GPU (default: config batch)")
    ap.add_argument("--fixed-k", type=int, default=0)
    ap.add_argument("--mode", choices=["fixed", "reference", "sqr"], default="fixed",
                    help="fixed: tol=0, K iterations (headline, SURVEY.md §8(d)(i)); reference: the "
                         "reference's stopping rule, tol=1e-5 absolute, maxit=40, per-problem masking (§8(d)(ii)); "
                         "sqr: the rank-update KKT plugin (socp_sqr_*, spsolver.jl) at the config's shape")
    ap.add_argument("--explicit-inverse", action="store_true",
                    help="SOCP_F_EXPLICIT_INVERSE: the reference's operation order (Li = H^-1 formed, "
                         "densesolver.jl:48) instead of the default H = L L' + triangular solves")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="per CPU line (two lines)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-ingest", action="store_true",
                    help="skip the PCIe-inclusive line (host batches through socp_ingest, N=1 only) and the "
                         "other-mode summaries (explicit inverse, rank-update plugin): only the timed solver launches")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic summary (tools/pmc_traffic.py); default: the newest profiles/rNN_pmc_traffic[_<config>].json")
    ap.add_argument("--stub-solve", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group of an N > 1 run: nccl (= RCCL, one GPU per rank; the product line) or "
                         "gloo (rehearsal: the ranks may share GPUs, outcomes exchanged through host memory; "
                         "the line says so and is not a scaling measurement)")
    args = ap.parse_args(argv)
    argv = sys.argv[1:] if argv is None else list(argv)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        if args.mode == "sqr":
            ap.error("--mode sqr is a one-GPU line (the rank-update plugin); run it with --gpus 1")
        return launch_ranks(args.gpus, argv)
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: the launcher and the flag disagree",
              file=sys.stderr, flush=True)
        return 2
    if args.mode == "sqr":
        if world > 1:
            print("bench.py: --mode sqr runs on one GPU", file=sys.stderr, flush=True)
            return 2
        sqr_bench(args)
        return 0
    return run_rank(args, world)


def run_rank(args, world):
    import torch
    import torch.distributed as dist
    from socp_amd.configs import CONFIGS

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    stub = args.stub_solve
    rehearsal = world > 1 and not stub and args.dist_backend == "gloo"
    if rehearsal:
        local = local % max(1, torch.cuda.device_count())  # ranks may share a GPU
    if world > 1:
        if stub or rehearsal:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    cfg = CONFIGS["C2" if args.config == "C3" else args.config]
    B = args.batch or cfg.batch
    ref_rule = args.mode == "reference"
    K = 40 if ref_rule else (args.fixed_k or cfg.fixed_k)  # solver.jl:105
    tol = 1e-5 if ref_rule else 0.0  # solver.jl:122
    n, m, k = cfg.n, cfg.m, cfg.k
    from socp_amd.dist import timed_shard_steps

    if stub:
        solve_shard = stub_shard_solver(B, K, 0.01)
        tr = timed_shard_steps(solve_shard, args.steps, args.warmup)
        kernel_ms = tr["step_ms"]
        kname = "stub (--stub-solve: no solver ran)"
        S = ctx = None
    else:
        import socp_amd as S
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        ctx = S.Context(local)
        c, A, b, G, h = S.generate(cfg.cones, B, n, m, k, cfg.seed, first_problem=rank * B, ctx=ctx)
        sing = torch.zeros(B, dtype=torch.uint8, device=dev)  # uniform G (k > n) has full column rank
        ctx.sync()
        prev = {"out": None}

        def solve_shard():
            # no host synchronisation inside a step: each launch records its own
            # HIP event pair on the solver's stream, read after the timed region
            prev["out"] = S.batch_solve(cfg.cones, n, m, k, c, A, b, G, h, sing, maxit=K, tol=tol, ctx=ctx,
                                        out=prev["out"], res=world > 1, explicit_inverse=args.explicit_inverse)
            return prev["out"]

        def sync():
            ctx.sync()
            torch.cuda.synchronize()

        # warm-up, the K timed steps between barriers, max-over-ranks time, summed
        # iterations, and (N > 1) the per-step outcome all-gather: socp_amd.dist
        tr = timed_shard_steps(solve_shard, args.steps, args.warmup, sync=sync)
        kernel_ms = ctx.kernel_times(args.steps)  # the timed steps' solver launches (the last 64 at most)
        kname = ctx.last_kernel_name()
    out, dt, iters_total = tr["out"], tr["dt"], tr["iters_total"]
    status_counts = torch.bincount(out["status"].long(), minlength=5).tolist()

    if rank == 0:
        kms = sum(kernel_ms) / len(kernel_ms)
        iters_per_launch = int(out["iters"].sum().item())
        F = flops_per_problem_iter(n, m, k)
        Fx = (F if args.explicit_inverse else
              flops_executed_per_problem_iter(n, m, k, large="large" in kname))
        Bq = bytes_per_problem_iter(n, m, k)
        # binding bound of the algorithmic model: FP64 when F/B is above the
        # ridge (C2, C4), HBM below it (C1)
        hbm_bound = F / Bq < FP64_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)
        if hbm_bound:
            achieved, peak, unit = Bq * iters_per_launch / (kms * 1e-3) / 1e9, HBM_PEAK_GBS, "GB/s"
        else:
            achieved, peak, unit = F * iters_per_launch / (kms * 1e-3) / 1e12, FP64_PEAK_TFLOPS, "TFLOP/s"
        traffic = None
        tj_path = args.traffic_json or latest_traffic_json(cfg.name)
        if os.path.exists(tj_path) and not stub:
            try:
                tj = json.load(open(tj_path))
                if tj.get("config") == cfg.name and tj.get("batch") == B and tj.get("fixed_k") == K:
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        hbm_gbs = traffic / (kms * 1e-3) / 1e9 if traffic else None
        line = {
            "metric": metric_name(cfg, B),
            "value": iters_total / dt,
            "unit": "problem-iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("stub: no solve ran (launcher / accounting test)" if stub else
                     "synthetic (device SplitMix64 generator, SURVEY.md §8(d); feasible by construction)"),
            "config": {
                "workload": f"{cfg.name}: {B} problems per GPU, n={n}, m={m}, k={k}, cones {cone_str(cfg.cones)}, "
                            + (f"initial point + reference stopping rule (tol=1e-5 abs, maxit={K}; "
                               f"value counts executed iterations)" if ref_rule else
                               f"initial point + fixed-K={K} IPM iterations (tol=0)")
                            + ("; explicit inverse Li = H^-1 (SOCP_F_EXPLICIT_INVERSE, the reference's "
                               "op order, densesolver.jl:47-48: Li from the Cholesky factor, L^-T L^-1)"
                               if args.explicit_inverse else ""),
                "operation_order": "explicit_inverse" if args.explicit_inverse else "cholesky",
                "global_batch": B * world,
                "parallelism": f"dp{world} (disjoint problem shards, status all-gather only)"
                               + ("; REHEARSAL: gloo process group, ranks sharing "
                                  f"{torch.cuda.device_count()} GPU(s) -- not a scaling measurement"
                                  if rehearsal else ""),
            },
            "kernel": kname,
            "kernel_ms": kms,
            "status_counts": status_counts,
            "roofline": {
                "bound": "hbm" if hbm_bound else "mfma",
                "achieved": achieved,
                "peak": peak,
                "unit": unit,
                "frac": achieved / peak,
                "traffic": traffic,
                "hbm_gbs": hbm_gbs,
                "traffic_source": os.path.relpath(tj_path, HERE) if traffic else None,
                "flops_per_problem_iter": F,
                # the same bound counting only the flops the kernel executes
                # (Cholesky + triangular solves: no explicit inverse, no A*Li)
                "flops_executed_per_problem_iter": Fx,
                "achieved_executed": Fx * iters_per_launch / (kms * 1e-3) / 1e12,
                "frac_executed": Fx * iters_per_launch / (kms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                "bytes_per_problem_iter": Bq,
                "problem_iters_per_launch": iters_per_launch,
            },
        }
        if world > 1 and tr.get("gathered") is not None:
            # every rank's outcome records as rank 0 received them (the exchange step)
            gst = tr["gathered"]["status"].reshape(-1).long().cpu()
            line["gathered"] = {"status_counts": torch.bincount(gst, minlength=5).tolist(),
                                "iters_sum": int(tr["gathered"]["iters"].long().sum().item()),
                                "problems": int(gst.numel())}
        extras = world == 1 and not stub
        if extras and not args.no_ingest:
            line["ingest"] = ingest_line(S, cfg, B, K, tol, (c, A, b, G, h), args.steps, ctx)
        if extras and not args.explicit_inverse and not ref_rule and not args.no_ingest:
            # the other operation order on the same batch (never `value`): the
            # reference's explicit Li = H^-1 (SOCP_F_EXPLICIT_INVERSE); its own
            # line is `--explicit-inverse`
            xi_ms, xo = [], None
            for rep in range(1 + args.steps):
                xo = S.batch_solve(cfg.cones, n, m, k, c, A, b, G, h, sing, maxit=K, tol=tol, ctx=ctx, out=xo,
                                   explicit_inverse=True)
                if rep:
                    xi_ms.append(ctx.last_kernel_ms())
            xi_kms = sum(xi_ms) / len(xi_ms)
            xi_it = int(xo["iters"].sum().item())
            line["explicit_inverse"] = {
                "kernel": ctx.last_kernel_name(), "kernel_ms": xi_kms,
                "value_kernel": xi_it / (xi_kms * 1e-3), "unit": "problem-iterations/s (solver kernel time)",
                "frac": F * xi_it / (xi_kms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                "mode": "bench.py --explicit-inverse: Li = H^-1 formed from the Cholesky factor as "
                        "densesolver.jl:47-48 forms it (potrf, then triangular solves against I); frac by the "
                        "SURVEY.md §8(d) formula (which this order executes)"}
        if extras and not args.no_ingest and cfg.name == "C2" and not ref_rule:
            # the rank-update plugin (SparseSolver + SqrScaling, socp_sqr_*) at the same shape: its
            # own line is `--mode sqr`; summarised here so every default run records it
            sq = sqr_bench(argparse.Namespace(config=cfg.name, batch=B, steps=args.steps, warmup=1, no_cpu=True,
                                              traffic_json=None), emit=False)
            line["rank_update_plugin"] = {"value": sq["value"], "unit": sq["unit"], "ms_per_step": sq["ms_per_step"],
                                          "kernels_ms": sq["kernels"], "status_counts": sq["status_counts"],
                                          "solve_socp": sq["solve_socp"],
                                          "mode": "bench.py --mode sqr (setup_iter + 2 x solve_kkt per problem)"}
        if not args.no_cpu and extras:  # the CPU leg: rank 0 at N=1 only
            line["cpu_baseline"] = cpu_baseline(cfg, K, budget_s=args.cpu_seconds, tol=tol)
            line["cpu_baseline_structured"] = cpu_baseline(cfg, K, budget_s=args.cpu_seconds, tol=tol,
                                                           structured=True)
            line["cpu_baseline_allcores"] = cpu_allcores(cfg, K, line["cpu_baseline"], tol=tol,
                                                         budget_s=args.cpu_seconds / 2)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
