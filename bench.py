#!/usr/bin/env python3
"""Benchmark: closed-loop GPC simulations/s over the Shell 3x3 tuning grid (BASELINE.json metric).

One step = score one batch of 4096 (N2=30, Nu=5, delta, lambda) candidates per GPU: a 500-step
constrained closed loop + its GAM cost J1 per candidate (GAM_fun.m:81-111 per candidate), then
one RCCL all-gather of the per-candidate costs and an identical stable ranking on every rank
(SURVEY §8e).  Inputs are resident in HBM before the timed region.  Weak scaling: every rank
scores its own strided 4096-candidate shard (candidates rank, rank + world, ...) of a
(4096 x world)-candidate grid.

Launch:  python bench.py [--gpus 1 --steps K --warmup W]
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "model-predictive-control-tuning_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (= FP64 matrix) dense peak, AMD spec; see DESIGN.md


def algorithmic_flops_per_sim(sc, N2, Nu, iters_per_step):
    """SURVEY §8(d) per-simulation flop count, evaluated on this scenario's tables:
    setup P*M*(M+1) + M^3/3; per step: plant 5*my*(nu+nd) + free response
    2*N2*(sum(na+1) + sum_ij cp_ij) + gradient 2*P*(M+1) + solve 2*M^2 + active set
    2*(2M*M + M^2)*I_as + cost 4*my."""
    my, nu, nin = sc.my, sc.nu, sc.nin
    M, P = nu * Nu, my * N2
    cp = sc.dp[:, :nu] + sc.nb[:, :nu]
    setup = P * M * (M + 1) + M ** 3 / 3.0
    per_step = (5 * my * nin + 2 * N2 * (int(np.sum(sc.na + 1)) + int(np.sum(np.maximum(cp, 1))))
                + 2 * P * (M + 1) + 2 * M * M + 2 * (2 * M * M + M * M) * iters_per_step + 4 * my)
    return setup + sc.nit * per_step


def band_flops_per_sim(sc, N2, Nu, iters):
    """Algorithmic flops of one config-3 simulation (mdband_kernel.hip): per step the
    free-response window update 2*P*nin (P = my*N2 output rows, nin = MVs + MDs), the feasibility
    scan of the 2P soft output rows against the M+1 QP variables 2*(2P)*(M+1), and per Goldfarb-
    Idnani iteration another scan plus the factor update 2*(2P)*(M+1) + 6*(M+1)^2; setup: the
    column-streamed QR of the M+1 weighted rows 2*(M+1)^3/3.  iters = measured GI iterations."""
    P, M1 = sc.my * N2, sc.nu * Nu + 1
    per_step = 2 * P * sc.nin + 4 * P * M1
    return 2 * M1 ** 3 / 3.0 + sc.nit * per_step + iters * (4 * P * M1 + 6 * M1 * M1)


def nmpc_flops_per_sim(N, Nu, gn_iters, nit=60, nsub=10, nx=3, ny=2, nu=2):
    """Algorithmic flops of one config-5 simulation (nmpc_kernel.hip), per Gauss-Newton
    iteration: the RK4 prediction over N steps x nsub sub-steps x 4 stages of the model (~40 flops)
    and of its M+1 forward tangents (2*nx^2 each), the streamed QR of the N*ny output rows into M+1
    columns (3*(M+1)^2 per row), an Armijo trial pass (prediction only); per closed-loop step the
    plant's own RK4 integration.  gn_iters = measured Gauss-Newton iterations of the simulation."""
    M1 = nu * Nu + 1
    rk = N * nsub * 4
    per_gn = rk * (40 + 2 * nx * nx * M1) + N * ny * 3 * M1 * M1 + rk * 40
    return gn_iters * per_gn + nit * nsub * 4 * 40


def dtc_flops_per_sim(sc, N2, Nu):
    """Algorithmic flops of one config-4 simulation as dtc_small_kernel computes it (the
    unconstrained DTC loop applies only the first-move rows of the gain): setup P*M*(M+1) + M^3/3
    (SURVEY §8d's term); per step 2 flops per term of every plant / disturbance-path entry and of
    every predictor entry Pz, Gz (nonzero numerator taps + denominator order), the filters
    2*(2*len - 1) per output, the y difference update 4 per output, the first-move product
    2*nu*nx, the costs 4*my."""
    def terms(t):
        return int(np.count_nonzero(np.asarray(t.num))) + len(t.den) - 1

    my, nu = sc.my, sc.nu
    nx = int(sc.table(2)[6])
    plant = sum(terms(t) for row in sc.plant for t in row) + sum(terms(t) for row in (sc.dist or []) for t in row)
    model = 2 * sum(terms(t) for row in sc.model for t in row[:nu])
    filt = sum(2 * (2 * len(f.den) - 1) for f in (sc.filters or []))
    M, P = nu * np.asarray(Nu, dtype=float), my * np.asarray(N2, dtype=float)
    per_step = 2 * (plant + model) + filt + 4 * my + 2 * nu * nx + 4 * my
    return P * M * (M + 1) + M ** 3 / 3.0 + sc.nit * per_step


def cpu_share():
    """(cpus, note): the CPUs this process may use -- its affinity set, limited by a cgroup CPU
    quota when one is set (the GPU box gives each GPU a share of the host)."""
    n = len(os.sched_getaffinity(0))
    note = "%d CPUs in the affinity set" % n
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
            note += ", cgroup quota %d CPUs" % quota
            n = min(n, quota)
    except (OSError, ValueError):
        pass
    return n, note


def reference_structured_baseline(N2v, Nuv, d, l, J1, seconds):
    """Config 2, reference-structured, 1 thread: the numpy restatement of
    closedloop_toolbox with the plant re-simulated over the whole input history every step
    (lsim, DTC_GPC_WW.m:130-136 structure, O(nit^2)) and the primal active-set QP, on seeded
    random candidates of the same grid for ~`seconds`."""
    from oracle.scenarios import shell3x3 as o_shell3x3
    from oracle.toolbox_gpc import closedloop_toolbox as o_cl

    osc, orr, oyref, _ = o_shell3x3()
    done, tc, rel = 0, 0.0, []
    for k in np.random.default_rng(20250307).permutation(len(N2v)):
        k = int(k)
        t1 = time.perf_counter()
        o = o_cl(osc, orr, None, int(N2v[k]), int(Nuv[k]), d[k], l[k], orr.shape[1], open_loop=False,
                 full_history=True)
        tc += time.perf_counter() - t1
        done += 1
        j = ((o.y - oyref) ** 2).sum(1)
        rel.append(float(np.max(np.abs(J1[k] - j) / np.abs(j))))
        if tc >= seconds:
            break
    return {"value": done / tc, "unit": "sims/s", "cores": 1, "kind": "port",
            "sample": "oracle/toolbox_gpc.py closedloop_toolbox(full_history=True): numpy, plant re-simulated "
                      "with lsim over the whole history every step (DTC_GPC_WW.m:130-136 structure), primal "
                      "active-set QP; %d seeded random candidates of the metric grid, 1 thread, %.1f s; max rel "
                      "|J1_gpu - J1_cpu| = %.1e" % (done, tc, max(rel))}


def other_cpu_baseline(workload, N2, Nu, d, l, refs, J1, st, seconds):
    """Single-thread CPU restatement (oracle/) of a config-3/4/5 simulation, timed on a bounded
    seeded sample of the same grid (rank 0, N = 1): the reference-structured numpy loops, i.e.
    toolbox_band.closedloop_band (config 3), nmpc_vdv.closedloop_nmpc (config 5) and
    dtcgpc.dtc_gpc_ww (config 4: DTC_GPC_WW.m's full-history lsim loop, nominal plant)."""
    rel = []
    if workload == "shell7x5":
        from oracle.scenarios import shell7x5 as o_shell7x5
        from oracle.toolbox_band import closedloop_band

        osc, orr, ov, _, _ = o_shell7x5()
        what = "oracle/toolbox_band.py closedloop_band (numpy, nit=200, closed loop only)"

        def run(k):
            closedloop_band(osc, orr, ov, int(N2[k]), int(Nu[k]), d[k], l[k], orr.shape[1], open_loop=False)
    elif workload == "vandevusse":
        from mpct.nmpc import steady_state, vandevusse_signals
        from oracle.nmpc_vdv import closedloop_nmpc

        _, yref = vandevusse_signals(steady_state())
        what = "oracle/nmpc_vdv.py closedloop_nmpc (numpy, nit=60 + open loop)"

        def run(k):
            o = closedloop_nmpc(refs[0], int(N2[k]), int(Nu[k]), d[k], l[k])
            if st[k] == 0:
                j1 = ((o.y - yref) ** 2).sum(1)
                rel.append(float(np.max(np.abs(J1[k] - j1) / np.maximum(np.abs(j1), 1e-300))))
    else:
        from oracle.dtcgpc import dtc_gpc_ww

        what = "oracle/dtcgpc.py dtc_gpc_ww (numpy, DTC_GPC_WW.m full-history lsim loop, nominal plant)"

        def run(k):
            p, m = int(N2[k]), int(Nu[k])
            dtc_gpc_ww(p=(p, p), m=(m, m), lam=tuple(l[k]), delta=tuple(d[k]))
    done, tc, picked = 0, 0.0, []
    for k in np.random.default_rng(20250307).permutation(len(N2)):
        k = int(k)
        t1 = time.perf_counter()
        try:
            run(k)
        except RuntimeError:
            continue  # an oracle self-check that gives up (toolbox_band's KKT NNLS) is not timed
        tc += time.perf_counter() - t1
        done += 1
        picked.append("%d/%d" % (N2[k], Nu[k]))
        if tc >= seconds:
            break
    if not done:
        return None
    sample = "%s on %d seeded random grid candidates (N/Nu %s), 1 thread, %.1f s" % (
        what, done, " ".join(picked), tc)
    if rel:
        sample += "; max rel |J1_gpu - J1_cpu| = %.1e" % max(rel)
    return {"value": done / tc, "unit": "sims/s", "cores": 1, "kind": "port", "sample": sample}


def lib_sha256() -> str:
    """sha256 of the libmpct.so this process loaded (mpct._lib.lib_path())."""
    import hashlib

    from mpct import _lib

    with open(_lib.lib_path(), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_traffic(C, n2, nu):
    """roofline.traffic from the committed PMC pass (profiles/pmc_latest.json, written by
    tools/pmc_summary.py from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes) -- accepted only
    when that pass profiled this very library (same sha256) on this workload; otherwise None.
    Returns (bytes per launch | None, source note, the pass's counter-derived FP64 rate | None)."""
    pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(pmc):
        return None, "no PMC pass committed", None
    try:
        with open(pmc) as f:
            pj = json.load(f)
    except (OSError, ValueError):
        return None, "unreadable profiles/pmc_latest.json", None
    mine = lib_sha256()
    src = "profiles/%s_pmc.json" % pj.get("tag", "?")
    if pj.get("lib_sha256") != mine:
        return None, "%s profiled libmpct.so sha256 %s, this run loaded %s: not used" % (
            src, str(pj.get("lib_sha256"))[:16], mine[:16]), None
    if (pj.get("candidates"), pj.get("n2"), pj.get("nu")) != (C, n2, nu):
        return None, "%s is for another workload: not used" % src, None
    return (pj.get("hbm_bytes_per_launch"), "%s (PMC pass of this libmpct.so, sha256 %s)" % (src, mine[:16]),
            pj.get("fp64_counter"))


def pmc_workload(workload, kms):
    """roofline.traffic and fp64_counter_tflops of the other §8d lines from the committed PMC pass over
    bench.py itself (profiles/pmc_workloads_latest.json, tools/pmc_workloads.sh: per-evaluation HBM bytes
    and FP64 instruction counts of the workload's kernel family) -- accepted only when that pass
    profiled this very library (same sha256); the counter rate is its flops over this run's kernel_ms.
    Returns (bytes per evaluation | None, source note, counter TFLOP/s | None)."""
    p = os.path.join(ROOT, "profiles", "pmc_workloads_latest.json")
    if not os.path.exists(p):
        return None, "no workload PMC pass committed", None
    try:
        with open(p) as f:
            pj = json.load(f)
    except (OSError, ValueError):
        return None, "unreadable profiles/pmc_workloads_latest.json", None
    mine = lib_sha256()
    src = "profiles/%s_pmc_workloads.json" % pj.get("tag", "?")
    if pj.get("lib_sha256") != mine:
        return None, "%s profiled libmpct.so sha256 %s, this run loaded %s: not used" % (
            src, str(pj.get("lib_sha256"))[:16], mine[:16]), None
    e = pj.get(workload) or {}
    fl = e.get("fp64_flops_per_evaluation")
    return (e.get("hbm_bytes_per_evaluation"),
            "%s (PMC pass of bench.py --workload %s on this libmpct.so, sha256 %s; bytes per evaluation)" % (
                src, workload, mine[:16]),
            fl / (kms * 1e-3) / 1e12 if fl else None)


def latency_roofline():
    """roofline.latency_frac from the committed latency model (profiles/latency_latest.json, written by
    tools/latency_model.py): the dependent chain of the heaviest 256 simulations priced with the
    measured primitive latencies (tools/latency_probe.hip), over their measured time -- accepted only
    when the model was fitted to this very library (same sha256).  Returns (frac | None, note)."""
    p = os.path.join(ROOT, "profiles", "latency_latest.json")
    if not os.path.exists(p):
        return None, "no latency model committed"
    try:
        with open(p) as f:
            lj = json.load(f)
    except (OSError, ValueError):
        return None, "unreadable profiles/latency_latest.json"
    mine = lib_sha256()
    if lj.get("lib_sha256") != mine:
        return None, "latency model fitted to libmpct.so sha256 %s, this run loaded %s: not used" % (
            str(lj.get("lib_sha256"))[:16], mine[:16])
    return lj.get("latency_frac"), "%s (chain model of the heaviest 256, libmpct.so sha256 %s)" % (
        lj.get("source", "profiles/latency_latest.json"), mine[:16])


def cpu_model() -> str:
    """The host CPU's model name (report the baseline's cores and CPU model)."""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--candidates", type=int, default=4096, help="candidates per GPU per step")
    ap.add_argument("--n2", type=int, default=30)
    ap.add_argument("--nu", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="thread-seconds of CPU baseline work")
    ap.add_argument("--ref-seconds", type=float, default=10.0,
                    help="seconds of the reference-structured single-thread CPU leg (0: skip)")
    ap.add_argument("--workload", default="shell3x3", choices=("shell3x3", "shell7x5", "vandevusse", "dtc-mc"),
                    help="shell3x3 = the BASELINE metric (config 2); the others are SURVEY §8d configs 3, 5, 4")
    args = ap.parse_args()
    if args.workload != "shell3x3":
        return other_workload(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        import torch.distributed as tdist

        tdist.init_process_group("nccl", device_id=dev)

    from mpct.dist import gather_costs, pad_shard, rank_candidates, shard_indices
    from mpct.engine import eval_batch_device
    from mpct.scenarios import candidate_grid, shell3x3

    sc, r, yref = shell3x3(n2_max=args.n2, nu_max=args.nu)
    Cg = args.candidates * world
    N2, Nu, d, l = candidate_grid(Cg, N2=args.n2, Nu=args.nu)
    sidx = shard_indices(Cg, world, rank)
    sN2, sNu, sd, sl = pad_shard(N2, Nu, d, l, sidx)
    # inputs resident in HBM before the timed region
    tN2 = torch.from_numpy(sN2).to(dev)
    tNu = torch.from_numpy(sNu).to(dev)
    td = torch.from_numpy(sd).to(dev)
    tl = torch.from_numpy(sl).to(dev)
    tr = torch.from_numpy(r[None].copy()).to(dev)
    C = sidx.size
    out = dict(J1=torch.empty((C, sc.my), dtype=torch.float64, device=dev),
               j22=torch.empty((C, sc.my), dtype=torch.float64, device=dev),
               status=torch.empty(C, dtype=torch.int32, device=dev),
               qp_iters=torch.empty(C, dtype=torch.int64, device=dev))
    w = torch.tensor([0.05, 0.40, 0.55], dtype=torch.float64, device=dev)  # Shell3x3.m:161
    stream = torch.cuda.current_stream(dev)
    kev = []

    def step(record):
        if record:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        eval_batch_device(sc, tN2, tNu, td, tl, tr, out, device=local, stream=stream)
        if record:
            e1.record(stream)
            kev.append((e0, e1))
        costs = gather_costs(out["J1"]) if dist else out["J1"]
        return rank_candidates(costs, w, Cg)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        order = step(True)
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist:
        te = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        tdist.all_reduce(te, op=tdist.ReduceOp.MAX)
        elapsed = float(te.item())
    kms = float(np.mean([a.elapsed_time(b) for a, b in kev]))  # ms per kernel launch
    status = out["status"].cpu().numpy()
    iters = out["qp_iters"].cpu().numpy()
    nbad = int(np.count_nonzero(status))
    I_as = float(iters.mean() / sc.nit)
    sims = world * C * args.steps
    value = sims / elapsed
    fl = algorithmic_flops_per_sim(sc, args.n2, args.nu, I_as) * C
    achieved = fl / (kms * 1e-3) / 1e12
    from mpct.engine import kernel_instance

    kernel_name = kernel_instance(sc)

    # PCIe-inclusive rate of the host-buffer entry point (mpct_eval_batch: H2D candidates,
    # kernel, D2H costs), after the timed region; reported beside `value`, never as `value`
    from mpct.engine import eval_batch

    hN2, hNu, hd, hl = sN2, sNu, sd, sl
    eval_batch(sc, hN2, hNu, hd, hl, r[None], device=local)
    t2 = time.perf_counter()
    for _ in range(3):
        eval_batch(sc, hN2, hNu, hd, hl, r[None], device=local)
    host_rate = 3 * C / (time.perf_counter() - t2)

    if rank != 0:
        if dist:
            tdist.destroy_process_group()
        return

    traffic, traffic_source, fp64c = pmc_traffic(C, args.n2, args.nu)
    lat_frac, lat_source = latency_roofline()

    cpu = None
    if not args.no_cpu_baseline and world == 1:
        # oracle/cgpc.c (C restatement of the same closed loop), timed on this host's cores
        from oracle.cport import CPort
        from oracle.scenarios import shell3x3 as o_shell3x3

        osc, orr, oyref, _ = o_shell3x3()
        cp = CPort(osc, args.n2, sc.nit, oyref)
        share, share_note = cpu_share()
        threads = max(1, args.cpu_threads or share)
        ncpu = C
        # bounded sample: repeat passes over the same batch until ~args.cpu_seconds of CPU work
        passes, tc = 0, 0.0
        while True:
            t1 = time.perf_counter()
            ref = cp.eval(N2[:ncpu], Nu[:ncpu], d[:ncpu], l[:ncpu], orr[None], threads=threads)
            tc += time.perf_counter() - t1
            passes += 1
            if tc * threads >= args.cpu_seconds or passes >= 50:
                break
        gpuJ = out["J1"].cpu().numpy()[:ncpu]
        rel = float(np.max(np.abs(gpuJ - ref["J1"]) / np.maximum(np.abs(ref["J1"]), 1e-12)))
        rate = passes * ncpu / tc
        cpu = {"value": rate, "unit": "sims/s", "cores": threads, "kind": "port",
               "per_core": rate / threads,
               "sample": "oracle/cgpc.c (C restatement, incremental recursions, same QR / dual active-set "
                         "arithmetic) on the same %d-candidate Shell 3x3 batch (N2=%d, Nu=%d, nit=500), %d passes, "
                         "%d OpenMP threads = every CPU this process may use (%s), %.2f s wall (%.0f thread-s), "
                         "%.0f sims/s per core; max rel |J1_gpu - J1_cpu| = %.1e; host %s, %d logical CPUs in "
                         "the machine" % (ncpu, args.n2, args.nu, passes, threads, share_note, tc, tc * threads,
                                          rate / threads, rel, cpu_model(), os.cpu_count() or 0)}

    cpu_ref = None
    if not args.no_cpu_baseline and world == 1 and args.ref_seconds > 0:
        cpu_ref = reference_structured_baseline(N2, Nu, d, l, out["J1"].cpu().numpy(), args.ref_seconds)

    line = {
        "metric": "closed-loop GPC sims/sec (Shell 3x3, N2=30 Nu=5) over tuning grid",
        "value": value,
        "unit": "sims/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic candidate grid (numpy default_rng(20250307)) on the reference's Shell 3x3 "
                "scenario (Shell3x3.m caso 2, L/R from Shell3x3_Tuning_25Jul2023_12_06.mat)",
        "config": {"workload": "Shell3x3 GAM scoring: %d candidates/GPU x nit=500 closed loop + J1 + "
                               "RCCL all-gather + ranking" % C,
                   "candidates_per_gpu": C, "N2": args.n2, "Nu": args.nu, "nit": sc.nit,
                   "parallelism": "dp%d" % world},
        "roofline": {"bound": "fp64-valu", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic, "traffic_source": traffic_source,
                     "kernel": kernel_name, "kernel_ms": kms,
                     "algorithmic_gflop_per_launch": fl / 1e9, "qp_iters_per_step": I_as,
                     # what the SIMDs issued, from the same sha-keyed PMC pass: every
                     # FP64 VALU wave-instruction at 64 lanes over the rocprof kernel time
                     "fp64_counter_tflops": fp64c.get("tflops") if fp64c else None,
                     # dependent-chain model time / measured time of the heaviest 256 simulations
                     # (tools/latency_model.py): how close the tail sits to its own chain
                     "latency_frac": lat_frac, "latency_source": lat_source,
                     "bound_note": "FP64 vector ALU issue + per-step dependent latency (no MFMA on this path: "
                                   "DESIGN §6); peak = MI355X FP64 vector dense peak"},
        "cpu_baseline": cpu,
        "cpu_baseline_reference_structured": cpu_ref,
        "host_api_sims_per_s": host_rate,
        "status_nonzero": nbad,
        "top_candidate": int(order[0].item()),
    }
    print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


def other_workload(args):
    """SURVEY §8d configs 3-5 through the same harness (barrier + synchronize around K timed steps,
    max over ranks, one JSON line on rank 0).  config 3 (shell7x5): the fixed 65,536-candidate
    grid of mpct.scenarios.config3_grid split over the ranks by whole cells (mpct.dist.plan_cells_lpt)
    (strong scaling, SURVEY: "65 536-candidate
    grid sharded over 8xMI355X via RCCL"); config 5 (vandevusse): 4096 NMPC candidates per GPU;
    config 4 (dtc-mc): 10,000 candidates x 32 plant-mismatch draws split over the ranks.  One
    all-gather of the per-candidate cost records, identical ranking on every rank."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        import torch.distributed as tdist

        tdist.init_process_group("nccl", device_id=dev)
    from mpct.dist import gather_and_rank, pad_shard, plan_shards
    from mpct.engine import eval_batch_device

    v = None
    nref = 1
    if args.workload == "shell7x5":
        from mpct.scenarios import SHELL7_W, config3_grid, shell7x5

        sc, r, vv, _ = shell7x5(n2_max=127, nu_max=15)
        N2, Nu, d, l = config3_grid(1024)
        refs, v = r[None], vv[None]
        w = SHELL7_W
        scaling, metric = "strong", "closed-loop band-MPC sims/sec (Shell 7x5, 65,536-candidate grid)"
        cfg = {"workload": "Shell7x5 band-mode MPC, N2 x Nu x 1024 lambda grid, nit=200, sharded", "candidates": 65536}
    elif args.workload == "vandevusse":
        from mpct.nmpc import VDV_W, nmpc_candidate_grid, vandevusse

        sc, r, _ = vandevusse()
        N2, Nu, d, l = nmpc_candidate_grid(args.candidates * world)
        refs = r[None]
        w = VDV_W
        scaling, metric = "weak", "closed-loop NMPC sims/sec (Van de Vusse, Gauss-Newton SQP)"
        cfg = {"workload": "VanDeVusse NMPC, N in 3..31, Nu in 2..15, nit=60 + open loop",
               "candidates_per_gpu": args.candidates}
    else:
        from mpct.dtc import config4_candidates, woodberry_mc

        D = 32
        sc, r, vv, _ = woodberry_mc(draws=D, n2_max=30, nu_max=10)
        Cc = 10000
        N2, Nu, d, l = config4_candidates(Cc)
        refs, v, nref = r, vv, D
        w = np.ones(2)
        scaling, metric = "strong", "closed-loop DTC-GPC sims/sec (WoodBerry, 10,000 candidates x 32 draws)"
        cfg = {"workload": "WoodBerry DTC-GPC Monte-Carlo, nit=200, sharded by candidate", "candidates": Cc,
               "draws": D}
    Cg = len(N2)
    # config 3's work varies ~100x over the grid: whole (N2, Nu) cells packed by their measured
    # one-GPU times (mpct.dist.plan_cells_lpt, the committed mpct/config3_cells.json); the others
    # strided (every rank gets the same mix of candidates)
    sidx, owners = plan_shards(N2, Nu, l, world, rank, keyed="cells" if args.workload == "shell7x5" else False,
                               nu=sc.nu)
    sN2, sNu, sd, sl = pad_shard(N2, Nu, d, l, sidx)
    C = sidx.size
    S = C * nref
    t = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in
         dict(N2=sN2, Nu=sNu, d=sd, l=sl, r=refs).items()}
    tv = torch.from_numpy(np.ascontiguousarray(v)).to(dev) if v is not None else None
    out = dict(J1=torch.empty((S, sc.my), dtype=torch.float64, device=dev),
               status=torch.empty(S, dtype=torch.int32, device=dev),
               qp_iters=torch.empty(S, dtype=torch.int64, device=dev))
    tw = torch.tensor(w, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    kev = []

    def step(record):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eval_batch_device(sc, t["N2"], t["Nu"], t["d"], t["l"], t["r"], out, v=tv, device=local, stream=stream)
        e1.record(stream)
        if record:
            kev.append((e0, e1))
        # worst case over the draws (config 4), all-gather, ranking (mpct.dist, gloo-tested)
        return gather_and_rank(out["J1"], C, nref, tw, Cg, owners=owners, distributed=dist)[1]

    steps = args.steps if args.steps != 20 else 2   # a step is a whole grid here (seconds)
    warm = args.warmup if args.warmup != 3 else 1
    for _ in range(warm):
        step(False)
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        order = step(True)
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist:
        te = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        tdist.all_reduce(te, op=tdist.ReduceOp.MAX)
        elapsed = float(te.item())
    kms = float(np.mean([a.elapsed_time(b) for a, b in kev]))
    st = out["status"].cpu().numpy()
    iters = out["qp_iters"].cpu().numpy()
    # algorithmic flops of the launch(es) over this rank's simulations (DESIGN §7 models)
    cN2 = np.repeat(sN2, nref).astype(np.int64)
    cNu = np.repeat(sNu, nref).astype(np.int64)
    live = cN2 > 0
    n_, u_, i_ = cN2[live].astype(float), cNu[live].astype(float), iters[live].astype(float)
    if args.workload == "shell7x5":
        fl = float(np.sum(band_flops_per_sim(sc, n_, u_, i_)))
        kname, ibound = "mdband_closed_loop_kernel (class launches)", "GI iterations"
    elif args.workload == "vandevusse":
        fl = float(np.sum(nmpc_flops_per_sim(n_, u_, i_, nit=sc.nit)))
        kname, ibound = "nmpc_closed_loop_kernel (class launches)", "Gauss-Newton iterations"
    else:
        from mpct.engine import kernel_instance

        kname = kernel_instance(sc)
        if kname.startswith("dtc_small_kernel"):
            # the unconstrained DTC loop as computed: no QP, first-move rows only
            fl = float(np.sum(dtc_flops_per_sim(sc, n_, u_)))
            ibound = "the DTC loop's terms (no QP)"
        else:
            # linear in the QP iterations: f(N2, Nu, 0) per horizon pair + 6 M^2 per iteration
            fl = 0.0
            for n, u in set(zip(cN2[live].tolist(), cNu[live].tolist())):
                sel = (cN2[live] == n) & (cNu[live] == u)
                fl += sel.sum() * algorithmic_flops_per_sim(sc, n, u, 0.0) + 6.0 * (sc.nu * u) ** 2 * i_[sel].sum()
            ibound = "QP iterations"
    achieved = fl / (kms * 1e-3) / 1e12
    # the PMC pass profiled one rank's whole grid: only a one-rank run evaluates the same launches
    traffic, traffic_source, fp64c = pmc_workload(args.workload, kms) if world == 1 else (
        None, "PMC pass profiled the one-GPU grid", None)
    roof = {"bound": "fp64-valu", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic, "traffic_source": traffic_source,
            "fp64_counter_tflops": fp64c, "kernel": kname, "kernel_ms": kms,
            "algorithmic_gflop_per_launch": fl / 1e9,
            "iterations_per_sim": float(iters[live].mean()) if live.any() else 0.0,
            "bound_note": "FP64 vector ALU + per-step latency; flops from the DESIGN §7 model with the "
                          "measured %s of every simulation; kernel_ms = HIP events around the whole "
                          "eval call (all class launches)" % ibound}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = other_cpu_baseline(args.workload, N2, Nu, d, l, refs, out["J1"].cpu().numpy(), st,
                                 args.cpu_seconds)
    if rank == 0:
        sims = (Cg * nref if scaling == "strong" else world * S) * steps
        line = {"metric": metric, "value": sims / elapsed, "unit": "sims/s", "n_gpus": world, "steps": steps,
                "warmup": warm, "ms_per_step": elapsed / steps * 1e3, "higher_is_better": True, "scaling": scaling,
                "vs_baseline": None, "dtype": "f64", "data": "synthetic candidate grid (seed 20250307) on the "
                "reference's scenario", "config": dict(cfg, parallelism="dp%d" % world),
                "roofline": roof, "kernel_ms_rank0": kms, "cpu_baseline": cpu,
                "status_codes": {int(k): int(n) for k, n in zip(*np.unique(st, return_counts=True))},
                "top_candidate": int(order[0].item())}
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
