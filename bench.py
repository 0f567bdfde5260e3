#!/usr/bin/env python3
"""Benchmark: MPC constraint-generation cycles/s (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): one scene, 4 obstacle vehicles, np = 5000 particles
per OV, ph = 8, v8ideal's Minkowski/MVOE constraint-generation cycle
(v8ideal/__init__.py:881-947 + the save_moments statistics): particle clouds already resident
in HBM -> per-cell moments -> every (cell, t, tau) MVOE half-space record.  One "step" = one
cycle, replayed as one hipGraph.  Synthetic seeded particle clouds (no Trajectron++ weights or
CARLA exist here).

Multi-GPU (one process per GPU): every rank plans its own independent scene (weak scaling, no
data-path collective); value = cycles completed by all ranks / max-over-ranks wall time.  Rank
0 prints ONE JSON line.  Under torchrun the ranks come from its env; `bench.py --gpus N` run
alone starts the N ranks itself as one child torchrun (launch_ranks) before any GPU call.
"""
import argparse
import glob
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "cc-mpc_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "MPC constraint-gen cycles/sec @20Hz (np=5000, ph=8); ellipsoid ΔF-norm vs ref"
HBM_PEAK = 8.0e12          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
HBM_ACHIEVABLE = 6.29e12   # MI355X_MICROARCH.md: 6.29 TB/s measured (float4 copy, 79 % of spec)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--O", type=int, default=4)
    ap.add_argument("--N", type=int, default=5000)
    ap.add_argument("--T", type=int, default=8)
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-cycles", type=int, default=200)
    ap.add_argument("--graph", action="store_true",
                    help="time hipGraph replays of the cycle instead of direct C-ABI calls")
    ap.add_argument("--no-sweep", action="store_true",
                    help="skip 'roofline_sweep' (the same kernel at C3's particle sweep, C5 and "
                         "the fused ideal rollout)")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip 'c4_sharded' (BASELINE configs[3] sharded over the ranks)")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default=None,
                    help="process-group backend for N > 1 (default nccl = RCCL; gloo only to "
                         "rehearse several ranks on one card)")
    ap.add_argument("--dist-always", action="store_true",
                    help="form the process group (nccl = RCCL) even at N = 1, so the one "
                         "exchange (c4_sharded's record all-gather) runs through RCCL on a "
                         "single card")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, report the world size and exit (no GPU work)")
    return ap.parse_args(argv)


MINPOS = np.array([150.0, -120.0])    # the sampler's scene offset (make_ovehicles' minpos)


def time_config(dev, seed, name, O, N, T, scenes, cold=True, f32=False):
    """Kernel time and algorithmic HBM rate of the one-launch cycle (and of the moment
    reduction alone) for one synthetic configuration: back to back on one store (warm: the
    Infinity Cache holds stores up to 256 MiB) and, for stores of >= 8 MB, rotating over
    distinct copies so that every launch streams from HBM (cold).  f32: the store in the
    sampler's format -- float32 relative to the scene's minpos, promoted to float64 in the
    kernel as the reference's `predictions + minpos` does (v8ideal/__init__.py:486) -- whose
    particles are 8 T bytes instead of 16 T."""
    from ccmpc import cycle, engine, synthetic
    cells, K, refs = [], [], []
    for sc in range(scenes):
        ovs, ref, _ = synthetic.scene(seed + 1000 + sc, O=O, N=N, T=T)
        cells += [c for o in ovs for c in o]
        K.append([len(o) for o in ovs])
        refs.append(ref)
    if f32:
        store = engine.ParticleStore.from_cells(cells, device=dev, dtype=torch.float32,
                                                origin=np.tile(MINPOS, (len(cells), 1)))
    else:
        store = engine.ParticleStore.from_cells(cells, device=dev)
    cyc = cycle.MinkowskiCycle(store, [k for ks in K for k in ks], np.array(refs),
                               scene_K=K)
    t = time_kernel_live(cyc.run, dev, per_graph=10, replays=5)
    tm = time_kernel_live(lambda: engine.moments(store, cyc.mean, cyc.cov, cyc.ws), dev,
                          per_graph=10, replays=5)
    b = int(sum(store.counts)) * 2 * T * (4 if f32 else 8)
    row = {"config": name, "particles": int(sum(store.counts)), "T": T,
           "halfspaces": cyc.n_constraints, "kernel_us": round(t * 1e6, 2),
           "alg_GBps": round(b / t / 1e9, 1), "frac": round(b / t / HBM_PEAK, 4),
           "moments_only_us": round(tm * 1e6, 2),
           "moments_only_frac": round(b / tm / HBM_PEAK, 4)}
    if cold:
        tc, k = cold_time(cyc, dev, store.pos.numel() * store.pos.element_size())
        if tc is not None:
            row.update({"cold_kernel_us": round(tc * 1e6, 2),
                        "cold_frac": round(b / tc / HBM_PEAK, 4), "cold_copies": k})
    return row


C4_GPU = ("C4/GPU@8: 8 scenes x 4 OVs np=20000 T=12", 4, 20000, 12, 8)


def sweep(dev, seed):
    """The one-launch cycle at the configs where the path is bandwidth-bound.
    Not part of `value`."""
    from ccmpc import engine, risk, synthetic
    configs = [("C3 np=1000 O=1 T=8", 1, 1000, 8, 1), ("C3 np=5000 O=1 T=8", 1, 5000, 8, 1),
               ("C3 np=20000 O=1 T=8", 1, 20000, 8, 1), ("C3 np=100000 O=1 T=8", 1, 100000, 8, 1),
               ("C5 O=8 np=50000 T=40", 8, 50000, 40, 1)]
    rows = [time_config(dev, seed, *c) for c in configs]
    # shrinking-horizon step: 1e6-sample ideal rollout fused with moments + half-spaces
    ovs, ref, _ = synthetic.scene(seed + 7, O=1, N=100000, T=8, K=2)
    store = engine.ParticleStore.from_cells(ovs[0], device=dev)
    mean, cov = engine.moments(store)
    src = torch.tensor([0, 1], dtype=torch.int32, device=dev)
    cr = torch.as_tensor(risk.cell_risk(risk.eps_ura([2]), [2], 8), device=dev)
    reft = torch.as_tensor(ref[None, :7], device=dev)
    ws = engine.Workspace(dev)
    fn = lambda: engine.ideal_minkowski_cycle(mean, cov, src, 7, 1_000_000, reft, cr, seed=3,
                                              workspace=ws)
    t = time_kernel_live(fn, dev, per_graph=4, replays=10)
    rows.append({"config": "ideal rollout 2 cells x 1e6 samples T=7 (fused rollout+moments+"
                           "half-spaces; 0 HBM bytes for trajectories)",
                 "particles": 2_000_000, "T": 7, "kernel_us": round(t * 1e6, 2),
                 "samples_per_s": round(2e6 * 7 / t, 1)})
    return rows


C4_FULL = {"scenes": 64, "O": 4, "N": 20000, "T": 12}


def c4_sharded(dev, seed, world, rank, steps=20, warmup=3, cfg=None, return_records=False):
    """BASELINE.json configs[3] as the node runs it: 64 independent scenes x 4 OVs x np=20000,
    ph=12, sharded over the ranks in contiguous scene blocks (ccmpc.dist.scene_range; strong
    scaling: the batch is fixed).  One step = every rank's ccmpc_minkowski_cycle over its
    scenes + the RCCL all-gather of the fixed-size half-space records (the north star's one
    exchange), timed between barriers, max over ranks.  Also the rank's kernel alone, back to
    back (warm) and rotating over distinct stores (cold HBM), as its HBM fraction."""
    from ccmpc import cycle, dist as cdist, engine, synthetic
    c = C4_FULL if cfg is None else cfg
    b, e = cdist.scene_range(c["scenes"], rank, world)
    cells, K, refs = [], [], []
    for sc in range(b, e):
        ovs, ref, _ = synthetic.scene(seed + 1000 + sc, O=c["O"], N=c["N"], T=c["T"])
        cells += [x for o in ovs for x in o]
        K.append([len(o) for o in ovs])
        refs.append(ref)
    store = engine.ParticleStore.from_cells(cells, device=dev)
    cyc = cycle.MinkowskiCycle(store, [k for ks in K for k in ks], np.array(refs), scene_K=K)
    launch = cyc.bind().launch
    gather = counts = None
    if world > 1 or _backend() is not None:     # a process group (also world 1: --dist-always)
        import torch.distributed as dist
        gloo = dist.get_backend() == "gloo"
        counts = cdist.record_counts(store.n_cells, "cpu" if gloo else dev)
        # the compact exchange: the QP's fields of each record packed to 32 bytes on the
        # device (ccmpc_compact_records) and all-gathered (a quarter of the 128-byte records)
        gather = ((lambda: cdist.gather_records(cdist.compact_records(cyc.rec).cpu(),
                                                counts=counts)) if gloo else
                  (lambda: cdist.gather_records(cyc.rec, counts=counts, compact=True)))
    gathered = [cyc.rec]

    def step():
        launch()
        if gather is not None:
            gathered[0] = gather()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev) / steps
    h = cyc.records().reshape(-1)
    ok = bool(np.all(h["status"] == 0))
    n_part = int(sum(store.counts))
    alg = n_part * 2 * c["T"] * 8
    t_warm = time_kernel_live(cyc.run, dev, per_graph=5, replays=4)
    t_cold, k = cold_time(cyc, dev, store.pos.numel() * store.pos.element_size())
    n_rec_local = cyc.n_constraints
    n_rec = sum_over_ranks(n_rec_local, world, dev)
    t_warm_max = max_over_ranks(t_warm, world, dev)
    out = {
        "config": "C4: 64 scenes x 4 OVs, np=20000/OV, ph=12, contiguous scene blocks per rank",
        "scaling": "strong", "n_gpus": world, "scenes_per_rank": e - b,
        "step_us": round(elapsed * 1e6, 2), "scenes_per_s": round(c["scenes"] / elapsed, 1),
        "constraints_per_step": int(n_rec),
        "constraints_per_s": round(n_rec / elapsed, 1),
        "record_gather": ("none (N=1)" if gather is None else
                          ("RCCL" if _backend() == "nccl" else _backend())
                          + " all_gather of every rank's compact (32-byte) records, inside the"
                          " step"),
        "gather_bytes_per_step": (None if gather is None else
                                  int(sum(counts) * (c["T"] * (c["T"] - 1) // 2) * 32)),
        "rank0": {"particles": n_part, "cells": store.n_cells, "alg_bytes_per_launch": alg,
                  "kernel_us_warm": round(t_warm * 1e6, 2),
                  "hbm_frac_warm": round(alg / t_warm / HBM_PEAK, 4)},
        "slowest_rank_kernel_us_warm": round(t_warm_max * 1e6, 2),
        "records_ok": ok,
    }
    if t_cold is not None:
        out["rank0"].update({"kernel_us_cold": round(t_cold * 1e6, 2),
                             "hbm_frac_cold": round(alg / t_cold / HBM_PEAK, 4),
                             "achievable_frac_cold": round(alg / t_cold / HBM_ACHIEVABLE, 4),
                             "cold_copies": k})
    if return_records:       # every scene's records, as the timed step's gather left them
        return out, gathered[0]
    return out


def _backend():
    import torch.distributed as dist
    return dist.get_backend() if dist.is_initialized() else None


def planning_qp(dev, seed, scenes=64, O=2, N=5000, T=8, with_cpu=True, first=0):
    """The caller side of the path: do_highlevel_control's QP
    (v8ideal/__init__.py:2850-2930) for `scenes` planning steps whose obstacles cross the ego's
    path (ccmpc.synthetic.crossing_scene: O OVs x 2 modes, N particles per OV, T steps), solved
    in one ccmpc_mpc_qp launch on the half-spaces one ccmpc_minkowski_cycle made for all of
    them.  Beside it, the oracle's dense SciPy solve of the first feasible scene (CPLEX itself
    is absent).  Not part of `value`."""
    from ccmpc import cycle, engine, mpc, synthetic
    cells, K, cps, x0s, goals, refs = [], [], [], [], [], []
    for sc in range(first, first + scenes):         # the batch's scenes first .. first+scenes-1
        c, k, ref, goal, x0, _ = synthetic.crossing_scene(seed + 5000 + sc, O=O, N=N, T=T)
        cells += c
        K.append(k)
        cps.append(len(c))
        refs.append(ref)
        goals.append(goal)
        x0s.append(x0)
    store = engine.ParticleStore.from_cells(cells, device=dev)
    cyc = cycle.MinkowskiCycle(store, [k for ks in K for k in ks], np.array(refs),
                               scene_K=K)
    cyc.run()
    xbar, gamma = mpc.ltv(np.array(x0s), T, lon=3.7)
    goal_t = torch.as_tensor(np.array(goals), device=dev)
    ref_t = torch.as_tensor(np.array(refs), device=dev)
    qp = mpc.PlanningQP(cps, T)
    fn = lambda: qp.solve(gamma, xbar, goal_t, ref_t, cyc.rec)
    t = time_kernel_live(fn, dev, per_graph=5, replays=5)
    fn()
    status, iters = qp.status.cpu().numpy(), qp.iters.cpu().numpy()
    ok = status == mpc.QP_OK
    out = {"config": f"{scenes} crossing scenes x {O} OVs x 2 modes, np={N}/OV, T={T}: one "
                     f"ccmpc_mpc_qp launch over {cyc.n_constraints} half-spaces",
           "scenes": scenes, "halfspaces": cyc.n_constraints, "kernel_us": round(t * 1e6, 2),
           "qps_per_s": round(scenes / t, 1), "solved": int(ok.sum()),
           "infeasible": int((status == mpc.QP_MAXITER).sum()),
           "iters_solved_max": int(iters[ok].max()) if ok.any() else None,
           "first_solved_scene": first + int(np.argmax(ok)) if ok.any() else None}
    if with_cpu and ok.any():
        from oracle import mpc_oracle as mo
        i = int(np.argmax(ok))
        recs = cyc.records().reshape(-1)
        xb, _, G, _, _ = mo.VehicleModel(T, 0.5, 1.85, 3.7).get_optimization_ltv(
            np.array(x0s[i]), np.zeros(2))
        P = T * (T - 1) // 2
        c0 = int(sum(cps[:i]))
        mine = recs[c0 * P:(c0 + cps[i]) * P]
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            r = mo.solve_step(G, xb, T, T, goals[i], refs[i], mine, "halfspace",
                              mo.DEFAULT_PARAMS)
            ts.append(time.perf_counter() - t0)
        out["cpu_oracle_qp_ms"] = round(statistics.median(ts) * 1e3, 2)
        out["max_abs_du_vs_oracle"] = float(np.max(np.abs(qp.u[i].cpu().numpy() - r["u"])))
        out["cpu_note"] = ("oracle/mpc_oracle.py dense assembly + SLSQP + active-set polish of "
                           "one scene, median of 5, 1 process (stand-in for cvxpy+CPLEX, absent)")
    return out


def bench_backend(args):
    """nccl (= RCCL over xGMI) unless --backend / CCMPC_BENCH_BACKEND says gloo, which exists
    only to rehearse the N > 1 code path with several ranks on one card (RCCL will not form a
    communicator from two ranks on one device)."""
    return args.backend or os.environ.get("CCMPC_BENCH_BACKEND", "nccl")


def launcher_argv(args, argv, env):
    """The child command that starts `--gpus N` ranks, or None when this process is already a
    rank (torchrun set WORLD_SIZE) or N == 1.  `python -m torch.distributed.run` as a CHILD
    process of a parent that has not touched the GPU (no exec; counting devices does not
    initialise HIP): one process per GPU, rendezvous on 127.0.0.1."""
    if args.gpus <= 1 or "WORLD_SIZE" in env:
        return None
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
            f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(args):
    """`bench.py --gpus N` run directly (not under torchrun): start the N ranks as one child
    torchrun and return its exit code; rank 0 of the child prints the JSON line on the inherited
    stdout.  None when this process should run the benchmark itself."""
    cmd = launcher_argv(args, sys.argv[1:], os.environ)
    if cmd is None:
        return None
    if bench_backend(args) == "nccl" and not args.launch_check:
        have = torch.cuda.device_count()          # does not initialise HIP on this image
        if have < args.gpus:
            raise SystemExit(f"--gpus {args.gpus} needs {args.gpus} visible GPUs, found {have} "
                             "(--backend gloo rehearses several ranks on one card)")
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["CCMPC_BENCH_SPAWNED"] = "1"
    if args.backend:
        env["CCMPC_BENCH_BACKEND"] = args.backend
    return subprocess.run(cmd, env=env).returncode


def init_dist(args):
    """One process per GPU (torchrun env), checked against --gpus on every path."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch with torchrun "
                         f"--nproc-per-node {args.gpus}, or run bench.py --gpus N alone")
    if world > 1 or getattr(args, "dist_always", False):
        import torch.distributed as dist
        backend = bench_backend(args)
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29531")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.launch_check:                       # launcher rehearsal: no GPU touched
            dist.init_process_group("gloo")
        elif backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:       # the one-card rehearsal: every rank on device 0 (device_count() may
            torch.cuda.set_device(0)   # count cards this process cannot open)
            dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    return world, rank, local


def launch_check(world, rank):
    """--launch-check: every rank reports what the launcher gave it (no GPU work); rank 0
    prints one JSON line.  Used by the CPU test of the launcher."""
    ranks = [rank]
    if world > 1:
        import torch.distributed as dist
        got = [None] * world
        dist.all_gather_object(got, {"rank": rank, "world": dist.get_world_size()})
        ranks = [g["rank"] for g in got]
        assert all(g["world"] == world for g in got)
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks": ranks}), flush=True)


def barrier(world):
    if world > 1 or _backend() is not None:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    import torch.distributed as dist
    gloo = dist.get_backend() == "gloo"
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if gloo else dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world, dev):
    if world == 1:
        return x
    import torch.distributed as dist
    gloo = dist.get_backend() == "gloo"
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if gloo else dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def time_kernel_live(fn, dev, per_graph=50, replays=20):
    """Average device time of one launch of `fn`: `per_graph` launches captured back to back
    into one hipGraph, replayed `replays` times between two HIP events on the capturing
    stream (no host launch overhead in the interval; each launch still pays its kernel
    boundary, which rocprof's per-kernel duration does not include).  `fn` may be a list of
    callables: launch i runs fn[i % len(fn)] (rotation over distinct buffers, cold_copies)."""
    fns = list(fn) if isinstance(fn, (list, tuple)) else [fn]
    per_graph = max(per_graph, len(fns))
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            for f in fns:
                f()
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(per_graph):
            fns[i % len(fns)]()
    g.replay()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(replays):
        g.replay()
    ev1.record()
    ev1.synchronize()
    return ev0.elapsed_time(ev1) * 1e-3 / (per_graph * replays)


MALL_BYTES = 256 << 20     # MI355X_MICROARCH.md: 256 MiB Infinity Cache in front of HBM


def cold_copies(store_bytes, cap=64):
    """Distinct copies of a store to rotate through so that every launch reads HBM, not the
    Infinity Cache (FETCH_SIZE counts its hits): >= 3 copies and >= 2x the cache in total; None
    when that would take more than `cap` copies (small stores are latency-bound anyway)."""
    k = max(3, -(-2 * MALL_BYTES // max(int(store_bytes), 1)))
    return k if k <= cap else None


def clone_cycle(cyc):
    """The same cycle over a fresh copy of its particle store (own buffers and workspace)."""
    import copy
    from ccmpc import cycle
    st = copy.copy(cyc.store)
    st.pos = cyc.store.pos.clone()
    c = cycle.MinkowskiCycle.__new__(cycle.MinkowskiCycle)
    c.__dict__.update(cyc.__dict__)
    c.store = st
    c.mean, c.cov = torch.empty_like(cyc.mean), torch.empty_like(cyc.cov)
    c.rec, c.prob_lower = torch.empty_like(cyc.rec), torch.empty_like(cyc.prob_lower)
    from ccmpc import engine
    c.ws = engine.Workspace(st.device)
    c.ws.get(cyc.ws.buf.numel())
    c.graph = None
    return c


def cold_time(cyc, dev, store_bytes):
    """Average launch time with every launch reading its particles from HBM (rotation over
    cold_copies distinct stores), or None for stores too small to rotate."""
    k = cold_copies(store_bytes)
    if k is None:
        return None, None
    cycles = [cyc] + [clone_cycle(cyc) for _ in range(k - 1)]
    t = time_kernel_live([c.run for c in cycles], dev, per_graph=4 * k, replays=3)
    del cycles
    torch.cuda.empty_cache()
    return t, k


def host_cpu():
    """CPU model and logical core count of this host (the box's CPU share is 16 of them)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "logical_cores": os.cpu_count()}


def cpu_baseline(ovs, ref, T, cycles):
    """The oracle's loop-faithful restatement of v8ideal/__init__.py:881-947 on this host:
    `cycles` full cycles with BLAS at 1 thread (~10 s at C2), then a short run with BLAS at
    min(16, cores) threads (the GPU box's CPU share is 16); the faster median is reported."""
    from threadpoolctl import threadpool_limits

    from oracle import ccmpc_oracle as orc
    import scipy.stats
    chi_p = scipy.stats.chi2.ppf(orc.TARGET_P, df=2)
    O = len(ovs)

    def one_cycle():
        for o, cells in enumerate(ovs):
            for k, traj in enumerate(cells):
                eps = (orc.EPS_TOTAL / O) / T
                chi_r = scipy.stats.chi2.ppf(1 - eps, df=2)
                orc.minkowski_cell(np.vstack(traj), T, T, ref, eps, chi_r, chi_p)

    best, total = None, 0.0
    for threads, n in ((1, cycles), (min(16, os.cpu_count() or 1), max(cycles // 5, 5))):
        with threadpool_limits(limits=threads):
            for _ in range(2):
                one_cycle()
            ts = []
            for _ in range(n):
                t0 = time.perf_counter()
                one_cycle()
                ts.append(time.perf_counter() - t0)
        total += sum(ts)
        med = statistics.median(ts)
        if best is None or med < best[0]:
            best = (med, threads, n)
    return best[0], best[1], best[2], total


def episode_c1(dev, cpu_steps=2, with_cpu=True, N=5000):
    """BASELINE configs[0] (tests/Hz20/test_montecarlo.py v8ideal scene4_ov1_brake ph8
    np5000): one obstacle, the full planning schedule of an episode through
    MidlevelAgent -- 8 shrinking Minkowski steps (T = 8..1; T < 8 on 1e6-sample predict_ideal
    rollouts) and 4 receding GMM-affine steps -- each step end to end (GPU sampler -> bucketing
    -> one fused launch -> host HalfSpace objects), synchronised.  Beside it, the oracle on the
    first `cpu_steps` planning steps with the same particles and the same Philox draws."""
    from ccmpc import episode
    rep = episode.EpisodeReplay(O=1, N=N, ph=8, n_ideal=1_000_000, receding_steps=4,
                                device=dev)
    first = rep.run()         # the first episode: allocations, every step's calls eager
    second = rep.run()        # the second: each shape's graphs captured at its second launch
    log = rep.run()           # from then on every step is a graph replay
    out = {"config": f"C1 schedule: 1 OV, np={N}, ph=8, n_ideal=1e6, 8 shrinking + 4 receding "
                     "planning steps (synthetic GMM predictions), each step one graph replay "
                     "(sampler -> bucketing -> generator) + the QP",
           "steps": [{k: (round(v, 3) if k in ("ms", "qp_ms") else v) for k, v in st.items()}
                     for st in log],
           "total_ms": round(sum(st["ms"] for st in log), 3),
           "total_qp_ms": round(sum(st.get("qp_ms", 0.0) for st in log), 3),
           "first_episode_total_ms": round(sum(st["ms"] + st.get("qp_ms", 0.0)
                                               for st in first), 3),
           "second_episode_total_ms": round(sum(st["ms"] + st.get("qp_ms", 0.0)
                                                for st in second), 3),
           "note": "total_ms = the generator side of every step (host clock, synchronised), "
                   "total_qp_ms the QP after it, in the agent's third episode (steady state: "
                   "every step a graph replay); a shape's first launch runs its calls eagerly "
                   "(first_episode_total_ms, allocations included), its second captures the "
                   "graphs (second_episode_total_ms, captures included)"}
    if not with_cpu:
        return out
    from oracle import ccmpc_oracle as orc
    rep = episode.EpisodeReplay(O=1, N=5000, ph=8, n_ideal=1_000_000, receding_steps=0,
                                device=dev, with_qp=False)
    cpu = []
    mom = None
    for frame, T, kind in rep.schedule()[:cpu_steps]:
        ovs, _ = rep.step(frame, T, kind)
        K = [ov.n_states for ov in ovs]
        cells = [[np.asarray(p, float) for p in ov.pred_positions] for ov in ovs]
        pasts = [np.asarray(ov.past, float).reshape(-1, 2) for ov in ovs]
        t0 = time.perf_counter()
        oovs = [orc.OVehicle(T, pasts[o], np.ones(K[o]) / K[o], cells[o],
                             [orc._step_yaws(c, pasts[o][-1], rep.ph) for c in cells[o]],
                             np.zeros((K[o], 2)), np.array([4.5, 2.5])) for o in range(len(K))]
        if T == rep.ph:
            orc.minkowski_generator(oovs, T, rep.ph, rep.ref_traj(frame), with_l4=False)
            mom = orc.save_moments(cells, T)
        else:
            ideal = orc.predict_ideal(mom, K, T, 1_000_000, seed=frame)
            orc.minkowski_generator(oovs, T, rep.ph, rep.ref_traj(frame), ideal_trajs=ideal,
                                    with_l4=False)
            mom = orc.save_moments([[ideal[o][k] for k in range(K[o])]
                                    for o in range(len(K))], T)
        cpu.append({"frame": frame, "T": T, "ms": round((time.perf_counter() - t0) * 1e3, 1)})
    out["cpu_oracle_sample"] = {
        "steps": cpu, "cores": 1, "kind": "port",
        "note": "oracle restatement of v8ideal/__init__.py:781-964 + :2620-2711 on the first "
                f"{cpu_steps} planning steps (generators only; no sampler, no bucketing)"}
    return out


def dropin_step_predictions(dev, steps=300, O=4, N=5000, ph=8, n_sets=8, on_device=False):
    """The planning step on the reference's own predictor output: generate_vehicle_latents'
    5-tuple (prediction.py:93-105) -- predictions (nodes, N, ph, 2) float32 and z (nodes, N)
    int64 as the host numpy arrays the reference returns, the ego's node in row 0 -- through
    MidlevelAgent.predict_and_constrain with StepGraph(source="predictions"): the arrays go into
    the pinned input pack, ccmpc_bucket_predictions (make_ovehicles, :469-505: one placement
    pass) -> the Minkowski cycle -> L4 -> 9-tuple; no sampler.  on_device: the same arrays as
    device tensors (generate_vehicle_latents(..., keep_on_device=True), a predictor on the same
    GPU): the step graph reads them in place (their addresses in the input pack,
    ccmpc_bucket_predictions_indirect), nothing crosses PCIe.  `n_sets` precomputed frames of particles (the sampler's own draws) are cycled, a
    different one each step."""
    from ccmpc import engine, episode, planner
    init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=20251015)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]])
             for o in range(O)]
    K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
    eps = np.full((O, max(K)), 0.05 / O)
    ego = np.array([165.0, -72.0])
    ref = np.array([ego + [4.0 * (t + 1), 0.5 * (t + 1)] for t in range(ph)])
    sets = []
    for k in range(n_sets):
        z, store = engine.sample_unicycle(init, pmf, gmm, N, ph, seed=900 + k, device=dev)
        pos = store.pos.cpu().numpy()
        pred = np.zeros((O + 1, N, ph, 2), np.float32)
        for o in range(O):
            off = store.offsets[o]
            pred[o + 1] = pos[:, off:off + N].reshape(ph, 2, N).transpose(2, 0, 1)
        zz = np.zeros((O + 1, N), np.int64)
        zz[1:] = z.cpu().numpy()
        if on_device:
            pred, zz = torch.as_tensor(pred, device=dev), torch.as_tensor(zz, device=dev)
        sets.append(dict(source="predictions", predictions=pred, z=zz,
                         rows=list(range(1, O + 1)), latent_pmf=pmf, N=N))
    agent = planner.MidlevelAgent(prediction_horizon=ph, device=dev)
    params = episode.Params(O, K, 0)

    def one(i):
        return agent.predict_and_constrain(params, sets[i % n_sets], eps, ph, ref, minpos,
                                           pasts)
    for i in range(20):
        one(i)
    ts = []
    for i in range(steps):
        t0 = time.perf_counter()
        _, out = one(i)
        ts.append(time.perf_counter() - t0)
    g = next(iter(agent._graphs.values()))
    t_graph = time_graph_replay(g, dev)
    cfg = ("step_pred_" + ("dev_" if on_device else "") +
           ("c2" if (O, N) == (4, 5000) else "100k" if (O, N) == (1, 100_000) else "x"))
    where = ("device tensors (keep_on_device) read in place" if on_device else
             "host numpy predictions / z in the pinned pack")
    return {"config": f"drop-in step on generate_vehicle_latents' 5-tuple: {O} OVs (+ the "
                      f"ego's node) x np={N} x ph={ph}, K={K}; {where} -> "
                      "ccmpc_bucket_predictions(_indirect) -> Minkowski cycle -> L4 -> 9-tuple",
            "steps": steps, "constraints_per_step": len(out[0]),
            "graph_branch": f"source={g.source}, fused={g.fused}",
            "input_pack_bytes": int(g.inp.nbytes),
            "dropin_step_us_median": round(statistics.median(ts) * 1e6, 1),
            "dropin_step_us_p90": round(float(np.percentile(ts, 90)) * 1e6, 1),
            "graph_replay_us": round(t_graph * 1e6, 1),
            "record_path_latency_us": round(time_record_path(g, dev) * 1e6, 1),
            "roofline": step_roofline(g, t_graph, cfg, predictions=True)}


def v8_milp(dev, with_cpu=True, seeds=range(20, 28), T=8, O=2):
    """v8's MILP (v8/__init__.py:692-873, road boundaries off) through
    MidlevelAgentV8.do_highlevel_control: big-M rows over the device L4 faces of crossing OV
    clouds, the exact branch and bound on the GPU (each round one batched mpc_qp_kernel launch).
    Beside it the oracle's branch and bound (SciPy QPs) on the same rows, on one host core."""
    from ccmpc import milp, ovehicle, synthetic
    from ccmpc.standins import AttrDict
    rows_ = []
    for seed in seeds:
        cells, K, ref, goal, x_init, pasts = synthetic.crossing_scene(seed, O=O, N=600, T=T, K=1,
                                                                      lateral=6.0)
        ovs = ovehicle.scene_from_positions([[c] for c in cells],
                                            [p.reshape(1, 2) for p in pasts], device=dev)
        agent = milp.MidlevelAgentV8(prediction_horizon=T, control_horizon=T, device=dev)
        params = AttrDict(x_init=x_init, goal=goal, diag=milp.ego_diag(3.7, 1.79), O=O, K=K)
        # warm: allocations, then the round graphs (each round shape is captured at its second
        # use): the timed call is a steady-state frame, on a fresh scene of the same particles
        # (so its L4 and the L4's copy to the host are inside the frame, as they are for a new
        # prediction)
        agent.do_highlevel_control(params, ovs)
        agent.do_highlevel_control(params, ovs)
        ovs = ovehicle.scene_from_positions([[c] for c in cells],
                                            [p.reshape(1, 2) for p in pasts], device=dev)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out, err = agent.do_highlevel_control(params, ovs)
        t_gpu = time.perf_counter() - t0
        r = {"seed": seed, "feasible": err is None, "ms": round(t_gpu * 1e3, 3),
             "nodes": agent.last_bnb["nodes"], "launches": agent.last_bnb["launches"]}
        if with_cpu:
            from oracle import mpc_oracle as mo
            rows = agent.compute_obstacle_constraints(params, ovs, None, None, None, None)[0]
            xb, _, G, _, _ = mo.VehicleModel(T, 0.5, 1.85, 3.7).get_optimization_ltv(
                x_init, np.zeros(2))
            t0 = time.perf_counter()
            want = mo.milp_bnb(G, xb, T, goal, rows.A, rows.rhs)
            r["oracle_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
            r["same_verdict"] = (want is None) == (err is not None)
            if want is not None and err is None:
                r["max_du"] = float(np.abs(out.U_star.reshape(-1) - want["u"]).max())
        rows_.append(r)
    solved = [r for r in rows_ if r["feasible"]]
    return {"config": f"v8 MILP: {O} crossing OVs x np=600, T={T}, L4 faces, big-M disjunction "
                      "(M_big = 1e4), road boundaries off; exact best-first branch and bound, "
                      "one batched QP launch per round (do_highlevel_control, host clock)",
            "scenes": rows_,
            "ms_median_solved": (round(statistics.median(r["ms"] for r in solved), 3)
                                 if solved else None)}


def harness_episode(dev, N=5000, run_interval=12, episodes=3):
    """The reference harness's own driver sequence (tests/Hz20/__init__.py:183-359) through the
    library: MidlevelAgent's reference constructor, then run_step(frame, offline_index, T,
    shrinking) every simulator frame (burn frames, 8 shrinking Minkowski plans, receding affine
    plans), CARLA / Trajectron++ replaced by ccmpc.standins (1 OV at C1's scene-4 shape,
    Trajectron++'s per-particle boundary as device tensors).  Reports run_step's host time per
    planning frame (prediction boundary -> graph step -> QP -> warm start) and per episode; each
    episode builds a fresh agent as the harness does and destroys it at the end, releasing its
    step graphs to the pool the next episode's agent takes them from."""
    from ccmpc import harness, standins
    stg = standins.SyntheticTrajectron(L=25, ph=8, seed=5, per_particle=True, device=dev)

    def make_world():
        return standins.town03_scene(n_ov=1, ego_xy=(60.0, 81.76), ego_speed=8.0, ov_gap=20.0,
                                     ov_speed=8.0, ov_lateral=40.0)
    route = make_world()[3].route_points[::2]
    res = []
    for e in range(episodes):
        scen = harness.MonteCarloScenario(
            harness.ScenarioParameters(n_burn_interval=4, run_interval=run_interval),
            harness.CtrlParameters(n_predictions=N, prediction_horizon=8, control_horizon=8),
            make_world, stg, agent_kwargs=dict(n_ideal=1_000_000, reference_trajectory=route,
                                               device=dev))
        t0 = time.perf_counter()
        stats = scen.episode(e)
        wall = time.perf_counter() - t0
        res.append({"episode": e, "wall_ms": round(wall * 1e3, 2), "plans": len(scen.steps),
                    "infeasible": bool(stats.infeasibility),
                    "plan_ms": [round(st["run_step_ms"], 3) for st in scen.steps],
                    "T": [st["T"] for st in scen.steps]})
    return {"config": f"tests/Hz20 MonteCarloScenario loop: 1 OV, n_predictions={N}, ph=8, "
                      f"n_ideal=1e6, {run_interval} planning periods after 4 burn periods "
                      "(10 simulator frames each), per-particle GMM boundary",
            "episodes": res,
            "note": "plan_ms = run_step's host time on a planning frame (synchronous: the QP's "
                    "answer is on the host when it returns); wall_ms = the whole episode "
                    "including the 10x more non-planning frames and the agent's construction; "
                    "each episode builds a fresh agent and destroys it at the end (tests/Hz20/"
                    "__init__.py:383-399): episode 0 runs every shape's calls eagerly, episode "
                    "1 takes the released graphs from the pool and captures them, episode 2 "
                    "replays them"}


def pp_sampler_draws(pmf, gmm, N, T, seed, dev):
    """Device tensors shaped as Trajectron++ hands them over (prediction.py:81-86): z ~ p(z|x)
    (torch.multinomial: the one-hot sample's argmax, :103), every sample's own GMM parameters
    (the latent's row + a per-sample perturbation, as an autoregressive decoder's outputs differ
    per sample), and GMM2D.rsample's standard-normal noise."""
    g = torch.Generator(device=dev).manual_seed(int(seed))
    O = pmf.shape[0]
    z = torch.multinomial(torch.as_tensor(pmf, device=dev), N, replacement=True,
                          generator=g).to(torch.int32)
    base = torch.as_tensor(gmm, device=dev)
    pp = torch.stack([base[o][z[o].long()] for o in range(O)])
    pp = pp + 0.02 * torch.randn(pp.shape, device=dev, generator=g)
    pp[..., 4].clamp_(-0.9, 0.9)
    eps = torch.randn((O, N, T, 2), device=dev, generator=g)
    return pp.float().contiguous(), z, eps


def dropin_step(dev, steps=300, with_cpu=True, O=4, N=5000, ph=8, per_particle=False,
                eager_steps=50, cpu_reps=5, label="C2 shape"):
    """The drop-in planning step through MidlevelAgent.predict_and_constrain: do_prediction
    (the sampler tail) + make_ovehicles + compute_obstacle_constraints_GMM_Minkowski_
    idealprediction (v8ideal/__init__.py:414-505, :781-964) -- one hipGraph replay per step
    with the packed input upload and the record / moment / L4 download inside it, then the
    9-tuple on the host (constraints built lazily).  Default: C2's shape (O = 4, np = 5000,
    ph = 8) in the synthetic per-latent sampler mode, a fresh Philox seed per step.
    per_particle: the upstream boundary instead -- every sample's GMM parameters, z and the
    noise as device tensors (pp_sampler_draws), copied device-to-device into the graph's
    buffers inside each timed step.  N > 8192 takes the graph's non-fused branch (sampler, then
    ccmpc_bucket).  Beside it: the same step through the eager drop-in calls, and the oracle's
    make_ovehicles + Minkowski generator (with vertices / L4) on the same sampler output, on one
    host core."""
    from ccmpc import engine, episode, ovehicle, planner
    init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=20251015)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]])
             for o in range(O)]
    K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
    eps = np.full((O, max(K)), 0.05 / O)
    ego = np.array([165.0, -72.0])
    ref = np.array([ego + [4.0 * (t + 1), 0.5 * (t + 1)] for t in range(ph)])
    agent = planner.MidlevelAgent(prediction_horizon=ph, device=dev)
    params = episode.Params(O, K, 0)
    draws = pp_sampler_draws(pmf, gmm, N, ph, 7, dev) if per_particle else None

    def sampler_of(seed):
        if per_particle:
            return dict(init_state=init, latent_pmf=pmf, gmm=draws[0], z=draws[1], eps=draws[2],
                        N=N, seed=seed, per_particle=True)
        return dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=seed)

    def graph_step(seed):
        return agent.predict_and_constrain(params, sampler_of(seed), eps, ph, ref, minpos,
                                           pasts)

    for i in range(20):
        graph_step(i)
    ts = []
    for i in range(steps):
        t0 = time.perf_counter()
        _, out = graph_step(1000 + i)
        ts.append(time.perf_counter() - t0)
    n_cons = len(out[0])
    g = next(iter(agent._graphs.values()))
    t_graph = time_graph_replay(g, dev)
    t_rec = time_record_path(g, dev)

    eager = planner.MidlevelAgent(prediction_horizon=ph, device=dev)

    def eager_step(seed):
        s = sampler_of(seed)
        z, store = engine.sample_unicycle(init, pmf, s["gmm"], N, ph, seed=seed, device=dev,
                                          z=s.get("z"), eps=s.get("eps"),
                                          per_particle=per_particle)
        ovs = ovehicle.make_ovehicles(store, z, pmf, minpos, pasts, device=dev)
        return eager.compute_obstacle_constraints_GMM_Minkowski_idealprediction(
            params, ovs, None, None, None, eps, None, ph, ref)

    for i in range(5):
        eager_step(i)
    te = []
    for i in range(eager_steps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        eager_step(2000 + i)
        te.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    mode = ("per-particle GMM parameters + z + noise as device tensors (Trajectron++'s "
            "boundary, prediction.py:81-86)" if per_particle
            else "synthetic per-latent GMM, Philox z and noise")
    res = {"config": f"{label} drop-in step: {O} OVs x np={N} x ph={ph}, L=25 latent values, "
                     f"K={K} kept modes; {mode}; sampler -> bucketing -> Minkowski cycle -> L4 "
                     "-> 9-tuple (MidlevelAgent.predict_and_constrain)",
           "steps": steps, "constraints_per_step": n_cons,
           "graph_branch": "fused sampler+bucketing" if g.fused else "sampler -> ccmpc_bucket",
           "dropin_step_us_median": round(med * 1e6, 1),
           "dropin_step_us_p90": round(float(np.percentile(ts, 90)) * 1e6, 1),
           "graph_replay_us": round(t_graph * 1e6, 1),
           "record_path_latency_us": round(t_rec * 1e6, 1),
           "roofline": step_roofline(g, t_graph, None if per_particle else (
               "step_c2" if (O, N) == (4, 5000) else
               "step_c1_100k" if (O, N) == (1, 100_000) else None)),
           "eager_calls_step_us_median": round(statistics.median(te) * 1e6, 1),
           "note": "wall clock per call on the host, host inputs from host memory (per-particle "
                   "tensors: device-to-device copies inside the step), outputs (records, "
                   "moments, statistics) on the host when it returns (polled signal), the L4 "
                   "outputs (the graph's parallel branch) read on access; graph_replay_us = HIP "
                   "events around back-to-back replays of the whole step graph (packed H2D + "
                   "sampler + bucketing, then the cycle + packed D2H beside L4 + its D2H); "
                   "record_path_latency_us = host time from launch to the records on the host "
                   "(launch + the record path's GPU time + the signal), no host work between"}
    if with_cpu:
        from oracle import ccmpc_oracle as orc
        s = sampler_of(7)
        z, store = engine.sample_unicycle(init, pmf, s["gmm"], N, ph, seed=7, device=dev,
                                          z=s.get("z"), eps=s.get("eps"),
                                          per_particle=per_particle)
        zc = z.cpu().numpy()
        pred = np.stack([store.cell_positions(o) for o in range(O)]).astype(np.float32)
        tc = []
        for _ in range(cpu_reps):
            t0 = time.perf_counter()
            oovs = orc.make_ovehicles(pred, zc, pmf, minpos, pasts, [np.array([4.5, 2.5])] * O,
                                      ph)
            orc.minkowski_generator(oovs, ph, ph, ref, with_l4=True)
            tc.append(time.perf_counter() - t0)
        cpu = statistics.median(tc)
        res["cpu_oracle_step_ms"] = round(cpu * 1e3, 2)
        res["speedup_vs_cpu_step"] = round(cpu / med, 1)
        res["cpu_note"] = ("oracle make_ovehicles + Minkowski generator with vertices/L4 on the "
                           "same sampler output, median of 5, 1 BLAS thread (the reference "
                           "path's own work; its Trajectron++ sampler is not counted)")
    return res


def time_graph_replay(g, dev, n=200):
    """HIP-event time per step of a captured planning step's graph (both branches: the record
    path and L4), the two parity graphs replayed back to back."""
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h = torch.cuda.current_stream(dev).cuda_stream

    def one(i):
        g.graphs[i & 1].replay(h)

    for i in range(10):
        one(i)
    torch.cuda.synchronize(dev)
    ev0.record()
    for i in range(n):
        one(i)
    ev1.record()
    ev1.synchronize()
    return ev0.elapsed_time(ev1) * 1e-3 / n


def time_record_path(g, dev, n=200):
    """Median host time from a step's launch to its records on the host (the graph's record-path
    signal; the L4 branch may still run), the inputs unchanged."""
    ts = []
    for _ in range(10):
        g.replay()
    for _ in range(n):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        g.launch()
        g.wait()
        ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize(dev)
    return statistics.median(ts)


def step_roofline(g, t_graph, config, predictions=False):
    """The planning step's roofline: ALGORITHMIC bytes per step over the graph's replay time
    (HIP events, both branches).  Per particle (T = ph steps, f32 positions): the placement's
    write of the bucketed store (8 T B), the cycle's read (8 T), the L4 passes' two reads
    (16 T) and the latent id written and read (8) = 32 T + 8 B; the predictor's route adds its
    input, the predictions and z read once (8 T + 8).  `traffic` = the HBM bytes per step of
    every kernel of the step from the committed PMC summary of this configuration
    (profiles/r*/configs/<config>_summary.json, tools/step_replay.py under
    profiles/collect_configs.sh: FETCH_SIZE x2 + WRITE_SIZE, each kernel weighted by its calls
    per step), with the kernels' summed time per step beside it."""
    T, n = g.ph, g.O * g.N
    alg = n * (32 * T + 8 + ((8 * T + 8) if predictions else 0))
    out = {"bound": "hbm", "alg_bytes_per_step": alg, "graph_us": round(t_graph * 1e6, 2),
           "achieved": round(alg / t_graph / 1e9, 2), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
           "frac": round(alg / t_graph / HBM_PEAK, 5), "traffic": None,
           "formula": "particles x (32 T + 8)" + (" + particles x (8 T + 8)" if predictions
                                                   else "")}
    rounds = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*")))
    for rdir in reversed(rounds):
        path = os.path.join(rdir, "configs", f"{config}_summary.json")
        if not os.path.exists(path):
            continue
        with open(path) as f:
            summ = json.load(f)
        steps = max((d.get("calls", 0) for k, d in summ.items()
                     if k.startswith("void ccmpc::latent_count_kernel")), default=0)
        if not steps:
            break
        b = sum(d.get("hbm_bytes_avg", 0.0) * d.get("calls", 0) / steps for d in summ.values())
        busy = sum(d.get("avg_ns", 0.0) * d.get("calls", 0) / steps for d in summ.values())
        out.update(traffic=int(b), counter_over_alg=round(b / alg, 3),
                   kernel_us_per_step=round(busy / 1e3, 2),
                   traffic_source=os.path.relpath(path, ROOT))
        break
    return out


def pmc_traffic(kernel_prefix, config=None):
    """HBM bytes per launch of a kernel from the newest committed PMC summary: the
    per-configuration one (profiles/<round>/configs/<config>_summary.json, written by
    profiles/collect_configs.sh: that configuration's launches only) when `config` is given and
    one exists, else profiles/<round>/summary.json (profiles/collect.sh).  FETCH_SIZE x2
    (gfx950) + WRITE_SIZE.  kernel_prefix stops before the balanced-mode template flag, so both
    names match.  (None, None) when nothing is committed."""
    rounds = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*")))
    for rdir in reversed(rounds):
        paths = ([os.path.join(rdir, "configs", f"{config}_summary.json")] if config else [])
        paths.append(os.path.join(rdir, "summary.json"))
        for path in paths:
            if not os.path.exists(path):
                continue
            with open(path) as f:
                summ = json.load(f)
            for name, d in summ.items():
                if name.startswith(kernel_prefix) and "hbm_bytes_avg" in d:
                    return int(d["hbm_bytes_avg"]), os.path.relpath(path, ROOT)
    return None, None


def pcie_inclusive(cyc, step, dev, iters=200):
    """Cycles/s when the boundary is handed HOST particles: pinned H2D of the whole particle
    store, the cycle step, pinned D2H of every record; synchronised per cycle (the planner
    needs the records before its QP).  Reported beside `value`, never as it."""
    host_pos = torch.empty(cyc.store.pos.shape, dtype=cyc.store.pos.dtype, pin_memory=True)
    host_pos.copy_(cyc.store.pos)
    host_rec = torch.empty(cyc.rec.shape, dtype=cyc.rec.dtype, pin_memory=True)
    for _ in range(5):
        cyc.store.pos.copy_(host_pos, non_blocking=True)
        step()
        host_rec.copy_(cyc.rec, non_blocking=True)
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(iters):
        cyc.store.pos.copy_(host_pos, non_blocking=True)
        step()
        host_rec.copy_(cyc.rec, non_blocking=True)
        torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / iters
    return {"cycles_per_s": round(1.0 / dt, 1), "us_per_cycle": round(dt * 1e6, 2),
            "h2d_bytes": host_pos.numel() * host_pos.element_size(),
            "d2h_bytes": host_rec.numel()}


def ellipsoid_parity(ovs, ref, T, h):
    """The metric's second half (BASELINE.json: "ellipsoid ΔF-norm vs ref"): the timed cycle's
    records against the oracle's restatement of v8ideal/__init__.py:881-947 on the same
    particles (golden-pinned to makeconstraint.py) -- the largest relative Frobenius error of
    the ellipsoid shapes Q and QR and of the centre, and whether record order, `which` and
    `side` agree bit for bit.  Bar: 1e-5 relative (BASELINE.json)."""
    import scipy.stats
    from oracle import ccmpc_oracle as orc
    chi_p = scipy.stats.chi2.ppf(orc.TARGET_P, df=2)
    eps = (orc.EPS_TOTAL / len(ovs)) / T
    chi_r = scipy.stats.chi2.ppf(1 - eps, df=2)
    want = []
    for cells in ovs:
        for traj in cells:
            want += orc.minkowski_cell(np.vstack(traj), T, T, ref, eps, chi_r, chi_p)[0]
    dq = dqr = dc = 0.0
    exact = len(want) == len(h)
    for r, g in zip(want, h):
        Q = np.array([[g["q00"], g["q01"]], [g["q01"], g["q11"]]])
        QR = np.array([[g["r00"], g["r01"]], [g["r01"], g["r11"]]])
        c = np.array([g["mean0"], g["mean1"]])
        dq = max(dq, float(np.linalg.norm(Q - r["Q"]) / np.linalg.norm(r["Q"])))
        dqr = max(dqr, float(np.linalg.norm(QR - r["QR"]) / np.linalg.norm(r["QR"])))
        dc = max(dc, float(np.linalg.norm(c - r["mean"]) / np.linalg.norm(r["mean"])))
        exact = exact and (int(g["which"]), int(g["side"]), int(g["t_tau"]) >> 16,
                           int(g["t_tau"]) & 0xFFFF) == (r["which"], r["side"], r["t"], r["tau"])
    return {"Q_rel_fro_max": dq, "QR_rel_fro_max": dqr, "centre_rel_max": dc,
            "order_which_side_exact": bool(exact), "records": len(want), "bar": 1e-5}


def spin_sync(local):
    """hipDeviceScheduleSpin on this rank's device, set before torch creates its context: a
    host thread waiting in hipDeviceSynchronize / hipStreamSynchronize spins instead of
    yielding, which is what a latency-bound planner (one ~10 us cycle per step) runs with.  The
    process has one HIP runtime (torch's libamdhip64.so.7, which libccmpc.so binds to by
    soname).  CCMPC_BENCH_SPIN=0 leaves the default (auto) schedule.  Returns True if set."""
    if os.environ.get("CCMPC_BENCH_SPIN", "1") != "1":
        return False
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so.7")
    except OSError:
        return False
    n = ctypes.c_int(0)
    if hip.hipGetDeviceCount(ctypes.byref(n)) != 0 or n.value < 1:
        hip.hipGetLastError()
        return False
    # the one-card rehearsal (--backend gloo) runs every rank on device 0; a failed call would
    # leave a sticky error that the next torch call reports
    if hip.hipSetDevice(ctypes.c_int(local % n.value)) != 0:
        hip.hipGetLastError()
        return False
    ok = hip.hipSetDeviceFlags(ctypes.c_uint(1)) == 0   # hipDeviceScheduleSpin
    if not ok:
        hip.hipGetLastError()
    return ok


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    spun = False if args.launch_check else spin_sync(int(os.environ.get("LOCAL_RANK", "0")))
    world, rank, local = init_dist(args)
    if args.launch_check:
        launch_check(world, rank)
        return
    dev = torch.device("cuda", torch.cuda.current_device() if world > 1 else local)
    torch.cuda.set_device(dev)

    from ccmpc import cycle, engine, synthetic

    # every rank plans its own scene: seed keyed by the global scene index
    ovs, ref, _ = synthetic.scene(args.seed + rank, O=args.O, N=args.N, T=args.T)
    K = [len(o) for o in ovs]
    store = engine.ParticleStore.from_cells([c for o in ovs for c in o], device=dev)
    # one step = one planning step's constraint generation = one ccmpc_minkowski_cycle call
    # (the drop-in call pattern; arguments pre-bound).  --graph replays a captured hipGraph
    # instead, which adds ~5 us of graph-launch gap per step on this stack.
    cyc = cycle.MinkowskiCycle(store, K, ref)
    if args.graph:
        cyc.capture()
        step = cyc.replay
    else:
        step = cyc.bind().launch

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)

    h = cyc.records().reshape(-1)
    assert np.all(h["status"] == 0), "non-ok constraint records"

    # dominant (and only) kernel of the cycle: moments_kernel<double,1,true> = the Gram
    # reduction with the fused half-space tail; algorithmic bytes = every particle coordinate
    # read once (2T float64 per particle) -- SURVEY.md 8d's 16 N T read term
    n_part = int(sum(store.counts))
    alg_bytes = n_part * 2 * args.T * 8
    t_kernel = time_kernel_live(cyc.run, dev)
    t_mom = time_kernel_live(lambda: engine.moments(store, cyc.mean, cyc.cov, cyc.ws), dev)

    pcie = pcie_inclusive(cyc, step, dev)
    traffic, traffic_src = pmc_traffic("void ccmpc::moments_kernel<double, 1, true", "C2")
    value = world * args.steps / elapsed
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "cycles/s",
        "n_gpus": world,
        "rccl_world_size": world if _backend() == "nccl" else None,
        "dist_backend": _backend() or "none (one rank)",
        "launcher": ("bench.py --gpus N (child torchrun)" if os.environ.get("CCMPC_BENCH_SPAWNED")
                     else ("torchrun" if world > 1 else "single process")),
        "steps": args.steps,
        "warmup": args.warmup,
        "host_sync": "spin (hipDeviceScheduleSpin)" if spun else "default",
        "ms_per_step": round(1e3 * elapsed / args.steps, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded particle clouds; no Trajectron++ weights / CARLA offline)",
        "config": {
            "workload": "C2: 1 scene x 4 OVs, np=5000/OV, ph=8, Minkowski/MVOE "
                        "constraint-gen cycle (moments + all (cell,t,tau) half-spaces), "
                        "one ccmpc_minkowski_cycle launch per step, particles resident in HBM",
            "scenes_per_gpu": 1, "O": args.O, "N_per_ov": args.N, "T": args.T, "K": K,
            "cells": store.n_cells, "halfspaces_per_cycle": cyc.n_constraints,
        },
        "constraints_per_s": round(value * cyc.n_constraints, 1),
        "pcie_inclusive": pcie,
        "roofline": {
            "bound": "hbm",
            "kernel": "moments_kernel<double,1,true> (ccmpc_minkowski_cycle: MFMA Gram + "
                      "last-arriver combine + MVOE half-spaces, one launch)",
            "achieved": round(alg_bytes / t_kernel / 1e9, 2),
            "peak": HBM_PEAK / 1e9,
            "unit": "GB/s",
            "frac": round(alg_bytes / t_kernel / HBM_PEAK, 5),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "alg_bytes_per_launch": alg_bytes,
            "avg_launch_us": round(t_kernel * 1e6, 3),
            "moments_only_avg_launch_us": round(t_mom * 1e6, 3),
            "achievable_peak": HBM_ACHIEVABLE / 1e9,
            "frac_of_achievable": round(alg_bytes / t_kernel / HBM_ACHIEVABLE, 5),
            "note": "C2 is a latency chain (DESIGN.md 4.1); the HBM-bound configs are c4_sharded "
                    "and roofline_sweep's C3 1e5 / C5 lines",
        },
    }
    if rank == 0:
        out["ellipsoid_parity"] = ellipsoid_parity(ovs, ref, args.T, h)
    if rank == 0 and world == 1 and not args.no_cpu:
        med, threads, n, total = cpu_baseline(ovs, ref, args.T, args.cpu_cycles)
        out["cpu_baseline"] = {
            "value": round(1.0 / med, 3), "unit": "cycles/s", "cores": threads, "kind": "port",
            "host_cpu": host_cpu(),
            "sample": f"median of {n} full C2 cycles (same scene) at BLAS threads={threads}; "
                      f"{total:.1f} s of CPU work in total (1 and min(16, cores) threads); "
                      "oracle restatement of v8ideal/__init__.py:881-947 (numpy/scipy)",
        }
        out["speedup_vs_cpu"] = round(value / (1.0 / med), 1)
    if not args.no_c4:
        # BASELINE configs[3]: the 64-scene batch sharded over the ranks, the record gather
        # (RCCL) inside the step; every rank takes part
        out["c4_sharded"] = c4_sharded(dev, args.seed, world, rank)
    if rank == 0:
        # C2 is launch/latency-bound (2.56 MB per cycle); the HBM roofline of the
        # same kernel is meaningful at the per-GPU C4 batch, reported beside it
        c4 = time_config(dev, args.seed, *C4_GPU)
        c4["traffic"], c4["traffic_source"] = pmc_traffic(
            "void ccmpc::moments4_kernel<double, 6, true", "C4")
        c4["alg_bytes_per_launch"] = c4["particles"] * 2 * C4_GPU[3] * 8
        out["roofline_c4_batch"] = c4
        # the same batch at the reference's own input precision (Trajectron++'s float32
        # predictions relative to minpos, promoted exactly): the f64 line above is the headline
        c4f = time_config(dev, args.seed, C4_GPU[0] + " (f32 store relative to minpos)",
                          *C4_GPU[1:], f32=True)
        c4f["alg_bytes_per_launch"] = c4f["particles"] * 2 * C4_GPU[3] * 4
        c4f["note"] = ("the sampler's store format: float32 positions relative to the scene's "
                       "minpos, promoted to float64 before use, as prediction + minpos does "
                       "(v8ideal/__init__.py:486); 8 T bytes per particle")
        out["roofline_c4_batch_f32"] = c4f
    if rank == 0 and world == 1:
        from threadpoolctl import threadpool_limits
        with threadpool_limits(limits=1):
            out["dropin_step_c2"] = dropin_step(dev, with_cpu=not args.no_cpu)
            out["dropin_step_c2_pp"] = dropin_step(dev, with_cpu=False, per_particle=True)
            # the reference's own predictor output (generate_vehicle_latents' 5-tuple)
            out["dropin_step_c2_predictions"] = dropin_step_predictions(dev)
            out["dropin_step_c2_predictions_device"] = dropin_step_predictions(dev,
                                                                               on_device=True)
            # C1's real particle count (tests/Hz20/params.py:377): the graph's non-fused branch
            out["dropin_step_c1_100k"] = dropin_step(
                dev, steps=100, with_cpu=not args.no_cpu, O=1, N=100_000, eager_steps=20,
                cpu_reps=2, label="C1 (n_predictions = 100 000)")
            out["dropin_step_c1_100k_predictions_device"] = dropin_step_predictions(
                dev, steps=100, O=1, N=100_000, n_sets=4, on_device=True)
            out["episode_c1"] = episode_c1(dev, with_cpu=not args.no_cpu)
            out["harness_episode"] = harness_episode(dev)
            # the reference's real particle count at the "np5000" label (params.py:377)
            out["episode_c1_np100k"] = episode_c1(dev, with_cpu=False, N=100_000)
            out["planning_qp"] = planning_qp(dev, args.seed, with_cpu=not args.no_cpu)
            # one frame's QP (the reference solves one per planning step) at T = 8 and at C4's
            # horizon T = 12 (n = 24: the active set on NM = 32 rows): the batch's first scene
            # (infeasible at T = 12: the certificate, then the interior point) and its first
            # solved scene, and the T = 12 batch
            out["planning_qp_single_t8"] = planning_qp(dev, args.seed, scenes=1, with_cpu=False)
            out["planning_qp_single_t12"] = planning_qp(dev, args.seed, scenes=1, T=12,
                                                        with_cpu=False)
            out["planning_qp_t12"] = planning_qp(dev, args.seed, T=12, with_cpu=False)
            f12 = out["planning_qp_t12"]["first_solved_scene"]
            if f12 is not None:
                out["planning_qp_single_t12_solved"] = planning_qp(
                    dev, args.seed, scenes=1, T=12, with_cpu=False, first=f12)
            out["v8_milp"] = v8_milp(dev, with_cpu=not args.no_cpu)
    if not args.no_sweep and rank == 0:
        out["roofline_sweep"] = sweep(dev, args.seed)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if _backend() is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
