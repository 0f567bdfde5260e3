"""A/B of libccmpc.so builds on the drop-in planning step's kernels (GPU box, repo root):
    python tools/ab_step.py main build_x ...
Each variant in its own process: the step graph's per-replay time (HIP events, back to back)
and ccmpc_l4 alone on the step's bucketed store."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
    import numpy as np
    import torch
    import bench
    from ccmpc import engine, episode, planner
    dev = torch.device("cuda", 0)
    O, N, ph = 4, 5000, 8
    init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=20251015)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]]) for o in range(O)]
    K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
    eps = np.full((O, max(K)), 0.05 / O)
    ref = np.array([[165.0 + 4.0 * (t + 1), -72.0 + 0.5 * (t + 1)] for t in range(ph)])
    agent = planner.MidlevelAgent(prediction_horizon=ph, device=dev)
    params = episode.Params(O, K, 0)
    for i in range(10):
        agent.predict_and_constrain(params, dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N,
                                                 seed=i), eps, ph, ref, minpos, pasts)
    g = next(iter(agent._graphs.values()))
    t_graph = bench.time_graph_replay(g, dev)
    lib, p, o, i, st = engine._lib.load(), engine._p, g.out, g.inp, g.store

    def l4():
        engine._lib.check(lib.ccmpc_l4(
            p(st.pos), engine.F32, st.ld, ph, p(st.origin), p(o.d("off")), p(o.d("cnt")), g.C,
            p(i.d("past")), p(i.d("bbox")), p(o.d("A")), p(o.d("b")), p(o.d("yaw_mean")),
            p(o.d("yaw0_var")), None, None, engine._stream()), "ccmpc_l4")
    t_l4 = bench.time_kernel_live(l4, dev, per_graph=20, replays=5)
    lws = g.l4_ws.buf

    def l4s():
        engine._lib.check(lib.ccmpc_l4_split(
            p(st.pos), engine.F32, st.ld, ph, p(st.origin), p(o.d("off")), p(o.d("cnt")), g.C,
            st.n_bound, p(i.d("past")), p(i.d("bbox")), p(lws), lws.numel(), p(o.d("A")),
            p(o.d("b")), p(o.d("yaw_mean")), p(o.d("yaw0_var")), None, None, engine._stream()),
            "ccmpc_l4_split")
    t_l4s = bench.time_kernel_live(l4s, dev, per_graph=20, replays=5)
    print(f"  graph replay {t_graph * 1e6:7.2f} us   l4 {t_l4 * 1e6:7.2f} us   "
          f"l4_split {t_l4s * 1e6:7.2f} us", flush=True)
    # a C1-sized cloud (one OV, 2 modes, 1e5 particles, ph = 8): both forms
    from ccmpc import synthetic
    ovs, _, pasts = synthetic.scene(5, O=1, N=100_000, T=ph, K=2)
    big = engine.ParticleStore.from_cells(ovs[0], device=dev)
    past = np.repeat(pasts, 2, axis=0)
    bb = np.tile([4.5, 2.5], (2, 1))
    ws = engine.Workspace(dev)
    for split in (False, True):
        fn = lambda: engine.l4(big, past, bb, split=split, workspace=ws)
        fn()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(20):
            fn()
        ev1.record()
        ev1.synchronize()
        print(f"  1e5-particle cells x 2, T = {ph}: {'split' if split else 'one workgroup'} "
              f"{ev0.elapsed_time(ev1) / 20 * 1e3:8.2f} us (with the wrapper's H2D copies)",
              flush=True)


def main():
    if sys.argv[1] == "--child":
        child()
        return
    for v in sys.argv[1:]:
        env = dict(os.environ)
        if v != "main":
            env["CCMPC_LIB"] = os.path.join(ROOT, "cc-mpc_amd", "csrc", v, "libccmpc.so")
        print(f"== {v}", flush=True)
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, text=True,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=300)
        print("\n".join(l for l in r.stdout.splitlines() if "amdgpu.ids" not in l), flush=True)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
