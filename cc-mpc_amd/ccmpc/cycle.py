"""Device-resident constraint-generation cycles with preallocated buffers.

A cycle is what one planning step of v8ideal spends on chance constraints:

  MinkowskiCycle  particles -> moments -> (cell, t, tau) MVOE half-spaces
                  (compute_obstacle_constraints_GMM_Minkowski_idealprediction,
                   v8ideal/__init__.py:881-947, plus the save_moments statistics :2575-2606
                   which are the same moments)
  AffineCycle     particles -> moments -> (cell, t) GMM-affine half-spaces (:1470-1515)

Every buffer is allocated up front and every call enqueues on the current stream, so
``capture()`` records the whole cycle into one hipGraph (torch.cuda.CUDAGraph) and ``replay()``
costs one graph launch.
"""
import ctypes

import numpy as np
import torch

from . import engine, risk


def _cell_ref(ref, n_cells, scene_K, cell_ref, device):
    """The per-cell reference-trajectory selector of a batched cycle (int32 [n_cells] on the
    device), or None when every cell uses ref[0].

    Each scene of a batch is its own planning step with its own ref_traj (the reference plans
    one scene per agent, v8ideal/__init__.py:2934-2976), so a batch of several scenes must say
    which row of `ref` [n_ref, T, 2] each cell reads: explicitly (cell_ref), or by scene when
    `ref` holds one row per scene of scene_K.  Indices are checked here, on the host: the kernel
    reads ref[cell_ref[c]] unchecked."""
    n_ref = int(ref.shape[0])
    if cell_ref is None and scene_K is not None and n_ref > 1:
        if n_ref != len(scene_K):
            raise ValueError(f"{n_ref} reference trajectories for {len(scene_K)} scenes")
        cell_ref = np.repeat(np.arange(n_ref), [sum(int(k) for k in K_s) for K_s in scene_K])
    if cell_ref is None:
        if n_ref != 1:
            raise ValueError(f"{n_ref} reference trajectories need cell_ref (or scene_K)")
        return None
    cell_ref = np.asarray(cell_ref, np.int64).reshape(-1)
    if cell_ref.shape[0] != n_cells:
        raise ValueError(f"cell_ref has {cell_ref.shape[0]} entries for {n_cells} cells")
    if n_cells and (cell_ref.min() < 0 or cell_ref.max() >= n_ref):
        raise ValueError(f"cell_ref indices must lie in [0, {n_ref})")
    return torch.as_tensor(cell_ref.astype(np.int32), device=device)


class MinkowskiCycle:
    def __init__(self, store, K, ref_traj, ph=None, R=risk.R_COLLISION, tol=1e-8, maxiter=1000,
                 scene_K=None, cell_ref=None):
        """scene_K: the per-scene split of K when several scenes' cells share one cycle (each
        scene then allocates its own risk, risk.scenes_cell_risk); None = one scene.
        ref_traj: (T, 2) for one scene, or (n_ref, T, 2) with cell_ref [n_cells] selecting each
        cell's row -- by default one row per scene of scene_K."""
        self.store = store
        self.device = store.device
        self.T = store.T
        self.K = [int(k) for k in K]
        assert sum(self.K) == store.n_cells
        ph = self.T if ph is None else ph
        C, T = store.n_cells, self.T
        self.ref = torch.as_tensor(np.asarray(ref_traj, np.float64).reshape(-1, T, 2),
                                   device=self.device)
        self.cell_ref = _cell_ref(self.ref, C, scene_K, cell_ref, self.device)
        if scene_K is None:
            cr = risk.cell_risk(risk.eps_ura(self.K), self.K, ph)
        else:
            assert [int(k) for K_s in scene_K for k in K_s] == self.K
            cr = risk.scenes_cell_risk(scene_K, ph)
        self.risk = torch.as_tensor(cr, device=self.device)
        self.R, self.tol, self.maxiter = R, tol, maxiter
        self.mean = torch.empty((C, T, 2), dtype=torch.float64, device=self.device)
        self.cov = torch.empty((C, 2 * T, 2 * T), dtype=torch.float64, device=self.device)
        P = max(T * (T - 1) // 2, 1)
        self.rec = torch.empty((C, P, 128), dtype=torch.uint8, device=self.device)
        self.prob_lower = torch.empty((C, T), dtype=torch.float64, device=self.device)
        self.ws = engine.Workspace(self.device)
        self.ws.get(engine._lib.load().ccmpc_moments_workspace_bytes(T, C, store.n_bound))
        self.graph = None

    def run(self):
        """One launch: moments + every (cell, t, tau) half-space (ccmpc_minkowski_cycle)."""
        engine.minkowski_cycle(self.store, self.ref, self.risk, cell_ref=self.cell_ref,
                               R=self.R, tol=self.tol,
                               maxiter=self.maxiter, workspace=self.ws, out_mean=self.mean,
                               out_cov=self.cov, out_rec=self.rec,
                               out_prob_lower=self.prob_lower)

    def bind(self):
        """Fill the one-launch C-ABI call's argument struct for the current stream once
        (ccmpc_minkowski_cycle_args), so `launch()` costs one single-pointer foreign call (the
        host side of a planning step: a 22-argument ctypes call is ~2-3 us of marshalling in
        front of every launch).  Rebind after changing streams or buffers."""
        from . import _lib as L
        lib = engine._lib.load()
        st = self.store
        ws = self.ws.get(lib.ccmpc_moments_workspace_bytes(self.T, st.n_cells, st.n_bound))
        p = engine._p
        self._fn = lib.ccmpc_minkowski_cycle_args
        self._argst = L.CycleArgs(
            positions=p(st.pos), dtype=st.ccmpc_dtype, maxiter=int(self.maxiter), ld=st.ld,
            T=self.T, origin=p(st.origin), cell_off=p(st.cell_off), cell_cnt=p(st.cell_cnt),
            n_cells=st.n_cells, n_particles_bound=st.n_bound, workspace=p(ws),
            workspace_bytes=ws.numel(), ref_traj=p(self.ref), cell_ref=p(self.cell_ref),
            cell_risk=p(self.risk), R=float(self.R), tol=float(self.tol), out_mean=p(self.mean),
            out_cov=p(self.cov), out_rec=p(self.rec), out_prob_lower=p(self.prob_lower),
            stream=engine._stream())
        self._args = (ctypes.addressof(self._argst),)
        self._keep = ws
        return self

    def launch(self):
        """One planning step's constraint generation: one C-ABI call, one kernel."""
        rc = self._fn(*self._args)
        if rc != 0:
            engine._lib.check(rc, "ccmpc_minkowski_cycle")

    def run_unfused(self):
        """Same cycle as two C-ABI calls (ccmpc_moments, ccmpc_minkowski)."""
        engine.moments(self.store, self.mean, self.cov, self.ws)
        engine.minkowski(self.mean, self.cov, self.ref, self.risk, cell_ref=self.cell_ref,
                         R=self.R, tol=self.tol,
                         maxiter=self.maxiter, out_rec=self.rec, out_prob_lower=self.prob_lower)

    def capture(self, warmup=2):
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.run()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.run()
        return self

    def replay(self):
        if self.graph is None:
            self.run()
        else:
            self.graph.replay()

    @property
    def n_constraints(self):
        return self.store.n_cells * (self.T * (self.T - 1) // 2)

    def records(self):
        return engine.halfspaces(self.rec)


class AffineCycle:
    def __init__(self, store, K, ref_traj, ph=None, R=risk.R_COLLISION, scene_K=None,
                 cell_ref=None):
        """scene_K / cell_ref as MinkowskiCycle."""
        self.store = store
        self.device = store.device
        self.T = store.T
        self.K = [int(k) for k in K]
        assert sum(self.K) == store.n_cells
        ph = self.T if ph is None else ph
        C, T = store.n_cells, self.T
        self.ref = torch.as_tensor(np.asarray(ref_traj, np.float64).reshape(-1, T, 2),
                                   device=self.device)
        self.cell_ref = _cell_ref(self.ref, C, scene_K, cell_ref, self.device)
        if scene_K is None:
            g = risk.cell_gamma(risk.eps_ura(self.K), self.K, ph)
        else:
            assert [int(k) for K_s in scene_K for k in K_s] == self.K
            g = risk.scenes_cell_risk(scene_K, ph)[:, 2].copy()
        self.gamma = torch.as_tensor(g, device=self.device)
        self.R = R
        self.mean = torch.empty((C, T, 2), dtype=torch.float64, device=self.device)
        self.cov = torch.empty((C, 2 * T, 2 * T), dtype=torch.float64, device=self.device)
        self.rec = torch.empty((C, T, 128), dtype=torch.uint8, device=self.device)
        self.ws = engine.Workspace(self.device)
        self.ws.get(engine._lib.load().ccmpc_moments_workspace_bytes(T, C, store.n_bound))

    def run(self):
        engine.moments(self.store, self.mean, self.cov, self.ws)
        engine.affine(self.mean, self.cov, self.ref, self.gamma, cell_ref=self.cell_ref,
                      R=self.R, out_rec=self.rec)

    def records(self):
        return engine.affine_records(self.rec)
