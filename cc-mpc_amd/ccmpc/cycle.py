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
import numpy as np
import torch

from . import engine, risk


class MinkowskiCycle:
    def __init__(self, store, K, ref_traj, ph=None, R=risk.R_COLLISION, tol=1e-8, maxiter=1000,
                 scene_K=None):
        """scene_K: the per-scene split of K when several scenes' cells share one cycle (each
        scene then allocates its own risk, risk.scenes_cell_risk); None = one scene."""
        self.store = store
        self.device = store.device
        self.T = store.T
        self.K = [int(k) for k in K]
        assert sum(self.K) == store.n_cells
        ph = self.T if ph is None else ph
        C, T = store.n_cells, self.T
        self.ref = torch.as_tensor(np.asarray(ref_traj, np.float64).reshape(-1, T, 2),
                                   device=self.device)
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
        engine.minkowski_cycle(self.store, self.ref, self.risk, R=self.R, tol=self.tol,
                               maxiter=self.maxiter, workspace=self.ws, out_mean=self.mean,
                               out_cov=self.cov, out_rec=self.rec,
                               out_prob_lower=self.prob_lower)

    def bind(self):
        """Pre-convert every argument of the one-launch C-ABI call for the current stream, so
        `launch()` costs one foreign call (the host side of a planning step, ~4x cheaper than
        re-deriving pointers per call).  Rebind after changing streams or buffers."""
        lib = engine._lib.load()
        st = self.store
        ws = self.ws.get(lib.ccmpc_moments_workspace_bytes(self.T, st.n_cells, st.n_bound))
        p = engine._p
        self._fn = lib.ccmpc_minkowski_cycle
        self._args = (p(st.pos), st.ccmpc_dtype, st.ld, self.T, p(st.origin), p(st.cell_off),
                      p(st.cell_cnt), st.n_cells, st.n_bound, p(ws), ws.numel(), p(self.ref),
                      p(None), p(self.risk), float(self.R), float(self.tol), int(self.maxiter),
                      p(self.mean), p(self.cov), p(self.rec), p(self.prob_lower),
                      engine._stream())
        return self

    def launch(self):
        """One planning step's constraint generation: one C-ABI call, one kernel."""
        rc = self._fn(*self._args)
        if rc != 0:
            engine._lib.check(rc, "ccmpc_minkowski_cycle")

    def run_unfused(self):
        """Same cycle as two C-ABI calls (ccmpc_moments, ccmpc_minkowski)."""
        engine.moments(self.store, self.mean, self.cov, self.ws)
        engine.minkowski(self.mean, self.cov, self.ref, self.risk, R=self.R, tol=self.tol,
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
    def __init__(self, store, K, ref_traj, ph=None, R=risk.R_COLLISION):
        self.store = store
        self.device = store.device
        self.T = store.T
        self.K = [int(k) for k in K]
        ph = self.T if ph is None else ph
        C, T = store.n_cells, self.T
        self.ref = torch.as_tensor(np.asarray(ref_traj, np.float64).reshape(-1, T, 2),
                                   device=self.device)
        self.gamma = torch.as_tensor(risk.cell_gamma(risk.eps_ura(self.K), self.K, ph),
                                     device=self.device)
        self.R = R
        self.mean = torch.empty((C, T, 2), dtype=torch.float64, device=self.device)
        self.cov = torch.empty((C, 2 * T, 2 * T), dtype=torch.float64, device=self.device)
        self.rec = torch.empty((C, T, 128), dtype=torch.uint8, device=self.device)
        self.ws = engine.Workspace(self.device)
        self.ws.get(engine._lib.load().ccmpc_moments_workspace_bytes(T, C, store.n_bound))

    def run(self):
        engine.moments(self.store, self.mean, self.cov, self.ws)
        engine.affine(self.mean, self.cov, self.ref, self.gamma, R=self.R, out_rec=self.rec)

    def records(self):
        return engine.affine_records(self.rec)
