"""Replay of one v8ideal episode's planning schedule through the drop-in surface.

SURVEY.md 3.1 (tests/Hz20/__init__.py:297-359 -> v8ideal/__init__.py:3163-3254): every 10
simulator frames the agent predicts (Trajectron++ sample -> make_ovehicles) and generates
chance constraints:

  shrinking phase  frames 0, 10, ..., 70 with Tsh = 8, 7, ..., 1: the Minkowski/MVOE generator;
                   at Tsh < ph it first rolls the moments saved at frame - 10 forward with
                   predict_ideal (1e6 samples)
  receding phase   every later planning frame: the GMM-affine generator at Tsh = ph

The CARLA world and the learned Trajectron++ encoder/decoder are outside this path; the replay
feeds the GPU sampler synthetic per-OV GMM action parameters (SURVEY.md 8d generator) and times
each planning step end to end (one step-graph replay: sampler -> bucketing -> the generator's
fused launch, then the host HalfSpace objects -> the QP on the device records,
do_highlevel_control :2850-3110).  The ego is not
simulated: each step plans from a synthetic state on the reference trajectory, and the
shrinking steps pass the first control of every earlier step as the executed controls
(U_prev, :3186).  The ego's lane (EGO_Y) keeps every QP of the default scene feasible; an
infeasible QP is logged (the reference raises InSimulationException and the episode ends; the
replay continues with a zero control for that step).
"""
import time

import numpy as np
import torch

from . import engine, ovehicle, planner


class Params:
    """The slice of the reference's `params` the generators read (O, K, frame)."""

    def __init__(self, O, K, frame):
        self.O, self.K, self.frame = O, np.asarray(K), frame


def synthetic_gmm(O, L=25, T=8, seed=20251015):
    """Per-OV inputs of the sampler boundary: initial unicycle state, latent pmf p(z|x) and
    per-(latent, step) GMM2D action parameters, drawn as SURVEY.md 8d specifies."""
    rng = np.random.default_rng(seed)
    init = np.stack([rng.uniform(180, 200, O) - 150.0, rng.uniform(-90, -70, O) + 120.0,
                     rng.uniform(-np.pi, np.pi, O), rng.uniform(3, 10, O)], axis=1)
    logits = rng.normal(0, 1.0, size=(O, L))
    for o in range(O):                       # keep >= 1 mode above the 0.1 filter
        logits[o, rng.integers(L)] += 3.0
    pmf = np.exp(logits)
    pmf /= pmf.sum(1, keepdims=True)
    gmm = np.zeros((O, L, T, 5), np.float32)
    gmm[..., 0] = rng.normal(0, 0.15, size=(O, L, T))
    gmm[..., 1] = rng.normal(0, 1.0, size=(O, L, T))
    gmm[..., 2:4] = rng.uniform(np.log(0.05), np.log(0.5), size=(O, L, T, 2))
    gmm[..., 4] = rng.uniform(-0.5, 0.5, size=(O, L, T))
    return init, pmf, gmm


class EpisodeReplay:
    def __init__(self, O=1, N=5000, ph=8, n_ideal=1_000_000, receding_steps=4, seed=0,
                 device="cuda", with_qp=True):
        self.O, self.N, self.ph = O, N, ph
        self.with_qp = with_qp
        self.u_prev = []
        self.device = engine.require_device(device)
        self.receding_steps = receding_steps
        self.seed = seed
        self.init, self.pmf, self.gmm = synthetic_gmm(O, T=ph, seed=20251015 + seed)
        self.minpos = np.array([150.0, -120.0])
        self.pasts = [np.array([[self.minpos[0] + self.init[o, 0] - 2.0,
                                 self.minpos[1] + self.init[o, 1]]]) for o in range(O)]
        self.agent = planner.MidlevelAgent(prediction_horizon=ph, n_ideal=n_ideal, seed=seed,
                                           device=self.device)

    # the ego's lane: 22 m north of where the OV's particle cloud crosses it, so the first
    # planning step's QP is feasible (the oracle's QP on the oracle's records: y = -72 and -60
    # are infeasible, -55 and -50 feasible) and the schedule is one the reference could run
    EGO_Y = -50.0

    def ref_traj(self, frame):
        """Ego reference over the horizon, placed so ref_y != mean_y."""
        ego = np.array([165.0 + 0.2 * frame, self.EGO_Y])
        return np.array([ego + [4.0 * (t + 1), 0.5 * (t + 1)] for t in range(self.ph)])

    def predict(self, frame):
        """do_prediction + make_ovehicles for one planning frame (sampler seed keyed by it)."""
        z, store = engine.sample_unicycle(self.init, self.pmf, self.gmm, self.N, self.ph,
                                          seed=self.seed * 7919 + frame, device=self.device)
        return ovehicle.make_ovehicles(store, z, self.pmf, self.minpos, self.pasts,
                                       device=self.device)

    def x_init(self, frame):
        """Synthetic ego state [x, y, psi, v] at the start of the reference trajectory."""
        ego = self.ref_traj(frame)[0] - np.array([4.0, 0.5])
        return np.array([ego[0], ego[1], np.arctan2(0.5, 4.0), 8.0])

    def plan(self, frame, T):
        """The planning step's QP on the generator's device records."""
        ref = self.ref_traj(frame)
        if T == self.ph:
            self.u_prev = []
        up = np.concatenate(self.u_prev) if self.u_prev else None
        try:
            res = self.agent.solve_planning_qp(self.x_init(frame), ref[-1] + [4.0, 0.5], ref,
                                               T, u_prev=up)
        except planner.InSimulationException:
            # the reference's episode ends here; the replay goes on timing the schedule with a
            # zero control standing in for the step that was not planned
            self.u_prev.append(np.zeros(2))
            return None
        self.u_prev.append(res["u"][:2])      # U_star.T.ravel()[:nu] (:3186)
        return res

    def schedule(self):
        """(frame, Tsh, generator) of every planning step of the episode."""
        steps = [(10 * s, self.ph - s, "minkowski") for s in range(self.ph)]
        steps += [(10 * (self.ph + r), self.ph, "affine") for r in range(self.receding_steps)]
        return steps

    def sampler(self, frame):
        """The frame's sampler-boundary inputs (seed keyed by the frame)."""
        return dict(init_state=self.init, latent_pmf=self.pmf, gmm=self.gmm, N=self.N,
                    seed=self.seed * 7919 + frame)

    def step(self, frame, T, kind, eager=False):
        """One planning step: do_prediction + make_ovehicles + the schedule's generator as a
        step-graph replay (MidlevelAgent.predict_and_constrain / _affine), or (eager) the
        separate calls -- the GPU sampler, the bucketing, then the generator method on the
        OVehicles -- which give the same bits."""
        if eager:
            ovs = self.predict(frame)
            K = [ov.n_states for ov in ovs]
        else:
            K = (self.pmf > 0.1).sum(1).tolist()
        eps = np.zeros((self.O, max(K)))
        eps[:, :] = 0.05 / self.O                    # eps_ura (v8ideal/__init__.py:2920-2926)
        params = Params(self.O, K, frame)
        ref = self.ref_traj(frame)
        if not eager:
            fn = (self.agent.predict_and_constrain if kind == "minkowski"
                  else self.agent.predict_and_constrain_affine)
            return fn(params, self.sampler(frame), eps, T, ref, self.minpos, self.pasts)
        gen = (self.agent.compute_obstacle_constraints_GMM_Minkowski_idealprediction
               if kind == "minkowski" else self.agent.compute_obstacle_constraints_GMM_affine)
        out = gen(params, ovs, None, None, None, eps, None, T, ref)
        return ovs, out

    def run(self, sync=True, eager=False):
        """Runs the whole schedule; returns one record per planning step."""
        log = []
        for frame, T, kind in self.schedule():
            if sync:
                torch.cuda.synchronize(self.device)
            t0 = time.perf_counter()
            ovs, out = self.step(frame, T, kind, eager=eager)
            if sync:
                torch.cuda.synchronize(self.device)
            t1 = time.perf_counter()
            entry = {"frame": frame, "T": T, "generator": kind,
                     "K": [ov.n_states for ov in ovs], "constraints": len(out[0]),
                     "ms": (t1 - t0) * 1e3}
            if self.with_qp:
                res = self.plan(frame, T)
                entry["qp_ms"] = (time.perf_counter() - t1) * 1e3
                entry["qp"] = "infeasible" if res is None else "solved"
            log.append(entry)
        return log
