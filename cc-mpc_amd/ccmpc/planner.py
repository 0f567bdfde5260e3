"""Drop-in constraint-generation surface of the v8ideal planner
(collect/in_simulation/midlevel/v8ideal/__init__.py, class MidlevelAgent).

The reference planner couples CARLA, Trajectron++, cvxpy and CPLEX; only its chance-constraint
path is in scope here.  This class keeps that path's Python call surface --
the two generator methods with their argument lists and 9-tuple results, save_moments and
predict_ideal -- and runs every numeric step on the GPU through libccmpc.so:

  compute_obstacle_constraints_GMM_Minkowski_idealprediction   v8ideal/__init__.py:781-964
      T == ph : ONE launch  (ccmpc_minkowski_cycle)        particles -> moments -> half-spaces
      T <  ph : ONE launch  (ccmpc_ideal_minkowski_cycle)  previous moments -> 1e6-sample
                                                            rollout -> moments -> half-spaces
      + ccmpc_l4 for vertices / A_union / b_union / yaw statistics
  compute_obstacle_constraints_GMM_affine                       v8ideal/__init__.py:1378-1539
  save_moments / predict_ideal                                  v8ideal/__init__.py:2575-2711

Differences from the reference, all at the boundary:
  * constraints are HalfSpace records (cvxpy is not part of the compute path and is not
    installed here); HalfSpace.expr(temp_x) builds the reference's cvxpy constraint when cvxpy
    is importable, HalfSpace.holds(x) evaluates it numerically;
  * the moments pickle (out/data/agent{id}_frame{f}_moments) is replaced by device-resident
    state keyed by frame (save_moments_npz / load_moments_npz keep the file format's keys);
  * the unseeded RNG of predict_ideal (:2664, :2699) is a Philox stream keyed by
    (seed, frame, cell), so runs are reproducible.
"""
import collections
import functools
import os

import numpy as np
import scipy.stats
import torch

from . import engine, mpc, risk
from .ovehicle import OVehicle, ScenePredictions


class InSimulationException(Exception):
    """collect/exception.py:11: the planner's failure (an infeasible QP, :3099-3110)."""


class HalfSpace:
    """One chance constraint on the ego position x_t (t = planning step):
    side = +1:  n . x_t >= rhs      side = -1:  n . x_t <= rhs
    Minkowski records have rhs = d (v8ideal/__init__.py:926-939); affine records have
    rhs = d +/- Gamma ||sqrtm(cov) [m, -1]|| (:1504-1515)."""

    __slots__ = ("ov", "k", "t", "tau", "n", "d", "rhs", "side", "which", "margin", "status")

    def __init__(self, ov, k, t, tau, n, d, rhs, side, which, margin=0.0, status=0):
        self.ov, self.k, self.t, self.tau = ov, k, t, tau
        self.n = n
        self.d, self.rhs, self.side, self.which = d, rhs, side, which
        self.margin, self.status = margin, status

    @property
    def A(self):
        """(A, b) of the reference's half-space bookkeeping (:931-939): A x <= b."""
        return -self.n if self.side > 0 else self.n

    @property
    def b(self):
        return -self.rhs if self.side > 0 else self.rhs

    def holds(self, xy, tol=0.0):
        v = float(self.n @ np.asarray(xy, float)[:2])
        return v >= self.rhs - tol if self.side > 0 else v <= self.rhs + tol

    def expr(self, temp_x):
        """The reference's cvxpy constraint n^T [x_t, y_t] >= / <= rhs."""
        import cvxpy as cp  # noqa: F401  (not installed in this image)
        lhs = self.n.T @ cp.vstack([temp_x[self.t][0], temp_x[self.t][1]])
        return lhs >= self.rhs if self.side > 0 else lhs <= self.rhs

    def __repr__(self):
        op = ">=" if self.side > 0 else "<="
        return (f"HalfSpace(ov={self.ov}, k={self.k}, t={self.t}, tau={self.tau}: "
                f"[{self.n[0]:.6g}, {self.n[1]:.6g}] . x {op} {self.rhs:.9g})")


class LazyVertices:
    """vertices[t][k][ov] -> (N_k, 4, 2) corners (v8ideal/__init__.py:627-640), copied from the
    device on first access only (100k particles x 8 corners is tens of MB per OV)."""

    def __init__(self, scene, ph):
        self.scene, self.ph = scene, ph

    def __len__(self):
        return self.ph

    def __getitem__(self, t):
        return _VertT(self, t)


class _VertT:
    def __init__(self, lv, t):
        self.lv, self.t = lv, t

    def __getitem__(self, k):
        return _VertTK(self.lv, self.t, k)


class _VertTK:
    def __init__(self, lv, t, k):
        self.lv, self.t, self.k = lv, t, k

    def __getitem__(self, ov):
        sc = self.lv.scene
        if self.k >= sc.K[ov]:
            return None
        v = sc.l4(with_yaw=True, with_vertices=True)["vertices"]
        st = sc.store
        c = sc.first_cell(ov) + self.k
        o, n = st.offsets[c], st.counts[c]
        return v[8 * self.t:8 * self.t + 8, o:o + n].T.cpu().numpy().reshape(n, 4, 2)


class HalfSpaceList:
    """The generator's `constraints` list over one host copy of the record block: HalfSpace
    objects are built when read (a planning step's records come back in one D2H; building
    hundreds of Python objects per step would cost more than the whole GPU step).  Checking
    the statuses happens up front, vectorised: the first failed record in the reference's
    (cell, t, tau) order raises the reference's exception (_lib.record_error)."""

    def __init__(self, h, cell_of, P, what="constraint"):
        self._h = h.reshape(len(cell_of), -1)[:, :P]
        self._cell_of = cell_of
        self._P = self._h.shape[1]
        st = self._h["status"].reshape(-1)
        bad = np.flatnonzero(st) if st.any() else ()
        if len(bad):
            c, p = divmod(int(bad[0]), self._P)
            r = self._h[c, p]
            o, k = cell_of[c]
            raise engine._lib.record_error(
                r["status"], f"{what} (ov={o}, k={k}, t={r['t_tau'] >> 16}, tau="
                             f"{r['t_tau'] & 0xFFFF})")

    def __len__(self):
        return len(self._cell_of) * self._P

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        c, p = divmod(i, self._P)
        r = self._h[c, p]
        o, k = self._cell_of[c]
        tt = int(r["t_tau"])
        return HalfSpace(o, k, tt >> 16, tt & 0xFFFF, np.array([r["n0"], r["n1"]]),
                         float(r["d"]), float(r["d"]), int(r["side"]), int(r["which"]))

    def __iter__(self):
        return (self[i] for i in range(len(self)))


class CellGrid:
    """A per-cell value as the reference's [ov][k] nested list (None where OV `ov` has no mode
    k), over a host array in (ov, k) cell order; rows are built on access."""

    def __init__(self, values, K, first=None):
        self._v, self._K = values, K
        self._first = first if first is not None else [sum(K[:o]) for o in range(len(K))]
        self._maxK = max(K)

    def __len__(self):
        return len(self._K)

    def __getitem__(self, o):
        if not 0 <= o < len(self._K):
            raise IndexError(o)
        f, k = self._first[o], self._K[o]
        return [float(x) for x in self._v[f:f + k]] + [None] * (self._maxK - k)

    def __iter__(self):
        return (self[o] for o in range(len(self._K)))


class UnionGrid:
    """A_union / b_union [t][k][ov] (v8ideal/__init__.py:627-736) over a host array [cell, t,
    ...]: None where OV `ov` has no mode k, as the reference's nested lists hold."""

    def __init__(self, arr, K, ph, first=None):
        self._arr, self._K, self._ph = arr, list(K), ph
        self._first = (first if first is not None
                       else np.concatenate([[0], np.cumsum(K)[:-1]]).astype(int))

    def __len__(self):
        return self._ph

    def __getitem__(self, t):
        if not 0 <= t < self._ph:
            raise IndexError(t)
        grid = self

        class _K:
            def __len__(self):
                return max(grid._K)

            def __getitem__(self, k):
                class _O:
                    def __len__(self):
                        return len(grid._K)

                    def __getitem__(self, ov):
                        if k >= grid._K[ov]:
                            return None
                        return grid._arr[grid._first[ov] + k, t]
                return _O()
        return _K()


class _LazyL4:
    """One step graph launch's L4 outputs (graph B), fetched on first use."""

    def __init__(self, graph, generation):
        self._g, self._gen, self._v = graph, generation, None

    def get(self):
        if self._v is None:
            self._v = self._g.l4_outputs(self._gen)
        return self._v


class _LazyCol:
    """A field (or one column of it) of a _LazyL4, indexed like the array it resolves to."""

    def __init__(self, l4, name, col):
        self._l4, self._name, self._col = l4, name, col

    def _arr(self):
        a = self._l4.get()[self._name]
        return a if self._col is None else a[:, self._col]

    def __getitem__(self, idx):
        return self._arr()[idx]

    def __array__(self, dtype=None, copy=None):
        a = self._arr()
        return a if dtype is None else a.astype(dtype)


def _match_modes(mean_loaded, x_init, cur_means, n_states, M_big):
    """Previous-frame mode per current mode: argmin of ||x_init - mean'_0|| + sum_t ||mean_t -
    mean'_{t+1}||, modes >= n_states (and missing ones) scored M_big, first minimum on ties
    (v8ideal/__init__.py:2190-2276)."""
    num_mode = len(mean_loaded)
    xi = np.asarray(x_init, np.float64).reshape(-1)[:2]
    picks = []
    for k in range(n_states):
        md = np.zeros(num_mode)
        for mode in range(num_mode):
            entry = mean_loaded[mode]
            if entry is None or entry[0] is None:
                md[mode] = M_big
                continue
            v = np.linalg.norm(xi - np.asarray(entry[0], np.float64))
            for t in range(len(cur_means[k])):
                v += np.linalg.norm(np.asarray(cur_means[k][t]) - np.asarray(entry[t + 1]))
            md[mode] = v
        md[n_states:] = M_big
        picks.append(int(np.argmin(md)))
    return picks


def _host(x):
    """NumPy view of a saved moment array (device tensor or host copy)."""
    return x.cpu().numpy() if torch.is_tensor(x) else np.asarray(x)


@functools.lru_cache(maxsize=64)
def _default_bboxes(O):
    """ovehicle.py:19's bbox for every OV (read-only: shared between calls)."""
    from . import ovehicle
    b = np.tile(ovehicle.DEFAULT_BBOX, (O, 1))
    b.setflags(write=False)
    return b


@functools.lru_cache(maxsize=256)
def _first_cells_t(K):
    return tuple(sum(K[:o]) for o in range(len(K)))


def _first_cells(K):
    """First cell of each OV for kept-mode counts K (a tuple)."""
    return list(_first_cells_t(tuple(K)))


@functools.lru_cache(maxsize=64)
def _last_cells(K):
    """Last cell (mode) of each OV."""
    return np.cumsum(K) - 1


def _object_grid(*shape):
    if len(shape) == 1:
        return [None] * shape[0]
    return np.empty(shape, dtype=object).tolist()


def _grid_cells(grid, K, shape):
    """[o][k][...] object grid -> (sum K, *shape) array in (ov, k) cell order."""
    out = np.zeros((sum(K),) + shape)
    c = 0
    for o, k_o in enumerate(K):
        for k in range(k_o):
            out[c] = np.asarray(grid[o][k], dtype=float).reshape(shape)
            c += 1
    return out


def _cells_grid(arr, K, T):
    """Inverse of _grid_cells for [o][k][t] leaves."""
    grid = _object_grid(len(K), max(K), T)
    c = 0
    for o, k_o in enumerate(K):
        for k in range(k_o):
            for t in range(T):
                grid[o][k][t] = arr[c, t]
            c += 1
    return grid


def _data_arrays(d, K):
    """Flatten the generator keys of a data_save dict into npz-safe arrays, cells in (ov, k)
    order: ovState*_tau_1 (C, 3) = (x, y, yaw); mnt_* = meanNtangent's (C, T, ...) fields."""
    out = {"K": np.asarray(K, np.int64), "MeanCov": np.bool_(d.get("MeanCov", False)),
           "shrinking": np.bool_(d.get("shrinking", False)),
           "OVconstraint": np.bool_(bool(d.get("OVconstraint", False)))}
    if "ovStateMean_tau_1" in d:
        out["ovStateMean_tau_1"] = np.stack([_grid_cells(g, K, ()) for g in d["ovStateMean_tau_1"]], 1)
        out["ovStateCov_tau_1"] = np.stack([_grid_cells(g, K, ()) for g in d["ovStateCov_tau_1"]], 1)
    if "meanNtangent" in d:
        mean_p, tangent, cov_p, _, const_idx = d["meanNtangent"]
        T = len(mean_p[0][0])
        out["mnt_mean"] = _grid_cells(mean_p, K, (T, 2))
        out["mnt_tangent"] = _grid_cells(tangent, K, (T,))
        out["mnt_cov"] = _grid_cells(cov_p, K, (T, 2, 2))
        out["mnt_const_idx"] = _grid_cells(const_idx, K, (T,)).astype(np.int32)
    if "x_init" in d:
        out["x_init"] = np.asarray(d["x_init"], float)
    for key in ("solve_time", "process_time", "cost", "timeout", "infeasible"):
        if d.get(key) is not None:
            out[key] = np.asarray(d[key])
    return out


def _mean_tangent_from_arrays(d):
    K = [int(k) for k in d["K"]]
    T = d["mnt_mean"].shape[1]
    const_idx = _cells_grid(d["mnt_const_idx"], K, T)
    for row in const_idx:
        for cell in row:
            if cell[0] is not None:
                cell[:] = [int(v) for v in cell]
    return (_cells_grid(d["mnt_mean"], K, T), _cells_grid(d["mnt_tangent"], K, T),
            _cells_grid(d["mnt_cov"], K, T), 0, const_idx)


def _flip_y_state(actor):
    """carlautil's location / rotation / speed with flip_y=True (python-utility is absent,
    restated): [x, -y, -yaw (rad), |v_xy|] -- make_local_params' x_init from the simulator
    (v8ideal/__init__.py:520-531, get_current_velocity :507-512)."""
    loc, rot, vel = actor.get_location(), actor.get_transform().rotation, actor.get_velocity()
    return np.array([loc.x, -loc.y, -np.deg2rad(rot.yaw), np.sqrt(vel.x ** 2 + vel.y ** 2)])


class PlanFollower:
    """Stand-in for the low-level VehiclePIDController (lowlevel/v1_1.py) the agent hands its
    plan to (:3255-3257, :3277-3279): set_plan(speeds, angles, step_period) keeps the plan,
    step() returns the control for the current frame as {target_speed, target_angle} (the
    planned speed / heading of the plan step the frame falls in).  The PID loop and CARLA's
    VehicleControl are outside the path."""

    def __init__(self):
        self.speeds = self.angles = None
        self.period, self.k = 1, 0

    def set_plan(self, speeds, angles, step_period):
        self.speeds, self.angles = np.asarray(speeds), np.asarray(angles)
        self.period, self.k = max(int(step_period), 1), 0

    def step(self):
        if self.speeds is None or len(self.speeds) == 0:
            return None
        i = min(self.k // self.period, len(self.speeds) - 1)
        self.k += 1
        return {"target_speed": float(self.speeds[i]), "target_angle": float(self.angles[i])}


class MidlevelAgent:
    """v8ideal.MidlevelAgent (v8ideal/__init__.py:202-235) with the reference's constructor:
    MidlevelAgent(ego_vehicle, map_reader, other_vehicle_ids, eval_stg, scene_builder_cls=...,
    scene_config=..., n_burn_interval=4, n_predictions=100, prediction_horizon=8,
    control_horizon=6, step_horizon=1, ..., **kwargs) -- the harness splats its scenario /
    control / debug dicts into it (tests/Hz20/__init__.py:183-193), unknown keys land in
    **kwargs as they do there (:234).

    The simulator-side arguments are duck-typed: ego_vehicle / map_reader / the scene builder
    / eval_stg need only the attributes ccmpc.standins documents (a real carla.Vehicle has
    them).  Without them the agent is the constraint-generation surface alone (every test
    that calls the generators directly builds it as MidlevelAgent(prediction_horizon=...)).

    Keyword extras of this implementation: n_ideal (predict_ideal's sample count, :2640),
    seed (the Philox streams that replace the reference's unseeded RNGs), device, data_dir
    (load_data from .npz files), reference_trajectory (load_refT's route, instead of the
    pickle at out/data/referenceTrajectory/T/refT), max_graphs (the step-graph cache size),
    record_interval / ego_vehicle_id when there is no scene_config / ego_vehicle."""

    def __init__(self, ego_vehicle=None, map_reader=None, other_vehicle_ids=(), eval_stg=None,
                 scene_builder_cls=None, scene_config=None, n_burn_interval=4,
                 n_predictions=100, prediction_horizon=8, control_horizon=None, step_horizon=1,
                 road_boundary_constraints=False, angle_boundary_constraints=False,
                 log_cplex=True, log_agent=False, plot_simulation=False, plot_boundary=False,
                 plot_scenario=False, plot_vertices=False, plot_overapprox=False,
                 get_computeTime=True, turn_choices=(), max_distance=100, *,
                 n_ideal=1_000_000, seed=0, device="cuda", data_dir=None, **kwargs):
        self.device = engine.require_device(device)
        self.prediction_horizon = int(prediction_horizon)
        # the reference's default is 6 (:215); clipped so a short-horizon agent built for the
        # generators alone stays valid under the reference's assert (:236)
        self.control_horizon = int(control_horizon if control_horizon is not None
                                   else min(6, self.prediction_horizon))
        if self.control_horizon > self.prediction_horizon:
            raise AssertionError("control_horizon <= prediction_horizon (:236)")
        self.n_predictions = int(n_predictions)
        self.n_burn_interval = int(n_burn_interval)
        self.step_horizon = int(step_horizon)
        self.n_ideal = int(n_ideal)
        self.scene_config = scene_config
        self.record_interval = int(scene_config.record_interval if scene_config is not None
                                   else kwargs.get("record_interval", 10))
        self._ego = ego_vehicle
        self.ego_vehicle_id = (ego_vehicle.id if ego_vehicle is not None
                               else kwargs.get("ego_vehicle_id", 0))
        self.seed = int(seed)
        self.road_boundary_constraints = road_boundary_constraints
        self.angle_boundary_constraints = angle_boundary_constraints
        self.log_cplex, self.log_agent = log_cplex, log_agent
        self.get_computeTime = get_computeTime
        self.plot_simulation = False           # plotting is outside the path (:305-310)
        self._map_reader, self._eval_stg = map_reader, eval_stg
        self._scene_builder_cls, self._scene_builder = scene_builder_cls, None
        self._first_frame = None
        self._other_vehicles = {}
        world = ego_vehicle.get_world() if ego_vehicle is not None else None
        if world is not None:
            ids = list(other_vehicle_ids)
            self._other_vehicles = dict(zip(ids, world.get_actors(ids)))     # :267-272
        # __steptime (:275-278): record_interval x the simulator's fixed step
        self.steptime = (self.record_interval * world.get_settings().fixed_delta_seconds
                         if world is not None else 0.5)
        self._sensor_listening = False
        self._lidar_feeds = collections.OrderedDict()
        self._local_planner = kwargs.get("local_planner") or PlanFollower()
        self._X_warm = None                    # __X_warmstarting (:290)
        self._U_warm = None                    # __U_warmstarting (:288)
        self.offline_index = 0
        self.refT = None
        self._ref_route = (None if kwargs.get("reference_trajectory") is None
                           else np.asarray(kwargs["reference_trajectory"], np.float64))
        self._road_boundary = None
        self._goal = None
        self._max_distance = float(max_distance)
        self._turn_choices = list(turn_choices)
        if ego_vehicle is not None:            # __make_global_params (:82-120), bbox / steer
            ext = ego_vehicle.bounding_box.extent
            self.ego_lon, self.ego_lat = 2.0 * ext.x, 2.0 * ext.y
            steer = ego_vehicle.get_physics_control().wheels[0].max_steer_angle
            self.mpc_params_steer = float(steer)
        else:
            self.ego_lon, self.ego_lat, self.mpc_params_steer = 3.7, 1.79, 70.0
        if map_reader is not None and ego_vehicle is not None:
            self._setup_road_boundary_conditions(self._turn_choices, self._max_distance)
        self.R = risk.R_COLLISION
        self._moments = {}                 # frame -> (mean [C,T,2], cov [C,2T,2T], K, T)
        self._mean_tangent = {}            # frame -> affine_scale meanNtangent (save_data)
        self._data = {}                    # frame -> data_save dict (save_data / load_data)
        self.data_dir = data_dir           # load_data from .npz files here (None: in memory)
        self.M_big = 10_000                # params.M_big (v8ideal/__init__.py:86)
        self._ws = engine.Workspace(self.device)
        self.prob_lower_save = None
        self.last_records = None
        self._last_rec = None              # (device records, kind, T) of the last generator
        self._last_sbig = False            # do its rows carry S_big (road boundaries)?
        self._qp_request = None            # the frame's QP inputs, set before its step graph
        self._qp_pending = None            # ((run, gen), records, (T, u_order)) enqueued
        self.mpc_params = mpc.MPCParams.reference_defaults(self.mpc_params_steer)
        self._ltv = None                   # (x_init, T_full) -> (xbar, Gamma), first step's
        self._qp = {}
        # step-graph key -> step.StepGraph, least recently used first: a graph holds pinned
        # packs, a device store and workspaces, and the kept modes per OV change from frame to
        # frame in an episode, so the cache is bounded.  One episode's schedule alone needs
        # ph + 1 shapes (T = ph Minkowski, T = ph-1 .. 1 shrinking, the receding affine step):
        # a bound below that recaptures a graph on every step (LRU over a cyclic schedule)
        self._graphs = collections.OrderedDict()
        self.max_graphs = int(kwargs.get("max_graphs", 2 * int(prediction_horizon) + 4))
        if self.max_graphs < 1:
            raise ValueError(f"max_graphs must be >= 1, got {self.max_graphs}")
        self._risk_memo = {}
        self._k_key = self._k_val = None   # _kept_counts' last pmf
        self._eps_memo = {}
        self._u_prev = []                  # executed controls of this shrinking episode (:3186)
        self.last_generator_output = None
        self.last_ctrl = None
        # the reference's prediction functions (prediction.py:19-105 and Trajectron++'s
        # prediction_output_to_trajectories), injectable; do_prediction calls them when eval_stg
        # is a Trajectron++ model (it has no sample_boundary)
        from . import prediction
        self._generate_vehicle_latents = kwargs.get("generate_vehicle_latents",
                                                    prediction.generate_vehicle_latents)
        # opt-in (not in the reference): the predictor's z / predictions stay on the GPU
        # (generate_vehicle_latents(..., keep_on_device=True)), so the step graph copies them
        # device to device instead of through the pinned input pack
        self.keep_predictions_on_device = bool(kwargs.get("keep_predictions_on_device", False))
        self._prediction_output_to_trajectories = kwargs.get(
            "prediction_output_to_trajectories", prediction.prediction_output_to_trajectories)

    # ------------------------------------------------------------------------------------
    # The harness-facing surface (tests/Hz20/__init__.py:183-359): construction, sensor and
    # goal accessors, run_step with the reference's frame gating, and the private
    # __compute_prediction_controls chain do_prediction -> make_ovehicles ->
    # make_local_params -> do_highlevel_control on the device path.

    def _setup_road_boundary_conditions(self, turn_choices, max_distance):
        """:170-200: the route's RoadBoundaryConstraint; its last point is the initial goal."""
        self._road_boundary = self._map_reader.road_boundary_constraints_from_actor(
            self._ego, max_distance, choices=turn_choices, flip_y=True)
        x, y = np.asarray(self._road_boundary.points)[-1]
        self._goal = {"x": float(x), "y": float(y), "is_relative": False}

    def start_sensor(self):
        """:359-363.  The semantic-lidar feed only shapes Trajectron++'s map input, which is
        outside the path: the stand-in just marks the sensor listening."""
        self._sensor_listening = True

    def stop_sensor(self):
        self._sensor_listening = False

    @property
    def sensor_is_listening(self):
        return self._sensor_listening

    def destroy(self):
        """:407-412 (no CARLA resources are held).  The step graphs go to the process's pool
        (step.pool_give), where the next agent of the same shapes takes them captured."""
        from . import step
        self._sensor_listening = False
        for key, g in self._graphs.items():
            step.pool_give(self.device, key + (self.R,), g)
        self._graphs.clear()
        if self._ltv is not None:
            step.ltv_give(self.device, self.prediction_horizon, self._ltv)
            self._ltv = None

    def get_goal(self):
        """:344-345: a copy, as an attribute dict (harness code writes goal.x / goal.y)."""
        from .standins import AttrDict
        return AttrDict(dict(self._goal)) if self._goal is not None else None

    def set_goal(self, x=None, y=None, distance=None, is_relative=True, **kwargs):
        """:350-357."""
        if x is not None and y is not None:
            self._goal = {"x": x, "y": y, "is_relative": is_relative}
        elif distance is not None:
            px, py = self._road_boundary.get_point_from_start(distance)
            self._goal = {"x": float(px), "y": float(py), "is_relative": False}
        else:
            raise NotImplementedError("Unknown method of setting motion planner goal.")

    def get_vehicle_state(self, flip_x=False, flip_y=False):
        """:331-341: the last planning step's x_init once one ran, else the simulator's state
        (flip_y as carlautil does)."""
        x = getattr(self, "x_init", None)
        if x is not None:
            return x
        if self._ego is None:
            raise AttributeError("no ego vehicle and no planning step yet")
        st = _flip_y_state(self._ego)
        if not flip_y:
            st = st * np.array([1.0, -1.0, -1.0, 1.0])
        return st

    def get_final_state(self):
        return self.planned_finalstate

    def do_first_step(self, frame):
        """:3212-3224."""
        self._first_frame = frame
        self._scene_builder = self._scene_builder_cls(
            self, self._map_reader, self._ego, self._other_vehicles, self._lidar_feeds,
            "test", self._first_frame, scene_config=self.scene_config, debug=False)

    def run_step(self, frame, offline_index=0, Tsh=6, shrinking=False, control=None):
        """:3226-3284.  Captures the scene every frame; plans when (frame - first_frame) is a
        multiple of record_interval, past n_burn_interval planning periods and on the
        step_horizon grid; hands the plan to the low-level follower; applies `control` (or the
        follower's) to the ego.  Returns the QP time-out flag; raises InSimulationException
        where the reference's CPLEX solve fails."""
        self.offline_index = offline_index
        if self._first_frame is None:
            self.do_first_step(frame)
        self._scene_builder.capture_trajectory(frame)
        timeout = False
        if (frame - self._first_frame) % self.record_interval == 0:
            frame_id = int((frame - self._first_frame) / self.record_interval)
            if frame_id < self.n_burn_interval:
                pass                                   # burn: collect data only (:3250-3252)
            elif (frame_id - self.n_burn_interval) % self.step_horizon == 0:
                speeds, angles, timeout = self.__compute_prediction_controls(frame, Tsh,
                                                                             shrinking)
                self._local_planner.set_plan(speeds, angles, self.record_interval)
        if not control:
            control = self._local_planner.step()
        if self._ego is not None and hasattr(self._ego, "apply_control"):
            self._ego.apply_control(control)
        return timeout

    def do_prediction(self, frame):
        """:414-467: the frame's scene from the scene builder, then the predictor.

        A Trajectron++ eval_stg (the reference's): generate_vehicle_latents(eval_stg, scene,
        timesteps, num_samples, ph, z_mode=False, gmm_mode=False, full_dist=False,
        all_z_sep=False) (prediction.py:19-105; injectable as the agent keyword
        generate_vehicle_latents) and prediction_output_to_trajectories, returned as the
        reference's AttrDict (scene, timestep, nodes, predictions, z, latent_probs, past_dict,
        ground_truth_dict); make_ovehicles then buckets predictions + z on the GPU.

        An eval_stg with sample_boundary (this library's sampler-tail boundary: per-OV latent
        pmf, initial state and GMM parameters, or Trajectron++'s per-sample parameters, z and
        noise as device tensors): the rollout itself (GMM2D.rsample + Unicycle) runs inside the
        planning step on the GPU, and `boundary` stands where `predictions` / `z` stand."""
        from .standins import AttrDict
        scene = self._scene_builder.get_scene()
        timestep = int((frame - self._first_frame) / self.record_interval)
        ph = self.prediction_horizon
        if hasattr(self._eval_stg, "sample_boundary"):
            b = self._eval_stg.sample_boundary(scene, timestep, self.n_predictions, ph)
            return AttrDict(scene=scene, timestep=timestep, nodes=list(b["nodes"]), boundary=b,
                            latent_probs=np.asarray(b["latent_probs"], np.float64),
                            past_dict={timestep: scene.past(timestep, max_h=10)})
        timesteps = np.array([timestep])
        extra = {"keep_on_device": True} if self.keep_predictions_on_device else {}
        with torch.no_grad():
            z, predictions, nodes, predictions_dict, latent_probs = \
                self._generate_vehicle_latents(self._eval_stg, scene, timesteps,
                                               num_samples=self.n_predictions, ph=ph,
                                               z_mode=False, gmm_mode=False, full_dist=False,
                                               all_z_sep=False, **extra)
        _, past_dict, ground_truth_dict = self._prediction_output_to_trajectories(
            predictions_dict, dt=scene.dt, max_h=10, ph=ph, map=None)
        return AttrDict(scene=scene, timestep=timestep, nodes=nodes, predictions=predictions,
                        z=z, latent_probs=latent_probs, past_dict=past_dict,
                        ground_truth_dict=ground_truth_dict)

    def make_ovehicles(self, result):
        """:469-505 (+ OVehicle.from_trajectron, ovehicle.py:24-117) on do_prediction's result:
        the non-ego nodes' predictions bucketed by z on the GPU (ccmpc_load_predictions +
        ccmpc_bucket), minpos = (x_min, y_min), pasts / ground truths + minpos, the OV actors'
        bboxes.  Returns list[OVehicle] (one device store).  The planning step itself
        (compute_prediction_controls) runs the same stages inside its step graph."""
        from . import ovehicle
        if "predictions" not in result:
            raise ValueError("make_ovehicles takes generate_vehicle_latents' result (this "
                             "do_prediction was given a sample_boundary eval_stg)")
        sampler, minpos, pasts, bboxes = self._ov_inputs(result)
        rows = sampler["rows"]
        pred, z = sampler["predictions"], sampler["z"]
        if torch.is_tensor(pred):
            pred, z = pred.cpu().numpy(), z.cpu().numpy()
        ovs = ovehicle.make_ovehicles(np.asarray(pred)[rows], np.asarray(z)[rows],
                                      sampler["latent_pmf"], minpos, pasts, bboxes=bboxes,
                                      device=self.device)
        gt, ts, nodes = result.get("ground_truth_dict"), result["timestep"], result["nodes"]
        for ov, r in zip(ovs, rows):
            ov.node = nodes[r]
            if gt is not None:
                ov.ground_truth = gt[ts][nodes[r]] + minpos
        return ovs

    def _ov_inputs(self, pred):
        """make_ovehicles (:469-505) up to the bucketing: the non-ego nodes' rows of the
        predictions + z (or of the sampler boundary), minpos = (x_min, y_min), pasts (+ minpos)
        and bboxes of the OV actors."""
        nodes, ts = pred["nodes"], pred["timestep"]
        sel = [i for i, n in enumerate(nodes) if n.id != "ego"]
        scene = pred["scene"]
        minpos = np.array([scene.x_min, scene.y_min])
        pasts = [pred["past_dict"][ts][nodes[i]] + minpos for i in sel]
        bboxes = []
        for i in sel:
            a = self._other_vehicles.get(int(nodes[i].id))
            ext = a.bounding_box.extent if a is not None else None
            bboxes.append([2.0 * ext.x, 2.0 * ext.y] if ext is not None else [4.5, 2.5])
        idx = np.asarray(sel)
        if "predictions" in pred:                # the reference's 5-tuple
            P = pred["predictions"]
            sampler = {"source": "predictions", "predictions": P, "z": pred["z"], "rows": sel,
                       "latent_pmf": np.asarray(pred["latent_probs"], np.float64).reshape(
                           len(nodes), -1)[idx], "N": int(P.shape[1])}
            return sampler, minpos, pasts, np.asarray(bboxes, np.float64)
        b = pred["boundary"]

        run = len(sel) > 0 and sel == list(range(sel[0], sel[0] + len(sel)))

        def rows(x):
            if x is None:
                return None
            if torch.is_tensor(x):
                if len(sel) == x.shape[0]:
                    return x
                if run:        # the OVs are one run of nodes (the ego first or last): a view,
                    return x[sel[0]:sel[0] + len(sel)].contiguous()  # no index upload
                return x[torch.as_tensor(idx, device=x.device)].contiguous()
            return np.asarray(x)[idx]

        sampler = {"init_state": rows(b["init_state"]), "latent_pmf": rows(b["latent_probs"]),
                   "gmm": rows(b["gmm"]), "N": int(b["N"]), "seed": int(b["seed"])}
        if b.get("per_particle"):
            sampler.update(per_particle=True, z=rows(b["z"]), eps=rows(b.get("eps")))
        if "filter_pmf" in b:
            sampler["filter_pmf"] = b["filter_pmf"]
        return sampler, minpos, pasts, np.asarray(bboxes, np.float64)

    def make_local_params(self, frame, Tsh):
        """:514-568 (the ego part): x_init is the previous plan's first state when there is
        one (:526-532, the reference's warm start), else the simulator's; the LTV model is
        built by the QP (solve_planning_qp) at Tsh == ph and kept below it (:2842-2871)."""
        if self._X_warm is not None:
            x_init = np.asarray(self._X_warm[0], np.float64)
        else:
            x_init = _flip_y_state(self._ego)
        self.x_init = x_init
        return x_init

    def load_refT(self, offline_idx, Tsh, x_init):
        """:2768-2787 on the route given as reference_trajectory=: the route point nearest
        x_init, or the next one when the nearest lies behind the third nearest (the
        reference's "closest ahead point"), and Tsh points from there."""
        ref = self._ref_route
        if ref is None:
            raise FileNotFoundError("no reference trajectory (reference_trajectory=) for "
                                    "load_refT (the reference reads out/data/"
                                    "referenceTrajectory/T/refT)")
        norm2 = np.linalg.norm(ref[:, :2] - np.asarray(x_init, np.float64)[:2], axis=1)
        s = np.argsort(norm2)
        if s[0] < s[2]:
            index_min = s[0]
        elif s[0] > s[2]:
            index_min = s[1]
        self.refT = ref[index_min:index_min + Tsh]
        if len(self.refT) < Tsh:
            raise IndexError(f"reference trajectory ends {Tsh - len(self.refT)} steps short of "
                             "the horizon (the reference's objective indexes past it)")
        return self.refT

    def compute_segs_polytopes_and_goal(self, x_init, Tsh):
        """:590-608: the route goal one horizon of speed-limited travel ahead of x_init."""
        v_lim = min(self._ego.get_speed_limit() * 0.28, self.mpc_params.max_v)
        distance = v_lim * self.steptime * Tsh + 1
        segments = self._road_boundary.collect_segs_polytopes_and_goal(
            np.asarray(x_init)[:2], distance)
        return segments, np.asarray(segments.goal, np.float64)

    def __compute_prediction_controls(self, frame, Tsh, shrinking):
        """:3163-3210 on the device path: prediction boundary -> (make_ovehicles + generator +
        QP in compute_prediction_controls) -> warm start (:3187-3193) -> speeds / angles."""
        pred = self.do_prediction(frame)
        sampler, minpos, pasts, bboxes = self._ov_inputs(pred)
        x_init = self.make_local_params(frame, Tsh)
        # do_highlevel_control (:2814, :2840): refT, then the route goal
        ref = self.load_refT(int(self.offline_index / 10) + 1, Tsh, x_init)
        segments, goal = self.compute_segs_polytopes_and_goal(x_init, Tsh)
        speeds, angles, timeout = self.compute_prediction_controls(
            frame, Tsh, shrinking, sampler, minpos, pasts, x_init, goal, ref, bboxes,
            segments=segments)
        self.control_horizon_last = Tsh        # __control_horizon = Tsh (:3170)
        c = self.last_ctrl
        self._U_warm, self._X_warm = c["U_star"], c["X_star"]
        self.planned_finalstate = c["X_star"][-1]
        log = getattr(self, "_step_log", None)
        if log is not None:                    # the harness replay's per-step record
            log.append({"frame": frame, "T": int(Tsh), "shrinking": bool(shrinking),
                        "sampler": sampler, "minpos": minpos, "pasts": pasts,
                        "bboxes": bboxes, "x_init": x_init.copy(), "goal": goal,
                        "ref": np.array(ref), "records": np.array(self.last_records),
                        "speeds": speeds, "angles": angles, "U_star": c["U_star"],
                        "X_star": c["X_star"], "u": c["u"], "segments": segments,
                        "polytopes": c.get("polytopes")})
        return speeds, angles, timeout

    # ------------------------------------------------------------------------------------
    def _saved(self, frame):
        """Saved moments of `frame` as device tensors (a graph step keeps host copies; they are
        uploaded once, when a later step first needs them), or None."""
        e = self._moments.get(frame)
        if e is not None and not torch.is_tensor(e[0]):
            e = (torch.as_tensor(e[0], device=self.device),
                 torch.as_tensor(e[1], device=self.device), e[2], e[3])
            self._moments[frame] = e
        return e

    def _scene(self, ovehicles):
        """All OVs must share one ScenePredictions (the fast path); otherwise pack them."""
        scenes = {id(ov.scene) for ov in ovehicles}
        if len(scenes) == 1 and [ov.ov for ov in ovehicles] == list(range(ovehicles[0].scene.O)):
            return ovehicles[0].scene
        cells = [[np.asarray(p) for p in ov.pred_positions] for ov in ovehicles]
        flat = [c for cs in cells for c in cs]
        store = engine.ParticleStore.from_cells(flat, device=self.device)
        return ScenePredictions(store, [len(c) for c in cells],
                                [ov.past[-1] for ov in ovehicles], [ov.bbox for ov in ovehicles])

    def _cell_risk_host(self, eps_ura, K):
        """Per-cell (chi_r, chi_p, gamma) from the caller's eps_ura (:910-913), host array
        (memoised per (eps_ura, K): a planner asks for the same allocation every step)."""
        key = (eps_ura.tobytes(), eps_ura.shape, tuple(K))
        hit = self._risk_memo.get(key)
        if hit is None:
            hit = self._risk_memo[key] = self._cell_risk_rows(eps_ura, K)
        return hit

    def _cell_risk_rows(self, eps_ura, K):
        ph = self.prediction_horizon
        chi_p = risk._chi2_ppf2(risk.TARGET_P)
        rows = []
        for o, k_o in enumerate(K):
            for k in range(k_o):
                e = float(eps_ura[o, k]) / ph
                rows.append((risk._chi2_ppf2(1 - e), chi_p, risk._norm_ppf(1 - e)))
        return np.asarray(rows, np.float64).reshape(-1, 3)

    def _cell_risk(self, eps_ura, K):
        return torch.as_tensor(self._cell_risk_host(eps_ura, K), device=self.device)

    def _ref(self, ref_traj, T):
        ref = np.asarray([[ref_traj[t][0], ref_traj[t][1]] for t in range(T)], np.float64)
        return torch.as_tensor(ref.reshape(1, T, 2), device=self.device)

    def _state_stats(self, scene, mean0, cov0, yaw=None):
        """ovStateMean/Cov_tau_1 (:864-875): t = 0 mean / variance of x, y, yaw per (ov, k).
        yaw = (yaw_mean at t = 0 [C], yaw0_var [C]) when already on the host."""
        K = scene.K
        if yaw is None:
            l4 = scene.l4_host()
            ym, yv = l4["yaw_mean"][:, 0], l4["yaw0_var"]
        else:
            ym, yv = yaw
        K = list(K)
        first = _first_cells(tuple(K))
        return tuple(tuple(CellGrid(v, K, first) for v in vals) for vals in (
            (mean0[:, 0], mean0[:, 1], np.asarray(ym)),
            (cov0[:, 0, 0], cov0[:, 1, 1], np.asarray(yv))))

    def _l4_lists(self, scene):
        ph = self.prediction_horizon
        l4 = scene.l4_host()
        A, b = l4["A"], l4["b"]
        A_union = _object_grid(ph, max(scene.K), scene.O)
        b_union = _object_grid(ph, max(scene.K), scene.O)
        for c, (o, k) in enumerate(scene.cell_of):
            for t in range(ph):
                A_union[t][k][o] = A[c, t]
                b_union[t][k][o] = b[c, t]
        return LazyVertices(scene, ph), A_union, b_union

    def _ov_in_junction(self, scene, mean0):
        """OVconstraint (:831-851): the Town03 scene-4 T-intersection test, last mode wins."""
        m = mean0[_last_cells(tuple(scene.K))].tolist()             # each OV's last mode
        return any(not (x >= 190 or y <= -80) for x, y in m)

    def _src_cells(self, prev_K, K):
        """data_idx fallback (:2648-2656): mode k reads saved mode k, or the last saved slot."""
        return torch.as_tensor(self._src_cells_host(prev_K, K), device=self.device)

    def _records_to_halfspaces(self, h, scene, T):
        return HalfSpaceList(h, scene.cell_of, T * (T - 1) // 2)

    # ------------------------------------------------------------------------------------
    def compute_obstacle_constraints_GMM_Minkowski_idealprediction(
            self, params, ovehicles, Delta2, Omicron, temp_x, eps_ura, segments, Tsh, ref_traj):
        """v8ideal/__init__.py:781-964.  Returns the reference's 9-tuple
        (constraints, vertices, A_union, b_union, OVconstraint, direct, ovStateMean_tau_1,
        ovStateCov_tau_1, 0)."""
        T, ph = int(Tsh), self.prediction_horizon
        scene = self._scene(ovehicles)
        K = scene.K
        cr = self._cell_risk(np.asarray(eps_ura), K)
        ref = self._ref(ref_traj, T)
        m_scene, c_scene = engine.moments(scene.store, workspace=self._ws) if T < ph else (None, None)
        if T < ph:
            prev = self._saved(params.frame - self.record_interval)
            if prev is None:
                raise KeyError(f"no moments saved for frame {params.frame - self.record_interval}"
                               " (the reference fails to load its pickle here)")
            src = self._src_cells(prev[2], K)
            seed = (self.seed * 1_000_003 + int(params.frame)) & (2**63 - 1)
            mean, cov, status, rec, pl = engine.ideal_minkowski_cycle(
                prev[0], prev[1], src, T, self.n_ideal, ref, cr, seed=seed, R=self.R,
                workspace=self._ws)
            st = status.cpu().numpy()
            if np.any(st != 0):
                raise np.linalg.LinAlgError(f"predict_ideal: conditional covariance not PD in "
                                            f"cells {np.nonzero(st)[0].tolist()}")
        else:
            mean, cov, rec, pl = engine.minkowski_cycle(scene.store, ref, cr, R=self.R,
                                                        workspace=self._ws)
            m_scene, c_scene = mean, cov
        # save_moments (:960): the moments of exactly the particles this step reduced
        self._moments[params.frame] = (mean, cov, list(K), T)
        h = engine.halfspaces(rec)[:, :T * (T - 1) // 2]     # T = 1 keeps one unused slot
        self.last_records = h
        self._last_rec = (rec, mpc.REC_HALFSPACE, T)
        self._last_sbig = False             # the Minkowski rows carry no S_big (:926-939)
        constraints = self._records_to_halfspaces(h, scene, T)
        pl_h = pl.cpu().numpy()
        if T == ph:
            self.prob_lower_save = list(pl_h[-1])          # last cell wins (:947, :961-962)
        mean0 = m_scene[:, 0, :].cpu().numpy()
        cov0 = c_scene[:, 0:2, 0:2].cpu().numpy()
        st_mean, st_cov = self._state_stats(scene, mean0, cov0)
        vertices, A_union, b_union = self._l4_lists(scene)
        direct = _object_grid(scene.O)
        return (constraints, vertices, A_union, b_union, self._ov_in_junction(scene, mean0),
                direct, st_mean, st_cov, 0)

    def compute_obstacle_constraints_GMM_affine(
            self, params, ovehicles, Delta2, Omicron, temp_x, eps_ura, segments, Tsh, ref_traj):
        """v8ideal/__init__.py:1378-1539.  The S_big_repeated term (zero with road boundaries
        off; M_big per chosen non-junction road polytope with them on) belongs to the caller's
        problem: solve_planning_qp adds it (milp.MilpBnB)."""
        T = int(Tsh)
        scene = self._scene(ovehicles)
        K = scene.K
        gamma = self._cell_risk(np.asarray(eps_ura), K)[:, 2].contiguous()
        ref = self._ref(ref_traj, T)
        mean, cov = engine.moments(scene.store, workspace=self._ws)
        if T != scene.T:
            raise ValueError("the affine generator runs on the prediction horizon's particles")
        rec = engine.affine(mean, cov, ref, gamma, R=self.R)
        h = engine.affine_records(rec)
        self.last_records = h
        self._last_rec = (rec, mpc.REC_AFFINE, T)
        self._last_sbig = True              # + S_big_repeated[0, t] on both sides (:1503-1515)
        cons = []
        for c, (o, k) in enumerate(scene.cell_of):
            for t in range(T):
                r = h[c, t]
                if r["status"] != 0:
                    raise engine._lib.record_error(r["status"],
                                                   f"affine constraint (ov={o}, k={k}, t={t})")
                cons.append(HalfSpace(o, k, t, -1, np.array([r["n0"], r["n1"]]), float(r["d"]),
                                      float(r["rhs"]), int(r["side"]), int(r["which"]),
                                      float(r["margin"])))
        mean0 = mean[:, 0, :].cpu().numpy()
        cov0 = cov[:, 0:2, 0:2].cpu().numpy()
        st_mean, st_cov = self._state_stats(scene, mean0, cov0)
        vertices, A_union, b_union = self._l4_lists(scene)
        return (cons, vertices, A_union, b_union, False, _object_grid(scene.O), st_mean, st_cov,
                0)

    def compute_obstacle_constraints_GMM_affine_scale_ideal(
            self, params, ovehicles, Delta2, Omicron, temp_x, eps_ura, segments, Tsh, ref_traj,
            Relax=None):
        """v8ideal/__init__.py:2074-2456: GMM-affine half-spaces with the recursive-feasibility
        covariance scale; at Tsh < ph on a 1e6-sample predict_ideal rollout, with the slopes
        and tangent indices of the previous frame's meanNtangent (save_data / load_data,
        :3064-3104) matched per mode.  Returns the 9-tuple with meanNtangent =
        (mean_p0p1, tangent, cov_p0p1, 0, const_idx)."""
        return self._affine_tangent_generator(params, ovehicles, eps_ura, Tsh, ref_traj,
                                              scaled=True)

    def compute_obstacle_constraints_GMM_affine_robust(
            self, params, ovehicles, Delta2, Omicron, temp_x, eps_ura, segments, Tsh, ref_traj):
        """v8ideal/__init__.py:1541-1878: the same generator without the covariance scale."""
        return self._affine_tangent_generator(params, ovehicles, eps_ura, Tsh, ref_traj,
                                              scaled=False)

    def _affine_tangent_generator(self, params, ovehicles, eps_ura, Tsh, ref_traj, scaled):
        T, ph = int(Tsh), self.prediction_horizon
        scene = self._scene(ovehicles)
        K = scene.K
        cr = self._cell_risk(np.asarray(eps_ura), K)
        ref = self._ref(ref_traj, T)
        m_scene, c_scene = engine.moments(scene.store, workspace=self._ws)
        tangent = const_idx = None
        if T < ph:
            prev = self._saved(params.frame - self.record_interval)
            if prev is None:
                raise KeyError(f"no moments saved for frame {params.frame - self.record_interval}")
            src = self._src_cells(prev[2], K)
            seed = (self.seed * 1_000_003 + int(params.frame)) & (2**63 - 1)
            mean, cov, status = engine.ideal_moments(prev[0], prev[1], src, T, self.n_ideal,
                                                     seed=seed, workspace=self._ws)
            if np.any(status.cpu().numpy() != 0):
                raise np.linalg.LinAlgError("predict_ideal: conditional covariance not PD")
            loaded = self.load_data(params, self.ego_vehicle_id, self.data_dir)
            tangent, const_idx = self._loaded_tangents(loaded, mean.cpu().numpy(), K, T,
                                                       getattr(params, "x_init", None),
                                                       ref.cpu().numpy()[0])
        else:
            mean, cov = m_scene, c_scene
        rec = engine.affine_scale(mean, cov, ref, cr, tangent, const_idx, R=self.R,
                                  scaled=scaled)
        h = engine.affine_records(rec)
        self.last_records = h
        self._last_rec = (rec, mpc.REC_AFFINE, T)
        # the scale-ideal rows carry + S_big_repeated[0, t] (:2394-2414), the robust ones
        # do not (:1828-1849)
        self._last_sbig = bool(scaled)
        cons = []
        O, maxK = scene.O, max(K)
        mean_p0p1 = _object_grid(O, maxK, T)
        tangent_s = _object_grid(O, maxK, T)
        cov_p0p1 = _object_grid(O, maxK, T)
        const_s = _object_grid(O, maxK, T)
        for c, (o, k) in enumerate(scene.cell_of):
            for t in range(T):
                r = h[c, t]
                if r["status"] != 0:
                    raise engine._lib.record_error(
                        r["status"], f"affine-scale constraint (ov={o}, k={k}, t={t})")
                cons.append(HalfSpace(o, k, t, -1, np.array([r["n0"], r["n1"]]), float(r["d"]),
                                      float(r["rhs"]), int(r["side"]), int(r["which"]),
                                      float(r["margin"])))
                mean_p0p1[o][k][t] = np.array([r["mean0"], r["mean1"]])
                tangent_s[o][k][t] = float(r["m"])
                cov_p0p1[o][k][t] = np.array([[r["c00"], r["c01"]], [r["c01"], r["c11"]]])
                const_s[o][k][t] = int(r["which"])
        meanNtangent = (mean_p0p1, tangent_s, cov_p0p1, 0, const_s)
        self._mean_tangent[params.frame] = meanNtangent
        self._moments[params.frame] = (mean, cov, list(K), T)   # save_moments (:2438)
        mean0 = m_scene[:, 0, :].cpu().numpy()
        cov0 = c_scene[:, 0:2, 0:2].cpu().numpy()
        st_mean, st_cov = self._state_stats(scene, mean0, cov0)
        vertices, A_union, b_union = self._l4_lists(scene)
        return (cons, vertices, A_union, b_union, self._ov_in_junction(scene, mean0),
                _object_grid(scene.O), st_mean, st_cov, meanNtangent)

    def predict_and_constrain(self, params, sampler, eps_ura, Tsh, ref_traj, minpos, pasts,
                              bboxes=None, filter_pmf=0.1):
        """One planning frame's prediction + Minkowski constraint generation, as
        do_highlevel_control runs them on the shrinking horizon (v8ideal/__init__.py:2934-2952):
        do_prediction (:414-467, the sampler tail of prediction.py:81-86), make_ovehicles
        (:469-505) and compute_obstacle_constraints_GMM_Minkowski_idealprediction (:781-964).

        sampler: the sampler tail's inputs, in one of two forms --
          per-latent (synthetic): dict(init_state (O, 4), latent_pmf (O, L), gmm (O, L, ph, 5),
              N, seed): z and the noise are Philox draws on the device;
          per-particle (Trajectron++'s boundary, prediction.py:81-86): dict(init_state,
              latent_pmf, gmm (O, N, ph, 5) per-sample parameters, z (O, N) latent ids, eps
              (O, N, ph, 2) or None, N, seed, per_particle=True), gmm / z / eps DEVICE tensors
              as p_y_xz and sample_p leave them (no host round trip); seed keys the noise
              when eps is None.
        Every step is a hipGraph replay (ccmpc.step.StepGraph, cached per shape and sampler
        mode in an LRU of `max_graphs`): inputs up in one copy (the per-particle tensors by
        device copies into the graph's buffers), the sampler + bucketing + generator kernels,
        the records / moments down in one copy, then the 9-tuple over host views (constraints
        built lazily).  At Tsh == ph the generator is the one-launch Minkowski cycle; below ph
        the 1e6-sample ideal rollout of the saved moments (predict_ideal, :2620-2711) fused with
        its moments and half-spaces, beside the sampled scene's moments (the t = 0 statistics).
        The L4 outputs (vertices / A_union / b_union, the heading statistics) come from a
        second graph on a side stream and are read on access.  Returns (ovehicles, 9-tuple);
        the OVehicles' device-backed fields (pred_positions, pred_yaws, vertices) must be read
        before the next step of the same shape -- after it they raise
        (ScenePredictions.check_live)."""
        T, ph = int(Tsh), self.prediction_horizon
        kind = "minkowski" if T == ph else "ideal"
        ovs, g, o, scene, K = self._graph_step(kind, params, sampler, eps_ura, T, ref_traj,
                                               minpos, pasts, bboxes, filter_pmf)
        h = o["records"]
        if kind == "ideal":
            st = o["status"]
            if st.any():
                raise np.linalg.LinAlgError(f"predict_ideal: conditional covariance not PD in "
                                            f"cells {np.nonzero(st)[0].tolist()}")
            self._moments[params.frame] = (o["imean"], o["icov"], list(K), T)   # :960
        else:
            self._moments[params.frame] = (o["mean"], o["cov"], list(K), T)     # :960
            self.prob_lower_save = o["pl"][-1].tolist()       # last cell wins (:947, :961)
        P = T * (T - 1) // 2
        constraints = HalfSpaceList(h, scene.cell_of, P)
        self.last_records = h[:, :P]
        self._last_rec = (g.out.d("rec"), mpc.REC_HALFSPACE, T)
        self._last_sbig = False
        return ovs, self._step_tuple(g, o, scene, K, 0, constraints=constraints)

    def predict_and_constrain_affine(self, params, sampler, eps_ura, Tsh, ref_traj, minpos,
                                     pasts, bboxes=None, filter_pmf=0.1):
        """The receding-horizon frame (do_highlevel_control :2954-2976): do_prediction +
        make_ovehicles + compute_obstacle_constraints_GMM_affine (:1378-1539) as one graph
        replay (sampler -> bucketing -> moments -> GMM-affine), the L4 graph beside it.
        Arguments and result as predict_and_constrain."""
        T = int(Tsh)
        if T != self.prediction_horizon:
            raise ValueError("the affine generator runs on the prediction horizon's particles")
        ovs, g, o, scene, K = self._graph_step("affine", params, sampler, eps_ura, T, ref_traj,
                                               minpos, pasts, bboxes, filter_pmf)
        h = o["records"]
        self.last_records = h
        self._last_rec = (g.out.d("rec"), mpc.REC_AFFINE, T)
        self._last_sbig = True
        st = h["status"]
        if st.any():
            c, t = divmod(int(np.flatnonzero(st.reshape(-1))[0]), T)
            ov, k = scene.cell_of[c]
            raise engine._lib.record_error(h[c, t]["status"],
                                           f"affine constraint (ov={ov}, k={k}, t={t})")
        cons = [HalfSpace(ov, k, t, -1, np.array([r["n0"], r["n1"]]), float(r["d"]),
                          float(r["rhs"]), int(r["side"]), int(r["which"]), float(r["margin"]))
                for c, (ov, k) in enumerate(scene.cell_of) for t, r in enumerate(h[c])]
        out = self._step_tuple(g, o, scene, K, 0, constraints=cons, ov_constraint=False)
        return ovs, out

    def _graph_step(self, kind, params, sampler, eps_ura, T, ref_traj, minpos, pasts, bboxes,
                    filter_pmf):
        """Inputs -> the cached StepGraph of this shape -> replay -> wait -> one snapshot of the
        record-path outputs.  Returns (ovehicles, graph, outputs, scene, K)."""
        from . import ovehicle, step
        ph = self.prediction_horizon
        source = sampler.get("source", "sampler")
        pmf = np.asarray(sampler["latent_pmf"], np.float64)
        O, L = pmf.shape
        N = int(sampler["N"])
        if source == "predictions":              # generate_vehicle_latents' 5-tuple
            init, seed, gmm, pp = None, 0, None, False
            z_in = eps_in = None
            pred_dev = torch.is_tensor(sampler["predictions"])
        else:
            init = np.asarray(sampler["init_state"], np.float64)
            seed, gmm = int(sampler["seed"]), sampler["gmm"]
            pp = bool(sampler.get("per_particle", False))
            z_in, eps_in = sampler.get("z"), sampler.get("eps")
            pred_dev = False
        if pp and z_in is None:
            raise ValueError("per-particle GMM parameters need the injected z (prediction.py:103)")
        if not pp and (z_in is not None or eps_in is not None):
            raise ValueError("injected z / eps go with per_particle=True at the graph step")
        # only the last past point goes into the step; the full pasts are converted for the
        # OVehicles after the launch, while the graph runs
        past_last = np.empty((len(pasts), 2))
        for j, p in enumerate(pasts):
            v = p[-1] if isinstance(p, np.ndarray) and p.ndim == 2 and p.shape[1] == 2 else None
            past_last[j] = v if v is not None else np.asarray(p, np.float64).reshape(-1, 2)[-1]
        bboxes = (_default_bboxes(O) if bboxes is None
                  else np.asarray(bboxes, np.float64).reshape(O, 2))
        K = self._kept_counts(pmf, filter_pmf)
        if min(K) == 0:
            raise ValueError("attempt to get argmin of an empty sequence: an OV has no latent "
                             f"mode with p(z|x) > {filter_pmf} (ovehicle.py:96-97)")
        prev = None
        extra = {}
        if kind == "ideal":
            prev = self._moments.get(params.frame - self.record_interval)
            if prev is None:
                raise KeyError(f"no moments saved for frame {params.frame - self.record_interval}"
                               " (the reference fails to load its pickle here)")
            extra = dict(prev_K=tuple(prev[2]), T_src=int(prev[3]), n_ideal=self.n_ideal)
        key = (kind, O, N, ph, T, L, tuple(K), pp, eps_in is not None, source, pred_dev) + tuple(
            sorted(extra.items()))
        req, self._qp_request = self._qp_request, None
        if req is not None and (req["T"] != T or (T < ph and req["u_prev"] is None)):
            req = None
        if req is not None:
            # the frame's QP inside the graph, right after the record path (before L4): the
            # records are final there and the answer is back before the host has built the
            # 9-tuple.  What the capture bakes in is in the key: the LTV buffers (this agent's,
            # so a pooled graph only serves the agent that took these buffers), whether the
            # frame rebuilds them, the QP parameters, Ts and the ego length
            xbar, gamma = self._ltv_buffers()
            build = T == ph or not self._ltv_built
            rec_kind = mpc.REC_AFFINE if kind == "affine" else mpc.REC_HALFSPACE
            key += ("qp", rec_kind, build, bytes(self.mpc_params), id(xbar),
                    float(self.steptime), float(req["lon"]))
        g = self._graphs.pop(key, None)
        if g is None:
            g = step.pool_take(self.device, key + (self.R,))
        if g is None:
            g = step.StepGraph(O, N, ph, L, K, device=self.device, R=self.R, per_particle=pp,
                               eps_in=eps_in is not None, kind=kind, T=T, source=source,
                               pred_device=pred_dev, **extra)
            while self._graphs and len(self._graphs) >= self.max_graphs:
                self._graphs.popitem(last=False)           # least recently used
        self._graphs[key] = g                              # most recently used
        if req is not None and g.qp is None:
            g.attach_qp(mpc.PlanningQPStep(g.out.d("rec").shape[0], T, ph, kind=rec_kind,
                                           params=self.mpc_params, u_order=mpc.U_ORDER_F,
                                           device=self.device),
                        xbar, gamma, build, Ts=self.steptime, lon=req["lon"])
        g.set_inputs(seed, init, pmf, None if pp else gmm, minpos, ref_traj,
                     self._cell_risk_host(np.asarray(eps_ura), K), past_last, bboxes,
                     filter_pmf=filter_pmf)
        if kind == "ideal":
            src = self._src_cells_host(prev[2], K)
            g.set_ideal_inputs(prev[0], prev[1], src,
                               (self.seed * 1_000_003 + int(params.frame)) & (2**63 - 1))
        if pp:
            g.set_device_inputs(gmm, z_in, eps_in)
        if source == "predictions":
            g.set_predictions(sampler["predictions"], sampler["z"], sampler.get("rows"))
        if req is not None:
            run = g.qp["step"]
            qgen = run.prepare(req["x_init"], req["goal"], req["ref"], req["u_prev"])
        g.launch()
        if req is not None:
            self._ltv_built = True
            self._qp_pending = ((run, qgen), g.out.d("rec"), (T, mpc.U_ORDER_F))
        # host objects that need no output are built while the graph runs
        pasts = [np.asarray(p, np.float64).reshape(-1, 2) for p in pasts]
        st = g.store
        scene = ovehicle.ScenePredictions(st, K, past_last, bboxes)
        scene.bind_generation(g)
        ovs = [ovehicle.OVehicle(scene, j, past=pasts[j]) for j in range(O)]
        g.wait()
        o = g.out.snapshot()            # the record path's outputs in one host copy
        if source == "predictions":      # make_ovehicles' list index on z (:488-491)
            engine.raise_bad_latents(o["zbad"][:O], L)
        ovehicle.check_kept_modes_drawn(o["centre"], K)
        st.counts = o["cnt"].tolist()
        st.offsets = o["off"].tolist()
        scene.cell_pmf, scene.init_center = o["pmf"], o["centre"]
        return ovs, g, o, scene, K

    def _step_tuple(self, g, o, scene, K, mean_tangent, constraints=None, ov_constraint=None):
        """The generator's 9-tuple over one step's outputs; vertices, A_union / b_union and the
        heading part of the state statistics read graph B's L4 outputs on access."""
        ph = self.prediction_horizon
        if constraints is None:
            constraints = HalfSpaceList(o["records"], scene.cell_of, g.T * (g.T - 1) // 2)
        gen = g.generation
        l4 = _LazyL4(g, gen)
        mean0, cov0 = o["mean"][:, 0, :], o["cov"][:, 0:2, 0:2]
        first = _first_cells(tuple(K))
        K = list(K)
        st_mean = (CellGrid(mean0[:, 0], K, first), CellGrid(mean0[:, 1], K, first),
                   CellGrid(_LazyCol(l4, "yaw_mean", 0), K, first))
        st_cov = (CellGrid(cov0[:, 0, 0], K, first), CellGrid(cov0[:, 1, 1], K, first),
                  CellGrid(_LazyCol(l4, "yaw0_var", None), K, first))
        occ = self._ov_in_junction(scene, mean0) if ov_constraint is None else ov_constraint
        return (constraints, LazyVertices(scene, ph), UnionGrid(_LazyCol(l4, "A", None), K, ph,
                                                                first),
                UnionGrid(_LazyCol(l4, "b", None), K, ph, first), occ, _object_grid(scene.O),
                st_mean, st_cov, mean_tangent)

    def _src_cells_host(self, prev_K, K):
        """_src_cells as a host int32 array."""
        maxK_prev = max(prev_K)
        starts = np.concatenate([[0], np.cumsum(prev_K)[:-1]])
        src = []
        for o, k_o in enumerate(K):
            for k in range(k_o):
                d = k if k < maxK_prev else max(maxK_prev - 1, 0)
                if d >= prev_K[o]:
                    raise ValueError(f"saved moments of OV {o} have no mode {d} (the reference "
                                     "reads None there and fails)")
                src.append(int(starts[o] + d))
        return np.asarray(src, np.int32)

    def compute_prediction_controls(self, frame, Tsh, shrinking, sampler, minpos, pasts, x_init,
                                    goal, ref_traj, bboxes=None, apply_robust=True,
                                    segments=None):
        """__compute_prediction_controls (v8ideal/__init__.py:3163-3210) without CARLA: one
        planning frame of the reference harness loop (tests/Hz20/__init__.py:297-359 ->
        run_step :3226-3284) from the sampler inputs on.

          do_prediction + make_ovehicles   the sampler tail and the bucketing (`sampler`: the
                                           dict predict_and_constrain takes)
          make_local_params                O, K, frame, x_init
          do_highlevel_control             shrinking and apply_robust: the Minkowski generator
                                           (:2934-2952; one graph replay at Tsh == ph), else the
                                           GMM-affine generator (:2954-2976); then the QP
                                           (:2850-3043) on the device records
          U_prev / warm start              the executed control U_star.T.ravel()[:nu] appended
                                           (:3186; reset at Tsh == ph, the first shrinking step)

        Returns (speeds, angles, timeout) as the reference does: X_star's speed column and its
        heading reflected about the x axis (utility.npu.reflect_radians_about_x_axis: -psi;
        python-utility is absent, restated), timeout False (the QP has no time limit here).
        Raises InSimulationException where the reference's CPLEX solve fails (:3099-3110).  The
        frame's 9-tuple and QP result stay on the agent (last_generator_output, last_ctrl)."""
        T, ph = int(Tsh), self.prediction_horizon
        pmf = np.asarray(sampler["latent_pmf"], np.float64)
        fp = float(sampler.get("filter_pmf", 0.1))     # one value for K, the graph and buckets
        if T == ph:
            self._u_prev = []
        up = np.concatenate(self._u_prev) if (T < ph and self._u_prev) else None
        self._qp_pending = None
        if not self.road_boundary_constraints:    # the QP's inputs are known before the step
            self._qp_request = dict(T=T, x_init=np.asarray(x_init, np.float64), goal=goal,
                                    ref=ref_traj, u_prev=up, lon=self.ego_lon)
        try:
            return self._prediction_controls(frame, T, shrinking, sampler, minpos, pasts,
                                             x_init, goal, ref_traj, bboxes, apply_robust,
                                             segments, pmf, fp, up)
        finally:
            # a frame that raised after the launch leaves no (run, gen) entry behind for a
            # later direct solve_planning_qp call to mistake for its own
            self._qp_request = self._qp_pending = None

    def _kept_counts(self, pmf, fp):
        """Kept modes per OV, (pmf > fp).sum(1) as a list; memoised on the last pmf (a frame
        asks twice, and small-array numpy reductions are microseconds each)."""
        key = (pmf.tobytes(), pmf.shape, fp)
        if key != self._k_key:
            self._k_val = (pmf > fp).sum(1).tolist()
            self._k_key = key
        return list(self._k_val)

    def _eps_ura(self, O, K):
        """:2909-2916's eps_ura, np.full((O, max K), 0.05 / O), shared read-only per shape."""
        key = (O, max(K))
        e = self._eps_memo.get(key)
        if e is None:
            e = self._eps_memo[key] = np.full(key, 0.05 / O)
            e.setflags(write=False)
        return e

    def _prediction_controls(self, frame, T, shrinking, sampler, minpos, pasts, x_init, goal,
                             ref_traj, bboxes, apply_robust, segments, pmf, fp, up):
        from . import episode
        O = pmf.shape[0]
        if shrinking and apply_robust:
            K = self._kept_counts(pmf, fp)
            eps_ura = self._eps_ura(O, K)                         # :2909-2916
            params = episode.Params(O, K, frame)
            params.x_init = np.asarray(x_init, np.float64)
            ovs, out = self.predict_and_constrain(params, sampler, eps_ura, T, ref_traj, minpos,
                                                  pasts, bboxes, filter_pmf=fp)
        else:
            K = self._kept_counts(pmf, fp)
            eps_ura = self._eps_ura(O, K)
            params = episode.Params(O, K, frame)
            params.x_init = np.asarray(x_init, np.float64)
            ovs, out = self.predict_and_constrain_affine(params, sampler, eps_ura, T, ref_traj,
                                                         minpos, pasts, bboxes, filter_pmf=fp)
        self.last_generator_output = (ovs, out)
        ctrl = self.solve_planning_qp(x_init, goal, ref_traj, T, u_prev=up, lon=self.ego_lon,
                                      segments=segments)
        self.last_ctrl = ctrl
        self._u_prev.append(np.asarray(ctrl["u"][:2]))        # U_star.T.ravel()[:nu] (:3186)
        X = ctrl["X_star"]
        return X[:, 3].copy(), -X[:, 2], False

    def solve_planning_qp(self, x_init, goal, ref_traj, Tsh, u_prev=None, lon=3.7,
                          u_order=mpc.U_ORDER_F, segments=None):
        """do_highlevel_control's QP (:2850-3043) on the device, on the records of the last
        generator call (read in place, never copied to the host).  The LTV model is the one of
        the first shrinking step (the reference keeps its Gamma/x_bar across T < ph steps,
        :2858-2891): it is recomputed when Tsh == ph and reused, sliced, below it, with u_prev
        the executed controls (the reference's U_prev, :3186).  Returns the reference's
        ctrl_result fields {cost, U_star (T, 2), X_star (T, 4), goal, u}; raises
        InSimulationException where CPLEX fails (:3099-3110).

        With road_boundary_constraints the problem is the reference's MILP over the Omicron
        binaries (:2906-2916, compute_road_boundary_constraints :738-758): `segments` (the map
        reader's polytopes and junction mask, compute_segs_polytopes_and_goal) is required and
        the solve is milp.MilpBnB's branch and bound over one road polytope per step, the
        generator's rows carrying S_big where the reference adds it; the result also holds
        `polytopes`, the polytope chosen per step."""
        if self._last_rec is None:
            raise RuntimeError("no constraint records: call a generator first")
        rec, kind, T = self._last_rec
        if int(Tsh) != T:
            raise ValueError(f"records are for T = {T}, not Tsh = {Tsh}")
        ph = self.prediction_horizon
        if self.road_boundary_constraints:
            return self._solve_road_milp(x_init, goal, ref_traj, T, rec, kind, u_prev, lon,
                                         u_order, segments)
        pend, self._qp_pending = self._qp_pending, None
        if pend is not None and pend[1] is rec and pend[2] == (T, u_order):
            run, gen = pend[0]            # enqueued behind the step graph (_graph_step)
        else:
            run, gen = self._qp_launch(x_init, goal, ref_traj, T, rec, kind, u_prev, lon,
                                       u_order)
        return self._qp_result(run.wait(gen), goal)

    def _qp_launch(self, x_init, goal, ref_traj, T, rec, kind, u_prev, lon, u_order):
        """Enqueue solve_planning_qp's device work on the current stream (no wait): the LTV
        rebuild at Tsh == ph, the QP on `rec`, the answer's copy-out and signal."""
        ph = self.prediction_horizon
        xbar, gamma = self._ltv_buffers()
        key = (rec.shape[0], T, kind, u_order)
        run = self._qp.get(key)
        if run is None:
            run = mpc.PlanningQPStep(rec.shape[0], T, ph, kind=kind, params=self.mpc_params,
                                     u_order=u_order, device=self.device)
            self._qp[key] = run
        if T < ph and u_prev is None:
            raise ValueError(f"Tsh = {T} < ph = {ph} needs u_prev, the controls executed "
                             "since the first shrinking step (:3186)")
        build = T == ph or not self._ltv_built
        gen = run.launch(x_init, goal, ref_traj, rec, xbar, gamma, u_prev=u_prev, ltv=build,
                         Ts=self.steptime, lon=lon)
        self._ltv_built = True
        return run, gen

    def _ltv_buffers(self):
        """The LTV model's device buffers (xbar [1, 4 ph], Gamma [1, 4 ph, 2 ph]), rebuilt in
        place at Tsh == ph.  A new agent takes a destroyed agent's from the pool, with them the
        step graphs whose captured QP reads them."""
        from . import step
        if self._ltv is None:
            ph = self.prediction_horizon
            self._ltv = step.ltv_take(self.device, ph) or (
                torch.empty((1, 4 * ph), dtype=torch.float64, device=self.device),
                torch.empty((1, 4 * ph, 2 * ph), dtype=torch.float64, device=self.device))
            self._ltv_built = False
        return self._ltv

    def _qp_result(self, res, goal):
        st = res["status"]
        if st & (mpc.QP_MAXITER | mpc.QP_NUMERIC):
            raise InSimulationException("Optimizer failed to find a solution")
        return {"cost": res["cost"], "U_star": res["U_star"], "X_star": res["X_star"],
                "goal": np.asarray(goal, np.float64), "u": res["u"],
                "skipped_rows": bool(st & mpc.QP_SKIPPED_ROWS)}

    def _solve_road_milp(self, x_init, goal, ref_traj, T, rec, kind, u_prev, lon, u_order,
                         segments):
        """solve_planning_qp with road boundaries: the generator's records packed on the
        device (ccmpc_compact_records) and read back as rows, a half-space (t, tau) record in
        pseudo-cell tau at step t; the LTV model as solve_planning_qp keeps it; MilpBnB."""
        from . import dist, milp
        if segments is None:
            raise ValueError("road_boundary_constraints: segments (compute_segs_polytopes_and_"
                             "goal's polytopes and mask) are required")
        ph = self.prediction_horizon
        if T < ph and u_prev is None:
            raise ValueError(f"Tsh = {T} < ph = {ph} needs u_prev, the controls executed "
                             "since the first shrinking step (:3186)")
        halfspace = kind == mpc.REC_HALFSPACE
        P = T * (T - 1) // 2 if halfspace else T
        C = rec.shape[0]
        Cb = C * (T - 1) if halfspace else C
        base = dict(n=np.zeros((Cb, T, 2)), rhs=np.zeros((Cb, T)), side=np.ones((Cb, T), int),
                    live=np.zeros((Cb, T), bool), sbig=np.full((Cb, T), bool(self._last_sbig)))
        if C and P:
            h = dist.compact_records(rec[:, :P].contiguous(), int(halfspace is False))
            h = h.cpu().numpy().reshape(-1).view(milp._GATHER).reshape(C, P)
            # record (c, p) -> base row (j, t): pseudo-cell c (T - 1) + tau at step t for a
            # half-space (t, tau) record, cell c at step p for an affine one (vectorised)
            if halfspace:
                tt = h["t_tau"].astype(np.int64)
                t, j = tt >> 16, np.arange(C)[:, None] * (T - 1) + (tt & 0xFFFF)
            else:
                t, j = np.broadcast_to(np.arange(P), (C, P)), np.broadcast_to(
                    np.arange(C)[:, None], (C, P))
            base["n"][j, t, 0], base["n"][j, t, 1] = h["n0"], h["n1"]
            base["rhs"][j, t], base["side"][j, t] = h["rhs"], h["side"]
            base["live"][j, t] = h["status"] == 0
        xbar, gamma = self._ltv_buffers()
        if T == ph or not self._ltv_built:
            xb, gm = mpc.ltv(np.asarray(x_init, np.float64).reshape(1, 4), ph, Ts=self.steptime,
                             lon=lon)
            xbar.copy_(xb)
            gamma.copy_(gm)
            self._ltv_built = True
        bnb = milp.MilpBnB(T, gamma, xbar, goal, ref=np.asarray(ref_traj, np.float64)[:T],
                           params=self.mpc_params, u_order=u_order, T_full=ph,
                           u_prev=None if T == ph else u_prev, base=base,
                           segments=milp.RoadSegments(segments), M_big=self.M_big,
                           device=self.device)
        sol = bnb.solve()
        self.last_bnb = dict(bnb.stats)
        if sol is None:
            raise InSimulationException("Optimizer failed to find a solution")
        u = np.asarray(sol["u"], np.float64)
        U = u.reshape(2, T).T.copy() if u_order == mpc.U_ORDER_F else u.reshape(T, 2).copy()
        return {"cost": sol["cost"], "U_star": U, "X_star": sol["X"],
                "goal": np.asarray(goal, np.float64), "u": u, "skipped_rows": False,
                "polytopes": sol["segments"]}

    def _loaded_tangents(self, loaded, mean, K, T, x_init, ref):
        """The previous frame's slopes / tangent indices for every (cell, t) of this frame
        (v8ideal/__init__.py:2190-2276 mode matching, :2349-2370 lookup); an OV without
        loaded data keeps slope-from-ref and const_idx = -1 (the reference's initial value)."""
        C = sum(K)
        tangent = np.zeros((C, T))
        const_idx = np.full((C, T), -1, np.int32)
        c0 = 0
        for o, k_o in enumerate(K):
            mean_l = loaded[0][o] if loaded is not None and o < len(loaded[0]) else None
            if mean_l is not None and len(mean_l) > 0 and x_init is not None:
                cur = [[mean[c0 + k, t] for t in range(T)] for k in range(k_o)]
                picks = _match_modes(mean_l, x_init, cur, k_o, self.M_big)
                for k, idx in enumerate(picks):
                    for t in range(T):
                        tangent[c0 + k, t] = loaded[1][o][idx][t + 1]
                        const_idx[c0 + k, t] = loaded[4][o][idx][t + 1]
            else:   # slope from ref (the same IEEE ops as the kernel's), const_idx stays -1
                for k in range(k_o):
                    tangent[c0 + k] = -(ref[:T, 0] - mean[c0 + k, :, 0]) / (
                        ref[:T, 1] - mean[c0 + k, :, 1])
            c0 += k_o
        return tangent, const_idx

    # ------------------------------------------------------------------------------------
    # Cross-step state: the `agent{id}_frame{f}_cov` data_save dict
    # (v8ideal/__init__.py:2979-3001, save_data :2559-2567, load_data :2547-2557).  It is kept
    # in memory by frame; with `directory` it is also written as an .npz with the generator
    # keys (no pickle).  The QP-side keys (cost, U_star, X_star, ...) belong to the solver,
    # which is outside this path; scalar ones are carried into the .npz when present.

    def data_save(self, out, params, shrinking=True, apply_robust=True):
        """The generator part of do_highlevel_control's data_save (:2979-2993) for a 9-tuple
        `out` returned by one of the compute_obstacle_constraints_* methods."""
        d = {"direct": out[5], "MeanCov": True, "OVconstraint": out[4],
             "ovStateMean_tau_1": out[6], "ovStateCov_tau_1": out[7], "shrinking": shrinking}
        if shrinking and apply_robust and not isinstance(out[8], int):
            d["meanNtangent"] = out[8]
        d["params"] = params
        if getattr(params, "x_init", None) is not None:
            d["x_init"] = np.asarray(params.x_init)
        return d

    def save_data(self, data_save, params, ego_vehicle_id, directory=None):
        """v8ideal/__init__.py:2559-2567 (the pickle is an .npz when `directory` is given)."""
        frame = int(params.frame)
        self._data[frame] = data_save
        if "meanNtangent" in data_save:
            self._mean_tangent[frame] = data_save["meanNtangent"]
        if directory is not None:
            np.savez(self._data_path(directory, ego_vehicle_id, frame),
                     **_data_arrays(data_save, [int(k) for k in np.asarray(params.K)]))

    def load_data(self, params, ego_vehicle_id, directory=None):
        """v8ideal/__init__.py:2547-2557: meanNtangent of frame - record_interval.  The
        reference's load fails (UnboundLocalError) when that frame saved none; so does this
        (KeyError)."""
        frame = int(params.frame) - self.record_interval
        if directory is not None:
            path = self._data_path(directory, ego_vehicle_id, frame)
            try:
                d = np.load(path, allow_pickle=False)
            except OSError as e:
                raise KeyError(f"no saved data for frame {frame}: {e}") from None
            if "mnt_mean" not in d:
                raise KeyError(f"frame {frame} saved no meanNtangent ({path})")
            return _mean_tangent_from_arrays(d)
        if frame not in self._mean_tangent:
            raise KeyError(f"no meanNtangent saved for frame {frame} (the reference fails to "
                           "load its _cov pickle here)")
        return self._mean_tangent[frame]

    @staticmethod
    def _data_path(directory, ego_vehicle_id, frame):
        return os.path.join(directory, f"agent{ego_vehicle_id}_frame{frame}_cov.npz")

    # ------------------------------------------------------------------------------------
    def save_moments(self, ovehicles, O, K, T, Tpred, ego_vehicle_id, params):
        """v8ideal/__init__.py:2575-2618: moments of the given OVs' first T steps, kept on the
        device under params.frame (the generator calls this implicitly)."""
        scene = self._scene(ovehicles)
        mean, cov = engine.moments(scene.store, workspace=self._ws)
        self._moments[params.frame] = (mean[:, :T].contiguous(),
                                       cov[:, :2 * T, :2 * T].contiguous(), list(scene.K), T)

    def saved_moments(self, frame):
        """The reference's pickle content for `frame`: dict(mean_p0p1, cov_p0p1, cross_cov)
        as nested lists [ov][k][t] (and [ov][k][t][tau])."""
        mean, cov, K, T = self._moments[frame]
        mean, cov = _host(mean), _host(cov)
        O, maxK = len(K), max(K)
        mp, cp_, xc = _object_grid(O, maxK, T), _object_grid(O, maxK, T), _object_grid(O, maxK, T, T - 1)
        c = 0
        for o in range(O):
            for k in range(K[o]):
                for t in range(T):
                    mp[o][k][t] = mean[c, t]
                    cp_[o][k][t] = cov[c, 2 * t:2 * t + 2, 2 * t:2 * t + 2]
                    for tau in range(t):
                        xc[o][k][t][tau] = cov[c, 2 * t:2 * t + 2, 2 * tau:2 * tau + 2]
                c += 1
        return dict(mean_p0p1=mp, cov_p0p1=cp_, cross_cov=xc)

    def save_moments_npz(self, frame, path):
        """Write the saved moments of `frame` with the reference pickle's keys (flattened)."""
        mean, cov, K, T = self._moments[frame]
        np.savez(path, mean=_host(mean), cov=_host(cov), K=np.asarray(K), T=T)

    def load_moments_npz(self, frame, path):
        d = np.load(path, allow_pickle=False)
        self._moments[frame] = (torch.as_tensor(d["mean"], device=self.device),
                                torch.as_tensor(d["cov"], device=self.device),
                                [int(k) for k in d["K"]], int(d["T"]))

    def predict_ideal(self, ovehicles, T, ego_vehicle_id, params):
        """v8ideal/__init__.py:2620-2711, materialised: traj_all[ov][k] = (n_ideal, T, 2).
        (The generator never materialises these; it fuses the rollout with the moments.)"""
        prev = self._saved(params.frame - self.record_interval)
        if prev is None:
            raise KeyError(f"no moments saved for frame {params.frame - self.record_interval}")
        K = [ov.n_states for ov in ovehicles]
        src = self._src_cells(prev[2], K)
        seed = (self.seed * 1_000_003 + int(params.frame)) & (2**63 - 1)
        store, status = engine.ideal_rollout(prev[0], prev[1], src, T, self.n_ideal, seed=seed)
        if np.any(status.cpu().numpy() != 0):
            raise np.linalg.LinAlgError("predict_ideal: conditional covariance not PD")
        out, c = {}, 0
        for o, k_o in enumerate(K):
            out[o] = {}
            for k in range(k_o):
                out[o][k] = store.cell_positions(c)
                c += 1
        return out
