"""Stand-ins for the simulator and the learned predictor around the planner's outer surface.

The reference harness (tests/Hz20/__init__.py:37-447) drives v8ideal.MidlevelAgent with
CARLA actors, a MapQuerier, a TrajectronPlusPlusSceneBuilder and a trained Trajectron++.
None of them exist here (no simulator, un-vendored Trajectron++ submodule, no weights), so
these classes supply exactly the attributes the agent reads, with CARLA's own names where
the agent reads CARLA objects:

  StubWorld / StubVehicle     carla.World / carla.Vehicle: tick(), get_settings()
                              .fixed_delta_seconds, get_actors(ids), get_location(),
                              get_transform().rotation, get_velocity(), bounding_box.extent,
                              get_physics_control().wheels[0].max_steer_angle,
                              get_speed_limit(), apply_control(), id
  OnlineConfig                collect/generate/scene/__init__.py OnlineConfig (record_interval)
  PolylineRoadBoundary        RoadBoundaryConstraint's goal rule (collect/generate/map/
                              road.py:621-677) over a polyline route; no road polytopes (the
                              road-boundary MILP variant is out of scope)
  StubMapReader               MapQuerier.road_boundary_constraints_from_actor
                              (collect/generate/map/__init__.py:392)
  ReplaySceneBuilder          TrajectronPlusPlusSceneBuilder's capture_trajectory / get_scene
                              over constant-velocity OV tracks (positions relative to the
                              scene's (x_min, y_min), as Trajectron++ scenes are)
  SyntheticTrajectron         eval_stg: hands the sampler tail the inputs p_y_xz produces
                              (prediction.py:70-86) -- per-OV latent pmf, the unicycle
                              initial state and either per-(latent, step) GMM2D parameters
                              (z and noise drawn on the GPU from a Philox stream keyed by
                              the timestep) or per-sample GMM parameters + z + noise as device
                              tensors, Trajectron++'s own boundary

Everything is seeded and deterministic.  None of this is on the compute path: it is the
replay's input side (SURVEY.md 8d's synthetic generator), like ccmpc.synthetic.
"""
import math

import numpy as np
import torch

from . import episode


class AttrDict(dict):
    """utility.AttrDict (python-utility, absent): a dict with attribute access."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v


class _Vec:
    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = float(x), float(y), float(z)


class _Rot:
    def __init__(self, pitch=0.0, yaw=0.0, roll=0.0):
        self.pitch, self.yaw, self.roll = float(pitch), float(yaw), float(roll)


class _Transform:
    def __init__(self, location, rotation):
        self.location, self.rotation = location, rotation


class OnlineConfig:
    """collect/generate/scene OnlineConfig: the planner reads record_interval (frames per
    planning step) from it."""

    def __init__(self, record_interval=10, node_type=None):
        self.record_interval = int(record_interval)
        self.node_type = node_type


class StubVehicle:
    """A carla.Vehicle with the attributes the agent reads.  Positions are CARLA's (left-handed,
    y down the map); the agent flips y as carlautil does (flip_y=True).  apply_control records
    the last control; tick() moves the vehicle by the control's target speed / angle (a
    kinematic stand-in for the PID follower and the physics)."""

    def __init__(self, world, actor_id, x, y, yaw_deg=0.0, speed=0.0, lon=3.7, lat=1.79,
                 max_steer_deg=70.0, speed_limit_kmh=30.0):
        self.world, self.id = world, int(actor_id)
        self._loc = _Vec(x, y, 0.0)
        self._rot = _Rot(0.0, yaw_deg, 0.0)
        self._speed = float(speed)
        self.bounding_box = AttrDict(extent=_Vec(lon / 2.0, lat / 2.0, 0.75))
        self._max_steer = float(max_steer_deg)
        self._speed_limit = float(speed_limit_kmh)
        self.controls = []

    def get_world(self):
        return self.world

    def get_location(self):
        return _Vec(self._loc.x, self._loc.y, self._loc.z)

    def get_transform(self):
        return _Transform(self.get_location(), _Rot(self._rot.pitch, self._rot.yaw, self._rot.roll))

    def get_velocity(self):
        h = math.radians(self._rot.yaw)
        return _Vec(self._speed * math.cos(h), self._speed * math.sin(h), 0.0)

    def get_physics_control(self):
        return AttrDict(wheels=[AttrDict(max_steer_angle=self._max_steer)])

    def get_speed_limit(self):
        return self._speed_limit

    def apply_control(self, control):
        self.controls.append(control)

    def _advance(self, dt):
        c = self.controls[-1] if self.controls else None
        if isinstance(c, dict) and "target_speed" in c:
            self._speed = float(c["target_speed"])
            # the agent already reflected the plan's heading back into CARLA's frame (:3208)
            self._rot.yaw = math.degrees(float(c["target_angle"]))
        h = math.radians(self._rot.yaw)
        self._loc.x += self._speed * math.cos(h) * dt
        self._loc.y += self._speed * math.sin(h) * dt

    def destroy(self):
        pass


class StubWorld:
    """carla.World in synchronous mode: tick() advances the frame counter (and the vehicles)."""

    def __init__(self, first_frame=1000, fixed_delta_seconds=0.05):
        self.frame = int(first_frame)
        self._settings = AttrDict(fixed_delta_seconds=float(fixed_delta_seconds),
                                  synchronous_mode=True)
        self.actors = {}

    def add(self, vehicle):
        self.actors[vehicle.id] = vehicle
        return vehicle

    def get_settings(self):
        return self._settings

    def get_actors(self, ids):
        return [self.actors[int(i)] for i in ids]

    def tick(self):
        for a in self.actors.values():
            a._advance(self._settings.fixed_delta_seconds)
        self.frame += 1
        return self.frame


class PolylineRoadBoundary:
    """RoadBoundaryConstraint over a polyline route (points in the planner's flipped frame):
    collect_segs_polytopes_and_goal's goal rule (road.py:663-666: the route point nearest the
    position, then the first point at or past min(its distance + distance, path length)), and
    get_point_from_start (:621-637, linear instead of the cubic spline between points).  The
    road segments (cover_along_path_varyingsize, :468-556, sizes from the spline curvature)
    are restated for a polyline: rectangles of `seg_len` metres along the route (one per run
    of route edges, `overlap` metres longer at each end so neighbours overlap), `lane_width`
    wide, in H-form A x <= b; a rectangle whose centre lies within one of the `junctions`
    (x, y, radius) discs is a junction polytope (mask True)."""

    def __init__(self, points, lane_width=3.5, seg_len=10.0, overlap=0.5, junctions=()):
        self.points = np.asarray(points, np.float64).reshape(-1, 2)
        seg = np.linalg.norm(np.diff(self.points, axis=0), axis=1)
        self.distances = np.concatenate([[0.0], np.cumsum(seg)])
        self._cover(float(lane_width), float(seg_len), float(overlap), junctions)

    def _cover(self, lane_width, seg_len, overlap, junctions):
        polys, mask, starts = [], [], []
        d, hw = self.distances, 0.5 * lane_width
        s0 = 0.0
        while s0 < d[-1] - 1e-9:
            s1 = min(s0 + seg_len, d[-1])
            p0, p1 = self.get_point_from_start(s0), self.get_point_from_start(s1)
            e = (p1 - p0) / max(np.linalg.norm(p1 - p0), 1e-12)
            nrm = np.array([-e[1], e[0]])
            A = np.stack([e, -e, nrm, -nrm])
            b = np.array([e @ p1 + overlap, -(e @ p0) + overlap, nrm @ p0 + hw, -(nrm @ p0) + hw])
            ctr = 0.5 * (p0 + p1)
            polys.append((A, b))
            mask.append(any(np.hypot(ctr[0] - jx, ctr[1] - jy) <= r for jx, jy, r in junctions))
            starts.append(s0)
            s0 = s1
        self.road_segs = AttrDict(polytopes=polys, mask=np.asarray(mask, bool),
                                  distances=np.asarray(starts))

    @property
    def path_length(self):
        return float(self.distances[-1])

    def get_point_from_start(self, distance):
        d = self.distances
        if not 0.0 <= distance <= d[-1]:
            return self.points[-1]
        return np.array([np.interp(distance, d, self.points[:, 0]),
                         np.interp(distance, d, self.points[:, 1])])

    def _poly_id(self, dist):
        return int(np.searchsorted(self.road_segs.distances, dist, side="right")) - 1

    def collect_segs_polytopes_and_goal(self, position, distance):
        beg_idx = int(np.argmin(np.linalg.norm(self.points - np.asarray(position)[:2], axis=1)))
        beg_dist = self.distances[beg_idx]
        end_dist = min(beg_dist + distance, self.path_length)
        # distance_to_point is indexed by the right-closed intervals (d[j-1], d[j]] -> point j
        j = max(int(np.searchsorted(self.distances, end_dist, side="left")), 1)
        n = len(self.road_segs.polytopes)
        beg_id = max(self._poly_id(beg_dist) - 1, 0)                # road.py:667-671
        end_id = min(self._poly_id(end_dist) + 1, n - 1)
        return AttrDict(polytopes=self.road_segs.polytopes[beg_id:end_id],
                        polytope_ids=list(range(beg_id, end_id)),
                        mask=self.road_segs.mask[beg_id:end_id], goal=self.points[j].copy())


class StubMapReader:
    """MapQuerier.road_boundary_constraints_from_actor (map/__init__.py:392) returning a
    PolylineRoadBoundary along the given route (road_kwargs: its lane width, segment length
    and junction discs)."""

    def __init__(self, route_points, **road_kwargs):
        self.route_points = np.asarray(route_points, np.float64)
        self.road_kwargs = road_kwargs

    def road_boundary_constraints_from_actor(self, actor, max_distance, choices=(), flip_y=True):
        return PolylineRoadBoundary(self.route_points, **self.road_kwargs)


def straight_route(start, heading, length=200.0, step=2.0):
    """A straight route from `start` (flipped frame) along `heading` (radians)."""
    s = np.arange(0.0, length + step, step)
    return np.stack([start[0] + s * math.cos(heading), start[1] + s * math.sin(heading)], 1)


class _Node:
    """A Trajectron++ scene node: id, and get(range, state) over the scene builder's track (the
    call prediction_output_to_trajectories makes): rows for timesteps lo .. hi inclusive, NaN
    outside the recorded track, as Trajectron++'s Node.get pads."""

    def __init__(self, node_id, tracks=None):
        self.id = node_id
        self._tracks = tracks

    def get(self, tr_scene, state):
        lo, hi = int(tr_scene[0]), int(tr_scene[1])
        tr = self._tracks[self.id]
        out = np.full((hi - lo + 1, 2), np.nan)
        for k, ts in enumerate(range(lo, hi + 1)):
            if 0 <= ts < len(tr):
                out[k] = tr[ts]
        return out

    def __repr__(self):
        return f"VEHICLE/{self.id}"


class ReplayScene:
    """The Trajectron++ scene of one planning frame: x_min / y_min (the offset its positions are
    relative to), dt, nodes, and each node's history (prediction_output_to_trajectories'
    past_dict, max_h steps, relative positions)."""

    def __init__(self, x_min, y_min, dt, nodes, tracks, timestep):
        self.x_min, self.y_min, self.dt = x_min, y_min, dt
        self.nodes = nodes
        self._tracks, self.timestep = tracks, timestep

    def past(self, timestep, max_h=10):
        out = {}
        for n in self.nodes:
            tr = self._tracks[n.id]
            lo = max(0, timestep - max_h)
            out[n] = np.asarray(tr[lo:timestep + 1], np.float64)
        return out

    def state(self, node, timestep):
        """Unicycle state [x, y, heading, speed] (relative) of `node` at `timestep`."""
        return self._tracks[node.id + "/state"][timestep]


class ReplaySceneBuilder:
    """TrajectronPlusPlusSceneBuilder (collect/generate/scene/v3_2/trajectron_scene.py) with the
    constructor the agent calls (v8ideal/__init__.py:3212-3224): capture_trajectory(frame)
    records every OV's position each record_interval frames; get_scene() returns the frame's
    ReplayScene.  OVs move at constant velocity from the world's actors' current states."""

    def __init__(self, agent, map_reader, ego_vehicle, other_vehicles, lidar_feeds, scene_name,
                 first_frame, scene_config=None, debug=False, minpos=(150.0, -120.0)):
        self.ego, self.other_vehicles = ego_vehicle, other_vehicles
        self.first_frame = int(first_frame)
        self.record_interval = scene_config.record_interval if scene_config else 10
        self.dt = self.record_interval * ego_vehicle.get_world().get_settings().fixed_delta_seconds
        self.minpos = np.asarray(minpos, np.float64)
        self.tracks = {}
        self.nodes = [_Node("ego", self.tracks)] + [_Node(str(i), self.tracks)
                                                    for i in other_vehicles]
        self.tracks.update({n.id: [] for n in self.nodes})
        for n in self.nodes:
            self.tracks[n.id + "/state"] = []
        self.timestep = -1

    def _actor(self, node):
        return self.ego if node.id == "ego" else self.other_vehicles[int(node.id)]

    def capture_trajectory(self, frame):
        if (frame - self.first_frame) % self.record_interval:
            return
        self.timestep = (frame - self.first_frame) // self.record_interval
        for n in self.nodes:
            a = self._actor(n)
            loc, rot, vel = a.get_location(), a.get_transform().rotation, a.get_velocity()
            rel = np.array([loc.x, -loc.y]) - self.minpos            # flip_y, scene-relative
            self.tracks[n.id].append(rel)
            self.tracks[n.id + "/state"].append(
                np.array([rel[0], rel[1], -math.radians(rot.yaw), math.hypot(vel.x, vel.y)]))

    def get_scene(self):
        return ReplayScene(self.minpos[0], self.minpos[1], self.dt, self.nodes, self.tracks,
                           self.timestep)


class SyntheticTrajectron:
    """eval_stg stand-in.  sample_boundary(scene, timestep, num_samples, ph) returns what the
    sampler tail receives from Trajectron++ (prediction.py:70-86) for every node of the scene
    (the ego included, as generate_vehicle_latents returns it; make_ovehicles skips it):

      nodes, init_state (n, 4) [x, y, heading, speed] relative to the scene, latent_probs (n, L)
      per_particle=False: gmm (n, L, ph, 5) per-(latent, step) GMM2D parameters, seed (the
          sampler draws z and the noise on the GPU from it)
      per_particle=True:  gmm (n, N, ph, 5), z (n, N) latent ids, eps (n, N, ph, 2) -- device
          tensors, drawn with torch on the device as p_y_xz leaves them

    The per-latent parameters are ccmpc.episode.synthetic_gmm's, fixed per node; the draws are
    keyed by (seed, timestep), so a frame's predictions are reproducible."""

    def __init__(self, L=25, ph=8, seed=0, per_particle=False, with_eps=True, device="cuda"):
        self.L, self.ph, self.seed = int(L), int(ph), int(seed)
        self.per_particle, self.with_eps = bool(per_particle), bool(with_eps)
        self.device = device
        self._gmm = {}

    def _node_params(self, i):
        if i not in self._gmm:
            _, pmf, gmm = episode.synthetic_gmm(1, L=self.L, T=self.ph,
                                                seed=20251015 + 97 * self.seed + i)
            self._gmm[i] = (pmf[0], gmm[0])
        return self._gmm[i]

    def sample_boundary(self, scene, timestep, num_samples, ph):
        assert ph == self.ph
        nodes = list(scene.nodes)
        n = len(nodes)
        init = np.stack([scene.state(nd, timestep) for nd in nodes])
        pmf = np.stack([self._node_params(i)[0] for i in range(n)])
        gmm = np.stack([self._node_params(i)[1] for i in range(n)])
        seed = (self.seed * 7919 + int(timestep)) & 0x7FFFFFFF
        out = AttrDict(nodes=nodes, init_state=init, latent_probs=pmf, N=int(num_samples),
                       seed=seed, per_particle=self.per_particle)
        if not self.per_particle:
            out.gmm = gmm
            return out
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        pmf_t = torch.as_tensor(pmf, device=self.device)
        z = torch.multinomial(pmf_t, int(num_samples), replacement=True, generator=g)
        base = torch.as_tensor(gmm, dtype=torch.float32, device=self.device)    # (n, L, ph, 5)
        pp = torch.gather(base, 1, z[:, :, None, None].expand(n, int(num_samples), ph, 5))
        # the GRU decoder conditions every sample on its own history: per-sample jitter
        pp = pp + 0.02 * torch.randn(pp.shape, generator=g, device=self.device,
                                     dtype=torch.float32)
        out.gmm, out.z = pp.contiguous(), z.to(torch.int32).contiguous()
        out.eps = (torch.randn((n, int(num_samples), ph, 2), generator=g, device=self.device,
                               dtype=torch.float32) if self.with_eps else None)
        return out


def town03_scene(world=None, n_ov=1, ego_xy=(140.0, 81.0), ego_yaw_deg=0.0, ego_speed=6.0,
                 ov_gap=25.0, ov_speed=4.0, ov_lateral=0.0, first_frame=1000):
    """A stand-in for the Town03 scene-4 setup of the Monte-Carlo test (tests/Hz20/params.py's
    MONTECARLO_scene4_*): the ego on a straight road (CARLA frame); n_ov OVs driving parallel
    to it, OV j ov_gap + 8 j metres ahead and ov_lateral metres to the side (alternating
    sides); and the route the map reader follows.  Returns (world, ego, ov_ids, map_reader)."""
    world = world or StubWorld(first_frame=first_frame)
    ego = world.add(StubVehicle(world, 1, ego_xy[0], ego_xy[1], ego_yaw_deg, ego_speed))
    ids = []
    h = math.radians(ego_yaw_deg)
    for j in range(n_ov):
        lat = ov_lateral * (1.0 if j % 2 == 0 else -1.0)
        x = ego_xy[0] + (ov_gap + 8.0 * j) * math.cos(h) - lat * math.sin(h)
        y = ego_xy[1] + (ov_gap + 8.0 * j) * math.sin(h) + lat * math.cos(h)
        ov = world.add(StubVehicle(world, 100 + j, x, y, ego_yaw_deg, ov_speed))
        ids.append(ov.id)
    start = np.array([ego_xy[0], -ego_xy[1]])
    route = straight_route(start, -math.radians(ego_yaw_deg))
    return world, ego, ids, StubMapReader(route)


class TrajectronModel:
    """eval_stg stand-in shaped like a real Trajectron++ model object: it has NO sample_boundary,
    so MidlevelAgent.do_prediction takes the reference's own route -- generate_vehicle_latents
    (prediction.py:19-105) -> the 5-tuple -> make_ovehicles on predictions + z.  `inner` (a
    SyntheticTrajectron) supplies the latent pmfs / GMM parameters that stand where the GRU
    decoder's outputs would; use it with generate_vehicle_latents below (agent keyword
    generate_vehicle_latents=standins.generate_vehicle_latents)."""

    def __init__(self, inner):
        self.inner = inner
        self.device = inner.device


def generate_vehicle_latents(eval_stg, scene, timesteps, num_samples=200, ph=8, z_mode=False,
                             gmm_mode=False, full_dist=False, all_z_sep=False,
                             keep_on_device=False):
    """prediction.py:19-105 for a TrajectronModel stand-in: the reference's 5-tuple
    (z (nodes, N) int64, predictions (nodes, N, ph, 2) float32 scene-relative, nodes,
    predictions_dict, latent_probs) as numpy arrays, the samples drawn by the library's own
    sampler tail (ccmpc_sample_unicycle_ex) from the inner stand-in's boundary.  The non-ego
    nodes are drawn as OVs 0 .. O-1 in node order (the Philox streams the sample_boundary route
    keys them by), so both routes see the same particles; the ego's row is drawn after them.
    keep_on_device: z and predictions as device tensors (ccmpc.prediction's opt-in), built on
    the GPU from the sampler's store without a host round trip."""
    from . import engine
    b = eval_stg.inner.sample_boundary(scene, int(np.asarray(timesteps).reshape(-1)[0]),
                                       num_samples, ph)
    nodes = list(b.nodes)
    N = int(b.N)
    n = len(nodes)
    rows = [i for i, nd in enumerate(nodes) if nd.id != "ego"]
    rows += [i for i, nd in enumerate(nodes) if nd.id == "ego"]
    pred = np.empty((n, N, ph, 2), np.float32)
    z = np.empty((n, N), np.int64)
    sel = np.asarray(rows)
    pp = bool(b.get("per_particle", False))

    def pick(x):
        if x is None:
            return None
        if isinstance(x, torch.Tensor):
            return x[torch.as_tensor(sel, device=x.device)]
        return np.asarray(x)[sel]
    zs, store = engine.sample_unicycle(
        np.asarray(b.init_state)[sel], np.asarray(b.latent_probs)[sel], pick(b.gmm), N, ph,
        seed=b.seed, device=eval_stg.device, z=pick(b.get("z")) if pp else None,
        eps=pick(b.get("eps")) if pp else None, per_particle=pp)
    ts = int(np.asarray(timesteps).reshape(-1)[0])
    if keep_on_device:
        dev = store.pos.device
        inv = torch.as_tensor(np.argsort(sel), device=dev)      # node i <- drawn row inv[i]
        off = torch.as_tensor(np.asarray(store.offsets[:n], np.int64), device=dev)
        idx = off[:, None] + torch.arange(N, device=dev)[None]  # (n, N) store columns
        cols = store.pos[:, idx]                                 # (2 ph, n, N)
        pred_d = cols.reshape(ph, 2, n, N).permute(2, 3, 0, 1)[inv].contiguous()
        z_d = zs.to(torch.int64)[inv].contiguous()
        pdict = {ts: {nd: pred_d[i][None] for i, nd in enumerate(nodes)}}
        return z_d, pred_d, nodes, pdict, np.asarray(b.latent_probs, np.float64)
    pos = store.pos.cpu().numpy()
    zh = zs.cpu().numpy()
    for j, r in enumerate(rows):
        o = store.offsets[j]
        pred[r] = pos[:, o:o + N].reshape(ph, 2, N).transpose(2, 0, 1)
        z[r] = zh[j]
    pdict = {ts: {nd: pred[i][None] for i, nd in enumerate(nodes)}}
    return z, pred, nodes, pdict, np.asarray(b.latent_probs, np.float64)
