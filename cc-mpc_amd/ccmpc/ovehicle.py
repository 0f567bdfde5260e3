"""Other-vehicle particle clouds, mirroring collect/in_simulation/midlevel/ovehicle.py.

The reference keeps each OV's bucketed predictions as Python lists of NumPy arrays
(pred_positions[k]: (N_k, T, 2) float64, pred_yaws[k]: (N_k, T)).  Here every OV of a planning
step shares ONE device-resident plane-major store (ScenePredictions); the list-of-arrays fields
the reference exposes are materialised on the host only when someone reads them.
"""
import numpy as np
import torch

from . import engine

DEFAULT_BBOX = np.array([4.5, 2.5])   # ovehicle.py:19


def _host(x):
    return x.cpu().numpy() if torch.is_tensor(x) else np.array(x)


class ScenePredictions:
    """Bucketed particle clouds of all OVs of one planning step (cells in (ov, k) order)."""

    def __init__(self, store, K, past_last, bbox, cell_pmf=None, init_center=None):
        self.store = store
        self.K = [int(k) for k in K]
        self.T = store.T
        self.cell_of = []                       # (ov, k) per cell
        for o, k in enumerate(self.K):
            self.cell_of += [(o, j) for j in range(k)]
        assert len(self.cell_of) == store.n_cells
        self.past_last = np.asarray(past_last, np.float64).reshape(len(self.K), 2)
        self.bbox = np.asarray(bbox, np.float64).reshape(len(self.K), 2)
        self.cell_pmf = cell_pmf
        self.init_center = init_center
        self._l4 = None
        self._owner = None                      # (graph, generation) when over a graph's buffers

    def bind_generation(self, owner):
        """This scene lives in the buffers of `owner` (a step.MinkowskiStepGraph) as its current
        launch left them; a later replay of the same graph overwrites them, after which every
        read of the device store raises instead of silently returning the newer frame's data
        (the reference's per-frame OVehicles are independent)."""
        self._owner = (owner, owner.generation)

    def check_live(self):
        if self._owner is not None and self._owner[0].generation != self._owner[1]:
            raise RuntimeError(
                "stale planning-step data: this frame's particle store was overwritten by a "
                "later step of the same shape (read vertices / pred_positions / pred_yaws "
                "before the next predict_and_constrain, or copy them)")

    @property
    def O(self):
        return len(self.K)

    def first_cell(self, ov):
        return int(sum(self.K[:ov]))

    def cell_past_last(self):
        return np.repeat(self.past_last, self.K, axis=0)

    def cell_bbox(self):
        return np.repeat(self.bbox, self.K, axis=0)

    def l4(self, with_yaw=False, with_vertices=False):
        """Headings / vertices / L4 over all ph steps (cached per scene)."""
        need = (self._l4 is None or (with_yaw and self._l4["yaw"] is None)
                or (with_vertices and self._l4["vertices"] is None))
        self.check_live()
        if need:
            self._l4 = engine.l4(self.store, self.cell_past_last(), self.cell_bbox(),
                                 with_yaw=with_yaw, with_vertices=with_vertices)
        return self._l4

    _L4_HOST = ("A", "b", "yaw_mean", "yaw0_var")

    def l4_host(self):
        """The per-(cell, t) L4 outputs (A, b, yaw_mean, yaw0_var) as host arrays, brought over
        in ONE device-to-host copy and kept with the scene's L4 (each .cpu() is a synchronising
        round trip of its own)."""
        l4 = self.l4()
        h = l4.get("_host")
        if h is None:
            flat = torch.cat([l4[k].reshape(-1) for k in self._L4_HOST]).cpu().numpy()
            h, o = {}, 0
            for k in self._L4_HOST:
                n = l4[k].numel()
                h[k] = flat[o:o + n].reshape(tuple(l4[k].shape))
                o += n
            l4["_host"] = h
        return h


class OVehicle:
    """Mirror of ovehicle.py:OVehicle (fields :119-131), backed by a ScenePredictions."""

    def __init__(self, scene, ov, node=None, past=None, ground_truth=None):
        self.scene = scene
        self.ov = ov
        self.node = node
        self.T = scene.T
        self.past = np.asarray(past if past is not None else scene.past_last[ov:ov + 1])
        self.ground_truth = ground_truth
        self.bbox = scene.bbox[ov]
        self.n_states = scene.K[ov]
        self._pos = None
        self._yaw = None

    @property
    def cells(self):
        c0 = self.scene.first_cell(self.ov)
        return list(range(c0, c0 + self.n_states))

    @property
    def latent_pmf(self):
        if self.scene.cell_pmf is None:
            st = self.scene.store
            st.sync_counts() if st.counts is None else None
            n = np.array([st.counts[c] for c in self.cells], float)
            return n / n.sum()
        return _host(self.scene.cell_pmf[self.cells[0]:self.cells[-1] + 1])

    @property
    def init_center(self):
        if self.scene.init_center is None:
            return np.array([self.pred_positions[k][:, self.T - 1].mean(0)
                             for k in range(self.n_states)])
        return _host(self.scene.init_center[self.cells[0]:self.cells[-1] + 1])

    @property
    def n_predictions(self):
        return int(sum(p.shape[0] for p in self.pred_positions))

    @property
    def pred_positions(self):
        """list over modes of (N_k, T, 2) float64 world positions (host copy, cached)."""
        if self._pos is None:
            self.scene.check_live()
            self._pos = [self.scene.store.cell_positions(c) for c in self.cells]
        return self._pos

    @property
    def pred_yaws(self):
        """list over modes of (N_k, T) headings (ovehicle.py:72-76), computed on the GPU."""
        if self._yaw is None:
            self.scene.check_live()
            st = self.scene.store
            if st.counts is None:
                st.sync_counts()
            yaw = self.scene.l4(with_yaw=True)["yaw"]
            self._yaw = [yaw[:, st.offsets[c]:st.offsets[c] + st.counts[c]].T.cpu().numpy()
                         for c in self.cells]
        return self._yaw


def scene_from_positions(ov_cells, pasts, bboxes=None, device="cuda", dtype=torch.float64):
    """Reference-format input (per OV a list over kept modes of (N_k, T, 2) world positions,
    i.e. ovehicle.pred_positions) -> list[OVehicle] sharing one device store."""
    K = [len(c) for c in ov_cells]
    flat = [c for cells in ov_cells for c in cells]
    store = engine.ParticleStore.from_cells(flat, device=device, dtype=dtype)
    bboxes = np.tile(DEFAULT_BBOX, (len(K), 1)) if bboxes is None else bboxes
    pasts = [np.asarray(p, np.float64).reshape(-1, 2) for p in pasts]
    scene = ScenePredictions(store, K, [p[-1] for p in pasts], bboxes)
    return [OVehicle(scene, o, past=pasts[o]) for o in range(len(K))]


def check_kept_modes_drawn(centre, K):
    """A kept mode (p(z|x) > filter) that drew no particle of its own: the reference builds
    `np.array([])` for it (v8ideal/__init__.py:493-494) and fails in from_trajectron at
    `ps[:,0,1]` (ovehicle.py:72, IndexError) before any rare particle is assigned.  The device
    bucketing gives that mode the centre 0 / 0 = NaN (the mean of its own particles, :80), so
    no rare particle is ever assigned to it; the drop-in raises the reference's error instead of
    returning that cell.  centre: per-cell init_center (host, (C, 2)), cells in (ov, k) order."""
    centre = np.asarray(centre, np.float64)
    # finite centres sum to a finite value; one NaN makes it NaN (a Python sum over the list:
    # numpy's reduction machinery costs ~2 us on these few values)
    s = sum(centre.reshape(-1).tolist())
    if s == s:
        return
    bad = np.flatnonzero(np.isnan(centre.reshape(-1, 2)).any(1))
    if bad.size:
        c = int(bad[0])
        first = np.concatenate([[0], np.cumsum(K)])
        o = int(np.searchsorted(first, c, side="right") - 1)
        raise IndexError(f"too many indices for array: kept mode {c - int(first[o])} of OV {o} "
                         "drew no particle (ovehicle.py:72 fails on its empty prediction array)")


def make_ovehicles(predictions, z, latent_probs, minpos, pasts, bboxes=None, T=None,
                   filter_pmf=0.1, device="cuda"):
    """v8ideal/__init__.py:469-505 + OVehicle.from_trajectron (ovehicle.py:24-117) on the GPU.

    predictions: either a sample-order F32 ParticleStore from engine.sample_unicycle (one cell
    per OV) with z [O, N] int32 on the device, or host arrays (O, N, T, 2) float32 + (O, N).
    latent_probs: (O, L) host p(z|x).  Returns list[OVehicle] sharing one ScenePredictions."""
    dev = engine.require_device(device)
    if isinstance(predictions, engine.ParticleStore):
        store_in, z_dev = predictions, z
    else:
        pred = np.asarray(predictions, np.float32)
        O, N, T_, _ = pred.shape
        store_in = engine.ParticleStore(T_, [N] * O, dtype=torch.float32, device=dev, align=4,
                                        origin=np.zeros((O, 2)))
        host = np.zeros((2 * T_, store_in.ld), np.float32)
        for o in range(O):
            host[:, store_in.offsets[o]:store_in.offsets[o] + N] = pred[o].transpose(1, 2, 0).reshape(2 * T_, N)
        store_in.pos.copy_(torch.from_numpy(host))
        z_dev = torch.as_tensor(np.asarray(z, np.int32), device=dev)
    O = z_dev.shape[0]
    mp = np.asarray(minpos, np.float64)
    mp = np.tile(mp.reshape(2), (O, 1)) if mp.size == 2 else mp.reshape(O, 2)
    store, K, pmf, centre = engine.bucket(z_dev, store_in, latent_probs, mp,
                                          filter_pmf=filter_pmf)
    store.sync_counts()
    check_kept_modes_drawn(centre.cpu().numpy(), K)
    pasts = [np.asarray(p, np.float64).reshape(-1, 2) for p in pasts]
    bboxes = np.tile(DEFAULT_BBOX, (O, 1)) if bboxes is None else np.asarray(bboxes)
    scene = ScenePredictions(store, K, [p[-1] for p in pasts], bboxes, pmf, centre)
    return [OVehicle(scene, o, past=pasts[o]) for o in range(O)]
