"""One planning step of v8ideal's prediction + constraint path as hipGraph replays.

Per planning frame the reference runs (v8ideal/__init__.py:2934-2976 -> :414-505, :781-964,
:1378-1539):

    do_prediction       Trajectron++ sample (prediction.py:81-86)
    make_ovehicles      bucketing by latent mode (:469-505, ovehicle.py:24-117)
    generator           compute_obstacle_constraints_GMM_Minkowski_idealprediction (shrinking,
                        robust) or compute_obstacle_constraints_GMM_affine (receding): the
                        half-spaces, vertices / L4 and the t = 0 state statistics

For a fixed shape (OVs, particles, horizon, latent count, kept modes per OV and, below ph, the
saved moments' cells) every stage is a kernel that needs nothing from the host between them:
the sampler, the bucketing, the moment / half-space kernels and the L4 kernel read the bucketed
cell counts on the device.  ``StepGraph`` captures, per kind,

    minkowski (T == ph)  copy-in -> sampler -> bucketing -> Minkowski cycle -> copy-out
    ideal     (T <  ph)  copy-in -> { ideal rollout + moments + half-spaces on the saved
                         moments (predict_ideal, :824-825) | sampler -> bucketing -> the scene's
                         moments (the t = 0 statistics, :864-875) } -> copy-out
    affine    (T == ph)  copy-in -> sampler -> bucketing -> moments -> GMM-affine -> copy-out

each as one linear graph that ends with the L4 outer approximation (vertices / A_union /
b_union and the heading statistics, :627-736):

    ... generator -> copy-out -> signal -> L4          (one stream; one hipGraphLaunch)

The host does not synchronise the stream: after the copy-out, ccmpc_signal_host writes the
step's generation number into a pinned word behind every output byte, and the host polls that
word.  So the records, moments and counts are read as soon as they land, while L4 (only
returned by the generator, never fed to the QP, :951-952) still runs; its device outputs are
read back on first access.  Two graphs alternate by the generation's parity, each with its own
L4 output buffers, so the previous step's L4 stays readable while the next step runs.

A step is: write the inputs into pinned memory, launch one graph, poll, read the outputs
through NumPy views of one snapshot.  The Philox seeds travel in the packed inputs (ccmpc_sample_unicycle_ex
and ccmpc_ideal_minkowski_cycle_ex read them on the device), so every replay draws afresh.

Outputs live in the graph's buffers until the next replay of the same graph; what the caller
keeps across steps (the saved moments) is copied out.
"""
import collections
import collections.abc
import os
import time

import numpy as np
import torch

from . import _lib, engine, risk

_ALIGN = 256
_STEP_PACKED = int(os.environ.get("CCMPC_STEP_PACKED", "1"))


class Pack:
    """Named, 256-byte aligned fields of one flat device buffer, mirrored in pinned host memory
    (one copy moves all of them)."""

    def __init__(self, fields, device, record_views=None):
        """record_views: {alias: (field, numpy record dtype)} -- snapshot-only views of a byte
        field as records (its last axis the record size), so a snapshot hands out the records
        without a per-call dtype view (~2.3 us each)."""
        self.spec, off = {}, 0
        for name, shape, dtype in fields:
            shape = tuple(int(s) for s in shape)
            n = int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()
            off = -(-off // _ALIGN) * _ALIGN
            self.spec[name] = (off, shape, dtype, n)
            off += max(n, 1)
        self.nbytes = -(-off // _ALIGN) * _ALIGN
        self.dev = torch.zeros(self.nbytes, dtype=torch.uint8, device=device)
        self.host = torch.zeros(self.nbytes, dtype=torch.uint8, pin_memory=True)
        raw = self.host.numpy()
        self._d, self._h = {}, {}
        for name, (off, shape, dtype, n) in self.spec.items():
            self._d[name] = self.dev[off:off + n].view(dtype).view(shape)
            npdt = torch.empty((), dtype=dtype).numpy().dtype
            self._h[name] = raw[off:off + n].view(npdt).reshape(shape)
        self._views = [(name, shape, self._h[name].dtype, off)
                       for name, (off, shape, dtype, n) in self.spec.items()]
        self._raw = raw
        # the whole buffer as one structured record: a snapshot is one copy and one array, its
        # fields views made on access (numpy's per-view constructor cost was most of it); a
        # record view is one more field over the same bytes
        views = [(name, shape, dt, off) for name, shape, dt, off in self._views]
        for alias, (field, rdt) in (record_views or {}).items():
            _, shape, dt, off = next(v for v in self._views if v[0] == field)
            rdt = np.dtype(rdt)
            if shape[-1] * dt.itemsize != rdt.itemsize:
                raise ValueError(f"{field}: last axis is not one {rdt.itemsize}-byte record")
            views.append((alias, shape[:-1], rdt, off))
        self._struct = np.dtype({"names": [v[0] for v in views],
                                 "formats": [(v[2], v[1]) for v in views],
                                 "offsets": [v[3] for v in views],
                                 "itemsize": self.nbytes})

    def d(self, name):
        """Device view of a field."""
        return self._d[name]

    def h(self, name):
        """Zero-copy NumPy view of the pinned host field."""
        return self._h[name]

    def snapshot(self, device=False):
        """One copy of the whole host buffer (device=True: of the device buffer, synchronously);
        returns a read-only mapping {field: view of the copy} (outputs that must outlive the
        next replay, for one memcpy instead of one per field)."""
        raw = self.dev.cpu().numpy() if device else self._raw.copy()
        return _Snapshot(np.ndarray((), self._struct, raw))


class _Snapshot(collections.abc.Mapping):
    """Pack.snapshot's result: field name -> array view of one copied buffer."""
    __slots__ = ("_a",)

    def __init__(self, a):
        self._a = a

    def __getitem__(self, name):
        if name not in self._a.dtype.fields:
            raise KeyError(name)
        return self._a[name]

    def __iter__(self):
        return iter(self._a.dtype.names)

    def __len__(self):
        return len(self._a.dtype.names)


class HipGraph:
    """An executable graph captured through ccmpc_graph_capture_* (the library's calls and the
    fork / join event pairs only), replayed on the current stream; destroyed with the object,
    after the device has drained (its last replay may still run)."""

    def __init__(self, device, fn, stream):
        """Capture fn() on `stream`."""
        import ctypes
        lib = _lib.load()
        self.device, self.exec = device, None
        with torch.cuda.stream(stream):
            s = engine._stream()
            _lib.check(lib.ccmpc_graph_capture_begin(s), "ccmpc_graph_capture_begin")
            ex = ctypes.c_void_p()
            try:
                fn()
            finally:
                rc = lib.ccmpc_graph_capture_end(s, ctypes.byref(ex))
            _lib.check(rc, "ccmpc_graph_capture_end")
        self.exec = ex.value
        self._launch = lib.ccmpc_graph_launch

    def replay(self, stream=None):
        """Launch on `stream` (a raw stream handle; default: torch's current stream)."""
        rc = self._launch(self.exec, engine._stream() if stream is None else stream)
        if rc != 0:
            _lib.check(rc, "ccmpc_graph_launch")

    def __del__(self):
        if self.exec:
            try:
                torch.cuda.synchronize(self.device)
                _lib.load().ccmpc_graph_destroy(self.exec)
            except Exception:       # interpreter shutdown: the process releases it
                pass
            self.exec = None


def poll_word(words, slot, gen, device, what):
    """Spin until the pinned signal word words[slot] (written by ccmpc_signal_host) reaches
    `gen`.  A word that does not arrive within 5 s (a faulted kernel never signals)
    synchronises the device, which raises the error, or else reports the missing signal."""
    if words[slot] >= gen:
        return
    deadline, n = None, 0
    while words[slot] < gen:
        n += 1
        if n & 0x3FF == 0:
            now = time.perf_counter()
            if deadline is None:
                deadline = now + 5.0
            elif now > deadline:
                torch.cuda.synchronize(device)
                if words[slot] < gen:
                    raise RuntimeError(f"{what} signal never came (word {slot} = "
                                       f"{int(words[slot])}, expected {gen})")


class StepGraph:
    """Sampler -> bucketing -> the step's generator kernels and, as a parallel branch, L4, for
    one shape.

    O OVs with N particles each over ph steps; L latent values; K kept modes per OV (the host
    decides them from p(z|x), as make_ovehicles does, so the shape is known before the step
    runs).  kind: "minkowski" (T == ph), "ideal" (T < ph, on the saved moments of prev_K cells
    over T_src steps, n_ideal rollout samples per cell) or "affine" (T == ph).

    Two sampler modes:
      per_particle=False  gmm (O, L, ph, 5) per-latent parameters, z and the noise drawn by
                          Philox on the device (the synthetic mode); gmm travels in the packed
                          host inputs.
      per_particle=True   the boundary Trajectron++ hands over on the GPU (prediction.py:81-86):
                          every sample's own GMM parameters gmm[o][t][5][n] (p_y_xz's
                          autoregressive decoder), the one-hot z's argmax (:103) and, with
                          eps_in, GMM2D.rsample's standard-normal draws -- all DEVICE tensors,
                          written into this graph's own device buffers (pp_gmm, pp_z, pp_eps)
                          by set_device_inputs, never through the host.

    source="predictions" takes the reference's own prediction boundary instead of the sampler
    tail: generate_vehicle_latents' predictions (O, N, ph, 2) float32 scene-relative and z
    (O, N) latent ids (prediction.py:93-105) -- host arrays written into the packed inputs
    (pred_device=False), or device tensors copied into the graph's own buffers -- moved into
    the sample-order store by ccmpc_load_predictions, then bucketed (ccmpc_bucket) as the
    sampler's output is: make_ovehicles (:469-505) with no sampler in the graph.

    ``generation`` counts launches: objects built over this graph's buffers (ScenePredictions)
    record the generation they belong to and refuse reads after a later replay."""

    def __init__(self, O, N, ph, L, K, device="cuda", dt=0.5, R=risk.R_COLLISION, tol=1e-8,
                 maxiter=1000, per_particle=False, eps_in=False, kind="minkowski", T=None,
                 prev_K=None, T_src=None, n_ideal=1_000_000, source="sampler",
                 pred_device=False):
        self.device = engine.require_device(device)
        self._dev_index = (self.device.index if self.device.index is not None
                           else torch.cuda.current_device())
        self.qp = None                       # attach_qp: the frame's QP inside the graph
        lib = _lib.load()
        if kind not in ("minkowski", "ideal", "affine"):
            raise ValueError(f"unknown step kind {kind!r}")
        self.kind = kind
        self.O, self.N, self.ph, self.L = int(O), int(N), int(ph), int(L)
        self.T = T = int(T if T is not None else ph)
        if (kind == "ideal") != (T < self.ph) or not 1 <= T <= self.ph:
            raise ValueError(f"kind {kind!r} with T = {T}, ph = {self.ph}")
        self.K = [int(k) for k in K]
        if len(self.K) != self.O or min(self.K) < 1:
            raise ValueError("K must give >= 1 kept mode for each OV")
        self.C = C = sum(self.K)
        self.P = P = max(T * (T - 1) // 2, 1)
        self.max_k = max(self.K)
        self.dt, self.R, self.tol, self.maxiter = float(dt), float(R), float(tol), int(maxiter)
        self.per_particle, self.eps_in = bool(per_particle), bool(eps_in)
        if self.eps_in and not self.per_particle:
            raise ValueError("eps_in is part of the per-particle (Trajectron++ boundary) mode")
        if source not in ("sampler", "predictions"):
            raise ValueError(f"unknown source {source!r}")
        self.source, self.pred_device = source, bool(pred_device)
        if source == "predictions" and self.per_particle:
            raise ValueError("the predictions source replaces the sampler tail: no per_particle")
        self.generation = 0
        f64, f32, i32, i64, u8 = torch.float64, torch.float32, torch.int32, torch.int64, torch.uint8
        ph_, L_ = self.ph, self.L
        gmm_field = ([] if self.per_particle or source == "predictions"
                     else [("gmm", (O, L_, ph_, 5), f32)])
        if source == "predictions" and not self.pred_device:
            gmm_field += [("pred", (O, N, ph_, 2), f32), ("zin", (O, N), i64)]
        O4 = -(-O // 4) * 4               # (16-byte copies)
        if source == "predictions":       # zeroed on the device by every copy-in
            gmm_field += [("zbad0", (O4,), i32)]
        if source == "predictions" and self.pred_device:
            # the addresses of this launch's predictions / z (ccmpc_bucket_predictions_indirect)
            gmm_field += [("pptr", (2,), i64)]
        fields = ([("gen", (2,), i64), ("seed", (1,), i64), ("init", (O, 4), f64),
                   ("cdf", (O, L_), f64)] + gmm_field +
                  [("keep", (O, L_), i32), ("nk", (O,), i32), ("base", (O,), i32),
                   ("minpos", (O, 2), f64), ("region", (O,), i64), ("origin", (C, 2), f64),
                   ("ref", (1, T, 2), f64), ("past", (C, 2), f64), ("bbox", (C, 2), f64)])
        fields += [("gamma", (C,), f64)] if kind == "affine" else [("risk", (C, 3), f64)]
        if kind == "ideal":
            self.prev_K = [int(k) for k in prev_K]
            self.T_src = int(T_src if T_src is not None else T + 1)
            if not T < self.T_src <= 40:
                raise ValueError(f"saved moments over T_src = {self.T_src} steps cannot roll "
                                 f"out T = {T}")
            self.n_ideal = int(n_ideal)
            Cp, Ts = sum(self.prev_K), self.T_src
            fields += [("iseed", (1,), i64), ("src", (C,), i32), ("pmean", (Cp, Ts, 2), f64),
                       ("pcov", (Cp, 2 * Ts, 2 * Ts), f64)]
        self.inp = Pack(fields, self.device)
        self.pp_gmm = self.pp_z = self.pp_eps = None
        if self.per_particle:       # device-side inputs (particle-minor, the sampler's layout)
            self.pp_gmm = torch.zeros((O, ph_, 5, N), dtype=f32, device=self.device)
            self.pp_z = torch.zeros((O, N), dtype=i32, device=self.device)
            if self.eps_in:
                self.pp_eps = torch.zeros((O, ph_, 2, N), dtype=f32, device=self.device)
        self.pr_pred = self.pr_z = None
        self._rows_idx = None                 # set_predictions' cached device row index
        self._held = None                     # the predictor's tensors the next launch reads
        if source == "predictions" and self.pred_device:
            self.pr_pred = torch.zeros((O, N, ph_, 2), dtype=f32, device=self.device)
            self.pr_z = torch.zeros((O, N), dtype=i64, device=self.device)
        out = [("cnt", (C,), i64), ("off", (C,), i64), ("pmf", (C,), f64),
               ("centre", (C, 2), f64), ("mean", (C, ph_, 2), f64),
               ("cov", (C, 2 * ph_, 2 * ph_), f64)]
        if kind == "affine":
            out += [("rec", (C, T, 128), u8)]
        else:
            out += [("rec", (C, P, 128), u8), ("pl", (C, T), f64)]
        if kind == "ideal":
            out += [("imean", (C, T, 2), f64), ("icov", (C, 2 * T, 2 * T), f64),
                    ("status", (C,), i32)]
        if source == "predictions":       # invalid latent ids per OV (make_ovehicles' index)
            out += [("zbad", (O4,), i32)]
        rdt = engine._lib.AFFINE_DTYPE if kind == "affine" else engine._lib.HALFSPACE_DTYPE
        self.out = Pack(out, self.device, record_views={"records": ("rec", rdt)})
        # one L4 output pack per generation parity (the two graphs alternate)
        self.out_l4s = [Pack([("A", (C, ph_, 4, 2), f64), ("b", (C, ph_, 4), f64),
                              ("yaw_mean", (C, ph_), f64), ("yaw0_var", (C,), f64)], self.device)
                        for _ in range(2)]
        # pinned signal word [0]: the record path's generation
        self.flags = torch.zeros(8, dtype=i64, pin_memory=True)
        self._flags = self.flags.numpy()
        # N <= 262144: sampler (or the predictor's output) + bucketing as one placement pass
        # (ccmpc_sample_bucket / ccmpc_bucket_predictions), whose cells need K (N + 4) slots per
        # OV; else the sample-order store + ccmpc_bucket
        fused_ws = lib.ccmpc_sample_bucket_workspace_bytes(O, N, ph_, self.max_k) \
            if self.max_k * (L_ + 1) <= 512 else 0
        self.fused = fused_ws > 0
        region, cur, n_bound = [], 0, 0
        for o in range(O):
            region.append(cur)
            cur = engine._round4(cur + (self.K[o] * (N + 4) if self.fused
                                        else N + 4 * self.K[o]))
            n_bound = engine._round4(n_bound + N + 4 * self.K[o])
        self.region = np.asarray(region, np.int64)
        st = engine.ParticleStore(ph_, [0] * C, dtype=f32, device=self.device,
                                  origin=np.zeros((C, 2)), capacity=cur)
        st.cell_off, st.cell_cnt, st.origin = self.out.d("off"), self.out.d("cnt"), \
            self.inp.d("origin")
        st.counts = st.offsets = None
        st.n_bound = n_bound
        self.store = st
        if self.fused:
            self.bucket_ws = torch.zeros(fused_ws, dtype=u8, device=self.device)
        else:
            self.z = torch.empty((O, N), dtype=i32, device=self.device)
            self.samples = engine.ParticleStore(ph_, [N] * O, dtype=f32, device=self.device,
                                                align=4, origin=np.zeros((O, 2)))
            self.bucket_ws = torch.zeros(
                max(lib.ccmpc_bucket_workspace_bytes(O, N, L_, self.max_k), 16), dtype=u8,
                device=self.device)
        self.ws = engine.Workspace(self.device)
        self.ws.get(lib.ccmpc_moments_workspace_bytes(ph_, C, st.n_bound))
        # fork / join events per parity graph, alive as long as the graphs are: an event
        # recorded into a capture and destroyed before the graph (what wait_stream's temporary
        # does) left a dangling reference that crashed the replay once the memory was reused
        self._ev = [{k: torch.cuda.Event() for k in ("fork", "join")}
                    for _ in range(2)]
        if kind == "ideal":         # its own: the rollout runs beside the scene's moments
            self.ideal_ws = engine.Workspace(self.device)
            self.ideal_ws.get(lib.ccmpc_ideal_moments_workspace_bytes(T, C, self.n_ideal))
            self.aux = torch.cuda.Stream(device=self.device)
            # the rollout as a branch beside the sampling, or (CCMPC_STEP_IDEAL_FORK=0) first on
            # the one stream
            self.ideal_fork = os.environ.get("CCMPC_STEP_IDEAL_FORK", "1") == "1"
        self.l4_ws = engine.Workspace(self.device)      # its own: layouts differ
        self.l4_ws.get(lib.ccmpc_l4_workspace_bytes(ph_, C, st.n_bound))
        self.side = torch.cuda.Stream(device=self.device)
        # the packed copies as copy kernels that read / write the pinned pack directly, or
        # (CCMPC_STEP_COPY_KERNEL=0) as memcpy nodes (a runtime blit of ~4.8 us each): the
        # kernels take ~8 us off a step (profiles/r02/v33_step_copy_kernel.txt)
        self.copy_kernel = os.environ.get("CCMPC_STEP_COPY_KERNEL", "1") == "1"
        # the multi-block copy kernel followed by ccmpc_signal_host, or (=1) both as one
        # single-workgroup launch: one CU's copy of the ~50 KB pack costs more than the launch
        # it saves (C2 step 100.4 vs 102.6 us, profiles/r04/ab_fused_signal.log); the QP's
        # sub-KB pack takes the fused form
        self.fused_signal = os.environ.get("CCMPC_STEP_FUSED_SIGNAL", "0") == "1"
        self.graphs = None                  # [parity 0, parity 1]
        # launches before this one run eagerly (the same calls, no capture): a shape used once
        # -- each shrinking horizon of an episode on a fresh agent -- never pays the capture
        # and instantiation (two graphs, ~2-3 ms), a shape that recurs is graphed from its
        # second launch on
        self.capture_at = int(os.environ.get("CCMPC_STEP_CAPTURE_AT", "2"))
        self._static_set = False
        self._l4_snap = {}                  # generation -> snapshot of its L4 outputs

    # ---------------------------------------------------------------------------------------
    def _packed_p0(self):
        """The input pack's copy in the placement's first launch (ccmpc_*_packed: the latent-id
        pass reads its inputs from the pinned host side meanwhile) instead of a copy kernel of
        its own -- for the fused placement of the predictor's output with the kernel copy, not
        beside the ideal rollout (whose fork waits on the copy).  Measured (profiles/r06/ab/
        packed_*): predictor output on the device, graph 64.8 -> 62.1 us at C2's shape with the
        same record path; the synthetic sampler's route, whose latent draws then wait on host
        reads of the CDF and seed, graph -1.4 us but record path +1.6 us, so not there.
        CCMPC_STEP_PACKED=0: never; =2: the sampler's route too (A/B)."""
        if not (_STEP_PACKED and self.fused and self.copy_kernel and self.kind != "ideal"):
            return False
        return self.source == "predictions" or _STEP_PACKED == 2

    def _sample_calls(self, s, pack=None):
        """The sampling + bucketing stage's C-ABI calls: [(fn, args)]; pack = (device side,
        host side, bytes) of the input pack to copy in the placement's first launch."""
        lib, p = _lib.load(), engine._p
        i, o, st = self.inp, self.out, self.store
        if pack is not None:
            return [(getattr(lib, fn.__name__ + "_packed"), tuple(pack) + args)
                    for fn, args in self._sample_calls(s)]
        O, N, T, L = self.O, self.N, self.ph, self.L
        ws = self.bucket_ws
        if self.source == "predictions":
            gmm = layout = z_in = eps = None
        elif self.per_particle:
            gmm, layout, z_in, eps = (p(self.pp_gmm), _lib.GMM_PER_PARTICLE, p(self.pp_z),
                                      p(self.pp_eps))
        else:
            gmm, layout, z_in, eps = p(i.d("gmm")), _lib.GMM_PER_LATENT, None, None
        if self.fused and self.source == "predictions":
            tail = (O, N, T, L, p(i.d("keep")), p(i.d("nk")), p(i.d("base")), self.max_k,
                    p(i.d("minpos")), p(i.d("region")), p(ws), ws.numel(), p(st.pos), st.ld,
                    p(o.d("off")), p(o.d("cnt")), p(o.d("pmf")), p(o.d("centre")),
                    p(o.d("zbad")), s)
            if self.pred_device:        # the tensors' addresses travel in the input pack
                return [(lib.ccmpc_bucket_predictions_indirect, (p(i.d("pptr")), 8, None) + tail)]
            return [(lib.ccmpc_bucket_predictions, (p(i.d("pred")), p(i.d("zin")), 8, None) +
                     tail)]
        if self.fused:
            return [(lib.ccmpc_sample_bucket, (
                p(i.d("init")), p(i.d("cdf")), L, gmm, layout, z_in, eps,
                O, N, T, self.dt, 0, p(i.d("seed")), 0, p(i.d("keep")), p(i.d("nk")),
                p(i.d("base")), self.max_k, p(i.d("minpos")), p(i.d("region")), p(ws),
                ws.numel(), None, p(st.pos), st.ld, p(o.d("off")), p(o.d("cnt")), p(o.d("pmf")),
                p(o.d("centre")), s))]
        sm = self.samples
        if self.source == "predictions":
            pred, z = ((self.pr_pred, self.pr_z) if self.pred_device
                       else (i.d("pred"), i.d("zin")))
            stride = sm.offsets[1] if O > 1 else N
            first = (lib.ccmpc_load_predictions, (p(pred), p(z), 8, None, O, N, T, L,
                                                  p(sm.pos), sm.ld, stride, p(self.z),
                                                  p(i.d("zbad0")), s))
        else:
            first = (lib.ccmpc_sample_unicycle_ex, (
                p(i.d("init")), p(i.d("cdf")), L, gmm, layout, z_in,
                eps, O, N, T, self.dt, 0, p(i.d("seed")), 0, p(self.z), p(sm.pos), sm.ld,
                s))
        calls = [first]
        if self.source == "predictions":   # the invalid-id counts into the output pack
            calls.append((lib.ccmpc_copy_kernel_async, (p(o.d("zbad")), p(i.d("zbad0")),
                                                        o.d("zbad").numel() * 4, s)))
        return calls + [
                (lib.ccmpc_bucket, (p(self.z), p(sm.pos), sm.ld, T, O, N, L, p(i.d("keep")),
                                    p(i.d("nk")), p(i.d("base")), self.max_k,
                                    p(i.d("minpos")), p(i.d("region")), p(ws), ws.numel(),
                                    p(st.pos), st.ld, p(o.d("off")), p(o.d("cnt")),
                                    p(o.d("pmf")), p(o.d("centre")), s))]

    def _enqueue(self, parity=0):
        """One step on the current stream (the graph of `parity`, or its eager form)."""
        lib, p, s = _lib.load(), engine._p, engine._stream()
        i, o, st = self.inp, self.out, self.store
        T, C, ph = self.T, self.C, self.ph
        ev = self._ev[parity]
        chk = engine._lib.check
        copy = lib.ccmpc_copy_kernel_async if self.copy_kernel else lib.ccmpc_copy_async
        packed = self._packed_p0()
        if not packed:
            chk(copy(p(i.dev), p(i.host), i.nbytes, s), "ccmpc_copy_async")
        main = torch.cuda.current_stream(self.device)
        if self.kind == "ideal":
            # the rollout needs only the saved moments: a branch beside the sampling
            if self.ideal_fork:
                ev["fork"].record(main)
                self.aux.wait_event(ev["fork"])
            with torch.cuda.stream(self.aux if self.ideal_fork else main):
                iws = self.ideal_ws.buf
                chk(lib.ccmpc_ideal_minkowski_cycle_ex(
                    p(i.d("pmean")), p(i.d("pcov")), self.T_src, p(i.d("src")), C, T,
                    self.n_ideal, None, 0, p(i.d("iseed")), None, p(iws), iws.numel(),
                    p(i.d("ref")), None, p(i.d("risk")), self.R, self.tol, self.maxiter,
                    p(o.d("imean")), p(o.d("icov")), p(o.d("status")), p(o.d("rec")),
                    p(o.d("pl")), engine._stream()), "ccmpc_ideal_minkowski_cycle_ex")
        for fn, args in self._sample_calls(s, (p(i.dev), p(i.host), i.nbytes) if packed
                                           else None):
            chk(fn(*args), fn.__name__)
        mws = self.ws.buf
        if self.kind == "minkowski":
            chk(lib.ccmpc_minkowski_cycle(
                p(st.pos), engine.F32, st.ld, ph, p(st.origin), p(o.d("off")), p(o.d("cnt")), C,
                st.n_bound, p(mws), mws.numel(), p(i.d("ref")), None, p(i.d("risk")), self.R,
                self.tol, self.maxiter, p(o.d("mean")), p(o.d("cov")), p(o.d("rec")),
                p(o.d("pl")), s), "ccmpc_minkowski_cycle")
        else:
            chk(lib.ccmpc_moments(p(st.pos), engine.F32, st.ld, ph, p(st.origin), p(o.d("off")),
                                  p(o.d("cnt")), C, st.n_bound, p(mws), mws.numel(),
                                  p(o.d("mean")), p(o.d("cov")), s), "ccmpc_moments")
            if self.kind == "affine":
                chk(lib.ccmpc_affine(p(o.d("mean")), p(o.d("cov")), T, C, p(i.d("ref")), None,
                                     p(i.d("gamma")), self.R, p(o.d("rec")), s), "ccmpc_affine")
            elif self.ideal_fork:
                ev["join"].record(self.aux)
                main.wait_event(ev["join"])
        if self.copy_kernel and self.fused_signal:   # one single-workgroup launch
            chk(lib.ccmpc_copy_signal_async(p(o.host), p(o.dev), o.nbytes, p(self.flags),
                                            p(i.d("gen")), s), "ccmpc_copy_signal_async")
        else:
            chk(copy(p(o.host), p(o.dev), o.nbytes, s), "ccmpc_copy_async")
            chk(lib.ccmpc_signal_host(p(self.flags), p(i.d("gen")), s), "ccmpc_signal_host")
        if self.qp is not None:              # the frame's QP on the records, before L4
            q = self.qp
            q["step"].enqueue(o.d("rec"), q["xbar"], q["gamma"], ltv=q["ltv"], Ts=q["Ts"],
                              lon=q["lon"])
        # L4 (which only reads the bucketed store) after the record path's signal, on the same
        # stream: the host's wait ends before it, and a linear graph launches in a fraction of
        # the host time a forked one takes (one branch for L4 cost ~25 us more per
        # hipGraphLaunch; with L4's nodes captured first, the cycle also started only after
        # L4's first pass, profiles/r04/probe_step_l4_first.log)
        self._enqueue_l4(parity)

    def attach_qp(self, qp_step, xbar, gamma, ltv, Ts=0.5, lon=3.7):
        """Put the planning frame's QP (an mpc.PlanningQPStep over this graph's records) into
        the step, right after the record path's signal and before L4: its inputs go in with
        qp_step.prepare() before each launch, its answer comes back with qp_step.wait().
        xbar / gamma: the LTV buffers (rebuilt by the graph when ltv).  Before the first
        launch only (the graph captures the calls)."""
        if self.generation or self.graphs is not None:
            raise RuntimeError("attach_qp before the graph's first launch")
        self.qp = dict(step=qp_step, xbar=xbar, gamma=gamma, ltv=bool(ltv), Ts=float(Ts),
                       lon=float(lon))

    def _enqueue_l4(self, parity):
        """The L4 branch on the current stream: L4 over the bucketed store into the parity's
        device pack (read back on access: two graph nodes, no copy-out or signal to launch)."""
        lib, p, s = _lib.load(), engine._p, engine._stream()
        i, o, q, st = self.inp, self.out, self.out_l4s[parity], self.store
        lws = self.l4_ws.buf
        chk = engine._lib.check
        if engine.l4_one_workgroup(self.C, st.n_bound):
            chk(lib.ccmpc_l4(p(st.pos), engine.F32, st.ld, self.ph, p(st.origin),
                             p(o.d("off")), p(o.d("cnt")), self.C, p(i.d("past")),
                             p(i.d("bbox")), p(q.d("A")), p(q.d("b")), p(q.d("yaw_mean")),
                             p(q.d("yaw0_var")), None, None, s), "ccmpc_l4")
            return
        chk(lib.ccmpc_l4_split(p(st.pos), engine.F32, st.ld, self.ph, p(st.origin),
                               p(o.d("off")), p(o.d("cnt")), self.C, st.n_bound,
                               p(i.d("past")), p(i.d("bbox")), p(lws), lws.numel(),
                               p(q.d("A")), p(q.d("b")), p(q.d("yaw_mean")),
                               p(q.d("yaw0_var")), None, None, s), "ccmpc_l4_split")

    def capture(self):
        """Record the two parity graphs (after one eager run that warms every kernel).

        torch hands out streams from a small pool, so this graph's capture / aux streams can be
        another graph's streams, which may still hold that graph's last L4 replay.  A fork into
        a stream with pending uncaptured work corrupted the captured graph (segfaults in the
        first replay once the pool had wrapped), so every stream the capture
        touches is drained first -- those streams only, not the device: another agent's work on
        other streams keeps running."""
        main = torch.cuda.current_stream(self.device)
        s = torch.cuda.Stream(device=self.device)
        used = [s, main] + [x for x in (getattr(self, "aux", None),) if x is not None]
        for x in used:
            x.synchronize()
        s.wait_stream(main)
        with torch.cuda.stream(s):
            self._enqueue(0)
        for x in used:
            x.synchronize()
        # the warm-up ran the whole step, including the signal of THIS launch's generation:
        # step the word back, so the poll can only be satisfied by the replay (else
        # wait() returned at once and the host read the output pack while the replay rewrote it)
        self._flags[0] = self.generation - 1
        if self.qp is not None:         # the attached QP signalled its own word the same way
            q = self.qp["step"]
            q._flags[0] = q.generation - 1
        self.graphs = [HipGraph(self.device, lambda par=par: self._enqueue(par), s)
                       for par in range(2)]
        return self

    # ---------------------------------------------------------------------------------------
    def set_inputs(self, seed, init_state, latent_pmf, gmm, minpos, ref_traj, cell_risk,
                   past_last, bbox, filter_pmf=0.1):
        """Write one step's host inputs into the pinned input pack (no device work; every field
        written in place, no temporaries).  The kept modes implied by latent_pmf must match the
        graph's K.  past_last / bbox: per cell (C, 2) or per OV (O, 2).  cell_risk: (C, 3)
        (chi2_r, chi2_p, Gamma) per cell; the affine kind reads its Gamma column."""
        i, O, L, C = self.inp, self.O, self.L, self.C
        if not self._static_set:       # shape-fixed fields and helpers: once
            i.h("nk")[:] = self.K
            i.h("base")[:] = np.concatenate([[0], np.cumsum(self.K)[:-1]])
            i.h("region")[:] = self.region
            self._K_arr = np.asarray(self.K)
            self._K_list = [int(k) for k in self.K]
            self._ov_of_cell = np.repeat(np.arange(O), self.K)
            self._pmf_key = self._bbox_key = None
            self._static_set = True
        pmf = np.asarray(latent_pmf, np.float64).reshape(O, L)
        # the fields that follow from the pmf are rewritten only when it changed (the pinned
        # pack keeps them between launches; small-array numpy calls are most of this method's
        # host time: add.accumulate is cumsum without its dispatch overhead, same sums)
        pk = (pmf.tobytes(), float(filter_pmf))
        if pk != self._pmf_key:
            self._pmf_key = None
            kept = pmf > filter_pmf
            keep = i.h("keep")           # kept: its rank among the kept latents; else -1
            np.add.accumulate(kept, axis=1, dtype=np.int32, out=keep)
            if keep[:, -1].tolist() != self._K_list:
                raise ValueError(f"kept modes per OV {keep[:, -1].tolist()}; this graph was "
                                 f"built for {self.K}")
            np.multiply(keep, kept, out=keep)
            keep -= 1
            np.add.accumulate(pmf, axis=1, out=i.h("cdf"))
            self._pmf_key = pk
        i.h("seed")[0] = _as_i64(seed)
        if init_state is not None:             # (the predictions source has no sampler)
            i.h("init").reshape(-1)[:] = np.asarray(init_state, np.float64).reshape(-1)
        if self.source == "predictions":
            if gmm is not None:
                raise ValueError("the predictions source takes set_predictions, not gmm")
        elif self.per_particle:
            if gmm is not None:
                raise ValueError("per-particle graph: pass the device parameters to "
                                 "set_device_inputs, not set_inputs")
        else:
            np.copyto(i.h("gmm").reshape(-1), np.asarray(gmm).reshape(-1), casting="same_kind")
        mp = np.asarray(minpos, np.float64)
        if mp.size == 2:
            i.h("minpos")[:] = mp.reshape(1, 2)
            i.h("origin")[:] = mp.reshape(1, 2)
        else:
            mp = mp.reshape(O, 2)
            i.h("minpos")[:] = mp
            np.take(mp, self._ov_of_cell, axis=0, out=i.h("origin"))
        i.h("ref").reshape(-1)[:] = np.asarray(ref_traj, np.float64)[:self.T].reshape(-1)
        cr = np.asarray(cell_risk, np.float64).reshape(C, 3)
        if self.kind == "affine":
            i.h("gamma")[:] = cr[:, 2]
        else:
            i.h("risk")[:] = cr
        for name, v in (("past", past_last), ("bbox", bbox)):
            v = np.asarray(v, np.float64)
            if name == "bbox":           # the OVs' boxes rarely change: skip an unchanged one
                bk = v.tobytes()
                if bk == self._bbox_key:
                    continue
                self._bbox_key = None
            if v.size == 2 * C:
                i.h(name).reshape(-1)[:] = v.reshape(-1)
            else:
                np.take(v.reshape(O, 2), self._ov_of_cell, axis=0, out=i.h(name))
            if name == "bbox":
                self._bbox_key = bk

    def set_ideal_inputs(self, prev_mean, prev_cov, src_cell, seed):
        """The shrinking step's saved moments (the previous frame's mean [Cp, T_src, 2] and cov
        [Cp, 2 T_src, 2 T_src], host arrays or device tensors), each current cell's source cell
        (the data_idx fallback, :2648-2656) and the rollout's Philox seed."""
        if self.kind != "ideal":
            raise ValueError("set_ideal_inputs belongs to the shrinking (ideal) step")
        i = self.inp
        for name, v in (("pmean", prev_mean), ("pcov", prev_cov)):
            v = v.cpu().numpy() if torch.is_tensor(v) else np.asarray(v, np.float64)
            if v.shape != i.h(name).shape:
                raise ValueError(f"{name}: shape {v.shape}, this graph holds {i.h(name).shape}")
            i.h(name)[...] = v
        src = src_cell.cpu().numpy() if torch.is_tensor(src_cell) else np.asarray(src_cell)
        i.h("src")[:] = src.reshape(-1)
        i.h("iseed")[0] = _as_i64(seed)

    def set_predictions(self, predictions, z, rows=None):
        """The predictions source's input for the next launch: generate_vehicle_latents'
        predictions (nodes, N, ph, 2) float32 scene-relative and z (nodes, N) latent ids
        (prediction.py:93-105), of which rows[o] is OV o's node (make_ovehicles skips the ego's,
        :475-477; default: rows 0 .. O-1).  Host arrays go into the pinned input pack (moved by
        the step's copy-in); device tensors are copied on the current stream into the graph's
        own buffers (a graph built with pred_device=True).  z is not validated on the host
        (that would synchronise): the kernels count the ids make_ovehicles' list index would
        refuse into the output pack's "zbad" (the planner raises IndexError on them)."""
        if self.source != "predictions":
            raise ValueError("set_predictions needs a graph built with source='predictions'")
        O, N, T = self.O, self.N, self.ph
        rows = list(range(O)) if rows is None else [int(r) for r in rows]
        if len(rows) != O:
            raise ValueError(f"{len(rows)} OV rows for a graph of {O} OVs")
        dev = torch.is_tensor(predictions)
        if dev != self.pred_device or torch.is_tensor(z) != dev:
            raise ValueError("predictions / z must both be device tensors on a pred_device "
                             "graph and host arrays otherwise")
        if tuple(predictions.shape[1:]) != (N, T, 2) or tuple(z.shape[1:]) != (N,):
            raise ValueError(f"predictions {tuple(predictions.shape)} / z {tuple(z.shape)}: "
                             f"expected (nodes, {N}, {T}, 2) / (nodes, {N})")
        nodes = int(predictions.shape[0])
        if int(z.shape[0]) != nodes or any(not 0 <= r < nodes for r in rows):
            # (on the device path an out-of-range row would reach index_select and abort the
            # process with a device-side assert)
            raise ValueError(f"OV rows {rows} out of range for {nodes} prediction nodes "
                             f"(z has {int(z.shape[0])})")
        if dev:
            if predictions.device != self.device or z.device != self.device:
                raise ValueError("predictions / z must be on the graph's device")
            run = rows == list(range(rows[0], rows[0] + O)) if O else True
            if (self.fused and run and predictions.dtype == torch.float32 and
                    z.dtype == torch.int64 and
                    predictions.is_contiguous() and z.is_contiguous()):
                # the OVs are one run of nodes (the ego's row first or last) of tensors in the
                # kernels' layout: the launch reads them in place -- their addresses go into
                # the input pack, nothing is copied (held until the next set_predictions; the
                # caller reads the outputs before that)
                r0 = rows[0] if O else 0
                pv, zv = predictions[r0:r0 + O], z[r0:r0 + O]
                self.inp.h("pptr")[:] = (pv.data_ptr(), zv.data_ptr())
                self._held = (predictions, z)
                return
            if run:
                # a view, one device-to-device copy each (converting), nothing uploaded
                self.pr_pred.copy_(predictions[rows[0]:rows[0] + O])
                self.pr_z.copy_(z[rows[0]:rows[0] + O])
            else:
                key = tuple(rows)
                if self._rows_idx is None or self._rows_idx[0] != key:
                    self._rows_idx = (key, torch.as_tensor(rows, device=self.device))
                idx = self._rows_idx[1]
                torch.index_select(predictions.to(torch.float32), 0, idx, out=self.pr_pred)
                torch.index_select(z.to(torch.int64), 0, idx, out=self.pr_z)
            self.inp.h("pptr")[:] = (self.pr_pred.data_ptr(), self.pr_z.data_ptr())
            self._held = None
            return
        hp, hz = self.inp.h("pred"), self.inp.h("zin")
        for o, r in enumerate(rows):             # straight into the pinned pack, no temporary
            np.copyto(hp[o], predictions[r], casting="same_kind")
            np.copyto(hz[o], z[r], casting="unsafe")

    def set_device_inputs(self, gmm, z, eps=None):
        """The per-particle mode's device inputs for the next launch, as Trajectron++ leaves
        them on the GPU (prediction.py:81-86): gmm (O, N, T, 5) -- or already the sampler's
        particle-minor (O, T, 5, N) -- z (O, N) latent ids (the one-hot z's argmax, :103) and,
        when the graph was built with eps_in, eps (O, N, T, 2) standard-normal draws (or (O, T,
        2, N)).  Each is one device-to-device copy on the current stream into the graph's own
        buffer, ordered before the replay; a tensor that already IS the buffer is not copied
        (an upstream that writes pp_gmm / pp_z / pp_eps directly costs nothing here).  z is not
        validated on the host (that would synchronise): the kernels clamp it into [0, L)."""
        if not self.per_particle:
            raise ValueError("set_device_inputs needs a graph built with per_particle=True")
        O, N, T = self.O, self.N, self.ph

        def put(dst, src, natural, minor, perm):
            if not torch.is_tensor(src) or src.device != self.device:
                raise ValueError("per-particle inputs must be tensors on the graph's device")
            if src.data_ptr() == dst.data_ptr() and tuple(src.shape) == tuple(dst.shape):
                return
            if tuple(src.shape) == minor:
                dst.copy_(src)
            elif tuple(src.shape) == natural:
                dst.copy_(src.permute(*perm))
            else:
                raise ValueError(f"shape {tuple(src.shape)}: expected {natural} or {minor}")

        put(self.pp_gmm, gmm, (O, N, T, 5), (O, T, 5, N), (0, 2, 3, 1))
        if not torch.is_tensor(z) or tuple(z.shape) != (O, N) or z.device != self.device:
            raise ValueError(f"z must be a ({O}, {N}) tensor on the graph's device")
        if z.data_ptr() != self.pp_z.data_ptr():
            self.pp_z.copy_(z)
        if self.eps_in:
            if eps is None:
                raise ValueError("this graph was built with eps_in: eps is required")
            put(self.pp_eps, eps, (O, N, T, 2), (O, T, 2, N), (0, 2, 3, 1))
        elif eps is not None:
            raise ValueError("this graph draws the noise itself (built without eps_in)")

    def launch(self, direct=False):
        """Enqueue one step on the current stream without waiting (the graph of this
        generation's parity).  direct: the same C-ABI calls enqueued eagerly instead."""
        self.generation += 1
        gen = self.generation
        self.inp.h("gen")[0] = gen      # read by this step's copy-in, then by its two signals
        if direct or (self.graphs is None and gen < self.capture_at):
            self._enqueue(gen & 1)
            return
        if self.graphs is None:
            self.capture()
        self.graphs[gen & 1].replay(engine._stream(self._dev_index))

    def _poll(self, slot, gen, what):
        poll_word(self._flags, slot, gen, self.device, f"planning step {gen}: the {what}")

    def wait(self):
        """Return when the launched step's output pack (records, moments, counts) is on the
        host; the L4 branch may still run."""
        self._poll(0, self.generation, "record path")

    def replay(self):
        """One step; returns when the output pack is on the host."""
        self.launch()
        self.wait()

    def l4_outputs(self, generation=None):
        """{A, b, yaw_mean, yaw0_var} host arrays of launch `generation` (default: the latest),
        waiting for its L4 branch; the latest two generations are readable (their parity packs
        are intact), older ones only if read before (snapshots), else they raise."""
        gen = self.generation if generation is None else generation
        snap = self._l4_snap.get(gen)
        if snap is not None:
            return snap
        if gen < 1 or gen < self.generation - 1 or gen > self.generation:
            raise RuntimeError(f"stale planning-step data: the L4 outputs of launch {gen} were "
                               f"overwritten (this graph is at launch {self.generation})")
        # the parity's pack is not rewritten before launch gen + 2: the stream's work up to now
        # includes gen's L4 branch (a step's graph joins its branches)
        torch.cuda.current_stream(self.device).synchronize()
        snap = self.out_l4s[gen & 1].snapshot(device=True)
        self._l4_snap = {k: v for k, v in self._l4_snap.items() if k >= self.generation - 1}
        self._l4_snap[gen] = snap
        return snap

    def records(self):
        return self.out.h("rec").reshape(-1).view(
            _lib.AFFINE_DTYPE if self.kind == "affine" else _lib.HALFSPACE_DTYPE).reshape(
            self.C, -1)


# Step graphs released by agents that were destroyed (MidlevelAgent.destroy), by (device,
# key): the reference harness builds a fresh agent per episode and destroys the last one
# (tests/Hz20/__init__.py:383-399), so the next agent takes the same shapes' graphs -- already
# captured -- instead of building them again.  A graph belongs to one agent at a time; its
# generation counter keeps counting, so objects the old agent handed out still refuse reads
# after the new owner's first replay.  Bounded: the least recently released go first.
_POOL = collections.OrderedDict()
POOL_MAX = 64


def pool_take(device, key):
    """A released graph of this shape, or None."""
    k = (str(device), key)
    lst = _POOL.get(k)
    if not lst:
        return None
    g = lst.pop()
    if not lst:
        del _POOL[k]
    return g


def pool_give(device, key, g):
    """Release a graph its agent no longer uses."""
    k = (str(device), key)
    _POOL.setdefault(k, []).append(g)
    _POOL.move_to_end(k)
    while sum(len(v) for v in _POOL.values()) > POOL_MAX:
        k0 = next(iter(_POOL))
        _POOL[k0].pop(0)
        if not _POOL[k0]:
            del _POOL[k0]


# The planners' LTV buffers (planner.MidlevelAgent._ltv_buffers), released with the agent's
# graphs: a graph holding the frame's QP reads one agent's buffers, so the next agent takes
# both (the graph key names the buffers it was captured with).
_LTV_POOL = collections.OrderedDict()


def ltv_take(device, ph):
    """A released agent's (xbar, Gamma) for this horizon, or None."""
    lst = _LTV_POOL.get((str(device), int(ph)))
    return lst.pop() if lst else None


def ltv_give(device, ph, bufs):
    lst = _LTV_POOL.setdefault((str(device), int(ph)), [])
    lst.append(bufs)
    del lst[:-4]


def _as_i64(seed):
    sd = int(seed) & (2**64 - 1)
    return sd - (1 << 64) if sd >= (1 << 63) else sd


class MinkowskiStepGraph(StepGraph):
    """The full-horizon (T == ph) Minkowski step: StepGraph(kind="minkowski")."""

    def __init__(self, O, N, T, L, K, device="cuda", dt=0.5, R=risk.R_COLLISION, tol=1e-8,
                 maxiter=1000, per_particle=False, eps_in=False):
        super().__init__(O, N, T, L, K, device=device, dt=dt, R=R, tol=tol, maxiter=maxiter,
                         per_particle=per_particle, eps_in=eps_in, kind="minkowski")
