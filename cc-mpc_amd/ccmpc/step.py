"""One planning step of v8ideal's prediction + constraint path as ONE hipGraph replay.

Per planning frame the reference runs (v8ideal/__init__.py:2934-2976 -> :414-505, :781-964):

    do_prediction       Trajectron++ sample (prediction.py:81-86)
    make_ovehicles      bucketing by latent mode (:469-505, ovehicle.py:24-117)
    generator           compute_obstacle_constraints_GMM_Minkowski_idealprediction at Tsh == ph
                        (moments -> MVOE half-spaces, vertices / L4, t = 0 state statistics)

For a fixed shape (OVs, particles, horizon, latent count and kept modes per OV) the whole chain
is five kernels that need nothing from the host between them: the sampler, the bucketing, the
one-launch Minkowski cycle and the L4 kernel read the bucketed cell counts on the device.  So
``MinkowskiStepGraph`` captures

    packed H2D of the step's host inputs  ->  sampler  ->  bucketing  ->  { cycle | L4 }
    ->  packed D2H of every output the 9-tuple needs

(the cycle and the L4 kernel are parallel branches of the graph: both only read the bucketed
store)

into one graph.  A step is: write the inputs into pinned memory, replay, wait for the stream,
read the outputs through zero-copy NumPy views.  The Philox seed travels in the packed inputs
(ccmpc_sample_unicycle_ex's seed_dev), so every replay draws a fresh particle set.

Outputs live in the graph's buffers until the next replay of the same graph; what the caller
keeps across steps (the saved moments) is copied out.
"""
import os

import numpy as np
import torch

from . import _lib, engine, risk

_ALIGN = 256


class Pack:
    """Named, 256-byte aligned fields of one flat device buffer, mirrored in pinned host memory
    (one copy moves all of them)."""

    def __init__(self, fields, device):
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

    def d(self, name):
        """Device view of a field."""
        return self._d[name]

    def h(self, name):
        """Zero-copy NumPy view of the pinned host field."""
        return self._h[name]

    def snapshot(self):
        """One copy of the whole host buffer; returns {field: view of the copy} (outputs that
        must outlive the next replay, for one memcpy instead of one per field)."""
        raw = self.host.numpy().copy()
        nd = np.ndarray
        return {name: nd(shape, dt, raw, off) for name, shape, dt, off in self._views}


class MinkowskiStepGraph:
    """Sampler -> bucketing -> Minkowski cycle -> L4 for a fixed shape, as one hipGraph.

    O OVs with N particles each over T = ph steps; L latent values; K kept modes per OV (the
    host decides them from p(z|x), as make_ovehicles does, so the shape is known before the
    step runs).

    Two sampler modes:
      per_particle=False  gmm (O, L, T, 5) per-latent parameters, z and the noise drawn by
                          Philox on the device (the synthetic mode); gmm travels in the packed
                          host inputs.
      per_particle=True   the boundary Trajectron++ hands over on the GPU (prediction.py:81-86):
                          every sample's own GMM parameters gmm[o][t][5][n] (p_y_xz's
                          autoregressive decoder), the one-hot z's argmax (:103) and, with
                          eps_in, GMM2D.rsample's standard-normal draws -- all DEVICE tensors,
                          written into this graph's own device buffers (pp_gmm, pp_z, pp_eps)
                          by set_device_inputs, never through the host.

    ``generation`` counts launches: objects built over this graph's buffers (ScenePredictions)
    record the generation they belong to and refuse reads after a later replay."""

    def __init__(self, O, N, T, L, K, device="cuda", dt=0.5, R=risk.R_COLLISION, tol=1e-8,
                 maxiter=1000, per_particle=False, eps_in=False):
        self.device = engine.require_device(device)
        lib = _lib.load()
        self.O, self.N, self.T, self.L = int(O), int(N), int(T), int(L)
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
        self.generation = 0
        f64, f32, i32, i64, u8 = torch.float64, torch.float32, torch.int32, torch.int64, torch.uint8
        gmm_field = [] if self.per_particle else [("gmm", (O, L, T, 5), f32)]
        self.inp = Pack([("seed", (1,), i64), ("init", (O, 4), f64), ("cdf", (O, L), f64)]
                        + gmm_field +
                        [("keep", (O, L), i32), ("nk", (O,), i32),
                         ("base", (O,), i32), ("minpos", (O, 2), f64), ("region", (O,), i64),
                         ("origin", (C, 2), f64), ("ref", (1, T, 2), f64), ("risk", (C, 3), f64),
                         ("past", (C, 2), f64), ("bbox", (C, 2), f64)], self.device)
        self.pp_gmm = self.pp_z = self.pp_eps = None
        if self.per_particle:       # device-side inputs (particle-minor, the sampler's layout)
            self.pp_gmm = torch.zeros((O, T, 5, N), dtype=f32, device=self.device)
            self.pp_z = torch.zeros((O, N), dtype=i32, device=self.device)
            if self.eps_in:
                self.pp_eps = torch.zeros((O, T, 2, N), dtype=f32, device=self.device)
        self.out = Pack([("rec", (C, P, 128), u8), ("pl", (C, T), f64), ("mean", (C, T, 2), f64),
                         ("cov", (C, 2 * T, 2 * T), f64), ("A", (C, T, 4, 2), f64),
                         ("b", (C, T, 4), f64), ("yaw_mean", (C, T), f64),
                         ("yaw0_var", (C,), f64), ("cnt", (C,), i64), ("off", (C,), i64),
                         ("pmf", (C,), f64), ("centre", (C, 2), f64)], self.device)
        # small clouds: sampler + bucketing in three short launches (ccmpc_sample_bucket), whose cells need
        # K (N + 4) slots per OV; else the sampler's sample-order store + ccmpc_bucket
        fused_ws = lib.ccmpc_sample_bucket_workspace_bytes(O, N, T, self.max_k) \
            if self.max_k * (L + 1) <= 512 else 0
        self.fused = fused_ws > 0
        region, cur, n_bound = [], 0, 0
        for o in range(O):
            region.append(cur)
            cur = engine._round4(cur + (self.K[o] * (N + 4) if self.fused
                                        else N + 4 * self.K[o]))
            n_bound = engine._round4(n_bound + N + 4 * self.K[o])
        self.region = np.asarray(region, np.int64)
        st = engine.ParticleStore(T, [0] * C, dtype=f32, device=self.device,
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
            self.samples = engine.ParticleStore(T, [N] * O, dtype=f32, device=self.device, align=4,
                                                origin=np.zeros((O, 2)))
            self.bucket_ws = torch.zeros(
                max(lib.ccmpc_bucket_workspace_bytes(O, N, L, self.max_k), 16), dtype=u8,
                device=self.device)
        self.ws = engine.Workspace(self.device)
        self.ws.get(lib.ccmpc_moments_workspace_bytes(T, C, st.n_bound))
        self.l4_ws = engine.Workspace(self.device)      # its own: layouts differ
        self.l4_ws.get(lib.ccmpc_l4_workspace_bytes(T, C, st.n_bound))
        self.side = torch.cuda.Stream(device=self.device)
        # the cycle and the L4 kernel as parallel graph branches, or (CCMPC_STEP_LINEAR=1) one
        # after the other on one stream
        self.branch = os.environ.get("CCMPC_STEP_LINEAR", "0") != "1"
        self.cycle_first = os.environ.get("CCMPC_STEP_CYCLE_FIRST", "0") == "1"
        # the packed copies as copy kernels that read / write the pinned pack directly, or
        # (CCMPC_STEP_COPY_KERNEL=0) as memcpy nodes (a runtime blit of ~4.8 us each): the
        # kernels take ~8 us off a step (profiles/r02/v33_step_copy_kernel.txt)
        self.copy_kernel = os.environ.get("CCMPC_STEP_COPY_KERNEL", "1") == "1"
        self.graph = None
        self._static_set = False

    # ---------------------------------------------------------------------------------------
    def _sample_calls(self, s):
        """The sampling + bucketing stage's C-ABI calls: [(fn, args)]."""
        lib, p = _lib.load(), engine._p
        i, o, st = self.inp, self.out, self.store
        O, N, T, L = self.O, self.N, self.T, self.L
        ws = self.bucket_ws
        if self.per_particle:
            gmm, layout, z_in, eps = (p(self.pp_gmm), _lib.GMM_PER_PARTICLE, p(self.pp_z),
                                      p(self.pp_eps))
        else:
            gmm, layout, z_in, eps = p(i.d("gmm")), _lib.GMM_PER_LATENT, None, None
        if self.fused:
            return [(lib.ccmpc_sample_bucket, (
                p(i.d("init")), p(i.d("cdf")), L, gmm, layout, z_in, eps,
                O, N, T, self.dt, 0, p(i.d("seed")), 0, p(i.d("keep")), p(i.d("nk")),
                p(i.d("base")), self.max_k, p(i.d("minpos")), p(i.d("region")), p(ws),
                ws.numel(), None, p(st.pos), st.ld, p(o.d("off")), p(o.d("cnt")), p(o.d("pmf")),
                p(o.d("centre")), s))]
        sm = self.samples
        return [(lib.ccmpc_sample_unicycle_ex, (
                    p(i.d("init")), p(i.d("cdf")), L, gmm, layout, z_in,
                    eps, O, N, T, self.dt, 0, p(i.d("seed")), 0, p(self.z), p(sm.pos), sm.ld,
                    s)),
                (lib.ccmpc_bucket, (p(self.z), p(sm.pos), sm.ld, T, O, N, L, p(i.d("keep")),
                                    p(i.d("nk")), p(i.d("base")), self.max_k,
                                    p(i.d("minpos")), p(i.d("region")), p(ws), ws.numel(),
                                    p(st.pos), st.ld, p(o.d("off")), p(o.d("cnt")),
                                    p(o.d("pmf")), p(o.d("centre")), s))]

    def _enqueue(self):
        lib, p, s = _lib.load(), engine._p, engine._stream()
        i, o, st = self.inp, self.out, self.store
        T, C = self.T, self.C
        chk = engine._lib.check
        copy = lib.ccmpc_copy_kernel_async if self.copy_kernel else lib.ccmpc_copy_async
        chk(copy(p(i.dev), p(i.host), i.nbytes, s), "ccmpc_copy_async")
        for fn, args in self._sample_calls(s):
            chk(fn(*args), fn.__name__)
        # the cycle and the L4 kernel only read the bucketed store: two graph branches (the
        # fork is taken after the sampling; which branch is captured first is a knob)
        main = torch.cuda.current_stream(self.device)
        side = self.side if self.branch else main
        side.wait_stream(main)

        def l4():
            with torch.cuda.stream(side):
                lws = self.l4_ws.buf
                chk(lib.ccmpc_l4_split(p(st.pos), engine.F32, st.ld, T, p(st.origin),
                                       p(o.d("off")), p(o.d("cnt")), C, st.n_bound,
                                       p(i.d("past")), p(i.d("bbox")), p(lws), lws.numel(),
                                       p(o.d("A")), p(o.d("b")), p(o.d("yaw_mean")),
                                       p(o.d("yaw0_var")), None, None, engine._stream()),
                    "ccmpc_l4_split")

        def cycle():
            mws = self.ws.buf
            chk(lib.ccmpc_minkowski_cycle(
                p(st.pos), engine.F32, st.ld, T, p(st.origin), p(o.d("off")), p(o.d("cnt")), C,
                st.n_bound, p(mws), mws.numel(), p(i.d("ref")), None, p(i.d("risk")), self.R,
                self.tol, self.maxiter, p(o.d("mean")), p(o.d("cov")), p(o.d("rec")),
                p(o.d("pl")), s), "ccmpc_minkowski_cycle")

        for stage in ((cycle, l4) if self.cycle_first else (l4, cycle)):
            stage()
        main.wait_stream(side)
        chk(copy(p(o.host), p(o.dev), o.nbytes, s), "ccmpc_copy_async")

    def capture(self):
        """Record the step into a hipGraph (after one eager run that warms every kernel)."""
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._enqueue()
        s.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=s):
            self._enqueue()
        torch.cuda.synchronize(self.device)
        return self

    # ---------------------------------------------------------------------------------------
    def set_inputs(self, seed, init_state, latent_pmf, gmm, minpos, ref_traj, cell_risk,
                   past_last, bbox, filter_pmf=0.1):
        """Write one step's host inputs into the pinned input pack (no device work; every field
        written in place, no temporaries).  The kept modes implied by latent_pmf must match the
        graph's K.  past_last / bbox: per cell (C, 2) or per OV (O, 2)."""
        i, O, L, C = self.inp, self.O, self.L, self.C
        if not self._static_set:       # shape-fixed fields and helpers: once
            i.h("nk")[:] = self.K
            i.h("base")[:] = np.concatenate([[0], np.cumsum(self.K)[:-1]])
            i.h("region")[:] = self.region
            self._K_arr = np.asarray(self.K)
            self._ov_of_cell = np.repeat(np.arange(O), self.K)
            self._static_set = True
        pmf = np.asarray(latent_pmf, np.float64).reshape(O, L)
        kept = pmf > filter_pmf
        kc = np.cumsum(kept, axis=1)
        if not (kc[:, -1] == self._K_arr).all():
            raise ValueError(f"kept modes per OV {kc[:, -1].tolist()}; this graph was built "
                             f"for {self.K}")
        keep = i.h("keep")               # kept: its rank among the kept latents; else -1
        np.multiply(kc, kept, out=keep, casting="unsafe")
        keep -= 1
        sd = int(seed) & (2**64 - 1)
        i.h("seed")[0] = sd - (1 << 64) if sd >= (1 << 63) else sd
        i.h("init").reshape(-1)[:] = np.asarray(init_state, np.float64).reshape(-1)
        np.cumsum(pmf, axis=1, out=i.h("cdf"))
        if self.per_particle:
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
        i.h("risk").reshape(-1)[:] = np.asarray(cell_risk, np.float64).reshape(3 * C)
        for name, v in (("past", past_last), ("bbox", bbox)):
            v = np.asarray(v, np.float64)
            if v.size == 2 * C:
                i.h(name).reshape(-1)[:] = v.reshape(-1)
            else:
                np.take(v.reshape(O, 2), self._ov_of_cell, axis=0, out=i.h(name))

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
        O, N, T = self.O, self.N, self.T

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

    def bind(self):
        """Pre-convert every argument of the step's C-ABI calls for the current stream (the
        direct-launch alternative to the graph: one foreign call per stage, the cycle and L4
        back to back on one stream)."""
        lib, p, s = _lib.load(), engine._p, engine._stream()
        i, o, st = self.inp, self.out, self.store
        T, C = self.T, self.C
        mws = self.ws.buf
        self._calls = [(lib.ccmpc_copy_async, (p(i.dev), p(i.host), i.nbytes, s))] + \
            self._sample_calls(s) + [
            (lib.ccmpc_minkowski_cycle, (
                p(st.pos), engine.F32, st.ld, T, p(st.origin), p(o.d("off")), p(o.d("cnt")), C,
                st.n_bound, p(mws), mws.numel(), p(i.d("ref")), None, p(i.d("risk")), self.R,
                self.tol, self.maxiter, p(o.d("mean")), p(o.d("cov")), p(o.d("rec")),
                p(o.d("pl")), s)),
            (lib.ccmpc_l4_split, (p(st.pos), engine.F32, st.ld, T, p(st.origin), p(o.d("off")),
                                  p(o.d("cnt")), C, st.n_bound, p(i.d("past")), p(i.d("bbox")),
                                  p(self.l4_ws.buf), self.l4_ws.buf.numel(), p(o.d("A")),
                                  p(o.d("b")), p(o.d("yaw_mean")), p(o.d("yaw0_var")), None,
                                  None, s)),
            (lib.ccmpc_copy_async, (p(o.host), p(o.dev), o.nbytes, s)),
        ]
        return self

    def launch(self, direct=False):
        """Enqueue one step (inputs up, the kernels, outputs down) without waiting: one graph
        replay, or (direct) the bound C-ABI calls."""
        self.generation += 1
        if direct:
            if getattr(self, "_calls", None) is None:
                self.bind()
            for fn, args in self._calls:
                rc = fn(*args)
                if rc != 0:
                    _lib.check(rc, fn.__name__)
            return
        if self.graph is None:
            self.capture()
        self.graph.replay()

    def wait(self):
        """Return when the launched step's output pack is on the host."""
        torch.cuda.current_stream(self.device).synchronize()

    def replay(self):
        """One step; returns when the output pack is on the host."""
        self.launch()
        self.wait()

    def records(self):
        return self.out.h("rec").reshape(-1).view(_lib.HALFSPACE_DTYPE).reshape(self.C, self.P)
