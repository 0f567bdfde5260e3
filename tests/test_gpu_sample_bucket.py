"""GPU tests of the two-launch sampler + bucketing (ccmpc_sample_bucket): on every shape it
must give what the sampler followed by the three-kernel bucketing gives (ccmpc_sample_unicycle_ex
+ ccmpc_bucket: prediction.py:81-86 -> v8ideal/__init__.py:469-505, ovehicle.py:24-117) --
the same particles in every cell, in the same order, the same pmf and init_center bits -- and
those are pinned against the oracle's make_ovehicles in test_gpu_planner.py."""
import numpy as np
import pytest
import torch

from oracle import ccmpc_oracle as orc

pytestmark = pytest.mark.gpu


def _inputs(O, L, T, seed, kept=None):
    rng = np.random.default_rng(seed)
    init = np.stack([rng.uniform(20, 60, O), rng.uniform(20, 60, O),
                     rng.uniform(-np.pi, np.pi, O), rng.uniform(3, 10, O)], axis=1)
    pmf = np.stack([np.exp(rng.normal(0, 1.6, L)) for _ in range(O)])
    pmf /= pmf.sum(1, keepdims=True)
    if kept == "heavy":                      # one kept mode, ~85% of the draws rare
        pmf[:] = 0.85 / (L - 1)
        pmf[:, 3] = 0.15
        pmf /= pmf.sum(1, keepdims=True)
    elif kept is not None:                   # exactly `kept` modes above the 0.1 filter
        for o in range(O):
            p = np.full(L, 0.0)
            hot = rng.choice(L, kept, replace=False)
            p[hot] = 0.9 / kept if kept > 1 else 0.9
            rest = np.setdiff1d(np.arange(L), hot)
            if rest.size:
                p[rest] = 0.1 / rest.size * rng.uniform(0.2, 1.0, rest.size)
            pmf[o] = p / p.sum()
    for o in range(O):
        if not np.any(pmf[o] > 0.1):
            pmf[o, rng.integers(L)] += 0.3
            pmf[o] /= pmf[o].sum()
    gmm = np.zeros((O, L, T, 5), np.float32)
    gmm[..., 0] = rng.normal(0, 0.3, size=(O, L, 1))
    gmm[..., 1] = rng.normal(0, 1.5, size=(O, L, 1))
    gmm[..., 2:4] = rng.uniform(np.log(0.05), np.log(0.5), size=(O, L, T, 2))
    gmm[..., 4] = rng.uniform(-0.5, 0.5, size=(O, L, T))
    return init, pmf, gmm


def _two_step(e, init, pmf, gmm, N, T, minpos, gpu, **kw):
    z, st = e.sample_unicycle(init, pmf, gmm, N, T, seed=kw.get("seed", 0), device=gpu,
                              z=kw.get("z"), eps=kw.get("eps"),
                              per_particle=kw.get("per_particle", False))
    bucketed, K, pmf_out, centre = e.bucket(z, st, pmf, minpos)
    return z, bucketed, K, pmf_out, centre


def _assert_same(got, want):
    (sg, Kg, pg, cg), (sw, Kw, pw, cw) = got, want
    assert Kg == Kw
    cnt_g, cnt_w = sg.sync_counts(), sw.sync_counts()
    assert cnt_g == cnt_w
    np.testing.assert_array_equal(pg.cpu().numpy(), pw.cpu().numpy())
    np.testing.assert_array_equal(cg.cpu().numpy(), cw.cpu().numpy())
    for j in range(len(cnt_g)):
        np.testing.assert_array_equal(sg.cell_positions(j), sw.cell_positions(j))
    offs = sg.offsets
    assert all(o % 4 == 0 for o in offs)
    # cells do not overlap
    spans = sorted((o, o + n) for o, n in zip(offs, cnt_g))
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))


@pytest.mark.parametrize("O,L,T,N,seed,kept", [
    (4, 25, 8, 5000, 1, None),       # the drop-in step's shape
    (3, 25, 8, 4097, 2, None),       # a partial last block
    (2, 12, 8, 8192, 3, None),       # the largest fused cloud
    (2, 7, 1, 300, 4, None),         # T = 1
    (2, 9, 40, 700, 5, None),        # T = 40 (80 coordinate rows; the serial chain)
    (2, 9, 16, 900, 11, None),       # T = 16: the parallel step terms' largest horizon
    (2, 9, 17, 900, 12, None),       # T = 17: the first serial one
    (3, 12, 12, 2500, 13, None),     # T = 12 (C4's horizon)
    (3, 25, 8, 3000, 6, 1),          # one kept mode: every rare particle is its
    (2, 10, 8, 2000, 7, 8),          # eight kept modes, few rare particles
    (2, 25, 8, 8192, 9, "heavy"),    # ~7000 rare particles: 28 rare-slot blocks per OV
    (2, 5, 8, 1000, 10, 5),          # every latent kept: no rare particle at all
    (1, 3, 6, 1, 8, None),           # a single particle
    # N > 8192: two chain waves per place block, the rare stage as keys + copy
    (2, 25, 8, 20_000, 21, None),
    (1, 25, 8, 100_000, 22, None),   # C1's np = 100 000 (tests/Hz20/params.py:377)
    (2, 25, 8, 30_000, 23, "heavy"), # ~26 000 rare particles per OV: 26 key blocks
    (2, 9, 40, 12_000, 24, None),    # T = 40: the serial chain, 80 coordinate rows
    (2, 9, 12, 9_000, 25, None),     # T = 12
    (2, 10, 8, 16_384, 26, 8),       # eight kept modes
    (2, 5, 8, 10_000, 27, 5),        # every latent kept: no rare particle
    (2, 25, 8, 8_193, 28, 1),        # the first wide N, one kept mode
    (1, 25, 8, 262_144, 29, None),   # the largest
])
def test_fused_equals_sampler_then_bucketing(gpu, O, L, T, N, seed, kept):
    from ccmpc import engine as e
    init, pmf, gmm = _inputs(O, L, T, seed, kept)
    minpos = np.tile([150.0, -120.0], (O, 1))
    z2, *want = _two_step(e, init, pmf, gmm, N, T, minpos, gpu, seed=seed)
    zf, *got = e.sample_bucket(init, pmf, gmm, N, T, minpos, seed=seed, device=gpu, with_z=True)
    np.testing.assert_array_equal(zf.cpu().numpy(), z2.cpu().numpy())
    _assert_same(got, want)


@pytest.mark.parametrize("N", [5000, 30_000])
def test_fused_with_injected_draws_and_per_particle_parameters(gpu, N):
    from ccmpc import engine as e
    O, L, T = 3, 25, 8
    init, pmf, gmm = _inputs(O, L, T, 9)
    g = torch.Generator().manual_seed(4)
    z = torch.multinomial(torch.as_tensor(pmf), N, replacement=True, generator=g).to(torch.int32)
    eps = torch.randn((O, N, T, 2), generator=g, dtype=torch.float32)
    minpos = np.tile([10.0, 20.0], (O, 1))
    _, *want = _two_step(e, init, pmf, gmm, N, T, minpos, gpu, z=z.numpy(), eps=eps.numpy())
    got = e.sample_bucket(init, pmf, gmm, N, T, minpos, device=gpu, z=z.numpy(), eps=eps.numpy())
    _assert_same(got, want)
    pp = np.stack([gmm[o][z[o].numpy()] for o in range(O)])           # (O, N, T, 5)
    pp[..., 0] += np.random.default_rng(2).normal(0, 0.05, pp[..., 0].shape).astype(np.float32)
    _, *want = _two_step(e, init, pmf, pp, N, T, minpos, gpu, z=z.numpy(), eps=eps.numpy(),
                         per_particle=True)
    got = e.sample_bucket(init, pmf, pp, N, T, minpos, device=gpu, z=z.numpy(),
                          eps=eps.numpy(), per_particle=True)
    _assert_same(got, want)


def test_fused_meets_the_oracle_bucketing(gpu):
    """Membership / order / pmf / centre against the oracle's make_ovehicles on the sampler's
    own draws (the same comparison test_gpu_planner.py makes for the three-kernel form)."""
    from ccmpc import engine as e
    O, L, T, N = 3, 25, 8, 6000
    init, pmf, gmm = _inputs(O, L, T, 11)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2, minpos[1] + init[o, 1]]]) for o in range(O)]
    z, st = e.sample_unicycle(init, pmf, gmm, N, T, seed=3, device=gpu)
    pred = np.stack([st.cell_positions(o).astype(np.float32) for o in range(O)])
    want = orc.make_ovehicles(pred, z.cpu().numpy(), pmf, minpos, pasts,
                              [np.array([4.5, 2.5])] * O, T)
    store, K, pmf_out, centre = e.sample_bucket(init, pmf, gmm, N, T, np.tile(minpos, (O, 1)),
                                                seed=3, device=gpu)
    store.sync_counts()
    pmf_h, centre_h = pmf_out.cpu().numpy(), centre.cpu().numpy()
    c = 0
    for o in range(O):
        assert K[o] == want[o].n_states
        for k in range(K[o]):
            np.testing.assert_allclose(pmf_h[c], want[o].latent_pmf[k], rtol=1e-15)
            np.testing.assert_allclose(centre_h[c], want[o].init_center[k], rtol=1e-12)
            np.testing.assert_array_equal(store.cell_positions(c), want[o].pred_positions[k])
            c += 1


def test_fused_repeat_calls_need_no_workspace_init(gpu):
    """The first launch writes everything the second reads: back-to-back calls on one workspace,
    first filled with garbage, agree."""
    from ccmpc import engine as e
    O, L, T, N = 2, 25, 8, 3000
    init, pmf, gmm = _inputs(O, L, T, 12)
    minpos = np.zeros((O, 2))
    lib = e._lib.load()
    ws = torch.full((lib.ccmpc_sample_bucket_workspace_bytes(O, N, T, 16),), 0xA5,
                    dtype=torch.uint8, device=gpu)
    a = e.sample_bucket(init, pmf, gmm, N, T, minpos, seed=5, device=gpu, workspace=ws)
    for _ in range(3):
        ws.fill_(0x5A)
        b = e.sample_bucket(init, pmf, gmm, N, T, minpos, seed=5, device=gpu, workspace=ws)
    _assert_same(a, b)


def test_fused_refuses_large_clouds_and_bad_args(gpu):
    from ccmpc import engine as e
    init, pmf, gmm = _inputs(1, 5, 4, 13)
    with pytest.raises(ValueError):
        e.sample_bucket(init, pmf, gmm, 262_145, 4, np.zeros((1, 2)), device=gpu)
    lib = e._lib.load()
    assert lib.ccmpc_sample_bucket_workspace_bytes(1, 262_145, 4, 1) == 0
    assert lib.ccmpc_sample_bucket_workspace_bytes(1, 100, 41, 1) == 0
    rc = lib.ccmpc_sample_bucket(None, None, 5, None, 0, None, None, 1, 300_000, 4, 0.5, 0, None, 0,
                                 None, None, None, 1, None, None, None, 0, None, None, 0, None,
                                 None, None, None, None)
    assert rc == -1


@pytest.mark.parametrize("T,mode", [(8, "philox"), (40, "philox"), (8, "injected"),
                                    (8, "per_particle")])
def test_wide_sampler_blocks_give_the_narrow_blocks_bits(gpu, T, mode):
    """Above 8192 particles per OV the sampler runs four chain waves per block (256 particles)
    instead of one; particle i's draws and chain depend only on (i, OV, seed), so the first
    8192 particles of a 20 000-particle call equal an 8192-particle call bit for bit, in every
    input mode (Philox, injected z / eps, per-particle parameters)."""
    from ccmpc import engine as e
    O, L, Nw, Nn = 2, 25, 20_000, 8192
    init, pmf, gmm = _inputs(O, L, T, 12)
    kw = {}
    if mode != "philox":
        g = torch.Generator().manual_seed(5)
        z = torch.multinomial(torch.as_tensor(pmf), Nw, replacement=True,
                              generator=g).to(torch.int32)
        eps = torch.randn((O, Nw, T, 2), generator=g, dtype=torch.float32)
        kw = dict(z=z, eps=eps)
        if mode == "per_particle":
            pp = np.stack([gmm[o][z[o].numpy()] for o in range(O)])
            pp[..., 1] += np.random.default_rng(3).normal(0, 0.05, pp[..., 1].shape).astype(
                np.float32)
            kw["per_particle"] = True
    gw = pp if kw.get("per_particle") else gmm
    zw, sw = e.sample_unicycle(init, pmf, gw, Nw, T, seed=77, device=gpu, **kw)
    kn = {k: (v[:, :Nn].contiguous() if torch.is_tensor(v) else v) for k, v in kw.items()}
    gn = pp[:, :Nn] if kw.get("per_particle") else gmm
    zn, sn = e.sample_unicycle(init, pmf, gn, Nn, T, seed=77, device=gpu, **kn)
    np.testing.assert_array_equal(zw.cpu().numpy()[:, :Nn], zn.cpu().numpy())
    for o in range(O):
        np.testing.assert_array_equal(sw.cell_positions(o)[:Nn], sn.cell_positions(o))
