"""ccmpc_load_predictions: the reference's prediction boundary (generate_vehicle_latents'
predictions (nodes, N, T, 2) float32 + z (nodes, N), prediction.py:93-105) into the sample-order
store ccmpc_bucket reads.  Integer / byte work: bit-exact against numpy, at every T the ABI takes,
ragged N (not a multiple of the 128-particle chunk), node rows gathered (the ego's skipped), both
z widths; then the GPU bucketing on it equals the oracle's make_ovehicles (:469-505)."""
import numpy as np
import pytest
import torch

from oracle import ccmpc_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,N,zdt", [(1, 1, np.int64), (8, 5000, np.int64), (8, 129, np.int32),
                                     (12, 20000, np.int64), (40, 333, np.int32)])
def test_load_predictions_bit_exact(gpu, T, N, zdt):
    from ccmpc import engine
    rng = np.random.default_rng(T * 1000 + N)
    nodes, L = 5, 25
    pred = rng.normal(0, 30, (nodes, N, T, 2)).astype(np.float32)
    z = rng.integers(0, L, (nodes, N)).astype(zdt)
    rows = [3, 0, 4]                               # node 1 and 2 skipped (e.g. the ego)
    for src in ("host", "device"):
        p_in, z_in = ((pred, z) if src == "host" else
                      (torch.as_tensor(pred, device=gpu), torch.as_tensor(z, device=gpu)))
        zo, st = engine.load_predictions(p_in, z_in, L, rows=rows, device=gpu)
        torch.cuda.synchronize()
        pos, zh = st.pos.cpu().numpy(), zo.cpu().numpy()
        for o, r in enumerate(rows):
            off = st.offsets[o]
            got = pos[:, off:off + N].reshape(T, 2, N).transpose(2, 0, 1)
            assert got.tobytes() == pred[r].tobytes()
            assert np.array_equal(zh[o], z[r].astype(np.int32))


def test_load_predictions_refuses_bad_latent_ids(gpu):
    """make_ovehicles indexes a list of L entries by z (v8ideal/__init__.py:488-491): an id in
    [-L, 0) wraps as a Python index does, any other id outside [0, L) raises IndexError there
    -- and here (counted on the device, not clamped into another mode's cloud)."""
    from ccmpc import _lib, engine
    pred = np.zeros((2, 64, 8, 2), np.float32)
    z = np.array([[-3, 0, 7, -8] * 16, [1] * 64], np.int64)
    zo, _ = engine.load_predictions(pred, z, 8, device=gpu)
    assert zo.cpu().numpy()[0, :4].tolist() == [5, 0, 7, 0]
    for bad in (8, -9, 100, -(2 ** 40)):
        zb = z.copy()
        zb[1, 17] = bad
        with pytest.raises(IndexError, match="OV 1"):
            engine.load_predictions(pred, zb, 8, device=gpu)
        with pytest.raises(IndexError, match="OV 1"):
            engine.load_predictions(torch.as_tensor(pred, device=gpu),
                                    torch.as_tensor(zb, device=gpu), 8, device=gpu)
    with pytest.raises(ValueError):
        engine.load_predictions(pred.astype(np.float64), z, 8, device=gpu)
    with pytest.raises(ValueError):
        engine.load_predictions(pred, z[:, :10], 8, device=gpu)
    with pytest.raises(_lib.CcmpcError):
        engine.load_predictions(np.zeros((1, 4, 41, 2), np.float32), np.zeros((1, 4), np.int64), 8,
                                device=gpu)


def test_bucketing_the_loaded_predictions_matches_oracle_make_ovehicles(gpu):
    from ccmpc import engine
    rng = np.random.default_rng(11)
    O, N, T, L = 3, 3000, 8, 6
    pmf = rng.dirichlet(np.ones(L), O)
    pmf[:, 0] += 0.3
    pmf /= pmf.sum(1, keepdims=True)
    z = np.stack([rng.choice(L, N, p=pmf[o]) for o in range(O)]).astype(np.int64)
    centres = rng.normal(0, 20, (O, L, 2))
    pred = (centres[np.arange(O)[:, None], z][:, :, None, :] * np.linspace(0.1, 1, T)[:, None]
            + rng.normal(0, 1, (O, N, T, 2))).astype(np.float32)
    minpos = np.array([150.0, -120.0])
    zo, st = engine.load_predictions(pred, z, L, device=gpu)
    store, K, cpmf, centre = engine.bucket(zo, st, pmf, np.tile(minpos, (O, 1)))
    store.sync_counts()
    pasts = [np.array([[minpos[0], minpos[1]]])] * O
    want = orc.make_ovehicles(pred, z, pmf, minpos, pasts, [np.array([4.5, 2.5])] * O, T)
    c = 0
    for o in range(O):
        assert K[o] == want[o].n_states
        np.testing.assert_array_equal(cpmf.cpu().numpy()[c:c + K[o]], want[o].latent_pmf)
        for k in range(K[o]):
            np.testing.assert_array_equal(store.cell_positions(c), want[o].pred_positions[k])
            c += 1


def _pred_scene(O, N, T, L, seed, heavy=False):
    rng = np.random.default_rng(seed)
    pmf = rng.dirichlet(np.ones(L), O)
    pmf[:, 0] += 0.05 if heavy else 0.3
    pmf /= pmf.sum(1, keepdims=True)
    for o in range(O):
        if not np.any(pmf[o] > 0.1):
            pmf[o, 1] += 0.3
            pmf[o] /= pmf[o].sum()
    z = np.stack([rng.choice(L, N, p=pmf[o]) for o in range(O)]).astype(np.int64)
    centres = rng.normal(0, 20, (O, L, 2))
    pred = (centres[np.arange(O)[:, None], z][:, :, None, :] * np.linspace(0.1, 1, T)[:, None]
            + rng.normal(0, 1, (O, N, T, 2))).astype(np.float32)
    return pred, z, pmf


@pytest.mark.parametrize("O,N,T,L", [
    (3, 3000, 8, 6), (4, 5000, 8, 25), (2, 129, 12, 9), (1, 1, 8, 4), (2, 700, 40, 9),
    (1, 100_000, 8, 25), (2, 20_000, 12, 25), (1, 30_000, 40, 9), (3, 8_193, 8, 25),
    (1, 262_144, 8, 25)])
def test_bucket_predictions_equals_load_then_bucket(gpu, O, N, T, L):
    """ccmpc_bucket_predictions (one placement pass: the predictor's coordinates written
    straight into the cells, the rare ones through a rare list) holds in every cell exactly the
    particles of ccmpc_load_predictions + ccmpc_bucket, in the same order, with the same pmf and
    centre bits; only the cell offsets differ.  Rows gathered with the ego's node skipped, both
    rare-stage forms (one pass <= 8192 particles, keys + copy above), ragged N."""
    from ccmpc import engine
    pred, z, pmf = _pred_scene(O + 1, N, T, L, N + T, heavy=N == 30_000)
    rows = list(range(1, O + 1))
    minpos = np.tile([150.0, -120.0], (O, 1))
    zo, st = engine.load_predictions(pred, z, L, rows=rows, device=gpu)
    want = engine.bucket(zo, st, pmf[1:], minpos)
    for src in ("host", "device"):
        p_in, z_in = ((pred, z) if src == "host" else
                      (torch.as_tensor(pred, device=gpu), torch.as_tensor(z, device=gpu)))
        got = engine.bucket_predictions(p_in, z_in, pmf[1:], minpos, rows=rows, device=gpu)
        (sg, Kg, pg, cg), (sw, Kw, pw, cw) = got, want
        assert Kg == Kw
        assert sg.sync_counts() == sw.sync_counts()
        assert pg.cpu().numpy().tobytes() == pw.cpu().numpy().tobytes()
        assert cg.cpu().numpy().tobytes() == cw.cpu().numpy().tobytes()
        for j in range(sum(Kg)):
            assert sg.cell_positions(j).tobytes() == sw.cell_positions(j).tobytes(), (src, j)


def test_bucket_predictions_matches_oracle_and_refuses_bad_ids(gpu):
    from ccmpc import engine
    O, N, T, L = 3, 12_000, 8, 6
    pred, z, pmf = _pred_scene(O, N, T, L, 5)
    minpos = np.array([150.0, -120.0])
    store, K, cpmf, _ = engine.bucket_predictions(pred, z, pmf, minpos, device=gpu)
    store.sync_counts()
    pasts = [np.array([[minpos[0], minpos[1]]])] * O
    want = orc.make_ovehicles(pred, z, pmf, minpos, pasts, [np.array([4.5, 2.5])] * O, T)
    c = 0
    for o in range(O):
        assert K[o] == want[o].n_states
        np.testing.assert_array_equal(cpmf.cpu().numpy()[c:c + K[o]], want[o].latent_pmf)
        for k in range(K[o]):
            np.testing.assert_array_equal(store.cell_positions(c), want[o].pred_positions[k])
            c += 1
    zw = z.copy()
    zw[1, :40] -= L                    # [-L, 0): a Python index wraps -- the same cells
    got = engine.bucket_predictions(pred, zw, pmf, minpos, device=gpu)[0]
    got.sync_counts()
    for j in range(sum(K)):
        assert got.cell_positions(j).tobytes() == store.cell_positions(j).tobytes()
    for n in (N - 1, 5):
        zb = z.copy()
        zb[2, n] = L
        with pytest.raises(IndexError, match="OV 2"):
            engine.bucket_predictions(pred, zb, pmf, minpos, device=gpu)
