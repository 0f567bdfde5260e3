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


def test_load_predictions_clamps_and_refuses(gpu):
    from ccmpc import _lib, engine
    pred = np.zeros((2, 64, 8, 2), np.float32)
    z = np.array([[-3, 0, 7, 100] * 16, [1] * 64], np.int64)
    zo, _ = engine.load_predictions(pred, z, 8, device=gpu)
    assert zo.cpu().numpy()[0, :4].tolist() == [0, 0, 7, 7]
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
