"""ccmpc.prediction.generate_vehicle_latents (the restated prediction.py:19-105 glue) against a
minimal stand-in of the Trajectron++ objects it drives (the submodule is absent here, so the
glue's calls are checked, not Trajectron++ itself -- parity unpinned upstream): the numpy
route returns the reference's 5-tuple layouts, and the keep_on_device opt-in returns the same
values as tensors on the model's device."""
import sys
import types

import numpy as np
import pytest
import torch

from ccmpc import prediction


class _Node:                        # hashable, as Trajectron++'s Node is
    def __init__(self, id):
        self.id = id


class _Latent:
    def __init__(self, L, seed):
        self.L, self.g = L, torch.Generator().manual_seed(seed)
        self.p_dist = None

    def get_p_dist_probs(self):
        return self.p_dist

    def sample_p(self, num_samples, mode, most_likely_z=False, full_dist=False,
                 all_z_sep=False):
        idx = torch.multinomial(self.p_dist[0], num_samples, replacement=True, generator=self.g)
        z = torch.nn.functional.one_hot(idx.T, self.L).to(torch.float32)  # (samples, nodes, L)
        return z, num_samples, 1


class _NodeModel:
    edge_types = ()

    def __init__(self, nodes, L, seed):
        self.n, self.latent = nodes, _Latent(L, seed)
        self.g = torch.Generator().manual_seed(seed + 1)

    def obtain_encoded_tensors(self, **kw):
        return (kw["inputs"], None, None, None, None, None)

    def p_z_x(self, mode, x):
        p = torch.rand((1, self.n, self.latent.L), generator=self.g) + 0.1
        return p / p.sum(-1, keepdim=True)

    def p_y_xz(self, mode, x, x_nr_t, y_r, n_s_t0, z, ph, n_samples, n_components, gmm_mode):
        # a deterministic function of z, so the two routes can be compared
        k = torch.argmax(z, -1).to(torch.float32)                      # (samples, nodes)
        t = torch.arange(1, ph + 1, dtype=torch.float32)
        pred = torch.stack([k[..., None] * t, -k[..., None] * 0.5 * t], -1)
        return None, pred + torch.randn(pred.shape, generator=self.g)


@pytest.fixture
def trajectron(monkeypatch):
    ds = types.ModuleType("model.dataset")
    mu = types.ModuleType("model.model_utils")
    mu.ModeKeys = types.SimpleNamespace(PREDICT="predict")
    nodes = [_Node(i) for i in ("ego", "3", "7")]

    def get_timesteps_data(env, scene, t, node_type, **kw):
        x = torch.zeros((len(nodes), 4))
        return (np.zeros(len(nodes), int), x, None, x, None, None, None, None, None), nodes, \
            [int(t[0])] * len(nodes)
    ds.get_timesteps_data = get_timesteps_data
    root = types.ModuleType("model")
    monkeypatch.setitem(sys.modules, "model", root)
    monkeypatch.setitem(sys.modules, "model.dataset", ds)
    monkeypatch.setitem(sys.modules, "model.model_utils", mu)
    return nodes


def _stg(nodes, seed):
    veh = "VEHICLE"
    return types.SimpleNamespace(
        env=types.SimpleNamespace(NodeType=types.SimpleNamespace(VEHICLE=veh)),
        pred_state={veh: {}}, state={}, max_ht=10, hyperparams={}, device="cpu",
        node_models_dict={veh: _NodeModel(len(nodes), 6, seed)})


def test_numpy_route_layouts(trajectron):
    z, pred, nodes, pdict, lp = prediction.generate_vehicle_latents(
        _stg(trajectron, 1), None, np.array([5]), num_samples=300, ph=8)
    assert isinstance(z, np.ndarray) and z.dtype == np.int64 and z.shape == (3, 300)
    assert pred.dtype == np.float32 and pred.shape == (3, 300, 8, 2)
    assert nodes == trajectron and lp.shape == (3, 6)
    for i, nd in enumerate(nodes):
        np.testing.assert_array_equal(pdict[5][nd], pred[i][None])


def test_keep_on_device_returns_the_same_values(trajectron):
    host = prediction.generate_vehicle_latents(_stg(trajectron, 2), None, np.array([5]),
                                               num_samples=257, ph=6)
    dev = prediction.generate_vehicle_latents(_stg(trajectron, 2), None, np.array([5]),
                                              num_samples=257, ph=6, keep_on_device=True)
    z, pred, nodes, pdict, lp = dev
    assert torch.is_tensor(z) and z.dtype == torch.int64 and tuple(z.shape) == (3, 257)
    assert torch.is_tensor(pred) and pred.dtype == torch.float32 and pred.is_contiguous()
    np.testing.assert_array_equal(z.numpy(), host[0])
    assert pred.numpy().tobytes() == host[1].tobytes()
    np.testing.assert_array_equal(lp, host[4])
    for i, nd in enumerate(nodes):
        np.testing.assert_array_equal(pdict[5][nd].numpy(), host[3][5][nd])
