"""Multi-rank layout of the path on the CPU (gloo, world_size 2): scene sharding, global-cell
keying and the record exchange of ccmpc.dist.  The per-cell compute is the
oracle here (no GPU); what is under test is the host logic around it."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ccmpc import dist as cdist
from ccmpc import _lib
from oracle import ccmpc_oracle as orc


def test_scene_range_partitions_every_scene_once():
    for n in (0, 1, 7, 8, 64, 65):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                b, e = cdist.scene_range(n, r, world)
                assert 0 <= b <= e <= n
                got += list(range(b, e))
            assert got == list(range(n))
            sizes = [np.subtract(*cdist.scene_range(n, r, world)[::-1]) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        cdist.scene_range(4, 2, 2)


def test_global_cell_ids():
    cells = [3, 1, 4, 2]
    assert cdist.global_cell_ids(cells, 0, 4) == list(range(10))
    assert cdist.global_cell_ids(cells, 1, 3) == [3, 4, 5, 6, 7]
    assert cdist.global_cell_ids(cells, 2, 2) == []


def _scene_records(scene, T=6):
    """Records of one synthetic scene: the oracle's Minkowski generator packed into the
    128-byte ccmpc_halfspace layout, shape (cells, T(T-1)/2, 128) uint8."""
    rng = np.random.default_rng(1000 + scene)
    O = 1 + scene % 2
    ovs, cells_per_ov = [], []
    for o in range(O):
        K = 1 + (scene + o) % 2
        cells = []
        for _ in range(K):
            steps = rng.normal(0, 0.3, size=(300, T, 2)) + np.array([2.0, 0.3])
            cells.append(np.cumsum(steps, axis=1) + np.array([190.0, -80.0]))
        past = np.array([[189.0, -80.0]])
        ovs.append(orc.OVehicle(T, past, np.ones(K) / K, cells,
                                [orc._step_yaws(c, past[-1], T) for c in cells],
                                np.zeros((K, 2)), np.array([4.5, 2.5])))
        cells_per_ov.append(K)
    ref = np.stack([np.array([170.0 + 4 * (t + 1), -70.0 + 0.5 * (t + 1)]) for t in range(T)])
    want = orc.minkowski_generator(ovs, T, T, ref, with_l4=False)
    P = T * (T - 1) // 2
    recs = np.zeros((sum(cells_per_ov), P), dtype=_lib.HALFSPACE_DTYPE)
    idx = {}
    for r in want["records"]:
        cell = sum(cells_per_ov[: r["ov"]]) + r["k"]
        j = idx.get(cell, 0)
        idx[cell] = j + 1
        rec = recs[cell, j]
        rec["n0"], rec["n1"], rec["d"] = r["n"][0], r["n"][1], r["d"]
        rec["which"], rec["side"], rec["t_tau"] = r["which"], r["side"], (r["t"] << 16) | r["tau"]
    return torch.from_numpy(recs.view(np.uint8).reshape(len(recs), P, 128).copy())


GATHER_DTYPE = np.dtype([("n0", "<f8"), ("n1", "<f8"), ("rhs", "<f8"), ("side", "<i2"),
                         ("status", "<i2"), ("t_tau", "<i4")])      # ccmpc_gather_rec


def _pack32(block):
    """The 32-byte ccmpc_gather_rec packing of a half-space block, restated in numpy: what
    ccmpc_compact_records writes on the GPU (tests/test_gpu_mpc.py checks the kernel against
    the records' own fields); here only the gather of packed blocks is under test."""
    h = block.numpy().reshape(-1, 128).view(_lib.HALFSPACE_DTYPE).reshape(-1)
    out = np.zeros(h.shape, GATHER_DTYPE)
    for f in ("n0", "n1", "side", "status", "t_tau"):
        out[f] = h[f]
    out["rhs"] = h["d"]
    return torch.from_numpy(out.view(np.uint8).reshape(block.shape[0], block.shape[1], 32).copy())


def _worker(rank, world, port, n_scenes, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b, e = cdist.scene_range(n_scenes, rank, world)
        local = [_scene_records(s) for s in range(b, e)]
        P = local[0].shape[1] if local else 15
        block = torch.cat(local) if local else torch.zeros((0, P, 128), dtype=torch.uint8)
        full = cdist.gather_records(block)
        compact = cdist.gather_records(_pack32(block))      # the 32-byte exchange
        if rank == 0:
            torch.save(full, os.path.join(out_dir, "gathered.pt"))
            torch.save(compact, os.path.join(out_dir, "gathered32.pt"))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n_scenes", [5, 1])
def test_gather_records_world2_equals_single_rank(tmp_path, n_scenes):
    """Two gloo ranks, each planning its own scene shard (uneven, or one rank empty), gather
    exactly the record block a single rank produces for all scenes, in global cell order."""
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), n_scenes, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    got = torch.load(os.path.join(tmp_path, "gathered.pt"), weights_only=True)
    want = torch.cat([_scene_records(s) for s in range(n_scenes)])
    assert got.shape == want.shape
    assert torch.equal(got, want)
    recs = got.numpy().view(_lib.HALFSPACE_DTYPE).reshape(got.shape[:2])
    assert np.all(np.isfinite(recs["d"]))
    got32 = torch.load(os.path.join(tmp_path, "gathered32.pt"), weights_only=True)
    assert got32.shape == want.shape[:2] + (32,)
    assert torch.equal(got32, _pack32(want))           # a quarter of the bytes, the same fields
    with pytest.raises(ValueError):
        cdist.gather_records(torch.zeros((1, 3, 64), dtype=torch.uint8))
