"""The sharded path on the device: two ranks on one card (gloo backend; RCCL will
not form a communicator from two ranks on one device), each running ONE batched HIP cycle over
its contiguous block of scenes (ccmpc.dist.scene_range) with every scene's own reference
trajectory, then the one exchange -- gather_records.  The gathered block must equal, bit for
bit, the single-rank batch of all scenes (the partition is invisible in the results)."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

T, O, N = 12, 4, 1500
SEEDS = list(range(4300, 4307))          # 7 scenes: an uneven 4 / 3 split


def _batch_records(seeds, device):
    from ccmpc import cycle, engine, synthetic
    scenes = [synthetic.scene(s, O=O, N=N, T=T) for s in seeds]
    cells = [c for ovs, _, _ in scenes for o in ovs for c in o]
    scene_K = [[len(o) for o in ovs] for ovs, _, _ in scenes]
    store = engine.ParticleStore.from_cells(cells, device=device)
    cyc = cycle.MinkowskiCycle(store, [k for K in scene_K for k in K],
                               np.array([r for _, r, _ in scenes]), scene_K=scene_K)
    cyc.run()
    return cyc.rec


def _worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "cc-mpc_amd")]
    import torch.distributed as dist
    from ccmpc import dist as cdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b, e = cdist.scene_range(len(SEEDS), rank, world)
        rec = _batch_records(SEEDS[b:e], torch.device("cuda:0"))
        full = cdist.gather_records(rec.cpu())
        if rank == 0:
            torch.save(full, os.path.join(out_dir, "gathered.pt"))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_shard_a_multi_scene_cycle(gpu, tmp_path):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    got = torch.load(os.path.join(tmp_path, "gathered.pt"), weights_only=True)
    want = _batch_records(SEEDS, gpu).cpu()
    assert got.shape == want.shape
    assert torch.equal(got, want)
    from ccmpc import _lib
    recs = got.numpy().view(_lib.HALFSPACE_DTYPE).reshape(got.shape[:2])
    assert np.all(recs["status"] == 0)


BENCH_CFG = {"scenes": 5, "O": 3, "N": 1200, "T": 12}


def _bench_worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "cc-mpc_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        out, full = bench.c4_sharded(torch.device("cuda:0"), 77, world, rank, steps=2, warmup=1,
                                     cfg=BENCH_CFG, return_records=True)
        if rank == 0:
            torch.save(full.cpu(), os.path.join(out_dir, "bench_gathered.pt"))
            assert out["records_ok"] and out["n_gpus"] == world
    finally:
        dist.destroy_process_group()


def test_bench_c4_shard_path_gathers_every_scene(gpu, tmp_path):
    """bench.py's c4_sharded (what the driver's SCALE run times at N > 1) on two gloo ranks:
    the records gathered inside the timed step are the single-rank batch's (packed to 32 bytes
    by ccmpc_compact_records), bit for bit."""
    import sys
    import torch.multiprocessing as mp
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    mp.start_processes(_bench_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2,
                       join=True, start_method="spawn")
    got = torch.load(os.path.join(tmp_path, "bench_gathered.pt"), weights_only=True)
    _, want = bench.c4_sharded(gpu, 77, 1, 0, steps=1, warmup=1, cfg=BENCH_CFG,
                               return_records=True)
    from ccmpc import dist as cdist
    assert got.shape[2] == 32           # the step gathers the compact (32-byte) records
    assert torch.equal(got, cdist.compact_records(want).cpu())
