"""The RCCL branch of the path's one exchange, on one card: a world-size-1 `nccl` process group
(RCCL; device_id = cuda:0) runs dist.record_counts / gather_records on device tensors, then
bench.c4_sharded with the compact record all-gather inside its step -- the code the 8-GPU
scaling run executes (bench.py c4_sharded, init_dist).  The gathered block must equal the rank's
own records (128-byte, or packed to 32 bytes by ccmpc_compact_records) bit for bit."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = {"scenes": 3, "O": 2, "N": 2000, "T": 12}


def _worker(rank, port, out_dir):
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "cc-mpc_amd")]
    import torch.distributed as dist
    import bench
    from ccmpc import dist as cdist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # the rank's records without any process group (no exchange)
    out0, rec0 = bench.c4_sharded(dev, 99, 1, 0, steps=2, warmup=1, cfg=CFG, return_records=True)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        counts = cdist.record_counts(rec0.shape[0], dev)              # device tensors
        got = cdist.gather_records(rec0, counts=counts)
        got_c = cdist.gather_records(rec0, counts=counts, compact=True)
        torch.cuda.synchronize(dev)
        same_direct = bool(torch.equal(got.cpu(), rec0.cpu()))
        c0 = cdist.compact_records(rec0)
        same_compact = bool(torch.equal(got_c.cpu(), c0.cpu())) and got_c.shape[2] == 32
        out1, rec1 = bench.c4_sharded(dev, 99, 1, 0, steps=3, warmup=1, cfg=CFG,
                                      return_records=True)
        torch.cuda.synchronize(dev)
        res = {"counts": counts, "same_direct": same_direct, "same_compact": same_compact,
               "same_step": bool(torch.equal(rec1.cpu(), c0.cpu())),
               "gather": out1["record_gather"], "gather0": out0["record_gather"],
               "device": str(rec1.device), "records_ok": out1["records_ok"]}
        with open(os.path.join(out_dir, "rccl.json"), "w") as f:
            json.dump(res, f)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_world1_record_gather(gpu, tmp_path):
    import json
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    res = json.load(open(os.path.join(tmp_path, "rccl.json")))
    assert res["counts"] == [res["counts"][0]] and res["counts"][0] > 0
    assert res["same_direct"] and res["same_compact"] and res["same_step"], res
    assert res["gather0"] == "none (N=1)"
    assert res["gather"].startswith("RCCL"), res
    assert res["device"].startswith("cuda") and res["records_ok"]
