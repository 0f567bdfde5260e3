"""Multi-GPU layout of the path: one process per GPU, scenes sharded.

Cells (scene, OV, mode) are independent, so a node runs the path as weak-scaled shards:

* ``scene_range`` gives each rank a contiguous block of scenes; particles are sampled, bucketed,
  reduced and turned into half-spaces on the rank that owns the scene and never leave its HBM.
* RNG streams are keyed by the GLOBAL cell id (``rng_cell`` of ccmpc_ideal_rollout /
  ccmpc_ideal_moments, the sampler's OV index), so every cell's draws -- and therefore every
  record -- are identical at 1, 2, 4 or 8 ranks.
* The planner's QP for a scene stays on the owning rank (v8ideal/__init__.py:2934-2976 solves
  one scene per agent), so the data path has NO collective.  ``gather_records`` is the one
  optional exchange, for a consumer that wants every scene's fixed-size half-space records on
  every rank (a fleet-level monitor, or a rank-0 logger): one all_gather of the padded record
  block, which RCCL runs over xGMI on a GPU node and gloo runs on the CPU in the tests.
"""
import torch

REC_BYTES = 128
COMPACT_BYTES = 32      # ccmpc_gather_rec: n0, n1, rhs, side, status, t_tau


def compact_records(rec, kind=0):
    """The QP-read fields of a record block, packed on the device (ccmpc_compact_records):
    uint8 (cells, P, 128) -> (cells, P, 32) ccmpc_gather_rec.  kind: 0 half-space, 1 affine
    (mpc.REC_HALFSPACE / REC_AFFINE).  The QP reads the result in place (mpc.REC_*_COMPACT)."""
    from . import _lib, engine
    if rec.dtype != torch.uint8 or rec.dim() != 3 or rec.shape[2] != REC_BYTES:
        raise ValueError("rec must be a uint8 (cells, P, 128) record block")
    if rec.device.type != "cuda":
        raise _lib.CcmpcError("compact_records runs on the GPU (ccmpc_compact_records)")
    rec = rec.contiguous()
    out = torch.empty(tuple(rec.shape[:2]) + (COMPACT_BYTES,), dtype=torch.uint8,
                      device=rec.device)
    with torch.cuda.device(rec.device):
        _lib.check(_lib.load().ccmpc_compact_records(
            engine._p(rec), int(kind), rec.shape[0] * rec.shape[1], engine._p(out),
            engine._stream()), "ccmpc_compact_records")
    return out


def scene_range(n_scenes, rank, world):
    """[begin, end) of the scenes owned by `rank`: contiguous blocks, sizes differ by <= 1."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    base, extra = divmod(int(n_scenes), world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def global_cell_ids(cells_per_scene, begin, end):
    """Global ids of the cells of scenes [begin, end), given every scene's cell count (the
    cells of scene s are numbered after those of scenes < s)."""
    first = sum(int(c) for c in cells_per_scene[:begin])
    n = sum(int(c) for c in cells_per_scene[begin:end])
    return list(range(first, first + n))


def record_counts(n_local, device, group=None):
    """Every rank's cell count (one small all_gather; synchronises).  A planner whose shard
    shapes are fixed exchanges them once and passes them to ``gather_records``."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([int(n_local)], dtype=torch.int64, device=device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    return [int(x.item()) for x in ns]


def gather_records(rec, group=None, counts=None, compact=False, kind=0):
    """All-gather every rank's record block.

    rec: uint8 tensor (n_local, P, 128) -- or (n_local, P, 32) already-packed ccmpc_gather_rec
    -- on this rank's device (CPU under gloo).  compact=True packs 128-byte records on the GPU
    first (compact_records; kind 0 half-space, 1 affine), so a quarter of the bytes cross xGMI.
    Ranks may hold different numbers of cells; blocks are padded to the largest and trimmed
    after the exchange.  ``counts`` (every rank's n_local, from ``record_counts``) skips the
    count exchange, so the call enqueues without a host synchronisation.  Returns the
    (sum n, P, bytes) block in rank order, i.e. the global cell order of contiguous
    ``scene_range`` shards.
    """
    import torch.distributed as dist
    if rec.dtype != torch.uint8 or rec.dim() != 3 or rec.shape[2] not in (REC_BYTES,
                                                                             COMPACT_BYTES):
        raise ValueError("rec must be a uint8 (cells, P, 128 or 32) record block")
    if compact and rec.shape[2] == REC_BYTES:
        rec = compact_records(rec, kind)
    world = dist.get_world_size(group)
    if counts is None:
        counts = record_counts(rec.shape[0], rec.device, group)
    elif len(counts) != world or counts[dist.get_rank(group)] != rec.shape[0]:
        raise ValueError(f"counts {counts} do not match this rank's {rec.shape[0]} cells")
    cap = max(counts)
    if rec.shape[0] == cap:
        padded = rec.contiguous()
    else:
        padded = rec.new_zeros((cap,) + tuple(rec.shape[1:]))
        padded[: rec.shape[0]] = rec
    out = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(out, padded, group=group)
    return torch.cat([o[:c] for o, c in zip(out, counts)], dim=0)
