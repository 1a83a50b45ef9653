"""Multi-GPU plumbing for bench.py: one process per GPU, streams sharded.

Streams are independent: each rank decodes a contiguous range
of a global batch with no data-path collective.  The only collectives are the
timing/verification reductions (barrier, MAX of elapsed time, MIN of the
verified flag), which work on both backends: "nccl" (RCCL over xGMI, CUDA
tensors) on the GPU box and "gloo" (CPU tensors) in the CPU test-suite.

Config 4 (LZMA2 dict-reset blocks) has the one real exchange:
the compressed file sits on rank 0 and each peer receives the byte range of its
blocks (and its block table) by point-to-point sends -- RCCL over xGMI on the
box, one link per peer, all sends posted as one group.  The optional last step
(8(e) step 5) gathers every rank's decoded blocks back to rank 0 the same way.
"""
import os


def world_info():
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(total, world, rank):
    """Contiguous, balanced [start, start+count) of `total` streams for `rank`."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def shard_by_weight(weights, world, rank):
    """Contiguous range of items whose cumulative weight (e.g. decompressed
    bytes) falls in rank's 1/world slice -- balances mixed-length batches."""
    total = float(sum(weights))
    lo, hi = total * rank / world, total * (rank + 1) / world
    acc, start, end = 0.0, None, len(weights)
    for i, w in enumerate(weights):
        mid = acc + w / 2.0
        if start is None and mid >= lo:
            start = i
        if mid >= hi:
            end = i
            break
        acc += w
    if start is None:
        start = len(weights)
    return start, max(0, end - start)


def _tensor(value, dtype, device):
    import torch
    return torch.tensor([value], dtype=dtype, device=device)


def reduce_max(value, device="cpu"):
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = _tensor(value, torch.float64, device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(value, device="cpu"):
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = _tensor(value, torch.float64, device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def all_true(flag, device="cpu"):
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return bool(flag)
    t = _tensor(1 if flag else 0, torch.int32, device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def barrier():
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def scatter_ranges(src, ranges, out, rank, world):
    """Rank 0 sends src[lo:hi] of ranges[r] = (lo, hi) to rank r; every rank
    gets its own range in `out` (rank 0 copies locally).  src is only read on
    rank 0 (None elsewhere); out has hi - lo elements on each rank.  All
    transfers are posted as one batch (grouped point-to-point)."""
    import torch.distributed as dist
    lo, hi = ranges[rank]
    if rank == 0:
        out.copy_(src[lo:hi])
    if world == 1:
        return
    ops = []
    if rank == 0:
        for r in range(1, world):
            a, b = ranges[r]
            if b > a:
                ops.append(dist.P2POp(dist.isend, src[a:b], r))
    elif hi > lo:
        ops.append(dist.P2POp(dist.irecv, out, 0))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()


def gather_ranges(mine, sizes, out, rank, world):
    """Every rank r sends its `mine` (sizes[r] elements) to rank 0, which lands
    it at out[sum(sizes[:r]) : + sizes[r]] (its own part by a local copy); out
    is only written on rank 0 (None elsewhere).  One grouped point-to-point
    batch, like scatter_ranges."""
    import torch.distributed as dist
    offs = [0]
    for n in sizes:
        offs.append(offs[-1] + n)
    if rank == 0:
        out[offs[0]:offs[1]].copy_(mine[:sizes[0]])
    if world == 1:
        return
    ops = []
    if rank == 0:
        for r in range(1, world):
            if sizes[r]:
                ops.append(dist.P2POp(dist.irecv, out[offs[r]:offs[r + 1]], r))
    elif sizes[rank]:
        ops.append(dist.P2POp(dist.isend, mine[:sizes[rank]], 0))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
