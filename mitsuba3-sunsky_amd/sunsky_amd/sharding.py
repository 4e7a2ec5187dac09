"""Ray-batch sharding across the GPUs of one node.

Directions / samples are independent and the per-emitter tables (<= 16 KB) are
staged identically on every rank, so a batch of N rays splits into contiguous
per-rank slices with no data-path collective; the only exchange is the
optional gather of the radiance buffer to one rank (the reference's
ncclGather of configs[4]), done here with torch.distributed (backend "nccl" =
RCCL over xGMI on MI355X, "gloo" for the CPU tests).

Slice starts are multiples of 4 rays so every rank's SoA planes keep the
16-byte alignment the VEC=4 eval kernel needs.
"""
import torch
import torch.distributed as dist

ALIGN = 4


def shard_range(n, rank, world):
    """[start, stop) of rank's contiguous slice of n rays (balanced, 4-aligned starts)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"invalid rank {rank} of world {world}")
    blocks = (n + ALIGN - 1) // ALIGN
    per, extra = divmod(blocks, world)
    b0 = rank * per + min(rank, extra)
    b1 = b0 + per + (1 if rank < extra else 0)
    return min(n, b0 * ALIGN), min(n, b1 * ALIGN)


def shard_sizes(n, world):
    return [shard_range(n, r, world)[1] - shard_range(n, r, world)[0] for r in range(world)]


def gather_shards(local, n_total, dst=0, group=None, bufs=None):
    """The collective alone: every rank's (C, n_r) shard, padded to the largest shard, into
    `dst`'s list of per-rank (C, m) buffers (rank-major, as ncclGather lays them out).
    Returns that list on `dst` (None elsewhere); `bufs` may be a preallocated list."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = shard_sizes(n_total, world)
    c = local.shape[0]
    if local.shape[1] != sizes[rank]:
        raise ValueError(f"rank {rank}: shard has {local.shape[1]} rays, expected {sizes[rank]}")
    m = max(sizes)
    send = local
    if local.shape[1] != m:
        send = torch.zeros((c, m), dtype=local.dtype, device=local.device)
        send[:, : local.shape[1]] = local
    send = send.contiguous()
    if rank == dst and bufs is None:
        bufs = [torch.empty((c, m), dtype=local.dtype, device=local.device) for _ in range(world)]
    dist.gather(send, bufs if rank == dst else None, dst=dst, group=group)
    return bufs if rank == dst else None


def gather_radiance(local, n_total, dst=0, group=None):
    """Gather every rank's (C, n_r) radiance shard into the (C, n_total) buffer on `dst`
    (None elsewhere).  Shards are padded to the largest size for the collective."""
    bufs = gather_shards(local, n_total, dst, group)
    if bufs is None:
        return None
    sizes = shard_sizes(n_total, dist.get_world_size(group))
    return torch.cat([b[:, :s] for b, s in zip(bufs, sizes)], dim=1)
