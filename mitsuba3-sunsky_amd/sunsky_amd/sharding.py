"""Ray-batch sharding across the GPUs of one node.

Directions / samples are independent and the per-emitter tables (<= 16 KB) are
staged identically on every rank, so a batch of N rays splits into contiguous
per-rank slices with no data-path collective; the only exchange is the
optional gather of the radiance buffer to one rank (the reference's
ncclGather of configs[4]).  On GPUs that gather is the C ABI's
sunsky_gather_radiance (grouped RCCL send/recv over xGMI straight into the
root's final [C][N] planes, csrc/sunsky_comm.cpp); torch.distributed only hands
the RCCL unique id to the ranks.  CPU tensors (the gloo tests) take a
torch.distributed.gather fallback with the same partitioning.

Slice starts are multiples of 4 rays so every rank's SoA planes keep the
16-byte alignment the VEC=4 eval kernel needs.
"""
import ctypes as C
import weakref

import torch
import torch.distributed as dist

from ._capi import check, lib

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


_COMMS = {}   # key -> (RadianceComm, weak reference to the process group it was built over)


def _group_key(group, dev):
    """Cache key of a communicator: the group object, the device and the group's current
    rank / size; a process without torch.distributed gets its own world-1 key."""
    if not dist.is_available() or not dist.is_initialized():
        return (None, dev.index, 0, 1)
    return (id(group) if group is not None else None, dev.index, dist.get_rank(group), dist.get_world_size(group))


def _world_group(group):
    """The process group object a communicator for `group` is built over (the default group
    for None), or None without torch.distributed."""
    if not dist.is_available() or not dist.is_initialized():
        return None
    return group if group is not None else dist.distributed_c10d._get_default_group()


def radiance_comm(group=None, device=None, _factory=None):
    """The process's RadianceComm for (group, device), created on first use and kept: a
    communicator costs an RCCL init plus connection setup, far more than one gather.
    Collective on first use (every rank of the group calls it).  A cached communicator is
    reused only while the process group object it was built over is still the current one:
    a world torn down and re-initialised with the same rank and size (a new group object,
    whose id() may even equal the old one's) gets a new communicator, and the stale one is
    closed.  _factory: the communicator class (tests)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    key = _group_key(group, dev)
    g = _world_group(group)
    entry = _COMMS.get(key)
    if entry is not None:
        comm, ref = entry
        if comm._h is not None and ref() is g:
            return comm
        comm.close()
        del _COMMS[key]
    comm = (_factory or RadianceComm)(group, dev)
    _COMMS[key] = (comm, weakref.ref(g) if g is not None else (lambda: None))
    return comm


def clear_radiance_comms():
    """Close every cached communicator (call before dist.destroy_process_group(): RCCL
    communicators must not outlive the world they were built for, nor run their
    destructors after RCCL itself is gone at interpreter teardown)."""
    while _COMMS:
        _, (comm, _) = _COMMS.popitem()
        comm.close()


def gather_radiance(local, n_total, dst=0, group=None, comm=None, out=None):
    """Gather every rank's (C, n_r) radiance shard into the (C, n_total) buffer on `dst`
    (None elsewhere).  GPU shards go through the C ABI's RCCL gather (`comm`, or the
    cached radiance_comm(group, device)); CPU shards (gloo) through
    torch.distributed.gather of padded shards."""
    if local.is_cuda:
        comm = comm if comm is not None else radiance_comm(group, local.device)
        return comm.gather(local, n_total, root=dst, out=out)
    bufs = gather_shards(local, n_total, dst, group)
    if bufs is None:
        return None
    sizes = shard_sizes(n_total, dist.get_world_size(group))
    return torch.cat([b[:, :s] for b, s in zip(bufs, sizes)], dim=1)


class RadianceComm:
    """An RCCL communicator of the C ABI (sunsky_comm_create) over the ranks of a
    torch.distributed group, on `device` (default: the current one).  Collective:
    every rank of the group constructs it."""

    def __init__(self, group=None, device=None):
        self.group = group
        single = not dist.is_available() or not dist.is_initialized()
        if single and group is not None:
            raise ValueError("a process group was given but torch.distributed is not initialised")
        # without torch.distributed the communicator is the process alone (world 1, rank 0):
        # a one-GPU job gathers its own shard into the output planes through the same call
        self.rank = 0 if single else dist.get_rank(group)
        self.world = 1 if single else dist.get_world_size(group)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        uid = C.create_string_buffer(128)
        if self.rank == 0:
            check(lib().sunsky_comm_get_unique_id(uid))
        box = [bytes(uid.raw)]
        if not single:
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                       group=group)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().sunsky_comm_create(box[0], self.world, self.rank, C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().sunsky_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def gather(self, local, n_total, root=0, out=None, stream=None):
        """Every rank's (C, n_r) shard (n_r = shard_sizes(n_total)[rank]) into root's (C,
        n_total) planes; returns them on root, None elsewhere.  Stream-ordered on the
        current stream (or `stream`)."""
        sizes = shard_sizes(n_total, self.world)
        if local.dim() != 2 or local.shape[1] != sizes[self.rank] or local.dtype != torch.float32:
            raise ValueError(f"rank {self.rank}: shard must be float32 (C, {sizes[self.rank]})")
        if local.shape[1] and local.stride(1) != 1:
            raise ValueError("shard planes must be contiguous")
        c = local.shape[0]
        if self.rank == root and out is None:
            out = torch.empty((c, n_total), dtype=torch.float32, device=self.device)
        if self.rank == root and (tuple(out.shape) != (c, n_total) or out.stride(1) != 1):
            raise ValueError(f"out must be a (C, {n_total}) tensor with contiguous planes")
        counts = (C.c_size_t * self.world)(*sizes)
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        send = C.c_void_p(local.data_ptr()) if local.numel() else C.c_void_p()
        recv = C.c_void_p(out.data_ptr()) if self.rank == root else C.c_void_p()
        check(lib().sunsky_gather_radiance(self._h, root, send, local.stride(0) if c > 1 else sizes[self.rank], c,
                                           counts, recv, out.stride(0) if self.rank == root else 0,
                                           C.c_void_p(st.cuda_stream)))
        return out if self.rank == root else None

