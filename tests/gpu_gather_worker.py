"""Worker of tests/test_gpu_gather.py: one rank of a multi-process run on the GPU box.
Each rank evaluates its shard of a spectral batch (C3 node kernel, 11 planes) with
the HIP kernels and the shards are gathered to the root (GATHER_ROOT, default 0) through
the C ABI's RCCL gather (sunsky_gather_radiance); the root compares with the whole batch
evaluated alone.  With SUNSKY_AMD_RCCL naming tests/cpp/build/libfake_rccl_ipc.so the
product's send/recv go through that multi-process test double instead of RCCL.
Exit 0 = bitwise equal, 3 = RCCL refused the configuration (e.g. two ranks on one
GPU), anything else = failure."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-sunsky_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import sunsky_amd as ss  # noqa: E402
from helpers import angles_dict, hemisphere_wo  # noqa: E402
from sunsky_amd.sharding import RadianceComm, shard_range  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    n = int(os.environ.get("GATHER_N", str((1 << 20) + 3)))
    root = int(os.environ.get("GATHER_ROOT", "0"))
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(rank % ndev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        em = ss.SunskyEmitter(angles_dict(3.0, 0.0, np.deg2rad(45), 0.3, 1.0, 1.0), "spectral")
        wi = torch.from_numpy(np.ascontiguousarray(-hemisphere_wo(n, seed=12).T)).cuda()
        lam = [float(x) for x in range(320, 721, 40)]
        a, b = shard_range(n, rank, world)
        local = em.eval_spectral_broadcast(wi[:, a:b].contiguous(), lam)
        try:
            comm = RadianceComm()
        except RuntimeError as e:
            print(f"rank {rank}: RCCL communicator refused: {e}", flush=True)
            return 3
        full = comm.gather(local, n, root=root)
        torch.cuda.synchronize()
        if rank == root:
            whole = em.eval_spectral_broadcast(wi, lam)
            torch.cuda.synchronize()
            ok = torch.equal(full, whole)
            print(f"rank {rank}: gathered {tuple(full.shape)} from {world} ranks, bitwise equal: {ok}", flush=True)
            if not ok:
                return 1
        comm.close()
        dist.barrier()
        return 0
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
