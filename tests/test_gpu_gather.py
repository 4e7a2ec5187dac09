"""The configs[4] gather through the C ABI (sunsky_gather_radiance, csrc/sunsky_comm.cpp;
SURVEY.md §8e): RCCL grouped send/recv of every rank's radiance planes into root's
final [C][N] planes.

* one rank (the communicator of a single process): root's own shard copied into place,
  and the in-place case (shard already at its columns) copies nothing;
* two processes on the box's GPU(s): shards evaluated by the HIP kernels, gathered to
  rank 0, bitwise equal to the whole batch evaluated alone.  With one GPU both ranks
  share it; if RCCL refuses two ranks on one device the test is skipped with its reason;
* the multi-rank send/recv branch itself on one GPU, 2-4 ranks in one process, with the
  RCCL entry points served by the test double tests/cpp/fake_rccl.cpp (linked by the
  test program tests/cpp/gather_double_check): ragged and empty shards, 3 and 11 planes,
  either root, either call order;
* the same branch with the ranks as separate PROCESSES on one GPU (the layout of a real
  multi-GPU job, and of bench.py's rehearsal with SUNSKY_BENCH_RCCL_DOUBLE): the product
  dlopens the multi-process double tests/cpp/fake_rccl_ipc.cpp through SUNSKY_AMD_RCCL,
  torch.distributed (gloo) carries the unique id as in a real job.
"""
import ctypes as C
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import sunsky_amd as ss
from sunsky_amd.sharding import shard_sizes

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def test_single_rank_gather_and_in_place():
    L = ss.lib()
    uid = C.create_string_buffer(128)
    ss._capi.check(L.sunsky_comm_get_unique_id(uid))
    h = C.c_void_p()
    ss._capi.check(L.sunsky_comm_create(uid.raw, 1, 0, C.byref(h)))
    try:
        r, w, d = C.c_int(), C.c_int(), C.c_int()
        ss._capi.check(L.sunsky_comm_info(h, C.byref(r), C.byref(w), C.byref(d)))
        assert (r.value, w.value, d.value) == (0, 1, 0)
        n, c = 1000 + 3, 11
        local = torch.randn((c, n), device="cuda")
        out = torch.full((c, n), -1.0, device="cuda")
        counts = (C.c_size_t * 1)(n)
        st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        ss._capi.check(L.sunsky_gather_radiance(h, 0, C.c_void_p(local.data_ptr()), n, c, counts,
                                                C.c_void_p(out.data_ptr()), n, st))
        torch.cuda.synchronize()
        assert torch.equal(out, local)
        # in place: the shard already sits at its columns of the output planes
        ss._capi.check(L.sunsky_gather_radiance(h, 0, C.c_void_p(out.data_ptr()), n, c, counts,
                                                C.c_void_p(out.data_ptr()), n, st))
        torch.cuda.synchronize()
        assert torch.equal(out, local)
        # argument checks
        with pytest.raises(ValueError):
            ss._capi.check(L.sunsky_gather_radiance(h, 1, C.c_void_p(local.data_ptr()), n, c, counts,
                                                    C.c_void_p(out.data_ptr()), n, st))
        with pytest.raises(ValueError):
            ss._capi.check(L.sunsky_gather_radiance(h, 0, C.c_void_p(local.data_ptr()), n, c, counts,
                                                    C.c_void_p(out.data_ptr()), n - 1, st))
    finally:
        L.sunsky_comm_destroy(h)


def run_workers(world, **extra):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), **extra)
    worker = os.path.join(ROOT, "tests", "gpu_gather_worker.py")
    procs = [subprocess.Popen([sys.executable, worker], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=150)
            outs.append((p.returncode, out))
    except subprocess.TimeoutExpired:
        for p in procs:
            p.kill()
        pytest.fail("gather workers timed out")
    codes = [c for c, _ in outs]
    text = "\n".join(o for _, o in outs)
    print(text)
    return codes, text


def test_two_ranks_rccl_gather_bitwise():
    codes, text = run_workers(2)
    if 3 in codes:
        pytest.skip("RCCL refused this configuration: " + text.strip().splitlines()[-1][:300])
    assert codes == [0, 0], text
    assert "bitwise equal: True" in text


@pytest.mark.parametrize("world,root", [(4, 0), (3, 2), (8, 5)])
def test_rank_processes_gather_through_ipc_double(world, root):
    """`world` rank processes on one GPU (8: the driver's node size), each evaluating a ragged
    shard of 2^20 + 3 rays;
    sunsky_gather_radiance's grouped send / recv served by tests/cpp/fake_rccl_ipc.cpp (device
    memory exported between the processes with hipIpc handles)."""
    so = os.path.join(ROOT, "tests", "cpp", "build", "libfake_rccl_ipc.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp"), "build/libfake_rccl_ipc.so"], check=True,
                       capture_output=True)
    codes, text = run_workers(world, SUNSKY_AMD_RCCL=so, GATHER_ROOT=str(root), SUNSKY_FAKE_RCCL_TIMEOUT="60")
    assert codes == [0] * world, text
    assert f"rank {root}: gathered (11, {(1 << 20) + 3}) from {world} ranks, bitwise equal: True" in text


def test_multi_rank_gather_through_rccl_double():
    """sunsky_gather_radiance's grouped ncclSend / ncclRecv branch (csrc/sunsky_comm.cpp) with
    2, 3 and 4 ranks on one GPU: tests/cpp/gather_double_check links the RCCL test double
    (tests/cpp/fake_rccl.cpp, soname librccl.so.1) so the product's dlopen finds it."""
    exe = os.path.join(ROOT, "tests", "cpp", "build", "gather_double_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp"), "build/gather_double_check"], check=True,
                       capture_output=True)
    p = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240)
    print(p.stdout)
    assert p.returncode == 0, p.stdout
    assert "48 cases bitwise equal" in p.stdout


def test_c5_sized_gather_through_rccl_double():
    """configs[4] at its own sizes: 4 ranks x 64M rays x the 11 node planes,
    each shard evaluated by the C3 node kernel on its own and gathered through the grouped
    send / recv branch into the root's (11, 256M) planes -- 2.95e9 floats, plane offsets past
    2^33 bytes -- then every gathered float compared with the whole batch evaluated alone,
    bitwise, for root 0 and root 3 (ranks calling in reverse order).  ~45 GB of HBM."""
    if torch.cuda.get_device_properties(0).total_memory < (64 << 30):
        pytest.skip("needs > 64 GiB of device memory")
    exe = os.path.join(ROOT, "tests", "cpp", "build", "gather_double_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp"), "build/gather_double_check"], check=True,
                       capture_output=True)
    p = subprocess.run([exe, "c5", "4", str(1 << 26)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=240)
    print(p.stdout)
    assert p.returncode == 0, p.stdout
    assert "c5 gather through the RCCL double: 2 cases bitwise equal" in p.stdout
