"""bench.py's configs[4] watchdog (VERDICT r03 weak 4 / ADVICE r03): a rank stuck in a
collective must not be reported as a success.  Past the limit rank 0 prints the bench line
with the C5 error and every rank exits non-zero (C5Watchdog.EXIT_CODE).  CPU only: one
process, then a gloo world-2 rehearsal in which rank 1 never reaches the barrier."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_ONE = """
import sys, time
sys.path.insert(0, {root!r})
import bench
bench.C5Watchdog(0.5, 0, {{"metric": "m", "value": 1.0}}).start()
time.sleep(60)
"""

_RANK = """
import os, sys, time
sys.path.insert(0, {root!r})
import torch.distributed as dist
import bench
rank = int(os.environ["RANK"])
dist.init_process_group("gloo")
result = {{"metric": "m", "value": 2.0}} if rank == 0 else None
bench.C5Watchdog(3.0, rank, result).start()
if rank == 1:
    time.sleep(60)          # never reaches the collective
dist.barrier()
print("barrier passed", flush=True)
"""


def _exit_code():
    sys.path.insert(0, ROOT)
    import bench
    return bench.C5Watchdog.EXIT_CODE


def test_watchdog_prints_the_line_and_exits_nonzero():
    p = subprocess.run([sys.executable, "-c", _ONE.format(root=ROOT)], capture_output=True, text=True, timeout=120)
    assert p.returncode == _exit_code() != 0, p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["value"] == 1.0 and "timed out" in line["c5_spectral_shard_gather"]["error"]


def test_watchdog_gloo_world2_rank_stuck_in_collective():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, "-c", _RANK.format(root=ROOT)], env=dict(env, RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    codes = [p.returncode for p in procs]
    assert codes == [_exit_code()] * 2, (codes, [e[-2000:] for _, e in outs])
    assert "barrier passed" not in outs[0][0]
    line = json.loads(outs[0][0].strip().splitlines()[-1])
    assert line["value"] == 2.0 and "timed out" in line["c5_spectral_shard_gather"]["error"]
    assert "c5_spectral_shard_gather" not in outs[1][0]        # only rank 0 prints the line
