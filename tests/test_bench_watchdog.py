"""bench.py's configs[4] watchdog (VERDICT r03 weak 4 / ADVICE r03): a rank stuck in a
collective must not be reported as a success.  Past the limit rank 0 prints the bench line
with the C5 error and every rank exits non-zero (C5Watchdog.EXIT_CODE).  CPU only: one
process, then a gloo world-2 rehearsal in which rank 1 never reaches the barrier."""
import json
import os
import subprocess
import sys

import numpy as np

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
dist.init_process_group("gloo", init_method="file://" + os.environ["SUNSKY_TEST_STORE"], rank=rank, world_size=2)
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


def test_watchdog_gloo_world2_rank_stuck_in_collective(tmp_path):
    # the ranks meet through a file store in the test's own directory (no port race under pytest -n)
    env = dict(os.environ, SUNSKY_TEST_STORE=str(tmp_path / "rdv"), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, "-c", _RANK.format(root=ROOT)], env=dict(env, RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    codes = [p.returncode for p in procs]
    assert codes == [_exit_code()] * 2, (codes, [e[-2000:] for _, e in outs])
    assert "barrier passed" not in outs[0][0]
    line = json.loads(outs[0][0].strip().splitlines()[-1])
    assert line["value"] == 2.0 and "timed out" in line["c5_spectral_shard_gather"]["error"]
    assert "c5_spectral_shard_gather" not in outs[1][0]        # only rank 0 prints the line


# ----------------------------------------------------------- bench.py --gpus N
def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def test_launch_plan():
    b = _bench()
    assert b.launch_plan(1, {}) == "single"
    assert b.launch_plan(8, {}) == "spawn"
    assert b.launch_plan(8, {"WORLD_SIZE": "8"}) == "rank"
    assert b.launch_plan(1, {"WORLD_SIZE": "1"}) == "rank"
    for gpus, ws in ((4, "8"), (8, "4"), (1, "2"), (2, "1")):
        try:
            b.launch_plan(gpus, {"WORLD_SIZE": ws})
        except b.LaunchError as e:
            assert f"--gpus {gpus}" in str(e) and f"WORLD_SIZE={ws}" in str(e)
        else:
            raise AssertionError(f"--gpus {gpus} with WORLD_SIZE={ws} accepted")


def test_gpus_and_world_size_mismatch_exits_nonzero_before_the_gpu():
    env = dict(os.environ, WORLD_SIZE="8", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "--gpus 4 but the launcher set WORLD_SIZE=8" in p.stderr, p.stderr[-2000:]
    assert p.stdout.strip() == ""


def test_gpus_n_without_a_launcher_spawns_n_ranks():
    """`bench.py --gpus 3` with no WORLD_SIZE starts 3 rank processes itself (the parent touches
    no GPU); --launch-check makes each print its launch environment and stop before the GPU."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--launch-check"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = sorted((json.loads(x) for x in p.stdout.strip().splitlines()), key=lambda d: d["rank"])
    assert [d["rank"] for d in lines] == [0, 1, 2] and [d["local_rank"] for d in lines] == [0, 1, 2]
    assert {d["world"] for d in lines} == {3} and {d["gpus"] for d in lines} == {3}
    assert {d["plan"] for d in lines} == {"rank"}
    assert len({d["master"] for d in lines}) == 1 and lines[0]["master"].startswith("127.0.0.1:")


def test_spawned_ranks_rendezvous_through_a_file_store():
    """spawn_ranks' ranks meet through a file store in a private temporary directory
    (no TCP port to lose to another process between picking and binding it): 3 ranks over gloo
    all-reduce their ranks and leave no store behind."""
    import glob
    import tempfile
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    before = set(glob.glob(os.path.join(tempfile.gettempdir(), "sunsky_bench_rdv_*")))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--rendezvous-check"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.strip().splitlines() if x.startswith("{")]   # (gloo logs too)
    assert sorted(d["rank"] for d in lines) == [0, 1, 2]
    assert {d["rank_sum"] for d in lines} == {3.0} and {d["rendezvous"] for d in lines} == {"file"}
    assert set(glob.glob(os.path.join(tempfile.gettempdir(), "sunsky_bench_rdv_*"))) == before


def test_spawned_rank_failure_fails_the_run():
    """A rank that exits non-zero makes the spawning parent exit non-zero (its peers are given
    the grace period, then killed).  Here every rank fails fast: no GPU in the CPU suite."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "-1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0, p.stderr[-2000:]


_TEARDOWN = """
import os, sys, time
sys.path.insert(0, {root!r})
import torch.distributed as dist
import bench
rank = int(os.environ["RANK"])
dist.init_process_group("gloo", init_method="file://" + os.environ["SUNSKY_TEST_STORE"], rank=rank, world_size=2)
result = {{"metric": "m", "value": 3.0}} if rank == 0 else None

def run():
    if rank == {bad}:
        raise RuntimeError("comm setup failed")
    dist.barrier()                 # the failing rank never joins
    return {{"ok": True}}

c5, wd, failed = bench.c5_phase(run, rank, result, 4.0)
if rank == 0:
    result["c5_spectral_shard_gather"] = c5
    print(__import__("json").dumps(result), flush=True)
    wd.printed = True
bench.teardown(2, rank, wd, failed)
print("teardown passed", flush=True)
"""


def test_c5_failure_on_one_rank_ends_every_rank_nonzero(tmp_path):
    """a rank whose configs[4] raised skips the teardown collectives and exits
    EXIT_CODE; its peer, left in C5's collective, ends non-zero too: gloo raises when the peer
    is gone (the same path as a C5 error), RCCL would wait and the still-armed watchdog ends it
    (test_watchdog_gloo_world2_rank_stuck_in_collective)."""
    for bad in (1, 0):
        env = dict(os.environ, SUNSKY_TEST_STORE=str(tmp_path / f"rdv{bad}"), WORLD_SIZE="2")
        procs = [subprocess.Popen([sys.executable, "-c", _TEARDOWN.format(root=ROOT, bad=bad)],
                                  env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
                 for r in range(2)]
        outs = [p.communicate(timeout=120) for p in procs]
        codes = [p.returncode for p in procs]
        assert all(c != 0 for c in codes), (bad, codes, [e[-1500:] for _, e in outs])
        assert codes[bad] == _exit_code(), (bad, codes)
        assert "teardown passed" not in outs[0][0] + outs[1][0]
        lines = [x for x in outs[0][0].splitlines() if x.startswith("{")]
        assert len(lines) == 1, outs[0][0]            # one bench line, from rank 0 only
        line = json.loads(lines[0])
        assert line["value"] == 3.0 and "error" in line["c5_spectral_shard_gather"]
        if bad == 0:
            assert "comm setup failed" in line["c5_spectral_shard_gather"]["error"]


def test_sigterm_to_the_spawning_parent_ends_every_rank():
    """A launcher's timeout (SIGTERM to `bench.py --gpus N`) must not leave rank processes behind:
    the parent forwards the signal and exits 128 + 15.  CPU: the ranks sleep in --launch-check
    (SUNSKY_BENCH_TEST_HOLD), so they are still running when the signal comes."""
    import signal as sg
    import time as tm
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SUNSKY_BENCH_TEST_HOLD"] = "60"
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    pids = []
    deadline = tm.time() + 120
    while len(pids) < 2 and tm.time() < deadline:
        line = p.stdout.readline()
        if line.startswith("{"):
            pids.append(json.loads(line)["pid"])
    assert len(pids) == 2
    p.send_signal(sg.SIGTERM)
    assert p.wait(timeout=60) == 128 + sg.SIGTERM
    for pid in pids:
        for _ in range(100):
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            tm.sleep(0.1)
        else:
            raise AssertionError(f"rank pid {pid} outlived the parent")


def test_secondary_bursts_span_the_timed_window():
    """Round 5: each secondary burst runs at least SECONDARY_TIMED_MS of launches (the shader clock
    drifts over tens of ms under sustained load), never fewer than the step-derived count."""
    bench = _bench()
    assert bench.timed_reps(0.8, 25) == int(np.ceil(bench.SECONDARY_TIMED_MS / 0.8))
    assert bench.timed_reps(0.8, 25) * 0.8 >= bench.SECONDARY_TIMED_MS
    assert bench.timed_reps(100.0, 25) == 25
    assert bench.timed_reps(0.0, 3) >= 3
