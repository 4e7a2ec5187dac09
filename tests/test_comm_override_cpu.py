"""SUNSKY_AMD_RCCL (csrc/sunsky_comm.cpp `rccl()`): the communicator entry points dlopen the
library it names and only that one, failing loudly when it is missing.  CPU only:
`sunsky_comm_get_unique_id` touches no GPU, and the multi-process test double
(tests/cpp/fake_rccl_ipc.cpp) answers it with a private directory.  Each case runs in its own
process, since the library is resolved once per process."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOUBLE = os.path.join(ROOT, "tests", "cpp", "build", "libfake_rccl_ipc.so")

_CODE = """
import ctypes as C, sys
sys.path.insert(0, {pkg!r})
import sunsky_amd as ss
uid = C.create_string_buffer(128)
rc = ss.lib().sunsky_comm_get_unique_id(uid)
print("rc", rc)
print("id", uid.value.decode(errors="replace"))
print("err", ss.lib().sunsky_last_error().decode(errors="replace"))
"""


def _run(path):
    env = dict(os.environ, SUNSKY_AMD_RCCL=path)
    code = _CODE.format(pkg=os.path.join(ROOT, "mitsuba3-sunsky_amd"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return dict(line.split(" ", 1) for line in r.stdout.strip().splitlines() if " " in line)


def test_named_rccl_is_the_one_loaded():
    if not os.path.exists(DOUBLE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp"), "build/libfake_rccl_ipc.so"], check=True,
                       capture_output=True)
    out = _run(DOUBLE)
    assert out["rc"] == "0", out
    # the double's unique id: a private directory it created
    assert out["id"].startswith("/tmp/fake_rccl_ipc_") and os.path.isdir(out["id"]), out
    os.rmdir(out["id"])


def test_missing_named_rccl_fails_loudly():
    out = _run("/nonexistent/librccl_missing.so")
    assert out["rc"] != "0", out
    assert "SUNSKY_AMD_RCCL=/nonexistent/librccl_missing.so" in out["err"], out
