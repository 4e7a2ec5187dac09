"""Profiler ranges (SURVEY.md §5 tracing): every C-ABI batch entry point opens a roctx range
named after the reference's ProfilerPhase scope (sunsky.cpp:304, 358, 402, 444, 454;
csrc/sunsky_profiler.h), so rocprofv3 --marker-trace attributes host time per call."""
import csv
import glob
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mitsuba3-sunsky_amd", "build", "libsunsky_amd.so")


def test_library_links_roctx():
    nm = shutil.which("nm")
    if nm is None:
        pytest.skip("nm not available")
    out = subprocess.run([nm, "-D", "--undefined-only", LIB], capture_output=True, text=True, check=True).stdout
    assert "roctxRangePushA" in out and "roctxRangePop" in out


@pytest.mark.gpu
def test_entry_points_emit_ranges(tmp_path):
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        pytest.skip("rocprofv3 not available")
    env = dict(os.environ, TMPDIR="/tmp")
    cmd = [prof, "--marker-trace", "--kernel-trace", "-d", str(tmp_path), "-o", "run", "--output-format", "csv",
           "--", sys.executable, os.path.join(ROOT, "tests", "roctx_worker.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=150, env=env, cwd="/tmp")
    assert r.returncode == 0 and "worker ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
    files = glob.glob(os.path.join(str(tmp_path), "**", "*marker_api_trace.csv"), recursive=True)
    assert files, os.listdir(str(tmp_path))
    names = set()
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                names.add(row.get("Function") or row.get("Message") or "")
    for want in ("InitScene:emitter_create", "EndpointEvaluate:eval", "EndpointSampleDirection:sample_direction",
                 "EndpointEvaluate:pdf_direction", "EndpointEvaluate:eval_direction",
                 "SamplingIntegratorSample:direct_diffuse"):
        assert want in names, (want, sorted(names))
