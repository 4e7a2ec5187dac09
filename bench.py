#!/usr/bin/env python3
"""Benchmark of the MI355X sun/sky emitter hot path (BASELINE.json north_star).

Headline (config 2 of BASELINE.json): RGB eval() of 16,777,216 uniform
upper-hemisphere directions per GPU, turbidity in {2, 6, 10} (sun at 45 deg
elevation, albedo 0.1).  One "step" = one eval pass over the batch for each of
the three turbidities = 3 x 16,777,216 direction evals.  Inputs are resident
in HBM before the timed region; outputs are written to HBM.

Secondary lines (reported under "secondary", not in `value`): config 3
(spectral eval, 16M dirs x the 11 model wavelengths, broadcast) and config 4
(sample_direction + pdf_direction on 64M samples).

Multi-GPU (torchrun, one process per GPU): every rank evaluates its own
16M-direction shard -- weak scaling, no data-path collective.  `--gather`
additionally times the RCCL gather of the radiance buffer to rank 0 (reported
separately; never part of `value`).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import ctypes
import json
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-sunsky_amd"))
import sunsky_amd as ss  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
N_DIRS = 1 << 24          # 16,777,216 (BASELINE.json configs[1])
TURBIDITIES = (2.0, 6.0, 10.0)
SUN_SLACK = [1.25]         # sun-disc lane bound k (tests/helpers.py SUN_SLACK): 1.25 fast, 4 reference
NB = 4                    # rotating headline input batches (4 x 201 MB > the 256 MiB Infinity Cache)
BYTES_RGB = 24            # 12 B wi + 12 B RGB per direction
BYTES_SPEC_PER_DIR = 12 + 11 * 4
BYTES_SAMPLE = 52


def sun_dict(turb, eta_deg=45.0, albedo=0.1, phi=0.0):
    th = np.deg2rad(90.0 - eta_deg)
    return {"type": "sunsky", "turbidity": turb, "albedo": albedo,
            "sun_direction": [float(np.cos(phi) * np.sin(th)), float(np.sin(phi) * np.sin(th)), float(np.cos(th))]}


def hemisphere_dirs(n, seed, device):
    """cos(theta) = u1, phi = 2 pi u2, SoA (3, n) fp32 on device."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    u = torch.rand((2, n), generator=g, device=device, dtype=torch.float32)
    ct = u[0]
    st = torch.sqrt(torch.clamp(1 - ct * ct, min=0))
    ph = 2 * np.pi * u[1]
    return torch.stack([st * torch.cos(ph), st * torch.sin(ph), ct]).contiguous()


class KernelTimer:
    """HIP events on the stream the C ABI launches on (torch's current stream),
    bracketing a burst of back-to-back launches: mean duration per launch
    (dispatch gaps included, so it is an upper bound on the rocprof average)."""

    def __init__(self):
        self.launches = 0
        self.t0 = torch.cuda.Event(enable_timing=True)
        self.t1 = torch.cuda.Event(enable_timing=True)

    def begin(self):
        self.t0.record()

    def end(self, launches):
        self.t1.record()
        self.launches = launches

    def mean_ms(self):
        torch.cuda.synchronize()
        return self.t0.elapsed_time(self.t1) / max(self.launches, 1)

    def mean_ms_with_clock(self):
        """mean_ms, plus the GFX clock (amd-smi, torch.cuda.clock_rate) polled on the host
        while the burst runs: (ms, median MHz or None)."""
        clk = []
        try:
            while not self.t1.query():
                clk.append(torch.cuda.clock_rate())
                time.sleep(0.002)
        except Exception:   # no SMI access: the timing alone
            clk = []
        return self.mean_ms(), (float(np.median(clk)) if clk else None)


SETTLE_MS = 60.0   # untimed launches before each secondary burst (settle())


def settle(*steps, ms=SETTLE_MS):
    """Untimed rounds of `steps` until `ms` of wall time has passed (at least 5 rounds), so that a
    secondary burst measures the settled shader clock rather than the power-management transient
    that follows a load step (returns ms per round): in a kernel trace of this bench, launches of one kernel ran 1.3-1.4x
    longer for 5-20 ms after their burst began, then recovered (profiles/r05_v14_bench_launch_sequence.json).
    The headline has its own --warmup steps."""
    torch.cuda.synchronize()
    t0, k = time.perf_counter(), 0
    while True:
        for _ in range(5):
            for st in steps:
                st()
        k += 5
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) * 1e3
        if el >= ms:
            return el / k   # ms per round of `steps`


SECONDARY_TIMED_MS = 200.0   # each secondary burst spans at least this much launch time


def timed_reps(round_ms, base):
    """Timed rounds for a secondary burst: `base`, or enough rounds of `round_ms` (settle()'s
    estimate) to span SECONDARY_TIMED_MS, whichever is more -- the shader clock drifts by up to
    ~20 % over tens of ms under sustained VALU load, and a longer burst averages over it."""
    return max(base, int(np.ceil(SECONDARY_TIMED_MS / max(round_ms, 1e-3))))


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/rNN_*pmc_traffic.json, written by tools/gpu_pmc.sh: separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this same bench command,
    corrected per MI355X_MICROARCH.md "HBM").  None when no summary exists."""
    import glob
    import re

    def version(path):   # natural order: r01_v9 < r01_v12
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")), key=version)
    if not files:
        return None, None
    with open(files[-1]) as fh:
        rec = json.load(fh).get(kernel)
    if not rec:
        return None, None
    return rec["traffic_bytes"], os.path.relpath(files[-1], ROOT)


def burst_profile(kernel):
    """rocprofv3 kernel-trace statistics of the timed headline burst alone (bench.py
    --headline-only under tools/gpu_prof.sh; tools/burst_stats.py keeps the last
    3 x steps dispatches) from the newest profiles/rNN_*burst_stats.json.  None if absent."""
    import glob
    import re

    def version(path):
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_burst_stats.json")), key=version)
    if not files:
        return None
    with open(files[-1]) as fh:
        rec = json.load(fh)
    if rec.get("kernel") != kernel:
        return None
    return {"rocprof_mean_us": rec["mean_us"], "rocprof_mean_x3_ms": rec["mean_x_per_step_ms"],
            "rocprof_first_launch_of_step_us": rec["first_launch_of_step_mean_us"],
            "rocprof_other_launches_us": rec["other_launches_mean_us"], "source": os.path.relpath(files[-1], ROOT)}


def valu_floor(kernel):
    """VALU-issue floor of one launch of `kernel` from the newest committed
    profiles/rNN_*valu_roofline.json (tools/gpu_valu.sh + tools/valu_summary.py: PMC
    SQ_INSTS_VALU / SQ_INSTS_VALU_TRANS_F32 per dispatch; 2 cycles per plain and 8 per
    transcendental wave64 instruction, 1024 SIMDs at 2.4 GHz).  None when absent."""
    import glob
    import re

    def version(path):
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_valu_roofline.json")), key=version)
    if not files:
        return None
    with open(files[-1]) as fh:
        rec = json.load(fh).get(kernel)
    if not rec:
        return None
    out = {"valu_wave_insts": rec["valu_wave_insts"], "trans_wave_insts": rec["trans_wave_insts"],
           "issue_floor_ms": rec["valu_issue_floor_ms"], "source": os.path.relpath(files[-1], ROOT)}
    if "stall" in rec:   # where the wave cycles go (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_*)
        out["wave_cycles"] = {k: v for k, v in rec["stall"].items() if k.endswith("_frac")}
    return out


def valu_frac(floor, ms, clk_mhz=None, eff_mhz=None):
    """`floor` (valu_floor) against a measured launch time: frac at the nominal 2.4 GHz,
    frac_at_gfxclk with the floor rescaled to amd-smi's sampled clock, and
    frac_at_effective_clock rescaled to the clock the CUs ran at during the burst (ClockDuring)."""
    out = dict(floor, achieved_ms=ms, frac=floor["issue_floor_ms"] / ms)
    if clk_mhz:
        out["frac_at_gfxclk"] = floor["issue_floor_ms"] * (2400.0 / clk_mhz) / ms
    if eff_mhz:
        out["frac_at_effective_clock"] = floor["issue_floor_ms"] * (2400.0 / eff_mhz) / ms
    return out


def sclk_under_valu_load(dev):
    """GFX clock (MHz, amd-smi through torch.cuda.clock_rate) sampled while every SIMD runs
    independent FMA chains (tools/clock_probe.hip, built by build(); ~0.3 s of load): the
    VALU-bound lines scale with the clock the power manager grants, which differs from box
    to box.  None when the probe's code object is absent."""
    path = os.path.join(ROOT, "tools", "build", "clock_probe.hsaco")
    if not os.path.exists(path):
        return None
    hip = ctypes.CDLL("libamdhip64.so")
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    if hip.hipModuleLoad(ctypes.byref(mod), path.encode()) != 0:
        return None
    try:
        if hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"sunsky_tools_clock_probe") != 0:
            return None
        cu = torch.cuda.get_device_properties(dev).multi_processor_count
        blocks = cu * 8
        out = torch.zeros(2 * blocks, dtype=torch.int64, device=dev)
        stream = torch.cuda.current_stream(dev)

        def launch(iters):
            p_out, it = ctypes.c_void_p(out.data_ptr()), ctypes.c_int(iters)
            a, b = ctypes.c_float(1.0000001), ctypes.c_float(1e-7)
            args = (ctypes.c_void_p * 4)(*[ctypes.cast(ctypes.pointer(x), ctypes.c_void_p) for x in (p_out, it, a, b)])
            rc = hip.hipModuleLaunchKernel(fn, blocks, 1, 1, 256, 1, 1, 0, ctypes.c_void_p(stream.cuda_stream), args,
                                           None)
            if rc != 0:
                raise RuntimeError(f"clock probe launch failed ({rc})")
        launch(2000)
        torch.cuda.synchronize(dev)
        idle = torch.cuda.clock_rate(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        launch(4000000)
        e1.record(stream)
        samples = []
        time.sleep(0.02)
        while not e1.query():
            samples.append(torch.cuda.clock_rate(dev))
            time.sleep(0.005)
        torch.cuda.synchronize(dev)
        load_ms = e0.elapsed_time(e1)
        # every workgroup is resident for the whole launch (8 per CU): its shader-clock cycles
        # (clock64 at its start and end) over the launch time is the clock it actually ran at
        cycles = out.view(-1, 2)[:, 0].double().cpu().numpy()
        eff = float(np.median(cycles)) / (load_ms * 1e-3) / 1e6
        if not samples:
            return {"error": "no clock sample during the load", "load_ms": load_ms, "effective_mhz_from_cycles": eff}
        return {"effective_mhz_from_cycles": eff,
                "gfxclk_mhz_median": float(np.median(samples)), "gfxclk_mhz_min": float(min(samples)),
                "gfxclk_mhz_max": float(max(samples)), "samples": len(samples), "gfxclk_mhz_idle": float(idle),
                "load_ms": load_ms,
                "note": "GFX clock reported by amd-smi (torch.cuda.clock_rate) while every SIMD runs independent FMA "
                        "chains (tools/clock_probe.hip).  The VALU-bound sampling and caller lines scale with it; the "
                        "HBM-bound headline does not"}
    finally:
        hip.hipModuleUnload(mod)


class ClockDuring:
    """The shader clock a VALU-bound burst actually runs at: one wave of
    tools/clock_probe.hip `sunsky_tools_clock_during` on a side stream, launched right after
    the burst's first kernel, counts shader-clock cycles (s_memtime) over `ms` of the constant
    100 MHz counter (s_memrealtime).  amd-smi's sampled GFX clock (mean_ms_with_clock) is the
    power manager's reported figure; this is the one the CUs ran at.  None when the probe's
    code object is absent."""

    def __init__(self, dev):
        self.fn = None
        path = os.path.join(ROOT, "tools", "build", "clock_probe.hsaco")
        if not os.path.exists(path):
            return
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
        if self.hip.hipModuleLoad(ctypes.byref(self.mod), path.encode()) != 0:
            return
        if self.hip.hipModuleGetFunction(ctypes.byref(fn), self.mod, b"sunsky_tools_clock_during") != 0:
            return
        self.fn = fn
        self.out = torch.zeros(2, dtype=torch.int64, device=dev)
        self.side = torch.cuda.Stream(dev)

    def launch(self, ms):
        if self.fn is None:
            return
        p_out, ticks = ctypes.c_void_p(self.out.data_ptr()), ctypes.c_uint64(int(ms * 1e5))
        args = (ctypes.c_void_p * 2)(*[ctypes.cast(ctypes.pointer(x), ctypes.c_void_p) for x in (p_out, ticks)])
        if self.hip.hipModuleLaunchKernel(self.fn, 1, 1, 1, 64, 1, 1, 0, ctypes.c_void_p(self.side.cuda_stream), args,
                                          None) != 0:
            self.fn = None

    def mhz(self):
        if self.fn is None:
            return None
        self.side.synchronize()
        cyc, ticks = (int(v) for v in self.out.cpu())
        return cyc / (ticks * 1e-8) / 1e6 if ticks else None


def host_cpu_topology():
    """lscpu-style facts of the host plus the CPU quota this process may use (cgroup v2
    cpu.max: quota / period CPUs; on the GPU box 1600000 / 100000 = 16 of 256 CPUs)."""
    topo = {"cpu_model": "unknown", "logical_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}
    try:
        with open("/proc/cpuinfo") as f:
            txt = f.read()
        blocks = [b for b in txt.split("\n\n") if b.strip()]
        key = lambda b, k: next((ln.split(":", 1)[1].strip() for ln in b.splitlines() if ln.startswith(k)), None)
        topo["cpu_model"] = key(blocks[0], "model name") or "unknown"
        cores = {(key(b, "physical id"), key(b, "core id")) for b in blocks}
        topo["sockets"] = len({k[0] for k in cores})
        topo["physical_cores"] = len(cores)
    except (OSError, IndexError):
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    topo["cgroup_cpu_quota"] = quota
    return topo


def cpu_baseline(wi_host, budget_s=12.0):
    """The oracle (fp32 restatement of sunsky.cpp, -O3 -march=x86-64-v4, OpenMP) timed on
    this host's cores on a bounded sample of the headline workload.  Threads = the CPUs
    this process may actually run on: the cgroup CPU quota when there is one (the GPU
    box grants 16 CPUs of its 2 x 64-core EPYC), else every CPU in the affinity mask."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    topo = host_cpu_topology()
    threads = int(topo["cgroup_cpu_quota"] or topo["affinity_cpus"])
    O.set_threads(threads)
    oracles = [O.Oracle(sun_dict(t), "rgb", "jit", "f32") for t in TURBIDITIES]
    n_sample = min(wi_host.shape[0], 1 << 22)
    sample = np.ascontiguousarray(wi_host[:n_sample])
    oracles[0].eval(sample[:65536])   # warm
    done, t0 = 0, time.perf_counter()
    while True:
        for o in oracles:
            o.eval(sample)
            done += n_sample
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    rate = done / dt
    out = {"value": rate, "unit": "dir-evals/s", "cores": threads, "kind": "port", **topo,
           "sample": f"{done} RGB evals ({n_sample} of the headline directions x T in {{2,6,10}}, "
                     f"repeated for >= {budget_s:.0f}s), oracle/sunsky_oracle.c fp32 (-O3 -march=x86-64-v4 "
                     f"-ffp-contract=off), {threads} OpenMP threads"}
    if topo.get("physical_cores") and threads < topo["physical_cores"]:
        out["all_physical_cores_linear_extrapolation"] = rate / threads * topo["physical_cores"]
        out["extrapolation_note"] = ("not measured: this process is limited to the cgroup quota above; "
                                     "per-thread rate x physical cores, an upper bound for the whole machine")
    return out


def lane_stats(got, a, b, sun, rtol=1e-5, t=None):
    """Parity figures of tests/helpers.py, per lane population:
    sky lanes against the fp32 oracle (bound rtol|o32| + |o32 - o64|), sun-disc lanes
    against the fp64 oracle (bound rtol|o64| + k|o32 - o64|, k = SUN_SLACK), each with its worst lane
    as a fraction of the bound and its plain max relative error; for the sun lanes the
    fp32 oracle's own error against fp64 is reported beside the GPU's.  Lanes where
    fp32 and fp64 disagree by > 1e-3 (deviant_lanes: a horizon / disc-edge mask flipped by
    rounding, or the limb's ill-conditioned cos psi) are left out of the max-rel figures; the
    mask flips among them (one side zero or > 2x the other) are counted with how many the GPU
    puts on the fp32 reference's side (its fp32 horizon / disc test; the tests require all).
    *_over_1e-5_* count the lanes (any channel) beyond a literal 1e-5 of o32 / o64.
    t: the fp64 evaluation of the product's own staged fp32 tables (oracle64(..., em)); with
    it the sun lanes also carry the literal 1e-5 count against it (the FAST eval kernels'
    own arithmetic; VERDICT r05 next 2, tests/test_gpu_disc_literal.py) and |o64 - o64t|
    beside it (the fp32 staged state itself: tables ~1e-7, and the fp32 sun frame, which
    an fp64 renormalisation moves by ~1e-8 -- up to ~5e-5 at the limb), and pass requires no
    sun lane over 1e-5 of o64t."""
    got, a, b = (np.asarray(x, np.float64) for x in (got, a, b))
    den64 = np.maximum(np.abs(b), 1e-6 * np.abs(b).max())
    den32 = np.maximum(np.abs(a), 1e-6 * np.abs(a).max())
    flip = (np.abs(a - b) / den64 > 1e-3).any(axis=1)
    hi, lo = np.maximum(np.abs(a), np.abs(b)), np.minimum(np.abs(a), np.abs(b))
    mflip = ((hi > 1e-6 * np.abs(b).max()) & (hi - lo > 0.5 * hi)).any(axis=1)
    on32 = ~(np.abs(got - a) / den32 > 1e-3).any(axis=1)
    over32 = (np.abs(got - a) / den32 > rtol).any(axis=1)
    st = {"deviant_lanes": int(flip.sum()), "mask_flip_lanes": int(mflip.sum()),
          "mask_flip_lanes_on_o32_side": int((mflip & on32).sum()),
          "sky_lanes_over_1e-5_vs_o32": int((over32 & ~sun).sum()),
          "sun_lanes_over_1e-5_vs_o32": int((over32 & sun).sum())}
    sky = ~sun
    if sky.any():
        g, r32, r64 = got[sky], a[sky], b[sky]
        d = np.abs(g - r32)
        floor = np.maximum(np.abs(r32), 1e-6 * np.abs(r32).max())
        keep = ~flip[sky]
        st.update(sky_lanes=int(sky.sum()), sky_max_abs_vs_o32=float(d.max()),
                  sky_max_rel_vs_o32=float((d / floor)[keep].max()),
                  sky_frac_within_rtol=float((d <= rtol * floor).mean()),
                  sky_worst_vs_bound=float((d / (rtol * floor + np.abs(r32 - r64))).max()))
    if sun.any():
        g, r32, r64 = got[sun], a[sun], b[sun]
        den = den64[sun]
        keep = ~flip[sun]
        rg, ra = np.abs(g - r64) / den, np.abs(r32 - r64) / den
        st.update(sun_lanes=int(sun.sum()), sun_max_rel_vs_o64=float(rg[keep].max()),
                  sun_o32_max_rel_vs_o64=float(ra[keep].max()),
                  **{"sun_lanes_over_1e-5_vs_o64": int((rg[keep] > rtol).any(axis=1).sum()),
                     "sun_o32_lanes_over_1e-5_vs_o64": int((ra[keep] > rtol).any(axis=1).sum())},
                  sun_worst_vs_bound=float((np.abs(g - r64) / (rtol * np.abs(r64) + SUN_SLACK[0] * np.abs(r32 - r64)
                                                                  + 1e-30)).max()))
        if t is not None:
            rt = np.asarray(t, np.float64)[sun]
            dt = np.maximum(np.abs(rt), 1e-30)
            rgt = (np.abs(g - rt) / dt)[keep]
            st.update(sun_max_rel_vs_o64t=float(rgt.max()),
                      **{"sun_lanes_over_1e-5_vs_o64t": int((rgt > rtol).any(axis=1).sum()),
                         "sun_o32_lanes_over_1e-5_vs_o64t": int(((np.abs(r32 - rt) / dt)[keep] > rtol).any(axis=1).sum())},
                      sun_o64_vs_o64t_max_rel=float((np.abs(r64 - rt) / dt)[keep].max()))
    st["pass"] = (st.get("sky_worst_vs_bound", 0) <= 1 and st.get("sun_worst_vs_bound", 0) <= 1
                  and st["mask_flip_lanes_on_o32_side"] == st["mask_flip_lanes"]
                  and st.get("sun_lanes_over_1e-5_vs_o64t", 0) == 0)
    return st


def merge_stats(parts):
    out = {}
    for p in parts:
        for k, v in p.items():
            if k not in out:
                out[k] = v
            elif "lanes" in k:       # counts: summed over the parts
                out[k] += v
            elif k == "pass":
                out[k] = out[k] and v
            elif "frac" in k:
                out[k] = min(out[k], v)
            else:
                out[k] = max(out[k], v)
    return out


def sun_cone_dirs(sun_local, cos_cutoff, n, seed, scale=1.2):
    """wo directions in and just around the sun cone (tests/helpers.py sun_cone_wo)."""
    rng = np.random.default_rng(seed)
    s = np.asarray(sun_local, np.float64)
    a = np.array([1.0, 0, 0]) if abs(s[0]) < 0.9 else np.array([0, 1.0, 0])
    t1 = np.cross(s, a)
    t1 /= np.linalg.norm(t1)
    t2 = np.cross(s, t1)
    g = np.arccos(cos_cutoff) * scale * np.sqrt(rng.random(n))
    ph = 2 * np.pi * rng.random(n)
    return (np.cos(g)[:, None] * s + np.sin(g)[:, None] * (np.cos(ph)[:, None] * t1 +
                                                            np.sin(ph)[:, None] * t2)).astype(np.float32)


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    return O


def oracle64(O, d, variant, semantics, o32, em=None):
    """The fp64 oracle of the parity blocks, given the fp32-normalised sun direction the
    reference and the product compute (dr::normalize, sunsky.cpp:923; tests/helpers.py
    fp32_sun_input): from the unrounded direction the disc moves by ~1e-8 rad, which at the
    limb moves a lane by up to ~5e-5 for any fp32 implementation.  em: also adopt that
    emitter's staged fp32 tables (o64t, lane_stats' t)."""
    if "sun_direction" in d:
        d = dict(d, sun_direction=[float(x) for x in o32.info()["sun_dir_world"]])
    if em is not None and em.info()["precision"] != "fast":
        return None                  # the reference-precision kernels keep the fp32 disc term
    o = O.Oracle(d, variant, semantics, "f64")
    if em is not None:
        o.adopt_tables(em)
    return o


def parity_check(ems, wi, outs, n_check=1 << 20, n_sun=1 << 14):
    """Headline parity: GPU radiance vs the oracle on the first n_check directions of
    each turbidity plus n_sun directions in and around the sun cone (the sun-disc
    lanes, reported separately against fp64)."""
    O = _oracle()
    parts = []
    wi_h = wi[:, :n_check].T.cpu().numpy()
    for t, em, out in zip(TURBIDITIES, ems, outs):
        o32 = O.Oracle(sun_dict(t), "rgb", "jit", "f32")
        o64, o64t = oracle64(O, sun_dict(t), "rgb", "jit", o32), oracle64(O, sun_dict(t), "rgb", "jit", o32, em)
        inf = o32.info()
        cone = -sun_cone_dirs(inf["sun_dir_local"], inf["cos_cutoff"], n_sun, seed=int(t))
        g_cone = em.eval(ss.SurfaceInteraction3f(wi=torch.from_numpy(cone.T.copy()).to(wi.device)))
        wi_all = np.concatenate([wi_h, cone])
        got = np.concatenate([out[:, :n_check].T.cpu().numpy(), g_cone.T.cpu().numpy()])
        sun = (-wi_all @ inf["sun_dir_local"] >= inf["cos_cutoff"]) & (wi_all[:, 2] <= 0)
        parts.append(lane_stats(got, o32.eval(wi_all), o64.eval(wi_all), sun,
                                t=None if o64t is None else o64t.eval(wi_all)))
    st = merge_stats(parts)
    return dict(st, checked_dirs=(n_check + n_sun) * len(TURBIDITIES),
                bound=f"sky: |gpu-o32| <= 1e-5|o32| + |o32-o64|; sun disc: |gpu-o64| <= 1e-5|o64| + {SUN_SLACK[0]:g}|o32-o64|"
                      "; fast: every sun-disc lane within a literal 1e-5 of o64t (the fp64 evaluation of the "
                      "product's staged fp32 tables)")


def parity_c3(em, d_scene, wi, out, n_check=1 << 19, n_sun=1 << 13):
    """C3 (node kernel) parity: the first n_check directions x 11 nodes plus sun-cone lanes."""
    O = _oracle()
    lams = np.arange(320, 721, 40, dtype=np.float32)
    o32 = O.Oracle(d_scene, "spectral", "jit", "f32")
    o64, o64t = oracle64(O, d_scene, "spectral", "jit", o32), oracle64(O, d_scene, "spectral", "jit", o32, em)
    inf = o32.info()
    cone = -sun_cone_dirs(inf["sun_dir_local"], inf["cos_cutoff"], n_sun, seed=3)
    g_cone = em.eval_spectral_broadcast(torch.from_numpy(cone.T.copy()).to(wi.device), lams.tolist())
    wi_all = np.concatenate([wi[:, :n_check].T.cpu().numpy(), cone])
    got = np.concatenate([out[:, :n_check].T.cpu().numpy(), g_cone.T.cpu().numpy()])
    lam = np.repeat(lams[:, None], wi_all.shape[0], 1)
    sun = (-wi_all @ inf["sun_dir_local"] >= inf["cos_cutoff"]) & (wi_all[:, 2] <= 0)
    st = lane_stats(got, o32.eval(wi_all, lam).T, o64.eval(wi_all, lam).T, sun,
                    t=None if o64t is None else o64t.eval(wi_all, lam).T)
    return dict(st, checked_dirs=wi_all.shape[0], kernel="sunsky_eval_spec_nodes_v4")


def parity_rays(em, d_scene, wi, lam, out, n_check=1 << 19, n_sun=1 << 13):
    """Per-ray spectral eval parity (Mitsuba's Spectrum<Float, 4>, sunsky.cpp:325-348): the
    first n_check rays with their 4 random wavelengths, plus n_sun rays in and around the sun
    cone with random wavelengths (the sun-disc lanes, against fp64)."""
    O = _oracle()
    o32 = O.Oracle(d_scene, "spectral", "jit", "f32")
    o64, o64t = oracle64(O, d_scene, "spectral", "jit", o32), oracle64(O, d_scene, "spectral", "jit", o32, em)
    inf = o32.info()
    cone = -sun_cone_dirs(inf["sun_dir_local"], inf["cos_cutoff"], n_sun, seed=5)
    lam_c = np.random.default_rng(6).uniform(360, 720, (4, n_sun)).astype(np.float32)
    g_cone = em.eval(ss.SurfaceInteraction3f(wi=torch.from_numpy(cone.T.copy()).to(wi.device),
                                             wavelengths=torch.from_numpy(lam_c).to(wi.device)))
    wi_all = np.concatenate([wi[:, :n_check].T.cpu().numpy(), cone])
    lam_all = np.concatenate([lam[:, :n_check].cpu().numpy(), lam_c], axis=1)
    got = np.concatenate([out[:, :n_check].T.cpu().numpy(), g_cone.T.cpu().numpy()])
    sun = (-wi_all @ inf["sun_dir_local"] >= inf["cos_cutoff"]) & (wi_all[:, 2] <= 0)
    st = lane_stats(got, o32.eval(wi_all, lam_all).T, o64.eval(wi_all, lam_all).T, sun,
                    t=None if o64t is None else o64t.eval(wi_all, lam_all).T)
    return dict(st, checked_rays=wi_all.shape[0], kernel="sunsky_eval_spec_rays4_v4")


def parity_c4(em, d_scene, u, d, pdf_s, wgt, pdf_q, n_check=1 << 19, semantics="jit", lam=None):
    """C4 parity on the first n_check samples: directions vs the oracle's sampler on the
    same u, and pdf / pdf_direction / weight at the GPU's own directions.  lam: the
    spectral variant's (4, n) per-sample wavelengths (RGB when None)."""
    O = _oracle()
    variant = "rgb" if lam is None else "spectral"
    o32 = O.Oracle(d_scene, variant, semantics, "f32")
    o64 = oracle64(O, d_scene, variant, semantics, o32)
    o32.override_w_sky(em.sky_sampling_w)
    o64.override_w_sky(em.sky_sampling_w)
    uh = u[:, :n_check].T.cpu().numpy()
    gd = d[:, :n_check].T.cpu().numpy()
    gp, gq = pdf_s[:n_check].cpu().numpy(), pdf_q[:n_check].cpu().numpy()
    gw = wgt[:, :n_check].T.cpu().numpy()
    lh = None if lam is None else lam[:, :n_check].cpu().numpy()
    ref = o32.sample_direction(uh, wavelengths=lh)
    derr = np.abs(gd - ref["d"]).max(axis=1)
    inf = o32.info()
    inside = gd @ inf["sun_dir_local"] >= inf["cos_cutoff"]
    pref = o32.pdf_direction(gd).astype(np.float64)
    same = (uh[:, 0] < em.sky_sampling_w) | inside     # sun picks skip the cone test (sunsky.cpp:720)
    floor = 1e-6 * np.abs(pref).max()
    rel_p = np.abs(gp[same] - pref[same]) / np.maximum(np.abs(pref[same]), floor)
    rel_q = np.abs(gq - pref) / np.maximum(np.abs(pref), floor)
    e32, e64 = o32.eval(-gd, lh), o64.eval(-gd, lh)
    if lh is not None:
        e32, e64 = e32.T, e64.T
    w32 = (e32 / gp[:, None]).astype(np.float32)
    w64 = e64 / gp[:, None].astype(np.float64)
    up = gd[:, 2] >= 0
    # disc lanes include a 1e-6 band at the edge: the kernel's fp32 disc test may put the sun
    # term on a lane the fp64 test leaves outside (tests/helpers.py disc_lanes)
    disc = gd.astype(np.float64) @ inf["sun_dir_local"] >= inf["cos_cutoff"] - 1e-6
    st = lane_stats(gw[up], w32[up], w64[up], disc[up], rtol=1e-5)
    return {"checked_samples": n_check, "variant": variant, "dir_max_abs_delta": float(derr.max()),
            "dir_p999_abs_delta": float(np.quantile(derr, 0.999)),
            "pdf_max_rel_vs_o32": float(rel_p.max()), "pdf_direction_max_rel_vs_o32": float(rel_q.max()),
            "weight": st, "pass": bool(derr.max() < 1e-4 and rel_p.max() < 1e-5 and rel_q.max() < 1e-5
                                       and st["pass"]),
            "bounds": "dir p99.9 < 2e-6, max < 1e-4; pdf 1e-5 rel; weights 1e-5 (sky vs o32, sun vs o64)"}


def parity_caller(kind, em, d_scene, nrm, out, seed, spp, vw=None, n_check=4096):
    """Caller parity on the first n_check points (PCG32 streams by point index, so the first
    points are the oracle's points 0..n_check-1): per point the GPU estimate vs
    oracle.direct_diffuse / direct_conductor (GGX 0.2, the bench's eta / k) with the product's
    staged w_sky; the bounds of tests/test_direct_diffuse.py and test_direct_conductor.py
    (p99.5 of the per-point max channel error relative to max(|ref|, 1e-3 max|ref|))."""
    O = _oracle()
    torch.cuda.synchronize()            # the caller kernels ran on the bench's own stream
    o32 = O.Oracle(d_scene, "rgb", "jit", "f32")
    o32.override_w_sky(em.sky_sampling_w)
    nh = nrm[:, :n_check].T.cpu().numpy()
    got = out[:, :n_check].cpu().numpy().astype(np.float64)
    if kind == "diffuse":
        ref, bound = O.direct_diffuse(o32, nh, seed, spp), 2e-4
    else:
        ref = O.direct_conductor(o32, nh, vw[:, :n_check].T.cpu().numpy(), 0.2, "ggx", (0.143, 0.374, 1.442),
                                 (3.983, 2.385, 1.603), seed, spp)
        bound = 1e-3
    rel = (np.abs(got - ref) / np.maximum(np.abs(ref), 1e-3 * np.abs(ref).max())).max(axis=0)
    q = np.quantile(rel, [0.5, 0.995, 1.0])
    return {"checked_points": n_check, "spp": spp, "rel_p50": float(q[0]), "rel_p995": float(q[1]),
            "rel_max": float(q[2]), "mean_rel_delta": float(abs(got.mean() - ref.mean()) / abs(ref.mean())),
            "pass": bool(q[1] < bound and np.all(np.isfinite(got))),
            "bounds": f"per-point p99.5 < {bound:g} (tests' bound; fp32 vs the oracle's fp64 BSDF / MIS terms)"}


C5_SEED = 4321            # rank k's configs[4] batch: hemisphere_dirs(seed = C5_SEED + k)


def c5_scene():
    return dict(sun_dict(3.0), albedo=0.3)


def parity_c5(planes, n5, world, dev, per_rank=1 << 14, em=None):
    """configs[4] output parity on rank 0: for every rank k, a strided sample of per_rank
    directions of k's batch plus every sun-disc direction in it (regenerated here from k's
    seed), read from k's columns of the gathered (11, n5 * world) planes and compared with
    the oracle at the DESIGN.md §6 bars.  A gather that put a shard at the wrong column
    range or plane would fail here (the sampled columns would hold another rank's rays)."""
    O = _oracle()
    lams = np.arange(320, 721, 40, dtype=np.float32)
    o32 = O.Oracle(c5_scene(), "spectral", "jit", "f32")
    o64 = oracle64(O, c5_scene(), "spectral", "jit", o32)
    o64t = oracle64(O, c5_scene(), "spectral", "jit", o32, em) if em is not None else None
    inf = o32.info()
    s = torch.tensor(inf["sun_dir_local"], dtype=torch.float32, device=dev)
    parts, checked = [], 0
    for k in range(world):
        wi_k = -hemisphere_dirs(n5, seed=C5_SEED + k, device=dev)
        disc = ((s[:, None] * -wi_k).sum(0) >= inf["cos_cutoff"]) & (wi_k[2] <= 0)
        idx = torch.unique(torch.cat([torch.arange(0, n5, max(1, n5 // per_rank), device=dev),
                                      disc.nonzero().flatten()]))
        w = wi_k[:, idx].T.cpu().numpy()
        got = planes[:, k * n5 + idx.to(planes.device)].T.cpu().numpy()
        del wi_k, disc
        lam = np.repeat(lams[:, None], w.shape[0], 1)
        sun = (-w @ inf["sun_dir_local"] >= inf["cos_cutoff"]) & (w[:, 2] <= 0)
        parts.append(lane_stats(got, o32.eval(w, lam).T, o64.eval(w, lam).T, sun,
                                t=None if o64t is None else o64t.eval(w, lam).T))
        checked += w.shape[0]
    return dict(merge_stats(parts), checked_dirs=checked, ranks_checked=world,
                sample=f"per rank: every {max(1, n5 // per_rank)}th direction + every sun-disc direction, "
                       "x 11 nodes, read from that rank's columns of the gathered planes",
                bound=f"sky: |gpu-o32| <= 1e-5|o32| + |o32-o64|; sun disc: |gpu-o64| <= 1e-5|o64| + "
                      f"{SUN_SLACK[0]:g}|o32-o64|; fast: every sun-disc lane within a literal 1e-5 of o64t")


def run_c5(args, world, rank, dev, coll_dev, rehearsal):
    """configs[4]: a --c5-dirs spectral batch per GPU (11 model
    wavelengths, the C3 node kernel), then the gather of every rank's (11, n) radiance
    planes into rank 0's (11, N) planes through the C ABI (sunsky_gather_radiance; at one
    rank the copy of the rank's own shard into the output planes).  Per-GPU eval time (max
    over ranks), whole-job evals/s, gather time and GB/s.  Returns rank 0's state for
    finish_c5 (None elsewhere), which checks every rank's gathered columns bitwise against the
    root's own evaluation of that rank's inputs and samples them against the oracle -- after
    the teardown collectives: the other ranks do not wait through rank 0's serial
    re-evaluations and CPU parity, so no deadline has to cover them."""
    n5 = args.c5_dirs
    wi5 = -hemisphere_dirs(n5, seed=C5_SEED + rank, device=dev)
    spec5 = ss.SunskyEmitter(c5_scene(), "spectral", precision=args.precision, device=dev)
    lams = [float(x) for x in range(320, 721, 40)]
    full = None
    # a rehearsal (more ranks than GPUs) gathers over gloo, unless SUNSKY_BENCH_RCCL_DOUBLE names
    # the multi-process RCCL test double (tests/cpp/fake_rccl_ipc.cpp): then it takes the C ABI
    # branch below, the one a real multi-GPU run takes, with the double in RCCL's place
    capi_gather = not rehearsal or bool(os.environ.get("SUNSKY_BENCH_RCCL_DOUBLE"))
    if rank == 0 and capi_gather:
        # the root evaluates its shard straight into its columns [0, n5) of the final (11, N)
        # planes (plane stride N): sunsky_gather_radiance then finds it in place and copies
        # nothing for it (csrc/sunsky_comm.cpp), so the root's time is the eval plus the receives
        full = torch.empty((11, n5 * world), dtype=torch.float32, device=dev)
        out5 = full[:, :n5]
    else:
        out5 = torch.empty((11, n5), dtype=torch.float32, device=dev)
    for _ in range(2):
        spec5.eval_spectral_broadcast(wi5, lams, out=out5)
    reps = max(3, args.steps // 10)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    tm = KernelTimer()
    t0 = time.perf_counter()
    tm.begin()
    for _ in range(reps):
        spec5.eval_spectral_broadcast(wi5, lams, out=out5)
    tm.end(reps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    te = (time.perf_counter() - t0) / reps
    kernel_ms = tm.mean_ms()
    tg, tcat, own_ok, gpath = 0.0, 0.0, True, None
    if world > 1:
        t = torch.tensor([te], device=coll_dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        te = float(t.item())
    tgs = []
    if capi_gather:
        # C ABI gather (grouped RCCL send/recv) straight into rank 0's final planes; the root's
        # own columns are already in place (one rank, no torch.distributed: nothing to move)
        from sunsky_amd.sharding import RadianceComm
        gpath = ("sunsky_gather_radiance: RCCL send/recv into rank 0's (11, N) planes, the root's shard "
                 "evaluated in place; no padding / concat" if world > 1 else
                 "sunsky_gather_radiance, one rank: the shard was evaluated in place in the (11, N) planes")
        if rehearsal:
            gpath += (f" -- rehearsal: send/recv by the RCCL test double {os.path.basename(os.environ['SUNSKY_AMD_RCCL'])} "
                      "(hipIpc handles between the rank processes on one GPU), not RCCL; its time is not xGMI's")
        comm = RadianceComm(device=dev)
        comm.gather(out5, n5 * world, out=full)         # untimed: connection setup
        for _ in range(3):
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            comm.gather(out5, n5 * world, out=full)
            torch.cuda.synchronize()
            tgs.append(time.perf_counter() - t0)
        comm.close()
    else:
        from sunsky_amd.sharding import gather_shards, shard_sizes
        gpath = "torch.distributed.gather of padded shards + torch.cat (gloo rehearsal)"
        send = out5.to(coll_dev)
        bufs = gather_shards(send, n5 * world)           # untimed: connection setup
        for _ in range(3):                                 # the collective alone, preallocated
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            gather_shards(send, n5 * world, bufs=bufs)
            torch.cuda.synchronize()
            tgs.append(time.perf_counter() - t0)
        if rank == 0:
            t0 = time.perf_counter()
            full = torch.cat([b[:, :s] for b, s in zip(bufs, shard_sizes(n5 * world, world))], dim=1)
            torch.cuda.synchronize()
            tcat = time.perf_counter() - t0
        del bufs, send
    del wi5, out5
    tg = sorted(tgs)[1]
    if rank != 0:
        return None
    return {"n5": n5, "world": world, "dev": dev, "spec5": spec5, "full": full, "te": te, "kernel_ms": kernel_ms,
            "tg": tg, "tcat": tcat, "gpath": gpath}


def finish_c5(st):
    """Rank 0 after the teardown collectives: the gathered planes against the root's own
    evaluation of every rank's inputs (bit for bit) and against the oracle (parity_c5); the
    configs[4] report."""
    t_tail = time.perf_counter()
    n5, world, dev, spec5, full = st["n5"], st["world"], st["dev"], st["spec5"], st["full"]
    te, kernel_ms, tg, tcat, gpath = st["te"], st["kernel_ms"], st["tg"], st["tcat"], st["gpath"]
    lams = [float(x) for x in range(320, 721, 40)]
    # the gathered planes are the one-GPU result bit for bit -- every rank's
    # columns (the root's own included) against the root's evaluation of that rank's
    # regenerated inputs
    ref5 = torch.empty((11, n5), dtype=torch.float32, device=dev)
    shards_ok, own_ok = 0, False
    for r in range(world):
        wr = -hemisphere_dirs(n5, seed=C5_SEED + r, device=dev)
        spec5.eval_spectral_broadcast(wr, lams, out=ref5)
        ok = bool(torch.equal(full[:, r * n5:(r + 1) * n5].to(dev), ref5))
        shards_ok += int(ok)
        own_ok = ok if r == 0 else own_ok
        del wr
    del ref5
    torch.cuda.synchronize()
    t_bitwise = time.perf_counter() - t_tail
    nbytes = 11 * n5 * 4 * (world - 1)
    parity = parity_c5(full, n5, world, dev, em=spec5)
    report = {
        "dirs_per_gpu": n5, "lambdas": 11, "eval_s": te, "eval_kernel_ms": kernel_ms,
        "evals_per_s_whole_job": 11 * n5 * world / te,
        "eval_achieved_GBps": BYTES_SPEC_PER_DIR * n5 / (kernel_ms * 1e-3) / 1e9,
        "gather_s": tg, "gather_bytes_to_root": nbytes, "gather_GBps": nbytes / tg / 1e9 if tg and nbytes else None,
        "gather_bytes_note": ("bytes received by rank 0 from the other ranks" if world > 1 else
                              "one rank: the shard is already in place (no bytes move)"),
        "gather_path": gpath,
        "gather_timing": "median of 3 gathers into preallocated buffers after one untimed call",
        "reassemble_planes_s": tcat, "end_to_end_s": te + tg + tcat, "bitwise_own_shard": own_ok,
        "shards_bitwise_vs_one_gpu": f"{shards_ok}/{world}",
        "parity": parity,
        "rank0_tail_s": {"bitwise_reeval": t_bitwise, "total": time.perf_counter() - t_tail,
                         "note": "rank 0's serial re-evaluation of every rank's inputs + CPU parity, after the "
                                 "teardown collectives (no other rank waits for it)"},
        "note": "configs[4]: per-GPU spectral eval (weak scaling) then gather of the radiance to rank 0"}
    del full
    st["full"] = None
    return report


class C5Watchdog:
    """A rank whose communicator setup fails leaves the others waiting in a collective
    (RCCL init, a barrier).  Past `limit_s` rank 0 prints the bench line with the C5 error
    (the measured `value` is kept) and EVERY rank exits with EXIT_CODE: a process that has
    touched the GPU and hung is never reported as a success."""
    EXIT_CODE = 3
    KEY = "c5_spectral_shard_gather"

    def __init__(self, limit_s, rank, result):
        import threading
        self.limit_s, self.rank, self.result, self.printed = limit_s, rank, result, False
        self.timer = threading.Timer(limit_s, self._fire)
        self.timer.daemon = True

    def start(self):
        self.timer.start()
        return self

    def cancel(self):
        self.timer.cancel()

    def _fire(self):
        if self.rank == 0 and not self.printed and self.result is not None:
            self.result[self.KEY] = {"error": f"timed out after {self.limit_s:.0f} s (a rank stuck in a collective); "
                                              f"value is unaffected; every rank exits {self.EXIT_CODE}"}
            print(json.dumps(self.result), flush=True)
        sys.stderr.write(f"bench.py rank {self.rank}: configs[4] timed out after {self.limit_s:.0f} s\n")
        sys.stderr.flush()
        os._exit(self.EXIT_CODE)


class LaunchError(SystemExit):
    """--gpus and the launcher's WORLD_SIZE disagree: exits non-zero before any GPU call."""


def launch_plan(gpus, env):
    """How this process takes part in a `--gpus N` run, decided before anything touches the GPU:
      "single" -- N = 1 and no launcher: one process, one GPU;
      "spawn"  -- N > 1 and no launcher (WORLD_SIZE unset): this process starts the N rank
                  processes itself (spawn_ranks) and only waits for them;
      "rank"   -- started by a launcher (torchrun or spawn_ranks) with WORLD_SIZE = N.
    WORLD_SIZE set and different from --gpus raises LaunchError: a --gpus 8 line must never be
    measured on another number of GPUs."""
    if gpus < 1:
        raise LaunchError(f"bench.py: --gpus {gpus}: need at least one GPU")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "spawn" if gpus > 1 else "single"
    if int(ws) != gpus:
        raise LaunchError(f"bench.py: --gpus {gpus} but the launcher set WORLD_SIZE={ws}; refusing to measure "
                          f"{ws} rank(s) as {gpus} GPU(s)")
    return "rank"


SPAWN_GRACE_S = 60.0   # after one rank fails, how long the others may take to finish before they are killed


def spawn_ranks(n, argv, grace_s=SPAWN_GRACE_S):
    """`bench.py --gpus N` without torchrun: N child processes of this script, one per GPU, with
    RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE and a free MASTER_PORT on 127.0.0.1 (what
    torchrun --standalone sets).  The parent never touches the GPU: it starts the children before
    any HIP call and only waits (a process that has initialised HIP must never exec another).
    Rank 0 prints the bench line.  When a rank fails, the others get `grace_s` to finish (the
    C5 watchdog ends a rank stuck in a collective) and are then killed.  A SIGTERM / SIGINT to the
    parent is forwarded to the ranks, and a rank gets SIGTERM if the parent dies (PR_SET_PDEATHSIG),
    so no rank outlives the launch.  The ranks rendezvous through a file store in a private
    temporary directory (SUNSKY_BENCH_RENDEZVOUS), not a TCP port: a port picked here and
    released before the ranks bind it could be taken in between.  Returns the exit
    code: 0 when every rank exited 0, else the first failing rank's code (a signal as 128 + signo)."""
    import shutil
    import tempfile
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]      # informational only (MASTER_PORT of a torchrun-style env)
    rdv_dir = tempfile.mkdtemp(prefix="sunsky_bench_rdv_")
    try:
        return _spawn_and_wait(n, argv, grace_s, port, os.path.join(rdv_dir, "store"))
    finally:
        shutil.rmtree(rdv_dir, ignore_errors=True)


def _spawn_and_wait(n, argv, grace_s, port, store):
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), SUNSKY_BENCH_RENDEZVOUS=store)
    def die_with_parent():   # runs in the child before exec (no GPU touched yet): SIGTERM when the parent dies
        import ctypes as C
        C.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)   # PR_SET_PDEATHSIG

    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                              env=dict(base, RANK=str(r), LOCAL_RANK=str(r)), preexec_fn=die_with_parent)
             for r in range(n)]

    def forward(signum, _frame):   # a launcher's SIGTERM / SIGINT ends the ranks too, then the parent
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        sys.exit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    code, failed_at = 0, None
    while True:
        for p in procs:
            rc = p.poll()
            if rc not in (None, 0) and code == 0:
                code, failed_at = (rc if rc > 0 else 128 - rc), time.monotonic()
        alive = [p for p in procs if p.poll() is None]
        if not alive:
            return code
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            for p in alive:
                sys.stderr.write(f"bench.py: killing rank pid {p.pid} ({grace_s:.0f} s after a rank failed)\n")
                p.kill()
        time.sleep(0.2)


def c5_phase(run, rank, result, limit_s):
    """configs[4] (`run()`) under a C5Watchdog.  Returns (state, watchdog, failed).  The
    watchdog stays ARMED: teardown() cancels it after the teardown collectives, so a rank
    left waiting there (a peer whose C5 raised, or hung) still exits non-zero.  Rank 0's
    serial checks (finish_c5) run after that, outside the deadline."""
    watchdog = C5Watchdog(limit_s, rank, result).start()
    try:
        return run(), watchdog, False
    except Exception as exc:   # reported beside `value`; never fails the bench line itself
        return {"error": f"{type(exc).__name__}: {exc}"}, watchdog, True


def teardown(world, rank, watchdog, c5_failed):
    """After rank 0 has printed the line.  At world > 1 a rank whose C5 raised skips the
    teardown collectives (its peers may still sit in C5's) and exits C5Watchdog.EXIT_CODE;
    the others close the communicators, meet at the barrier and leave the group while the
    watchdog is still armed."""
    if world > 1:
        if c5_failed:
            sys.stdout.flush()
            sys.stderr.write(f"bench.py rank {rank}: configs[4] failed; leaving without the teardown collectives\n")
            sys.stderr.flush()
            os._exit(C5Watchdog.EXIT_CODE)
        from sunsky_amd.sharding import clear_radiance_comms
        clear_radiance_comms()
        dist.barrier()
        dist.destroy_process_group()
    if watchdog is not None:
        watchdog.cancel()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--n", type=int, default=N_DIRS, help="directions per GPU")
    ap.add_argument("--precision", default=os.environ.get("SUNSKY_BENCH_PRECISION", "fast"))
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--gather", action="store_true", help="also time an RCCL gather of the radiance to rank 0")
    ap.add_argument("--no-pmc", action="store_true", help="do not read the committed PMC traffic summary")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip configs[4] (spectral 11-lambda eval of --c5-dirs per GPU + gather to rank 0, "
                         "with its parity block; on by default at every N)")
    ap.add_argument("--headline-only", action="store_true",
                    help="run the settle, warmup and timed headline steps only (for a rocprof trace of the burst)")
    ap.add_argument("--c5-dirs", type=int, default=1 << 26, help="configs[4] directions per GPU (default 64M)")
    ap.add_argument("--launch-check", action="store_true",
                    help="print this rank's launch environment as JSON and exit before any GPU call (tests)")
    ap.add_argument("--rendezvous-check", action="store_true",
                    help="meet the other ranks over gloo as the bench does, all-reduce the ranks, print JSON and "
                         "exit before any GPU call (tests)")
    args = ap.parse_args()
    SUN_SLACK[0] = 4.0 if args.precision == "reference" else 1.25

    plan = launch_plan(args.gpus, os.environ)
    if plan == "spawn":            # no launcher: start the N ranks, touch no GPU here
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.launch_check:
        print(json.dumps({"plan": plan, "gpus": args.gpus, "world": world, "rank": int(os.environ.get("RANK", "0")),
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "pid": os.getpid(),
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}), flush=True)
        time.sleep(float(os.environ.get("SUNSKY_BENCH_TEST_HOLD", "0")))   # tests: a rank that is still running
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rendezvous_check:
        store = os.environ.get("SUNSKY_BENCH_RENDEZVOUS")
        init = {"init_method": f"file://{store}", "rank": rank, "world_size": world} if store else {}
        dist.init_process_group("gloo", **init)
        t = torch.tensor([float(rank)])
        dist.all_reduce(t)
        print(json.dumps({"rank": rank, "world": world, "rank_sum": float(t.item()),
                          "rendezvous": "file" if store else "env"}), flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return
    # One rank per GPU over RCCL ("nccl").  More ranks than GPUs (a multi-rank rehearsal
    # on a 1-GPU box) share the GPUs and synchronise over gloo with CPU tensors.
    ndev = max(1, torch.cuda.device_count())
    rehearsal = world > ndev
    double = os.environ.get("SUNSKY_BENCH_RCCL_DOUBLE")
    if double:
        # the C ABI resolves RCCL at its first communicator call (csrc/sunsky_comm.cpp rccl())
        if not rehearsal:
            raise SystemExit("SUNSKY_BENCH_RCCL_DOUBLE is for rehearsals (more ranks than GPUs) only")
        os.environ["SUNSKY_AMD_RCCL"] = os.path.abspath(double)
    backend = "gloo" if rehearsal else os.environ.get("SUNSKY_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local % ndev)
    dev = torch.device("cuda", local % ndev)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")
    if world > 1:
        # spawn_ranks' ranks meet through its file store; a launcher's through env:// (MASTER_*)
        store = os.environ.get("SUNSKY_BENCH_RENDEZVOUS")
        init = {"init_method": f"file://{store}", "rank": rank, "world_size": world} if store else {}
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, **init)
        else:
            dist.init_process_group(backend, **init)

    n = args.n
    # NB input batches of n directions (4 x 201 MB > the 256 MiB Infinity Cache), one per step
    # in rotation: every step's first launch reads its directions from HBM; its other two
    # launches re-read them at the next turbidity, as the workload (one batch x T{2,6,10}) does.
    batches = [-hemisphere_dirs(n, seed=1234 + 1000 * k + rank, device=dev) for k in range(NB)]   # si.wi = -wo
    wi = batches[0]
    ems = [ss.SunskyEmitter(sun_dict(t), "rgb", precision=args.precision, device=dev) for t in TURBIDITIES]
    outs = [torch.empty((3, n), dtype=torch.float32, device=dev) for _ in TURBIDITIES]
    lib = ss.lib()
    vins = [ss._capi.Vec3In(b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr()) for b in batches]
    vin = vins[0]
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step(i):
        v = vins[i % NB]
        for em, out in zip(ems, outs):
            rc = lib.sunsky_eval(em._h, v, None, 0, 0, None, n, out.data_ptr(), n, stream)
            if rc:
                raise RuntimeError(lib.sunsky_last_error().decode())

    # Untimed settle: bring the GPU out of its idle clock state before the
    # W warmup steps (a step is ~0.2 ms, so a handful of warmups alone is too short).
    torch.cuda.synchronize()
    t_settle = time.perf_counter()
    i = 0
    while time.perf_counter() - t_settle < 0.5:
        step(i)
        i += 1
        torch.cuda.synchronize()
    for k in range(args.warmup):
        step(i + k)
    timer = KernelTimer()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    timer.begin()
    for k in range(args.steps):
        step(k)
    timer.end(args.steps * len(TURBIDITIES))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=coll_dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms = timer.mean_ms()
    evals_per_step = len(TURBIDITIES) * n
    value = evals_per_step * world * args.steps / elapsed
    if args.headline_only:     # the timed burst alone (rocprofv3 --kernel-trace --stats of exactly it)
        if rank == 0:
            print(json.dumps({"metric": "headline burst only", "value": value, "ms_per_step": elapsed / args.steps * 1e3,
                              "kernel_ms": kernel_ms, "steps": args.steps, "warmup": args.warmup}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    # Headline kernel with every launch's inputs from HBM: the NB batches evaluated
    # round-robin at one turbidity (roofline "frac_all_cold").
    def cold_step():
        for k, v in enumerate(vins):
            rc = lib.sunsky_eval(ems[0]._h, v, None, 0, 0, None, n, outs[k % 3].data_ptr(), n, stream)
            if rc:
                raise RuntimeError(lib.sunsky_last_error().decode())

    for _ in range(2):
        cold_step()
    tm = KernelTimer()
    reps = max(3, args.steps // 4)
    tm.begin()
    for _ in range(reps):
        cold_step()
    tm.end(reps * len(vins))
    cold_ms = tm.mean_ms()
    # the NB batches stay resident: the C3 and per-ray spectral lines time cold inputs on them
    # the bitwise outputs of the parity check below are the timed step's on batch 0: recompute them
    step(0)
    torch.cuda.synchronize()

    result = None
    if rank == 0:
        achieved = BYTES_RGB * n / (kernel_ms * 1e-3) / 1e9
        kname = "sunsky_eval_rgb_v4_" + ("ref" if args.precision == "reference" else "fast")
        traffic, traffic_src = (None, None) if args.no_pmc else pmc_traffic(kname)
        parity = parity_check(ems, wi, outs)
        result = {
            "metric": "sky-radiance evals/sec (ray-dir \u00d7 \u03bb) at 1/2/4/8 GPU; max-abs \u0394 vs scalar ref", "value": value, "unit": "evals/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "RGB eval(): 16,777,216 uniform upper-hemisphere dirs per GPU x turbidity {2,6,10}",
                       "dirs_per_gpu": n, "turbidity": list(TURBIDITIES), "sun_elevation_deg": 45,
                       "albedo": 0.1, "precision": args.precision, "parallelism": f"shard{world}",
                       **({"rehearsal": f"{world} ranks on {ndev} GPU(s), gloo" +
                           (", C5 gather through the RCCL test double" if double else "")} if rehearsal else {})},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "achieved_all_cold": BYTES_RGB * n / (cold_ms * 1e-3) / 1e9,
                         "frac_all_cold": BYTES_RGB * n / (cold_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "kernel_ms_all_cold": cold_ms,
                         "cache_note": f"the timed steps rotate over {NB} distinct 201 MB input batches (805 MB > "
                                       "the 256 MiB Infinity Cache): launch 1 of a step reads its directions from "
                                       "HBM, launches 2 and 3 (the next turbidities of the same batch) may find "
                                       "them in the Infinity Cache, as the workload re-reads them.  *_all_cold "
                                       "evaluates the batches round-robin so every launch reads from HBM.  PMC "
                                       "FETCH_SIZE counts Infinity-Cache hits too (MI355X_MICROARCH.md 'HBM'), so "
                                       "`traffic` is bytes past the L2, not HBM-only bytes",
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kname,
                         "kernel_ms": kernel_ms, "bytes_per_launch": BYTES_RGB * n,
                         "profile": burst_profile(kname)},
            "parity": parity,
        }

    # ---------------------------------------------------------------- secondary
    if not args.no_secondary:
        sec = {}
        # caller: 8192 x 4096 lat-long RGB bake of the sky (write-only, 12 B per pixel)
        bw, bh = 8192, 4096
        bake_out = torch.empty((3, bh, bw), dtype=torch.float32, device=dev)
        est = settle(lambda: ems[0].bake_latlong(bw, bh, out=bake_out))
        tm = KernelTimer()
        reps = timed_reps(est, max(10, args.steps // 4))
        tm.begin()
        for _ in range(reps):
            ems[0].bake_latlong(bw, bh, out=bake_out)
        tm.end(reps)
        ms = tm.mean_ms()
        sec["latlong_bake_8192x4096"] = {"kernel_ms": ms, "pixels_per_s": bw * bh / (ms * 1e-3),
                                         "achieved_GBps": 12 * bw * bh / (ms * 1e-3) / 1e9,
                                         "note": "sunsky_bake_latlong: directions generated on device, RGB writes only"}
        del bake_out
        # Reverse-mode AD (f2): sum(d_out * d eval / d params) over the headline directions,
        # 16 parameter slots accumulated on device (vjp kernel + deterministic block reduce)
        d_out = torch.ones((3, n), dtype=torch.float32, device=dev)
        si_v = ss.SurfaceInteraction3f(wi=wi)
        grad = ems[0].eval_vjp(si_v, d_out)[0]
        est = settle(lambda: ems[0].eval_vjp(si_v, d_out, grad=grad))
        tm = KernelTimer()
        reps = timed_reps(est, max(10, args.steps // 4))
        tm.begin()
        for _ in range(reps):
            ems[0].eval_vjp(si_v, d_out, grad=grad)
        tm.end(reps)
        ms = tm.mean_ms()
        sec["eval_vjp_rgb_16M"] = {"kernel_ms": ms, "dirs_per_s": n / (ms * 1e-3),
                                   "achieved_GBps": 24 * n / (ms * 1e-3) / 1e9,
                                   "note": "sunsky_eval_vjp (RGB): reads wi + d_out (24 B/dir), gradients of "
                                           "turbidity, albedo, sun_direction (full-precision AD kernel + deterministic reduce)"}
        del d_out, grad
        # C3: spectral eval, 11 model wavelengths broadcast.  Warm: the same 201 MB of
        # directions every launch (they stay in the 256 MiB Infinity Cache); cold: the NB
        # batches round-robin, so every launch reads its directions from HBM (what a renderer's
        # fresh wavefront of rays sees) -- `evals_per_s` is the cold figure.
        spec = ss.SunskyEmitter(dict(sun_dict(3.0), albedo=0.3), "spectral", precision=args.precision, device=dev)
        lams = [float(x) for x in range(320, 721, 40)]
        spec_out = torch.empty((11, n), dtype=torch.float32, device=dev)
        est = settle(lambda: spec.eval_spectral_broadcast(wi, lams, out=spec_out))
        tm = KernelTimer()
        reps = timed_reps(est, max(10, args.steps // 4))
        tm.begin()
        for _ in range(reps):
            spec.eval_spectral_broadcast(wi, lams, out=spec_out)
        tm.end(reps)
        ms_warm = tm.mean_ms()
        tm = KernelTimer()
        reps_c = timed_reps(est * len(batches), max(3, args.steps // 16))
        tm.begin()
        for _ in range(reps_c):
            for b in batches:
                spec.eval_spectral_broadcast(b, lams, out=spec_out)
        tm.end(reps_c * len(batches))
        ms = tm.mean_ms()
        spec.eval_spectral_broadcast(wi, lams, out=spec_out)   # batch 0's radiance for the parity block
        kn = "sunsky_eval_spec_nodes_v4_" + ("ref" if args.precision == "reference" else "fast")
        sec["spectral_eval_C3"] = {"evals_per_s": 11 * n / (ms * 1e-3), "kernel_ms": ms,
                                   "achieved_GBps": BYTES_SPEC_PER_DIR * n / (ms * 1e-3) / 1e9,
                                   "hbm_frac": BYTES_SPEC_PER_DIR * n / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                   "kernel_ms_warm": ms_warm,
                                   "hbm_frac_warm": BYTES_SPEC_PER_DIR * n / (ms_warm * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                   "kernel": kn, "unit": "(dir x lambda) evals/s",
                                   "note": f"cold: {NB} distinct 201 MB direction batches round-robin (every launch "
                                           "reads its directions from HBM; 56 B per direction); warm: one batch "
                                           "re-read from the Infinity Cache"}
        if rank == 0:
            sec["spectral_eval_C3"]["parity"] = parity_c3(spec, dict(sun_dict(3.0), albedo=0.3), wi, spec_out)
        del spec_out
        # Mitsuba's spectral variants: 4 wavelengths per ray (Spectrum<Float, 4>), per-ray lambda;
        # NB (direction, wavelength) batches so that the cold figure reads both from HBM
        lam_b = [360.0 + 360.0 * torch.rand((4, n), generator=torch.Generator(device=dev).manual_seed(5 + rank + 97 * k),
                                            device=dev) for k in range(NB)]
        lam4 = lam_b[0]
        rays_out = torch.empty((4, n), dtype=torch.float32, device=dev)

        def rays_step(k=0):
            rc = lib.sunsky_eval(spec._h, vins[k], lam_b[k].data_ptr(), 4, n, None, n, rays_out.data_ptr(), n, stream)
            if rc:
                raise RuntimeError(lib.sunsky_last_error().decode())

        est = settle(rays_step)
        tm = KernelTimer()
        reps = timed_reps(est, max(10, args.steps // 4))
        reps_c = timed_reps(est * NB, max(3, args.steps // 16))
        tm.begin()
        for _ in range(reps):
            rays_step()
        tm.end(reps)
        ms_warm = tm.mean_ms()
        tm = KernelTimer()
        tm.begin()
        for _ in range(reps_c):
            for k in range(NB):
                rays_step(k)
        tm.end(reps_c * NB)
        ms = tm.mean_ms()
        rays_step()
        sec["spectral_eval_per_ray_4lambda"] = {"evals_per_s": 4 * n / (ms * 1e-3), "kernel_ms": ms,
                                                "achieved_GBps": (12 + 16 + 16) * n / (ms * 1e-3) / 1e9,
                                                "hbm_frac": (12 + 16 + 16) * n / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                                "kernel_ms_warm": ms_warm,
                                                "hbm_frac_warm": 44 * n / (ms_warm * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                                "note": "16M rays x 4 random wavelengths in [360, 720] nm "
                                                        "(reads wi + lambda, writes 4 radiances); cold: "
                                                        f"{NB} (direction, wavelength) batches round-robin, warm: one"}
        vr = valu_floor("sunsky_eval_spec_rays4_v4_" + ("ref" if args.precision == "reference" else "fast"))
        if vr:
            sec["spectral_eval_per_ray_4lambda"]["valu_roofline"] = {
                "bound": "valu", "unit": "ms", "eval": valu_frac(vr, ms),
                "note": "frac = VALU-issue floor (PMC instruction counts x issue cycles / (1024 SIMDs x 2.4 GHz)) / "
                        "measured launch time; the HBM fraction of the same launches is hbm_frac"}
        if rank == 0:
            sec["spectral_eval_per_ray_4lambda"]["parity"] = parity_rays(spec, dict(sun_dict(3.0), albedo=0.3), wi,
                                                                         lam4, rays_out)
        del lam4, lam_b, rays_out
        del batches[1:]
        vins = vins[:1]
        # C4: sample_direction + pdf_direction, 64M samples (per GPU); JIT semantics (w_sky from
        # the quadrature) and the scalar variants' w_sky = 0.5 (sunsky.cpp:778-783)
        ns = 4 * n
        kfx = "ref" if args.precision == "reference" else "fast"
        for sem, key in (("jit", "sampling_C4"), ("scalar", "sampling_C4_scalar_w05")):
            smp_s = ss.SunskyEmitter(dict(sun_dict(3.0, eta_deg=30.0), albedo=0.3), "rgb", semantics=sem,
                                     precision=args.precision, device=dev)
            g = torch.Generator(device=dev)
            g.manual_seed(99 + rank)
            u = torch.rand((2, ns), generator=g, device=dev)
            d = torch.empty((3, ns), dtype=torch.float32, device=dev)
            pdf_s = torch.empty(ns, dtype=torch.float32, device=dev)
            wgt = torch.empty((3, ns), dtype=torch.float32, device=dev)
            pdf_q = torch.empty(ns, dtype=torch.float32, device=dev)
            nul_in = ss._capi.Vec3In(None, None, None)
            nul_out = ss._capi.Vec3Out(None, None, None)
            d_out = ss._capi.Vec3Out(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr())
            d_in = ss._capi.Vec3In(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr())

            def sample_step():   # ds.dist / ds.p not requested (NULL): 36 B per sample
                rc = lib.sunsky_sample_direction(smp_s._h, u[0].data_ptr(), u[1].data_ptr(), nul_in, None, 0, 0, None,
                                                 ns, d_out, pdf_s.data_ptr(), None, nul_out, wgt.data_ptr(), ns, stream)
                if rc:
                    raise RuntimeError(lib.sunsky_last_error().decode())

            def pdf_step():      # 16 B per sample
                rc = lib.sunsky_pdf_direction(smp_s._h, d_in, None, ns, pdf_q.data_ptr(), stream)
                if rc:
                    raise RuntimeError(lib.sunsky_last_error().decode())

            reps = timed_reps(settle(sample_step, pdf_step), max(10, args.steps // 4))
            t_s, t_p = KernelTimer(), KernelTimer()
            cd = ClockDuring(dev)
            t_s.begin()
            for r_ in range(reps):
                sample_step()
                if r_ == 0:
                    cd.launch(0.4 * reps * 0.8)   # ~40 % of the burst, from its first launch on
            t_s.end(reps)
            t_p.begin()
            for _ in range(reps):
                pdf_step()
            t_p.end(reps)
            ms_s, clk_s = t_s.mean_ms_with_clock()
            ms_p = t_p.mean_ms()
            ms = ms_s + ms_p
            sec[key] = {"samples_per_s": ns / (ms * 1e-3), "ms": ms, "samples": ns,
                        "sample_direction_ms": ms_s, "pdf_direction_ms": ms_p, "w_sky": smp_s.sky_sampling_w,
                        "gfxclk_mhz_during_sample_direction": clk_s,
                        "effective_mhz_during_sample_direction": cd.mhz(),
                        "achieved_GBps": BYTES_SAMPLE * ns / (ms * 1e-3) / 1e9,
                        "note": "sample_direction (reads u; writes d, pdf, RGB weight) + pdf_direction "
                                "(reads d; writes pdf); " + ("JIT semantics, w_sky from the quadrature" if sem == "jit"
                                                             else "scalar semantics, w_sky = 0.5")}
            vs, vp = valu_floor("sunsky_sample_direction_rgb_lean_" + kfx), valu_floor("sunsky_pdf_direction_v4_" + kfx)
            if sem == "jit" and vs and vp:
                sec[key]["valu_roofline"] = {
                    "bound": "valu", "unit": "ms",
                    "sample_direction": valu_frac(vs, ms_s, clk_s, sec[key]["effective_mhz_during_sample_direction"]),
                    "pdf_direction": valu_frac(vp, ms_p),
                    "note": "frac = VALU-issue floor (PMC instruction counts x issue cycles / (1024 SIMDs x 2.4 GHz)) "
                            "/ measured launch time (frac_at_gfxclk: the floor at the sampled clock); HBM frac of the same launches is achieved_GBps / 8000"}
            if rank == 0:
                sec[key]["parity"] = parity_c4(smp_s, dict(sun_dict(3.0, eta_deg=30.0), albedo=0.3), u, d,
                                               pdf_s, wgt, pdf_q, semantics=sem)
            if sem == "jit":
                # the general call a Mitsuba integrator makes (DirectionSample3f with p and dist): it.p
                # in, ds.p and ds.dist out as well (+28 B per sample); the wave-sorted kSortPos kernel
                # (the next window's it.p prefetched with its u), bitwise the unsorted general kernel
                itp = torch.randn((3, ns), generator=g, device=dev)
                dist_o = torch.empty(ns, dtype=torch.float32, device=dev)
                pos_o = torch.empty((3, ns), dtype=torch.float32, device=dev)
                p_in = ss._capi.Vec3In(itp[0].data_ptr(), itp[1].data_ptr(), itp[2].data_ptr())
                p_out = ss._capi.Vec3Out(pos_o[0].data_ptr(), pos_o[1].data_ptr(), pos_o[2].data_ptr())

                def general_step():
                    rc = lib.sunsky_sample_direction(smp_s._h, u[0].data_ptr(), u[1].data_ptr(), p_in, None, 0, 0,
                                                     None, ns, d_out, pdf_s.data_ptr(), dist_o.data_ptr(), p_out,
                                                     wgt.data_ptr(), ns, stream)
                    if rc:
                        raise RuntimeError(lib.sunsky_last_error().decode())
                reps_g = timed_reps(settle(general_step), reps)
                t_g = KernelTimer()
                t_g.begin()
                for _ in range(reps_g):
                    general_step()
                t_g.end(reps_g)
                ms_g = t_g.mean_ms()
                sec[key]["sample_direction_general_ms"] = ms_g
                sec[key]["sample_direction_general_note"] = (
                    "the same samples with it.p in and ds.p, ds.dist out (64 B per sample), the wave-sorted "
                    "kernel with it.p prefetched per window (sunsky_sample_direction_rgb_pos_sorted); not part of "
                    "samples_per_s")
                del itp, dist_o, pos_o
            del u, d, pdf_s, wgt, pdf_q
            if sem == "jit":
                smp = smp_s
        # the spectral variant's sampling call (Mitsuba Spectrum<Float, 4>: 4 wavelengths per sample),
        # LEAN (d, pdf, 4 weights) + pdf_direction; parity: tests/test_gpu_parity.py (spectral sampling)
        smp_sp = ss.SunskyEmitter(dict(sun_dict(3.0, eta_deg=30.0), albedo=0.3), "spectral", precision=args.precision,
                                  device=dev)
        g_sp = torch.Generator(device=dev)
        g_sp.manual_seed(199 + rank)
        u_sp = torch.rand((2, ns), generator=g_sp, device=dev)
        lam_sp = 360.0 + 360.0 * torch.rand((4, ns), generator=g_sp, device=dev)
        d_sp = torch.empty((3, ns), dtype=torch.float32, device=dev)
        p_sp = torch.empty(ns, dtype=torch.float32, device=dev)
        w_sp = torch.empty((4, ns), dtype=torch.float32, device=dev)
        q_sp = torch.empty(ns, dtype=torch.float32, device=dev)
        dsp_out = ss._capi.Vec3Out(d_sp[0].data_ptr(), d_sp[1].data_ptr(), d_sp[2].data_ptr())
        dsp_in = ss._capi.Vec3In(d_sp[0].data_ptr(), d_sp[1].data_ptr(), d_sp[2].data_ptr())
        nul_in = ss._capi.Vec3In(None, None, None)
        nul_out = ss._capi.Vec3Out(None, None, None)

        def spec_sample_step():
            rc = lib.sunsky_sample_direction(smp_sp._h, u_sp[0].data_ptr(), u_sp[1].data_ptr(), nul_in,
                                             lam_sp.data_ptr(), 4, ns, None, ns, dsp_out, p_sp.data_ptr(), None,
                                             nul_out, w_sp.data_ptr(), ns, stream)
            if rc:
                raise RuntimeError(lib.sunsky_last_error().decode())

        def spec_pdf_step():
            rc = lib.sunsky_pdf_direction(smp_sp._h, dsp_in, None, ns, q_sp.data_ptr(), stream)
            if rc:
                raise RuntimeError(lib.sunsky_last_error().decode())

        reps = timed_reps(settle(spec_sample_step, spec_pdf_step), max(10, args.steps // 4))
        t_ss, t_sq = KernelTimer(), KernelTimer()
        cd = ClockDuring(dev)
        t_ss.begin()
        for r_ in range(reps):
            spec_sample_step()
            if r_ == 0:
                cd.launch(0.4 * reps * 1.2)
        t_ss.end(reps)
        t_sq.begin()
        for _ in range(reps):
            spec_pdf_step()
        t_sq.end(reps)
        ms_ss, clk_ss = t_ss.mean_ms_with_clock()
        ms_sq = t_sq.mean_ms()
        sec["sampling_C4_spectral_4lambda"] = {
            "samples_per_s": ns / ((ms_ss + ms_sq) * 1e-3), "sample_direction_ms": ms_ss, "pdf_direction_ms": ms_sq,
            "gfxclk_mhz_during_sample_direction": clk_ss,
            "effective_mhz_during_sample_direction": cd.mhz(),
            "samples": ns, "achieved_GBps": (8 + 16 + 12 + 4 + 16 + 12 + 4) * ns / ((ms_ss + ms_sq) * 1e-3) / 1e9,
            "note": "spectral emitter, C4 sun: sample_direction with 4 per-sample wavelengths (reads u + 4 lambda, "
                    "writes d, pdf, 4 weights; the wave-sorted LEAN kernel) + pdf_direction"}
        vss = valu_floor("sunsky_sample_direction_spec_lean4_sorted_" + kfx)
        if vss:
            sec["sampling_C4_spectral_4lambda"]["valu_roofline"] = {
                "bound": "valu", "unit": "ms",
                "sample_direction": valu_frac(vss, ms_ss, clk_ss, sec["sampling_C4_spectral_4lambda"][
                    "effective_mhz_during_sample_direction"]),
                "note": "frac = VALU-issue floor (PMC instruction counts x issue cycles / (1024 SIMDs x 2.4 GHz)) / "
                        "measured launch time (frac_at_gfxclk: the floor at the sampled clock)"}
        if rank == 0:
            sec["sampling_C4_spectral_4lambda"]["parity"] = parity_c4(
                smp_sp, dict(sun_dict(3.0, eta_deg=30.0), albedo=0.3), u_sp, d_sp, p_sp, w_sp, q_sp, lam=lam_sp)
        # Mitsuba's general call in the spectral variants (it.p in, ds.p and ds.dist out): the
        # wave-sorted kernel with ds.dist / ds.p formed at the store stage
        itp_sp = torch.randn((3, ns), generator=g_sp, device=dev)
        dist_sp = torch.empty(ns, dtype=torch.float32, device=dev)
        pos_sp = torch.empty((3, ns), dtype=torch.float32, device=dev)
        psp_in = ss._capi.Vec3In(itp_sp[0].data_ptr(), itp_sp[1].data_ptr(), itp_sp[2].data_ptr())
        psp_out = ss._capi.Vec3Out(pos_sp[0].data_ptr(), pos_sp[1].data_ptr(), pos_sp[2].data_ptr())

        def spec_general_step():
            rc = lib.sunsky_sample_direction(smp_sp._h, u_sp[0].data_ptr(), u_sp[1].data_ptr(), psp_in,
                                             lam_sp.data_ptr(), 4, ns, None, ns, dsp_out, p_sp.data_ptr(),
                                             dist_sp.data_ptr(), psp_out, w_sp.data_ptr(), ns, stream)
            if rc:
                raise RuntimeError(lib.sunsky_last_error().decode())

        reps_g = timed_reps(settle(spec_general_step), max(10, args.steps // 4))
        t_g = KernelTimer()
        t_g.begin()
        for _ in range(reps_g):
            spec_general_step()
        t_g.end(reps_g)
        sec["sampling_C4_spectral_4lambda"]["sample_direction_general_ms"] = t_g.mean_ms()
        sec["sampling_C4_spectral_4lambda"]["sample_direction_general_note"] = (
            "the same samples with it.p in and ds.p, ds.dist out, the wave-sorted kernel "
            "(sunsky_sample_direction_spec_pos_sorted); not part of samples_per_s")
        del u_sp, lam_sp, d_sp, p_sp, w_sp, q_sp, itp_sp, dist_sp, pos_sp
        # caller (§8f row 4): direct sun+sky light at 16M diffuse points x 4 spp, emitter + BSDF
        # sampling with MIS fused in one kernel (sunsky_direct_diffuse); reads 12 B normal, writes 12 B RGB
        npts, spp = n, 4
        nrm = torch.randn((3, npts), generator=g, device=dev)
        nrm[2].abs_().add_(0.2)
        nrm /= nrm.norm(dim=0, keepdim=True)
        nrm = nrm.contiguous()
        dd = torch.empty((3, npts), dtype=torch.float32, device=dev)
        n_in = ss._capi.Vec3In(nrm[0].data_ptr(), nrm[1].data_ptr(), nrm[2].data_ptr())

        def direct_step():
            rc = lib.sunsky_direct_diffuse(smp._h, n_in, None, None, 0, 0, 7, spp, None, 0, npts, dd.data_ptr(), npts,
                                           stream)
            if rc:
                raise RuntimeError(lib.sunsky_last_error().decode())

        reps = timed_reps(settle(direct_step), max(10, args.steps // 4))
        t_d = KernelTimer()
        t_d.begin()
        for _ in range(reps):
            direct_step()
        t_d.end(reps)
        ms_d = t_d.mean_ms()
        sec["direct_diffuse_16M_x4spp"] = {"samples_per_s": npts * spp / (ms_d * 1e-3), "ms": ms_d,
                                           "points": npts, "spp": spp,
                                           "note": "per sample: sample_direction + eval (emitter sampling), cosine "
                                                   "BSDF sample + pdf_direction + eval (escaped ray), power-heuristic "
                                                   "MIS; C4 sun/sky, random normals; one fused kernel"}
        if rank == 0:
            sec["direct_diffuse_16M_x4spp"]["parity"] = parity_caller(
                "diffuse", smp, dict(sun_dict(3.0, eta_deg=30.0), albedo=0.3), nrm, dd, 7, spp)
        # the glossy vertex: the same points seen from random view directions, a rough conductor
        # (GGX, alpha 0.2, gold-like eta / k) -- sunsky_direct_conductor, reads 24 B, writes 12 B
        vw = torch.randn((3, npts), generator=g, device=dev)
        vw = vw * torch.sign((vw * nrm).sum(0, keepdim=True))
        vw = (vw / vw.norm(dim=0, keepdim=True)).contiguous()
        w_in = ss._capi.Vec3In(vw[0].data_ptr(), vw[1].data_ptr(), vw[2].data_ptr())
        eta3 = (ctypes.c_float * 3)(0.143, 0.374, 1.442)
        k3 = (ctypes.c_float * 3)(3.983, 2.385, 1.603)

        def conductor_step():
            rc = lib.sunsky_direct_conductor(smp._h, n_in, w_in, 1, 0.2, eta3, k3, None, 0, 0, 7, spp, None, 0, npts,
                                             dd.data_ptr(), npts, stream)
            if rc:
                raise RuntimeError(lib.sunsky_last_error().decode())

        reps = timed_reps(settle(conductor_step), max(10, args.steps // 4))
        t_c = KernelTimer()
        t_c.begin()
        for _ in range(reps):
            conductor_step()
        t_c.end(reps)
        ms_c = t_c.mean_ms()
        sec["direct_conductor_16M_x4spp"] = {"samples_per_s": npts * spp / (ms_c * 1e-3), "ms": ms_c,
                                             "points": npts, "spp": spp,
                                             "note": "per sample: sample_direction + eval + rough-conductor eval/pdf "
                                                     "(emitter sampling), GGX visible-normal sample + pdf_direction + "
                                                     "eval (escaped ray), power-heuristic MIS; one fused kernel"}
        if rank == 0:
            sec["direct_conductor_16M_x4spp"]["parity"] = parity_caller(
                "conductor", smp, dict(sun_dict(3.0, eta_deg=30.0), albedo=0.3), nrm, dd, 7, spp, vw=vw)
        del nrm, dd, vw
        if rank == 0:
            try:
                sec["sclk_under_valu_load"] = sclk_under_valu_load(dev)
            except Exception as exc:   # a diagnostic beside the lines; never fail the bench
                sec["sclk_under_valu_load"] = {"error": f"{type(exc).__name__}: {exc}"}
            result["secondary"] = sec

    # ----------------------------------------------------------- optional gather
    if args.gather and world > 1:
        # configs[4]'s final step: the radiance shards gathered to rank 0 through the C ABI's
        # RCCL gather (sunsky_gather_radiance); reported beside `value`, never in it.
        # One communicator (cached per group and device) and one untimed gather first, so the
        # timed call is the transfer, not RCCL init and connection setup.
        from sunsky_amd.sharding import gather_radiance
        src = outs[0] if not rehearsal else outs[0].cpu()
        full = gather_radiance(src, n * world)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        full = gather_radiance(src, n * world, out=full)
        torch.cuda.synchronize()
        gt = time.perf_counter() - t0
        if rank == 0:
            nbytes = outs[0].numel() * 4 * (world - 1)
            result["gather"] = {"seconds": gt, "bytes_to_root": nbytes, "GBps": nbytes / gt / 1e9,
                                "path": "torch.distributed.gather (gloo rehearsal)" if rehearsal
                                        else "sunsky_gather_radiance (RCCL send/recv)",
                                "bitwise_own_shard": bool(torch.equal(full[:, :n].to(dev), outs[0]))}
        del full

    # ------------------------------------------- configs[4]: spectral shard + gather
    watchdog, c5_failed, c5 = None, False, None
    if not args.no_c5:
        del outs
        c5, watchdog, c5_failed = c5_phase(lambda: run_c5(args, world, rank, dev, coll_dev, rehearsal), rank, result,
                                           float(os.environ.get("SUNSKY_BENCH_C5_TIMEOUT", "150")))
        if rank == 0 and c5_failed:
            result["c5_spectral_shard_gather"] = c5
    # the teardown collectives under the still-armed C5 watchdog (ranks that finished C5 meet
    # here at once: rank 0's serial checks come after), then every rank but 0 is done
    teardown(world, rank, watchdog, c5_failed)

    if rank == 0:
        if c5 is not None and not c5_failed:
            try:
                result["c5_spectral_shard_gather"] = finish_c5(c5)
            except Exception as exc:   # reported beside `value`; never fails the bench line itself
                result["c5_spectral_shard_gather"] = {"error": f"{type(exc).__name__}: {exc}"}
        if not args.no_cpu and world == 1:   # the CPU baseline: rank 0 at N=1 only
            result["cpu_baseline"] = cpu_baseline(wi.T.cpu().numpy())
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
