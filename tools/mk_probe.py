#!/usr/bin/env python3
"""Probe builds of the product kernels, made OUTSIDE the product source.

The shipped `mitsuba3-sunsky_amd/csrc/sunsky_kernels.hip` holds no probe code.  A probe
(cost ablation, compute-only build, layout experiment) is a list of textual edits applied
here to a copy of it in tools/build/, which is then compiled to tools/build/probe_<name>.hsaco
for tools/gpu_ab.sh / kbench.  An edit whose anchor is missing fails loudly, so a probe
never silently measures the unmodified product.  Probes whose anchors a later change removed
are dropped from the table (their A/B logs stay in profiles/, their edits in git history).

usage: python tools/mk_probe.py <name> [--src FILE]   (tools/Makefile: make build/probe_<name>.hsaco)
"""
import argparse
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "mitsuba3-sunsky_amd", "csrc")

# name -> [(anchor, replacement)]: each anchor must occur exactly once in the product source
PROBES = {
    # compute-only: every global store suppressed (kept live by an impossible compare), for
    # the roofline splits of DESIGN.md §3
    "nostore": [
        ("__device__ __forceinline__ void store_vec(float* p, size_t i, const float v[VEC]) {\n",
         "__device__ __forceinline__ void store_vec(float* p, size_t i, const float v[VEC]) {\n"
         "    if (v[0] != -1234.5f) return;\n"),
        ("__device__ __forceinline__ void store_nt(float v, float* p) {\n",
         "__device__ __forceinline__ void store_nt(float v, float* p) {\n"
         "    if (v != -1234.5f) return;\n"),
    ],
    # the general RGB call (kSortPos) in windows of 3 / 2 x 64 samples
    "pos_r3": [("SS_SAMPLE_DIRECTION_SORTED(sunsky_sample_direction_rgb_pos_sorted_fast, true, SS_SORT_R, kSortPos)",
                "SS_SAMPLE_DIRECTION_SORTED(sunsky_sample_direction_rgb_pos_sorted_fast, true, 3, kSortPos)")],
    "pos_r2": [("SS_SAMPLE_DIRECTION_SORTED(sunsky_sample_direction_rgb_pos_sorted_fast, true, SS_SORT_R, kSortPos)",
                "SS_SAMPLE_DIRECTION_SORTED(sunsky_sample_direction_rgb_pos_sorted_fast, true, 2, kSortPos)")],
    # pdf_direction with the node kernel's contiguous span per workgroup instead of its grid-stride loop
    "pdf_span": [("""    const float3_ sn = mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]);
    const size_t nvec = n / VEC;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
""", """    const float3_ sn = mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]);
    const size_t nvec = n / VEC;
    const size_t lanes_ = (size_t)gridDim.x * blockDim.x, G_ = (nvec + lanes_ - 1) / lanes_;
    for (size_t g_ = 0; g_ < G_; ++g_) {
        const size_t v = ((size_t)blockIdx.x * G_ + g_) * blockDim.x + threadIdx.x;
        if (v >= nvec) break;
""")],
    # cost split of the general RGB call (kSortPos): no it.p loads (it.p = 0) / no ds.dist, ds.p stores
    "pos_noload": [("""                npx[r] = in ? px[i] : 0.f;
                npy[r] = in ? py[i] : 0.f;
                npz[r] = in ? pz[i] : 0.f;
""", """                npx[r] = 0.f * (float)in;
                npy[r] = 0.f;
                npz[r] = 0.f;
""")],
    # the spectral general call with it.p prefetched one window ahead (as the RGB kSortPos) instead
    # of read at the store stage: +3 R VGPRs over the passes
    "spec_pos_prefetch": [
        ("""    float na[R], nb[R], nl[4][R];""",
         """    float na[R], nb[R], nl[4][R];
    float npx[POS ? R : 1], npy[POS ? R : 1], npz[POS ? R : 1];"""),
        ("""            for (int k = 0; k < 4; ++k) nl[k][r] = i < n ? lam[(size_t)k * lstride + i] : 500.f;""",
         """            for (int k = 0; k < 4; ++k) nl[k][r] = i < n ? lam[(size_t)k * lstride + i] : 500.f;
            if constexpr (POS) {
                const bool in = px && i < n;
                npx[r] = in ? px[i] : 0.f;
                npy[r] = in ? py[i] : 0.f;
                npz[r] = in ? pz[i] : 0.f;
            }"""),
        ("""        const size_t base = w * W;
        int slot[R], nsky = 0;
        {
            float a[R], b[R], l[4][R];""",
         """        const size_t base = w * W;
        int slot[R], nsky = 0;
        float qpx[POS ? R : 1], qpy[POS ? R : 1], qpz[POS ? R : 1];
        if constexpr (POS) {
#pragma unroll
            for (int r = 0; r < R; ++r) { qpx[r] = npx[r]; qpy[r] = npy[r]; qpz[r] = npz[r]; }
        }
        {
            float a[R], b[R], l[4][R];"""),
        ("""                    const float3_ itp = px ? mk3(px[i], py[i], pz[i]) : mk3(0.f, 0.f, 0.f);""",
         """                    const float3_ itp = mk3(qpx[POS ? r : 0], qpy[POS ? r : 0], qpz[POS ? r : 0]);"""),
    ],
    # the spectral sorted passes specialised by class (as the RGB kernel's KIND 1 / 2 passes)
    "spec_kind_passes": [
        ("""            sample_one_spec4<FAST>(K, S, Y[0][q], Y[1][q], l4, inv_w, inv_w_sun, o);""",
         """            if (p * 64 + 64 <= nsky) sample_one_spec4<FAST, 1>(K, S, Y[0][q], Y[1][q], l4, inv_w, inv_w_sun, o);
            else if (p * 64 >= nsky) sample_one_spec4<FAST, 2>(K, S, Y[0][q], Y[1][q], l4, inv_w, inv_w_sun, o);
            else sample_one_spec4<FAST, 0>(K, S, Y[0][q], Y[1][q], l4, inv_w, inv_w_sun, o);"""),
    ],
    # pdf_direction with the next grid-stride step's directions loaded before this step's work
    "pdf_prefetch": [
        ("""    const float3_ sn = mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]);
    const size_t nvec = n / VEC;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        const size_t i = v * VEC;
        float x[VEC], y[VEC], z[VEC];
        bool m[VEC];
        load_dirs<VEC>(dx, dy, dz, active, i, x, y, z, m);""",
         """    const float3_ sn = mk3(K.sun_n[0], K.sun_n[1], K.sun_n[2]);
    const size_t nvec = n / VEC;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    float nx[VEC], ny[VEC], nz[VEC];
    bool nm[VEC];
    const size_t v0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v0 < nvec) load_dirs<VEC>(dx, dy, dz, active, v0 * VEC, nx, ny, nz, nm);
    for (size_t v = v0; v < nvec; v += stride) {
        const size_t i = v * VEC;
        float x[VEC], y[VEC], z[VEC];
        bool m[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) { x[j] = nx[j]; y[j] = ny[j]; z[j] = nz[j]; m[j] = nm[j]; }
        if (v + stride < nvec) load_dirs<VEC>(dx, dy, dz, active, (v + stride) * VEC, nx, ny, nz, nm);"""),
    ],
    # the general RGB call (kSortPos) with the hoisted sun rows, held to 4 waves/SIMD
    "pos_hoist": [
        ("""    constexpr bool kHoist = MODE == kSortLean;""", """    constexpr bool kHoist = MODE != kSortFull;"""),
        ("""#ifndef SS_RGB_SORTED_ATTR   // probe builds (tools/build) set occupancy attributes here
#define SS_RGB_SORTED_ATTR
""", """#ifndef SS_RGB_SORTED_ATTR   // probe builds (tools/build) set occupancy attributes here
#define SS_RGB_SORTED_ATTR __attribute__((amdgpu_waves_per_eu(4)))
"""),
    ],
    # the RGB eval in span_steps form (measured 4 % slower at 16M; the product keeps grid-stride)
    "rgb_span": [("""                                              float* __restrict__ out, size_t ostride) {
    const size_t nvec = n / VEC;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        const size_t i = v * VEC;
        float x[VEC], y[VEC], z[VEC], r[VEC], g[VEC], b[VEC];""", """                                              float* __restrict__ out, size_t ostride) {
    const size_t nvec = n / VEC, G = span_steps(nvec);
    for (size_t gs = 0; gs < G; ++gs) {
        const size_t v = ((size_t)blockIdx.x * G + gs) * blockDim.x + threadIdx.x;
        if (v >= nvec) break;
        const size_t i = v * VEC;
        float x[VEC], y[VEC], z[VEC], r[VEC], g[VEC], b[VEC];""")],
}


def make_source(name, src_path):
    text = open(src_path).read()
    for anchor, repl in PROBES[name]:
        if text.count(anchor) != 1:
            sys.exit(f"mk_probe: probe '{name}': anchor found {text.count(anchor)} times (want 1):\n{anchor}")
        text = text.replace(anchor, repl)
    return text


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name", choices=sorted(PROBES))
    ap.add_argument("--src", default=os.path.join(CSRC, "sunsky_kernels.hip"))
    ap.add_argument("--general", action="store_true", help="the general-to_world code object (default: identity)")
    args = ap.parse_args()
    build = os.path.join(HERE, "build")
    os.makedirs(build, exist_ok=True)
    hip = os.path.join(build, f"probe_{args.name}.hip")
    with open(hip, "w") as fh:
        fh.write(make_source(args.name, args.src))
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--genco",
           "-I" + CSRC, "-I" + os.path.join(ROOT, "include"), "-o", os.path.join(build, f"probe_{args.name}.hsaco"), hip]
    if not args.general:
        cmd.insert(5, "-DSS_XFORM_IDENTITY")
    subprocess.check_call(cmd)


if __name__ == "__main__":
    main()
