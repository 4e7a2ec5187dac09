#!/usr/bin/env python3
"""Probe builds of the product kernels, made OUTSIDE the product source.

The shipped `mitsuba3-sunsky_amd/csrc/sunsky_kernels.hip` holds no probe code.  A probe
(cost ablation, compute-only build, layout experiment) is a list of textual edits applied
here to a copy of it in tools/build/, which is then compiled to tools/build/probe_<name>.hsaco
for tools/gpu_ab.sh / kbench.  An edit whose anchor is missing fails loudly, so a probe
never silently measures the unmodified product.

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
    # round 6 fp64 disc fix-up variants (A/B against the product build)
    "rgb_jbarrier": [("""            float o[3];
            if constexpr (FAST) {
                bool h;""", """            float o[3];
            if constexpr (FAST) {
                __builtin_amdgcn_sched_barrier(0);
                bool h;""")],
    "rays_nofix": [("""        // FAST: the disc lanes again with the fp64 disc term (fixup_rgb_disc)
        if (FAST && any_sun) {""", """        if (false && FAST && any_sun) {""")],
    "rays_noinline_fix": [("""        // FAST: the disc lanes again with the fp64 disc term (fixup_rgb_disc)
        if (FAST && any_sun) {
#pragma unroll 1
            for (int j = 0; j < VEC; ++j) {""", """        // FAST: the disc lanes again with the fp64 disc term (fixup_rgb_disc)
        if (FAST && any_sun) fixup_rays_noinline<VEC, FAST, NEG>(K, chans, wx, wy, wz, active, i, lam, lstride, nlam, out, ostride);
        if (false) {
#pragma unroll 1
            for (int j = 0; j < VEC; ++j) {"""),
        ("""// ======================================================================
// eval(): spectral with per-ray wavelengths (Mitsuba Spectrum<Float, k>):""", """template <int VEC, bool FAST, bool NEG>
__device__ __noinline__ void fixup_rays_noinline(const SunskyKArgs& K, const typename ChanSel<FAST>::T* chans,
    const float* __restrict__ wx, const float* __restrict__ wy, const float* __restrict__ wz, const uint8_t* __restrict__ active,
    size_t i, const float* __restrict__ lam, size_t lstride, int nlam, float* __restrict__ out, size_t ostride) {
#pragma unroll 1
    for (int j = 0; j < VEC; ++j) {
        const size_t q = i + j;
        const DirTerms tj = refetch_terms<NEG>(K, wx, wy, wz, active, q);
        if (!tj.hit_sun) continue;
        const SunDisc64 d = sun_disc64(K, tj.wx, tj.wy, tj.cos_theta);
#pragma unroll 1
        for (int k = 0; k < nlam; ++k)
            out[(size_t)k * ostride + q] = eval_spec_one_flat<FAST, kSunF64>(K, chans, K.sun_table, K.sun_ld, tj,
                                                                              lam[(size_t)k * lstride + q], &d, &K);
    }
}

// ======================================================================
// eval(): spectral with per-ray wavelengths (Mitsuba Spectrum<Float, k>):""")],
    # the node kernel with the next step's directions loaded before this
    # step's 11 stores (vmcnt counts loads and stores in order: a load issued after the stores
    # waits for them); rolled channel loop / unrolled with a scheduling barrier per channel
    "nodes_pf": [('    const size_t nvec = n / VEC, G = span_steps(nvec);\n    {\n#pragma unroll 1\n      for (size_t g = 0; g < G; ++g) {', '    const size_t nvec = n / VEC, G = span_steps(nvec);\n    {\n      float px_[VEC], py_[VEC], pz_[VEC];\n      bool pm_[VEC];\n#pragma unroll 1\n      for (size_t g = 0; g < G; ++g) {'), ("        const size_t v = ((size_t)blockIdx.x * G + g) * blockDim.x + threadIdx.x;\n        if (v >= nvec) break;\n        const size_t i = v * VEC;\n        float x[VEC], y[VEC], z[VEC];\n        bool m[VEC];\n        load_dirs<VEC>(wx, wy, wz, active, i, x, y, z, m);\n        DirTerms t[VEC];\n        bool any_sun = false;\n#pragma unroll\n        for (int j = 0; j < VEC; ++j) {\n            t[j] = dir_terms<FAST>(K, to_local(K, flip3<NEG>(x[j], y[j], z[j])), m[j]);\n            any_sun |= t[j].hit_sun;\n        }\n        if (any_sun) {\n#pragma unroll\n            for (int j = 0; j < VEC; ++j) add_sun_terms<FAST>(K, t[j]);\n        }\n        // Rolled: one channel's constants (LDS broadcast reads) live at a time;\n        // unrolling lets the compiler hoist all 110 out of the ray loop (184 VGPRs).\n#pragma unroll 1\n        for (int c = 0; c < kNbWavelengths; ++c) {", "        const size_t v = ((size_t)blockIdx.x * G + g) * blockDim.x + threadIdx.x;\n        if (v >= nvec) break;\n        const size_t i = v * VEC;\n        if (g == 0) load_dirs<VEC>(wx, wy, wz, active, i, px_, py_, pz_, pm_);\n        DirTerms t[VEC];\n        bool any_sun = false;\n#pragma unroll\n        for (int j = 0; j < VEC; ++j) {\n            t[j] = dir_terms<FAST>(K, to_local(K, flip3<NEG>(px_[j], py_[j], pz_[j])), pm_[j]);\n            any_sun |= t[j].hit_sun;\n        }\n        // the next step's directions, issued before this step's stores\n        if (g + 1 < G && v + blockDim.x < nvec) load_dirs<VEC>(wx, wy, wz, active, i + (size_t)blockDim.x * VEC, px_, py_, pz_, pm_);\n        if (any_sun) {\n#pragma unroll\n            for (int j = 0; j < VEC; ++j) add_sun_terms<FAST>(K, t[j]);\n        }\n#pragma unroll 1\n        for (int c = 0; c < kNbWavelengths; ++c) {\n            ")],
    "nodes_pf_unroll": [('    const size_t nvec = n / VEC, G = span_steps(nvec);\n    {\n#pragma unroll 1\n      for (size_t g = 0; g < G; ++g) {', '    const size_t nvec = n / VEC, G = span_steps(nvec);\n    {\n      float px_[VEC], py_[VEC], pz_[VEC];\n      bool pm_[VEC];\n#pragma unroll 1\n      for (size_t g = 0; g < G; ++g) {'), ("        const size_t v = ((size_t)blockIdx.x * G + g) * blockDim.x + threadIdx.x;\n        if (v >= nvec) break;\n        const size_t i = v * VEC;\n        float x[VEC], y[VEC], z[VEC];\n        bool m[VEC];\n        load_dirs<VEC>(wx, wy, wz, active, i, x, y, z, m);\n        DirTerms t[VEC];\n        bool any_sun = false;\n#pragma unroll\n        for (int j = 0; j < VEC; ++j) {\n            t[j] = dir_terms<FAST>(K, to_local(K, flip3<NEG>(x[j], y[j], z[j])), m[j]);\n            any_sun |= t[j].hit_sun;\n        }\n        if (any_sun) {\n#pragma unroll\n            for (int j = 0; j < VEC; ++j) add_sun_terms<FAST>(K, t[j]);\n        }\n        // Rolled: one channel's constants (LDS broadcast reads) live at a time;\n        // unrolling lets the compiler hoist all 110 out of the ray loop (184 VGPRs).\n#pragma unroll 1\n        for (int c = 0; c < kNbWavelengths; ++c) {", "        const size_t v = ((size_t)blockIdx.x * G + g) * blockDim.x + threadIdx.x;\n        if (v >= nvec) break;\n        const size_t i = v * VEC;\n        if (g == 0) load_dirs<VEC>(wx, wy, wz, active, i, px_, py_, pz_, pm_);\n        DirTerms t[VEC];\n        bool any_sun = false;\n#pragma unroll\n        for (int j = 0; j < VEC; ++j) {\n            t[j] = dir_terms<FAST>(K, to_local(K, flip3<NEG>(px_[j], py_[j], pz_[j])), pm_[j]);\n            any_sun |= t[j].hit_sun;\n        }\n        // the next step's directions, issued before this step's stores\n        if (g + 1 < G && v + blockDim.x < nvec) load_dirs<VEC>(wx, wy, wz, active, i + (size_t)blockDim.x * VEC, px_, py_, pz_, pm_);\n        if (any_sun) {\n#pragma unroll\n            for (int j = 0; j < VEC; ++j) add_sun_terms<FAST>(K, t[j]);\n        }\n#pragma unroll \n        for (int c = 0; c < kNbWavelengths; ++c) {\n            __builtin_amdgcn_sched_barrier(0);")],
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
    "pos_nostore": [("""                    if (dist) store_nt(dd, dist + i);
                    if (opx) { store_nt(fmaf(d.x, dd, itp.x), opx + i); store_nt(fmaf(d.y, dd, itp.y), opy + i); store_nt(fmaf(d.z, dd, itp.z), opz + i); }
""", """                    const float s_ = fmaf(d.x, dd, itp.x) + fmaf(d.y, dd, itp.y) + fmaf(d.z, dd, itp.z);
                    if (dist && s_ == -1234.5f) store_nt(dd, dist + i);
""")],
    # the wave-sorted RGB kernels' un-sort stores as plain stores: ds.dist / ds.p only, or all planes
    "sorted_plain_pos": [("""                    if (dist) store_nt(dd, dist + i);
                    if (opx) { store_nt(fmaf(d.x, dd, itp.x), opx + i); store_nt(fmaf(d.y, dd, itp.y), opy + i); store_nt(fmaf(d.z, dd, itp.z), opz + i); }
                }""", """                    if (dist) dist[i] = dd;
                    if (opx) { opx[i] = fmaf(d.x, dd, itp.x); opy[i] = fmaf(d.y, dd, itp.y); opz[i] = fmaf(d.z, dd, itp.z); }
                }""")],
    "sorted_plain_all": [("""                    if (dist) store_nt(dd, dist + i);
                    if (opx) { store_nt(fmaf(d.x, dd, itp.x), opx + i); store_nt(fmaf(d.y, dd, itp.y), opy + i); store_nt(fmaf(d.z, dd, itp.z), opz + i); }
                }""", """                    if (dist) dist[i] = dd;
                    if (opx) { opx[i] = fmaf(d.x, dd, itp.x); opy[i] = fmaf(d.y, dd, itp.y); opz[i] = fmaf(d.z, dd, itp.z); }
                }"""),
        ("""                for (int k = 0; k < 7; ++k) store_nt(Y[k][slot[r]], planes[k] + i);""",
         """                for (int k = 0; k < 7; ++k) planes[k][i] = Y[k][slot[r]];""")],
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
    # the per-ray spectral eval's and the node kernel's grid-stride loops (the split before round 5), for A/B
    "evals_gridstride": [
        ("""    if constexpr (NL > 0) nlam = NL;
    const size_t nvec = n / VEC, G = span_steps(nvec);
    for (size_t gs = 0; gs < G; ++gs) {
        const size_t v = ((size_t)blockIdx.x * G + gs) * blockDim.x + threadIdx.x;
        if (v >= nvec) break;""",
         """    if constexpr (NL > 0) nlam = NL;
    const size_t nvec = n / VEC;
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (size_t)gridDim.x * blockDim.x) {"""),
        ("""    const size_t nvec = n / VEC, G = span_steps(nvec);
    {
#pragma unroll 1
      for (size_t g = 0; g < G; ++g) {
        const size_t v = ((size_t)blockIdx.x * G + g) * blockDim.x + threadIdx.x;
        if (v >= nvec) break;""",
         """    const size_t nvec = n / VEC;
    {
#pragma unroll 1
      for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (size_t)gridDim.x * blockDim.x) {"""),
    ],
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
