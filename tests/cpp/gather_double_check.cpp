// gather_double_check.cpp -- test program for tests/test_gpu_gather.py: the multi-rank
// branch of sunsky_gather_radiance (grouped ncclSend / ncclRecv, csrc/sunsky_comm.cpp)
// on ONE GPU.  The program links the RCCL test double (build/librccl.so.1, soname
// librccl.so.1), so the product's dlopen("librccl.so.1") finds the double already loaded;
// no product code changes.  Ranks are communicators of one unique id in this process,
// each gathering from its own stream.  Cases: 2-4 ranks, ragged and empty shards
// (shard_range's 4-aligned split), RGB eval (3 planes) and the C3 node kernel (11
// planes), root first or last, ranks calling in either order.  Exit 0 when every
// gathered buffer equals the whole batch evaluated alone, bit for bit.
//
// `gather_double_check c5 [world] [rays_per_rank]` runs the same check at configs[4]'s
// sizes instead: `world` ranks (default 4) of 64M rays x the 11 node wavelengths each,
// so the root's planes hold more than 2^31 floats (plane offsets past 2^33 bytes), every
// shard evaluated on its own and gathered, then compared with the whole batch bitwise.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "sunsky_amd.h"

#define CK(x)                                                                              \
    do {                                                                                   \
        int rc_ = (x);                                                                     \
        if (rc_ != SUNSKY_OK) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, sunsky_last_error());                      \
            return 2;                                                                      \
        }                                                                                  \
    } while (0)
#define HK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            return 3;                                                                      \
        }                                                                                  \
    } while (0)

// sunsky_amd/sharding.py shard_range: balanced, 4-aligned starts
static void shard_range(size_t n, int r, int world, size_t* a, size_t* b) {
    const size_t blocks = (n + 3) / 4, per = blocks / world, extra = blocks % world;
    const size_t b0 = r * per + std::min<size_t>(r, extra), b1 = b0 + per + ((size_t)r < extra ? 1 : 0);
    *a = std::min(n, b0 * 4);
    *b = std::min(n, b1 * 4);
}

static int eval(sunsky_emitter* em, bool spec, const float* wi, size_t stride, size_t n, float* out) {
    static const float nodes[11] = {320, 360, 400, 440, 480, 520, 560, 600, 640, 680, 720};
    sunsky_vec3_in v{wi, wi + stride, wi + 2 * stride};
    if (spec) CK(sunsky_eval_spectral_broadcast(em, v, nodes, 11, nullptr, n, out, n, nullptr));
    else CK(sunsky_eval(em, v, nullptr, 0, 0, nullptr, n, out, n, nullptr));
    return 0;
}

extern "C" int ncclGetUniqueId(void*);   // the double this program links

// configs[4] sizes: world x n rays x 11 planes; the inputs tile a host pattern whose length
// (2^20 + 7) divides neither a shard nor a plane, so a shard landing at a wrong column range
// or plane would not compare equal by accident
static int run_c5(sunsky_emitter* spec, int world, size_t per) {
    const int np = 11;
    const size_t n = per * world, tile = (1u << 20) + 7;
    std::printf("c5: %d ranks x %zu rays x %d planes: root planes %zu floats (%.2f GB)\n", world, per, np,
                (size_t)np * n, np * n * 4.0 / 1e9);
    std::fflush(stdout);
    std::vector<float> h(3 * tile);
    std::mt19937 rng(4321);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    for (size_t i = 0; i < tile; ++i) {
        float ct = U(rng), ph = 6.2831853f * U(rng), st = std::sqrt(std::max(0.f, 1 - ct * ct));
        h[i] = -st * std::cos(ph); h[tile + i] = -st * std::sin(ph); h[2 * tile + i] = -ct;
    }
    float *wi, *whole, *out;
    HK(hipMalloc(&wi, 3 * n * 4));
    for (int c = 0; c < 3; ++c)
        for (size_t i = 0; i < n; i += tile)
            HK(hipMemcpy(wi + c * n + i, h.data() + c * tile, std::min(tile, n - i) * 4, hipMemcpyHostToDevice));
    HK(hipMalloc(&whole, (size_t)np * n * 4));
    if (eval(spec, true, wi, n, n, whole)) return 2;
    unsigned char uid[SUNSKY_COMM_ID_BYTES];
    CK(sunsky_comm_get_unique_id(uid));
    std::vector<sunsky_comm*> comms(world);
    for (int r = 0; r < world; ++r) CK(sunsky_comm_create(uid, world, r, &comms[r]));
    std::vector<hipStream_t> streams(world);
    for (auto& st : streams) HK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::vector<float*> shard(world, nullptr);
    std::vector<size_t> counts(world);
    for (int r = 0; r < world; ++r) {
        size_t a, b;
        shard_range(n, r, world, &a, &b);
        counts[r] = b - a;
        float* wr;
        HK(hipMalloc(&wr, 3 * counts[r] * 4));
        for (int c = 0; c < 3; ++c)
            HK(hipMemcpy(wr + c * counts[r], wi + c * n + a, counts[r] * 4, hipMemcpyDeviceToDevice));
        HK(hipMalloc(&shard[r], (size_t)np * counts[r] * 4));
        if (eval(spec, true, wr, counts[r], counts[r], shard[r])) return 2;
        HK(hipDeviceSynchronize());
        (void)hipFree(wr);
    }
    (void)hipFree(wi);
    HK(hipMalloc(&out, (size_t)np * n * 4));
    const size_t chunk = (size_t)1 << 26;   // compared through pinned 256 MB host buffers
    float *ha, *hb;
    HK(hipHostMalloc(&ha, chunk * 4, 0));
    HK(hipHostMalloc(&hb, chunk * 4, 0));
    int cases = 0;
    for (int root : {0, world - 1}) {
        const bool rev = root != 0;
        HK(hipMemset(out, 0xff, (size_t)np * n * 4));   // NaN
        HK(hipDeviceSynchronize());
        for (int k = 0; k < world; ++k) {
            const int r = rev ? world - 1 - k : k;
            CK(sunsky_gather_radiance(comms[r], root, shard[r], counts[r], np, counts.data(), r == root ? out : nullptr,
                                      r == root ? n : 0, streams[r]));
        }
        HK(hipDeviceSynchronize());
        for (size_t off = 0; off < (size_t)np * n; off += chunk) {
            const size_t m = std::min(chunk, (size_t)np * n - off);
            HK(hipMemcpy(ha, out + off, m * 4, hipMemcpyDeviceToHost));
            HK(hipMemcpy(hb, whole + off, m * 4, hipMemcpyDeviceToHost));
            if (std::memcmp(ha, hb, m * 4) != 0) {
                std::printf("c5 root %d: gathered planes differ in floats [%zu, %zu) (plane %zu)\n", root, off,
                            off + m, off / n);
                return 1;
            }
        }
        ++cases;
        std::printf("c5 case %d: world %d root %d order %d: %zu floats bitwise equal\n", cases, world, root, (int)rev,
                    (size_t)np * n);
        std::fflush(stdout);
    }
    (void)hipHostFree(ha); (void)hipHostFree(hb);
    for (float* x : shard) (void)hipFree(x);
    (void)hipFree(out); (void)hipFree(whole);
    for (auto* c : comms) sunsky_comm_destroy(c);
    for (auto st : streams) (void)hipStreamDestroy(st);
    std::printf("c5 gather through the RCCL double: %d cases bitwise equal\n", cases);
    return 0;
}

int main(int argc, char** argv) {
    const bool c5 = argc > 1 && std::strcmp(argv[1], "c5") == 0;
    // the product resolves RCCL with dlopen("librccl.so.1"): it must get the double, or the
    // communicators below would be real ones waiting for ranks that never come
    void* so = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!so || dlsym(so, "ncclGetUniqueId") != (void*)&ncclGetUniqueId) {
        std::fprintf(stderr, "librccl.so.1 does not resolve to the test double (see tests/cpp/Makefile)\n");
        return 4;
    }
    sunsky_props* p = nullptr;
    CK(sunsky_props_create(&p));
    const float th = (float)(45.0 * M_PI / 180.0);
    CK(sunsky_props_set_float(p, "turbidity", 3.0));
    CK(sunsky_props_set_float(p, "albedo", 0.3));
    CK(sunsky_props_set_vector3(p, "sun_direction", std::sin(th), 0.f, std::cos(th)));
    sunsky_emitter *rgb = nullptr, *spec = nullptr;
    CK(sunsky_emitter_create(p, 0, 0, nullptr, &rgb));
    CK(sunsky_props_set_float(p, "turbidity", 3.0));   // properties are queried once per create
    CK(sunsky_props_set_float(p, "albedo", 0.3));
    CK(sunsky_props_set_vector3(p, "sun_direction", std::sin(th), 0.f, std::cos(th)));
    CK(sunsky_emitter_create(p, 1, 0, nullptr, &spec));
    std::printf("emitters staged\n");
    std::fflush(stdout);
    if (c5) {
        const int world = argc > 2 ? std::atoi(argv[2]) : 4;
        const size_t per = argc > 3 ? (size_t)std::atoll(argv[3]) : ((size_t)1 << 26);
        if (world < 2 || world > 16 || per < 4 || per % 4) {
            std::fprintf(stderr, "c5: world in [2, 16], rays per rank a positive multiple of 4\n");
            return 5;
        }
        const int rc = run_c5(spec, world, per);
        sunsky_emitter_destroy(rgb);
        sunsky_emitter_destroy(spec);
        sunsky_props_destroy(p);
        return rc;
    }
    int cases = 0;
    for (int world = 2; world <= 4; ++world) {
        unsigned char uid[SUNSKY_COMM_ID_BYTES];
        CK(sunsky_comm_get_unique_id(uid));
        std::vector<sunsky_comm*> comms(world);
        for (int r = 0; r < world; ++r) CK(sunsky_comm_create(uid, world, r, &comms[r]));
        std::vector<hipStream_t> streams(world);
        for (auto& s : streams) HK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        for (int sp = 0; sp < 2; ++sp) {
            const int nplanes = sp ? 11 : 3;
            for (size_t n : {(size_t)(1 << 18) + 3, (size_t)(4 * world - 2)}) {   // the second leaves a rank empty
                std::vector<float> h(3 * n);
                std::mt19937 rng((unsigned)(world * 1000 + n));
                std::uniform_real_distribution<float> U(0.f, 1.f);
                for (size_t i = 0; i < n; ++i) {
                    float ct = U(rng), ph = 6.2831853f * U(rng), st = std::sqrt(std::max(0.f, 1 - ct * ct));
                    h[i] = -st * std::cos(ph); h[n + i] = -st * std::sin(ph); h[2 * n + i] = -ct;
                }
                float *wi, *whole;
                HK(hipMalloc(&wi, 3 * n * 4));
                HK(hipMalloc(&whole, nplanes * n * 4));
                HK(hipMemcpy(wi, h.data(), 3 * n * 4, hipMemcpyHostToDevice));
                if (eval(sp ? spec : rgb, sp, wi, n, n, whole)) return 2;
                std::vector<float*> shard(world, nullptr);
                std::vector<size_t> counts(world);
                for (int r = 0; r < world; ++r) {
                    size_t a, b;
                    shard_range(n, r, world, &a, &b);
                    counts[r] = b - a;
                    if (!counts[r]) continue;
                    float* wr;
                    HK(hipMalloc(&wr, 3 * counts[r] * 4));
                    for (int c = 0; c < 3; ++c)
                        HK(hipMemcpy(wr + c * counts[r], wi + c * n + a, counts[r] * 4, hipMemcpyDeviceToDevice));
                    HK(hipMalloc(&shard[r], nplanes * counts[r] * 4));
                    if (eval(sp ? spec : rgb, sp, wr, counts[r], counts[r], shard[r])) return 2;
                    HK(hipDeviceSynchronize());
                    (void)hipFree(wr);
                }
                std::vector<float> ref(nplanes * n), got(nplanes * n);
                HK(hipDeviceSynchronize());
                HK(hipMemcpy(ref.data(), whole, ref.size() * 4, hipMemcpyDeviceToHost));
                float* out;
                HK(hipMalloc(&out, nplanes * n * 4));
                for (int root : {0, world - 1}) {
                    for (int rev = 0; rev < 2; ++rev) {
                        HK(hipMemset(out, 0xff, nplanes * n * 4));   // NaN
                        HK(hipDeviceSynchronize());   // the gather streams are non-blocking: order the fill first
                        for (int k = 0; k < world; ++k) {
                            const int r = rev ? world - 1 - k : k;
                            CK(sunsky_gather_radiance(comms[r], root, shard[r], std::max<size_t>(counts[r], 1), nplanes,
                                                      counts.data(), r == root ? out : nullptr, r == root ? n : 0,
                                                      streams[r]));
                        }
                        HK(hipDeviceSynchronize());
                        HK(hipMemcpy(got.data(), out, got.size() * 4, hipMemcpyDeviceToHost));
                        if (std::memcmp(got.data(), ref.data(), got.size() * 4) != 0) {
                            std::printf("world %d planes %d n %zu root %d order %d: gathered planes differ\n", world,
                                        nplanes, n, root, rev);
                            return 1;
                        }
                        ++cases;
                        std::printf("case %d: world %d planes %d n %zu root %d order %d ok\n", cases, world, nplanes, n,
                                    root, rev);
                        std::fflush(stdout);
                    }
                }
                for (float* s : shard) if (s) (void)hipFree(s);
                (void)hipFree(out); (void)hipFree(wi); (void)hipFree(whole);
            }
        }
        for (auto* c : comms) sunsky_comm_destroy(c);
        for (auto s : streams) (void)hipStreamDestroy(s);
    }
    sunsky_emitter_destroy(rgb);
    sunsky_emitter_destroy(spec);
    sunsky_props_destroy(p);
    std::printf("multi-rank gather through the RCCL double: %d cases bitwise equal\n", cases);
    return 0;
}
