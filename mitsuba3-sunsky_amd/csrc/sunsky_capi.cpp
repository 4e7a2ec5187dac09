// sunsky_capi.cpp -- the C ABI (include/sunsky_amd.h): host staging through
// SunskyModel, device tables, and kernel launches through hipModule.
#include "sunsky_amd.h"

#include <dlfcn.h>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <sys/stat.h>

#include "sunsky_dataset.h"
#include "sunsky_errors.h"
#include "sunsky_model.h"
#include "sunsky_profiler.h"
#include "sunsky_props.h"
#include "sunsky_types.h"

using namespace sunsky;

// ---------------------------------------------------------------- errors
namespace sunsky {
double hosek_solar_radiance(const std::string& datasets, double turbidity, double wavelength, double elevation,
                            double gamma);
}

namespace sunsky {
namespace capi {
std::string& last_error() {
    thread_local std::string g_error;
    return g_error;
}
}  // namespace capi
}  // namespace sunsky

namespace {
using namespace sunsky::capi;

// ---------------------------------------------------------------- paths
std::string library_dir() {
    Dl_info info;
    if (dladdr((const void*)&library_dir, &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        size_t s = p.rfind('/');
        return s == std::string::npos ? std::string(".") : p.substr(0, s);
    }
    return ".";
}

bool file_exists(const std::string& p) {
    struct stat st;
    return ::stat(p.c_str(), &st) == 0;
}

std::string default_pack_path() {
    if (const char* env = std::getenv("SUNSKY_AMD_DATASET")) return env;
    std::string d = library_dir();
    for (const char* rel : {"/sunsky_datasets.pack", "/../data/sunsky_datasets.pack", "/data/sunsky_datasets.pack"})
        if (file_exists(d + rel)) return d + rel;
    return d + "/../data/sunsky_datasets.pack";
}

std::string code_object_path() {
    if (const char* env = std::getenv("SUNSKY_AMD_CODE_OBJECT")) return env;
    return library_dir() + "/sunsky_kernels.hsaco";
}

// The same kernels compiled with to_world / to_local as the identity (SS_XFORM_IDENTITY),
// launched for emitters whose to_world is the identity: the same bits without the
// per-direction identity test.  SUNSKY_AMD_CODE_OBJECT_IDENT (a probe build) replaces it.
std::string ident_code_object_path() {
    if (const char* env = std::getenv("SUNSKY_AMD_CODE_OBJECT_IDENT")) return env;
    const std::string path = library_dir() + "/sunsky_kernels_ident.hsaco";
    // an A/B run that overrides only the general module would otherwise time the installed
    // identity module for every identity-to_world emitter without noticing
    if (std::getenv("SUNSKY_AMD_CODE_OBJECT"))
        std::fprintf(stderr, "sunsky_amd: SUNSKY_AMD_CODE_OBJECT is set but SUNSKY_AMD_CODE_OBJECT_IDENT is not: "
                             "emitters with an identity to_world use %s\n", path.c_str());
    return path;
}

// An SS_XFORM_IDENTITY build exports sunsky_xform_identity_marker.  Such an object as the
// general module would drop every rotated to_world without an error, and a general build
// as the identity module would only be slower: both are refused at load.
void check_xform_form(hipModule_t mod, const std::string& path, bool want_identity) {
    hipFunction_t f = nullptr;
    const bool is_identity = hipModuleGetFunction(&f, mod, "sunsky_xform_identity_marker") == hipSuccess;
    (void)hipGetLastError();
    if (is_identity != want_identity)
        throw HipError("code object " + path + (is_identity
            ? " is an identity-to_world build (SS_XFORM_IDENTITY); it cannot serve emitters with a rotated to_world "
              "(SUNSKY_AMD_CODE_OBJECT takes a general build, SUNSKY_AMD_CODE_OBJECT_IDENT an identity build)"
            : " is not an identity-to_world build (SUNSKY_AMD_CODE_OBJECT_IDENT takes an SS_XFORM_IDENTITY build)"));
}

// ---------------------------------------------------------------- kernels
// The sampling kernels are instantiated per variant (RGB / spectral) so each
// carries only its own tables and registers.
enum KernelId {
    K_EVAL_RGB_V4, K_EVAL_RGB_V1, K_EVAL_SPEC_BCAST_V4, K_EVAL_SPEC_BCAST_V1, K_EVAL_SPEC_NODES_V4,
    K_EVAL_SPEC_RAYS_V4, K_EVAL_SPEC_RAYS_V1, K_SAMPLE_DIRECTION_RGB, K_SAMPLE_DIRECTION_SPEC, K_PDF_DIRECTION_V4, K_PDF_DIRECTION_V1, K_SAMPLE_WAVELENGTHS_RGB,
    K_SAMPLE_WAVELENGTHS_SPEC, K_SAMPLE_RAY_RGB, K_SAMPLE_RAY_SPEC, K_BAKE_RGB, K_BAKE_SPEC,
    K_DIRECT_DIFFUSE_RGB, K_DIRECT_DIFFUSE_SPEC, K_SAMPLE_DIRECTION_RGB_LEAN, K_SAMPLE_DIRECTION_SPEC_LEAN,
    K_DIRECT_DIFFUSE_RAYS, K_SAMPLE_DIRECTION_RGB_LEAN_PLAIN, K_DIRECT_CONDUCTOR_RGB, K_DIRECT_CONDUCTOR_SPEC,
    K_DIRECT_CONDUCTOR_RAYS, K_SAMPLE_DIRECTION_SPEC_LEAN4_SORTED, K_SAMPLE_RAY_RGB_SORTED,
    K_SAMPLE_DIRECTION_RGB_FULL_SORTED, K_EVAL_SPEC_RAYS4_V4, K_DEBUG_SUN_SEGMENTS, K_SAMPLE_DIRECTION_RGB_POS_SORTED,
    K_SAMPLE_DIRECTION_SPEC_POS_SORTED, K_COUNT
};
const char* kKernelNames[K_COUNT] = {
    "sunsky_eval_rgb_v4", "sunsky_eval_rgb_v1", "sunsky_eval_spec_bcast_v4", "sunsky_eval_spec_bcast_v1",
    "sunsky_eval_spec_nodes_v4", "sunsky_eval_spec_rays_v4", "sunsky_eval_spec_rays_v1", "sunsky_sample_direction_rgb",
    "sunsky_sample_direction_spec", "sunsky_pdf_direction_v4", "sunsky_pdf_direction_v1",
    "sunsky_sample_wavelengths_rgb",
    "sunsky_sample_wavelengths_spec", "sunsky_sample_ray_rgb", "sunsky_sample_ray_spec",
    "sunsky_bake_latlong_rgb", "sunsky_bake_latlong_spec", "sunsky_direct_diffuse_rgb", "sunsky_direct_diffuse_spec",
    "sunsky_sample_direction_rgb_lean", "sunsky_sample_direction_spec_lean", "sunsky_direct_diffuse_rays",
    "sunsky_sample_direction_rgb_lean_plain", "sunsky_direct_conductor_rgb", "sunsky_direct_conductor_spec",
    "sunsky_direct_conductor_rays", "sunsky_sample_direction_spec_lean4_sorted", "sunsky_sample_ray_rgb_sorted",
    "sunsky_sample_direction_rgb_full_sorted", "sunsky_eval_spec_rays4_v4", "sunsky_debug_sun_segments",
    "sunsky_sample_direction_rgb_pos_sorted", "sunsky_sample_direction_spec_pos_sorted"};

// eval kernels instantiated twice: eval(si) negates wi at compile time,
// eval_direction(ds) uses ds.d as is (the "_dir" kernels)
bool has_dir_form(KernelId k) {
    return k == K_EVAL_RGB_V4 || k == K_EVAL_RGB_V1 || k == K_EVAL_SPEC_RAYS_V4 || k == K_EVAL_SPEC_RAYS_V1 ||
           k == K_EVAL_SPEC_RAYS4_V4;
}

struct DeviceModule {
    hipModule_t module = nullptr, module_ident = nullptr;
    // [identity to_world][precision][kernel]: [1] from sunsky_kernels_ident.hsaco
    hipFunction_t fn[2][2][K_COUNT] = {};
    hipFunction_t fn_dir[2][2][K_COUNT] = {};   // eval_direction forms (wo = +d) of the eval kernels
    hipFunction_t jvp_rgb = nullptr, jvp_spec = nullptr;   // eval_jvp (reference operation order)
    hipFunction_t vjp_rgb = nullptr, vjp_spec = nullptr, grad_reduce = nullptr;   // eval_vjp
    hipFunction_t latlong_tables = nullptr;                                     // bake_latlong
    hipFunction_t stage_radiance = nullptr, quad_points = nullptr, quad_finish = nullptr;   // parameters_changed
    hipFunction_t stage_tangent = nullptr;                                      // eval_jvp / eval_vjp tables
    int cu_count = 256;
};

std::mutex g_module_mutex;
std::map<int, DeviceModule*> g_modules;

DeviceModule* module_for_device(int dev) {
    std::lock_guard<std::mutex> lock(g_module_mutex);
    auto it = g_modules.find(dev);
    if (it != g_modules.end()) return it->second;
    std::unique_ptr<DeviceModule> m(new DeviceModule());
    const std::string path = code_object_path(), ipath = ident_code_object_path();
    for (const std::string& p : {path, ipath})
        if (!file_exists(p)) throw HipError("kernel code object not found: " + p + " (run the build)");
    hip_check(hipModuleLoad(&m->module, path.c_str()), "hipModuleLoad(sunsky_kernels.hsaco)");
    check_xform_form(m->module, path, false);
    hip_check(hipModuleLoad(&m->module_ident, ipath.c_str()), "hipModuleLoad(sunsky_kernels_ident.hsaco)");
    check_xform_form(m->module_ident, ipath, true);
    for (int id = 0; id < 2; ++id)
        for (int p = 0; p < 2; ++p)
            for (int k = 0; k < K_COUNT; ++k) {
                hipModule_t mod = id ? m->module_ident : m->module;
                std::string name = std::string(kKernelNames[k]) + (p == SUNSKY_PRECISION_FAST ? "_fast" : "_ref");
                hip_check(hipModuleGetFunction(&m->fn[id][p][k], mod, name.c_str()), name.c_str());
                if (has_dir_form((KernelId)k)) {
                    std::string dn = std::string(kKernelNames[k]) + (p == SUNSKY_PRECISION_FAST ? "_dir_fast" : "_dir_ref");
                    hip_check(hipModuleGetFunction(&m->fn_dir[id][p][k], mod, dn.c_str()), dn.c_str());
                }
            }
    hip_check(hipModuleGetFunction(&m->jvp_rgb, m->module, "sunsky_eval_jvp_rgb"), "sunsky_eval_jvp_rgb");
    hip_check(hipModuleGetFunction(&m->jvp_spec, m->module, "sunsky_eval_jvp_spec"), "sunsky_eval_jvp_spec");
    hip_check(hipModuleGetFunction(&m->vjp_rgb, m->module, "sunsky_eval_vjp_rgb"), "sunsky_eval_vjp_rgb");
    hip_check(hipModuleGetFunction(&m->vjp_spec, m->module, "sunsky_eval_vjp_spec"), "sunsky_eval_vjp_spec");
    hip_check(hipModuleGetFunction(&m->grad_reduce, m->module, "sunsky_grad_reduce"), "sunsky_grad_reduce");
    hip_check(hipModuleGetFunction(&m->latlong_tables, m->module, "sunsky_latlong_tables"), "sunsky_latlong_tables");
    hip_check(hipModuleGetFunction(&m->stage_tangent, m->module, "sunsky_stage_tangent"), "sunsky_stage_tangent");
    hip_check(hipModuleGetFunction(&m->stage_radiance, m->module, "sunsky_stage_radiance"), "sunsky_stage_radiance");
    hip_check(hipModuleGetFunction(&m->quad_points, m->module, "sunsky_stage_quad_points"), "sunsky_stage_quad_points");
    hip_check(hipModuleGetFunction(&m->quad_finish, m->module, "sunsky_stage_quad_finish"), "sunsky_stage_quad_finish");
    hip_check(hipDeviceGetAttribute(&m->cu_count, hipDeviceAttributeMultiprocessorCount, dev),
              "hipDeviceGetAttribute");
    DeviceModule* raw = m.release();
    g_modules[dev] = raw;
    return raw;
}

constexpr int kBlock = 256;

// Grid-stride launches sized to fill every CU several times over
// (cdna_hip_programming.md Guideline 11).  Workgroups per CU from the
// tools/kbench.cpp sweep on MI355X (profiles/r01_v2_kbench_grid_sweep.log):
// RGB eval 64 (60.4 us vs 64.9 us at 16 for 16M directions), spectral 64,
// sampling 64 (profiles/r01_v5_kbench.log, r01_v7_tune.log).
// SUNSKY_AMD_BLOCKS_PER_CU overrides every kernel class.
int blocks_per_cu(KernelId k) {
    static const int env = [] {
        const char* e = std::getenv("SUNSKY_AMD_BLOCKS_PER_CU");
        return e ? std::max(1, std::atoi(e)) : 0;
    }();
    if (env) return env;
    switch (k) {
        case K_EVAL_RGB_V4: case K_EVAL_RGB_V1: return 64;
        case K_EVAL_SPEC_BCAST_V4: case K_EVAL_SPEC_BCAST_V1: case K_EVAL_SPEC_NODES_V4: return 64;
        case K_SAMPLE_DIRECTION_RGB: case K_SAMPLE_DIRECTION_SPEC: case K_PDF_DIRECTION_V4: case K_PDF_DIRECTION_V1:
        case K_SAMPLE_DIRECTION_RGB_LEAN: case K_SAMPLE_DIRECTION_SPEC_LEAN:
        case K_SAMPLE_DIRECTION_RGB_LEAN_PLAIN: case K_SAMPLE_DIRECTION_SPEC_LEAN4_SORTED:
        case K_SAMPLE_RAY_RGB_SORTED: case K_SAMPLE_DIRECTION_RGB_FULL_SORTED: case K_SAMPLE_DIRECTION_RGB_POS_SORTED:
        case K_SAMPLE_DIRECTION_SPEC_POS_SORTED:
            return 64;
        case K_BAKE_RGB: case K_BAKE_SPEC: return 64;
        case K_DIRECT_DIFFUSE_RGB: case K_DIRECT_DIFFUSE_SPEC: case K_DIRECT_DIFFUSE_RAYS: return 64;
        case K_DIRECT_CONDUCTOR_RGB: case K_DIRECT_CONDUCTOR_SPEC: case K_DIRECT_CONDUCTOR_RAYS: return 64;
        case K_EVAL_SPEC_RAYS_V4: case K_EVAL_SPEC_RAYS_V1: case K_EVAL_SPEC_RAYS4_V4: return 64;
        // kbench sweep over 8/16/32/64 (profiles/r03_v18_kbench_grid_ray_wavelengths.log)
        case K_SAMPLE_RAY_RGB: case K_SAMPLE_RAY_SPEC: return 32;
        case K_SAMPLE_WAVELENGTHS_SPEC: return 64;
        default: return 16;
    }
}

unsigned grid_for(const DeviceModule* m, KernelId k, size_t work_items) {
    size_t need = (work_items + kBlock - 1) / kBlock;
    size_t cap = (size_t)m->cu_count * (size_t)blocks_per_cu(k);
    return (unsigned)std::max<size_t>(1, std::min(need, cap));
}

void launch(hipFunction_t f, unsigned grid, hipStream_t stream, void** args, unsigned dyn_lds = 0) {
    hip_check(hipModuleLaunchKernel(f, grid, 1, 1, kBlock, 1, 1, dyn_lds, stream, args, nullptr),
              "hipModuleLaunchKernel");
}

// The 11-node spectral kernel with more than one step per lane (configs[4]'s 64M directions
// per GPU): unused dynamic LDS that holds it to 5 workgroups (5 waves/SIMD) per CU.  Fewer
// concurrent 11-plane write streams per CU write HBM faster there: 64M x 11 cold, 774 ->
// 750 us at 5 and 745 us at 4 workgroups per CU, 806 us at 2; at one step per lane (16M)
// neutral (profiles/r06_v8_nodes_occupancy_cold.log, r06_v7_ab_nodes_lds_cap.log).
constexpr unsigned kNodesLdsCap = 32000;

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

struct LambdaSet {   // mirrors the kernel-side struct
    int m;
    int lo[kMaxBroadcastLambda];
    float f[kMaxBroadcastLambda];
};

struct LatLong {     // mirrors the kernel-side struct
    int w, h;
    float theta0, dtheta, phi0, dphi;
    const float* tab;
};

// normalized_wavelengths / floor2int / lerp factor of eval, sunsky.cpp:326-332
LambdaSet make_lambda_set(const float* lam, int m) {
    LambdaSet L;
    std::memset(&L, 0, sizeof(L));
    L.m = m;
    for (int k = 0; k < m; ++k) {
        float nw = (lam[k] - kWavelength0) / kWavelengthStep;
        bool valid = (0.f <= nw) && (nw <= (float)(kNbWavelengths - 1));
        int lo = valid ? (int)std::floor(nw) : 0;
        L.lo[k] = lo;
        L.f[k] = valid ? nw - (float)lo : -1.f;
    }
    return L;
}

// Makes the emitter's device current for the scope of an entry point: every
// allocation, event and launch of an emitter happens on its own GPU whatever the
// caller's current device is.
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        if (dev < 0) return;
        int cur = 0;
        hip_check(hipGetDevice(&cur), "hipGetDevice");
        if (cur != dev) {
            hip_check(hipSetDevice(dev), "hipSetDevice");
            prev = cur;
        }
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

struct StageArgs {   // mirrors the kernel-side struct (sunsky_kernels.hip)
    SunskyKArgs* state;
    float* sun_table;
    const float* sky_params_ds;
    const float* sky_rad_ds;
    const float* sun_rad_ds;
    RadianceStage rs;
    float albedo[kNbWavelengths];
    int nch, variant, sun_block;
    float sky_scale;
};

constexpr int kQuadBlock = 256;   // sunsky_kernels.hip: one quadrature row per workgroup
struct QuadArgs {    // mirrors the kernel-side struct (sunsky_kernels.hip)
    SunskyKArgs* state;
    const float* qx;
    const float* qw;
    float* rows;
    int nq, nch;
    float cie_y[kNbWavelengths];
    float sky_scale, sun_scale;
    int* status;
};

}  // namespace

// ---------------------------------------------------------------- handles
struct sunsky_props {
    Properties props;
};

struct sunsky_emitter {
    std::unique_ptr<SunskyModel> model;
    // Host mirror of the state: geometry, dispatch fields (variant, semantics, nch) and,
    // once read back (sync_host), the device-staged radiance fields.
    SunskyKArgs kargs;
    DeviceModule* mod = nullptr;
    int device = 0;
    int precision = SUNSKY_PRECISION_FAST;
    // ---- device state (one per emitter per GPU).  Every kernel reads the emitter
    // through `d_state` (SunskyKArgs in device memory, s_load'ed by the kernels);
    // parameters_changed rewrites it in place, ordered on the caller's stream.
    SunskyKArgs* d_state = nullptr;
    float* d_sun_table = nullptr;
    float* d_sun_ld = nullptr;
    float* d_datasets = nullptr;          // sky params | sky radiance | sun table | quadrature x | w
    const float *d_sky_params_ds = nullptr, *d_sky_rad_ds = nullptr, *d_sun_rad_ds = nullptr;
    const float *d_qx = nullptr, *d_qw = nullptr;
    float* d_quad_part = nullptr;         // quadrature row sums [2][200][nch]
    int* d_status = nullptr;              // device staging status (0 ok)
    static constexpr int kRing = 4;       // pinned host images of the state for the async copy
    SunskyKArgs* h_ring = nullptr;
    hipEvent_t ring_ev[kRing] = {};
    bool ring_used[kRing] = {};
    int ring_i = 0;
    bool restoring = false;                    // restaging the accepted state after a rejection
    int inject_faults = 0;                     // testing: stagings left that report a rejection
    mutable hipEvent_t stage_done = nullptr;   // recorded after the last device staging
    mutable float* d_jvp = nullptr;   // eval_jvp tangent tables (layout: sunsky_kernels.hip)
    mutable float* d_vjp = nullptr;   // eval_vjp basis-tangent tables
    mutable float* d_partials = nullptr;   // eval_vjp per-workgroup gradient partials
    mutable size_t partials_cap = 0;
    mutable float* d_bake = nullptr;       // bake_latlong angle tables
    mutable size_t bake_cap = 0;
    // AD tangent tables depend only on the emitter state: restaged when `rev` (bumped by
    // every staging) or, for the JVP, the requested tangent changes.  `ad_done` is recorded
    // after each AD launch; the next AD call's stream waits on it, so a later call on
    // another stream cannot overwrite d_jvp / d_partials under an in-flight kernel.  The
    // bakes order their angle tables the same way (`bake_done`).
    uint64_t rev = 0;
    mutable uint64_t vjp_rev = ~0ull, jvp_rev = ~0ull;
    mutable std::vector<float> jvp_key;
    mutable hipEvent_t ad_done = nullptr, bake_done = nullptr;

    static constexpr int kJvpFloats = kJvpSunOffset + kSunRgbTableSize;   // AD tangent buffers
    static constexpr int kVjpFloats = kVjpSunOffset + kSunRgbTableSize;

    // Allocations of a GPU emitter (once, at creation): state, tables, the raw datasets
    // the staging kernels read, quadrature nodes, scratch, pinned ring, events.
    void init_device() {
        const bool spec = model->variant() == kSpectral;
        hip_check(hipMalloc(&d_state, sizeof(SunskyKArgs)), "hipMalloc");
        hip_check(hipMalloc(&d_sun_table, sizeof(float) * kSunRgbTableSize), "hipMalloc");
        hip_check(hipMalloc(&d_sun_ld, sizeof(float) * kNbWavelengths * kNbSunLdParams), "hipMalloc");
        const std::vector<float>& sp = model->sky_params_ds();
        const std::vector<float>& sr = model->sky_rad_ds();
        const std::vector<float>& su = model->sun_rad_ds();
        std::vector<float> qx, qw;
        SunskyModel::quadrature_nodes(&qx, &qw);
        std::vector<float> all;
        all.reserve(sp.size() + sr.size() + su.size() + qx.size() + qw.size());
        all.insert(all.end(), sp.begin(), sp.end());
        all.insert(all.end(), sr.begin(), sr.end());
        all.insert(all.end(), su.begin(), su.end());
        all.insert(all.end(), qx.begin(), qx.end());
        all.insert(all.end(), qw.begin(), qw.end());
        hip_check(hipMalloc(&d_datasets, sizeof(float) * all.size()), "hipMalloc");
        hip_check(hipMemcpy(d_datasets, all.data(), sizeof(float) * all.size(), hipMemcpyHostToDevice), "hipMemcpy");
        d_sky_params_ds = d_datasets;
        d_sky_rad_ds = d_sky_params_ds + sp.size();
        d_sun_rad_ds = d_sky_rad_ds + sr.size();
        d_qx = d_sun_rad_ds + su.size();
        d_qw = d_qx + qx.size();
        const std::vector<float>& ld = model->sun_ld();
        if (spec)
            hip_check(hipMemcpy(d_sun_ld, ld.data(), sizeof(float) * std::min<size_t>(ld.size(), kNbWavelengths * kNbSunLdParams),
                                hipMemcpyHostToDevice), "hipMemcpy");
        const size_t nq = qx.size();
        hip_check(hipMalloc(&d_quad_part, sizeof(float) * 2 * nq * model->nch()), "hipMalloc");
        hip_check(hipMalloc(&d_status, sizeof(int)), "hipMalloc");
        hip_check(hipMemset(d_status, 0, sizeof(int)), "hipMemset");
        hip_check(hipHostMalloc((void**)&h_ring, sizeof(SunskyKArgs) * kRing, hipHostMallocDefault), "hipHostMalloc");
        for (int i = 0; i < kRing; ++i)
            hip_check(hipEventCreateWithFlags(&ring_ev[i], hipEventDisableTiming), "hipEventCreate");
        hip_check(hipEventCreateWithFlags(&stage_done, hipEventDisableTiming), "hipEventCreate");
    }

    // parameters_changed on the device, ordered on `s`: the host-staged part of the
    // state (geometry, TGMM, discrete distribution) by an async copy from a pinned image,
    // then the staging kernels write the sky channels, the sun table and (JIT) the
    // sampling weight and wavelength distribution.  Nothing here waits for the device,
    // except for a pinned image still in flight kRing updates later.
    void stage_async(hipStream_t s) {
        kargs = model->kargs();
        kargs.sun_table = d_sun_table;
        kargs.sun_ld = d_sun_ld;
        const int slot = ring_i;
        ring_i = (ring_i + 1) % kRing;
        if (ring_used[slot]) hip_check(hipEventSynchronize(ring_ev[slot]), "hipEventSynchronize");
        h_ring[slot] = kargs;
        hip_check(hipMemcpyAsync(d_state, &h_ring[slot], sizeof(SunskyKArgs), hipMemcpyHostToDevice, s),
                  "hipMemcpyAsync");
        hip_check(hipEventRecord(ring_ev[slot], s), "hipEventRecord");
        ring_used[slot] = true;
        const bool spec = model->variant() == kSpectral;
        StageArgs A;
        std::memset(&A, 0, sizeof(A));
        A.state = d_state;
        A.sun_table = d_sun_table;
        A.sky_params_ds = d_sky_params_ds;
        A.sky_rad_ds = d_sky_rad_ds;
        A.sun_rad_ds = d_sun_rad_ds;
        A.rs = model->radiance_stage();
        const std::vector<float>& alb = model->albedo();
        for (int c = 0; c < model->nch(); ++c) A.albedo[c] = alb[c];
        A.nch = model->nch();
        A.variant = model->variant();
        A.sun_block = spec ? kSunSpecTableSize : kSunRgbTableSize;
        A.sky_scale = model->sky_scale();
        void* sargs[] = {&A};
        hip_check(hipModuleLaunchKernel(mod->stage_radiance, 1, 1, 1, 256, 1, 1, 0, s, sargs, nullptr),
                  "hipModuleLaunchKernel(sunsky_stage_radiance)");
        if (model->semantics() == kJit) {
            QuadArgs Q;
            std::memset(&Q, 0, sizeof(Q));
            Q.state = d_state;
            Q.qx = d_qx;
            Q.qw = d_qw;
            Q.rows = d_quad_part;
            Q.nq = 200;
            Q.nch = model->nch();
            std::memcpy(Q.cie_y, model->cie_y(), sizeof(Q.cie_y));
            Q.sky_scale = model->sky_scale();
            Q.sun_scale = model->sun_scale();
            Q.status = d_status;
            void* qargs[] = {&Q};
            static_assert(200 <= kQuadBlock, "one quadrature row per workgroup");
            hip_check(hipModuleLaunchKernel(mod->quad_points, (unsigned)Q.nq, 1, 1, kQuadBlock, 1, 1, 0, s, qargs, nullptr),
                      "hipModuleLaunchKernel(sunsky_stage_quad_points)");
            hip_check(hipModuleLaunchKernel(mod->quad_finish, 1, 1, 1, 256, 1, 1, 0, s, qargs, nullptr),
                      "hipModuleLaunchKernel(sunsky_stage_quad_finish)");
        }
        if (inject_faults > 0 && model->semantics() == kJit && !restoring) {   // sunsky_emitter_inject_staging_fault
            --inject_faults;
            hip_check(hipMemsetAsync(d_status, 1, 1, s), "hipMemsetAsync");
        }
        hip_check(hipEventRecord(stage_done, s), "hipEventRecord");
        ++rev;
    }

    // Bring the device-staged fields back into the host model (get_info / get_table /
    // to_string): waits for the last staging only.
    void sync_host() const {
        if (!model->radiance_stale() || !d_state) return;
        DeviceScope g(device);
        hip_check(hipEventSynchronize(stage_done), "hipEventSynchronize");
        SunskyKArgs dk;
        hip_check(hipMemcpy(&dk, d_state, sizeof(dk), hipMemcpyDeviceToHost), "hipMemcpy");
        std::vector<float> st(kSunRgbTableSize);
        hip_check(hipMemcpy(st.data(), d_sun_table, sizeof(float) * st.size(), hipMemcpyDeviceToHost), "hipMemcpy");
        int status = 0;
        hip_check(hipMemcpy(&status, d_status, sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy");
        auto* self = const_cast<sunsky_emitter*>(this);
        if (status) {
            // A device staging since the last read-back rejected its update (a negative
            // wavelength-distribution node, the check of ContinuousDistribution's
            // constructor); the status is sticky, so which one is unknown.  As the reference
            // throws from parameters_changed and keeps its old state: restore the parameters
            // of the last staging known to be accepted, restage them, report the error once.
            hip_check(hipMemset(d_status, 0, sizeof(int)), "hipMemset");
            if (restoring || !model->has_accepted())   // the accepted state itself is rejected (e.g. at creation)
                throw std::runtime_error("ContinuousDistribution: entries must be non-negative!");
            model->revert_to_accepted();
            self->restoring = true;
            try {
                // batch kernels queued on any stream may still read d_state: let them drain
                // before it is rewritten (a rare error path; no stream of the caller is known)
                hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
                self->stage_async(nullptr);
                hip_check(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
                sync_host();
            } catch (...) {
                self->restoring = false;
                throw;
            }
            self->restoring = false;
            throw std::runtime_error("ContinuousDistribution: entries must be non-negative! (update rejected by the "
                                     "device staging; the parameters of the last accepted update were restored)");
        }
        model->mark_accepted();
        model->adopt_device_stage(dk, st.data());
        const SunskyKArgs& hk = model->kargs();
        std::memcpy(self->kargs.sky, hk.sky, sizeof(hk.sky));
        std::memcpy(self->kargs.fsky, hk.fsky, sizeof(hk.fsky));
        self->kargs.w_sky = hk.w_sky;
        self->kargs.sun_sky_fit_on = hk.sun_sky_fit_on;
        self->kargs.spec_size = hk.spec_size;
        std::memcpy(self->kargs.spec_pdf, hk.spec_pdf, sizeof(hk.spec_pdf));
        std::memcpy(self->kargs.spec_cdf, hk.spec_cdf, sizeof(hk.spec_cdf));
        self->kargs.spec_integral = hk.spec_integral;
        self->kargs.spec_norm = hk.spec_norm;
        self->kargs.spec_interval = hk.spec_interval;
        self->kargs.spec_inv_interval = hk.spec_inv_interval;
    }

    // the identity-to_world code object for emitters whose to_world is the identity
    // (SUNSKY_AMD_GENERAL_XFORM=1: the general one always; the bitwise test of the two)
    // A launch being captured into a hipGraph takes the general code object: the graph may be
    // replayed after an update that gives the emitter a non-identity to_world (captured
    // launches read the current state), which the identity kernels would not apply.
    int xform_form(hipStream_t s) const {
        const char* g = std::getenv("SUNSKY_AMD_GENERAL_XFORM");
        if (!kargs.identity_xform || (g && g[0] == '1')) return 0;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        hip_check(hipStreamIsCapturing(s, &cs), "hipStreamIsCapturing");
        return cs == hipStreamCaptureStatusNone ? 1 : 0;
    }
    hipFunction_t fn(KernelId k, hipStream_t s) const {
        if (!mod) throw std::invalid_argument("host-only emitter (sunsky_emitter_create_host) cannot launch kernels");
        return mod->fn[xform_form(s)][precision][k];
    }
    // eval (sign < 0: wo = -wi) or eval_direction (sign > 0: wo = d) form of an eval kernel
    hipFunction_t fn_eval(KernelId k, float sign, hipStream_t s) const {
        if (!mod) throw std::invalid_argument("host-only emitter (sunsky_emitter_create_host) cannot launch kernels");
        const int x = xform_form(s);
        return sign < 0.f ? mod->fn[x][precision][k] : mod->fn_dir[x][precision][k];
    }

    ~sunsky_emitter() {
        if (device < 0) return;
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != device) (void)hipSetDevice(device);
        // a destroyed emitter may still be read by launches in flight on any stream
        (void)hipDeviceSynchronize();
        for (void* p : {(void*)d_state, (void*)d_sun_table, (void*)d_sun_ld, (void*)d_datasets, (void*)d_quad_part,
                        (void*)d_status, (void*)d_jvp, (void*)d_vjp, (void*)d_partials, (void*)d_bake})
            if (p) (void)hipFree(p);
        if (h_ring) (void)hipHostFree(h_ring);
        for (hipEvent_t ev : ring_ev)
            if (ev) (void)hipEventDestroy(ev);
        for (hipEvent_t ev : {stage_done, ad_done, bake_done})
            if (ev) (void)hipEventDestroy(ev);
        if (cur >= 0 && cur != device) (void)hipSetDevice(cur);
    }

    // Order this AD call after the previous one (any stream), then mark its end.
    void ad_begin(hipStream_t st) const {
        if (!ad_done) hip_check(hipEventCreateWithFlags(&ad_done, hipEventDisableTiming), "hipEventCreate");
        else hip_check(hipStreamWaitEvent(st, ad_done, 0), "hipStreamWaitEvent");
    }
    void ad_end(hipStream_t st) const { hip_check(hipEventRecord(ad_done, st), "hipEventRecord"); }
    // Device tangent staging into an AD table buffer (sunsky_stage_tangent, sunsky_staging.h):
    // the arguments for `nbasis` bases over this emitter's datasets, then the launch.
    TangentArgs tangent_args(float* out, int nbasis, int sun_local_off, int sun_local_first, int sun_off,
                             int total) const {
        TangentArgs A;
        std::memset(&A, 0, sizeof(A));
        A.sky_params_ds = d_sky_params_ds;
        A.sky_rad_ds = d_sky_rad_ds;
        A.sun_rad_ds = d_sun_rad_ds;
        A.out = out;
        A.nbasis = A.nsky = nbasis;
        A.sun_local_off = sun_local_off;
        A.sun_local_first = sun_local_first;
        A.sun_off = sun_off;
        A.sun_block = model->variant() == kSpectral ? kSunSpecTableSize : kSunRgbTableSize;
        A.total = total;
        return A;
    }
    void stage_tangent(TangentArgs& A, hipStream_t st) const {
        void* args[] = {&A};
        const unsigned grid = (unsigned)((A.total + 255) / 256);
        hip_check(hipModuleLaunchKernel(mod->stage_tangent, grid, 1, 1, 256, 1, 1, 0, st, args, nullptr),
                  "hipModuleLaunchKernel(sunsky_stage_tangent)");
    }
};

// Batch calls need the emitter's device state: a host-only emitter
// (sunsky_emitter_create_host) has none and rejects them.
void require_device(const sunsky_emitter* e) {
    if (!e->mod) throw std::invalid_argument("host-only emitter (sunsky_emitter_create_host) cannot launch kernels");
}

extern "C" {

int sunsky_abi_version(void) { return SUNSKY_AMD_ABI_VERSION; }
const char* sunsky_last_error(void) { return last_error().c_str(); }

int sunsky_props_create(sunsky_props** out) {
    if (!out) return fail(SUNSKY_ERROR_INVALID_VALUE, "null output pointer");
    return guarded([&] { *out = new sunsky_props(); });
}
void sunsky_props_destroy(sunsky_props* p) { delete p; }

#define PROPS_GUARD(p, name)                                                                   \
    if (!(p) || !(name)) return fail(SUNSKY_ERROR_INVALID_VALUE, "null props / property name")

int sunsky_props_set_float(sunsky_props* p, const char* name, double v) {
    PROPS_GUARD(p, name);
    return guarded([&] { p->props.set_float(name, v); });
}
int sunsky_props_set_int(sunsky_props* p, const char* name, int64_t v) {
    PROPS_GUARD(p, name);
    return guarded([&] { p->props.set_int(name, v); });
}
int sunsky_props_set_vector3(sunsky_props* p, const char* name, float x, float y, float z) {
    PROPS_GUARD(p, name);
    return guarded([&] { p->props.set_vector3(name, x, y, z); });
}
int sunsky_props_set_transform(sunsky_props* p, const char* name, const float m[16]) {
    PROPS_GUARD(p, name);
    if (!m) return fail(SUNSKY_ERROR_INVALID_VALUE, "null matrix");
    return guarded([&] { p->props.set_transform(name, m); });
}
int sunsky_props_set_spectrum(sunsky_props* p, const char* name, const float* v, int n) {
    PROPS_GUARD(p, name);
    if (!v || n <= 0) return fail(SUNSKY_ERROR_INVALID_VALUE, "empty spectrum");
    return guarded([&] { p->props.set_spectrum(name, v, n); });
}
int sunsky_props_set_irregular_spectrum(sunsky_props* p, const char* name, const float* wl, const float* v, int n) {
    PROPS_GUARD(p, name);
    if (!wl || !v || n <= 0) return fail(SUNSKY_ERROR_INVALID_VALUE, "empty spectrum");
    return guarded([&] { p->props.set_irregular(name, wl, v, n); });
}

int sunsky_emitter_create(const sunsky_props* props, int variant, int semantics, const char* dataset_path,
                          sunsky_emitter** out) {
    SUNSKY_PHASE("InitScene", "emitter_create");
    if (!props || !out) return fail(SUNSKY_ERROR_INVALID_VALUE, "null props / output pointer");
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<sunsky_emitter> e(new sunsky_emitter());
        std::string ds = dataset_path && *dataset_path ? std::string(dataset_path) : default_pack_path();
        // radiance tables + quadrature are staged on the device (stage_async)
        e->model.reset(new SunskyModel(props->props, variant, semantics, ds, /*radiance_on_host=*/false));
        hip_check(hipGetDevice(&e->device), "hipGetDevice");
        e->mod = module_for_device(e->device);
        if (const char* env = std::getenv("SUNSKY_AMD_PRECISION"))
            e->precision = std::strcmp(env, "reference") == 0 ? SUNSKY_PRECISION_REFERENCE : SUNSKY_PRECISION_FAST;
        e->init_device();
        e->stage_async(nullptr);
        hip_check(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
        e->sync_host();
        for (const std::string& w : e->model->warnings) std::fprintf(stderr, "WARN sunsky: %s\n", w.c_str());
        *out = e.release();
    });
}

int sunsky_emitter_create_host(const sunsky_props* props, int variant, int semantics, const char* dataset_path,
                               sunsky_emitter** out) {
    if (!props || !out) return fail(SUNSKY_ERROR_INVALID_VALUE, "null props / output pointer");
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<sunsky_emitter> e(new sunsky_emitter());
        std::string ds = dataset_path && *dataset_path ? std::string(dataset_path) : default_pack_path();
        e->model.reset(new SunskyModel(props->props, variant, semantics, ds));
        e->device = -1;
        e->kargs = e->model->kargs();
        *out = e.release();
    });
}

void sunsky_emitter_destroy(sunsky_emitter* e) { delete e; }

int sunsky_emitter_set_param(sunsky_emitter* e, const char* name, const float* v, int count) {
    if (!e || !name || !v) return fail(SUNSKY_ERROR_INVALID_VALUE, "null argument");
    return guarded([&] { e->model->set_param(name, v, count); });
}

int sunsky_emitter_parameters_changed_async(sunsky_emitter* e, void* stream) {
    SUNSKY_PHASE("InitScene", "emitter_parameters_changed_async");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    return guarded([&] {
        const bool gpu = e->device >= 0;
        if (gpu) {
            // The update is a host + stream operation (pinned-image copy, events), not a
            // graph node: refuse it during capture before anything is committed or queued.
            DeviceScope g(e->device);
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            hip_check(hipStreamIsCapturing((hipStream_t)stream, &cs), "hipStreamIsCapturing");
            if (cs != hipStreamCaptureStatusNone) {
                e->model->discard_pending();
                throw std::invalid_argument("parameters_changed cannot be captured into a hipGraph: update the "
                                            "emitter outside the capture (a captured graph reads the current state)");
            }
        }
        e->model->parameters_changed(/*radiance_on_host=*/!gpu);   // keeps the scene bounding sphere
        if (gpu) {
            DeviceScope g(e->device);
            e->stage_async((hipStream_t)stream);
        } else {
            e->kargs = e->model->kargs();
        }
    });
}

int sunsky_emitter_inject_staging_fault(sunsky_emitter* e, int count) {
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (count < 0) return fail(SUNSKY_ERROR_INVALID_VALUE, "count must be >= 0");
    e->inject_faults = count;
    return SUNSKY_OK;
}

int sunsky_emitter_sun_segments(const sunsky_emitter* e, const float* cos_theta, size_t n, int* pos, void* stream) {
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (n == 0) return SUNSKY_OK;
    if (!cos_theta || !pos) return fail(SUNSKY_ERROR_INVALID_VALUE, "null input / output pointer");
    return guarded([&] {
        require_device(e);
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        hipStream_t s = (hipStream_t)stream;
        void* args[] = {&K, &cos_theta, &n, &pos};
        launch(e->fn(K_DEBUG_SUN_SEGMENTS, s), grid_for(e->mod, K_DEBUG_SUN_SEGMENTS, n), s, args);
    });
}

int sunsky_emitter_parameters_changed(sunsky_emitter* e) {
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    int rc = sunsky_emitter_parameters_changed_async(e, nullptr);
    if (rc != SUNSKY_OK || e->device < 0) return rc;
    return guarded([&] {
        DeviceScope g(e->device);
        hip_check(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
        e->sync_host();
    });
}

int sunsky_emitter_get_param(const sunsky_emitter* e, const char* name, float* out, int cap, int* count) {
    if (!e || !name || !count) return fail(SUNSKY_ERROR_INVALID_VALUE, "null argument");
    return guarded([&] { *count = e->model->get_param(name, out, out ? cap : 0); });
}

int sunsky_emitter_set_scene(sunsky_emitter* e, int bbox_valid, const float center[3], float radius) {
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    float zero[3] = {0, 0, 0};
    return guarded([&] {
        e->model->set_scene(bbox_valid != 0, center ? center : zero, radius);
        const SunskyKArgs& k = e->model->kargs();
        std::memcpy(e->kargs.bs_center, k.bs_center, sizeof(k.bs_center));
        e->kargs.bs_radius = k.bs_radius;
        if (e->device >= 0) {   // the 4 bounding-sphere floats of the device state, in place
            DeviceScope g(e->device);
            static_assert(offsetof(SunskyKArgs, bs_radius) == offsetof(SunskyKArgs, bs_center) + 3 * sizeof(float),
                          "bounding sphere layout");
            float bs[4] = {k.bs_center[0], k.bs_center[1], k.bs_center[2], k.bs_radius};
            // a staging still queued on another stream copies the whole state block (with
            // the old sphere): let it land first, then write the sphere in place
            hip_check(hipEventSynchronize(e->stage_done), "hipEventSynchronize");
            hip_check(hipMemcpy((char*)e->d_state + offsetof(SunskyKArgs, bs_center), bs, sizeof(bs),
                                hipMemcpyHostToDevice), "hipMemcpy");
        }
    });
}

int sunsky_emitter_set_precision(sunsky_emitter* e, int precision) {
    if (!e || (precision != SUNSKY_PRECISION_FAST && precision != SUNSKY_PRECISION_REFERENCE))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "invalid precision mode");
    e->precision = precision;
    return SUNSKY_OK;
}

int sunsky_emitter_get_info(const sunsky_emitter* e, sunsky_info* out) {
    if (!e || !out) return fail(SUNSKY_ERROR_INVALID_VALUE, "null argument");
    int rc = guarded([&] { e->sync_host(); });
    if (rc != SUNSKY_OK) return rc;
    const SunskyKArgs& k = e->kargs;
    std::memset(out, 0, sizeof(*out));
    out->variant = e->model->variant();
    out->semantics = k.semantics;
    out->nb_channels = e->model->nch();
    out->active_record = e->model->active_record();
    out->turbidity = e->model->turbidity();
    out->sky_scale = k.sky_scale;
    out->sun_scale = k.sun_scale;
    out->sun_half_aperture = k.half_aperture;
    out->cos_cutoff = k.cos_cutoff;
    out->area_ratio = k.area_ratio;
    std::memcpy(out->sun_dir_world, e->model->sun_dir_world(), 3 * sizeof(float));
    std::memcpy(out->sun_dir_local, k.sun_n, 3 * sizeof(float));
    out->sun_angles[0] = k.sun_phi;
    out->sun_angles[1] = k.sun_theta;
    out->sky_sampling_w = k.w_sky;
    std::memcpy(out->bsphere_center, k.bs_center, 3 * sizeof(float));
    out->bsphere_radius = k.bs_radius;
    out->flags = SUNSKY_FLAG_INFINITE | SUNSKY_FLAG_SPATIALLY_VARYING;
    out->device = e->device;
    out->precision = e->precision;
    return SUNSKY_OK;
}

int sunsky_emitter_get_table(const sunsky_emitter* e, int id, float* out, size_t cap, size_t* count) {
    if (!e || !count) return fail(SUNSKY_ERROR_INVALID_VALUE, "null argument");
    int rc = guarded([&] { e->sync_host(); });
    if (rc != SUNSKY_OK) return rc;
    std::vector<float> v;
    const SunskyKArgs& k = e->kargs;
    switch (id) {
        case SUNSKY_TABLE_SKY_PARAMS: v = e->model->sky_params(); break;
        case SUNSKY_TABLE_SKY_RADIANCE: v = e->model->sky_radiance(); break;
        case SUNSKY_TABLE_SUN_RADIANCE: v = e->model->sun_table(); break;
        case SUNSKY_TABLE_SUN_LD: v = e->model->sun_ld(); break;
        case SUNSKY_TABLE_GAUSSIANS: v.assign(e->model->gaussians_raw(), e->model->gaussians_raw() + kNbMixture * kNbGaussianParams); break;
        case SUNSKY_TABLE_GAUSSIAN_CDF: v.assign(k.gauss_cdf, k.gauss_cdf + kNbMixture); break;
        case SUNSKY_TABLE_SPECTRAL_PDF: v.assign(k.spec_pdf, k.spec_pdf + k.spec_size); break;
        case SUNSKY_TABLE_SPECTRAL_CDF: v.assign(k.spec_cdf, k.spec_cdf + std::max(0, k.spec_size - 1)); break;
        case SUNSKY_TABLE_ALBEDO: v = e->model->albedo(); break;
        case SUNSKY_TABLE_SUN_SKY_FIT:
            v.assign(k.sun_sky_fit, k.sun_sky_fit + 6);
            v.insert(v.end(), {k.sun_sky_fit_dev, k.sun_sky_fit_fmin, (float)k.sun_sky_fit_ok, (float)k.sun_sky_fit_on});
            break;
        case SUNSKY_TABLE_SUN_SEGMENTS:
            v.assign(k.sun_seg_z, k.sun_seg_z + kNbSunSegments);
            v.insert(v.end(), {(float)k.sun_row_lo, (float)k.sun_row_hi});
            break;
        default: return fail(SUNSKY_ERROR_INVALID_VALUE, "unknown table id");
    }
    *count = v.size();
    if (out && !v.empty()) std::memcpy(out, v.data(), sizeof(float) * std::min(cap, v.size()));
    return SUNSKY_OK;
}

int sunsky_emitter_to_string(const sunsky_emitter* e, char* buf, size_t cap) {
    if (!e || !buf || !cap) return fail(SUNSKY_ERROR_INVALID_VALUE, "null argument");
    int rc = guarded([&] { e->sync_host(); });
    if (rc != SUNSKY_OK) return rc;
    std::string s = e->model->to_string();
    std::snprintf(buf, cap, "%s", s.c_str());
    return SUNSKY_OK;
}

int sunsky_emitter_bbox(const sunsky_emitter* e, float mn[3], float mx[3]) {
    if (!e || !mn || !mx) return fail(SUNSKY_ERROR_INVALID_VALUE, "null argument");
    for (int i = 0; i < 3; ++i) { mn[i] = INFINITY; mx[i] = -INFINITY; }
    return SUNSKY_OK;
}

// ---------------------------------------------------------------- hot path
static int eval_impl(const sunsky_emitter* e, sunsky_vec3_in w, const float* lam, int nlam, size_t lstride,
                     const uint8_t* active, size_t n, float* out, size_t ostride, void* stream, float sign) {
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (n == 0) return SUNSKY_OK;
    if (!w.x || !w.y || !w.z || !out) return fail(SUNSKY_ERROR_INVALID_VALUE, "null ray / output pointer");
    const bool spec = e->kargs.variant == kSpectral;
    if (spec && (!lam || nlam < 1 || nlam > kMaxLambdaPerRay))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "spectral eval needs 1..16 wavelength planes");
    const size_t nout = spec ? (size_t)nlam : 3;
    if (nout > 1 && ostride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "out_stride < n");
    if (spec && nlam > 1 && lstride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "wl_stride < n");
    return guarded([&] {
        require_device(e);
        hipStream_t s = (hipStream_t)stream;
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        if (!spec) {
            bool vec = n >= 4 && aligned16(w.x) && aligned16(w.y) && aligned16(w.z) && aligned16(out) &&
                       (ostride % 4) == 0 && (!active || ((uintptr_t)active & 3u) == 0);
            size_t n4 = vec ? (n & ~(size_t)3) : 0;
            if (n4) {
                const float *x = w.x, *y = w.y, *z = w.z;
                void* args[] = {&K, &x, &y, &z, &active, &n4, &out, &ostride, &sign};
                launch(e->fn_eval(K_EVAL_RGB_V4, sign, s), grid_for(e->mod, K_EVAL_RGB_V4, n4 / 4), s, args);
            }
            if (n4 < n) {
                const float *x = w.x + n4, *y = w.y + n4, *z = w.z + n4;
                const uint8_t* a = active ? active + n4 : nullptr;
                float* o = out + n4;
                size_t rem = n - n4;
                void* args[] = {&K, &x, &y, &z, &a, &rem, &o, &ostride, &sign};
                launch(e->fn_eval(K_EVAL_RGB_V1, sign, s), grid_for(e->mod, K_EVAL_RGB_V1, rem), s, args);
            }
        } else {
            // VEC = 4 over rays when every plane is 16-byte aligned; VEC = 1 tail
            bool vec = n >= 4 && aligned16(w.x) && aligned16(w.y) && aligned16(w.z) && aligned16(out) &&
                       aligned16(lam) && (ostride % 4) == 0 && (nlam == 1 || (lstride % 4) == 0) &&
                       (!active || ((uintptr_t)active & 3u) == 0);
            size_t n4 = vec ? (n & ~(size_t)3) : 0;
            int nl = nlam;
            if (n4) {
                const float *x = w.x, *y = w.y, *z = w.z;
                void* args[] = {&K, &x, &y, &z, &lam, &lstride, &nl, &active, &n4, &out, &ostride, &sign};
                // Mitsuba's Spectrum<Float, 4>: the kernel with the count compiled in
                const KernelId kr = nlam == 4 ? K_EVAL_SPEC_RAYS4_V4 : K_EVAL_SPEC_RAYS_V4;
                launch(e->fn_eval(kr, sign, s), grid_for(e->mod, kr, n4 / 4), s, args);
            }
            if (n4 < n) {
                const float *x = w.x + n4, *y = w.y + n4, *z = w.z + n4, *l = lam + n4;
                const uint8_t* a = active ? active + n4 : nullptr;
                float* o = out + n4;
                size_t rem = n - n4;
                void* args[] = {&K, &x, &y, &z, &l, &lstride, &nl, &a, &rem, &o, &ostride, &sign};
                launch(e->fn_eval(K_EVAL_SPEC_RAYS_V1, sign, s), grid_for(e->mod, K_EVAL_SPEC_RAYS_V1, rem), s, args);
            }
        }
    });
}

int sunsky_eval(const sunsky_emitter* e, sunsky_vec3_in wi, const float* lam, int nlam, size_t lstride,
                const uint8_t* active, size_t n, float* out, size_t ostride, void* stream) {
    SUNSKY_PHASE("EndpointEvaluate", "eval");
    return eval_impl(e, wi, lam, nlam, lstride, active, n, out, ostride, stream, -1.f);
}

int sunsky_eval_direction(const sunsky_emitter* e, sunsky_vec3_in d, const float* lam, int nlam, size_t lstride,
                          const uint8_t* active, size_t n, float* out, size_t ostride, void* stream) {
    SUNSKY_PHASE("EndpointEvaluate", "eval_direction");
    return eval_impl(e, d, lam, nlam, lstride, active, n, out, ostride, stream, 1.f);
}

int sunsky_eval_spectral_broadcast(const sunsky_emitter* e, sunsky_vec3_in w, const float* lam_host, int m,
                                   const uint8_t* active, size_t n, float* out, size_t ostride, void* stream) {
    SUNSKY_PHASE("EndpointEvaluate", "eval_spectral_broadcast");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (e->kargs.variant != kSpectral) return fail(SUNSKY_ERROR_INVALID_VALUE, "broadcast eval needs a spectral emitter");
    if (!lam_host || m < 1 || m > kMaxBroadcastLambda)
        return fail(SUNSKY_ERROR_INVALID_VALUE, "1..32 broadcast wavelengths required");
    if (n == 0) return SUNSKY_OK;
    if (!w.x || !w.y || !w.z || !out) return fail(SUNSKY_ERROR_INVALID_VALUE, "null ray / output pointer");
    if (m > 1 && ostride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "out_stride < n");
    LambdaSet L = make_lambda_set(lam_host, m);
    // The 11 model wavelengths 320:40:720 in order: compile-time channel kernel.
    bool nodes = m == kNbWavelengths;
    for (int k = 0; nodes && k < m; ++k) nodes = L.lo[k] == k && L.f[k] == 0.f;
    return guarded([&] {
        require_device(e);
        hipStream_t s = (hipStream_t)stream;
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        float sign = -1.f;
        bool vec = n >= 4 && aligned16(w.x) && aligned16(w.y) && aligned16(w.z) && aligned16(out) &&
                   (ostride % 4) == 0 && (!active || ((uintptr_t)active & 3u) == 0);
        size_t n4 = vec ? (n & ~(size_t)3) : 0;
        if (n4) {
            const float *x = w.x, *y = w.y, *z = w.z;
            void* args[] = {&K, &L, &x, &y, &z, &active, &n4, &out, &ostride, &sign};
            const unsigned grid = grid_for(e->mod, K_EVAL_SPEC_BCAST_V4, n4 / 4);
            const bool multi_step = n4 / 4 > (size_t)grid * kBlock;
            launch(e->fn(nodes ? K_EVAL_SPEC_NODES_V4 : K_EVAL_SPEC_BCAST_V4, s), grid, s, args,
                   nodes && multi_step ? kNodesLdsCap : 0u);
        }
        if (n4 < n) {
            const float *x = w.x + n4, *y = w.y + n4, *z = w.z + n4;
            const uint8_t* a = active ? active + n4 : nullptr;
            float* o = out + n4;
            size_t rem = n - n4;
            void* args[] = {&K, &L, &x, &y, &z, &a, &rem, &o, &ostride, &sign};
            launch(e->fn(K_EVAL_SPEC_BCAST_V1, s), grid_for(e->mod, K_EVAL_SPEC_BCAST_V1, rem), s, args);
        }
    });
}

int sunsky_sample_direction(const sunsky_emitter* e, const float* ux, const float* uy, sunsky_vec3_in it_p,
                            const float* lam, int nlam, size_t lstride, const uint8_t* active, size_t n,
                            sunsky_vec3_out ds_d, float* ds_pdf, float* ds_dist, sunsky_vec3_out ds_p,
                            float* weight, size_t wstride, void* stream) {
    SUNSKY_PHASE("EndpointSampleDirection", "sample_direction");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (n == 0) return SUNSKY_OK;
    const bool spec = e->kargs.variant == kSpectral;
    if (!ux || !uy || !ds_d.x || !ds_d.y || !ds_d.z || !ds_pdf || !weight)
        return fail(SUNSKY_ERROR_INVALID_VALUE, "null sample / output pointer");
    if (spec && (!lam || nlam < 1 || nlam > kMaxLambdaPerRay))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "spectral sample_direction needs 1..16 wavelength planes");
    if (wstride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "weight_stride < n");
    if ((it_p.x != nullptr) != (it_p.y != nullptr) || (it_p.x != nullptr) != (it_p.z != nullptr))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "it_p must be all-NULL or all-set");
    if ((ds_p.x != nullptr) != (ds_p.y != nullptr) || (ds_p.x != nullptr) != (ds_p.z != nullptr))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "ds_p must be all-NULL or all-set");
    return guarded([&] {
        require_device(e);
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        int nl = spec ? nlam : 0;
        void* args[] = {&K, &ux, &uy, (void*)&it_p.x, (void*)&it_p.y, (void*)&it_p.z, &lam, &lstride, &nl, &active, &n,
                        &ds_d.x, &ds_d.y, &ds_d.z, &ds_pdf, &ds_dist, &ds_p.x, &ds_p.y, &ds_p.z, &weight, &wstride};
        // the common call (no it.p, ds.dist, ds.p or mask) takes the kernel with those
        // paths compiled out: same results, no SGPR spills (sampling)
        const bool lean = !it_p.x && !ds_dist && !ds_p.x && !active;
        // SUNSKY_AMD_UNSORTED_SAMPLING=1: the unsorted LEAN kernels (A/B timing and the bitwise
        // sorted-vs-unsorted tests); read per call so a test can switch it
        const char* uns = std::getenv("SUNSKY_AMD_UNSORTED_SAMPLING");
        const bool unsorted = uns && uns[0] == '1';
        // SUNSKY_AMD_SORTED_GENERAL_SAMPLING=1: the masked general RGB call through the wave-sorted
        // kernel (10 % slower than the unsorted one; bitwise tests only)
        const char* sgs = std::getenv("SUNSKY_AMD_SORTED_GENERAL_SAMPLING");
        const bool sorted_general = sgs && sgs[0] == '1' && !unsorted;
        // spectral at Mitsuba's 4 wavelengths per sample: the wave-sorted kernel, LEAN or (no mask)
        // with ds.dist / ds.p from it.p read at the store stage.  RGB
        // without a mask (Mitsuba's DirectionSample call: it.p in, ds.dist / ds.p out) takes the
        // LEAN windows with each window's it.p loaded with its u, one window ahead (kSortPos); with
        // a mask, the unsorted general kernel.
        const KernelId k = spec ? (lean ? (nlam == 4 && !unsorted ? K_SAMPLE_DIRECTION_SPEC_LEAN4_SORTED
                                                                  : K_SAMPLE_DIRECTION_SPEC_LEAN)
                                        : (nlam == 4 && !active && !unsorted) ? K_SAMPLE_DIRECTION_SPEC_POS_SORTED
                                                                              : K_SAMPLE_DIRECTION_SPEC)
                                : (lean ? (unsorted ? K_SAMPLE_DIRECTION_RGB_LEAN_PLAIN : K_SAMPLE_DIRECTION_RGB_LEAN)
                                        : sorted_general ? K_SAMPLE_DIRECTION_RGB_FULL_SORTED
                                        : (!active && !unsorted) ? K_SAMPLE_DIRECTION_RGB_POS_SORTED
                                                                 : K_SAMPLE_DIRECTION_RGB);
        // the wave-sorted kernels: one wave takes a window of 4 (RGB) or 3 (spectral) x 64 samples
        const size_t items = (k == K_SAMPLE_DIRECTION_RGB_LEAN || k == K_SAMPLE_DIRECTION_RGB_FULL_SORTED ||
                              k == K_SAMPLE_DIRECTION_RGB_POS_SORTED) ? (n + 3) / 4
                             : (k == K_SAMPLE_DIRECTION_SPEC_LEAN4_SORTED || k == K_SAMPLE_DIRECTION_SPEC_POS_SORTED)
                                   ? (n + 2) / 3 : n;
        launch(e->fn(k, (hipStream_t)stream), grid_for(e->mod, k, items), (hipStream_t)stream, args);
    });
}

int sunsky_pdf_direction(const sunsky_emitter* e, sunsky_vec3_in d, const uint8_t* active, size_t n, float* pdf,
                         void* stream) {
    SUNSKY_PHASE("EndpointEvaluate", "pdf_direction");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (n == 0) return SUNSKY_OK;
    if (!d.x || !d.y || !d.z || !pdf) return fail(SUNSKY_ERROR_INVALID_VALUE, "null direction / output pointer");
    return guarded([&] {
        require_device(e);
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        hipStream_t s = (hipStream_t)stream;
        bool vec = n >= 4 && aligned16(d.x) && aligned16(d.y) && aligned16(d.z) && aligned16(pdf) &&
                   (!active || ((uintptr_t)active & 3u) == 0);
        size_t n4 = vec ? (n & ~(size_t)3) : 0;
        if (n4) {
            void* args[] = {&K, (void*)&d.x, (void*)&d.y, (void*)&d.z, &active, &n4, &pdf};
            launch(e->fn(K_PDF_DIRECTION_V4, s), grid_for(e->mod, K_PDF_DIRECTION_V4, n4 / 4), s, args);
        }
        if (n4 < n) {
            const float *x = d.x + n4, *y = d.y + n4, *z = d.z + n4;
            const uint8_t* a = active ? active + n4 : nullptr;
            float* p = pdf + n4;
            size_t rem = n - n4;
            void* args[] = {&K, &x, &y, &z, &a, &rem, &p};
            launch(e->fn(K_PDF_DIRECTION_V1, s), grid_for(e->mod, K_PDF_DIRECTION_V1, rem), s, args);
        }
    });
}

int sunsky_sample_ray(const sunsky_emitter* e, const float* wls, const float* s2x, const float* s2y,
                      const float* s3x, const float* s3y, const uint8_t* active, size_t n, sunsky_vec3_out o,
                      sunsky_vec3_out d, float* lam, size_t lstride, float* weight, size_t wstride, void* stream) {
    SUNSKY_PHASE("EndpointSampleRay", "sample_ray");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (n == 0) return SUNSKY_OK;
    if (!s2x || !s2y || !s3x || !s3y || !o.x || !o.y || !o.z || !d.x || !d.y || !d.z || !lam || !weight)
        return fail(SUNSKY_ERROR_INVALID_VALUE, "null sample / output pointer");
    if (e->kargs.variant == kSpectral && !wls) return fail(SUNSKY_ERROR_INVALID_VALUE, "null wavelength sample");
    if (lstride < n || wstride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "stride < n");
    return guarded([&] {
        require_device(e);
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        void* args[] = {&K, &wls, &s2x, &s2y, &s3x, &s3y, &active, &n, &o.x, &o.y, &o.z,
                        &d.x, &d.y, &d.z, &lam, &lstride, &weight, &wstride};
        // RGB without a mask: the wave-sorted kernel (one wave per window of 4 x 64 rays);
        // SUNSKY_AMD_UNSORTED_SAMPLING=1 keeps the unsorted one (A/B, the bitwise test)
        const char* uns = std::getenv("SUNSKY_AMD_UNSORTED_SAMPLING");
        const bool unsorted = uns && uns[0] == '1';
        const KernelId k = e->kargs.variant == kSpectral ? K_SAMPLE_RAY_SPEC
                           : (!active && !unsorted) ? K_SAMPLE_RAY_RGB_SORTED : K_SAMPLE_RAY_RGB;
        launch(e->fn(k, (hipStream_t)stream), grid_for(e->mod, k, k == K_SAMPLE_RAY_RGB_SORTED ? (n + 3) / 4 : n), (hipStream_t)stream,
               args);
    });
}

int sunsky_sample_wavelengths(const sunsky_emitter* e, sunsky_vec3_in w, const float* sample, const uint8_t* active,
                              size_t n, float* lam, size_t lstride, float* weight, size_t wstride, void* stream) {
    SUNSKY_PHASE("EndpointSampleRay", "sample_wavelengths");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (n == 0) return SUNSKY_OK;
    if (!w.x || !w.y || !w.z || !lam || !weight) return fail(SUNSKY_ERROR_INVALID_VALUE, "null pointer");
    if (e->kargs.variant == kSpectral && !sample) return fail(SUNSKY_ERROR_INVALID_VALUE, "null sample");
    if (lstride < n || wstride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "stride < n");
    return guarded([&] {
        require_device(e);
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        void* args[] = {&K, (void*)&w.x, (void*)&w.y, (void*)&w.z, &sample, &active, &n, &lam, &lstride, &weight, &wstride};
        const KernelId k = e->kargs.variant == kSpectral ? K_SAMPLE_WAVELENGTHS_SPEC : K_SAMPLE_WAVELENGTHS_RGB;
        launch(e->fn(k, (hipStream_t)stream), grid_for(e->mod, k, n), (hipStream_t)stream, args);
    });
}

int sunsky_eval_jvp(const sunsky_emitter* e, int param, const float* tangent, int tangent_count, sunsky_vec3_in wi,
                    const float* lam, int nlam, size_t lstride, const uint8_t* active, size_t n, float* out,
                    float* d_out, size_t ostride, void* stream) {
    SUNSKY_PHASE("EndpointEvaluate", "eval_jvp");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (!tangent) return fail(SUNSKY_ERROR_INVALID_VALUE, "null tangent");
    const bool spec = e->kargs.variant == kSpectral;
    if (spec && (!lam || nlam < 1 || nlam > kMaxLambdaPerRay))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "spectral eval needs 1..16 wavelength planes");
    const size_t nout = spec ? (size_t)nlam : 3;
    if (n && (!wi.x || !wi.y || !wi.z || !out || !d_out))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "null ray / output pointer");
    if (n && nout > 1 && ostride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "out_stride < n");
    if (n && spec && nlam > 1 && lstride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "wl_stride < n");
    return guarded([&] {
        std::vector<float> key(tangent, tangent + std::max(0, tangent_count));
        key.push_back((float)param);
        const bool stage = !e->d_jvp || e->jvp_rev != e->rev || key != e->jvp_key;
        TangentStage ts;
        if (stage || n == 0) ts = e->model->tangent_stage(param, tangent, tangent_count);   // validates param / count
        if (n == 0) return;
        require_device(e);
        hipStream_t st = (hipStream_t)stream;
        DeviceScope dev_scope(e->device);
        e->ad_begin(st);   // ordered after the previous AD call (which may read d_jvp), any stream
        if (stage) {   // the tangent tables, staged on the device (sunsky_stage_tangent)
            if (!e->d_jvp) hip_check(hipMalloc(&e->d_jvp, sizeof(float) * sunsky_emitter::kJvpFloats), "hipMalloc");
            TangentArgs A = e->tangent_args(e->d_jvp, 1, kTanSunLocal, 0, kJvpSunOffset, sunsky_emitter::kJvpFloats);
            A.st[0] = ts;
            e->stage_tangent(A, st);
            e->jvp_key = key;
            e->jvp_rev = e->rev;
        }
        const SunskyKArgs* K = e->d_state;
        const float* jvp = e->d_jvp;
        const float *x = wi.x, *y = wi.y, *z = wi.z;
        float sign = -1.f;
        if (!spec) {
            void* args[] = {&K, &jvp, &x, &y, &z, &active, &n, &out, &d_out, &ostride, &sign};
            launch(e->mod->jvp_rgb, grid_for(e->mod, K_EVAL_RGB_V1, n), (hipStream_t)stream, args);
        } else {
            int nl = nlam;
            void* args[] = {&K, &jvp, &x, &y, &z, &lam, &lstride, &nl, &active, &n, &out, &d_out, &ostride, &sign};
            launch(e->mod->jvp_spec, grid_for(e->mod, K_EVAL_SPEC_RAYS_V1, n), (hipStream_t)stream, args);
        }
        e->ad_end(st);
    });
}

int sunsky_emitter_tangent_tables(const sunsky_emitter* e, int param, const float* tangent, int tangent_count,
                                  int on_device, float* out, size_t cap, size_t* count) {
    if (!e || !count) return fail(SUNSKY_ERROR_INVALID_VALUE, "null argument");
    if (!tangent) return fail(SUNSKY_ERROR_INVALID_VALUE, "null tangent");
    return guarded([&] {
        e->sync_host();
        const int total = sunsky_emitter::kJvpFloats;
        static_assert(sunsky_emitter::kJvpFloats == SUNSKY_TANGENT_FLOATS, "tangent buffer layout");
        std::vector<float> v(total, 0.f);
        if (on_device) {
            require_device(e);
            DeviceScope g(e->device);
            float* d = nullptr;
            hip_check(hipMalloc(&d, sizeof(float) * total), "hipMalloc");
            TangentArgs A = e->tangent_args(d, 1, kTanSunLocal, 0, kJvpSunOffset, total);
            A.st[0] = e->model->tangent_stage(param, tangent, tangent_count);
            e->stage_tangent(A, nullptr);
            hipError_t rc = hipMemcpy(v.data(), d, sizeof(float) * total, hipMemcpyDeviceToHost);
            (void)hipFree(d);
            hip_check(rc, "hipMemcpy");
        } else {
            const EvalTangent t = e->model->eval_tangent(param, tangent, tangent_count);
            std::memcpy(v.data(), t.dsky.data(), sizeof(float) * t.dsky.size());
            std::memcpy(v.data() + kTanSunLocal, t.dsun_local, 3 * sizeof(float));
            std::memcpy(v.data() + kJvpSunOffset, t.dsun.data(), sizeof(float) * t.dsun.size());
        }
        *count = v.size();
        if (out) std::memcpy(out, v.data(), sizeof(float) * std::min(cap, v.size()));
    });
}

int sunsky_eval_vjp(const sunsky_emitter* e, sunsky_vec3_in wi, const float* lam, int nlam, size_t lstride,
                    const uint8_t* active, size_t n, const float* d_out, size_t ostride, float* grad, void* stream) {
    SUNSKY_PHASE("EndpointEvaluate", "eval_vjp");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (!grad) return fail(SUNSKY_ERROR_INVALID_VALUE, "null gradient buffer");
    const bool spec = e->kargs.variant == kSpectral;
    if (n == 0) return SUNSKY_OK;
    if (spec && (!lam || nlam < 1 || nlam > kMaxLambdaPerRay))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "spectral eval needs 1..16 wavelength planes");
    const size_t nout = spec ? (size_t)nlam : 3;
    if (!wi.x || !wi.y || !wi.z || !d_out) return fail(SUNSKY_ERROR_INVALID_VALUE, "null ray / cotangent pointer");
    if (nout > 1 && ostride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "out_stride < n");
    if (spec && nlam > 1 && lstride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "wl_stride < n");
    return guarded([&] {
        require_device(e);
        // basis tangents: turbidity, albedo (all channels at once: channel c's tables depend on
        // albedo[c] only, so the all-ones tangent is the diagonal), sun_direction x / y / z
        const SunskyModel& M = *e->model;
        const int nch = M.nch();
        // 6 workgroups per CU (the RGB kernel holds 3 per CU at a time, 134 VGPRs): few per-block
        // partials, so the one-workgroup reduce below stays short (16384 partials took 0.3 ms)
        const unsigned grid = (unsigned)std::max<size_t>(
            1, std::min<size_t>((n + kBlock - 1) / kBlock, (size_t)e->mod->cu_count * 6));
        hipStream_t st = (hipStream_t)stream;
        DeviceScope dev_scope(e->device);
        const bool stage = !e->d_vjp || e->vjp_rev != e->rev;
        const bool had_ad = e->ad_done != nullptr;
        e->ad_begin(st);   // ordered after the previous AD call (d_vjp / d_partials readers), any stream
        if (e->partials_cap < grid) {
            // the host frees the old partials only once the previous AD call is done with them
            if (had_ad) hip_check(hipEventSynchronize(e->ad_done), "hipEventSynchronize");
            if (e->d_partials) hip_check(hipFree(e->d_partials), "hipFree");
            e->d_partials = nullptr;
            hip_check(hipMalloc(&e->d_partials, sizeof(float) * 16 * grid), "hipMalloc");
            e->partials_cap = grid;
        }
        if (stage) {   // the 5 basis tangents, staged on the device (sunsky_stage_tangent)
            if (!e->d_vjp) hip_check(hipMalloc(&e->d_vjp, sizeof(float) * sunsky_emitter::kVjpFloats), "hipMalloc");
            const int nb = M.active_record() ? 2 : kVjpBases;   // sun_direction is not exposed in time mode
            TangentArgs A = e->tangent_args(e->d_vjp, nb, kVjpSunLocal, 2, kVjpSunOffset, sunsky_emitter::kVjpFloats);
            const float one = 1.f;
            A.st[0] = M.tangent_stage(kJvpTurbidity, &one, 1);
            std::vector<float> ones(nch, 1.f);
            A.st[1] = M.tangent_stage(kJvpAlbedo, ones.data(), nch);
            for (int k = 0; k + 2 < nb; ++k) {
                float axis[3] = {0.f, 0.f, 0.f};
                axis[k] = 1.f;
                A.st[2 + k] = M.tangent_stage(kJvpSunDirection, axis, 3);
            }
            if (nb == kVjpBases) {
                // the sky tables of sun axis k are d eta_k times those of a unit elevation
                // tangent: basis 2 holds the latter and the kernels scale by d eta_k
                // (kVjpSunEta), one sky tangent per channel for the 3 axes instead of 3
                A.eta_off = kVjpSunEta;
                A.st[2].dx = A.st[2].dx_per_eta;
                A.nsky = 3;   // the sky blocks of bases 3 and 4 are never read: written 0, not staged
            }
            e->stage_tangent(A, st);
            e->vjp_rev = e->rev;
        }
        const SunskyKArgs* K = e->d_state;
        const float* vjp = e->d_vjp;
        float* partials = e->d_partials;
        const float *x = wi.x, *y = wi.y, *z = wi.z;
        float sign = -1.f;
        if (!spec) {
            void* args[] = {&K, &vjp, &x, &y, &z, &active, &n, &d_out, &ostride, &sign, &partials};
            launch(e->mod->vjp_rgb, grid, st, args);
        } else {
            int nl = nlam;
            void* args[] = {&K, &vjp, &x, &y, &z, &lam, &lstride, &nl, &active, &n, &d_out, &ostride, &sign, &partials};
            launch(e->mod->vjp_spec, grid, st, args);
        }
        unsigned nb = grid;
        void* rargs[] = {&partials, &nb, &grad};
        hip_check(hipModuleLaunchKernel(e->mod->grad_reduce, 1, 1, 1, 256, 1, 1, 0, st, rargs, nullptr),
                  "hipModuleLaunchKernel");
        e->ad_end(st);
    });
}

int sunsky_bake_latlong(const sunsky_emitter* e, int width, int height, float theta0, float theta1, float phi0,
                        float phi1, const float* lam_host, int m, float* out, size_t ostride, void* stream) {
    SUNSKY_PHASE("EndpointEvaluate", "bake_latlong");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (width < 1 || height < 1) return fail(SUNSKY_ERROR_INVALID_VALUE, "image size must be >= 1 x 1");
    if ((int64_t)width * height >= (int64_t)1 << 31) return fail(SUNSKY_ERROR_INVALID_VALUE, "image larger than 2^31 pixels");
    const bool spec = e->kargs.variant == kSpectral;
    if (spec && (!lam_host || m < 1 || m > kMaxBroadcastLambda))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "1..32 wavelengths required for a spectral bake");
    if (!spec && lam_host && m) return fail(SUNSKY_ERROR_INVALID_VALUE, "RGB bake takes no wavelengths");
    const size_t n = (size_t)width * (size_t)height;
    if (!out) return fail(SUNSKY_ERROR_INVALID_VALUE, "null output pointer");
    if (ostride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "out_stride < width * height");
    // dr::linspace(start, end, count): step = (end - start) / (count - 1) in fp32
    LatLong G = {width, height, theta0, height > 1 ? (theta1 - theta0) / (float)(height - 1) : 0.f,
                 phi0, width > 1 ? (phi1 - phi0) / (float)(width - 1) : 0.f, nullptr};
    return guarded([&] {
        require_device(e);
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        hipStream_t s = (hipStream_t)stream;
        const size_t need = 2 * (size_t)width + 2 * (size_t)height;
        // the angle tables are per emitter: order this bake after the previous one (any
        // stream), so a bake on another stream cannot rewrite them under a running kernel
        const bool had_bake = e->bake_done != nullptr;
        if (!had_bake) hip_check(hipEventCreateWithFlags(&e->bake_done, hipEventDisableTiming), "hipEventCreate");
        else hip_check(hipStreamWaitEvent(s, e->bake_done, 0), "hipStreamWaitEvent");
        if (e->bake_cap < need) {
            // the host frees the old tables only once the previous bake is done with them
            if (had_bake) hip_check(hipEventSynchronize(e->bake_done), "hipEventSynchronize");
            if (e->d_bake) hip_check(hipFree(e->d_bake), "hipFree");
            e->d_bake = nullptr;
            hip_check(hipMalloc(&e->d_bake, sizeof(float) * need), "hipMalloc");
            e->bake_cap = need;
        }
        float* tab = e->d_bake;
        G.tab = tab;
        {
            void* targs[] = {&G, &tab};
            const unsigned tg = (unsigned)((std::max(width, height) + kBlock - 1) / kBlock);
            launch(e->mod->latlong_tables, tg, s, targs);
        }
        if (!spec) {
            void* args[] = {&K, &G, &out, &ostride};
            launch(e->fn(K_BAKE_RGB, s), grid_for(e->mod, K_BAKE_RGB, (size_t)((width + 3) / 4) * height), s, args);
        } else {
            LambdaSet L = make_lambda_set(lam_host, m);
            void* args[] = {&K, &G, &L, &out, &ostride};
            launch(e->fn(K_BAKE_SPEC, s), grid_for(e->mod, K_BAKE_SPEC, n), s, args);
        }
        hip_check(hipEventRecord(e->bake_done, s), "hipEventRecord");
    });
}

int sunsky_direct_diffuse(const sunsky_emitter* e, sunsky_vec3_in nrm, const float* rho, const float* lam, int nlam,
                          size_t lstride, uint32_t seed, uint32_t spp, const uint8_t* vis, size_t vstride, size_t n,
                          float* out, size_t ostride, void* stream) {
    SUNSKY_PHASE("SamplingIntegratorSample", "direct_diffuse");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (n == 0) return SUNSKY_OK;
    const bool spec = e->kargs.variant == kSpectral;
    if (!nrm.x || !nrm.y || !nrm.z || !out) return fail(SUNSKY_ERROR_INVALID_VALUE, "null normal / output pointer");
    if (spp < 1) return fail(SUNSKY_ERROR_INVALID_VALUE, "spp must be >= 1");
    if (n > 0xffffffffull) return fail(SUNSKY_ERROR_INVALID_VALUE, "more than 2^32 points (the sampler's lane index is 32-bit)");
    if (spec && (!lam || nlam < 1 || nlam > 4))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "spectral direct lighting needs 1..4 wavelength planes");
    if (!spec && (lam || nlam)) return fail(SUNSKY_ERROR_INVALID_VALUE, "RGB direct lighting takes no wavelengths");
    if (ostride < n || (spec && lstride < n)) return fail(SUNSKY_ERROR_INVALID_VALUE, "stride < n");
    if (vis && vstride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "vis_stride < n");
    return guarded([&] {
        require_device(e);
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        int nl = spec ? nlam : 0;
        void* args[] = {&K, (void*)&nrm.x, (void*)&nrm.y, (void*)&nrm.z, &rho, &lam, &lstride, &nl, &seed, &spp, &vis,
                        &vstride, &n, &out, &ostride};
        const KernelId k = spec ? K_DIRECT_DIFFUSE_SPEC : K_DIRECT_DIFFUSE_RGB;
        launch(e->fn(k, (hipStream_t)stream), grid_for(e->mod, k, n), (hipStream_t)stream, args);
    });
}

int sunsky_direct_diffuse_rays(const sunsky_emitter* e, sunsky_vec3_in nrm, uint32_t seed, uint32_t spp, size_t n,
                               sunsky_vec3_out em, sunsky_vec3_out bs, size_t rstride, void* stream) {
    SUNSKY_PHASE("SamplingIntegratorSample", "direct_diffuse_rays");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (n == 0) return SUNSKY_OK;
    if (!nrm.x || !nrm.y || !nrm.z) return fail(SUNSKY_ERROR_INVALID_VALUE, "null normal pointer");
    if (!em.x || !em.y || !em.z || !bs.x || !bs.y || !bs.z) return fail(SUNSKY_ERROR_INVALID_VALUE, "null ray pointer");
    if (spp < 1) return fail(SUNSKY_ERROR_INVALID_VALUE, "spp must be >= 1");
    if (n > 0xffffffffull) return fail(SUNSKY_ERROR_INVALID_VALUE, "more than 2^32 points (the sampler's lane index is 32-bit)");
    if (rstride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "ray_stride < n");
    return guarded([&] {
        require_device(e);
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        void* args[] = {&K, (void*)&nrm.x, (void*)&nrm.y, (void*)&nrm.z, &seed, &spp, &n, &em.x, &em.y, &em.z,
                        &bs.x, &bs.y, &bs.z, &rstride};
        launch(e->fn(K_DIRECT_DIFFUSE_RAYS, (hipStream_t)stream), grid_for(e->mod, K_DIRECT_DIFFUSE_RAYS, n), (hipStream_t)stream, args);
    });
}

// The rough conductor of the glossy caller (mirrors the kernel-side ConductorArgs; alpha_v
// after the IOR so the isotropic layout's offsets stay)
struct ConductorArgs {
    int type;
    float alpha_u;
    float eta[4], k[4];
    float alpha_v;
};
static_assert(sizeof(ConductorArgs) == 44 && offsetof(ConductorArgs, alpha_v) == 40, "ConductorArgs layout");

static int conductor_args(const sunsky_emitter* e, int distribution, float alpha_u, float alpha_v, const float* eta,
                          const float* k, ConductorArgs* c) {
    if (distribution != SUNSKY_MICROFACET_BECKMANN && distribution != SUNSKY_MICROFACET_GGX)
        return fail(SUNSKY_ERROR_INVALID_VALUE, "distribution must be SUNSKY_MICROFACET_BECKMANN or _GGX");
    if (!(alpha_u > 0.f) || !(alpha_v > 0.f) || std::isinf(alpha_u) || std::isinf(alpha_v))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "alpha (alpha_u, alpha_v) must be finite and > 0");
    if (!eta || !k) return fail(SUNSKY_ERROR_INVALID_VALUE, "null eta / k");
    std::memset(c, 0, sizeof(*c));
    c->type = distribution;
    // microfacet.h clamps alpha_u, alpha_v to 1e-4 (MicrofacetDistribution::configure, :424-428)
    c->alpha_u = std::max(alpha_u, 1e-4f);
    c->alpha_v = std::max(alpha_v, 1e-4f);
    const int nc = e->kargs.variant == kSpectral ? 1 : 3;
    for (int i = 0; i < nc; ++i) { c->eta[i] = eta[i]; c->k[i] = k[i]; }
    return SUNSKY_OK;
}

static int direct_conductor_impl(const sunsky_emitter* e, sunsky_vec3_in nrm, sunsky_vec3_in wi, int distribution,
                                 float alpha_u, float alpha_v, const float* eta, const float* k, const float* lam,
                                 int nlam, size_t lstride, uint32_t seed, uint32_t spp, const uint8_t* vis,
                                 size_t vstride, size_t n, float* out, size_t ostride, void* stream) {
    SUNSKY_PHASE("SamplingIntegratorSample", "direct_conductor");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    ConductorArgs C;
    int rc = conductor_args(e, distribution, alpha_u, alpha_v, eta, k, &C);
    if (rc != SUNSKY_OK) return rc;
    if (n == 0) return SUNSKY_OK;
    const bool spec = e->kargs.variant == kSpectral;
    if (!nrm.x || !nrm.y || !nrm.z || !wi.x || !wi.y || !wi.z || !out)
        return fail(SUNSKY_ERROR_INVALID_VALUE, "null normal / view direction / output pointer");
    if (spp < 1) return fail(SUNSKY_ERROR_INVALID_VALUE, "spp must be >= 1");
    if (n > 0xffffffffull) return fail(SUNSKY_ERROR_INVALID_VALUE, "more than 2^32 points (the sampler's lane index is 32-bit)");
    if (spec && (!lam || nlam < 1 || nlam > 4))
        return fail(SUNSKY_ERROR_INVALID_VALUE, "spectral direct lighting needs 1..4 wavelength planes");
    if (!spec && (lam || nlam)) return fail(SUNSKY_ERROR_INVALID_VALUE, "RGB direct lighting takes no wavelengths");
    if (ostride < n || (spec && lstride < n)) return fail(SUNSKY_ERROR_INVALID_VALUE, "stride < n");
    if (vis && vstride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "vis_stride < n");
    return guarded([&] {
        require_device(e);
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        int nl = spec ? nlam : 0;
        void* args[] = {&K, &C, (void*)&nrm.x, (void*)&nrm.y, (void*)&nrm.z, (void*)&wi.x, (void*)&wi.y, (void*)&wi.z,
                        &lam, &lstride, &nl, &seed, &spp, &vis, &vstride, &n, &out, &ostride};
        const KernelId kid = spec ? K_DIRECT_CONDUCTOR_SPEC : K_DIRECT_CONDUCTOR_RGB;
        launch(e->fn(kid, (hipStream_t)stream), grid_for(e->mod, kid, n), (hipStream_t)stream, args);
    });
}

static int direct_conductor_rays_impl(const sunsky_emitter* e, sunsky_vec3_in nrm, sunsky_vec3_in wi,
                                      int distribution, float alpha_u, float alpha_v, const float* eta, const float* k,
                                      uint32_t seed, uint32_t spp, size_t n, sunsky_vec3_out em, sunsky_vec3_out bs,
                                      float* bw, size_t rstride, void* stream) {
    SUNSKY_PHASE("SamplingIntegratorSample", "direct_conductor_rays");
    if (!e) return fail(SUNSKY_ERROR_INVALID_VALUE, "null emitter");
    if (bw && (!eta || !k)) return fail(SUNSKY_ERROR_INVALID_VALUE, "the BSDF weights need eta / k");
    const float one[3] = {1.f, 1.f, 1.f};
    ConductorArgs C;
    // the directions do not depend on eta / k; the weights do
    int rc = conductor_args(e, distribution, alpha_u, alpha_v, bw ? eta : one, bw ? k : one, &C);
    if (rc != SUNSKY_OK) return rc;
    int nw = e->kargs.variant == kSpectral ? 1 : 3;
    if (n == 0) return SUNSKY_OK;
    if (!nrm.x || !nrm.y || !nrm.z || !wi.x || !wi.y || !wi.z)
        return fail(SUNSKY_ERROR_INVALID_VALUE, "null normal / view direction pointer");
    if (!em.x || !em.y || !em.z || !bs.x || !bs.y || !bs.z) return fail(SUNSKY_ERROR_INVALID_VALUE, "null ray pointer");
    if (spp < 1) return fail(SUNSKY_ERROR_INVALID_VALUE, "spp must be >= 1");
    if (n > 0xffffffffull) return fail(SUNSKY_ERROR_INVALID_VALUE, "more than 2^32 points (the sampler's lane index is 32-bit)");
    if (rstride < n) return fail(SUNSKY_ERROR_INVALID_VALUE, "ray_stride < n");
    return guarded([&] {
        require_device(e);
        DeviceScope dev_scope(e->device);
        const SunskyKArgs* K = e->d_state;
        void* args[] = {&K, &C, (void*)&nrm.x, (void*)&nrm.y, (void*)&nrm.z, (void*)&wi.x, (void*)&wi.y, (void*)&wi.z,
                        &seed, &spp, &n, &em.x, &em.y, &em.z, &bs.x, &bs.y, &bs.z, &rstride, &bw, &nw};
        launch(e->fn(K_DIRECT_CONDUCTOR_RAYS, (hipStream_t)stream), grid_for(e->mod, K_DIRECT_CONDUCTOR_RAYS, n), (hipStream_t)stream, args);
    });
}

int sunsky_direct_conductor(const sunsky_emitter* e, sunsky_vec3_in nrm, sunsky_vec3_in wi, int distribution,
                            float alpha, const float* eta, const float* k, const float* lam, int nlam, size_t lstride,
                            uint32_t seed, uint32_t spp, const uint8_t* vis, size_t vstride, size_t n, float* out,
                            size_t ostride, void* stream) {
    return direct_conductor_impl(e, nrm, wi, distribution, alpha, alpha, eta, k, lam, nlam, lstride, seed, spp, vis,
                                 vstride, n, out, ostride, stream);
}

int sunsky_direct_conductor_aniso(const sunsky_emitter* e, sunsky_vec3_in nrm, sunsky_vec3_in wi, int distribution,
                                  float alpha_u, float alpha_v, const float* eta, const float* k, const float* lam,
                                  int nlam, size_t lstride, uint32_t seed, uint32_t spp, const uint8_t* vis,
                                  size_t vstride, size_t n, float* out, size_t ostride, void* stream) {
    return direct_conductor_impl(e, nrm, wi, distribution, alpha_u, alpha_v, eta, k, lam, nlam, lstride, seed, spp,
                                 vis, vstride, n, out, ostride, stream);
}

int sunsky_direct_conductor_rays(const sunsky_emitter* e, sunsky_vec3_in nrm, sunsky_vec3_in wi, int distribution,
                                 float alpha, const float* eta, const float* k, uint32_t seed, uint32_t spp, size_t n,
                                 sunsky_vec3_out em, sunsky_vec3_out bs, float* bw, size_t rstride, void* stream) {
    return direct_conductor_rays_impl(e, nrm, wi, distribution, alpha, alpha, eta, k, seed, spp, n, em, bs, bw, rstride,
                                      stream);
}

int sunsky_direct_conductor_rays_aniso(const sunsky_emitter* e, sunsky_vec3_in nrm, sunsky_vec3_in wi,
                                       int distribution, float alpha_u, float alpha_v, const float* eta,
                                       const float* k, uint32_t seed, uint32_t spp, size_t n, sunsky_vec3_out em,
                                       sunsky_vec3_out bs, float* bw, size_t rstride, void* stream) {
    return direct_conductor_rays_impl(e, nrm, wi, distribution, alpha_u, alpha_v, eta, k, seed, spp, n, em, bs, bw,
                                      rstride, stream);
}

int sunsky_sample_position(const sunsky_emitter* e) {
    (void)e;
    return fail(SUNSKY_ERROR_NOT_IMPLEMENTED, "sample_position");
}

int sunsky_array_from_file(const char* path, int file_dtype, double* out, size_t cap, size_t* count, uint64_t* shape,
                           int* ndims) {
    if (!path || !count) return fail(SUNSKY_ERROR_INVALID_VALUE, "null argument");
    Table t;
    std::string err;
    if (!read_array_file(path, file_dtype, &t, &err))
        return fail(err.find("does not exist") != std::string::npos ? SUNSKY_ERROR_FILE : SUNSKY_ERROR_FORMAT, err);
    *count = t.size();
    if (out) std::memcpy(out, t.data.data(), sizeof(double) * std::min(cap, t.size()));
    if (ndims) *ndims = (int)t.shape.size();
    if (shape)
        for (size_t i = 0; i < t.shape.size() && i < 16; ++i) shape[i] = t.shape[i];
    return SUNSKY_OK;
}

int sunsky_array_to_file(const char* path, const float* data, size_t count, const uint64_t* shape, int ndims) {
    if (!path || (!data && count)) return fail(SUNSKY_ERROR_INVALID_VALUE, "null argument");
    std::vector<size_t> sh;
    for (int i = 0; i < ndims; ++i) sh.push_back((size_t)shape[i]);
    std::string err;
    if (!write_array_file(path, data, count, sh.empty() ? nullptr : sh.data(), (int)sh.size(), &err))
        return fail(SUNSKY_ERROR_FILE, err);
    return SUNSKY_OK;
}

const char* plugin_name(void) { return "sunsky"; }
const char* plugin_descr(void) { return "Sun and Sky dome background emitter (MI355X)"; }

int sunsky_hosek_sun_rad(const char* dataset_path, double turbidity, double wavelength, double elevation,
                         double gamma, double* out) {
    if (!out) return fail(SUNSKY_ERROR_INVALID_VALUE, "null output pointer");
    return guarded([&] {
        std::string ds = dataset_path && *dataset_path ? std::string(dataset_path) : default_pack_path();
        *out = hosek_solar_radiance(ds, turbidity, wavelength, elevation, gamma);
    });
}

int sunsky_default_dataset_path(char* buf, size_t cap) {
    if (!buf || !cap) return fail(SUNSKY_ERROR_INVALID_VALUE, "null buffer");
    std::snprintf(buf, cap, "%s", default_pack_path().c_str());
    return SUNSKY_OK;
}

}  // extern "C"
