// sunsky_comm.cpp -- the one data-path exchange of the multi-GPU workload
// (BASELINE.json configs[4]): every rank's radiance shard gathered
// into the root's final [C][N] planes over RCCL (xGMI between the GPUs of a node).
//
// The reference's equivalent is a single ncclGather of equal, padded shards
// (rccl.h:745-746) followed by a re-layout; here each rank's C planes go straight to
// their column range of the root's planes with grouped ncclSend / ncclRecv, so the
// shards need no padding and the root no concatenation copy.  RCCL is opened with
// dlopen on first use: the eval / sampling path never needs it, and inside a PyTorch
// process the soname resolves to the RCCL torch already loaded (one RCCL per process).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <type_traits>
#include <string>
#include <vector>

#include "sunsky_amd.h"
#include "sunsky_profiler.h"
#include "sunsky_errors.h"

using namespace sunsky::capi;

namespace {

// The RCCL symbols used here (rccl.h): opaque handles, results as int.
typedef struct ncclComm* ncclComm_t;
typedef int ncclResult_t;
constexpr int kNcclSuccess = 0;
constexpr int kNcclFloat32 = 7;     // ncclFloat32, rccl.h:466
struct ncclUniqueId { char internal[SUNSKY_COMM_ID_BYTES]; };

struct Rccl {
    void* so = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    static std::string err;
    std::call_once(once, [] {
        // SUNSKY_AMD_RCCL: the RCCL library to use, by path (a specific RCCL build; the tests'
        // multi-process double on a one-GPU box).  Only that one is tried.
        const char* forced = std::getenv("SUNSKY_AMD_RCCL");
        if (forced && *forced) {
            r.so = dlopen(forced, RTLD_NOW | RTLD_LOCAL);
            if (!r.so) {
                err = std::string("RCCL not found (dlopen SUNSKY_AMD_RCCL=") + forced + "): " + dlerror();
                return;
            }
        }
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            if (r.so) break;
            r.so = dlopen(name, RTLD_NOW | RTLD_LOCAL);
        }
        if (!r.so) {
            err = std::string("RCCL not found (dlopen librccl.so.1): ") + dlerror();
            return;
        }
        auto sym = [&](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(r.so, name));
            if (!fp && err.empty()) err = std::string("RCCL symbol missing: ") + name;
        };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.GetErrorString, "ncclGetErrorString");
    });
    if (!err.empty()) throw CommError(err);
    return r;
}

void nccl_check(ncclResult_t res, const char* what) {
    if (res != kNcclSuccess) {
        const char* msg = rccl().GetErrorString ? rccl().GetErrorString(res) : "unknown";
        throw CommError(std::string(what) + ": " + msg);
    }
}

}  // namespace

struct sunsky_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1, device = 0;
};

extern "C" {

int sunsky_comm_get_unique_id(unsigned char id[SUNSKY_COMM_ID_BYTES]) {
    if (!id) return fail(SUNSKY_ERROR_INVALID_VALUE, "null id buffer");
    return guarded([&] {
        ncclUniqueId u;
        nccl_check(rccl().GetUniqueId(&u), "ncclGetUniqueId");
        std::memcpy(id, u.internal, SUNSKY_COMM_ID_BYTES);
    });
}

int sunsky_comm_create(const unsigned char id[SUNSKY_COMM_ID_BYTES], int nranks, int rank, sunsky_comm** out) {
    if (!id || !out) return fail(SUNSKY_ERROR_INVALID_VALUE, "null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(SUNSKY_ERROR_INVALID_VALUE, "invalid rank / nranks");
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<sunsky_comm> c(new sunsky_comm());
        hip_check(hipGetDevice(&c->device), "hipGetDevice");
        ncclUniqueId u;
        std::memcpy(u.internal, id, SUNSKY_COMM_ID_BYTES);
        nccl_check(rccl().CommInitRank(&c->comm, nranks, u, rank), "ncclCommInitRank");
        c->rank = rank;
        c->nranks = nranks;
        *out = c.release();
    });
}

void sunsky_comm_destroy(sunsky_comm* c) {
    if (!c) return;
    if (c->comm) {
        try {
            (void)rccl().CommDestroy(c->comm);
        } catch (...) {
        }
    }
    delete c;
}

int sunsky_comm_info(const sunsky_comm* c, int* rank, int* nranks, int* device) {
    if (!c) return fail(SUNSKY_ERROR_INVALID_VALUE, "null communicator");
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    if (device) *device = c->device;
    return SUNSKY_OK;
}

int sunsky_gather_radiance(sunsky_comm* c, int root, const float* send, size_t send_stride, int nplanes,
                           const size_t* counts, float* recv, size_t recv_stride, void* stream) {
    SUNSKY_PHASE("Gather", "gather_radiance");
    if (!c || !counts) return fail(SUNSKY_ERROR_INVALID_VALUE, "null communicator / counts");
    if (root < 0 || root >= c->nranks) return fail(SUNSKY_ERROR_INVALID_VALUE, "invalid root rank");
    if (nplanes < 1) return fail(SUNSKY_ERROR_INVALID_VALUE, "nplanes must be >= 1");
    std::vector<size_t> offset(c->nranks + 1, 0);
    for (int r = 0; r < c->nranks; ++r) offset[r + 1] = offset[r] + counts[r];
    const size_t mine = counts[c->rank];
    if (mine && !send) return fail(SUNSKY_ERROR_INVALID_VALUE, "null send buffer");
    if (nplanes > 1 && mine && send_stride < mine) return fail(SUNSKY_ERROR_INVALID_VALUE, "send_stride < shard size");
    if (c->rank == root) {
        if (!recv && offset[c->nranks]) return fail(SUNSKY_ERROR_INVALID_VALUE, "null receive buffer on root");
        if (nplanes > 1 && recv_stride < offset[c->nranks])
            return fail(SUNSKY_ERROR_INVALID_VALUE, "recv_stride < total rays");
    }
    return guarded([&] {
        int cur = 0;
        hip_check(hipGetDevice(&cur), "hipGetDevice");
        if (cur != c->device) hip_check(hipSetDevice(c->device), "hipSetDevice");
        struct Restore {
            int dev, prev;
            ~Restore() { if (dev != prev) (void)hipSetDevice(prev); }
        } restore{c->device, cur};
        hipStream_t s = (hipStream_t)stream;
        const Rccl& R = rccl();
        if (c->rank == root) {
            // own shard: a device copy into its columns (skipped when already in place)
            for (int p = 0; p < nplanes && mine; ++p) {
                float* dst = recv + (size_t)p * recv_stride + offset[root];
                const float* src = send + (size_t)p * send_stride;
                if (dst != src)
                    hip_check(hipMemcpyAsync(dst, src, sizeof(float) * mine, hipMemcpyDeviceToDevice, s),
                              "hipMemcpyAsync");
            }
        }
        if (c->nranks == 1) return;
        nccl_check(R.GroupStart(), "ncclGroupStart");
        if (c->rank == root) {
            for (int r = 0; r < c->nranks; ++r) {
                if (r == root || counts[r] == 0) continue;
                for (int p = 0; p < nplanes; ++p)
                    nccl_check(R.Recv(recv + (size_t)p * recv_stride + offset[r], counts[r], kNcclFloat32, r, c->comm, s),
                               "ncclRecv");
            }
        } else if (mine) {
            for (int p = 0; p < nplanes; ++p)
                nccl_check(R.Send(send + (size_t)p * send_stride, mine, kNcclFloat32, root, c->comm, s), "ncclSend");
        }
        nccl_check(R.GroupEnd(), "ncclGroupEnd");
    });
}

}  // extern "C"
