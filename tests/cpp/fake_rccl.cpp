// fake_rccl.cpp -- TEST DOUBLE of the RCCL entry points csrc/sunsky_comm.cpp resolves
// with dlopen (ncclGetUniqueId, ncclCommInitRank, ncclCommDestroy, ncclGroupStart,
// ncclGroupEnd, ncclSend, ncclRecv, ncclGetErrorString).  Built as tests/cpp/build/
// librccl.so.1 and linked only by the test program gather_double_check, where the
// product's dlopen("librccl.so.1") finds it already loaded; never shipped.
//
// It lets the multi-rank branch of sunsky_gather_radiance (grouped send/recv) run on a
// one-GPU box, where real RCCL refuses two ranks on one device: several "ranks" live in
// one process (one communicator each, created with the same unique id), and a send and
// the receive it pairs with (same sender, receiver and position in their order, as NCCL
// matches point-to-point operations) become one hipMemcpyAsync.  The copy runs on the
// receiver's stream after an event recorded on the sender's stream at its ncclGroupEnd,
// whichever of the two groups ends last issues it.  Only float32 (datatype 7) is handled.
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

namespace {

constexpr int kOk = 0, kInvalidArgument = 4, kInternal = 3, kFloat32 = 7;

struct World;
struct Comm {
    World* world;
    int rank, nranks, device;
};

struct Send {
    const void* buf;
    size_t bytes;
    hipEvent_t ready;
};
struct Recv {
    void* buf;
    size_t bytes;
    hipStream_t stream;
};

struct World {
    int nranks;
    int joined = 0;
    // per (sender, receiver): posted and not yet matched, in posting order
    std::map<std::pair<int, int>, std::deque<Send>> sends;
    std::map<std::pair<int, int>, std::deque<Recv>> recvs;
    std::vector<hipEvent_t> spent;
};

std::mutex g_mu;
std::map<std::string, World*> g_worlds;
unsigned g_next_id = 1;

// operations posted since ncclGroupStart on this thread
struct Pending {
    bool send;
    Comm* comm;
    int peer;
    void* buf;
    size_t bytes;
    hipStream_t stream;
};
thread_local int t_depth = 0;
thread_local std::vector<Pending> t_ops;

int match(World* w, int src, int dst) {
    auto& S = w->sends[{src, dst}];
    auto& R = w->recvs[{src, dst}];
    while (!S.empty() && !R.empty()) {
        Send s = S.front();
        Recv r = R.front();
        S.pop_front();
        R.pop_front();
        if (s.bytes != r.bytes) {
            std::fprintf(stderr, "fake_rccl: send of %zu bytes paired with a receive of %zu\n", s.bytes, r.bytes);
            return kInvalidArgument;
        }
        if (hipStreamWaitEvent(r.stream, s.ready, 0) != hipSuccess) return kInternal;
        if (hipMemcpyAsync(r.buf, s.buf, s.bytes, hipMemcpyDeviceToDevice, r.stream) != hipSuccess) return kInternal;
        w->spent.push_back(s.ready);   // destroyed with the world, after a device synchronisation
    }
    return kOk;
}

int post(const Pending& p) {
    World* w = p.comm->world;
    const int me = p.comm->rank;
    if (p.send) {
        hipEvent_t ev;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return kInternal;
        if (hipEventRecord(ev, p.stream) != hipSuccess) return kInternal;
        w->sends[{me, p.peer}].push_back({p.buf, p.bytes, ev});
        return match(w, me, p.peer);
    }
    w->recvs[{p.peer, me}].push_back({p.buf, p.bytes, p.stream});
    return match(w, p.peer, me);
}

}  // namespace

extern "C" {

struct ncclUniqueId { char internal[128]; };
typedef Comm* ncclComm_t;

int ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return kInvalidArgument;
    std::lock_guard<std::mutex> lock(g_mu);
    std::memset(id->internal, 0, sizeof(id->internal));
    std::snprintf(id->internal, sizeof(id->internal), "fake-rccl-%u", g_next_id++);
    return kOk;
}

int ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return kInvalidArgument;
    std::lock_guard<std::mutex> lock(g_mu);
    std::string key(id.internal, strnlen(id.internal, sizeof(id.internal)));
    World*& w = g_worlds[key];
    if (!w) {
        w = new World();
        w->nranks = nranks;
    }
    if (w->nranks != nranks || w->joined >= nranks) return kInvalidArgument;
    ++w->joined;
    int dev = 0;
    (void)hipGetDevice(&dev);
    *comm = new Comm{w, rank, nranks, dev};
    return kOk;
}

int ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return kInvalidArgument;
    std::lock_guard<std::mutex> lock(g_mu);
    World* w = comm->world;
    delete comm;
    if (--w->joined == 0) {   // the last rank of the world: nothing can wait on its events any more
        (void)hipDeviceSynchronize();
        for (hipEvent_t e : w->spent) (void)hipEventDestroy(e);
        for (auto& kv : g_worlds)
            if (kv.second == w) {
                g_worlds.erase(kv.first);
                break;
            }
        delete w;
    }
    return kOk;
}

int ncclGroupStart() {
    ++t_depth;
    return kOk;
}

int ncclGroupEnd() {
    if (t_depth == 0) return kInvalidArgument;
    if (--t_depth > 0) return kOk;
    std::lock_guard<std::mutex> lock(g_mu);
    int rc = kOk;
    for (const Pending& p : t_ops)
        if (rc == kOk) rc = post(p);
    t_ops.clear();
    return rc;
}

static int enqueue(bool send, const void* buf, size_t count, int datatype, int peer, ncclComm_t comm,
                   hipStream_t stream) {
    if (!comm || datatype != kFloat32 || peer < 0 || peer >= comm->nranks || peer == comm->rank) return kInvalidArgument;
    Pending p{send, comm, peer, const_cast<void*>(buf), count * sizeof(float), stream};
    if (t_depth > 0) {
        t_ops.push_back(p);
        return kOk;
    }
    std::lock_guard<std::mutex> lock(g_mu);
    return post(p);
}

int ncclSend(const void* buf, size_t count, int datatype, int peer, ncclComm_t comm, hipStream_t stream) {
    return enqueue(true, buf, count, datatype, peer, comm, stream);
}

int ncclRecv(void* buf, size_t count, int datatype, int peer, ncclComm_t comm, hipStream_t stream) {
    return enqueue(false, buf, count, datatype, peer, comm, stream);
}

const char* ncclGetErrorString(int result) {
    switch (result) {
        case kOk: return "no error (fake_rccl)";
        case kInvalidArgument: return "invalid argument (fake_rccl)";
        default: return "internal error (fake_rccl)";
    }
}

}  // extern "C"
