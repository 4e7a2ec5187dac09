// fake_rccl_ipc.cpp -- TEST DOUBLE of the RCCL entry points csrc/sunsky_comm.cpp resolves
// (ncclGetUniqueId, ncclCommInitRank, ncclCommDestroy, ncclGroupStart, ncclGroupEnd, ncclSend,
// ncclRecv, ncclGetErrorString) for ranks that are separate PROCESSES on one GPU, where real
// RCCL refuses two ranks on one device.  Built as tests/cpp/build/libfake_rccl_ipc.so and loaded
// by the product only when SUNSKY_AMD_RCCL names it (tests/test_gpu_gather.py, bench.py's
// multi-rank rehearsal with SUNSKY_BENCH_RCCL_DOUBLE); never shipped.  fake_rccl.cpp is the
// one-process form (ranks as communicators of one process).
//
// The unique id is a private directory (mkdtemp).  A send and the receive it pairs with (same
// sender, receiver and position in their order, as NCCL matches point-to-point operations)
// meet through it: at ncclGroupEnd the sender copies the send into an allocation of its own
// (exporting the caller's allocation directly hung hipIpcOpenMemHandle for allocations past
// 2 GiB -- configs[4]'s 2.95 GB shard planes -- while 1.5 GB ones worked), exports it with
// hipIpcGetMemHandle and publishes (handle, bytes) in a file named by (sender, receiver,
// sequence); the receiver waits for that file, opens the handle, copies on its stream, waits for
// the copy, closes the handle and answers with a "done" file; the sender frees its copy when
// every one of its sends is answered.  All
// of a group's sends are published before any of its receives waits, so no rank waits on a
// peer that is itself waiting.  Only float32 (datatype 7).  A missing peer times out (120 s,
// SUNSKY_FAKE_RCCL_TIMEOUT) with an error instead of hanging.
#include <hip/hip_runtime_api.h>

#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int kOk = 0, kInternal = 3, kInvalidArgument = 4, kFloat32 = 7;

struct Comm {
    std::string dir;
    int rank, nranks;
    std::map<int, unsigned> send_seq, recv_seq;   // per peer: operations posted so far
};

struct Op {
    bool send;
    Comm* comm;
    int peer;
    void* buf;
    size_t bytes;
    hipStream_t stream;
    unsigned seq;
    void* stage;   // the sender's exported copy
};

struct Published {
    hipIpcMemHandle_t handle;
    size_t offset, bytes;
};

thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;

std::string path(const Comm* c, const char* kind, int from, int to, unsigned seq) {
    return c->dir + "/" + kind + "_" + std::to_string(from) + "_" + std::to_string(to) + "_" + std::to_string(seq);
}

// SUNSKY_FAKE_RCCL_DEBUG=1: per-operation timings on stderr
bool debug() {
    static const bool on = std::getenv("SUNSKY_FAKE_RCCL_DEBUG") != nullptr;
    return on;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool wait_for(const std::string& p) {
    const char* t = std::getenv("SUNSKY_FAKE_RCCL_TIMEOUT");
    const double limit = t ? std::atof(t) : 120.0;
    const auto t0 = std::chrono::steady_clock::now();
    struct stat st;
    while (stat(p.c_str(), &st) != 0) {
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
            std::fprintf(stderr, "fake_rccl_ipc: timed out waiting for %s\n", p.c_str());
            return false;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    return true;
}

bool write_atomic(const std::string& p, const void* data, size_t n) {
    const std::string tmp = p + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(data, 1, n, f) == n;
    std::fclose(f);
    return ok && std::rename(tmp.c_str(), p.c_str()) == 0;
}

int publish(Op& s) {
    const double t0 = now_s();
    if (hipMalloc(&s.stage, s.bytes ? s.bytes : 4) != hipSuccess) return kInternal;
    if (hipMemcpyAsync(s.stage, s.buf, s.bytes, hipMemcpyDeviceToDevice, s.stream) != hipSuccess ||
        hipStreamSynchronize(s.stream) != hipSuccess)
        return kInternal;
    Published m{};
    const double t1 = now_s();
    if (hipIpcGetMemHandle(&m.handle, s.stage) != hipSuccess) return kInternal;
    m.offset = 0;
    m.bytes = s.bytes;
    if (debug())
        std::fprintf(stderr, "fake_rccl_ipc: rank %d send %u to %d: %zu B, stage %.3f s, export %.3f s\n",
                     s.comm->rank, s.seq, s.peer, s.bytes, t1 - t0, now_s() - t1);
    return write_atomic(path(s.comm, "send", s.comm->rank, s.peer, s.seq), &m, sizeof m) ? kOk : kInternal;
}

int receive(const Op& r) {
    const std::string p = path(r.comm, "send", r.peer, r.comm->rank, r.seq);
    if (!wait_for(p)) return kInternal;
    Published m{};
    FILE* f = std::fopen(p.c_str(), "rb");
    if (!f) return kInternal;
    const bool ok = std::fread(&m, 1, sizeof m, f) == sizeof m;
    std::fclose(f);
    if (!ok) return kInternal;
    if (m.bytes != r.bytes) {
        std::fprintf(stderr, "fake_rccl_ipc: send of %zu bytes paired with a receive of %zu\n", m.bytes, r.bytes);
        return kInvalidArgument;
    }
    void* mapped = nullptr;
    const double t0 = now_s();
    if (hipIpcOpenMemHandle(&mapped, m.handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return kInternal;
    const double t1 = now_s();
    int rc = kOk;
    if (hipMemcpyAsync(r.buf, (char*)mapped + m.offset, m.bytes, hipMemcpyDeviceToDevice, r.stream) != hipSuccess ||
        hipStreamSynchronize(r.stream) != hipSuccess)
        rc = kInternal;
    const double t2 = now_s();
    (void)hipIpcCloseMemHandle(mapped);
    if (debug())
        std::fprintf(stderr, "fake_rccl_ipc: rank %d recv %u from %d: %zu B, open %.3f s, copy %.3f s, close %.3f s\n",
                     r.comm->rank, r.seq, r.peer, m.bytes, t1 - t0, t2 - t1, now_s() - t2);
    std::remove(p.c_str());
    const char one = 1;
    if (!write_atomic(path(r.comm, "done", r.peer, r.comm->rank, r.seq), &one, 1)) rc = kInternal;
    return rc;
}

int run(std::vector<Op>& ops) {
    struct Free {   // the sender's copies, whatever the outcome
        std::vector<Op>& ops;
        ~Free() {
            for (Op& o : ops)
                if (o.stage) (void)hipFree(o.stage);
        }
    } release{ops};
    for (Op& o : ops)
        if (o.send)
            if (int rc = publish(o)) return rc;
    for (const Op& o : ops)
        if (!o.send)
            if (int rc = receive(o)) return rc;
    for (const Op& o : ops)
        if (o.send) {
            const std::string d = path(o.comm, "done", o.comm->rank, o.peer, o.seq);
            if (!wait_for(d)) return kInternal;
            std::remove(d.c_str());
        }
    return kOk;
}

}  // namespace

extern "C" {

struct ncclUniqueId { char internal[128]; };
typedef Comm* ncclComm_t;

int ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return kInvalidArgument;
    char tmpl[] = "/tmp/fake_rccl_ipc_XXXXXX";
    if (!mkdtemp(tmpl)) return kInternal;
    std::memset(id->internal, 0, sizeof(id->internal));
    std::snprintf(id->internal, sizeof(id->internal), "%s", tmpl);
    return kOk;
}

int ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return kInvalidArgument;
    std::string dir(id.internal, strnlen(id.internal, sizeof(id.internal)));
    struct stat st;
    if (dir.rfind("/tmp/fake_rccl_ipc_", 0) != 0 || stat(dir.c_str(), &st) != 0) return kInvalidArgument;
    *comm = new Comm{dir, rank, nranks, {}, {}};
    return kOk;
}

int ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return kInvalidArgument;
    // every exchange of this communicator has completed (each side waited for its peer's file):
    // whichever rank destroys its communicator last finds the directory empty and removes it
    (void)rmdir(comm->dir.c_str());
    delete comm;
    return kOk;
}

int ncclGroupStart() {
    ++t_depth;
    return kOk;
}

int ncclGroupEnd() {
    if (t_depth == 0) return kInvalidArgument;
    if (--t_depth > 0) return kOk;
    std::vector<Op> ops;
    ops.swap(t_ops);
    return run(ops);
}

static int enqueue(bool send, const void* buf, size_t count, int datatype, int peer, ncclComm_t comm,
                   hipStream_t stream) {
    if (!comm || datatype != kFloat32 || peer < 0 || peer >= comm->nranks || peer == comm->rank) return kInvalidArgument;
    const unsigned seq = send ? comm->send_seq[peer]++ : comm->recv_seq[peer]++;
    Op o{send, comm, peer, const_cast<void*>(buf), count * sizeof(float), stream, seq, nullptr};
    if (t_depth > 0) {
        t_ops.push_back(o);
        return kOk;
    }
    std::vector<Op> one{o};
    return run(one);
}

int ncclSend(const void* buf, size_t count, int datatype, int peer, ncclComm_t comm, hipStream_t stream) {
    return enqueue(true, buf, count, datatype, peer, comm, stream);
}

int ncclRecv(void* buf, size_t count, int datatype, int peer, ncclComm_t comm, hipStream_t stream) {
    return enqueue(false, buf, count, datatype, peer, comm, stream);
}

const char* ncclGetErrorString(int result) {
    switch (result) {
        case kOk: return "no error (fake_rccl_ipc)";
        case kInvalidArgument: return "invalid argument (fake_rccl_ipc)";
        default: return "internal error (fake_rccl_ipc)";
    }
}

}  // extern "C"
