// fake_rccl.cpp — TEST INFRASTRUCTURE ONLY: an in-process stand-in for the
// nine RCCL entry points libgolhip.so binds (gol_runtime.cpp rccl()), so the
// library's one-process-per-rank transport (GOL_XPORT_RCCL: the halo exchange
// of gol_runtime.cpp exchange(), the per-rank slabs, the event ordering around
// it) can run on ONE GPU.  Real RCCL refuses two ranks on one device
// ("Duplicate GPU detected"), and the GPU box has one GPU.
//
// Ranks are host threads of one process (one gol_ctx each, all on device 0).
// ncclSend/ncclRecv are collected per thread between ncclGroupStart/End; at
// ncclGroupEnd every rank of the communicator meets at a host barrier (one
// round per group), then each receive is matched with its peer's send (FIFO
// per (src, dst) channel) and enqueued on the RECEIVER's stream as:
//   wait(event recorded on the sender's stream at ncclSend) -> D2D copy
//   -> event; the sender's stream then waits for that event.
// Nothing waits on the device for work that is not yet enqueued, so the shim
// cannot hang the GPU.  Loaded with RTLD_GLOBAL before libgolhip.so resolves
// RCCL (it looks in the global scope first).
#include <hip/hip_runtime.h>
#include <string.h>

#include <condition_variable>
#include <map>
#include <mutex>
#include <string>
#include <vector>

extern "C" {
typedef enum { ncclSuccess = 0, ncclUnhandledCudaError = 1, ncclSystemError = 2, ncclInternalError = 3,
               ncclInvalidArgument = 4, ncclInvalidUsage = 5 } ncclResult_t;
typedef struct { char internal[128]; } ncclUniqueId;
typedef int ncclDataType_t;   // ncclUint8 / ncclInt8 for halos; ncclFloat64 (8) for the trial agreement
typedef int ncclRedOp_t;      // ncclSum (0), ncclMax (2)
struct FakeComm;
typedef FakeComm *ncclComm_t;
}

namespace {
struct Op {
    bool send;
    void *buf;
    size_t bytes;
    int peer;
    hipStream_t stream;
    hipEvent_t ready = nullptr;   // send: recorded on the sender's stream at ncclSend
};

struct Hub {
    std::mutex mu;
    std::condition_variable cv;
    int world = 0;
    int arrived = 0;
    unsigned long long round = 0;
    std::vector<std::vector<Op>> posted;   // per rank, this round
    std::vector<hipEvent_t> events;        // destroyed with the last communicator
    int live = 0;
    // ncclAllReduce: its own barrier (one collective per round)
    int ar_arrived = 0;
    unsigned long long ar_round = 0;
    std::vector<const void *> ar_send;
    std::vector<void *> ar_recv;
    std::vector<hipStream_t> ar_stream;
};

std::mutex g_mu;
std::map<std::string, Hub *> g_hubs;
unsigned long long g_next_id = 1;
}

struct FakeComm {
    Hub *hub;
    std::string key;
    int rank, world;
};

namespace {
thread_local int t_depth = 0;
thread_local FakeComm *t_comm = nullptr;
thread_local std::vector<Op> t_ops;

ncclResult_t run_round(FakeComm *c, std::vector<Op> ops) {
    Hub *h = c->hub;
    std::unique_lock<std::mutex> lk(h->mu);
    const unsigned long long my_round = h->round;
    h->posted[c->rank] = std::move(ops);
    if (++h->arrived < h->world) {
        h->cv.wait(lk, [&] { return h->round != my_round; });
        return ncclSuccess;
    }
    // last arriver: match every receive with its peer's send, in FIFO order per channel
    ncclResult_t rc = ncclSuccess;
    std::vector<std::vector<size_t>> next(h->world, std::vector<size_t>(h->world, 0));
    for (int r = 0; r < h->world && rc == ncclSuccess; ++r) {
        for (Op &rv : h->posted[r]) {
            if (rv.send) continue;
            const int p = rv.peer;
            Op *sd = nullptr;
            size_t &i = next[p][r];
            for (; i < h->posted[p].size(); ++i) {
                Op &o = h->posted[p][i];
                if (o.send && o.peer == r) {
                    sd = &o;
                    ++i;
                    break;
                }
            }
            if (!sd || sd->bytes != rv.bytes) {
                rc = ncclInvalidUsage;
                break;
            }
            hipEvent_t done;
            if (hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess ||
                hipStreamWaitEvent(rv.stream, sd->ready, 0) != hipSuccess ||
                hipMemcpyAsync(rv.buf, sd->buf, rv.bytes, hipMemcpyDeviceToDevice, rv.stream) != hipSuccess ||
                hipEventRecord(done, rv.stream) != hipSuccess || hipStreamWaitEvent(sd->stream, done, 0) != hipSuccess) {
                rc = ncclUnhandledCudaError;
                break;
            }
            h->events.push_back(done);
        }
    }
    // every send must have been consumed
    for (int p = 0; p < h->world && rc == ncclSuccess; ++p)
        for (int r = 0; r < h->world; ++r) {
            size_t n = 0;
            for (const Op &o : h->posted[p]) n += (o.send && o.peer == r);
            size_t used = 0;
            for (size_t i = 0; i < next[p][r]; ++i) used += (h->posted[p][i].send && h->posted[p][i].peer == r);
            if (used != n) rc = ncclInvalidUsage;
        }
    h->arrived = 0;
    h->round++;
    for (auto &v : h->posted) v.clear();
    lk.unlock();
    h->cv.notify_all();
    return rc;
}

ncclResult_t post(bool send, void *buf, size_t count, int peer, FakeComm *c, hipStream_t s) {
    if (!c || peer < 0 || peer >= c->world || peer == c->rank) return ncclInvalidArgument;
    Op o{send, buf, count, peer, s};
    if (send) {
        if (hipEventCreateWithFlags(&o.ready, hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(o.ready, s) != hipSuccess)
            return ncclUnhandledCudaError;
        std::lock_guard<std::mutex> lk(c->hub->mu);
        c->hub->events.push_back(o.ready);
    }
    if (t_depth == 0) return run_round(c, {o});
    if (t_comm && t_comm != c) return ncclInvalidUsage;   // one communicator per group in this shim
    t_comm = c;
    t_ops.push_back(o);
    return ncclSuccess;
}
}

extern "C" {
ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    if (!id) return ncclInvalidArgument;
    memset(id->internal, 0, sizeof id->internal);
    std::lock_guard<std::mutex> lk(g_mu);
    snprintf(id->internal, sizeof id->internal, "fake-rccl-%llu", g_next_id++);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    std::string key(id.internal, strnlen(id.internal, sizeof id.internal));
    std::lock_guard<std::mutex> lk(g_mu);
    Hub *&h = g_hubs[key];
    if (!h) {
        h = new Hub();
        h->world = nranks;
        h->posted.resize(nranks);
    }
    if (h->world != nranks) return ncclInvalidUsage;
    h->live++;
    *comm = new FakeComm{h, key, rank, nranks};
    return ncclSuccess;
}

ncclResult_t ncclSend(const void *buf, size_t count, ncclDataType_t, int peer, ncclComm_t comm, hipStream_t s) {
    return post(true, const_cast<void *>(buf), count, peer, comm, s);
}

ncclResult_t ncclRecv(void *buf, size_t count, ncclDataType_t, int peer, ncclComm_t comm, hipStream_t s) {
    return post(false, buf, count, peer, comm, s);
}

// Every rank of the communicator meets at a host barrier; the last arriver
// drains each rank's stream (everything they wait for is enqueued: every rank
// thread is inside this call), reduces on the host and writes every result
// buffer.  float64 MAX / SUM only (what libgolhip uses).
ncclResult_t ncclAllReduce(const void *sendbuff, void *recvbuff, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t s) {
    if (!comm || dt != 8 || (op != 0 && op != 2) || t_depth != 0) return ncclInvalidArgument;
    Hub *h = comm->hub;
    std::unique_lock<std::mutex> lk(h->mu);
    if (h->ar_send.empty()) {
        h->ar_send.resize(h->world);
        h->ar_recv.resize(h->world);
        h->ar_stream.resize(h->world);
    }
    const unsigned long long my_round = h->ar_round;
    h->ar_send[comm->rank] = sendbuff;
    h->ar_recv[comm->rank] = recvbuff;
    h->ar_stream[comm->rank] = s;
    if (++h->ar_arrived < h->world) {
        h->cv.wait(lk, [&] { return h->ar_round != my_round; });
        return ncclSuccess;
    }
    ncclResult_t rc = ncclSuccess;
    std::vector<double> acc(count), v(count);
    for (int r = 0; r < h->world && rc == ncclSuccess; ++r) {
        if (hipStreamSynchronize(h->ar_stream[r]) != hipSuccess ||
            hipMemcpy(v.data(), h->ar_send[r], count * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
            rc = ncclUnhandledCudaError;
            break;
        }
        for (size_t i = 0; i < count; ++i)
            acc[i] = r == 0 ? v[i] : (op == 2 ? (v[i] > acc[i] ? v[i] : acc[i]) : acc[i] + v[i]);
    }
    for (int r = 0; r < h->world && rc == ncclSuccess; ++r)
        if (hipMemcpy(h->ar_recv[r], acc.data(), count * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
            rc = ncclUnhandledCudaError;
    h->ar_arrived = 0;
    h->ar_round++;
    lk.unlock();
    h->cv.notify_all();
    return rc;
}

ncclResult_t ncclGroupStart() {
    t_depth++;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_depth <= 0) return ncclInvalidUsage;
    if (--t_depth > 0) return ncclSuccess;
    FakeComm *c = t_comm;
    std::vector<Op> ops;
    ops.swap(t_ops);
    t_comm = nullptr;
    if (!c) return ncclSuccess;
    return run_round(c, std::move(ops));
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(g_mu);
    Hub *h = comm->hub;
    if (--h->live == 0) {
        (void)hipDeviceSynchronize();
        for (hipEvent_t e : h->events) (void)hipEventDestroy(e);
        g_hubs.erase(comm->key);
        delete h;
    }
    delete comm;
    return ncclSuccess;
}

const char *ncclGetErrorString(ncclResult_t r) {
    switch (r) {
    case ncclSuccess: return "fake-rccl: success";
    case ncclInvalidArgument: return "fake-rccl: invalid argument";
    case ncclInvalidUsage: return "fake-rccl: unmatched send/recv";
    default: return "fake-rccl: hip error";
    }
}
}
