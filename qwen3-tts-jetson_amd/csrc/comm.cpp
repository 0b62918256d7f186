// comm.cpp — RCCL (librccl) transport of comm.h.  Collectives run on the caller's stream and are waited for before
// returning: they are start-up / end-of-run steps, never inside the frame loop.
#include "comm.h"

#include <rccl/rccl.h>

#include <cstring>
#include <string>

namespace q3t {

struct Comm {
    ncclComm_t nc = nullptr;
    int world = 1, rank = 0, device = 0;
    void *scratch = nullptr;   // device scratch for small collectives (64 doubles)
};

#define Q3T_NCCL(call)                                                                                    \
    do {                                                                                                  \
        ncclResult_t r__ = (call);                                                                        \
        if (r__ != ncclSuccess) {                                                                         \
            set_error(std::string(#call) + ": " + ncclGetErrorString(r__));                               \
            return false;                                                                                 \
        }                                                                                                 \
    } while (0)

static_assert(sizeof(ncclUniqueId) == COMM_ID_BYTES, "ncclUniqueId size");

bool comm_unique_id(uint8_t *id) {
    ncclUniqueId u;
    Q3T_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof u);
    return true;
}

bool comm_init(Comm **out, int world, int rank, const uint8_t *id, int device) {
    *out = nullptr;
    if (world < 1 || rank < 0 || rank >= world || !id) { set_error("comm_init: bad rank/world"); return false; }
    Q3T_HIP(hipSetDevice(device));
    Comm *c = new Comm();
    c->world = world;
    c->rank = rank;
    c->device = device;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    const ncclResult_t r = ncclCommInitRank(&c->nc, world, u, rank);
    if (r != ncclSuccess) {
        set_error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        delete c;
        return false;
    }
    if (hipMalloc(&c->scratch, 64 * sizeof(double)) != hipSuccess) {
        set_error("comm_init: scratch allocation failed");
        ncclCommDestroy(c->nc);
        delete c;
        return false;
    }
    *out = c;
    return true;
}

void comm_destroy(Comm *c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->nc) ncclCommDestroy(c->nc);
    if (c->scratch) hipFree(c->scratch);
    delete c;
}

int comm_rank(const Comm *c) { return c ? c->rank : 0; }
int comm_world(const Comm *c) { return c ? c->world : 1; }

bool comm_bcast_arenas(Comm *c, const std::vector<WeightArena *> &arenas, hipStream_t s) {
    // 1) every rank must have laid out the same blobs (same GGUF shapes): max and -min of each size must agree
    const int n = (int)arenas.size();
    if (n > 16) { set_error("comm_bcast_arenas: too many arenas"); return false; }
    double v[32];
    for (int i = 0; i < n; ++i) {
        v[i] = (double)arenas[i]->used;
        v[16 + i] = -(double)arenas[i]->used;
    }
    for (int i = n; i < 16; ++i) v[i] = v[16 + i] = 0.0;
    if (!comm_allreduce_max(c, v, 32, s)) return false;
    for (int i = 0; i < n; ++i)
        if (v[i] != -v[16 + i]) {
            set_error("comm_bcast_arenas: ranks laid out different weight blobs (different GGUF files?)");
            return false;
        }
    // 2) one broadcast per blob (>= hundreds of MB each: ring bandwidth over xGMI, not latency)
    // the group is closed on every path: an enqueue error must not leave the communicator inside ncclGroupStart
    Q3T_NCCL(ncclGroupStart());
    ncclResult_t first = ncclSuccess;
    for (WeightArena *a : arenas) {
        const ncclResult_t r = ncclBroadcast(a->base, a->base, a->used, ncclUint8, 0, c->nc, s);
        if (r != ncclSuccess) { first = r; break; }
    }
    const ncclResult_t end = ncclGroupEnd();
    if (first != ncclSuccess) { set_error(std::string("ncclBroadcast: ") + ncclGetErrorString(first)); return false; }
    if (end != ncclSuccess) { set_error(std::string("ncclGroupEnd: ") + ncclGetErrorString(end)); return false; }
    Q3T_HIP(hipStreamSynchronize(s));
    return true;
}

bool comm_allreduce_max(Comm *c, double *v, int n, hipStream_t s) {
    if (n <= 0) return true;
    if (n > 64) { set_error("comm_allreduce_max: n > 64"); return false; }
    Q3T_HIP(hipMemcpyAsync(c->scratch, v, n * sizeof(double), hipMemcpyHostToDevice, s));
    Q3T_NCCL(ncclAllReduce(c->scratch, c->scratch, n, ncclFloat64, ncclMax, c->nc, s));
    Q3T_HIP(hipMemcpyAsync(v, c->scratch, n * sizeof(double), hipMemcpyDeviceToHost, s));
    Q3T_HIP(hipStreamSynchronize(s));
    return true;
}

}  // namespace q3t
