// zr_comm.cpp -- the shared-table exchange of the multi-GPU path on RCCL.
//
// One process per GPU. Every rank counts its own shard's bytes on its device;
// the shared frequency table is the table of the SUM of those histograms
// (RansBlobStore::train counts its whole training set, blob_store/entropy.rs:
// 212-219; AdaptiveRans64Encoder counts all its data, rans.rs:708-714), so one
// in-place all-reduce of 256 u32 counters over xGMI gives every rank the same
// histogram and each then builds the identical table on its device
// (zr_rans_dtab_from_hist_dev: normalize_frequencies is deterministic).
//
// librccl is opened with dlopen on the first zr_comm_* call, so the codec
// library itself loads on hosts without RCCL and a single-GPU user never
// initialises it. The unique id travels between the ranks' processes by any
// host channel the caller has (a file, a socket, torch.distributed, an env
// var): the same contract as ncclGetUniqueId / ncclCommInitRank.
#include <dlfcn.h>

#include <cstring>
#include <mutex>

#include <rccl/rccl.h>

#include "zr_internal.h"

namespace zr {
namespace {

struct Rccl {
    void *h = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommCount) comm_count = nullptr;
    std::string err;
};

Rccl &rccl_state() {
    static Rccl r;
    return r;
}

Rccl *rccl() {
    Rccl &r = rccl_state();
    static std::once_flag once;
    std::call_once(once, [&r] {
        const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        for (const char *n : names)
            if ((r.h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!r.h) {
            const char *e = dlerror();
            r.err = std::string("cannot load librccl: ") + (e ? e : "?");
            return;
        }
        auto sym = [&](const char *n) { return dlsym(r.h, n); };
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
        r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
        r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
        r.broadcast = reinterpret_cast<decltype(r.broadcast)>(sym("ncclBroadcast"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
        r.comm_count = reinterpret_cast<decltype(r.comm_count)>(sym("ncclCommCount"));
        if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce || !r.broadcast ||
            !r.error_string || !r.comm_count)
            r.err = "librccl lacks an entry point";
    });
    return r.err.empty() ? &r : nullptr;
}

int32_t rccl_missing() { return set_error(ZR_UNSUPPORTED, "RCCL unavailable: " + rccl_state().err); }

int32_t rccl_fail(Rccl *r, ncclResult_t e, const char *what) {
    return set_error(ZR_INTERNAL, std::string(what) + ": " + (r->error_string ? r->error_string(e) : "?"));
}

}  // namespace
}  // namespace zr

struct zr_comm {
    ncclComm_t comm;
    int32_t nranks, rank, device;
};

using namespace zr;

extern "C" {

int32_t zr_comm_unique_id(uint8_t id[ZR_COMM_ID_BYTES]) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!id) return set_error(ZR_INVALID_INPUT, "null argument");
    Rccl *r = rccl();
    if (!r) return rccl_missing();
    static_assert(sizeof(ncclUniqueId) == ZR_COMM_ID_BYTES, "unique id size");
    ncclUniqueId u;
    const ncclResult_t e = r->get_unique_id(&u);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclGetUniqueId");
    memcpy(id, &u, ZR_COMM_ID_BYTES);
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_comm_init(const uint8_t id[ZR_COMM_ID_BYTES], int32_t nranks, int32_t rank, zr_comm **comm) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!id || !comm) return set_error(ZR_INVALID_INPUT, "null argument");
    *comm = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return set_error(ZR_INVALID_INPUT, "rank outside 0..nranks-1");
    Rccl *r = rccl();
    if (!r) return rccl_missing();
    int dev = 0;
    ZR_HIP(hipGetDevice(&dev));
    ncclUniqueId u;
    memcpy(&u, id, ZR_COMM_ID_BYTES);
    ncclComm_t c = nullptr;
    const ncclResult_t e = r->comm_init_rank(&c, nranks, u, rank);  // collective over the ranks
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclCommInitRank");
    *comm = new zr_comm{c, nranks, rank, dev};
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_comm_count(const zr_comm *comm, int32_t *nranks) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!comm || !nranks) return set_error(ZR_INVALID_INPUT, "null argument");
    *nranks = 0;
    Rccl *r = rccl();
    if (!r) return rccl_missing();
    int n = 0;  // RCCL's own view of the communicator, not the count the caller passed
    const ncclResult_t e = r->comm_count(comm->comm, &n);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclCommCount");
    *nranks = n;
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_histogram_allreduce_dev(zr_comm *comm, uint32_t *hist_dev, uint32_t n_bins, void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!comm || (!hist_dev && n_bins)) return set_error(ZR_INVALID_INPUT, "null argument");
    if (n_bins == 0) return ZR_OK;
    Rccl *r = rccl();
    if (!r) return rccl_missing();
    // u32 SUM wraps mod 2^32 per bin, as the reference's u32 counters do
    const ncclResult_t e =
        r->all_reduce(hist_dev, hist_dev, n_bins, ncclUint32, ncclSum, comm->comm, (hipStream_t)stream);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclAllReduce");
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_table_broadcast_dev(zr_comm *comm, void *dtabs_dev, uint32_t n_tables, int32_t root, void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!comm || (!dtabs_dev && n_tables)) return set_error(ZR_INVALID_INPUT, "null argument");
    if (root < 0 || root >= comm->nranks) return set_error(ZR_INVALID_INPUT, "root outside 0..nranks-1");
    if (n_tables == 0) return ZR_OK;
    Rccl *r = rccl();
    if (!r) return rccl_missing();
    const size_t bytes = (size_t)n_tables * sizeof(RansDTab);
    const ncclResult_t e =
        r->broadcast(dtabs_dev, dtabs_dev, bytes, ncclUint8, root, comm->comm, (hipStream_t)stream);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclBroadcast");
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_comm_destroy(zr_comm *comm) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!comm) return ZR_OK;
    Rccl *r = rccl();
    int32_t st = ZR_OK;
    if (r) {
        const ncclResult_t e = r->comm_destroy(comm->comm);
        if (e != ncclSuccess) st = rccl_fail(r, e, "ncclCommDestroy");
    }
    delete comm;
    return st;
    ZR_GUARD_END
}

}  // extern "C"
