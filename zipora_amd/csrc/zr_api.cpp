// zr_api.cpp -- host side of the C ABI: error state, table construction,
// host-memory entry points, device helpers and synthetic inputs.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "zr_internal.h"

namespace zr {

// ---------------------------------------------------------------- errors
// thread-local last error + optional callback (src/ffi/c_api.rs:17-42)
static thread_local std::string g_last_error;
static zr_error_cb g_cb = nullptr;

int32_t set_error(int32_t code, const std::string &msg) {
    g_last_error = msg;
    if (g_cb) g_cb(code, g_last_error.c_str());
    return code;
}
void clear_error() { g_last_error.clear(); }

// compute units of the current device (cached per device)
uint32_t cu_count() {
    // (atomic slots: the thread-safe host entry points may fill them concurrently;
    // every writer stores the same value)
    static std::atomic<int> cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int n = cached[dev].load(std::memory_order_relaxed);
    if (!n) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cached[dev].store(n, std::memory_order_relaxed);
    }
    return (uint32_t)n;
}

// ---------------------------------------------------------------- allocations
static std::atomic<uint64_t> g_dev_allocs{0};

hipError_t dev_alloc(void **p, size_t bytes) {
    g_dev_allocs.fetch_add(1, std::memory_order_relaxed);
    return hipMalloc(p, bytes ? bytes : 16);
}

// ---------------------------------------------------------------- call contexts
namespace {
std::mutex g_ctx_mx;
std::map<int, std::vector<CallCtx *>> g_ctx_free;  // per device; contexts live for the process
}  // namespace

int32_t CallLease::acquire() {
    int dev = 0;
    ZR_HIP(hipGetDevice(&dev));
    {
        std::lock_guard<std::mutex> g(g_ctx_mx);
        auto &v = g_ctx_free[dev];
        if (!v.empty()) {
            c_ = v.back();
            v.pop_back();
            return ZR_OK;
        }
    }
    CallCtx *c = new CallCtx;
    c->device = dev;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return set_error(ZR_INTERNAL, "hipStreamCreate failed");
    }
    c_ = c;
    return ZR_OK;
}

// buffers larger than this are returned when the lease ends (a rare huge call
// must not pin GiBs of device memory in an idle pooled context for the life of
// the process); smaller ones stay cached for the next call
constexpr size_t LEASE_KEEP = size_t(1) << 30;

CallLease::~CallLease() {
    if (!c_) return;
    for (int i = 0; i < CallCtx::NBUF; i++)
        if (c_->buf[i] && c_->cap[i] > LEASE_KEEP) {
            (void)hipFreeAsync(c_->buf[i], c_->stream);  // after the call's work, in stream order
            c_->buf[i] = nullptr;
            c_->cap[i] = 0;
        }
    (void)hipStreamSynchronize(c_->stream);  // nothing of this call may still run
    std::lock_guard<std::mutex> g(g_ctx_mx);
    g_ctx_free[c_->device].push_back(c_);
}

int32_t CallLease::get(int slot, size_t bytes, void **p) {
    if (bytes == 0) bytes = 16;
    if (bytes > c_->cap[slot]) {
        // grow to the next power of two (at least 64 KiB) so that a run of
        // growing calls reallocates rarely. Stream-ordered free and allocation
        // (hipFreeAsync / hipMallocAsync on the context's own stream): growing
        // never synchronises the device, only this call's stream orders it
        size_t want = 64 << 10;
        while (want < bytes) want <<= 1;
        if (c_->buf[slot]) {
            ZR_HIP(hipFreeAsync(c_->buf[slot], c_->stream));
            c_->buf[slot] = nullptr;
            c_->cap[slot] = 0;
        }
        g_dev_allocs.fetch_add(1, std::memory_order_relaxed);
        if (hipMallocAsync(&c_->buf[slot], want, c_->stream) != hipSuccess) {
            c_->buf[slot] = nullptr;
            return set_error(ZR_MEMORY_ERROR, "hipMallocAsync failed");
        }
        c_->cap[slot] = want;
    }
    *p = c_->buf[slot];
    return ZR_OK;
}

// every idle pooled context of every device: buffers freed, streams destroyed,
// the devices' default memory pools trimmed (contexts in use are not in the
// pool and are left alone)
int32_t release_call_contexts() {
    std::map<int, std::vector<CallCtx *>> take;
    {
        std::lock_guard<std::mutex> g(g_ctx_mx);
        take.swap(g_ctx_free);
    }
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) {  // nothing released: the contexts go back
        std::lock_guard<std::mutex> g(g_ctx_mx);
        for (auto &kv : take) g_ctx_free[kv.first].insert(g_ctx_free[kv.first].end(), kv.second.begin(), kv.second.end());
        return set_error(ZR_INTERNAL, "HIP error: hipGetDevice failed");
    }
    // a device that cannot be selected keeps its contexts in the pool (never
    // leaked); the other devices are still released; the first error is reported
    int32_t st = ZR_OK;
    for (auto &kv : take) {
        if (hipSetDevice(kv.first) != hipSuccess) {
            std::lock_guard<std::mutex> g(g_ctx_mx);
            auto &v = g_ctx_free[kv.first];
            v.insert(v.end(), kv.second.begin(), kv.second.end());
            if (st == ZR_OK) st = set_error(ZR_INTERNAL, "HIP error: hipSetDevice failed");
            continue;
        }
        for (CallCtx *c : kv.second) {
            for (int i = 0; i < CallCtx::NBUF; i++)
                if (c->buf[i]) (void)hipFreeAsync(c->buf[i], c->stream);
            (void)hipStreamSynchronize(c->stream);
            (void)hipStreamDestroy(c->stream);
            delete c;
        }
        hipMemPool_t pool;
        if (hipDeviceGetDefaultMemPool(&pool, kv.first) == hipSuccess) (void)hipMemPoolTrimTo(pool, 0);
    }
    if (hipSetDevice(cur) != hipSuccess && st == ZR_OK) st = set_error(ZR_INTERNAL, "HIP error: hipSetDevice failed");
    return st;
}

int32_t CallLease::sync() {
    ZR_HIP(hipStreamSynchronize(c_->stream));
    return ZR_OK;
}

// ---------------------------------------------------------------- rANS table
// Rans64Encoder::new (rans.rs:208-235) with normalize_frequencies (rans.rs:238-299).
int32_t rans_normalize_host(const uint32_t raw[256], zr_rans_table *out) {
    std::memset(out, 0, sizeof(*out));
    uint32_t total = 0;  // wrapping u32 sum (rans.rs:209)
    for (int i = 0; i < 256; i++) total += raw[i];
    if (total == 0) return ZR_OK;  // empty encoder (rans.rs:210-216)
    uint32_t *norm = out->freq;
    uint32_t remaining = TOTFREQ;
    int used = 0;
    for (int i = 0; i < 256; i++)
        if (raw[i]) {
            norm[i] = 1;
            remaining--;
            used++;
        }
    if (!used) return set_error(ZR_INVALID_INPUT, "No symbols with non-zero frequency");
    const uint64_t ir = remaining;
    for (int i = 0; i < 256; i++)
        if (raw[i] && remaining) {
            uint32_t add = (uint32_t)(((uint64_t)raw[i] * ir) / total);
            add = std::min(add, remaining);
            norm[i] += add;
            remaining -= add;
        }
    // third pass, with the repeated +1 on one argmax batched up to the 1024 cap
    while (remaining) {
        uint32_t mf = 0;
        int mi = -1;
        for (int i = 0; i < 256; i++)
            if (raw[i] > mf && norm[i] < TOTFREQ / 4) {
                mf = raw[i];
                mi = i;
            }
        if (mi < 0) {
            for (int i = 0; i < 256; i++)
                if (raw[i]) {
                    norm[i] += remaining;
                    break;
                }
            remaining = 0;
        } else {
            const uint32_t give = std::min(remaining, TOTFREQ / 4 - norm[mi]);
            norm[mi] += give;
            remaining -= give;
        }
    }
    uint32_t cum = 0;
    for (int i = 0; i < 256; i++) {
        out->start[i] = cum;
        cum += norm[i];
    }
    out->total_freq = TOTFREQ;
    return ZR_OK;
}

void rans_dtab_from_table(const zr_rans_table *t, RansDTab *d) {
    std::memset(d, 0, sizeof(*d));
    d->status = ZR_OK;
    bool single = false;
    for (int s = 0; s < 256; s++) {
        const uint32_t f = t->freq[s];
        d->freq[s] = f;
        d->start[s] = t->start[s];
        d->rsh[s] = enc_rsh(f);
        d->rcp[s] = enc_rcp(f);
        if (f == TOTFREQ) single = true;
        for (uint32_t i = 0; i < f && t->start[s] + i < TOTFREQ; i++) {
            const uint32_t j = t->start[s] + i;
            d->slot[j] = (uint32_t)s | (i << 8) | ((f < TOTFREQ ? f : 0u) << 20);
        }
    }
    d->kind = t->total_freq == 0 ? DT_EMPTY : (single ? DT_SINGLE : DT_NORMAL);
}

// ---------------------------------------------------------------- synthetic inputs
static inline uint64_t xs64(uint64_t &s) {  // tests/fse_tests.rs:711-717
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}

static void synth(int kind, uint64_t seed, uint8_t *out, size_t n) {
    uint64_t s = seed ? seed : 0x9E3779B97F4A7C15ull;
    if (kind == 0) {
        for (size_t i = 0; i < n; i++) out[i] = (uint8_t)(xs64(s) >> 32);
    } else if (kind == 1) {
        // Zipf(1.1) over ranks 1..256 by inverse CDF, rank k -> byte k-1
        double cdf[256], acc = 0;
        for (int k = 0; k < 256; k++) acc += std::pow((double)(k + 1), -1.1);
        double run = 0;
        for (int k = 0; k < 256; k++) {
            run += std::pow((double)(k + 1), -1.1);
            cdf[k] = run / acc;
        }
        cdf[255] = 1.0;
        for (size_t i = 0; i < n; i++) {
            const double u = (double)(xs64(s) >> 11) * (1.0 / 9007199254740992.0);
            int lo = 0, hi = 255;
            while (lo < hi) {
                int mid = (lo + hi) >> 1;
                if (cdf[mid] > u) hi = mid;
                else lo = mid + 1;
            }
            out[i] = (uint8_t)lo;
        }
    } else {
        // text-like: order-1 Markov chain over 64 printable symbols; each
        // context prefers 8 successors (3/4 of the mass), spaces every ~6 bytes
        static const char alpha[] =
            " etaoinshrdlcumwfgypbvkjxqzETAOINSHRDLCUMWFGYPBVKJXQZ.,;:'!?-\n0";
        uint8_t succ[64][8];
        uint64_t t = 1;
        for (int c = 0; c < 64; c++)
            for (int j = 0; j < 8; j++) succ[c][j] = (uint8_t)(xs64(t) % 64);
        int cur = 0;
        for (size_t i = 0; i < n; i++) {
            const uint64_t r = xs64(s);
            int nxt;
            const uint32_t u = (uint32_t)(r >> 40) & 0xFFFF;
            if (u < 10923) nxt = 0;                                   // ~1/6 spaces
            else if (u < 10923 + 40960) nxt = succ[cur][(r >> 8) & 7]; // preferred successors
            else nxt = (int)((r >> 16) % 48) + 1;                      // letters / punctuation
            out[i] = (uint8_t)alpha[nxt];
            cur = nxt;
        }
    }
}

}  // namespace zr

using namespace zr;

// ======================================================================
// C ABI
// ======================================================================
extern "C" {

const char *zr_last_error(void) { return g_last_error.c_str(); }
void zr_set_error_callback(zr_error_cb cb) { g_cb = cb; }
const char *zr_version(void) { return "zipora_amd 0.1.0 (gfx950)"; }

int32_t zr_device_count(int32_t *count) {
    ZR_GUARD_BEGIN
    int n = 0;
    ZR_HIP(hipGetDeviceCount(&n));
    *count = n;
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_set_device(int32_t device) {
    ZR_GUARD_BEGIN
    ZR_HIP(hipSetDevice(device));
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_rans_table_build(const uint32_t raw[256], zr_rans_table *out) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!raw || !out) return set_error(ZR_INVALID_INPUT, "null argument");
    return rans_normalize_host(raw, out);
    ZR_GUARD_END
}

size_t zr_rans_encode_bound(size_t n, uint32_t n_streams) {
    // <= 2 renorm bytes per symbol (state stays in [2^16, 2^24)) + header/state
    const size_t N = n_streams ? n_streams : 1;
    return 2 * n + 12 * N + 16;
}

int32_t zr_rans_dtab_upload(const zr_rans_table *tables, uint32_t n_tables, void *dtabs_dev,
                            void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (n_tables == 0) return ZR_OK;
    // the tables leave from a heap copy that a stream-ordered host callback
    // frees after the copy (no host synchronisation); a captured graph would
    // replay the copy from freed memory, so capture is refused
    if (capturing((hipStream_t)stream))
        return set_error(ZR_UNSUPPORTED, "zr_rans_dtab_upload stages host tables: not capturable");
    auto *h = new std::vector<RansDTab>(n_tables);
    for (uint32_t i = 0; i < n_tables; i++) rans_dtab_from_table(&tables[i], &(*h)[i]);
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemcpyAsync(dtabs_dev, h->data(), sizeof(RansDTab) * n_tables, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) {
        delete h;
        ZR_HIP(e);
    }
    ZR_HIP(hipLaunchHostFunc(
        s, [](void *p) { delete static_cast<std::vector<RansDTab> *>(p); }, h));
    return ZR_OK;
    ZR_GUARD_END
}

// ---- host-memory rANS (synchronous; Rans64Encoder::encode / Rans64Decoder::decode)
namespace {
// one-buffer batch run on a leased call context (no allocation in steady state,
// synchronisation on the context's stream only)
int32_t run_single(bool encode, const zr_rans_table *t, uint32_t N, const uint8_t *in, size_t in_len,
                   uint8_t *out, size_t out_cap, size_t n, size_t *out_len) {
    if (N == 0) N = 1;
    const size_t raw_len = encode ? in_len : n;
    const size_t enc_cap = encode ? zr_rans_encode_bound(in_len, N) : in_len;
    CallLease L;
    int32_t st = L.acquire();
    if (st) return st;
    void *d_raw, *d_enc, *d_meta, *d_tab, *d_ws;
    const size_t wsb = rans_workspace_bytes(1, N, raw_len);
    if ((st = L.get(0, raw_len, &d_raw)) || (st = L.get(1, enc_cap, &d_enc)) || (st = L.get(2, 64, &d_meta)) ||
        (st = L.get(3, sizeof(RansDTab), &d_tab)) || (st = L.get(4, wsb, &d_ws)))
        return st;
    CallCtx *c = L.ctx();
    hipStream_t s = L.stream();
    c->host_stage.resize(sizeof(RansDTab));
    RansDTab *h = reinterpret_cast<RansDTab *>(&c->host_stage[0]);
    rans_dtab_from_table(t, h);
    ZR_HIP(hipMemcpyAsync(d_tab, h, sizeof(RansDTab), hipMemcpyHostToDevice, s));
    uint64_t *meta = c->meta;
    meta[0] = raw_len;
    meta[1] = 0;
    meta[2] = 0;
    meta[3] = encode ? 0 : (uint64_t)in_len;
    meta[4] = 0;
    ZR_HIP(hipMemcpyAsync(d_meta, meta, 5 * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    uint64_t *m = reinterpret_cast<uint64_t *>(d_meta);
    zr_rans_batch bt;
    bt.n_buffers = 1;
    bt.n_streams = N;
    bt.max_len = raw_len;
    bt.len = m + 0;
    bt.raw_off = m + 1;
    bt.enc_off = m + 2;
    bt.enc_len = m + 3;
    bt.status = reinterpret_cast<int32_t *>(m + 4);
    bt.tables = d_tab;
    bt.table_stride = 0;
    bt.min_len = raw_len;
    if (encode) {
        if (in_len) ZR_HIP(hipMemcpyAsync(d_raw, in, in_len, hipMemcpyHostToDevice, s));
        st = zr_rans_encode_batch_dev(&bt, (const uint8_t *)d_raw, (uint8_t *)d_enc, d_ws, wsb, s);
    } else {
        if (in_len) ZR_HIP(hipMemcpyAsync(d_enc, in, in_len, hipMemcpyHostToDevice, s));
        st = zr_rans_decode_batch_dev(&bt, (const uint8_t *)d_enc, (uint8_t *)d_raw, d_ws, wsb, s);
    }
    if (st) return st;
    ZR_HIP(hipMemcpyAsync(meta, d_meta, 5 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    if ((st = L.sync())) return st;
    const int32_t status = (int32_t)(meta[4] & 0xFFFFFFFFu);
    if (status != 0) {
        if (encode) return set_error(ZR_INVALID_INPUT, "Symbol not in frequency table");
        return set_error(ZR_INVALID_INPUT, "Invalid or insufficient rANS data");
    }
    if (encode) {
        if (meta[3] > out_cap) return set_error(ZR_INVALID_INPUT, "output capacity too small");
        ZR_HIP(hipMemcpyAsync(out, d_enc, meta[3], hipMemcpyDeviceToHost, s));
        *out_len = meta[3];
    } else if (n) {
        ZR_HIP(hipMemcpyAsync(out, d_raw, n, hipMemcpyDeviceToHost, s));
    }
    return L.sync();
}
}  // namespace

int32_t zr_rans_encode(const zr_rans_table *t, uint32_t n_streams, const uint8_t *in, size_t n,
                       uint8_t *out, size_t out_cap, size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!t || (!in && n) || !out || !out_len) return set_error(ZR_INVALID_INPUT, "null argument");
    return run_single(true, t, n_streams, in, n, out, out_cap, 0, out_len);
    ZR_GUARD_END
}

int32_t zr_rans_decode(const zr_rans_table *t, uint32_t n_streams, const uint8_t *in, size_t in_len,
                       uint8_t *out, size_t n) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!t || (!in && in_len) || (!out && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    if (n == 0) return ZR_OK;  // rans.rs:511-513
    size_t dummy = 0;
    return run_single(false, t, n_streams, in, in_len, out, n, n, &dummy);
    ZR_GUARD_END
}

uint32_t zr_rans_adaptive_streams(size_t data_size) {
    // AdaptiveRans64Encoder::select_variant (rans.rs:669-681)
    if (data_size < 73) return 1;
    if (data_size < 73ull * 73) return 2;
    if (data_size < 73ull * 73 * 73 * 73) return 4;
    return 8;
}

int32_t zr_rans_encode_adaptive(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap, size_t *out_len,
                                uint32_t *n_streams) {
    ZR_GUARD_BEGIN
    clear_error();
    if ((!in && n) || !out || !out_len) return set_error(ZR_INVALID_INPUT, "null argument");
    // encode_adaptive (rans.rs:684-706): calculate_frequencies (:708-714, on
    // the device), Rans64Encoder::<P>::new, encode with P = select_variant
    uint32_t f[256];
    int32_t st = zr_byte_histogram(in, n, f);
    if (st) return st;
    zr_rans_table t;
    if ((st = rans_normalize_host(f, &t))) return st;
    const uint32_t N = zr_rans_adaptive_streams(n);
    if (n_streams) *n_streams = N;
    return run_single(true, &t, N, in, n, out, out_cap, 0, out_len);
    ZR_GUARD_END
}

int32_t zr_device_alloc_count(uint64_t *count) {
    if (!count) return set_error(ZR_INVALID_INPUT, "null argument");
    *count = g_dev_allocs.load(std::memory_order_relaxed);
    return ZR_OK;
}

// ---- device helpers
int32_t zr_malloc_dev(void **ptr, size_t bytes) {
    ZR_GUARD_BEGIN
    hipError_t e = dev_alloc(ptr, bytes);
    if (e != hipSuccess) return set_error(ZR_MEMORY_ERROR, "hipMalloc failed");
    return ZR_OK;
    ZR_GUARD_END
}
int32_t zr_free_dev(void *ptr) {
    ZR_GUARD_BEGIN
    ZR_HIP(hipFree(ptr));
    return ZR_OK;
    ZR_GUARD_END
}
int32_t zr_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream) {
    ZR_GUARD_BEGIN
    ZR_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    return ZR_OK;
    ZR_GUARD_END
}
int32_t zr_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream) {
    ZR_GUARD_BEGIN
    ZR_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    return ZR_OK;
    ZR_GUARD_END
}
int32_t zr_release_call_contexts(void) {
    ZR_GUARD_BEGIN
    clear_error();
    return release_call_contexts();
    ZR_GUARD_END
}
int32_t zr_memset_dev(void *dst, int value, size_t bytes, void *stream) {
    ZR_GUARD_BEGIN
    fill_dev(dst, value, bytes, (hipStream_t)stream);  // (a kernel: graph-capturable, see fill_dev)
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}
// device-to-device copy, 16 B per lane, four loads in flight per lane, grid
// sized to the chip (the one-pass streaming ceiling bench.py reports beside
// the 8 TB/s spec peak)
}  // extern "C"
namespace zr {
typedef unsigned cv4u __attribute__((ext_vector_type(4)));
// Each wave copies its own contiguous chunk in rounds of 8 KiB (eight 16-B
// loads per lane in flight, then eight stores): the access order that reads
// fastest on the box (tools/micro/sweep.hip: 6.1-6.4 TB/s per-wave chunks
// against 5.4 TB/s for a grid-wide in-order sweep). The remainder below a
// whole round per wave is copied grid-strided.
__global__ __launch_bounds__(256) void k_copy_stream(const cv4u *__restrict__ src, cv4u *__restrict__ dst,
                                                     uint64_t n16) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4, w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t per = (n16 / W) / 512 * 512;  // 16-B units per wave, whole 8 KiB rounds
    const cv4u *p = src + w * per + lane;
    cv4u *q = dst + w * per + lane;
    for (uint64_t u = 0; u < per; u += 512) {
        cv4u v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = __builtin_nontemporal_load(p + u + 64 * k);
#pragma unroll
        for (int k = 0; k < 8; k++) __builtin_nontemporal_store(v[k], q + u + 64 * k);
    }
    for (uint64_t i = W * per + (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        dst[i] = src[i];
}
__global__ void k_copy_tail(const uint8_t *src, uint8_t *dst, uint64_t n) {
    if (threadIdx.x < n) dst[threadIdx.x] = src[threadIdx.x];
}
}  // namespace zr
extern "C" {
int32_t zr_memcpy_dev(void *dst, const void *src, size_t bytes, uint32_t grid, void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (bytes == 0) return ZR_OK;
    if (!dst || !src) return set_error(ZR_INVALID_INPUT, "null argument");
    hipStream_t s = (hipStream_t)stream;
    const bool al = ((((uintptr_t)dst) | ((uintptr_t)src)) & 15) == 0;
    if (!al) {
        ZR_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
        return ZR_OK;
    }
    const uint64_t n16 = bytes / 16;
    if (grid == 0) grid = 8u * (uint32_t)cu_count();
    if (n16)
        hipLaunchKernelGGL(k_copy_stream, dim3(grid), dim3(256), 0, s, reinterpret_cast<const cv4u *>(src),
                           reinterpret_cast<cv4u *>(dst), n16);
    if (bytes % 16)
        hipLaunchKernelGGL(k_copy_tail, dim3(1), dim3(64), 0, s, reinterpret_cast<const uint8_t *>(src) + 16 * n16,
                           reinterpret_cast<uint8_t *>(dst) + 16 * n16, (uint64_t)(bytes % 16));
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}
int32_t zr_stream_sync(void *stream) {
    ZR_GUARD_BEGIN
    ZR_HIP(hipStreamSynchronize((hipStream_t)stream));
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_synth_fill(int32_t kind, uint64_t seed, uint8_t *out, size_t n) {
    ZR_GUARD_BEGIN
    if (kind < 0 || kind > 2 || (!out && n)) return set_error(ZR_INVALID_INPUT, "bad synth kind");
    synth(kind, seed, out, n);
    return ZR_OK;
    ZR_GUARD_END
}

}  // extern "C"

// ======================================================================
// kernel timers
// ======================================================================
namespace zr {
namespace {
struct TimerRec {
    std::string name;
    hipEvent_t a, b;
};
std::mutex g_tm;
bool g_timer_on = false;
std::string g_sel;  // ",name,name," : the timed kernels; empty = all
std::vector<TimerRec> g_recs;
std::vector<hipEvent_t> g_pool;
bool selected(const char *name) {
    return g_sel.empty() || g_sel.find("," + std::string(name) + ",") != std::string::npos;
}
hipEvent_t ev_get() {
    if (!g_pool.empty()) {
        hipEvent_t e = g_pool.back();
        g_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
}
}  // namespace

TimerPair timer_pair(const char *name) {
    std::lock_guard<std::mutex> g(g_tm);
    if (!g_timer_on || !selected(name)) return TimerPair{nullptr, nullptr};
    TimerRec r{name, ev_get(), ev_get()};
    g_recs.push_back(r);
    return TimerPair{r.a, r.b};
}
void timer_begin(const char *name, hipStream_t s) {
    std::lock_guard<std::mutex> g(g_tm);
    if (!g_timer_on || !selected(name)) return;
    TimerRec r{name, ev_get(), ev_get()};
    (void)hipEventRecord(r.a, s);
    g_recs.push_back(r);
}
void timer_end(const char *name, hipStream_t s) {
    std::lock_guard<std::mutex> g(g_tm);
    if (!g_timer_on || !selected(name)) return;
    for (auto it = g_recs.rbegin(); it != g_recs.rend(); ++it)
        if (it->name == name) {
            (void)hipEventRecord(it->b, s);
            return;
        }
}
}  // namespace zr

extern "C" {
int32_t zr_timer_enable(int32_t on) {
    std::lock_guard<std::mutex> g(g_tm);
    g_timer_on = on != 0;
    // events are created here, not per launch inside a timed region
    while (g_timer_on && g_pool.size() + 2 * g_recs.size() < 1024) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) break;
        g_pool.push_back(e);
    }
    return ZR_OK;
}
int32_t zr_timer_select(const char *names) {
    std::lock_guard<std::mutex> g(g_tm);
    g_sel.clear();
    if (names && *names) g_sel = "," + std::string(names) + ",";
    return ZR_OK;
}
int32_t zr_timer_reset(void) {
    std::lock_guard<std::mutex> g(g_tm);
    for (auto &r : g_recs) {
        (void)hipEventSynchronize(r.b);
        g_pool.push_back(r.a);
        g_pool.push_back(r.b);
    }
    g_recs.clear();
    return ZR_OK;
}
int32_t zr_timer_read(const char *kernel, double *total_ms, uint64_t *launches) {
    ZR_GUARD_BEGIN
    std::lock_guard<std::mutex> g(g_tm);
    double tot = 0;
    uint64_t n = 0;
    for (auto &r : g_recs)
        if (r.name == kernel) {
            ZR_HIP(hipEventSynchronize(r.b));
            float ms = 0;
            ZR_HIP(hipEventElapsedTime(&ms, r.a, r.b));
            tot += ms;
            n++;
        }
    *total_ms = tot;
    *launches = n;
    return ZR_OK;
    ZR_GUARD_END
}
}  // extern "C"
