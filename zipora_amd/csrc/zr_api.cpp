// zr_api.cpp -- host side of the C ABI: error state, table construction,
// host-memory entry points, device helpers and synthetic inputs.
#include <algorithm>
#include <cmath>
#include <cstring>
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
        const uint32_t l = f <= 1 ? 0u : 32u - (uint32_t)__builtin_clz(f - 1);
        d->rsh[s] = l;
        d->rcp[s] = f ? (uint32_t)(((1ull << (24 + l)) + f - 1) / f) : 0u;
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
    std::vector<RansDTab> h(n_tables);
    for (uint32_t i = 0; i < n_tables; i++) rans_dtab_from_table(&tables[i], &h[i]);
    ZR_HIP(hipMemcpyAsync(dtabs_dev, h.data(), sizeof(RansDTab) * n_tables, hipMemcpyHostToDevice,
                          (hipStream_t)stream));
    ZR_HIP(hipStreamSynchronize((hipStream_t)stream));
    return ZR_OK;
    ZR_GUARD_END
}

// ---- host-memory rANS (synchronous; Rans64Encoder::encode / Rans64Decoder::decode)
namespace {
struct DevBuf {
    void *p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t n) { return hipMalloc(&p, n ? n : 16); }
};

// one-buffer batch run against device copies of the arguments
int32_t run_single(bool encode, const zr_rans_table *t, uint32_t N, const uint8_t *in, size_t in_len,
                   uint8_t *out, size_t out_cap, size_t n, size_t *out_len) {
    if (N == 0) N = 1;
    const size_t raw_len = encode ? in_len : n;
    const size_t enc_cap = encode ? zr_rans_encode_bound(in_len, N) : in_len;
    DevBuf d_raw, d_enc, d_meta, d_tab, d_ws;
    ZR_HIP(d_raw.alloc(raw_len));
    ZR_HIP(d_enc.alloc(enc_cap));
    ZR_HIP(d_meta.alloc(64));
    ZR_HIP(d_tab.alloc(sizeof(RansDTab)));
    const size_t wsb = rans_workspace_bytes(1, N, raw_len);
    ZR_HIP(d_ws.alloc(wsb));
    RansDTab *h = new RansDTab;
    rans_dtab_from_table(t, h);
    hipError_t e = hipMemcpy(d_tab.p, h, sizeof(RansDTab), hipMemcpyHostToDevice);
    delete h;
    ZR_HIP(e);
    uint64_t meta[5] = {raw_len, 0, 0, encode ? 0 : (uint64_t)in_len, 0};
    ZR_HIP(hipMemcpy(d_meta.p, meta, sizeof(meta), hipMemcpyHostToDevice));
    uint64_t *m = reinterpret_cast<uint64_t *>(d_meta.p);
    zr_rans_batch bt;
    bt.n_buffers = 1;
    bt.n_streams = N;
    bt.max_len = raw_len;
    bt.len = m + 0;
    bt.raw_off = m + 1;
    bt.enc_off = m + 2;
    bt.enc_len = m + 3;
    bt.status = reinterpret_cast<int32_t *>(m + 4);
    bt.tables = d_tab.p;
    bt.table_stride = 0;
    bt.min_len = raw_len;
    int32_t st;
    if (encode) {
        if (in_len) ZR_HIP(hipMemcpy(d_raw.p, in, in_len, hipMemcpyHostToDevice));
        st = zr_rans_encode_batch_dev(&bt, (const uint8_t *)d_raw.p, (uint8_t *)d_enc.p, d_ws.p, wsb, nullptr);
    } else {
        if (in_len) ZR_HIP(hipMemcpy(d_enc.p, in, in_len, hipMemcpyHostToDevice));
        st = zr_rans_decode_batch_dev(&bt, (const uint8_t *)d_enc.p, (uint8_t *)d_raw.p, d_ws.p, wsb, nullptr);
    }
    if (st) return st;
    ZR_HIP(hipDeviceSynchronize());
    ZR_HIP(hipMemcpy(meta, d_meta.p, sizeof(meta), hipMemcpyDeviceToHost));
    const int32_t status = (int32_t)(meta[4] & 0xFFFFFFFFu);
    if (status != 0) {
        if (encode) return set_error(ZR_INVALID_INPUT, "Symbol not in frequency table");
        return set_error(ZR_INVALID_INPUT, "Invalid or insufficient rANS data");
    }
    if (encode) {
        if (meta[3] > out_cap) return set_error(ZR_INVALID_INPUT, "output capacity too small");
        ZR_HIP(hipMemcpy(out, d_enc.p, meta[3], hipMemcpyDeviceToHost));
        *out_len = meta[3];
    } else if (n) {
        ZR_HIP(hipMemcpy(out, d_raw.p, n, hipMemcpyDeviceToHost));
    }
    return ZR_OK;
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

// ---- device helpers
int32_t zr_malloc_dev(void **ptr, size_t bytes) {
    ZR_GUARD_BEGIN
    hipError_t e = hipMalloc(ptr, bytes ? bytes : 16);
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
int32_t zr_memset_dev(void *dst, int value, size_t bytes, void *stream) {
    ZR_GUARD_BEGIN
    ZR_HIP(hipMemsetAsync(dst, value, bytes, (hipStream_t)stream));
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
std::vector<TimerRec> g_recs;
std::vector<hipEvent_t> g_pool;
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

void timer_begin(const char *name, hipStream_t s) {
    std::lock_guard<std::mutex> g(g_tm);
    if (!g_timer_on) return;
    TimerRec r{name, ev_get(), ev_get()};
    (void)hipEventRecord(r.a, s);
    g_recs.push_back(r);
}
void timer_end(const char *name, hipStream_t s) {
    std::lock_guard<std::mutex> g(g_tm);
    if (!g_timer_on) return;
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
