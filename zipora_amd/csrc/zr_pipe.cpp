// zr_pipe.cpp -- host-resident rANS batches with overlapped copies
// (blob-store records and file buffers start and end in
// host memory).
//
// The buffers of a call are cut into groups of whole buffers (contiguous in
// host memory). Each group goes through one of ZR_PIPE_SLOTS (3) device slots
// on three HIP streams, so group g+1's host-to-device copy, group g's coding
// and group g-1's device-to-host copy run at the same time:
//
//   s_in : input span H2D -> event in_done
//   s_cmp: wait in_done, meta in, zr_rans_{encode,decode}_batch_dev, lengths and
//          statuses out -> event code_done
//   s_out: wait code_done, output span D2H -> event out_done
//
// A slot is reused only after its out_done: by then its device buffers and its
// pinned meta staging are free. The device layout of a group mirrors the
// caller's host offsets (relative to the group's first buffer), so each span
// moves with one copy. Host buffers should be pinned (zr_host_register) for the
// full PCIe rate; pageable memory works but copies through a driver bounce.
#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "zr_internal.h"

using namespace zr;

namespace {

struct Slot {
    uint8_t *raw = nullptr, *enc = nullptr;  // device spans
    size_t raw_cap = 0, enc_cap = 0;
    void *ws = nullptr;
    size_t ws_cap = 0;
    uint8_t *pack = nullptr;    // packed encode output (device)
    size_t pack_cap = 0;
    void *poff = nullptr;       // packed offsets (device)
    size_t poff_cap = 0;
    uint64_t *meta = nullptr;   // device: len | raw_off | enc_off | enc_len, then int32 status
    uint64_t *hmeta = nullptr;  // pinned host mirror
    uint64_t *hmeta_dev = nullptr;  // its device-side address
    uint32_t meta_cap = 0;      // buffers
    hipEvent_t in_done = nullptr, code_done = nullptr, out_done = nullptr;
    bool busy = false;          // a group is in flight
    uint32_t b0 = 0, nb = 0;    // the group in flight (for collecting results)
};

size_t meta_bytes(uint32_t nb) { return (size_t)nb * 4 * 8 + round_up((size_t)nb * 4, 8); }

// Meta moves between the pinned staging and the slot by kernels on the coding
// stream (the staging is mapped into the device address space): small
// hipMemcpyAsync calls are serviced synchronously by the runtime and would
// serialise the copy streams.
__global__ void k_words(const uint64_t *__restrict__ src, uint64_t *__restrict__ dst, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = src[i];
}

// Packed encode output (records back to back, the ZipOffset content layout:
// offsets = exclusive scan of the lengths): the group's exclusive scan of the
// encoded lengths (failed buffers count 0), then one wave per buffer moves its
// bytes from the bound-sized slot to the packed position.
__global__ __launch_bounds__(1024) void k_pack_scan(const uint64_t *enc_len, const int32_t *status, uint32_t nb,
                                                    uint64_t *poff) {
    __shared__ unsigned long long wsum[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    unsigned long long carry = 0;
    for (uint32_t base = 0; base < nb; base += 1024) {
        const uint32_t i = base + tid;
        const unsigned long long v = (i < nb && status[i] == 0) ? enc_len[i] : 0;
        unsigned long long inc = v;
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const unsigned long long t = __shfl_up(inc, d, 64);
            if (lane >= d) inc += t;
        }
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        unsigned long long before = 0, total = 0;
        for (uint32_t w = 0; w < 16; w++) {
            before += w < wv ? wsum[w] : 0;
            total += wsum[w];
        }
        if (i < nb) poff[i] = carry + before + inc - v;
        carry += total;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_pack_copy(const uint8_t *src, const uint64_t *slot_off,
                                                   const uint64_t *enc_len, const int32_t *status,
                                                   const uint64_t *poff, uint8_t *dst, uint32_t nb) {
    const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= nb || status[i] != 0) return;
    const uint64_t L = enc_len[i];
    const uint8_t *sp = src + slot_off[i];
    uint8_t *dp = dst + poff[i];
    for (uint64_t k = lane; k < L; k += 64) dp[k] = sp[k];
}

int32_t copy_words(const uint64_t *src, uint64_t *dst, size_t n, hipStream_t s) {
    if (!n) return ZR_OK;
    const uint32_t grid = (uint32_t)std::min<size_t>(ceil_div(n, 256), 64);
    hipLaunchKernelGGL(k_words, dim3(grid), dim3(256), 0, s, src, dst, (uint32_t)n);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
}

}  // namespace

// device slots: a group's input copy waits for the copy back of the group
// ZR_PIPE_SLOTS earlier (the slot it reuses). With two, group g+1's input copy
// waited for group g-1's copy back, which waits for group g-1's coding: the
// input link idled for a coding time per group. Same box, 64 x 4 MiB x4096,
// pinned (tools/pipe_ab.py): encode 26-27.5 -> 36-37 GiB/s, decode 37 -> 39.5,
// both 15.5 -> 19.0; 1 M x 1 KiB records 16.4 -> 19.2; four slots: the same
// as three.
#ifndef ZR_PIPE_SLOTS
#define ZR_PIPE_SLOTS 3
#endif
struct zr_rans_pipe {
    uint32_t N = 1;
    uint64_t group_cap = 0;
    hipStream_t s_in = nullptr, s_cmp = nullptr, s_out = nullptr;
    Slot slot[ZR_PIPE_SLOTS];
    void *dtab = nullptr;  // the shared device table
};

namespace {

// Slot buffers are whole 2 MiB multiples: an odd-sized hipMalloc is backed by
// small pages and the copy engines crawl through it (measured: 30 GB/s instead
// of 56 GB/s for a 32.4 MiB span).
int32_t grow(void **p, size_t *cap, size_t need) {
    if (need <= *cap) return ZR_OK;
    need = round_up(need, (size_t)2 << 20);
    if (*p) ZR_HIP(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    ZR_HIP(dev_alloc(p, need));
    *cap = need;
    return ZR_OK;
}

int32_t slot_meta(Slot &S, uint32_t nb) {
    if (nb <= S.meta_cap) return ZR_OK;
    if (S.meta) ZR_HIP(hipFree(S.meta));
    if (S.hmeta) ZR_HIP(hipHostFree(S.hmeta));
    S.meta = nullptr;
    S.hmeta = nullptr;
    ZR_HIP(dev_alloc(reinterpret_cast<void **>(&S.meta), meta_bytes(nb)));
    ZR_HIP(hipHostMalloc(reinterpret_cast<void **>(&S.hmeta), meta_bytes(nb),
                         hipHostMallocMapped | hipHostMallocCoherent));
    ZR_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&S.hmeta_dev), S.hmeta, 0));
    S.meta_cap = nb;
    return ZR_OK;
}

// Results of the group a slot last carried (valid after its out_done).
void collect(const Slot &S, uint64_t *enc_len, int32_t *status) {
    const uint64_t *h = S.hmeta;
    const int32_t *st = reinterpret_cast<const int32_t *>(h + 4 * (size_t)S.nb);
    for (uint32_t i = 0; i < S.nb; i++) {
        if (enc_len) enc_len[S.b0 + i] = h[3 * (size_t)S.nb + i];
        if (status) status[S.b0 + i] = st[i];
    }
}

// Cut [0, B) into groups of whole buffers: at most group_cap raw bytes each
// (a larger buffer forms a group of its own).
std::vector<std::pair<uint32_t, uint32_t>> groups(const uint64_t *len, uint32_t B, uint64_t cap) {
    std::vector<std::pair<uint32_t, uint32_t>> g;
    uint32_t b0 = 0;
    uint64_t acc = 0;
    for (uint32_t b = 0; b < B; b++) {
        if (b > b0 && acc + len[b] > cap) {
            g.push_back({b0, b});
            b0 = b;
            acc = 0;
        }
        acc += len[b];
    }
    if (B > b0) g.push_back({b0, B});
    return g;
}

// ZR_PIPE_TRACE=1: per-group timeline of the three streams on stderr (diagnostic)
struct Trace {
    bool on = std::getenv("ZR_PIPE_TRACE") != nullptr;
    std::vector<std::array<hipEvent_t, 6>> ev;  // per group: in, code, out (start, end)
    void mark(size_t g, int k, hipStream_t s) {
        if (!on) return;
        if (ev.size() <= g) ev.resize(g + 1, std::array<hipEvent_t, 6>{});
        (void)hipEventCreate(&ev[g][k]);
        (void)hipEventRecord(ev[g][k], s);
    }
    void dump() {
        if (!on || ev.empty()) return;
        (void)hipDeviceSynchronize();
        for (size_t g = 0; g < ev.size(); g++) {
            float t[6] = {};
            for (int k = 0; k < 6; k++)
                if (ev[g][k]) (void)hipEventElapsedTime(&t[k], ev[0][0], ev[g][k]);
            std::fprintf(stderr, "zr_pipe group %zu: in %.3f-%.3f code %.3f-%.3f out %.3f-%.3f ms\n", g, t[0], t[1],
                         t[2], t[3], t[4], t[5]);
        }
        for (auto &a : ev)
            for (hipEvent_t e : a)
                if (e) (void)hipEventDestroy(e);
        ev.clear();
    }
};

// Extents of a group's buffers in one area ([off, off + n) each, relative to
// the group's lowest offset), sorted and merged across gaps under kGap so that
// runs of small records move in one copy and the slack of bound-sized encoded
// slots does not cross PCIe.
constexpr uint64_t kGap = 256 << 10;

std::vector<std::pair<uint64_t, uint64_t>> extents(const uint64_t *off, const uint64_t *n, uint32_t b0,
                                                   uint32_t b1, uint64_t base) {
    std::vector<std::pair<uint64_t, uint64_t>> v;
    v.reserve(b1 - b0);
    for (uint32_t b = b0; b < b1; b++)
        if (n[b]) v.push_back({off[b] - base, off[b] - base + n[b]});
    if (!std::is_sorted(v.begin(), v.end())) std::sort(v.begin(), v.end());
    std::vector<std::pair<uint64_t, uint64_t>> m;
    for (const auto &e : v) {
        if (!m.empty() && e.first <= m.back().second + kGap)
            m.back().second = std::max(m.back().second, e.second);
        else
            m.push_back(e);
    }
    return m;
}

int32_t copy_extents(uint8_t *dst, const uint8_t *src, const std::vector<std::pair<uint64_t, uint64_t>> &ex,
                     hipMemcpyKind kind, hipStream_t s) {
    for (const auto &e : ex)
        ZR_HIP(hipMemcpyAsync(dst + e.first, src + e.first, e.second - e.first, kind, s));
    return ZR_OK;
}

// One direction of the pipeline. Group g's input copy and coding are issued,
// then group g-1's copy back (encode first waits for g-1's coding on the host:
// only then are its encoded lengths, and so the extents to copy, known).
// packed encode: the caller gets enc_off back (records back to back from 0)
struct Packed {
    bool on = false;
    size_t cap = 0;
    uint64_t *off_out = nullptr;
    uint64_t pos = 0;
};

int32_t run_impl(zr_rans_pipe *p, bool encode, uint32_t B, const uint64_t *len, uint8_t *raw,
                 const uint64_t *raw_off, uint8_t *enc, const uint64_t *enc_off, uint64_t *enc_len,
                 int32_t *status, Packed *pk) {
    const uint32_t N = p->N;
    const auto gs = groups(len, B, p->group_cap);
    Trace tr;
    std::vector<uint64_t> bound(encode ? B : 0);
    for (uint32_t b = 0; b < (encode ? B : 0); b++) bound[b] = zr_rans_encode_bound(len[b], N);
    const bool packed = pk && pk->on;
    std::vector<uint64_t> slots;  // packed: the device slot layout (16-byte aligned bound slots)
    if (packed) {
        slots.resize(B);
        uint64_t o = 0;
        for (uint32_t b = 0; b < B; b++) {
            slots[b] = o;
            o += round_up(bound[b], 16);
        }
        enc_off = slots.data();
    }
    const uint64_t *enc_n = encode ? bound.data() : enc_len;  // encoded extent per buffer, device side
    std::vector<uint64_t> rbase(gs.size()), ebase(gs.size());
    std::vector<uint8_t> use_pack(gs.size(), 0);  // packed groups of small records: device packing

    auto issue_out = [&](size_t gi) -> int32_t {
        Slot &S = p->slot[gi % ZR_PIPE_SLOTS];
        const uint32_t b0 = gs[gi].first, b1 = gs[gi].second, nb = b1 - b0;
        ZR_HIP(hipStreamWaitEvent(p->s_out, S.code_done, 0));
        tr.mark(gi, 4, p->s_out);
        if (encode && packed) {
            ZR_HIP(hipEventSynchronize(S.code_done));
            const uint64_t *el = S.hmeta + 3 * (size_t)nb;
            const int32_t *stt = reinterpret_cast<const int32_t *>(S.hmeta + 4 * (size_t)nb);
            uint64_t tot = 0;
            for (uint32_t i = 0; i < nb; i++) {
                pk->off_out[b0 + i] = pk->pos + tot;
                tot += stt[i] == 0 ? el[i] : 0;
            }
            if (pk->pos + tot > pk->cap) return set_error(ZR_INVALID_INPUT, "packed output buffer too small");
            if (use_pack[gi]) {
                if (tot) ZR_HIP(hipMemcpyAsync(enc + pk->pos, S.pack, tot, hipMemcpyDeviceToHost, p->s_out));
            } else {  // large records: each straight from its slot to its packed place
                for (uint32_t i = 0; i < nb; i++) {
                    const uint64_t L = stt[i] == 0 ? el[i] : 0;
                    if (L)
                        ZR_HIP(hipMemcpyAsync(enc + pk->off_out[b0 + i], S.enc + (enc_off[b0 + i] - ebase[gi]), L,
                                              hipMemcpyDeviceToHost, p->s_out));
                }
            }
            pk->pos += tot;
        } else if (encode) {
            ZR_HIP(hipEventSynchronize(S.code_done));
            const uint64_t *el = S.hmeta + 3 * (size_t)nb;
            std::vector<uint64_t> off(nb), n(nb);
            for (uint32_t i = 0; i < nb; i++) {
                off[i] = enc_off[b0 + i] - ebase[gi];
                n[i] = std::min(el[i], bound[b0 + i]);
            }
            const auto ex = extents(off.data(), n.data(), 0, nb, 0);
            if (int32_t st = copy_extents(enc + ebase[gi], S.enc, ex, hipMemcpyDeviceToHost, p->s_out)) return st;
        } else {
            const auto ex = extents(raw_off, len, b0, b1, rbase[gi]);
            if (int32_t st = copy_extents(raw + rbase[gi], S.raw, ex, hipMemcpyDeviceToHost, p->s_out)) return st;
        }
        tr.mark(gi, 5, p->s_out);
        ZR_HIP(hipEventRecord(S.out_done, p->s_out));
        return ZR_OK;
    };

    for (size_t gi = 0; gi < gs.size(); gi++) {
        Slot &S = p->slot[gi % ZR_PIPE_SLOTS];
        if (S.busy) {  // the slot's previous group: wait for its copies back, keep its results
            ZR_HIP(hipEventSynchronize(S.out_done));
            collect(S, encode ? enc_len : nullptr, status);
            S.busy = false;
        }
        const uint32_t b0 = gs[gi].first, b1 = gs[gi].second, nb = b1 - b0;
        uint64_t max_len = 0, min_len = ~0ull, rb = ~0ull, re = 0, eb = ~0ull, ee = 0;
        for (uint32_t b = b0; b < b1; b++) {
            max_len = std::max(max_len, len[b]);
            min_len = std::min(min_len, len[b]);
            rb = std::min(rb, raw_off[b]);
            re = std::max(re, raw_off[b] + len[b]);
            eb = std::min(eb, enc_off[b]);
            ee = std::max(ee, enc_off[b] + enc_n[b]);
        }
        rbase[gi] = rb;
        ebase[gi] = eb;
        int32_t st;
        if ((st = grow(reinterpret_cast<void **>(&S.raw), &S.raw_cap, std::max<uint64_t>(re - rb, 16)))) return st;
        if ((st = grow(reinterpret_cast<void **>(&S.enc), &S.enc_cap, std::max<uint64_t>(ee - eb, 16)))) return st;
        if ((st = grow(&S.ws, &S.ws_cap, rans_workspace_bytes(nb, N, max_len)))) return st;
        if ((st = slot_meta(S, nb))) return st;
        // meta: len | raw_off | enc_off | enc_len (relative to the slot areas), statuses
        uint64_t *h = S.hmeta;
        for (uint32_t i = 0; i < nb; i++) {
            const uint32_t b = b0 + i;
            h[i] = len[b];
            h[nb + i] = raw_off[b] - rb;
            h[2 * (size_t)nb + i] = enc_off[b] - eb;
            h[3 * (size_t)nb + i] = encode ? 0 : enc_len[b];
        }
        std::memset(h + 4 * (size_t)nb, 0, round_up((size_t)nb * 4, 8));
        tr.mark(gi, 0, p->s_in);
        if (encode) {
            const auto ex = extents(raw_off, len, b0, b1, rb);
            if ((st = copy_extents(S.raw, raw + rb, ex, hipMemcpyHostToDevice, p->s_in))) return st;
        } else {
            const auto ex = extents(enc_off, enc_len, b0, b1, eb);
            if ((st = copy_extents(S.enc, enc + eb, ex, hipMemcpyHostToDevice, p->s_in))) return st;
        }
        tr.mark(gi, 1, p->s_in);
        ZR_HIP(hipEventRecord(S.in_done, p->s_in));
        // coding
        ZR_HIP(hipStreamWaitEvent(p->s_cmp, S.in_done, 0));
        tr.mark(gi, 2, p->s_cmp);
        if ((st = copy_words(S.hmeta_dev, S.meta, meta_bytes(nb) / 8, p->s_cmp))) return st;
        zr_rans_batch bt;
        bt.n_buffers = nb;
        bt.n_streams = N;
        bt.max_len = max_len;
        bt.min_len = min_len;
        bt.len = S.meta;
        bt.raw_off = S.meta + nb;
        bt.enc_off = S.meta + 2 * (size_t)nb;
        bt.enc_len = S.meta + 3 * (size_t)nb;
        bt.status = reinterpret_cast<int32_t *>(S.meta + 4 * (size_t)nb);
        bt.tables = p->dtab;
        bt.table_stride = 0;
        st = encode ? zr_rans_encode_batch_dev(&bt, S.raw, S.enc, S.ws, S.ws_cap, p->s_cmp)
                    : zr_rans_decode_batch_dev(&bt, S.enc, S.raw, S.ws, S.ws_cap, p->s_cmp);
        if (st) return st;
        // lengths and statuses back to the staging
        if ((st = copy_words(S.meta + 3 * (size_t)nb, S.hmeta_dev + 3 * (size_t)nb,
                             meta_bytes(nb) / 8 - 3 * (size_t)nb, p->s_cmp)))
            return st;
        use_pack[gi] = packed && max_len <= (64u << 10);
        if (use_pack[gi]) {  // small records: back to back in S.pack (group-relative offsets)
            if ((st = grow(reinterpret_cast<void **>(&S.pack), &S.pack_cap, std::max<uint64_t>(ee - eb, 16))))
                return st;
            if ((st = grow(&S.poff, &S.poff_cap, 8 * (size_t)nb))) return st;
            const int32_t *dst = reinterpret_cast<const int32_t *>(S.meta + 4 * (size_t)nb);
            hipLaunchKernelGGL(k_pack_scan, dim3(1), dim3(1024), 0, p->s_cmp, S.meta + 3 * (size_t)nb, dst, nb,
                               reinterpret_cast<uint64_t *>(S.poff));
            hipLaunchKernelGGL(k_pack_copy, dim3((nb + 3) / 4), dim3(256), 0, p->s_cmp, S.enc, S.meta + 2 * (size_t)nb,
                               S.meta + 3 * (size_t)nb, dst, reinterpret_cast<const uint64_t *>(S.poff), S.pack,
                               nb);
            ZR_HIP(hipGetLastError());
        }
        tr.mark(gi, 3, p->s_cmp);
        ZR_HIP(hipEventRecord(S.code_done, p->s_cmp));
        S.busy = true;
        S.b0 = b0;
        S.nb = nb;
        if (gi > 0 && (st = issue_out(gi - 1))) return st;
    }
    if (!gs.empty()) {
        if (int32_t st = issue_out(gs.size() - 1)) return st;
    }
    for (Slot &S : p->slot) {
        if (!S.busy) continue;
        ZR_HIP(hipEventSynchronize(S.out_done));
        collect(S, encode ? enc_len : nullptr, status);
        S.busy = false;
    }
    tr.dump();
    return ZR_OK;
}

// Any error return leaves copies in flight on the three streams and slots
// marked busy with this call's group geometry. Drain every stream before
// returning (no copy may land in caller memory after the error is reported)
// and forget the slots, so the next call starts clean.
int32_t run(zr_rans_pipe *p, bool encode, uint32_t B, const uint64_t *len, uint8_t *raw, const uint64_t *raw_off,
            uint8_t *enc, const uint64_t *enc_off, uint64_t *enc_len, int32_t *status, Packed *pk = nullptr) {
    const int32_t st = run_impl(p, encode, B, len, raw, raw_off, enc, enc_off, enc_len, status, pk);
    if (st != ZR_OK) {
        (void)hipStreamSynchronize(p->s_in);
        (void)hipStreamSynchronize(p->s_cmp);
        (void)hipStreamSynchronize(p->s_out);
        for (Slot &S : p->slot) {
            S.busy = false;
            S.b0 = S.nb = 0;
        }
    }
    return st;
}

void release(zr_rans_pipe *p) {
    for (Slot &S : p->slot) {
        if (S.raw) (void)hipFree(S.raw);
        if (S.enc) (void)hipFree(S.enc);
        if (S.ws) (void)hipFree(S.ws);
        if (S.meta) (void)hipFree(S.meta);
        if (S.hmeta) (void)hipHostFree(S.hmeta);
        if (S.pack) (void)hipFree(S.pack);
        if (S.poff) (void)hipFree(S.poff);
        if (S.in_done) (void)hipEventDestroy(S.in_done);
        if (S.code_done) (void)hipEventDestroy(S.code_done);
        if (S.out_done) (void)hipEventDestroy(S.out_done);
    }
    if (p->dtab) (void)hipFree(p->dtab);
    if (p->s_in) (void)hipStreamDestroy(p->s_in);
    if (p->s_cmp) (void)hipStreamDestroy(p->s_cmp);
    if (p->s_out) (void)hipStreamDestroy(p->s_out);
    delete p;
}

}  // namespace

extern "C" {

int32_t zr_rans_pipe_create(const zr_rans_table *table, uint32_t n_streams, uint64_t group_bytes,
                            zr_rans_pipe **out) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!table || !out) return set_error(ZR_INVALID_INPUT, "null argument");
    *out = nullptr;
    zr_rans_pipe *p = new zr_rans_pipe;
    p->N = n_streams ? n_streams : 1;
    p->group_cap = group_bytes ? group_bytes : (32ull << 20);
    auto fail = [&](int32_t st) {
        release(p);
        return st;
    };
    if (hipStreamCreateWithFlags(&p->s_in, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&p->s_cmp, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&p->s_out, hipStreamNonBlocking) != hipSuccess)
        return fail(set_error(ZR_INTERNAL, "hipStreamCreate failed"));
    for (Slot &S : p->slot) {
        if (hipEventCreateWithFlags(&S.in_done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&S.code_done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&S.out_done, hipEventDisableTiming) != hipSuccess)
            return fail(set_error(ZR_INTERNAL, "hipEventCreate failed"));
    }
    if (dev_alloc(&p->dtab, zr_rans_dtab_bytes()) != hipSuccess)
        return fail(set_error(ZR_MEMORY_ERROR, "hipMalloc failed"));
    int32_t st = zr_rans_dtab_upload(table, 1, p->dtab, p->s_cmp);
    if (st) return fail(st);
    if (hipStreamSynchronize(p->s_cmp) != hipSuccess) return fail(set_error(ZR_INTERNAL, "table upload failed"));
    *out = p;
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_rans_pipe_destroy(zr_rans_pipe *p) {
    ZR_GUARD_BEGIN
    if (p) release(p);
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_rans_pipe_encode(zr_rans_pipe *p, uint32_t n_buffers, const uint64_t *len, const uint8_t *raw,
                            const uint64_t *raw_off, uint8_t *enc, const uint64_t *enc_off, uint64_t *enc_len,
                            int32_t *status) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!p || (n_buffers && (!len || !raw || !raw_off || !enc || !enc_off || !enc_len || !status)))
        return set_error(ZR_INVALID_INPUT, "null argument");
    return run(p, true, n_buffers, len, const_cast<uint8_t *>(raw), raw_off, enc, enc_off, enc_len, status);
    ZR_GUARD_END
}

int32_t zr_rans_pipe_encode_packed(zr_rans_pipe *p, uint32_t n_buffers, const uint64_t *len, const uint8_t *raw,
                                   const uint64_t *raw_off, uint8_t *enc, size_t enc_cap, uint64_t *enc_off,
                                   uint64_t *enc_len, int32_t *status, uint64_t *enc_total) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!p || !enc_total ||
        (n_buffers && (!len || !raw || !raw_off || !enc || !enc_off || !enc_len || !status)))
        return set_error(ZR_INVALID_INPUT, "null argument");
    Packed pk;
    pk.on = true;
    pk.cap = enc_cap;
    pk.off_out = enc_off;
    int32_t st = run(p, true, n_buffers, len, const_cast<uint8_t *>(raw), raw_off, enc, nullptr, enc_len, status, &pk);
    *enc_total = pk.pos;
    if (!st)  // failed buffers hold no bytes in the packed layout
        for (uint32_t b = 0; b < n_buffers; b++)
            if (status[b] != 0) enc_len[b] = 0;
    return st;
    ZR_GUARD_END
}

int32_t zr_rans_pipe_decode(zr_rans_pipe *p, uint32_t n_buffers, const uint64_t *len, const uint8_t *enc,
                            const uint64_t *enc_off, const uint64_t *enc_len, uint8_t *raw,
                            const uint64_t *raw_off, int32_t *status) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!p || (n_buffers && (!len || !raw || !raw_off || !enc || !enc_off || !enc_len || !status)))
        return set_error(ZR_INVALID_INPUT, "null argument");
    return run(p, false, n_buffers, len, raw, raw_off, const_cast<uint8_t *>(enc), enc_off,
               const_cast<uint64_t *>(enc_len), status);
    ZR_GUARD_END
}

int32_t zr_host_register(void *ptr, size_t bytes) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!ptr || !bytes) return ZR_OK;
    ZR_HIP(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_host_unregister(void *ptr) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!ptr) return ZR_OK;
    ZR_HIP(hipHostUnregister(ptr));
    return ZR_OK;
    ZR_GUARD_END
}

}  // extern "C"
