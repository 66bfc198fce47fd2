// zr_rans.hip -- rANS order-0 (src/entropy/rans.rs) on MI355X / gfx950.
//
// Layout in HBM (bit-exact with the reference, rans.rs:402-419 / Appendix A):
//   xN (len >= N > 1): state[0..N]:u64 LE | len[0..N]:u32 LE | stream_0 | ... | stream_{N-1}
//   x1 (N == 1 or len < N): renorm bytes in emission order | state:u64 LE
// Stream s holds symbols s, s+N, s+2N, ...; encoded last-to-first, decoded first-to-last
// reading its bytes backwards.
//
// Work decomposition: one lane = one coder state = one stream. A 256-thread
// workgroup owns 256 consecutive streams of one buffer, so step k of the
// workgroup touches 256 consecutive bytes raw[k*N + 256*blk ...]: the raw side
// is staged through an LDS tile and moved with 16-byte coalesced accesses.
// The decode slot table (16 KiB) and encode symbol table (2 KiB) live in LDS.
// Per-buffer x1 streams (blob records) run one lane per buffer.
#include <cstdlib>

#include "zr_internal.h"

namespace zr {

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t ld_u32_u(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint64_t ld_u64_u(const uint8_t *p) {
    return (uint64_t)ld_u32_u(p) | ((uint64_t)ld_u32_u(p + 4) << 32);
}
__device__ __forceinline__ void st_u32_u(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

__device__ __forceinline__ unsigned long long wave_incl_scan(unsigned long long v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        unsigned long long t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// exclusive scan over a 256-thread block; sh must hold 4 entries
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, unsigned long long *sh,
                                                    uint64_t *total) {
    unsigned long long inc = wave_incl_scan(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) sh[w] = inc;
    __syncthreads();
    unsigned long long base = 0;
    for (int i = 0; i < w; i++) base += sh[i];
    if (total) *total = sh[0] + sh[1] + sh[2] + sh[3];
    __syncthreads();
    return base + inc - v;
}

__device__ __forceinline__ uint64_t block_sum(uint64_t v, unsigned long long *sh) {
    uint64_t t;
    block_excl_scan(v, sh, &t);
    return t;
}

__device__ __forceinline__ const RansDTab *tab_for(const void *tables, uint32_t stride, uint32_t b) {
    return reinterpret_cast<const RansDTab *>(tables) + (size_t)stride * b;
}

__device__ __forceinline__ bool single_mode(uint64_t n, uint32_t N) { return N <= 1 || n < N; }

struct KArgs {  // kernel-side copy of zr_rans_batch
    uint32_t B, N;
    uint64_t max_len;
    const uint64_t *len, *raw_off, *enc_off;
    uint64_t *enc_len;
    int32_t *status;
    const void *tables;
    uint32_t table_stride;
};

// ======================================================================
// histogram (the callers' [u32;256] counts: compression/mod.rs:433-436,
// blob_store/entropy.rs:213-216, rans.rs:708-714)
// ======================================================================
__device__ __forceinline__ void hist_range(const uint8_t *p, uint64_t lo, uint64_t hi, uint32_t *mine) {
    // head bytes up to 16-byte alignment
    const uint64_t mis = (16 - (((uintptr_t)(p + lo)) & 15)) & 15;
    const uint64_t body_lo = min(hi, lo + mis);
    if (threadIdx.x < body_lo - lo) atomicAdd(&mine[p[lo + threadIdx.x]], 1u);
    const uint64_t units = (hi - body_lo) / 16;
    const uint4 *q = reinterpret_cast<const uint4 *>(p + body_lo);
    for (uint64_t u = threadIdx.x; u < units; u += 256) {
        uint4 v = q[u];
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            atomicAdd(&mine[w[j] & 0xFF], 1u);
            atomicAdd(&mine[(w[j] >> 8) & 0xFF], 1u);
            atomicAdd(&mine[(w[j] >> 16) & 0xFF], 1u);
            atomicAdd(&mine[w[j] >> 24], 1u);
        }
    }
    const uint64_t tail_lo = body_lo + units * 16;
    if (threadIdx.x < hi - tail_lo) atomicAdd(&mine[p[tail_lo + threadIdx.x]], 1u);
}

// Work item = (buffer, 64 KiB chunk). Per-buffer histograms: one workgroup
// per item. Shared histogram: a grid-stride loop over the items with one LDS
// histogram per workgroup and one global add per bin at the end (a batch of
// a million 1 KiB records would otherwise send a global atomic per bin per
// record to the same 256 counters).
__global__ __launch_bounds__(256) void k_hist(const uint8_t *raw, KArgs a, int shared,
                                              uint32_t *hist, uint64_t chunk, uint32_t nchunk) {
    __shared__ uint32_t h[4][257];
    for (int i = threadIdx.x; i < 4 * 257; i += 256) (&h[0][0])[i] = 0;
    __syncthreads();
    uint32_t *mine = h[threadIdx.x >> 6];
    const uint64_t items = (uint64_t)a.B * nchunk;
    const uint64_t step = shared ? gridDim.x : items;
    for (uint64_t it = blockIdx.x; it < items; it += step) {
        const uint32_t b = (uint32_t)(it / nchunk), c = (uint32_t)(it % nchunk);
        const uint64_t n = a.len[b];
        const uint64_t lo = (uint64_t)c * chunk;
        if (lo >= n) continue;
        hist_range(raw + a.raw_off[b], lo, min(n, lo + chunk), mine);
        if (!shared) break;
    }
    __syncthreads();
    const uint32_t v = threadIdx.x;
    const uint32_t s = h[0][v] + h[1][v] + h[2][v] + h[3][v];
    if (s) {
        const uint32_t b = (uint32_t)(blockIdx.x / nchunk);
        atomicAdd(&hist[(shared ? 0 : (size_t)b * 256) + v], s);
    }
}

// ======================================================================
// table build on device: Rans64Encoder::new (rans.rs:208-235) with
// normalize_frequencies (rans.rs:238-299) and the symbol starts (rans.rs:225-228)
// ======================================================================
__global__ __launch_bounds__(256) void k_tab(const uint32_t *hist, RansDTab *tabs) {
    __shared__ unsigned long long sh[4];
    __shared__ uint32_t norm_s[256], start_s[256], freq_raw[256];
    __shared__ unsigned long long best;
    const uint32_t v = threadIdx.x;
    RansDTab *d = tabs + blockIdx.x;
    const uint32_t f = hist[(size_t)blockIdx.x * 256 + v];
    freq_raw[v] = f;
    // total_freq: u32 wrapping sum (rans.rs:209)
    const uint32_t total = (uint32_t)block_sum(f, sh);
    if (total == 0) {  // empty encoder (rans.rs:210-216)
        d->freq[v] = 0;
        d->start[v] = 0;
        d->rcp[v] = 0;
        d->rsh[v] = 0;
        for (int j = v; j < (int)TOTFREQ; j += 256) d->slot[j] = 0;
        if (v == 0) {
            d->kind = DT_EMPTY;
            d->status = ZR_OK;
        }
        return;
    }
    // pass 1: one slot per present symbol (rans.rs:244-250)
    const uint32_t used = (uint32_t)block_sum(f > 0, sh);
    const uint64_t ir = TOTFREQ - used;  // initial_remaining (rans.rs:263)
    // pass 2: proportional share of the initial budget (rans.rs:264-271). The
    // min(remaining) clamp never binds because sum(f*ir/total) <= ir.
    uint32_t add = f > 0 ? (uint32_t)(((uint64_t)f * ir) / (uint64_t)total) : 0;
    uint32_t norm = (f > 0 ? 1u : 0u) + add;
    uint32_t remaining = (uint32_t)(ir - block_sum(add, sh));
    norm_s[v] = norm;
    __syncthreads();
    // pass 3 (rans.rs:274-296): +1 to the largest raw freq (lowest index on ties)
    // whose normalised freq is < 1024; repeated +1 on the same argmax is batched.
    while (remaining > 0) {
        if (v == 0) best = 0;
        __syncthreads();
        const uint32_t fv = freq_raw[v];
        if (fv > 0 && norm_s[v] < TOTFREQ / 4)
            atomicMax(&best, ((unsigned long long)fv << 8) | (255 - v));
        __syncthreads();
        const unsigned long long bk = best;
        __syncthreads();
        if (bk == 0) {  // fallback: first non-zero symbol (rans.rs:284-292)
            if (v == 0) {
                for (int i = 0; i < 256; i++)
                    if (freq_raw[i] > 0) {
                        norm_s[i] += remaining;
                        break;
                    }
            }
            remaining = 0;
        } else {
            const uint32_t idx = 255 - (uint32_t)(bk & 0xFF);
            const uint32_t give = min(remaining, TOTFREQ / 4 - norm_s[idx]);
            if (v == 0) norm_s[idx] += give;
            remaining -= give;
        }
        __syncthreads();
    }
    norm = norm_s[v];
    uint64_t tot;
    const uint32_t start = (uint32_t)block_excl_scan(norm, sh, &tot);
    start_s[v] = start;
    d->freq[v] = norm;
    d->start[v] = start;
    uint32_t l = norm <= 1 ? 0u : 32u - __clz(norm - 1);
    d->rsh[v] = l;
    d->rcp[v] = norm ? (uint32_t)(((1ull << (24 + l)) + norm - 1) / norm) : 0u;
    const uint32_t maxn = (uint32_t)__syncthreads_or(norm == TOTFREQ);
    __syncthreads();
    for (uint32_t j = v; j < TOTFREQ; j += 256) {
        // owner of slot j: last symbol with start <= j (zero-freq symbols share the next start)
        int lo = 0, hi = 255;
        while (lo < hi) {
            int mid = (lo + hi + 1) >> 1;
            if (start_s[mid] <= j) lo = mid;
            else hi = mid - 1;
        }
        const uint32_t fs = norm_s[lo];
        d->slot[j] = (uint32_t)lo | ((j - start_s[lo]) << 8) | ((fs < TOTFREQ ? fs : 0u) << 20);
    }
    if (v == 0) {
        d->kind = maxn ? DT_SINGLE : DT_NORMAL;
        d->status = ZR_OK;
    }
}

typedef unsigned v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void asm_load16(v4u &dst, uintptr_t addr) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst) : "v"(addr) : "memory");
}

// s_waitcnt vmcnt(min(n, 12)) with a runtime, wave-uniform n
#define ZR_WAITC(k) \
    case k:         \
        asm volatile("s_waitcnt vmcnt(" #k ")" : "+v"(reg)::"memory"); \
        break;
__device__ __forceinline__ void wait_vmcnt_le(uint32_t n, v4u &reg) {
    switch (n > 12 ? 12 : n) {
        ZR_WAITC(0) ZR_WAITC(1) ZR_WAITC(2) ZR_WAITC(3) ZR_WAITC(4) ZR_WAITC(5) ZR_WAITC(6)
        ZR_WAITC(7) ZR_WAITC(8) ZR_WAITC(9) ZR_WAITC(10) ZR_WAITC(11) ZR_WAITC(12)
    }
}

// ======================================================================
// encode, xN layout: one lane per stream (rans.rs:369-420, encode_symbol :303-335)
// ======================================================================
__global__ __launch_bounds__(256) void k_enc_xn(const uint8_t *raw, KArgs a, RansWork w, int ablate) {
    const uint32_t nblk = w.nblk;
    const uint32_t b = blockIdx.x / nblk, blk = blockIdx.x % nblk;
    if (b >= a.B) return;
    const uint64_t n = a.len[b];
    const uint32_t N = a.N;
    if (single_mode(n, N)) return;
    // per symbol: x = xmax = freq << 12 (0 = not in table), y = xmax << 8 (two
    // renorm bytes at or above it), z = reciprocal,
    // w = start | (4096 - freq) << 12 | rsh << 24
    __shared__ uint4 et[256];
    __shared__ unsigned long long sh[4];
    const RansDTab *T = tab_for(a.tables, a.table_stride, b);
    {
        const uint32_t v = threadIdx.x, f = T->freq[v];
        et[v] = make_uint4(f << TF_SHIFT, f >= TOTFREQ ? 0xFFFFFFFFu : f << (TF_SHIFT + 8), T->rcp[v],
                           T->start[v] | (((TOTFREQ - f) & 0xFFF) << 12) | (T->rsh[v] << 24));
    }
    __syncthreads();
    // Input rows k*N + 256*blk .. +255 are staged through an LDS tile of ETILE rows:
    // each thread moves one 16-byte piece per tile (coalesced), loaded into
    // registers one tile ahead (the loads fly while the previous tile is coded).
    constexpr uint32_t ETILE = 16;
    __shared__ __attribute__((aligned(16))) uint8_t itile[ETILE * 256];
    const uint32_t s = blk * 256 + threadIdx.x;
    const bool active = s < N;
    const uint64_t c = active ? (n - s - 1) / N + 1 : 0;  // symbols s, s+N, ... < n
    const uint64_t cmax = (n - 1) / N + 1;
    const uint8_t *inb = raw + a.raw_off[b];
    const bool vec_in = ((((uintptr_t)inb) | N) & 15) == 0;
    const uint32_t lr = threadIdx.x >> 4, lp = (threadIdx.x & 15) * 16;  // my piece: row, column
    auto load_piece = [&](uint64_t t) -> uint4 {
        const uint64_t k = t * ETILE + lr;
        const uint64_t p = k * N + (uint64_t)blk * 256 + lp;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (k < cmax && blk * 256 + lp < N) {
            if (vec_in && p + 16 <= n) {
                v = *reinterpret_cast<const uint4 *>(inb + p);
            } else {
                uint32_t wv[4] = {0, 0, 0, 0};
                for (uint32_t j = 0; j < 16; j++)
                    if (p + j < n && blk * 256 + lp + j < N) wv[j >> 2] |= (uint32_t)inb[p + j] << (8 * (j & 3));
                v = make_uint4(wv[0], wv[1], wv[2], wv[3]);
            }
        }
        return v;
    };
    uint32_t *out = reinterpret_cast<uint32_t *>(w.scratch + (size_t)b * w.region + (size_t)s * w.cap);
    uint32_t x = RANS_L, nout = 0;  // nout = dwords stored
    uint64_t acc = 0;               // pending output bits (emission order from bit 0)
    uint32_t nacc = 0;              // valid bits in acc, < 32 after every flush
    bool err = false;
    // encode_symbol (rans.rs:303-335), branchless: at most two renorm bytes
    // (x < 2^24, xmax >= 2^12); q = x / f by the exact 24-bit reciprocal.
    // renorm bytes: x >= xmax << 8 -> 2, x >= xmax -> 1 (y >> 8 >= xmax <=> y >= xmax << 8)
    uint32_t xmin = 0xFFFFFFFFu;  // min xmax over coded symbols: 0 = a symbol not in the table
    auto enc_fast = [&](const uint4 e) {
        xmin = min(xmin, e.x);
        const uint32_t nb = x >= e.y ? 16u : (x >= e.x ? 8u : 0u);
        acc |= (uint64_t)__builtin_amdgcn_ubfe(x, 0, nb) << nacc;
        nacc += nb;
        const uint32_t y = x >> nb;
        const uint32_t q = __umulhi(y << 8, e.z) >> (e.w >> 24);          // y / f
        x = y + (e.w & 0xFFF) + __umul24(q, (e.w >> 12) & 0xFFF);         // (y/f)*4096 + y%f + start
    };
    auto enc_step = [&](const uint4 e, bool valid) {
        err |= valid && e.x == 0;  // "Symbol {} not in frequency table" (rans.rs:311-316)
        const uint32_t nb = valid ? (x >= e.y ? 16u : (x >= e.x ? 8u : 0u)) : 0u;
        acc |= (uint64_t)__builtin_amdgcn_ubfe(x, 0, nb) << nacc;
        nacc += nb;
        const uint32_t y = x >> nb;
        const uint32_t q = __umulhi(y << 8, e.z) >> (e.w >> 24);
        const uint32_t xn = y + (e.w & 0xFFF) + __umul24(q, (e.w >> 12) & 0xFFF);
        x = valid ? xn : x;
    };
    uint32_t sc = 0;  // store instructions this wave issued since the last piece load
    // full dwords queue in a 4-dword shift register; every 16 bytes move to an
    // LDS staging row ([chunk][lane], 1 KiB per wave store: conflict-free), and
    // every 64 bytes a lane stores its 4 staged chunks back to back, so each
    // 64-B segment of the scratch reaches the L2 in one burst (16-B stores
    // spread over time were written back as partial lines: 2.4x the bytes).
    __shared__ v4u stg[4 * 256];
    uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0, nq = 0, nstg = 0;
    v4u *out4 = reinterpret_cast<v4u *>(out);
    auto flush = [&]() {
        if (nacc >= 32) {
            q0 = q1;
            q1 = q2;
            q2 = q3;
            q3 = (uint32_t)acc;
            acc >>= 32;
            nacc -= 32;
            nq++;
        }
        const bool need = nq == 4;
        if (__builtin_amdgcn_ballot_w64(need) != 0) {  // wave-uniform
            if (need) {
                stg[(nstg & 3) * 256 + threadIdx.x] = v4u{q0, q1, q2, q3};
                nstg++;
                nq = 0;
            }
            const bool full = need && (nstg & 3) == 0;
            if (__builtin_amdgcn_ballot_w64(full) != 0) {
                sc += 4;
                if (full) {
                    const uint32_t o = nout >> 2;
                    if (ablate & 1) {  // diagnostic
                        asm volatile("" ::"v"(stg[threadIdx.x]));
                    } else {
                        out4[o + 0] = stg[0 * 256 + threadIdx.x];
                        out4[o + 1] = stg[1 * 256 + threadIdx.x];
                        out4[o + 2] = stg[2 * 256 + threadIdx.x];
                        out4[o + 3] = stg[3 * 256 + threadIdx.x];
                    }
                    nout += 16;
                }
            }
        }
    };
    // piece prefetch: inline-asm loads (no compiler vmcnt(0) that would also
    // wait for the scratch stores); the wait counts this wave's stores since.
    auto issue_piece = [&](uint64_t t, v4u &dst) {
        const uint64_t k = t * ETILE + lr;
        const uint64_t p = k * N + (uint64_t)blk * 256 + lp;
        if (vec_in && k < cmax && blk * 256 + lp + 16 <= N && p + 16 <= n) {
            asm_load16(dst, (uintptr_t)(inb + p));
        } else {
            const uint4 v = load_piece(t);
            dst = v4u{v.x, v.y, v.z, v.w};
        }
    };
    const uint64_t ntiles = (cmax + ETILE - 1) / ETILE;
    v4u pend;
    issue_piece(ntiles - 1, pend);
    for (uint64_t t = ntiles; t-- > 0;) {
        __syncthreads();
        wait_vmcnt_le(sc, pend);
        *reinterpret_cast<v4u *>(&itile[lr * 256 + lp]) = pend;
        __syncthreads();
        sc = 0;
        if (t > 0) issue_piece(t - 1, pend);
        const uint32_t rtop = (uint32_t)min((uint64_t)ETILE, cmax - t * ETILE);
        const bool wave_all = (uint64_t)blk * 256 + (threadIdx.x & ~63u) + 64 <= N;  // wave-uniform
        if (rtop == ETILE && t * ETILE + ETILE < cmax && wave_all) {
            // full tile, every lane of the wave a stream: no per-lane predicates
#pragma unroll
            for (int g = ETILE - 4; g >= 0; g -= 4) {
                const uint32_t s3 = itile[(g + 3) * 256 + threadIdx.x], s2 = itile[(g + 2) * 256 + threadIdx.x];
                const uint32_t s1 = itile[(g + 1) * 256 + threadIdx.x], s0 = itile[g * 256 + threadIdx.x];
                const uint4 e3 = et[s3], e2 = et[s2], e1 = et[s1], e0 = et[s0];
                enc_fast(e3);
                enc_fast(e2);
                flush();
                enc_fast(e1);
                enc_fast(e0);
                flush();
            }
        } else if (rtop == ETILE && t * ETILE + ETILE < cmax) {
            // full tile: every row is complete for every stream (rows < cmax - 1)
#pragma unroll
            for (int g = ETILE - 4; g >= 0; g -= 4) {
                const uint32_t s3 = itile[(g + 3) * 256 + threadIdx.x], s2 = itile[(g + 2) * 256 + threadIdx.x];
                const uint32_t s1 = itile[(g + 1) * 256 + threadIdx.x], s0 = itile[g * 256 + threadIdx.x];
                const uint4 e3 = et[s3], e2 = et[s2], e1 = et[s1], e0 = et[s0];
                enc_step(e3, active);
                enc_step(e2, active);
                flush();
                enc_step(e1, active);
                enc_step(e0, active);
                flush();
            }
        } else {
            for (uint32_t r = rtop; r-- > 0;) {
                const uint64_t k = t * ETILE + r;
                const uint32_t sym = itile[r * 256 + threadIdx.x];
                enc_step(et[sym], k < c);
                flush();
            }
        }
    }
    wait_vmcnt_le(0, pend);
    // drain: staged chunks, queued dwords (oldest in q[4-nq]), the partial dword
    for (uint32_t i = 0; i < (nstg & 3); i++) out4[(nout >> 2) + i] = stg[i * 256 + threadIdx.x];
    nout += 4 * (nstg & 3);
    {
        const uint32_t qs[4] = {q0, q1, q2, q3};
        for (uint32_t i = 0; i < nq; i++) out[nout + i] = qs[4 - nq + i];
        nout += nq;
    }
    if (nacc) out[nout] = (uint32_t)acc;
    const uint32_t nacc_bytes = nacc / 8;
    if (err || xmin == 0) atomicOr(&a.status[b], 1);  // marked; converted to ZR_INVALID_INPUT by the scan
    const uint32_t bytes = nout * 4 + nacc_bytes;
    if (active) {
        w.st_state[(size_t)b * N + s] = x;
        w.st_len[(size_t)b * N + s] = bytes;
    }
    const uint64_t bs = block_sum(active ? bytes : 0, sh);
    if (threadIdx.x == 0) w.blocksum[(size_t)b * nblk + blk] = bs;
}

// ======================================================================
// encode/decode, x1 layout: one lane per buffer (encode_single rans.rs:354-366)
// ======================================================================
__global__ __launch_bounds__(64) void k_enc_x1_generic(const uint8_t *raw, KArgs a, RansWork w) {
    const uint32_t b = blockIdx.x * 64 + threadIdx.x;
    if (b >= a.B) return;
    const uint64_t n = a.len[b];
    if (!single_mode(n, a.N)) return;
    const RansDTab *T = tab_for(a.tables, a.table_stride, b);
    const uint8_t *in = raw + a.raw_off[b];
    uint8_t *out = w.scratch + (size_t)b * w.region;
    uint32_t x = RANS_L;
    uint64_t no = 0;
    bool err = false;
    for (uint64_t i = n; i-- > 0;) {
        const uint32_t sym = in[i];
        const uint32_t f = T->freq[sym];
        if (f == 0) {
            err = true;
            break;
        }
        const uint32_t xmax = f << TF_SHIFT;
        while (x >= xmax) {
            out[no++] = (uint8_t)x;
            x >>= 8;
        }
        const uint32_t q = __umulhi(x << 8, T->rcp[sym]) >> T->rsh[sym];
        x = x + T->start[sym] + q * (TOTFREQ - f);
    }
    if (err) a.status[b] = ZR_INVALID_INPUT;
    w.st_state[(size_t)b * a.N] = x;
    w.blocksum[(size_t)b * w.nblk] = no;  // x1: renorm byte count
    a.enc_len[b] = no + 8;
}

// per-buffer exclusive scan of block sums; validates decode headers
__global__ __launch_bounds__(256) void k_scan(KArgs a, RansWork w, int decode) {
    const uint32_t b = blockIdx.x;
    if (b >= a.B) return;
    const uint64_t n = a.len[b];
    const uint32_t N = a.N;
    if (single_mode(n, N)) return;
    __shared__ unsigned long long sh[4];
    const uint32_t nblk = w.nblk;
    uint64_t carry = 0;
    for (uint32_t base = 0; base < nblk; base += 256) {
        const uint32_t i = base + threadIdx.x;
        const uint64_t v = i < nblk ? w.blocksum[(size_t)b * nblk + i] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan(v, sh, &tot);
        if (i < nblk) w.blockoff[(size_t)b * nblk + i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        const uint64_t hdr = (uint64_t)N * 12;
        if (!decode) {
            a.enc_len[b] = hdr + carry;
            if (a.status[b] != 0) a.status[b] = ZR_INVALID_INPUT;
        } else if (a.status[b] == 0 && hdr + carry > a.enc_len[b]) {
            a.status[b] = ZR_INVALID_INPUT;  // "Invalid stream data length" (rans.rs:608-610)
        }
    }
}

// header + stream compaction of the xN layout (rans.rs:402-419)
constexpr uint32_t CSPLIT = 4;  // workgroups per 256-stream block (more bytes in flight per CU)
__global__ __launch_bounds__(256) void k_enc_compact(uint8_t *enc, KArgs a, RansWork w) {
    const uint32_t nblk = w.nblk;
    const uint32_t part = blockIdx.x % CSPLIT;
    const uint32_t b = blockIdx.x / CSPLIT / nblk, blk = (blockIdx.x / CSPLIT) % nblk;
    if (b >= a.B) return;
    const uint64_t n = a.len[b];
    const uint32_t N = a.N;
    if (single_mode(n, N) || a.status[b] != 0) return;
    __shared__ unsigned long long sh[4];
    __shared__ uint64_t soff[256];
    __shared__ uint32_t slen[256];
    const uint32_t s = blk * 256 + threadIdx.x;
    const bool active = s < N;
    const uint32_t L = active ? w.st_len[(size_t)b * N + s] : 0;
    const uint64_t off = block_excl_scan(L, sh, nullptr) + w.blockoff[(size_t)b * nblk + blk];
    soff[threadIdx.x] = off;
    slen[threadIdx.x] = L;
    uint8_t *e = enc + a.enc_off[b];
    if (active && part == 0) {
        const uint32_t x = w.st_state[(size_t)b * N + s];
        st_u32_u(e + 8 * (size_t)s, x);
        st_u32_u(e + 8 * (size_t)s + 4, 0);
        st_u32_u(e + 8 * (size_t)N + 4 * (size_t)s, L);
    }
    __syncthreads();
    // The block's 256 streams are contiguous in the destination. Each thread
    // owns aligned 16-byte destination units (unit u = thread + 256 i) and
    // finds the stream holding it by a forward scan of the stream offsets in
    // LDS; interior units gather 16 source bytes with 5 dword loads +
    // v_alignbyte, units crossing a stream boundary go byte by byte.
    __shared__ uint64_t send_s[256];
    send_s[threadIdx.x] = off + L;  // (exclusive end offsets, relative to the buffer's stream area)
    __syncthreads();
    uint8_t *dbase = e + 12 * (size_t)N;
    const uint32_t nstream = min(256u, N - blk * 256);
    const uint64_t r0 = soff[0], r1 = send_s[nstream - 1];  // destination range [r0, r1)
    if (r1 > r0) {
        const uintptr_t ua0 = ((uintptr_t)dbase + r0) & ~(uintptr_t)15;
        const uint64_t nunits = ((uintptr_t)dbase + r1 - ua0 + 15) / 16;
        const uint64_t ulo = nunits * part / CSPLIT, uhi = nunits * (part + 1) / CSPLIT;
        uint32_t sj = 0;
        for (uint64_t u = ulo + threadIdx.x; u < uhi; u += 256) {
            const uintptr_t ua = ua0 + 16 * u;
            // destination offset of the unit; negative for a first unit that starts in the header
            const int64_t p0 = (int64_t)(ua - (uintptr_t)dbase);
            while (sj + 1 < nstream && (int64_t)send_s[sj] <= p0) sj++;
            const int64_t o = p0 - (int64_t)soff[sj];  // source offset in stream sj
            const uint8_t *src = w.scratch + (size_t)b * w.region + (size_t)(blk * 256 + sj) * w.cap;
            const uint8_t *sbase = w.scratch + (size_t)b * w.region + (size_t)(blk * 256) * w.cap;
            // 16 source bytes of stream j starting at source offset o (o may be
            // negative: bytes before the stream are read but masked off later)
            auto gather16 = [&](uint32_t j, int64_t o) -> uint4 {
                const uint8_t *src = sbase + (size_t)j * w.cap;
                const uint32_t *s4 = reinterpret_cast<const uint32_t *>(src + (o & ~(int64_t)3));
                const uint32_t r = (uint32_t)(o & 3) * 8;
                const uint32_t w0 = s4[0], w1 = s4[1], w2 = s4[2], w3 = s4[3], w4 = s4[4];
                uint4 v;
                v.x = (uint32_t)((((uint64_t)w1 << 32) | w0) >> r);
                v.y = (uint32_t)((((uint64_t)w2 << 32) | w1) >> r);
                v.z = (uint32_t)((((uint64_t)w3 << 32) | w2) >> r);
                v.w = (uint32_t)((((uint64_t)w4 << 32) | w3) >> r);
                return v;
            };
            const int64_t endj = (int64_t)send_s[sj] - p0;  // unit bytes [0, endj) lie in stream sj
            const bool inside = p0 >= (int64_t)r0 && p0 + 16 <= (int64_t)r1;
            if (o >= 0 && endj >= 16) {
                *reinterpret_cast<uint4 *>(ua) = gather16(sj, o);  // interior unit
            } else if (inside && o >= 0 && sj + 1 < nstream &&
                       ((int64_t)send_s[sj + 1] - p0 >= 16 || sj + 2 == nstream)) {
                // unit crossing one stream boundary at byte endj: merge two gathers
                const uint4 A = gather16(sj, o), Bv = gather16(sj + 1, -endj);
                auto msk = [&](int i) -> uint32_t {
                    const int64_t k = endj - 4 * i;  // bytes of dword i taken from A
                    return k >= 4 ? 0xFFFFFFFFu : (k <= 0 ? 0u : (1u << (8 * k)) - 1u);
                };
                uint4 v;
                v.x = (A.x & msk(0)) | (Bv.x & ~msk(0));
                v.y = (A.y & msk(1)) | (Bv.y & ~msk(1));
                v.z = (A.z & msk(2)) | (Bv.z & ~msk(2));
                v.w = (A.w & msk(3)) | (Bv.w & ~msk(3));
                *reinterpret_cast<uint4 *>(ua) = v;
            } else {
                // range edge or a unit spanning three or more streams: byte by byte
                uint32_t sk = sj;
                for (int t = 0; t < 16; t++) {
                    const int64_t p = p0 + t;
                    if (p < (int64_t)r0 || p >= (int64_t)r1) continue;
                    while (sk + 1 < nstream && (int64_t)send_s[sk] <= p) sk++;
                    reinterpret_cast<uint8_t *>(ua)[t] = sbase[(size_t)sk * w.cap + (p - (int64_t)soff[sk])];
                }
            }
        }
    }
}

__global__ __launch_bounds__(64) void k_enc_x1_compact(uint8_t *enc, KArgs a, RansWork w) {
    const uint32_t b = blockIdx.x;
    if (b >= a.B) return;
    const uint64_t n = a.len[b];
    if (!single_mode(n, a.N) || a.status[b] != 0) return;
    const uint64_t L = w.blocksum[(size_t)b * w.nblk];
    const uint8_t *src = w.scratch + (size_t)b * w.region;
    uint8_t *dst = enc + a.enc_off[b];
    for (uint64_t i = threadIdx.x; i < L; i += 64) dst[i] = src[i];
    if (threadIdx.x < 8) {
        const uint64_t x = w.st_state[(size_t)b * a.N];
        dst[L + threadIdx.x] = (uint8_t)(x >> (8 * threadIdx.x));
    }
}

// ======================================================================
// decode
// ======================================================================
// block sums of the xN stream lengths read from the encoded header (rans.rs:589-606)
__global__ __launch_bounds__(256) void k_dec_hdr(const uint8_t *enc, KArgs a, RansWork w) {
    const uint32_t nblk = w.nblk;
    const uint32_t b = blockIdx.x / nblk, blk = blockIdx.x % nblk;
    if (b >= a.B) return;
    const uint64_t n = a.len[b];
    const uint32_t N = a.N;
    if (n == 0 || single_mode(n, N)) return;
    __shared__ unsigned long long sh[4];
    const uint64_t hdr = (uint64_t)N * 12;
    const bool hdr_ok = a.enc_len[b] >= hdr;  // min_header_size (rans.rs:563-568)
    const uint32_t s = blk * 256 + threadIdx.x;
    uint64_t L = 0;
    if (hdr_ok && s < N) L = ld_u32_u(enc + a.enc_off[b] + 8 * (size_t)N + 4 * (size_t)s);
    const uint64_t bs = block_sum(L, sh);
    if (threadIdx.x == 0) {
        w.blocksum[(size_t)b * nblk + blk] = bs;
        w.redo[(size_t)b * nblk + blk] = 0;
        if (!hdr_ok && blk == 0) a.status[b] = ZR_INVALID_INPUT;
    }
}

constexpr int TILE = 16;  // decode steps staged per LDS tile

// Writes rows [k0, k0+rows) of the staged tile to raw (row k -> raw[k*N + 256*blk ...]).
__device__ __forceinline__ void flush_tile(const uint8_t *tile, uint8_t *outb, uint64_t n, uint32_t N,
                                           uint32_t blk, uint64_t k0, uint32_t rows, bool vec_ok) {
    const uint32_t col0 = blk * 256;
    const uint32_t width = min(256u, N - col0);
    if (vec_ok && width == 256) {
        // 16 threads per row, 16 bytes each
        const uint32_t r = threadIdx.x >> 4, cc = (threadIdx.x & 15) * 16;
        if (r < rows) {
            const uint64_t k = k0 + r;
            const uint64_t rowbase = k * N + col0;
            if (rowbase + 256 <= n) {
                *reinterpret_cast<uint4 *>(outb + rowbase + cc) =
                    *reinterpret_cast<const uint4 *>(tile + r * 256 + cc);
            } else {
                for (uint32_t j = 0; j < 16; j++)
                    if (rowbase + cc + j < n) outb[rowbase + cc + j] = tile[r * 256 + cc + j];
            }
        }
    } else {
        const uint32_t t = threadIdx.x;
        if (t < width) {
            for (uint32_t r = 0; r < rows; r++) {
                const uint64_t pos = (k0 + r) * N + col0 + t;
                if (pos < n) outb[pos] = tile[r * 256 + t];
            }
        }
    }
}

// Fast path: 32-bit state in [2^16, 2^24), packed LDS slot table, 64-bit MSB-first
// register window over the stream bytes refilled by aligned dword loads.
// GENERIC: u64 state, any table kind, byte-wise renormalisation exactly as
// decode_symbol (rans.rs:472-507). Workgroups the fast path cannot take are
// flagged in w.redo and re-run by the GENERIC instance.
template <bool GENERIC>
__global__ __launch_bounds__(256) void k_dec_xn(const uint8_t *enc, uint8_t *raw, KArgs a, RansWork w) {
    const uint32_t nblk = w.nblk;
    const uint32_t b = blockIdx.x / nblk, blk = blockIdx.x % nblk;
    if (b >= a.B) return;
    const uint64_t n = a.len[b];
    const uint32_t N = a.N;
    if (n == 0 || single_mode(n, N) || a.status[b] != 0) return;
    if (GENERIC && !w.redo[(size_t)b * nblk + blk]) return;
    __shared__ uint32_t stab[TOTFREQ];
    __shared__ uint8_t tile[TILE * 256];
    __shared__ unsigned long long sh[4];
    __shared__ uint32_t gfreq[GENERIC ? 256 : 1], gstart[GENERIC ? 256 : 1];
    const RansDTab *T = tab_for(a.tables, a.table_stride, b);
    for (uint32_t j = threadIdx.x; j < TOTFREQ; j += 256) stab[j] = T->slot[j];
    if (GENERIC) {
        gfreq[threadIdx.x] = T->freq[threadIdx.x];
        gstart[threadIdx.x] = T->start[threadIdx.x];
    }
    const uint32_t kind = T->kind;
    const uint32_t s = blk * 256 + threadIdx.x;
    const bool active = s < N;
    const uint8_t *e = enc + a.enc_off[b];
    const uint32_t L = active ? ld_u32_u(e + 8 * (size_t)N + 4 * (size_t)s) : 0;
    const uint64_t off = block_excl_scan(L, sh, nullptr) + w.blockoff[(size_t)b * nblk + blk];
    uint64_t X = active ? ld_u64_u(e + 8 * (size_t)s) : RANS_L;
    if (!GENERIC) {
        const bool fast = kind == DT_NORMAL && X >= RANS_L && X < (1ull << 24);
        if (__syncthreads_or(!fast)) {
            if (threadIdx.x == 0) w.redo[(size_t)b * nblk + blk] = 1;
            return;
        }
    }
    __syncthreads();
    const uint64_t c = active ? (n - s - 1) / N + 1 : 0;
    const uint64_t cmax = (n - 1) / N + 1;
    const uint8_t *sb = e + 12 * (size_t)N + off;  // stream start
    uint8_t *outb = raw + a.raw_off[b];
    const bool vec_ok = ((((uintptr_t)outb) | N) & 15) == 0;
    bool err = false;

    // ---- fast-path lane state
    uint32_t x = (uint32_t)X;
    uint64_t win = 0;
    uint32_t nbits = 0;
    uint64_t consumed = 0;  // bits
    const uintptr_t lo_lim = ((uintptr_t)a.enc_off[b] + (uintptr_t)enc) & ~(uintptr_t)3;
    uintptr_t rp = 0;
    // ---- generic lane state
    uint64_t pos = L;

    if (!GENERIC && active) {
        const uintptr_t pend = (uintptr_t)sb + L;
        const uintptr_t a0 = (pend - 1) & ~(uintptr_t)3;
        const uint32_t v = (uint32_t)(pend - a0);  // 1..4 valid bytes in the first dword
        const uint32_t w0 = *reinterpret_cast<const uint32_t *>(a0 > lo_lim ? a0 : lo_lim);
        win = (uint64_t)(w0 << (32 - 8 * v)) << 32;
        nbits = 8 * v;
        rp = a0 - 4;
    }

    for (uint64_t k0 = 0; k0 < cmax; k0 += TILE) {
        const uint32_t rows = (uint32_t)min((uint64_t)TILE, cmax - k0);
        for (uint32_t r = 0; r < rows; r++) {
            const uint64_t k = k0 + r;
            uint8_t sym = 0;
            if (k < c) {
                if (!GENERIC) {
                    // renormalise before decoding (rans.rs:479-485): x in [16, 2^24) needs
                    // 0, 1 or 2 bytes: sh = 8 * (#bytes) from the leading-zero count
                    const uint32_t sh8 = (__clz(x) & 24) - 8;
                    const uint32_t t = __builtin_amdgcn_ubfe((uint32_t)(win >> 32), 32 - sh8, sh8);
                    x = (x << sh8) | t;
                    win <<= sh8;
                    nbits -= sh8;
                    consumed += sh8;
                    if (nbits <= 32) {
                        const uintptr_t ra = rp > lo_lim ? rp : lo_lim;
                        const uint32_t ww = *reinterpret_cast<const uint32_t *>(ra);
                        win |= (uint64_t)ww << (32 - nbits);
                        nbits += 32;
                        rp -= 4;
                    }
                    const uint32_t ent = stab[x & (TOTFREQ - 1)];
                    x = __umul24(ent >> 20, x >> TF_SHIFT) + ((ent >> 8) & 0xFFF);
                    sym = (uint8_t)ent;
                } else if (!err) {
                    while (X < RANS_L) {
                        if (pos == 0) {  // "Insufficient data for decoding" (rans.rs:480-482)
                            err = true;
                            break;
                        }
                        pos--;
                        X = (X << 8) | sb[pos];
                    }
                    if (!err) {
                        const uint32_t slot = (uint32_t)(X & (TOTFREQ - 1));
                        const uint32_t sy = stab[slot] & 0xFF;
                        X = (uint64_t)gfreq[sy] * (X >> TF_SHIFT) + slot - gstart[sy];
                        sym = (uint8_t)sy;
                    }
                }
            }
            tile[r * 256 + threadIdx.x] = sym;
        }
        __syncthreads();
        flush_tile(tile, outb, n, N, blk, k0, rows, vec_ok);
        __syncthreads();
    }
    if (!GENERIC && active && consumed > 8ull * L) err = true;
    if (err) a.status[b] = ZR_INVALID_INPUT;
}

// ----------------------------------------------------------------------
// Fast xN decode. One lane = one stream, FW = 512 lanes per workgroup share
// one 16 KiB LDS slot table (2 workgroups per CU hold 1024 streams).
//   * stream bytes: per-lane ring of RSLOTS x 16 B in LDS, laid out
//     [dword][lane] (bank = lane: conflict-free whatever each lane reads).
//     Ring refills are wave-UNIFORM: every DTILE steps each lane writes the
//     chunks it loaded DTILE steps earlier (register staged, so the global
//     load latency overlaps a whole tile) and issues loads for up to two more.
//     A lane only ever reads its own ring column, so no barrier is needed.
//   * window: 64-bit MSB-first bit window. A step consumes at most 16 bits
//     (x >= 16 after a decode), so one 32-bit refill per PAIR of steps keeps
//     it >= 32 bits at every pair start; the next dword is prefetched from the
//     ring one pair ahead.
//   * output: step k of stream s is byte k*N + s, so at every step a wave
//     stores 64 consecutive bytes (one coalesced byte-store instruction, row
//     base in SGPRs, no VALU work).
// ----------------------------------------------------------------------
constexpr int FW = 512;
constexpr int RSLOTS = 8;
constexpr int DTILE = 16;


__global__ __launch_bounds__(FW) void k_dec_fast(const uint8_t *enc, uint8_t *raw, KArgs a, RansWork w,
                                                 uint32_t nblkF) {
    const uint32_t b = blockIdx.x / nblkF, blkF = blockIdx.x % nblkF;
    if (b >= a.B) return;
    const uint64_t n = a.len[b];
    const uint32_t N = a.N;
    if (n == 0 || single_mode(n, N) || a.status[b] != 0) return;
    constexpr uint32_t RD = RSLOTS * 4;  // ring dwords per lane
    __shared__ uint32_t stab[TOTFREQ];
    __shared__ __attribute__((aligned(16))) uint32_t ringw[RD * FW];  // [dword][lane]
    // scan scratch and flag alias the ring (used before it is filled): keeps the
    // workgroup at exactly 80 KiB of LDS so two fit on a CU
    unsigned long long *sh = reinterpret_cast<unsigned long long *>(ringw);
    uint32_t *flag = ringw + 64;
    const uint32_t tid = threadIdx.x;
    const RansDTab *T = tab_for(a.tables, a.table_stride, b);
    for (uint32_t j = tid; j < TOTFREQ; j += FW) stab[j] = T->slot[j];
    const uint32_t kind = T->kind;
    const uint32_t s = blkF * FW + tid;
    const bool active = s < N;
    const uint8_t *e = enc + a.enc_off[b];
    const uint32_t L = active ? ld_u32_u(e + 8 * (size_t)N + 4 * (size_t)s) : 0;
    // 512-lane exclusive scan of the stream lengths + base of the first 256-block
    unsigned long long inc = wave_incl_scan(L);
    const int wv = tid >> 6;
    if ((tid & 63) == 63) sh[wv] = inc;
    if (tid == 0) *flag = 0;
    __syncthreads();
    unsigned long long base = 0;
    for (int i = 0; i < wv; i++) base += sh[i];
    const uint64_t off = base + inc - L + w.blockoff[(size_t)b * w.nblk + 2 * blkF];
    const uint64_t X = active ? ld_u64_u(e + 8 * (size_t)s) : RANS_L;
    uint8_t *outb = raw + a.raw_off[b];
    const bool fast = kind == DT_NORMAL && X >= RANS_L && X < (1ull << 24);
    if (!fast) atomicOr(flag, 1u);
    __syncthreads();
    const uint32_t any_slow = *flag;
    __syncthreads();  // scan/flag reads complete before the ring is written
    if (any_slow) {
        if (tid == 0) {
            w.redo[(size_t)b * w.nblk + 2 * blkF] = 1;
            if (2 * blkF + 1 < w.nblk) w.redo[(size_t)b * w.nblk + 2 * blkF + 1] = 1;
        }
        return;
    }
    const uint64_t c = active ? (n - s - 1) / N + 1 : 0;
    const uint64_t cmax = (n - 1) / N + 1;
    const uintptr_t sb = (uintptr_t)e + 12 * (size_t)N + off;  // stream start
    const uintptr_t lo_lim = ((uintptr_t)e) & ~(uintptr_t)15;     // safe lower bound for loads
    uint32_t *ring = ringw + tid;
    // byte address -> this lane's ring dword (the dword holding that address)
    auto rdw = [&](uint32_t addr) -> uint32_t { return ring[((addr >> 2) & (RD - 1)) * FW]; };
    auto put16 = [&](uint32_t addr, const v4u v) {  // chunk at 16-aligned addr
        const uint32_t d = (addr >> 2) & (RD - 1);
        ring[(d + 0) * FW] = v.x;
        ring[(d + 1) * FW] = v.y;
        ring[(d + 2) * FW] = v.z;
        ring[(d + 3) * FW] = v.w;
    };
    auto clampa = [&](uintptr_t addr) -> uintptr_t { return addr > lo_lim ? addr : lo_lim; };
    // ---- ring prologue (synchronous): the 64-B segment holding the stream's
    // last byte, and the segment below it. Later refills move whole 64-B
    // segments (4 chunks issued back to back), so each L2 line is requested
    // in one burst instead of chunk by chunk across tiles.
    const uintptr_t pend = sb + L;
    const uintptr_t top = ((pend - 1) & ~(uintptr_t)15) + 16;  // end of the last chunk
    uintptr_t lo = (top - 1) & ~(uintptr_t)63;                   // lowest byte loaded or in flight
    {
        for (uintptr_t cpos = top - 16; cpos + 1 > lo; cpos -= 16)
            put16((uint32_t)cpos, *reinterpret_cast<const v4u *>(clampa(cpos)));
        const uintptr_t g = lo - 64;
        const v4u c0 = *reinterpret_cast<const v4u *>(clampa(g + 48));
        const v4u c1 = *reinterpret_cast<const v4u *>(clampa(g + 32));
        const v4u c2 = *reinterpret_cast<const v4u *>(clampa(g + 16));
        const v4u c3 = *reinterpret_cast<const v4u *>(clampa(g));
        put16((uint32_t)(g + 48), c0);
        put16((uint32_t)(g + 32), c1);
        put16((uint32_t)(g + 16), c2);
        put16((uint32_t)g, c3);
        lo = g;
    }
    // window: the dword holding the last stream byte, its garbage top bytes shifted out
    const uintptr_t a0 = (pend - 1) & ~(uintptr_t)3;
    const uint32_t v0 = (uint32_t)(pend - a0);
    uint32_t x = (uint32_t)X;
    uint64_t win = (uint64_t)(rdw((uint32_t)a0) << (32 - 8 * v0)) << 32;
    uint32_t nbits = 8 * v0;
    const uint32_t pend32 = (uint32_t)pend;
    uint32_t cons = (uint32_t)a0;  // (low 32 bits) bytes [cons, pend) have entered the window
    uint32_t nextw = rdw(cons - 4);
    // a staged segment in flight. Inline asm so hipcc inserts no conservative
    // vmcnt(0) (it would also wait for the tile's stores); the boundary below
    // waits with an exact count instead.
    v4u st0 = {0, 0, 0, 0}, st1 = st0, st2 = st0, st3 = st0;
    bool pending = false;
    uint32_t stlo = 0;
    const bool wave_live = (uint64_t)blkF * FW + (tid & ~63u) < N;  // wave-uniform

    // one 32-bit refill (branchless), then prefetch the next ring dword
    auto refill = [&]() {
        const bool need = nbits <= 32;
        win |= (uint64_t)(need ? nextw : 0u) << ((32 - nbits) & 63);
        nbits += need ? 32u : 0u;
        cons -= need ? 4u : 0u;
        nextw = rdw(cons - 4);
    };
    refill();  // >= 32 bits before the first pair
    uint32_t cons_snap = cons;
    uint32_t nbits_snap = nbits;
    // one decode step: renormalise (rans.rs:479-485) then decode (rans.rs:488-504);
    // returns the slot entry (its low byte is the symbol)
    auto step = [&]() -> uint32_t {
        // x in [16, 2^24) needs 0, 1 or 2 bytes; the shift is 8 * #bytes
        const uint32_t sh8 = (__builtin_clz(x) & 24) - 8;
        x = (uint32_t)(((((uint64_t)x) << 32) | (uint32_t)(win >> 32)) << sh8 >> 32);
        win <<= sh8;
        nbits -= sh8;
        const uint32_t ent = stab[x & (TOTFREQ - 1)];
        x = __umul24(ent >> 20, x >> TF_SHIFT) + ((ent >> 8) & 0xFFF);
        return ent;
    };
    // output: at step k the wave's lanes write bytes k*N + s .. +63 -- one
    // coalesced 64-byte byte-store per wave per step, row base in SGPRs
    const bool wave_all = (uint64_t)blkF * FW + (tid & ~63u) + 64 <= N;  // wave-uniform

    bool prev_full = true;
    for (uint64_t k0 = 0; k0 < cmax; k0 += DTILE) {
        // ---- ring maintenance (wave-uniform position, per-lane masks)
        if (k0 > 0) {
            // the previous boundary's segment loads are followed by exactly DTILE
            // byte stores of this wave when that tile was full and the wave is live
            if (prev_full && wave_live)
                asm volatile("s_waitcnt vmcnt(16)" : "+v"(st0), "+v"(st1), "+v"(st2), "+v"(st3)::"memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" : "+v"(st0), "+v"(st1), "+v"(st2), "+v"(st3)::"memory");
            if (pending) {
                put16(stlo + 48, st0);
                put16(stlo + 32, st1);
                put16(stlo + 16, st2);
                put16(stlo, st3);
            }
            // <= 4 chunks still unread: the next 64-B segment fits the 8-chunk ring
            const uint32_t occ = ((cons - 1 - (uint32_t)lo) >> 4) + 1;
            pending = occ <= 4;
            if (pending) {
                asm_load16(st0, clampa(lo - 16));
                asm_load16(st1, clampa(lo - 32));
                asm_load16(st2, clampa(lo - 48));
                asm_load16(st3, clampa(lo - 64));
                lo -= 64;
                stlo = (uint32_t)lo;
            }
        }
        const bool full = k0 + DTILE < cmax;  // every row of the tile is complete for every stream
        if (full && wave_all) {
#pragma unroll
            for (int j = 0; j < DTILE; j++) {
                const uint32_t ent = step();
                if (j & 1) refill();
                (outb + (k0 + j) * N)[s] = (uint8_t)ent;
            }
        } else if (full) {
#pragma unroll
            for (int j = 0; j < DTILE; j++) {
                const uint32_t ent = step();
                if (j & 1) refill();
                if (active) (outb + (k0 + j) * N)[s] = (uint8_t)ent;
            }
        } else {
            const uint32_t nsteps = (uint32_t)(cmax - k0);
            for (uint32_t j = 0; j < nsteps; j++) {
                const uint64_t k = k0 + j;
                if (k == c) {  // first step past this lane's symbols
                    cons_snap = cons;
                    nbits_snap = nbits;
                }
                const uint32_t ent = step();
                if (j & 1) refill();
                if (k < c) (outb + k * N)[s] = (uint8_t)ent;
            }
        }
        prev_full = full;
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(st0), "+v"(st1), "+v"(st2), "+v"(st3)::"memory");
    if (c == cmax) {  // no step past the end was executed for this lane
        cons_snap = cons;
        nbits_snap = nbits;
    }
    // bytes consumed by renormalisation = bytes moved into the window - bits still there
    if (active) {
        const uint64_t consumed = (uint64_t)(pend32 - cons_snap) - nbits_snap / 8;
        if (consumed > L) a.status[b] = ZR_INVALID_INPUT;  // "Insufficient data" (rans.rs:480-482)
    }
}

__global__ __launch_bounds__(64) void k_dec_x1_generic(const uint8_t *enc, uint8_t *raw, KArgs a) {
    const uint32_t b = blockIdx.x * 64 + threadIdx.x;
    if (b >= a.B) return;
    const uint64_t n = a.len[b];
    if (n == 0 || !single_mode(n, a.N)) return;
    const uint64_t len = a.enc_len[b];
    if (len < 8) {  // "rANS data too short" (rans.rs:524-526)
        a.status[b] = ZR_INVALID_INPUT;
        return;
    }
    const RansDTab *T = tab_for(a.tables, a.table_stride, b);
    const uint8_t *e = enc + a.enc_off[b];
    uint64_t X = ld_u64_u(e + len - 8);
    uint64_t pos = len - 8;
    uint8_t *out = raw + a.raw_off[b];
    for (uint64_t i = 0; i < n; i++) {
        while (X < RANS_L) {
            if (pos == 0) {
                a.status[b] = ZR_INVALID_INPUT;
                return;
            }
            pos--;
            X = (X << 8) | e[pos];
        }
        const uint32_t slot = (uint32_t)(X & (TOTFREQ - 1));
        const uint32_t sy = T->slot[slot] & 0xFF;
        X = (uint64_t)T->freq[sy] * (X >> TF_SHIFT) + slot - T->start[sy];
        out[i] = (uint8_t)sy;
    }
}

// ----------------------------------------------------------------------
// x1 layout, shared table (record batches: RansBlobStore / RansCompressor
// records). One lane per buffer, 256 buffers per
// workgroup sharing the LDS table. Input and output move in 16-byte chunks
// (the generic kernels above move single bytes with global table reads).
// The encoder writes straight into the final "bytes || state" layout: its
// destination offset is known before encoding, so x1 needs no compaction.
// ----------------------------------------------------------------------
typedef unsigned x4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_enc_x1_fast(const uint8_t *raw, uint8_t *enc, KArgs a, RansWork w) {
    __shared__ uint4 et[256];
    const RansDTab *T = reinterpret_cast<const RansDTab *>(a.tables);  // table 0 (stride 0)
    {
        const uint32_t v = threadIdx.x, f = T->freq[v];
        et[v] = make_uint4(f << TF_SHIFT, f >= TOTFREQ ? 0xFFFFFFFFu : f << (TF_SHIFT + 8), T->rcp[v],
                           T->start[v] | (((TOTFREQ - f) & 0xFFF) << 12) | (T->rsh[v] << 24));
    }
    __syncthreads();
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= a.B) return;
    const uint64_t n = a.len[b];
    if (!single_mode(n, a.N)) return;
    const uint8_t *in = raw + a.raw_off[b];
    uint8_t *out = enc + a.enc_off[b];
    const bool vec_out = (((uintptr_t)out) & 15) == 0;
    uint32_t x = RANS_L;
    uint32_t xmin = 0xFFFFFFFFu;
    uint64_t acc = 0;
    uint32_t nacc = 0, q0 = 0, q1 = 0, q2 = 0, q3 = 0, nq = 0;
    uint64_t nout = 0;  // bytes stored
    auto enc_step = [&](const uint4 e) {  // rans.rs:303-335 (see k_enc_xn)
        xmin = min(xmin, e.x);
        const uint32_t nb = x >= e.y ? 16u : (x >= e.x ? 8u : 0u);
        acc |= (uint64_t)__builtin_amdgcn_ubfe(x, 0, nb) << nacc;
        nacc += nb;
        const uint32_t y = x >> nb;
        const uint32_t q = __umulhi(y << 8, e.z) >> (e.w >> 24);
        x = y + (e.w & 0xFFF) + __umul24(q, (e.w >> 12) & 0xFFF);
    };
    auto push = [&]() {  // move whole dwords of acc to the queue, 16 bytes to memory
        if (nacc >= 32) {
            q0 = q1;
            q1 = q2;
            q2 = q3;
            q3 = (uint32_t)acc;
            acc >>= 32;
            nacc -= 32;
            if (++nq == 4) {
                if (vec_out) {
                    *reinterpret_cast<x4u *>(out + nout) = x4u{q0, q1, q2, q3};
                } else {
                    const uint32_t qs[4] = {q0, q1, q2, q3};
                    for (int i = 0; i < 16; i++) out[nout + i] = (uint8_t)(qs[i >> 2] >> (8 * (i & 3)));
                }
                nout += 16;
                nq = 0;
            }
        }
    };
    const uint64_t full = n & ~15ull;
    for (uint64_t i = n; i > full;) {  // ragged top, < 16 symbols
        enc_step(et[in[--i]]);
        push();
    }
    if (full) {
        int64_t c = (int64_t)(full >> 4) - 1;
        if ((((uintptr_t)in) & 15) == 0) {
            const x4u *in4 = reinterpret_cast<const x4u *>(in);
            const x4u z = {0, 0, 0, 0};
            x4u cur = in4[c];
            x4u n1 = c >= 1 ? in4[c - 1] : z;
            for (; c >= 0; c--) {
                const x4u wv = cur;
                cur = n1;
                if (c >= 2) n1 = in4[c - 2];
                uint4 e[16];
#pragma unroll
                for (int k = 15; k >= 0; k--) e[k] = et[(wv[k >> 2] >> (8 * (k & 3))) & 0xFF];
#pragma unroll
                for (int k = 15; k >= 0; k--) {
                    enc_step(e[k]);
                    if (k & 1) push();
                }
                push();
            }
        } else {
            for (uint64_t i = full; i-- > 0;) {
                enc_step(et[in[i]]);
                push();
            }
        }
    }
    // drain: queued dwords, the partial dword, then the u64 state
    {
        const uint32_t qs[4] = {q0, q1, q2, q3};
        for (uint32_t i = 0; i < nq; i++) {
            const uint32_t d = qs[4 - nq + i];
            for (int t = 0; t < 4; t++) out[nout + 4 * i + t] = (uint8_t)(d >> (8 * t));
        }
        nout += 4 * nq;
    }
    for (uint32_t t = 0; t < nacc / 8; t++) out[nout + t] = (uint8_t)(acc >> (8 * t));
    nout += nacc / 8;
    for (int t = 0; t < 8; t++) out[nout + t] = (uint8_t)((uint64_t)x >> (8 * t));
    if (xmin == 0 && n) a.status[b] = ZR_INVALID_INPUT;  // "Symbol {} not in frequency table"
    a.enc_len[b] = nout + 8;
}

// rans.rs:523-560 decode_single: state = last 8 bytes; renormalisation bytes
// are read backwards from len - 8 through a 16-byte register window
__global__ __launch_bounds__(256) void k_dec_x1_fast(const uint8_t *enc, uint8_t *raw, KArgs a) {
    __shared__ uint32_t stab[TOTFREQ];
    const RansDTab *T = reinterpret_cast<const RansDTab *>(a.tables);
    for (uint32_t j = threadIdx.x; j < TOTFREQ; j += 256) stab[j] = T->slot[j];
    const bool single = T->kind != DT_NORMAL;  // single-symbol / empty tables: global reads
    __syncthreads();
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= a.B) return;
    const uint64_t n = a.len[b];
    if (n == 0 || !single_mode(n, a.N)) return;
    const uint64_t len = a.enc_len[b];
    if (len < 8) {  // "rANS data too short" (rans.rs:524-526)
        a.status[b] = ZR_INVALID_INPUT;
        return;
    }
    const uint8_t *e = enc + a.enc_off[b];
    uint64_t X = ld_u64_u(e + len - 8);
    uint64_t pos = len - 8;  // bytes [0, pos) unread
    // backward byte reader: chunk cur holds the aligned 16 bytes containing pos - 1
    const x4u *e4 = reinterpret_cast<const x4u *>(e - (((uintptr_t)e) & 15));
    const uint64_t ebias = ((uintptr_t)e) & 15;  // e[i] = bytes of e4 at ebias + i
    int64_t cidx = ((int64_t)(pos + ebias) - 1) >> 4;
    x4u cur = {0, 0, 0, 0};
    if (pos) cur = e4[cidx];
    auto rd = [&]() -> uint32_t {  // pos > 0: return e[--pos]
        pos--;
        const uint64_t ab = pos + ebias;
        const int64_t ci = (int64_t)(ab >> 4);
        if (ci != cidx) {
            cidx = ci;
            cur = e4[ci];
        }
        const uint32_t k = (uint32_t)(ab & 15);
        const uint32_t dw = (k >> 2) == 0 ? cur.x : (k >> 2) == 1 ? cur.y : (k >> 2) == 2 ? cur.z : cur.w;
        return (dw >> (8 * (k & 3))) & 0xFF;
    };
    uint8_t *out = raw + a.raw_off[b];
    const bool vec_out = (((uintptr_t)out) & 15) == 0;
    uint32_t w0 = 0, w1 = 0, w2 = 0, acc = 0;
    bool err = false;
    uint64_t i = 0;
    for (; i < n; i++) {
        // renormalise first (rans.rs:479-485)
        while (X < RANS_L) {
            if (pos == 0) {
                err = true;
                break;
            }
            X = (X << 8) | rd();
        }
        if (err) break;
        uint32_t sy;
        if (single) {
            const uint32_t slot = (uint32_t)(X & (TOTFREQ - 1));
            sy = T->slot[slot] & 0xFF;
            X = (uint64_t)T->freq[sy] * (X >> TF_SHIFT) + slot - T->start[sy];
        } else {
            const uint32_t ent = stab[X & (TOTFREQ - 1)];
            sy = ent & 0xFF;
            X = (uint64_t)(ent >> 20) * (X >> TF_SHIFT) + ((ent >> 8) & 0xFFF);
        }
        if (vec_out) {
            acc = (acc >> 8) | (sy << 24);
            if ((i & 15) == 15) {
                *reinterpret_cast<x4u *>(out + i - 15) = x4u{w0, w1, w2, acc};
            } else if ((i & 3) == 3) {
                w0 = w1;
                w1 = w2;
                w2 = acc;
            }
        } else {
            out[i] = (uint8_t)sy;
        }
    }
    if (err) {
        a.status[b] = ZR_INVALID_INPUT;  // "Insufficient data" (rans.rs:480-482)
        return;
    }
    const uint32_t rem = (uint32_t)(n & 15);
    if (vec_out && rem) {
        const uint64_t g = n - rem;
        const uint32_t cq = rem >> 2, r = rem & 3;
        const uint32_t ws[3] = {w0, w1, w2};
        for (uint32_t k = 0; k < cq; k++)
            for (int t = 0; t < 4; t++) out[g + 4 * k + t] = (uint8_t)(ws[3 - cq + k] >> (8 * t));
        for (uint32_t t = 0; t < r; t++) out[g + 4 * cq + t] = (uint8_t)(acc >> (8 * (4 - r + t)));
    }
}

// ======================================================================
// host launchers
// ======================================================================
size_t rans_workspace_bytes(uint32_t B, uint32_t N, uint64_t max_len) {
    if (N == 0) N = 1;
    const uint64_t nblk = ceil_div(N, 256);
    const uint64_t cmax = ceil_div(max_len ? max_len : 1, N);
    const uint64_t cap = round_up(2 * cmax + 16, 16);
    const uint64_t region = std::max<uint64_t>(round_up((uint64_t)N * cap, 256),
                                               round_up(2 * max_len + 16, 256));
    size_t t = 0;
    t += round_up((uint64_t)B * N * 4, 256) * 2;
    t += round_up((uint64_t)B * nblk * 8, 256) * 2;
    t += round_up((uint64_t)B * nblk * 4, 256);
    t += (size_t)B * region;
    return t + 256;
}

int32_t rans_carve(uint32_t B, uint32_t N, uint64_t max_len, void *ws, size_t bytes, RansWork *w) {
    if (N == 0) N = 1;
    if (bytes < rans_workspace_bytes(B, N, max_len))
        return set_error(ZR_INVALID_INPUT, "rANS workspace too small");
    const uint64_t nblk = ceil_div(N, 256);
    const uint64_t cmax = ceil_div(max_len ? max_len : 1, N);
    w->cap = (uint32_t)round_up(2 * cmax + 16, 16);
    w->region = std::max<uint64_t>(round_up((uint64_t)N * w->cap, 256), round_up(2 * max_len + 16, 256));
    w->nblk = (uint32_t)nblk;
    uint8_t *p = reinterpret_cast<uint8_t *>(round_up((uintptr_t)ws, 256));
    auto take = [&](uint64_t n) {
        uint8_t *r = p;
        p += round_up(n, 256);
        return r;
    };
    w->st_state = reinterpret_cast<uint32_t *>(take((uint64_t)B * N * 4));
    w->st_len = reinterpret_cast<uint32_t *>(take((uint64_t)B * N * 4));
    w->blocksum = reinterpret_cast<uint64_t *>(take((uint64_t)B * nblk * 8));
    w->blockoff = reinterpret_cast<uint64_t *>(take((uint64_t)B * nblk * 8));
    w->redo = reinterpret_cast<uint32_t *>(take((uint64_t)B * nblk * 4));
    w->scratch = take((uint64_t)B * w->region);
    return ZR_OK;
}

static KArgs kargs(const zr_rans_batch *bt) {
    KArgs a;
    a.B = bt->n_buffers;
    a.N = bt->n_streams ? bt->n_streams : 1;
    a.max_len = bt->max_len;
    a.len = bt->len;
    a.raw_off = bt->raw_off;
    a.enc_off = bt->enc_off;
    a.enc_len = bt->enc_len;
    a.status = bt->status;
    a.tables = bt->tables;
    a.table_stride = bt->table_stride;
    return a;
}

}  // namespace zr

using namespace zr;

extern "C" {

size_t zr_rans_dtab_bytes(void) { return sizeof(RansDTab); }

size_t zr_rans_workspace_bytes(uint32_t n_buffers, uint32_t n_streams, uint64_t max_len) {
    return rans_workspace_bytes(n_buffers, n_streams, max_len);
}

int32_t zr_histogram_dev(const uint8_t *raw, const zr_rans_batch *bt, int32_t shared,
                         uint32_t *hist_dev, void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!bt || !hist_dev) return set_error(ZR_INVALID_INPUT, "null argument");
    if (bt->n_buffers == 0 || bt->max_len == 0) return ZR_OK;
    KArgs a = kargs(bt);
    const uint64_t chunk = 64 * 1024;
    const uint32_t nchunk = (uint32_t)ceil_div(bt->max_len, chunk);
    const uint64_t items = (uint64_t)nchunk * a.B;
    const uint64_t grid = shared ? std::min<uint64_t>(items, 8192) : items;
    timer_begin("histogram", (hipStream_t)stream);
    hipLaunchKernelGGL(k_hist, dim3((uint32_t)grid), dim3(256), 0, (hipStream_t)stream, raw, a,
                       shared, hist_dev, chunk, nchunk);
    timer_end("histogram", (hipStream_t)stream);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_rans_dtab_from_hist_dev(const uint32_t *hist_dev, uint32_t n_tables, void *dtabs_dev,
                                   void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (n_tables == 0) return ZR_OK;
    hipLaunchKernelGGL(k_tab, dim3(n_tables), dim3(256), 0, (hipStream_t)stream, hist_dev,
                       reinterpret_cast<RansDTab *>(dtabs_dev));
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_rans_encode_batch_dev(const zr_rans_batch *bt, const uint8_t *raw, uint8_t *enc,
                                 void *ws, size_t ws_bytes, void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!bt) return set_error(ZR_INVALID_INPUT, "null batch");
    if (bt->n_buffers == 0) return ZR_OK;
    KArgs a = kargs(bt);
    RansWork w;
    int32_t st = rans_carve(a.B, a.N, bt->max_len, ws, ws_bytes, &w);
    if (st) return st;
    hipStream_t s = (hipStream_t)stream;
    ZR_HIP(hipMemsetAsync(bt->status, 0, sizeof(int32_t) * a.B, s));
    const uint64_t gx = (uint64_t)w.nblk * a.B;
    if (bt->max_len >= a.N && a.N > 1) {
        timer_begin("rans_encode", s);
        static const int ablate = getenv("ZR_ABLATE") ? atoi(getenv("ZR_ABLATE")) : 0;  // diagnostics only
        hipLaunchKernelGGL(k_enc_xn, dim3((uint32_t)gx), dim3(256), 0, s, raw, a, w, ablate);
        timer_end("rans_encode", s);
        hipLaunchKernelGGL(k_scan, dim3(a.B), dim3(256), 0, s, a, w, 0);
        timer_begin("rans_compact", s);
        hipLaunchKernelGGL(k_enc_compact, dim3((uint32_t)gx * CSPLIT), dim3(256), 0, s, enc, a, w);
        timer_end("rans_compact", s);
    }
    timer_begin("rans_encode_x1", s);
    if (!(bt->min_len >= a.N && a.N > 1)) {  // some buffer may take the x1 layout
        if (a.table_stride == 0) {
            hipLaunchKernelGGL(k_enc_x1_fast, dim3((uint32_t)ceil_div(a.B, 256)), dim3(256), 0, s, raw, enc, a, w);
        } else {
            hipLaunchKernelGGL(k_enc_x1_generic, dim3((uint32_t)ceil_div(a.B, 64)), dim3(64), 0, s, raw, a, w);
            hipLaunchKernelGGL(k_enc_x1_compact, dim3(a.B), dim3(64), 0, s, enc, a, w);
        }
    }
    timer_end("rans_encode_x1", s);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_rans_decode_batch_dev(const zr_rans_batch *bt, const uint8_t *enc, uint8_t *raw, void *ws,
                                 size_t ws_bytes, void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!bt) return set_error(ZR_INVALID_INPUT, "null batch");
    if (bt->n_buffers == 0) return ZR_OK;
    KArgs a = kargs(bt);
    RansWork w;
    int32_t st = rans_carve(a.B, a.N, bt->max_len, ws, ws_bytes, &w);
    if (st) return st;
    hipStream_t s = (hipStream_t)stream;
    ZR_HIP(hipMemsetAsync(bt->status, 0, sizeof(int32_t) * a.B, s));
    const uint64_t gx = (uint64_t)w.nblk * a.B;
    if (bt->max_len >= a.N && a.N > 1) {
        hipLaunchKernelGGL(k_dec_hdr, dim3((uint32_t)gx), dim3(256), 0, s, enc, a, w);
        hipLaunchKernelGGL(k_scan, dim3(a.B), dim3(256), 0, s, a, w, 1);
        timer_begin("rans_decode", s);
        const uint32_t nblkF = (uint32_t)ceil_div(a.N, FW);
        hipLaunchKernelGGL(k_dec_fast, dim3(nblkF * a.B), dim3(FW), 0, s, enc, raw, a, w, nblkF);
        timer_end("rans_decode", s);
        hipLaunchKernelGGL(k_dec_xn<true>, dim3((uint32_t)gx), dim3(256), 0, s, enc, raw, a, w);
    }
    timer_begin("rans_decode_x1", s);
    if (!(bt->min_len >= a.N && a.N > 1)) {
        if (a.table_stride == 0)
            hipLaunchKernelGGL(k_dec_x1_fast, dim3((uint32_t)ceil_div(a.B, 256)), dim3(256), 0, s, enc, raw, a);
        else
            hipLaunchKernelGGL(k_dec_x1_generic, dim3((uint32_t)ceil_div(a.B, 64)), dim3(64), 0, s, enc, raw, a);
    }
    timer_end("rans_decode_x1", s);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

}  // extern "C"
