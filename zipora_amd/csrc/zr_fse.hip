// zr_fse.hip -- "FSE" (src/entropy/fse.rs) on MI355X / gfx950.
//
// The reference FSE is a ryg-style rANS64: 32-bit renormalisation words,
// initial state 1, tables normalised to 4096 (fse.rs:411-735). Formats
// (Appendix A):
//   0xF5 | body                          (single serial chain)
//   0xF6 | nblocks:u32 | size:u32 x nblocks | body x nblocks
//   body = len:u32 | 0xFF | raw                      (len < 100)
//        = len:u32 | 12 | nsym:u16 | (sym:u8, freq:u32) x nsym | words | state:u64
// A body is ONE serial coder chain, so the only parallel unit is the 0xF6
// block: one lane per block. The shared table lives in LDS.
//
// Encode: device histogram -> k_fse_tab (normalize_frequencies_exact,
// init_enc_symbol with the portable wrapping mul_hi) -> k_fse_enc (lane per
// block, words to 16-byte queued scratch stores) -> k_fse_scan (framing) ->
// k_fse_compact (coalesced body assembly).
// Decode: k_fse_frame -> k_fse_parse (one workgroup per block; dedupes tables
// whose header bytes equal block 0's) -> k_fse_tabs -> k_fse_dec (lane per
// block) .
#include <algorithm>
#include <cstring>
#include <vector>

#include "zr_internal.h"

namespace zr {

constexpr uint32_t FSE_MODE_SINGLE = 0xF5;    // fse.rs:15
constexpr uint32_t FSE_MODE_PARALLEL = 0xF6;  // fse.rs:17

struct alignas(16) FseDTab {
    uint32_t status, nsym, max_symbol, hdr_len;  // hdr_len = 3 + 5 * nsym
    uint32_t freq[256];                          // normalised (header content)
    uint32_t start[256];
    uint64_t rcp[256];                           // init_enc_symbol (fse.rs:583-615)
    uint32_t shift[256];
    uint32_t bias[256];
    uint32_t cmpl[256];
    // encode entry per symbol: {rcp lo, rcp hi, bias | cmpl << 16, freq | shift << 16}
    uint4 enc[256];
    // decode slot per state: sym | (freq & 4095) << 8 | (slot - start) << 20
    // (freq 4096, a table of one symbol, is stored as 0: the fast decoder takes
    // the frequency as is and leaves such tables to the generic lane loop)
    uint32_t slot[4096];
    uint8_t hdr[3 + 5 * 256];  // table_log(12) | nsym:u16 | (sym, freq:u32) pairs
};

// FseTable::mul_hi (fse.rs:618-628): the middle sum wraps in release builds.
__device__ __forceinline__ uint64_t mul_hi_portable(uint64_t a, uint64_t b) {
    const uint64_t a_lo = a & 0xFFFFFFFFull, a_hi = a >> 32;
    const uint64_t b_lo = b & 0xFFFFFFFFull, b_hi = b >> 32;
    const uint64_t x0 = b_lo * a_lo;
    const uint64_t x1 = (b_lo * a_hi) + (b_hi * a_lo) + (x0 >> 32);
    return (b_hi * a_hi) + (x1 >> 32);
}

__device__ __forceinline__ uint64_t blk_sum64(uint64_t v, unsigned long long *sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor((unsigned long long)v, d, 64);
    if (lane == 0) sh[w] = v;
    __syncthreads();
    const uint64_t t = sh[0] + sh[1] + sh[2] + sh[3];
    __syncthreads();
    return t;
}

__device__ __forceinline__ uint64_t blk_excl_scan64(uint64_t v, unsigned long long *sh, uint64_t *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned long long inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        unsigned long long t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    unsigned long long base = 0;
    for (int i = 0; i < w; i++) base += sh[i];
    if (total) *total = sh[0] + sh[1] + sh[2] + sh[3];
    __syncthreads();
    return base + inc - v;
}

// FseTable::new for the 256 frequencies f (one per thread of a 256-thread
// block): normalize_frequencies_exact (fse.rs:513-580), init_enc_symbol
// (fse.rs:583-615), alias table and the header pair list (fse.rs:909-928).
__device__ void fse_build_table(uint32_t f, FseDTab *d, unsigned long long *sh, uint32_t *norm_s,
                                uint32_t *raw_s, unsigned long long *best) {
    const uint32_t v = threadIdx.x;
    raw_s[v] = f;
    const uint64_t total = blk_sum64(f, sh);
    if (total == 0) {  // "No symbols found in frequency table" (fse.rs:415-422)
        if (v == 0) d->status = ZR_INVALID_INPUT;
        return;
    }
    const uint32_t scaled = f ? (uint32_t)(((uint64_t)f * 4096) / total) : 0u;
    uint32_t norm = f ? (scaled > 1 ? scaled : 1u) : 0u;
    norm_s[v] = norm;
    const uint64_t assigned = blk_sum64(norm, sh);
    if (assigned > 4096) {
        // repeatedly shrink the current largest (lowest index on ties) by
        // min(excess, max - 1) (fse.rs:542-560)
        uint64_t excess = assigned - 4096;
        while (excess > 0) {
            if (v == 0) *best = 0;
            __syncthreads();
            if (norm_s[v]) atomicMax(best, ((unsigned long long)norm_s[v] << 8) | (255 - v));
            __syncthreads();
            const unsigned long long bk = *best;
            __syncthreads();
            const uint32_t idx = 255 - (uint32_t)(bk & 0xFF), mv = (uint32_t)(bk >> 8);
            const uint64_t take = excess < (uint64_t)(mv - 1) ? excess : (uint64_t)(mv - 1);
            if (v == 0) norm_s[idx] -= (uint32_t)take;
            excess -= take;
            __syncthreads();
            if (take == 0) break;  // unreachable for <= 256 symbols (guard against a hang)
        }
    } else if (assigned < 4096) {
        // whole deficit to the largest raw frequency, lowest index on ties (fse.rs:561-573)
        if (v == 0) *best = 0;
        __syncthreads();
        if (f) atomicMax(best, ((unsigned long long)f << 8) | (255 - v));
        __syncthreads();
        if (v == 0) norm_s[255 - (uint32_t)(*best & 0xFF)] += (uint32_t)(4096 - assigned);
        __syncthreads();
    }
    norm = norm_s[v];
    // max_symbol: last symbol with a raw frequency (fse.rs:415)
    if (v == 0) *best = 0;
    __syncthreads();
    if (f) atomicMax(best, (unsigned long long)v + 1);
    __syncthreads();
    const uint32_t max_symbol = (uint32_t)*best - 1;
    __syncthreads();
    const uint32_t present = (norm > 0 && v <= max_symbol) ? 1u : 0u;
    const uint32_t nf = present ? norm : 0u;
    uint64_t tot;
    const uint32_t start = (uint32_t)blk_excl_scan64(nf, sh, &tot);
    const uint32_t rank = (uint32_t)blk_excl_scan64(present, sh, &tot);
    const uint32_t nsym = (uint32_t)tot;
    d->freq[v] = norm;
    d->start[v] = start;
    uint64_t rcp = 0;
    uint32_t shift = 0, bias = 0, cmpl = 0;
    if (present) {
        cmpl = 4096 - nf;
        if (nf < 2) {
            rcp = ~0ull;
            shift = 0;
            bias = start + 4096 - 1;
        } else {
            uint32_t sh2 = 0;
            while (nf > (1u << sh2)) sh2++;
            const uint64_t x0 = nf - 1, x1 = 1ull << (sh2 + 31);
            const uint64_t t1 = x1 / nf;
            const uint64_t x0e = x0 + ((x1 % nf) << 32);
            const uint64_t t0 = x0e / nf;
            rcp = t0 + (t1 << 32);
            shift = sh2 - 1;
            bias = start;
        }
        for (uint32_t i = 0; i < nf; i++) d->slot[start + i] = v | ((nf & 4095) << 8) | (i << 20);
        uint8_t *e = d->hdr + 3 + 5 * rank;
        e[0] = (uint8_t)v;
        e[1] = (uint8_t)norm;
        e[2] = (uint8_t)(norm >> 8);
        e[3] = (uint8_t)(norm >> 16);
        e[4] = (uint8_t)(norm >> 24);
    }
    d->rcp[v] = rcp;
    d->shift[v] = shift;
    d->bias[v] = bias;
    d->cmpl[v] = cmpl;
    // w: shift | the renorm threshold on the high word << 16, (nf << 4) - 1 (x >= nf
    // << 36 <=> x_hi > it), 0 for a symbol not in the table (encode_symbol -> None);
    // the 64-bit shift reads w's low 6 bits and the compare w's high half in place
    d->enc[v] = make_uint4((uint32_t)rcp, (uint32_t)(rcp >> 32), bias | (cmpl << 16),
                           shift | ((nf ? (nf << 4) - 1 : 0u) << 16));
    if (v == 0) {
        d->status = ZR_OK;
        d->nsym = nsym;
        d->max_symbol = max_symbol;
        d->hdr_len = 3 + 5 * nsym;
        d->hdr[0] = 12;  // table.table_log is always TF_SHIFT (fse.rs:491)
        d->hdr[1] = (uint8_t)nsym;
        d->hdr[2] = (uint8_t)(nsym >> 8);
    }
}

__global__ __launch_bounds__(256) void k_fse_tab(const uint32_t *hist, FseDTab *d) {
    __shared__ unsigned long long sh[4], best;
    __shared__ uint32_t norm_s[256], raw_s[256];
    fse_build_table(hist[threadIdx.x], d, sh, norm_s, raw_s, &best);
}

// F1 histogram (fse.rs:796-851): 32 bank-spread LDS copies per workgroup (bin b,
// copy c at b * 32 + c: lanes of a wave hit different banks even when they all
// count the same byte, which the skewed data FSE is run on does constantly),
// 16-byte loads, four in flight per thread, 256 KiB per workgroup.
constexpr uint32_t FH_COPY = 32;
constexpr uint64_t FH_CHUNK = 256 * 1024;
__device__ __forceinline__ void fh_add4(uint32_t *h, uint32_t w, uint32_t cp) {
    atomicAdd(&h[((w & 0xFF) << 5) + cp], 1u);
    atomicAdd(&h[(((w >> 8) & 0xFF) << 5) + cp], 1u);
    atomicAdd(&h[(((w >> 16) & 0xFF) << 5) + cp], 1u);
    atomicAdd(&h[((w >> 24) << 5) + cp], 1u);
}
__global__ __launch_bounds__(256) void k_fse_hist(const uint8_t *in, uint64_t n, uint32_t *hist) {
    typedef unsigned hv4u __attribute__((ext_vector_type(4)));
    __shared__ uint32_t h[256 * FH_COPY];
    const uint32_t tid = threadIdx.x, cp = tid & (FH_COPY - 1);
    for (uint32_t i = tid; i < 256 * FH_COPY; i += 256) h[i] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * FH_CHUNK, hi = min(n, lo + FH_CHUNK);
    const uint64_t mis = (16 - (((uintptr_t)(in + lo)) & 15)) & 15;
    const uint64_t blo = min(hi, lo + mis);
    if (lo + tid < blo) atomicAdd(&h[((uint32_t)in[lo + tid] << 5) + cp], 1u);
    const uint64_t units = (hi - blo) / 16;
    const hv4u *q = reinterpret_cast<const hv4u *>(in + blo);
    uint64_t u = tid;
    for (; u + 768 < units; u += 1024) {
        const hv4u v0 = __builtin_nontemporal_load(q + u);
        const hv4u v1 = __builtin_nontemporal_load(q + u + 256);
        const hv4u v2 = __builtin_nontemporal_load(q + u + 512);
        const hv4u v3 = __builtin_nontemporal_load(q + u + 768);
        fh_add4(h, v0.x, cp); fh_add4(h, v0.y, cp); fh_add4(h, v0.z, cp); fh_add4(h, v0.w, cp);
        fh_add4(h, v1.x, cp); fh_add4(h, v1.y, cp); fh_add4(h, v1.z, cp); fh_add4(h, v1.w, cp);
        fh_add4(h, v2.x, cp); fh_add4(h, v2.y, cp); fh_add4(h, v2.z, cp); fh_add4(h, v2.w, cp);
        fh_add4(h, v3.x, cp); fh_add4(h, v3.y, cp); fh_add4(h, v3.z, cp); fh_add4(h, v3.w, cp);
    }
    for (; u < units; u += 256) {
        const hv4u v = q[u];
        fh_add4(h, v.x, cp); fh_add4(h, v.y, cp); fh_add4(h, v.z, cp); fh_add4(h, v.w, cp);
    }
    const uint64_t tlo = blo + units * 16;
    if (tlo + tid < hi) atomicAdd(&h[((uint32_t)in[tlo + tid] << 5) + cp], 1u);
    __syncthreads();
    // bin tid: its 32 copies, read rotated so the threads of a wave use different banks
    uint32_t sum = 0;
    for (uint32_t i = 0; i < FH_COPY; i++) sum += h[(tid << 5) + ((i + tid) & (FH_COPY - 1))];
    if (sum) atomicAdd(&hist[tid], sum);
}

struct FseEncArgs {
    const uint8_t *in;
    uint64_t n, bs, nb;  // block size, block count (nb == 1: single body over all of in)
    const FseDTab *tab;
    uint8_t *scratch;    // per block: words (emission order) at scratch + j * cap
    uint64_t cap;
    uint32_t *wlen;      // bytes of words per block
    uint64_t *state;     // final state per block
    uint64_t *body;      // body bytes per block
    int32_t *status;
};

typedef unsigned fv4u __attribute__((ext_vector_type(4)));

// compress_single_internal (fse.rs:887-966): reverse scan, renormalize_encode
// (fse.rs:680-700) then encode_symbol (fse.rs:632-648), one lane per block.
// The input is read backwards in aligned 16-byte chunks with two chunks of
// prefetch; each chunk's 16 steps are unrolled so the LDS entry reads (which
// depend only on the symbols) are off the state's dependency chain.
__global__ __launch_bounds__(64) void k_fse_enc(FseEncArgs a) {
    __shared__ uint4 s_e[256];
    for (int i = threadIdx.x; i < 256; i += 64) s_e[i] = a.tab->enc[i];
    __syncthreads();
    const uint64_t j = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (j >= a.nb || a.tab->status != ZR_OK) return;
    const uint64_t lo = j * a.bs, len = min(a.bs, a.n - lo);
    if (len < 100) {  // raw marker body (fse.rs:892-904)
        a.wlen[j] = 0;
        a.state[j] = 0;
        a.body[j] = 5 + len;
        return;
    }
    const uint8_t *in = a.in + lo;
    uint32_t *out = reinterpret_cast<uint32_t *>(a.scratch + j * a.cap);
    fv4u *out4 = reinterpret_cast<fv4u *>(out);
    // renorm words go to a per-lane LDS ring ([slot][lane], conflict-free):
    // every step writes its candidate word to slot nw unconditionally and
    // advances nw only when it emits, so the step has no branch; complete
    // 16-byte chunks leave for the scratch once per 16-symbol group.
    __shared__ uint32_t wq[64 * 64];
    const uint32_t lane = threadIdx.x;
    uint32_t wa = 4 * lane;  // byte address of ring slot nw (mod 64 slots) = 4 * lane + 256 * nw
    uint64_t nout = 0;  // words stored to the scratch (multiple of 4 until the tail)
    uint64_t x = 1;  // fse.rs:931
    bool err = false;
    auto step_e = [&](const uint4 e) {
        const uint32_t thr = e.w >> 16;
        err |= (thr == 0);  // encode_symbol returns None (fse.rs:946-953)
        // renormalize_encode: x_max = ((RANS_L >> 12) << 32) * freq = freq << 36.
        // The word shift is branch-free (selects); only the 16-byte store of a
        // full queue branches, once per four words.
        // x < 2^48 between steps, so x >= f << 36 compares the high word only
        const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
        const bool emit = xh > thr;
        *reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(wq) + (wa & 0x3FFF)) = xl;
        const uint32_t lo = emit ? xh : xl, hi = emit ? 0u : xh;
        wa += emit ? 256u : 0u;
        // mul_hi_portable(x, rcp) as three 32x32->64 multiply-adds: the middle
        // sum u wraps mod 2^64 exactly like the reference's (fse.rs:618-628)
        const uint64_t t = (uint64_t)lo * e.y + __umulhi(lo, e.x);
        const uint64_t u = (uint64_t)hi * e.x + t;
        uint64_t uh;  // u >> 32 as an aligned register pair in one shift (not two moves)
        asm("v_lshrrev_b64 %0, 32, %1" : "=v"(uh) : "v"(u));
        const uint64_t m = (uint64_t)hi * e.y + uh;
        const uint64_t q = m >> (e.w & 63);  // shift < 64
        // x + bias + q * cmpl (wrapping); q <= x < 2^48, so q_hi * cmpl fits 24 bits
        const uint32_t cm = e.z >> 16;
        const uint64_t xb = (((uint64_t)hi << 32) | lo) + (e.z & 0xFFFF);
        const uint64_t r = (uint64_t)(uint32_t)q * cm + xb;
        x = ((uint64_t)(__umul24((uint32_t)(q >> 32), cm) + (uint32_t)(r >> 32)) << 32) | (uint32_t)r;
    };
    auto step = [&](uint32_t sym) { step_e(s_e[sym]); };
    auto flush = [&]() {  // complete chunks of the ring -> scratch (at most 5 per group)
        while ((wa >> 8) - (uint32_t)nout >= 4) {
            const uint32_t k = (uint32_t)nout & 63;
            out4[nout >> 2] = fv4u{wq[(k << 6) | lane], wq[(((k + 1) & 63) << 6) | lane],
                                   wq[(((k + 2) & 63) << 6) | lane], wq[(((k + 3) & 63) << 6) | lane]};
            nout += 4;
        }
    };
    const uint64_t full = len & ~15ull;
    for (uint64_t i = len; i > full;) step(in[--i]);  // ragged top, < 16 symbols
    flush();
    if (full && !err) {
        int64_t c = (int64_t)(full >> 4) - 1;
        if ((((uintptr_t)in) & 15) == 0) {
            const fv4u *in4 = reinterpret_cast<const fv4u *>(in);
            const fv4u z = {0, 0, 0, 0};
            fv4u cur = in4[c];
            fv4u n1 = c >= 1 ? in4[c - 1] : z;
            fv4u n2 = c >= 2 ? in4[c - 2] : z;
            for (; c >= 0; c--) {
                const fv4u w = cur;
                cur = n1;
                n1 = n2;
                if (c >= 3) n2 = in4[c - 3];
                uint4 e[16];  // table entries depend only on the symbols: read them all first
#pragma unroll
                for (int k = 15; k >= 0; k--) e[k] = s_e[(w[k >> 2] >> (8 * (k & 3))) & 0xFF];
#pragma unroll
                for (int k = 15; k >= 0; k--) step_e(e[k]);
                flush();
                if (err) break;
            }
        } else {
            for (uint64_t i = full; i-- > 0;) {
                step(in[i]);
                if ((i & 15) == 0) flush();
            }
        }
    }
    flush();
    for (; (uint32_t)nout != (wa >> 8); nout++) out[nout] = wq[(((uint32_t)nout & 63) << 6) | lane];
    if (err) *a.status = ZR_INVALID_INPUT;
    a.wlen[j] = (uint32_t)(nout * 4);
    a.state[j] = x;
    a.body[j] = 4 + a.tab->hdr_len + nout * 4 + 8;
}

// framing: body offsets, sizes table and total length (fse.rs:877-883, :1026-1044)
// mode: 0 = 0xF5 single, 1 = 0xF6 parallel, 2 = body only (parallel_blocks = Some(1) quirk)
__global__ __launch_bounds__(256) void k_fse_scan(const uint64_t *body, uint64_t nb, int mode, uint8_t *out,
                                                  uint64_t *boff, uint64_t *out_len, int32_t *status,
                                                  const FseDTab *tab) {
    __shared__ unsigned long long sh[4];
    const uint64_t pre = mode == 1 ? 5 + 4 * nb : (mode == 0 ? 1 : 0);
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nb; base += 256) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t v = i < nb ? body[i] : 0;
        uint64_t tot;
        const uint64_t ex = blk_excl_scan64(v, sh, &tot);
        if (i < nb) {
            boff[i] = pre + carry + ex;
            if (mode == 1) {
                uint8_t *p = out + 5 + 4 * i;
                p[0] = (uint8_t)v;
                p[1] = (uint8_t)(v >> 8);
                p[2] = (uint8_t)(v >> 16);
                p[3] = (uint8_t)(v >> 24);
            }
        }
        carry += tot;
    }
    if (threadIdx.x == 0) {
        if (mode == 0) out[0] = FSE_MODE_SINGLE;
        if (mode == 1) {
            out[0] = FSE_MODE_PARALLEL;
            out[1] = (uint8_t)nb;
            out[2] = (uint8_t)(nb >> 8);
            out[3] = (uint8_t)(nb >> 16);
            out[4] = (uint8_t)(nb >> 24);
        }
        if (tab->status != ZR_OK) *status = tab->status;
        *out_len = *status == ZR_OK ? pre + carry : 0;
    }
}

// body assembly: len | header | words | state, or len | FF | raw. One
// workgroup per block; the words are moved as aligned 16-byte destination units.
__global__ __launch_bounds__(256) void k_fse_compact(FseEncArgs a, uint8_t *out, const uint64_t *boff) {
    const uint64_t j = blockIdx.x;
    if (j >= a.nb || *a.status != ZR_OK) return;
    const uint64_t lo = j * a.bs, len = min(a.bs, a.n - lo);
    uint8_t *dst = out + boff[j];
    if (threadIdx.x < 4) dst[threadIdx.x] = (uint8_t)(len >> (8 * threadIdx.x));
    if (len < 100) {
        if (threadIdx.x == 0) dst[4] = 0xFF;
        for (uint64_t i = threadIdx.x; i < len; i += 256) dst[5 + i] = a.in[lo + i];
        return;
    }
    const uint32_t hl = a.tab->hdr_len;
    for (uint32_t i = threadIdx.x; i < hl; i += 256) dst[4 + i] = a.tab->hdr[i];
    const uint64_t W = a.wlen[j];
    uint8_t *wd = dst + 4 + hl;
    const uint8_t *src = a.scratch + j * a.cap;
    const uintptr_t ua0 = ((uintptr_t)wd) & ~(uintptr_t)15;
    const uint64_t nunits = ((uintptr_t)wd + W - ua0 + 15) / 16;
    for (uint64_t u = threadIdx.x; u < nunits; u += 256) {
        const uintptr_t ua = ua0 + 16 * u;
        const int64_t o = (int64_t)(ua - (uintptr_t)wd);
        if (o >= 0 && (uint64_t)o + 16 <= W) {
            const uint32_t *s4 = reinterpret_cast<const uint32_t *>(src + (o & ~(int64_t)3));
            const uint32_t r = (uint32_t)(o & 3) * 8;
            const uint32_t w0 = s4[0], w1 = s4[1], w2 = s4[2], w3 = s4[3], w4 = s4[4];
            uint4 v;
            v.x = (uint32_t)((((uint64_t)w1 << 32) | w0) >> r);
            v.y = (uint32_t)((((uint64_t)w2 << 32) | w1) >> r);
            v.z = (uint32_t)((((uint64_t)w3 << 32) | w2) >> r);
            v.w = (uint32_t)((((uint64_t)w4 << 32) | w3) >> r);
            *reinterpret_cast<uint4 *>(wd + o) = v;  // (rebased on wd: a global, not flat, store)
        } else {
            for (int t = 0; t < 16; t++) {
                const int64_t p = o + t;
                if (p >= 0 && (uint64_t)p < W) wd[p] = src[p];
            }
        }
    }
    if (threadIdx.x < 8) wd[W + threadIdx.x] = (uint8_t)(a.state[j] >> (8 * threadIdx.x));
}

// ---------------------------------------------------------------- decode
struct FseBlk {         // parsed block
    uint64_t body;      // offset of the body in the stream
    uint64_t blen;      // body length
    uint64_t orig;      // decoded length
    uint64_t words;     // offset of the word area in the stream
    uint64_t wbytes;    // word area length
    uint64_t state;
    uint32_t raw, table;  // raw body; table index (0 = shared with block 0)
};

struct FseDecArgs {
    const uint8_t *in;
    uint64_t n, max_blocks, out_cap;
    uint8_t *out;
    uint64_t *nblocks;  // device scalar
    FseBlk *blk;
    uint32_t *freqs;    // [max_blocks][256] raw header frequencies (table builds)
    FseDTab *tabs;      // [max_blocks] (only built where blk.table == index)
    uint64_t *ooff;     // output offset per block
    uint64_t *out_len;
    int32_t *status;
};

__device__ __forceinline__ uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint64_t rd64(const uint8_t *p) { return rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

// mode byte, block count and body offsets (FseDecoder::decompress fse.rs:1105-1148,
// decompress_parallel fse.rs:1284-1312)
__global__ __launch_bounds__(256) void k_fse_frame(FseDecArgs a) {
    __shared__ unsigned long long sh[4];
    __shared__ int s_mode;
    __shared__ uint64_t s_nb;
    const uint8_t *in = a.in;
    const uint64_t n = a.n;
    if (threadIdx.x == 0) {
        int mode = -1;
        uint64_t nb = 0;
        if (n == 0) {
            mode = 0;  // empty -> empty output
        } else if (in[0] == FSE_MODE_SINGLE) {
            mode = 1;
            nb = 1;
        } else if (in[0] == FSE_MODE_PARALLEL) {
            if (n - 1 < 4) {
                mode = -1;  // "truncated before block count"
            } else {
                nb = rd32(in + 1);
                if (nb == 0 || nb > (n - 1 - 4) / 4) mode = -1;  // zero blocks / claims too many
                else if (nb > a.max_blocks) mode = -2;
                else mode = 2;
            }
        }  // else: unknown mode byte
        s_mode = mode;
        s_nb = nb;
        *a.status = mode == -1 ? ZR_INVALID_INPUT : (mode == -2 ? ZR_UNSUPPORTED : ZR_OK);
        *a.nblocks = mode > 0 ? nb : 0;
        if (mode == 1) {
            a.blk[0].body = 1;
            a.blk[0].blen = n - 1;
        }
    }
    __syncthreads();
    if (s_mode != 2) return;
    const uint64_t nb = s_nb;
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nb; base += 256) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t v = i < nb ? rd32(in + 5 + 4 * i) : 0;
        uint64_t tot;
        const uint64_t ex = blk_excl_scan64(v, sh, &tot);
        if (i < nb) {
            a.blk[i].body = 5 + 4 * nb + carry + ex;
            a.blk[i].blen = v;
        }
        carry += tot;
    }
    if (threadIdx.x == 0 && 5 + 4 * nb + carry > n) *a.status = ZR_INVALID_INPUT;  // "Invalid block data"
}

// decompress_single header parsing (fse.rs:1151-1249), one workgroup per block
__global__ __launch_bounds__(256) void k_fse_parse(FseDecArgs a) {
    const uint64_t j = blockIdx.x;
    __shared__ int s_go;
    // other workgroups of this grid may flip *status: read it once per workgroup
    if (threadIdx.x == 0) s_go = j < *a.nblocks && *a.status == ZR_OK;
    __syncthreads();
    if (!s_go) return;
    __shared__ int s_err, s_diff;
    __shared__ uint32_t s_nsym, s_last[256];
    const uint8_t *d = a.in + a.blk[j].body;
    const uint64_t len = a.blk[j].blen;
    FseBlk &B = a.blk[j];
    if (threadIdx.x == 0) {
        int err = 0;
        B.raw = 0;
        B.orig = 0;
        B.wbytes = 0;
        B.table = 0;
        s_nsym = 0;
        if (len == 0) {
            B.raw = 2;  // empty body -> empty output
        } else if (len < 5) {
            err = 1;  // "Data too short for FSE header"
        } else {
            const uint64_t orig = rd32(d);
            if (orig == 0) {
                B.raw = 2;
            } else if (d[4] == 0xFF) {
                if (5 + orig > len) err = 1;  // "Incomplete uncompressed data"
                B.raw = 1;
                B.orig = orig;
            } else if (d[4] < 5 || d[4] > 15) {
                err = 1;  // "Invalid table log"
            } else if (7 > len) {
                err = 1;  // "Missing frequency table size"
            } else {
                const uint32_t nsym = (uint32_t)d[5] | ((uint32_t)d[6] << 8);
                if (nsym == 0) err = 1;  // all-zero table: "No symbols found"
                else if (7 + 5 * (uint64_t)nsym > len) err = 1;  // "Incomplete frequency table"
                else if (7 + 5 * (uint64_t)nsym + 8 > len) err = 1;  // "Missing final state"
                else {
                    s_nsym = nsym;
                    B.orig = orig;
                    const uint64_t ss = len - 8;
                    uint64_t st = rd64(d + ss);
                    if (st == 0) st = 1;  // fse.rs:1247-1249
                    B.state = st;
                    B.words = a.blk[j].body + 7 + 5 * (uint64_t)nsym;
                    B.wbytes = ss - (7 + 5 * (uint64_t)nsym);
                }
            }
        }
        s_err = err;
        s_diff = 0;
        if (err) *a.status = ZR_INVALID_INPUT;
    }
    __syncthreads();
    if (s_err || s_nsym == 0) return;  // raw / empty / error: no table
    const uint32_t nsym = s_nsym;
    // same pair bytes as block 0 -> share table 0
    if (j != 0) {
        // block 0's header is re-read from the stream (its FseBlk is being
        // written by another workgroup of this grid). Sharing needs a coded
        // block 0 whose pair list is complete; any block-0 error fails the
        // whole stream anyway.
        const uint8_t *d0 = a.in + a.blk[0].body;
        const uint64_t len0 = a.blk[0].blen;
        const bool comparable = len0 >= 7 && rd32(d0) != 0 && d0[4] != 0xFF && d0[5] == d[5] &&
                                d0[6] == d[6] && 7 + 5 * (uint64_t)nsym <= len0;
        if (!comparable) {
            if (threadIdx.x == 0) s_diff = 1;
        } else {
            for (uint32_t i = threadIdx.x; i < 5 * nsym; i += 256)
                if (d0[7 + i] != d[7 + i]) s_diff = 1;
        }
        __syncthreads();
        if (!s_diff) return;
    }
    if (threadIdx.x == 0) B.table = (uint32_t)j;
    // raw frequencies: later entries for the same symbol win (fse.rs:1200-1215)
    s_last[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nsym; i += 256) atomicMax(&s_last[d[7 + 5 * i]], i + 1);
    __syncthreads();
    const uint32_t li = s_last[threadIdx.x];
    a.freqs[j * 256 + threadIdx.x] = li ? rd32(d + 7 + 5 * (li - 1) + 1) : 0u;
}

__global__ __launch_bounds__(256) void k_fse_tabs(FseDecArgs a) {
    const uint64_t j = blockIdx.x;
    __shared__ int s_go;
    if (threadIdx.x == 0) {
        s_go = j < *a.nblocks && *a.status == ZR_OK;
        if (s_go) {
            const FseBlk &B = a.blk[j];
            s_go = !(B.raw || B.table != j || B.orig == 0);
        }
    }
    __syncthreads();
    if (!s_go) return;
    __shared__ unsigned long long sh[4], best;
    __shared__ uint32_t norm_s[256], raw_s[256];
    fse_build_table(a.freqs[j * 256 + threadIdx.x], &a.tabs[j], sh, norm_s, raw_s, &best);
    __syncthreads();
    if (threadIdx.x == 0 && a.tabs[j].status != ZR_OK) *a.status = ZR_INVALID_INPUT;
}

__global__ __launch_bounds__(256) void k_fse_outscan(FseDecArgs a) {
    __shared__ unsigned long long sh[4];
    if (*a.status != ZR_OK) {
        if (threadIdx.x == 0) *a.out_len = 0;
        return;
    }
    const uint64_t nb = *a.nblocks;
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nb; base += 256) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t v = i < nb ? a.blk[i].orig : 0;
        uint64_t tot;
        const uint64_t ex = blk_excl_scan64(v, sh, &tot);
        if (i < nb) a.ooff[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        *a.out_len = carry;
        if (carry > a.out_cap) *a.status = ZR_INVALID_INPUT;  // output buffer too small
    }
}

// decode loop of decompress_single (fse.rs:1258-1278): decode_symbol
// (fse.rs:664-676) then renormalize_decode (fse.rs:704-735), one lane per
// block. One LDS slot read per symbol; the word area is read backwards as
// aligned 16-byte chunks (three chunks prefetched) and the 32-bit words are
// funnel-shifted out of them (their misalignment is fixed for the block).
template <bool SHARED>
__device__ __forceinline__ void fse_dec_lane(const uint32_t *slot, const uint8_t *in, const uint8_t *wd, uint64_t bp,
                                             uint64_t x, uint8_t *out, uint64_t orig) {
    const fv4u z = {0, 0, 0, 0};
    const uintptr_t wbase = (uintptr_t)wd;
    const uintptr_t cmin = wbase >> 4;  // lowest chunk of the word area
    // chunks are addressed from the (16-aligned-down) stream pointer so the
    // loads stay in the global address space (no flat loads)
    const fv4u *in4 = reinterpret_cast<const fv4u *>(in - (((uintptr_t)in) & 15));
    const uintptr_t c0 = ((uintptr_t)in4) >> 4;
    auto ld = [&](uintptr_t c) -> fv4u { return c >= cmin ? in4[c - c0] : z; };
    uint32_t r8 = 0;
    uintptr_t m = 0;  // absolute dword index of the next word's low dword
    fv4u hi = z, cur = z, n1 = z, n2 = z, n3 = z;
    if (bp >= 4) {
        const uintptr_t a0 = wbase + bp - 4;
        r8 = (uint32_t)(a0 & 3) * 8;
        m = a0 >> 2;
        const uintptr_t c = m >> 2;
        // the chunk above is only needed when the first word's low dword is
        // the last of its chunk; it then starts at or below the state bytes
        if ((m & 3) == 3) hi = in4[c + 1 - c0];
        cur = ld(c);
        n1 = ld(c - 1);
        n2 = ld(c - 2);
        n3 = ld(c - 3);
    }
    auto step = [&]() -> uint32_t {
        const uint32_t e = slot[x & 4095];
        const uint32_t fq = (e >> 8) & 4095;
        x = (uint64_t)(fq ? fq : 4096u) * (x >> 12) + (e >> 20);
        if (x < 65536 && bp > 0) {
            if (bp >= 4) {
                bp -= 4;
                const uint32_t k = (uint32_t)(m & 3);
                const uint32_t lo32 = k == 0 ? cur.x : k == 1 ? cur.y : k == 2 ? cur.z : cur.w;
                const uint32_t hi32 = k == 0 ? cur.y : k == 1 ? cur.z : k == 2 ? cur.w : hi.x;
                x = (x << 32) | (uint32_t)((((uint64_t)hi32 << 32) | lo32) >> r8);
                m -= 1;
                if (k == 0) {
                    hi = cur;
                    cur = n1;
                    n1 = n2;
                    n2 = n3;
                    n3 = ld((m >> 2) - 3);
                }
            } else {
                bp -= 1;
                x = (x << 8) | wd[bp];
            }
        }
        if (x < 1) x = 1;
        return e & 0xFF;
    };
    uint64_t i = 0;
    if ((((uintptr_t)out) & 15) == 0) {
        const uint64_t groups = orig >> 4;
        fv4u *o4 = reinterpret_cast<fv4u *>(out);
        for (uint64_t g = 0; g < groups; g++) {
            uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < 16; k++) o[k >> 2] |= step() << (8 * (k & 3));
            o4[g] = fv4u{o[0], o[1], o[2], o[3]};
        }
        i = groups << 4;
    }
    for (; i < orig; i++) out[i] = (uint8_t)step();
}

__device__ __forceinline__ void fse_asm_load16(fv4u &dst, const fv4u *p) {
    // issued behind the compiler's back: the group pipeline below waits for it
    // with a counted vmcnt instead of the vmcnt(0) the compiler would emit
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst) : "v"(p) : "memory");
}

#ifndef ZR_FSE_PK
#define ZR_FSE_PK 1
#endif
// Fast path for blocks coded with block 0's table (every block of a stream
// this library or the reference wrote from one histogram). Per lane: a
// 64-dword LDS ring of the word area indexed by absolute dword index mod 64
// ([dword][lane] layout: conflict-free), refilled once per 16-symbol group by
// two wave-uniform 16-byte loads that land two groups later behind
// `s_waitcnt vmcnt(2)`. The next renormalisation word is read from the ring
// one renormalisation ahead, so a step's dependency chain is one LDS slot read
// plus integer arithmetic.
__global__ __launch_bounds__(64) void k_fse_dec(FseDecArgs a) {
    __shared__ uint32_t s_slot[4096];
    __shared__ uint32_t s_ring[65 * 64];  // [slot][lane], slot 64 mirrors slot 0
    const uint32_t lane = threadIdx.x;
    const uint64_t j = (uint64_t)blockIdx.x * 64 + lane;
    const uint64_t nb = *a.nblocks;
    if (*a.status != ZR_OK) return;  // uniform: status is not written by this kernel
    const FseDTab *T0 = &a.tabs[0];
    const bool t0 = nb > 0 && a.blk[0].raw == 0 && a.blk[0].orig > 0;
    if (t0) {
        const uint4 *src = reinterpret_cast<const uint4 *>(T0->slot);
        for (int i = lane; i < 1024; i += 64) reinterpret_cast<uint4 *>(s_slot)[i] = src[i];
    }
    __syncthreads();
    FseBlk B = {};
    if (j < nb) B = a.blk[j];
    const bool coded = j < nb && B.raw == 0 && B.orig > 0;
    const bool fast = coded && B.table == 0 && T0->nsym > 1;  // (one symbol: freq 4096, generic loop)
    uint8_t *out = a.out + (j < nb ? a.ooff[j] : 0);

    const fv4u *in4 = reinterpret_cast<const fv4u *>(a.in - (((uintptr_t)a.in) & 15));
    const uintptr_t c0 = ((uintptr_t)in4) >> 4;
    const uintptr_t wbase = (uintptr_t)(a.in + B.words);
    const uintptr_t cmin = wbase >> 4;
    uint64_t x = fast ? B.state : 1, bp = fast ? B.wbytes : 0;
    uint32_t *ring = s_ring + lane;
    auto rd = [&](uintptr_t d) -> uint32_t { return ring[(d & 63) * 64]; };
    auto land = [&](const fv4u v, uintptr_t c) {
        if (((4 * c) & 63) == 0) ring[64 * 64] = v.x;  // the mirror of slot 0
        ring[((4 * c + 0) & 63) * 64] = v.x;
        ring[((4 * c + 1) & 63) * 64] = v.y;
        ring[((4 * c + 2) & 63) * 64] = v.z;
        ring[((4 * c + 3) & 63) * 64] = v.w;
    };
    const uint32_t r8 = (uint32_t)((wbase + bp) & 3) * 8;
    uintptr_t m = (wbase + bp - 4) >> 2;  // dword index of the next word's low dword
    const uintptr_t ctop = (wbase + bp + 3) >> 4;
    uintptr_t fc = ctop;  // next chunk to fetch (downwards)
    if (fast) {
        // initial fill: 16 chunks (state bytes follow the words, so ctop is in bounds)
        for (int i = 0; i < 16 && fc >= cmin; i++, fc--) land(in4[fc - c0], fc);
    }
    // the word at dword mm (low) and mm + 1 (high), realigned: slots mm and
    // mm + 1 are one ds_read2st64 thanks to the mirror slot
    auto read_word = [&](uint32_t mm) -> uint32_t {
        const uint32_t *q = ring + (mm & 63) * 64;
        return __builtin_amdgcn_alignbit(q[64], q[0], r8);
    };
    uint32_t nw = fast && bp >= 4 ? read_word(m) : 0u;
    auto step = [&]() -> uint32_t {
        const uint32_t e = s_slot[x & 4095];
        x = (uint64_t)((e >> 8) & 4095) * (x >> 12) + (e >> 20);
        // the common 32-bit renormalisation, branchless: the next word is
        // re-read from the ring every step (LDS bandwidth is idle here)
        const bool small = x < 65536;
        const bool w4 = small && bp >= 4;
        const bool w1 = small && bp > 0 && bp < 4;
        x = w4 ? ((x << 32) | nw) : x;
        bp -= w4 ? 4 : 0;
        m -= w4 ? 1 : 0;
        nw = read_word(m);
        if (w1) {  // the last 1..3 bytes of a stream
            bp -= 1;
            const uintptr_t ad = wbase + bp;
            x = (x << 8) | ((rd(ad >> 2) >> ((ad & 3) * 8)) & 0xFF);
        }
        x |= (x == 0) ? 1u : 0u;  // x = max(x, 1)
        return e & 0xFF;
    };
    // a group that starts with >= 68 unread bytes never reaches the stream's
    // last 1..3 bytes (one word per step at most): renormalise without that
    // branch, and with max(x, 1) folded into the word merge (after a word
    // merge x is 0 only when the decoded x and the word both are)
    // bp and m are settled once per group from the 32-bit word position m32
    // The word is read before the slot entry (both LDS reads land by the one
    // wait the entry needs), and max(x, 1) is a select between the word and
    // max(word, 1) on the low dword of xd (xd < 2^16 whenever it is merged).
    auto step_bulk = [&](uint32_t &m32) -> uint32_t {
        const uint32_t w = read_word(m32);
        const uint32_t e = s_slot[x & 4095];
        const uint64_t xd = (uint64_t)((e >> 8) & 4095) * (x >> 12) + (e >> 20);
        const bool small = xd < 65536;
        const uint32_t xl = (uint32_t)xd;
        // max(x, 1) after the merge: the low word is max(w, [xl == 0]), with
        // [xl == 0] = 1 -sat xl (one clamped subtract)
        const uint64_t merged = ((uint64_t)xl << 32) | max(w, __builtin_elementwise_sub_sat(1u, xl));
        x = small ? merged : xd;
        m32 -= small ? 1 : 0;
        return e;  // (the symbol is the low byte; the caller packs)
    };
    const uint32_t G = fast ? (uint32_t)(B.orig >> 4) : 0u;
    const bool vec = (((uintptr_t)out) & 15) == 0;
    uint32_t Gmax = vec ? G : 0u;  // unaligned output: everything in the tail loop
    const uint32_t Gl = Gmax;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) Gmax = max(Gmax, (uint32_t)__shfl_xor((int)Gmax, d, 64));
    fv4u A0 = {0, 0, 0, 0}, A1 = A0, B0 = A0, B1 = A0;
    uint32_t fa = 0, fb = 0;
    uintptr_t ca = 0, cb = 0;
    auto issue = [&](fv4u &R0, fv4u &R1, uint32_t &fl, uintptr_t &cc) {
        const uintptr_t need = (m + 1) >> 2;  // highest chunk still read
        const bool f0 = fast && fc >= cmin && fc + 16 > need;
        const bool f1 = f0 && fc >= cmin + 1 && fc + 15 > need;
        cc = fc;
        fse_asm_load16(R0, f0 ? in4 + (fc - c0) : in4);
        fse_asm_load16(R1, f1 ? in4 + (fc - 1 - c0) : in4);
        fl = (f0 ? 1u : 0u) | (f1 ? 2u : 0u);
        fc -= (f0 ? 1 : 0) + (f1 ? 1 : 0);
    };
    auto settle = [&](const fv4u R0, const fv4u R1, uint32_t &fl, uintptr_t cc) {
        if (fl & 1) land(R0, cc);
        if (fl & 2) land(R1, cc - 1);
        fl = 0;
    };
    // explicit global address space: a flat store would also count in lgkmcnt
    // and every LDS wait of the next steps would wait for it
    typedef __attribute__((address_space(1))) fv4u gfv4u;
    typedef __attribute__((address_space(1))) uint8_t gu8;
    gfv4u *o4 = (gfv4u *)(out);
    gu8 *ob = (gu8 *)(out);
    auto group = [&](uint32_t g) {
        if (g < Gl) {
            uint32_t o[4] = {0, 0, 0, 0};
            if (bp >= 68) {
                uint32_t m32 = (uint32_t)m;
                if (ZR_FSE_PK) {
                    // the step returns the slot entry e (symbol in its low
                    // byte); four symbols pack into a dword with two v_perm
                    // and an or instead of a mask and a shift-or each
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const uint32_t e0 = step_bulk(m32), e1 = step_bulk(m32);
                        const uint32_t lo = __builtin_amdgcn_perm(e1, e0, 0x0c0c0400u);  // [e0, e1, 0, 0]
                        const uint32_t e2 = step_bulk(m32), e3 = step_bulk(m32);
                        o[q] = __builtin_amdgcn_perm(e3, e2, 0x04000c0cu) | lo;  // [.., .., e2, e3]
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 16; k++) o[k >> 2] |= (step_bulk(m32) & 0xFF) << (8 * (k & 3));
                }
                const uint32_t used = (uint32_t)m - m32;  // words merged by the group
                m -= used;
                bp -= 4ull * used;
                nw = read_word(m);  // the generic step's look-ahead word
            } else {
#pragma unroll
                for (int k = 0; k < 16; k++) o[k >> 2] |= step() << (8 * (k & 3));
            }
            o4[g] = fv4u{o[0], o[1], o[2], o[3]};
        }
    };
    for (uint32_t g = 0; g < Gmax; g += 2) {
        if (g >= 2) {
            asm volatile("s_waitcnt vmcnt(2)" : "+v"(A0), "+v"(A1)::"memory");
            settle(A0, A1, fa, ca);
        }
        group(g);
        issue(A0, A1, fa, ca);
        if (g + 1 < Gmax) {
            if (g + 1 >= 2) {
                asm volatile("s_waitcnt vmcnt(2)" : "+v"(B0), "+v"(B1)::"memory");
                settle(B0, B1, fb, cb);
            }
            group(g + 1);
            issue(B0, B1, fb, cb);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(A0), "+v"(A1), "+v"(B0), "+v"(B1)::"memory");
    settle(A0, A1, fa, ca);
    settle(B0, B1, fb, cb);
    if (fast) {
        // tail (and every symbol of an unaligned output), refilling per symbol as needed
        for (uint64_t i = (uint64_t)Gl << 4; i < B.orig; i++) {
            if ((i & 15) == 0) {
                const uintptr_t need = (m + 1) >> 2;
                while (fc >= cmin && fc + 16 > need) {
                    land(in4[fc - c0], fc);
                    fc--;
                }
            }
            ob[i] = (uint8_t)step();
        }
    } else if (coded) {
        fse_dec_lane<false>(a.tabs[B.table].slot, a.in, a.in + B.words, B.wbytes, B.state, out, B.orig);
    } else if (j < nb && B.raw == 1) {
        const uint8_t *src = a.in + B.body + 5;
        for (uint64_t i = 0; i < B.orig; i++) out[i] = src[i];
    }
}

size_t fse_dec_ws_bytes(uint64_t maxb) {
    return 256 + round_up(sizeof(FseBlk) * maxb, 256) + round_up(4ull * 256 * maxb, 256) +
           round_up(sizeof(FseDTab) * maxb, 256) + round_up(8 * maxb, 256) + 256;
}

struct FsePlan {
    uint64_t nb, bs;
    int mode;  // 0 F5, 1 F6, 2 body only
};
static FsePlan fse_plan(const zr_fse_config *c, uint64_t n) {
    FsePlan p;
    if (c->parallel_blocks != 0 && c->block_size > 0 && n > c->block_size * 2) {
        p.bs = c->block_size;
        p.nb = (n + p.bs - 1) / p.bs;
        p.mode = c->parallel_blocks <= 1 ? 2 : 1;  // Some(1): single body, no mode byte (fse.rs:975-977)
        if (p.mode == 2) {
            p.nb = 1;
            p.bs = n;
        }
    } else {
        p.bs = n;
        p.nb = 1;
        p.mode = 0;
    }
    return p;
}

static int32_t fse_validate(const zr_fse_config *c) {  // FseConfig::validate (fse.rs:317-348)
    if (c->table_log < 5 || c->table_log > 15) return set_error(ZR_INVALID_INPUT, "Table log must be 5-15");
    if (c->compression_level < 1 || c->compression_level > 22)
        return set_error(ZR_INVALID_INPUT, "Compression level must be 1-22");
    if ((1ull << c->table_log) > c->max_table_size) return set_error(ZR_INVALID_INPUT, "Table size exceeds max");
    return ZR_OK;
}

static uint64_t fse_cap(uint64_t bs) { return round_up(bs + bs / 2 + 64, 16); }

}  // namespace zr

using namespace zr;

extern "C" {

void zr_fse_config_default(zr_fse_config *c) {
    c->table_log = 12;
    c->compression_level = 3;
    c->max_table_size = 64 * 1024;
    c->parallel_blocks = 0;
    c->block_size = 64 * 1024;
    c->adaptive = 1;
}

size_t zr_fse_compress_bound(size_t n, const zr_fse_config *c) {
    const FsePlan p = fse_plan(c, n);
    // per block: len + header(3 + 5*256) + words (<= 1.5 B/symbol) + state, + framing
    return n + n / 2 + p.nb * (4 + 3 + 5 * 256 + 8 + 4 + 16) + 64;
}

size_t zr_fse_workspace_bytes(size_t n, const zr_fse_config *c) {
    const FsePlan p = fse_plan(c, n);
    return 1024 + round_up(sizeof(FseDTab), 256) + round_up(p.nb * fse_cap(p.bs), 256) +
           round_up(4 * p.nb, 256) + 3 * round_up(8 * p.nb, 256) + 512;
}

int32_t zr_fse_compress_dev(const zr_fse_config *c, const uint32_t *freqs_dev, const uint8_t *in, size_t n,
                            uint8_t *out, uint64_t *out_len_dev, int32_t *status_dev, void *ws, size_t ws_bytes,
                            void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (capturing((hipStream_t)stream))
        return set_error(ZR_UNSUPPORTED, "zr_fse_compress_dev on a capturing stream");
    int32_t st = fse_validate(c);  // FseEncoder::new (fse.rs:773-786)
    if (st) return st;
    hipStream_t s = (hipStream_t)stream;
    ZR_HIP(hipMemsetAsync(status_dev, 0, 4, s));
    if (n == 0) {  // empty input -> empty output (fse.rs:855-857)
        ZR_HIP(hipMemsetAsync(out_len_dev, 0, 8, s));
        return ZR_OK;
    }
    if (ws_bytes < zr_fse_workspace_bytes(n, c)) return set_error(ZR_INVALID_INPUT, "FSE workspace too small");
    const FsePlan p = fse_plan(c, n);
    uint8_t *w = reinterpret_cast<uint8_t *>(round_up((uintptr_t)ws, 256));
    uint32_t *hist = reinterpret_cast<uint32_t *>(w);
    w += 1024;
    FseDTab *tab = reinterpret_cast<FseDTab *>(w);
    w += round_up(sizeof(FseDTab), 256);
    FseEncArgs a;
    a.in = in;
    a.n = n;
    a.bs = p.bs;
    a.nb = p.nb;
    a.tab = tab;
    a.cap = fse_cap(p.bs);
    a.scratch = w;
    w += round_up(p.nb * a.cap, 256);
    a.wlen = reinterpret_cast<uint32_t *>(w);
    w += round_up(4 * p.nb, 256);
    a.state = reinterpret_cast<uint64_t *>(w);
    w += round_up(8 * p.nb, 256);
    a.body = reinterpret_cast<uint64_t *>(w);
    w += round_up(8 * p.nb, 256);
    uint64_t *boff = reinterpret_cast<uint64_t *>(w);
    a.status = status_dev;
    if (freqs_dev) {
        hist = const_cast<uint32_t *>(freqs_dev);
    } else {
        ZR_HIP(hipMemsetAsync(hist, 0, 1024, s));
        launch_timed("fse_histogram", k_fse_hist, dim3((uint32_t)ceil_div(n, FH_CHUNK)), dim3(256), 0, s, in,
                     (uint64_t)n, hist);
    }
    hipLaunchKernelGGL(k_fse_tab, dim3(1), dim3(256), 0, s, hist, tab);
    launch_timed("fse_encode", k_fse_enc, dim3((uint32_t)ceil_div(p.nb, 64)), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_fse_scan, dim3(1), dim3(256), 0, s, a.body, p.nb, p.mode, out, boff, out_len_dev,
                       status_dev, tab);
    hipLaunchKernelGGL(k_fse_compact, dim3((uint32_t)p.nb), dim3(256), 0, s, a, out, boff);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

size_t zr_fse_decode_workspace_bytes(uint64_t max_blocks) { return fse_dec_ws_bytes(max_blocks ? max_blocks : 1); }

int32_t zr_fse_decompress_dev(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap, uint64_t max_blocks,
                              uint64_t *out_len_dev, int32_t *status_dev, void *ws, size_t ws_bytes,
                              void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (capturing((hipStream_t)stream))
        return set_error(ZR_UNSUPPORTED, "zr_fse_decompress_dev on a capturing stream");
    if (max_blocks == 0) max_blocks = 1;
    if (ws_bytes < fse_dec_ws_bytes(max_blocks)) return set_error(ZR_INVALID_INPUT, "FSE workspace too small");
    hipStream_t s = (hipStream_t)stream;
    uint8_t *w = reinterpret_cast<uint8_t *>(round_up((uintptr_t)ws, 256));
    FseDecArgs a;
    a.in = in;
    a.n = n;
    a.max_blocks = max_blocks;
    a.out_cap = out_cap;
    a.out = out;
    a.nblocks = reinterpret_cast<uint64_t *>(w);
    w += 256;
    a.blk = reinterpret_cast<FseBlk *>(w);
    w += round_up(sizeof(FseBlk) * max_blocks, 256);
    a.freqs = reinterpret_cast<uint32_t *>(w);
    w += round_up(4ull * 256 * max_blocks, 256);
    a.tabs = reinterpret_cast<FseDTab *>(w);
    w += round_up(sizeof(FseDTab) * max_blocks, 256);
    a.ooff = reinterpret_cast<uint64_t *>(w);
    a.out_len = out_len_dev;
    a.status = status_dev;
    const uint32_t gb = (uint32_t)max_blocks;
    hipLaunchKernelGGL(k_fse_frame, dim3(1), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_fse_parse, dim3(gb), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_fse_tabs, dim3(gb), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_fse_outscan, dim3(1), dim3(256), 0, s, a);
    launch_timed("fse_decode", k_fse_dec, dim3((uint32_t)ceil_div(max_blocks, 64)), dim3(64), 0, s, a);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

// ---- host-memory entry points (synchronous, on a leased call context:
// zr_internal.h CallLease -- no allocation in steady state, stream-scoped sync)

int32_t zr_fse_decompressed_size(const uint8_t *in, size_t n, size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    *out_len = 0;
    if (n == 0) return ZR_OK;
    auto body_size = [&](const uint8_t *d, size_t len) -> size_t {
        if (len < 5) return 0;
        return (size_t)d[0] | ((size_t)d[1] << 8) | ((size_t)d[2] << 16) | ((size_t)d[3] << 24);
    };
    if (in[0] == FSE_MODE_SINGLE) {
        *out_len = body_size(in + 1, n - 1);
        return ZR_OK;
    }
    if (in[0] != FSE_MODE_PARALLEL || n < 5) return set_error(ZR_INVALID_INPUT, "unknown FSE stream mode byte");
    const size_t nb = (size_t)in[1] | ((size_t)in[2] << 8) | ((size_t)in[3] << 16) | ((size_t)in[4] << 24);
    if (nb == 0 || nb > (n - 5) / 4) return set_error(ZR_INVALID_INPUT, "invalid FSE block count");
    size_t pos = 5 + 4 * nb, tot = 0;
    for (size_t b = 0; b < nb; b++) {
        const uint8_t *q = in + 5 + 4 * b;
        const size_t bs = (size_t)q[0] | ((size_t)q[1] << 8) | ((size_t)q[2] << 16) | ((size_t)q[3] << 24);
        if (pos + bs > n) return set_error(ZR_INVALID_INPUT, "Invalid block data");
        tot += body_size(in + pos, bs);
        pos += bs;
    }
    *out_len = tot;
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_fse_compress(const zr_fse_config *c, const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                        size_t *out_len) {
    return zr_fse_compress_freqs(c, nullptr, in, n, out, out_cap, out_len);
}

int32_t zr_byte_histogram(const uint8_t *in, size_t n, uint32_t freqs[256]) {
    ZR_GUARD_BEGIN
    clear_error();
    memset(freqs, 0, 1024);
    if (n == 0) return ZR_OK;
    CallLease L;
    int32_t st = L.acquire();
    if (st) return st;
    void *din, *dh;
    if ((st = L.get(0, n, &din)) || (st = L.get(2, 1024, &dh))) return st;
    hipStream_t s = L.stream();
    ZR_HIP(hipMemcpyAsync(din, in, n, hipMemcpyHostToDevice, s));
    ZR_HIP(hipMemsetAsync(dh, 0, 1024, s));
    hipLaunchKernelGGL(k_fse_hist, dim3((uint32_t)ceil_div(n, FH_CHUNK)), dim3(256), 0, s, (const uint8_t *)din,
                       (uint64_t)n, (uint32_t *)dh);
    ZR_HIP(hipGetLastError());
    ZR_HIP(hipMemcpyAsync(freqs, dh, 1024, hipMemcpyDeviceToHost, s));
    return L.sync();
    ZR_GUARD_END
}

int32_t zr_fse_compress_freqs(const zr_fse_config *c, const uint32_t *freqs, const uint8_t *in, size_t n,
                              uint8_t *out, size_t out_cap, size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    int32_t st = fse_validate(c);
    if (st) return st;
    *out_len = 0;
    if (n == 0) return ZR_OK;
    const size_t wsb = zr_fse_workspace_bytes(n, c), cap = zr_fse_compress_bound(n, c);
    CallLease L;
    if ((st = L.acquire())) return st;
    void *din, *dout, *dws, *dm;
    if ((st = L.get(0, n, &din)) || (st = L.get(1, cap, &dout)) || (st = L.get(4, wsb, &dws)) ||
        (st = L.get(2, 64 + 1024, &dm)))
        return st;
    hipStream_t s = L.stream();
    CallCtx *cx = L.ctx();
    ZR_HIP(hipMemcpyAsync(din, in, n, hipMemcpyHostToDevice, s));
    uint64_t *olen = reinterpret_cast<uint64_t *>(dm);
    int32_t *dst = reinterpret_cast<int32_t *>(olen + 1);
    uint32_t *dfreq = nullptr;
    if (freqs) {
        dfreq = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(dm) + 64);
        cx->host_stage.assign(reinterpret_cast<const char *>(freqs), 1024);
        ZR_HIP(hipMemcpyAsync(dfreq, cx->host_stage.data(), 1024, hipMemcpyHostToDevice, s));
    }
    st = zr_fse_compress_dev(c, dfreq, (const uint8_t *)din, n, (uint8_t *)dout, olen, dst, dws, wsb, s);
    if (st) return st;
    uint64_t *meta = cx->meta;
    ZR_HIP(hipMemcpyAsync(meta, dm, 16, hipMemcpyDeviceToHost, s));
    if ((st = L.sync())) return st;
    if ((int32_t)meta[1] != 0) return set_error(ZR_INVALID_INPUT, "FSE compression failed");
    if (meta[0] > out_cap) return set_error(ZR_INVALID_INPUT, "output capacity too small");
    ZR_HIP(hipMemcpyAsync(out, dout, meta[0], hipMemcpyDeviceToHost, s));
    if ((st = L.sync())) return st;
    *out_len = meta[0];
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_fse_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap, size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    *out_len = 0;
    if (n == 0) return ZR_OK;
    // block count bound from the framing (host side)
    uint64_t maxb = 1;
    if (in[0] == FSE_MODE_PARALLEL && n >= 5) {
        const uint64_t nb = (uint64_t)in[1] | ((uint64_t)in[2] << 8) | ((uint64_t)in[3] << 16) | ((uint64_t)in[4] << 24);
        if (nb <= (n - 5) / 4 && nb > 0) maxb = nb;
    }
    const size_t wsb = fse_dec_ws_bytes(maxb);
    CallLease L;
    int32_t st = L.acquire();
    if (st) return st;
    void *din, *dout, *dws, *dm;
    if ((st = L.get(0, n, &din)) || (st = L.get(1, out_cap, &dout)) || (st = L.get(4, wsb, &dws)) ||
        (st = L.get(2, 64, &dm)))
        return st;
    hipStream_t s = L.stream();
    ZR_HIP(hipMemcpyAsync(din, in, n, hipMemcpyHostToDevice, s));
    uint64_t *olen = reinterpret_cast<uint64_t *>(dm);
    int32_t *dst = reinterpret_cast<int32_t *>(olen + 1);
    st = zr_fse_decompress_dev((const uint8_t *)din, n, (uint8_t *)dout, out_cap, maxb, olen, dst, dws, wsb, s);
    if (st) return st;
    uint64_t *meta = L.ctx()->meta;
    ZR_HIP(hipMemcpyAsync(meta, dm, 16, hipMemcpyDeviceToHost, s));
    if ((st = L.sync())) return st;
    if ((int32_t)meta[1] != 0) return set_error((int32_t)meta[1], "FSE decompression failed: invalid data");
    if (meta[0]) ZR_HIP(hipMemcpyAsync(out, dout, meta[0], hipMemcpyDeviceToHost, s));
    if ((st = L.sync())) return st;
    *out_len = meta[0];
    return ZR_OK;
    ZR_GUARD_END
}


// ---- FSE as the PA-Zip second stage (dict_zip/compression_types.rs:2272-2340)
// dict_zip's FseConfig maps to the entropy config with parallel_blocks None and
// 64 KiB blocks/tables (compression_types.rs:2107-2123).
static zr_fse_config pazip_cfg(const zr_fse_config *c) {
    zr_fse_config e = *c;
    e.parallel_blocks = 0;
    e.block_size = 64 * 1024;
    e.max_table_size = 64 * 1024;
    return e;
}

size_t zr_pazip_fse_bound(size_t n, const zr_fse_config *c) {
    const zr_fse_config e = pazip_cfg(c);
    return 2 + std::max(n, zr_fse_compress_bound(n, &e));
}

// apply_fse_compression: "UN" | raw below 32 bytes or when FSE does not shrink
// the data, else "FS" | FseCompressor::compress (a fresh encoder per call)
int32_t zr_pazip_fse_apply(const zr_fse_config *c, const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                           size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!c || !out_len || (!in && n) || (!out && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *out_len = 0;
    if (n == 0) return ZR_OK;
    auto raw = [&]() -> int32_t {
        if (out_cap < n + 2) return set_error(ZR_INVALID_INPUT, "output buffer too small");
        out[0] = 0x55;
        out[1] = 0x4E;
        memcpy(out + 2, in, n);
        *out_len = n + 2;
        return ZR_OK;
    };
    if (n < 32) return raw();
    const zr_fse_config e = pazip_cfg(c);
    int32_t st = fse_validate(&e);  // FseCompressor::with_config -> FseEncoder::new
    if (st) return st;
    std::vector<uint8_t> tmp(zr_fse_compress_bound(n, &e));
    size_t cl = 0;
    if ((st = zr_fse_compress(&e, in, n, tmp.data(), tmp.size(), &cl))) return st;
    if (cl >= n) return raw();
    if (out_cap < cl + 2) return set_error(ZR_INVALID_INPUT, "output buffer too small");
    out[0] = 0xFE;
    out[1] = 0x53;
    memcpy(out + 2, tmp.data(), cl);
    *out_len = cl + 2;
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_pazip_fse_removed_size(const uint8_t *in, size_t n, size_t *size) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!size || (!in && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *size = 0;
    if (n < 2) {
        *size = n;
        return ZR_OK;
    }
    if (in[0] == 0x55 && in[1] == 0x4E) {
        *size = n - 2;
        return ZR_OK;
    }
    if (in[0] == 0xFE && in[1] == 0x53) return zr_fse_decompressed_size(in + 2, n - 2, size);
    return zr_fse_decompressed_size(in, n, size);
    ZR_GUARD_END
}

// remove_fse_compression: "UN" -> raw, "FS" -> FseCompressor::decompress, no
// magic -> decompress the whole input (older format), < 2 bytes -> as is
int32_t zr_pazip_fse_remove(const zr_fse_config *c, const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                            size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!c || !out_len || (!in && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *out_len = 0;
    if (n == 0) return ZR_OK;
    auto copy = [&](const uint8_t *p, size_t len) -> int32_t {
        if (len > out_cap || (!out && len)) return set_error(ZR_INVALID_INPUT, "output buffer too small");
        if (len) memcpy(out, p, len);
        *out_len = len;
        return ZR_OK;
    };
    if (n < 2) return copy(in, n);
    if (in[0] == 0x55 && in[1] == 0x4E) return copy(in + 2, n - 2);
    const zr_fse_config e = pazip_cfg(c);
    int32_t st = fse_validate(&e);
    if (st) return st;
    const bool fs = in[0] == 0xFE && in[1] == 0x53;
    const uint8_t *p = fs ? in + 2 : in;
    const size_t len = fs ? n - 2 : n;
    if (len == 0) return ZR_OK;  // FseCompressor::decompress(&[]) -> empty
    return zr_fse_decompress(p, len, out, out_cap, out_len);
    ZR_GUARD_END
}

}  // extern "C"
