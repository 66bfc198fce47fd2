// zr_compressor.hip -- RansCompressor record format:
// compression/mod.rs:416-512.
//
//   record = 256 x u32 LE normalised frequencies | u32 LE original size | x1 stream
//   (empty input <-> empty record)
//
// compress writes the compressor's *normalised* table; decompress rebuilds
// the coder with Rans64Encoder::new on those stored frequencies, i.e. it
// normalises an already-normalised table again (mod.rs:514). That second
// normalisation is not the identity for skewed tables (SURVEY.md finding 0.9),
// and it is reproduced here, not repaired: the device batch path runs the same
// k_tab on the stored frequencies that builds every other table.
#include <cstring>

#include "zr_internal.h"

using namespace zr;

namespace {

constexpr uint64_t RC_HDR = 256 * 4 + 4;  // frequency table + original size

__device__ __forceinline__ uint32_t ld32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ void st32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

// per-record body offsets for the inner x1 batch
__global__ void k_rc_enc_prep(uint32_t B, const uint64_t *enc_off, uint64_t *body_off) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < B) body_off[b] = enc_off[b] + RC_HDR;
}

// headers of the encoded records: one wave per record
__global__ void k_rc_enc_hdr(uint32_t B, const uint64_t *len, const uint64_t *enc_off, uint64_t *enc_len,
                             const int32_t *status, const RansDTab *T, uint8_t *enc) {
    const uint32_t b = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64, l = threadIdx.x & 63;
    if (b >= B) return;
    const uint64_t n = len[b];
    if (n == 0) {  // Compressor::compress: empty data -> empty output (mod.rs:458-460)
        if (l == 0) enc_len[b] = 0;
        return;
    }
    if (status[b] != 0) return;
    uint8_t *e = enc + enc_off[b];
    for (uint32_t v = l; v < 256; v += 64) st32(e + 4 * v, T->freq[v]);
    if (l == 0) {
        st32(e + 1024, (uint32_t)n);  // `data.len() as u32` (mod.rs:470)
        enc_len[b] += RC_HDR;
    }
}

// decode side: validate headers, pick the first non-empty record as the table source
__global__ void k_rc_dec_prep(uint32_t B, const uint64_t *len, const uint64_t *enc_off, const uint64_t *enc_len,
                              const uint8_t *enc, uint64_t *body_off, uint64_t *body_len, uint64_t *len_in,
                              int32_t *pstat, uint32_t *first) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const uint64_t n = len[b], el = enc_len[b];
    int32_t st = ZR_OK;
    bool live = false;
    if (el == 0) {
        st = n == 0 ? ZR_OK : ZR_INVALID_INPUT;  // empty record decodes to empty data (mod.rs:479-481)
    } else if (el < RC_HDR) {
        st = ZR_INVALID_INPUT;  // "Invalid rANS compressed data format" (mod.rs:483-487)
    } else {
        const uint32_t size = ld32(enc + enc_off[b] + 1024);
        if ((uint64_t)size != n) st = ZR_INVALID_INPUT;  // the caller's length must be the stored size
        else live = true;
    }
    body_off[b] = enc_off[b] + RC_HDR;
    body_len[b] = live ? el - RC_HDR : 0;
    len_in[b] = live ? n : 0;
    pstat[b] = st;
    if (live) atomicMin(first, b);
}

__global__ void k_rc_dec_hist(const uint32_t *first, const uint64_t *enc_off, const uint8_t *enc, uint32_t *hist) {
    const uint32_t f = *first, v = threadIdx.x;
    hist[v] = f == 0xFFFFFFFFu ? 0u : ld32(enc + enc_off[f] + 4 * v);
}

// every live record must carry the table source's frequencies (one compressor
// per batch): one wave per record compares the 1 KiB table
__global__ void k_rc_dec_check(uint32_t B, const uint32_t *first, const uint64_t *enc_off, const uint8_t *enc,
                               uint64_t *len_in, int32_t *pstat) {
    const uint32_t b = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64, l = threadIdx.x & 63;
    if (b >= B || len_in[b] == 0) return;
    const uint8_t *p = enc + enc_off[b], *q = enc + enc_off[*first];
    bool same = true;
    for (uint32_t i = l; i < 256; i += 64) same = same && ld32(p + 4 * i) == ld32(q + 4 * i);
    if (__builtin_amdgcn_ballot_w64(!same) != 0 && l == 0) {
        pstat[b] = ZR_UNSUPPORTED;
        len_in[b] = 0;
    }
}

__global__ void k_rc_dec_merge(uint32_t B, const int32_t *pstat, int32_t *status) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < B && pstat[b] != 0) status[b] = pstat[b];
}

struct RcWork {
    uint64_t *body_off, *body_len, *len_in;
    int32_t *pstat;
    uint32_t *first, *hist;
    void *dtab;
    void *inner;
    size_t inner_bytes;
};

size_t rc_fixed_bytes(uint32_t B) {
    return round_up(8 * (size_t)B, 256) * 3 + round_up(4 * (size_t)B, 256) + 256 + 1024 +
           round_up(sizeof(RansDTab), 256);
}

RcWork rc_carve(uint32_t B, void *ws, size_t ws_bytes) {
    RcWork w;
    uint8_t *p = static_cast<uint8_t *>(ws);
    auto take = [&](size_t n) {
        uint8_t *r = p;
        p += round_up(n, 256);
        return r;
    };
    w.body_off = reinterpret_cast<uint64_t *>(take(8 * (size_t)B));
    w.body_len = reinterpret_cast<uint64_t *>(take(8 * (size_t)B));
    w.len_in = reinterpret_cast<uint64_t *>(take(8 * (size_t)B));
    w.pstat = reinterpret_cast<int32_t *>(take(4 * (size_t)B));
    w.first = reinterpret_cast<uint32_t *>(take(256));
    w.hist = reinterpret_cast<uint32_t *>(take(1024));
    w.dtab = take(sizeof(RansDTab));
    w.inner = p;
    const size_t used = (size_t)(p - static_cast<uint8_t *>(ws));
    w.inner_bytes = ws_bytes > used ? ws_bytes - used : 0;
    return w;
}

}  // namespace

extern "C" {

int32_t zr_rans_compressor_train(const uint8_t *train, size_t n, zr_rans_table *out) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!out || (!train && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    if (n == 0) return set_error(ZR_INVALID_INPUT, "rANS compressor requires training data");  // mod.rs:426-430
    uint32_t f[256];
    int32_t st = zr_byte_histogram(train, n, f);  // mod.rs:433-436 (the min-1 fix-up at :438-448 never fires)
    if (st) return st;
    return zr_rans_table_build(f, out);
    ZR_GUARD_END
}

// a record slot: header + x1 bound (also for empty input, whose inner x1 stream is
// written to the slot before the record is cut back to empty)
size_t zr_rans_compressor_bound(size_t n) { return RC_HDR + zr_rans_encode_bound(n, 1); }

int32_t zr_rans_compressor_compress(const zr_rans_table *t, const uint8_t *in, size_t n, uint8_t *out,
                                    size_t out_cap, size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!t || (!in && n) || !out_len || (!out && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *out_len = 0;
    if (n == 0) return ZR_OK;
    if (out_cap < RC_HDR) return set_error(ZR_INVALID_INPUT, "output buffer too small");
    for (int v = 0; v < 256; v++) {
        const uint32_t f = t->freq[v];
        for (int k = 0; k < 4; k++) out[4 * v + k] = (uint8_t)(f >> (8 * k));
    }
    const uint32_t size = (uint32_t)n;
    for (int k = 0; k < 4; k++) out[1024 + k] = (uint8_t)(size >> (8 * k));
    size_t body = 0;
    int32_t st = zr_rans_encode(t, 1, in, n, out + RC_HDR, out_cap - RC_HDR, &body);
    if (st) return st;
    *out_len = RC_HDR + body;
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_rans_compressor_decompressed_size(const uint8_t *in, size_t n, size_t *size) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!size || (!in && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *size = 0;
    if (n == 0) return ZR_OK;
    if (n < RC_HDR) return set_error(ZR_INVALID_INPUT, "Invalid rANS compressed data format");
    *size = (size_t)in[1024] | ((size_t)in[1025] << 8) | ((size_t)in[1026] << 16) | ((size_t)in[1027] << 24);
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_rans_compressor_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                                      size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!out_len || (!in && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *out_len = 0;
    size_t size = 0;
    int32_t st = zr_rans_compressor_decompressed_size(in, n, &size);
    if (st || n == 0) return st;
    if (size > out_cap || (!out && size)) return set_error(ZR_INVALID_INPUT, "output buffer too small");
    uint32_t f[256];
    for (int v = 0; v < 256; v++)
        f[v] = (uint32_t)in[4 * v] | ((uint32_t)in[4 * v + 1] << 8) | ((uint32_t)in[4 * v + 2] << 16) |
               ((uint32_t)in[4 * v + 3] << 24);
    zr_rans_table t;
    if ((st = zr_rans_table_build(f, &t))) return st;  // Rans64Encoder::new on stored freqs (mod.rs:514)
    if ((st = zr_rans_decode(&t, 1, in + RC_HDR, n - RC_HDR, out, size))) return st;
    *out_len = size;
    return ZR_OK;
    ZR_GUARD_END
}

size_t zr_rans_compressor_workspace_bytes(uint32_t n_buffers, uint64_t max_len) {
    return rc_fixed_bytes(n_buffers) + rans_workspace_bytes(n_buffers, 1, max_len);
}

int32_t zr_rans_compressor_compress_batch_dev(const zr_rans_batch *bt, const uint8_t *raw, uint8_t *enc,
                                              void *ws, size_t ws_bytes, void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (capturing((hipStream_t)stream))
        return set_error(ZR_UNSUPPORTED, "zr_rans_compressor_compress_batch_dev on a capturing stream");
    if (!bt) return set_error(ZR_INVALID_INPUT, "null batch");
    if (bt->n_streams != 1 || bt->table_stride != 0)
        return set_error(ZR_INVALID_INPUT, "RansCompressor batches are x1 with one shared table");
    const uint32_t B = bt->n_buffers;
    if (B == 0) return ZR_OK;
    if (ws_bytes < zr_rans_compressor_workspace_bytes(B, bt->max_len))
        return set_error(ZR_INVALID_INPUT, "workspace too small");
    RcWork w = rc_carve(B, ws, ws_bytes);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_rc_enc_prep, dim3((uint32_t)ceil_div(B, 256)), dim3(256), 0, s, B, bt->enc_off,
                       w.body_off);
    ZR_HIP(hipGetLastError());
    zr_rans_batch in = *bt;
    in.enc_off = w.body_off;
    int32_t st = zr_rans_encode_batch_dev(&in, raw, enc, w.inner, w.inner_bytes, stream);
    if (st) return st;
    hipLaunchKernelGGL(k_rc_enc_hdr, dim3((uint32_t)ceil_div(B, 4)), dim3(256), 0, s, B, bt->len, bt->enc_off,
                       bt->enc_len, bt->status, reinterpret_cast<const RansDTab *>(bt->tables), enc);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_rans_compressor_decompress_batch_dev(const zr_rans_batch *bt, const uint8_t *enc, uint8_t *raw,
                                                void *ws, size_t ws_bytes, void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (capturing((hipStream_t)stream))
        return set_error(ZR_UNSUPPORTED, "zr_rans_compressor_decompress_batch_dev on a capturing stream");
    if (!bt) return set_error(ZR_INVALID_INPUT, "null batch");
    if (bt->n_streams != 1) return set_error(ZR_INVALID_INPUT, "RansCompressor batches are x1");
    const uint32_t B = bt->n_buffers;
    if (B == 0) return ZR_OK;
    if (ws_bytes < zr_rans_compressor_workspace_bytes(B, bt->max_len))
        return set_error(ZR_INVALID_INPUT, "workspace too small");
    RcWork w = rc_carve(B, ws, ws_bytes);
    hipStream_t s = (hipStream_t)stream;
    ZR_HIP(hipMemsetAsync(w.first, 0xFF, 4, s));
    hipLaunchKernelGGL(k_rc_dec_prep, dim3((uint32_t)ceil_div(B, 256)), dim3(256), 0, s, B, bt->len, bt->enc_off,
                       bt->enc_len, enc, w.body_off, w.body_len, w.len_in, w.pstat, w.first);
    hipLaunchKernelGGL(k_rc_dec_hist, dim3(1), dim3(256), 0, s, w.first, bt->enc_off, enc, w.hist);
    ZR_HIP(hipGetLastError());
    int32_t st = zr_rans_dtab_from_hist_dev(w.hist, 1, w.dtab, stream);
    if (st) return st;
    hipLaunchKernelGGL(k_rc_dec_check, dim3((uint32_t)ceil_div(B, 4)), dim3(256), 0, s, B, w.first, bt->enc_off,
                       enc, w.len_in, w.pstat);
    ZR_HIP(hipGetLastError());
    zr_rans_batch in = *bt;
    in.len = w.len_in;
    in.enc_off = w.body_off;
    in.enc_len = w.body_len;
    in.tables = w.dtab;
    in.table_stride = 0;
    in.min_len = 0;
    if ((st = zr_rans_decode_batch_dev(&in, enc, raw, w.inner, w.inner_bytes, stream))) return st;
    hipLaunchKernelGGL(k_rc_dec_merge, dim3((uint32_t)ceil_div(B, 256)), dim3(256), 0, s, B, w.pstat, bt->status);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

}  // extern "C"
