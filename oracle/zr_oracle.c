/*
 * zr_oracle.c -- CPU restatement of infinilabs/zipora src/entropy.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py. Never linked into or called by the product.
 *
 * Every function cites the reference file:line it restates. Rust release
 * semantics are kept: u64/u32 arithmetic wraps (Cargo.toml [profile.release]
 * has no overflow checks), integer division truncates, to_le_bytes is LE.
 *
 * Parity is pinned by SURVEY.md Appendix B and the reference's exact asserts
 * (see zr_oracle.h header and tests/test_oracle_kats.py).
 */
#include "zr_oracle.h"

#include <stdlib.h>
#include <string.h>

#define OK 0
#define EINVAL_DATA (-1)
#define EUNSUP (-4)

/* ------------------------------------------------------------------------ */
/* small growable byte vector                                                */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint8_t *p;
    size_t n, cap;
} bvec;

static int bv_reserve(bvec *v, size_t need) {
    if (need <= v->cap) return 0;
    size_t c = v->cap ? v->cap : 64;
    while (c < need) c *= 2;
    uint8_t *q = (uint8_t *)realloc(v->p, c);
    if (!q) return -1;
    v->p = q;
    v->cap = c;
    return 0;
}
static void bv_push(bvec *v, uint8_t b) {
    if (v->n == v->cap) bv_reserve(v, v->n + 1);
    v->p[v->n++] = b;
}
static void bv_put(bvec *v, const void *src, size_t k) {
    bv_reserve(v, v->n + k);
    memcpy(v->p + v->n, src, k);
    v->n += k;
}
static void bv_u32(bvec *v, uint32_t x) {
    uint8_t b[4] = {(uint8_t)x, (uint8_t)(x >> 8), (uint8_t)(x >> 16), (uint8_t)(x >> 24)};
    bv_put(v, b, 4);
}
static void bv_u64(bvec *v, uint64_t x) {
    for (int i = 0; i < 8; i++) bv_push(v, (uint8_t)(x >> (8 * i)));
}
static uint32_t rd_u32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint64_t rd_u64(const uint8_t *p) {
    uint64_t x = 0;
    for (int i = 7; i >= 0; i--) x = (x << 8) | p[i];
    return x;
}

/* ======================================================================== */
/* rANS -- src/entropy/rans.rs                                               */
/* ======================================================================== */
#define RANS64_L (1ull << 16) /* rans.rs:14 */
#define TOTFREQ 4096u         /* rans.rs:15-16 */

/* Rans64Encoder::normalize_frequencies, rans.rs:238-299. */
static int rans_normalize(const uint32_t f[256], uint32_t total_freq, uint32_t norm[256]) {
    uint32_t remaining = TOTFREQ;
    int used = 0;
    memset(norm, 0, 256 * sizeof(uint32_t));
    for (int i = 0; i < 256; i++) /* first pass, rans.rs:244-250 */
        if (f[i] > 0) {
            norm[i] = 1;
            remaining -= 1;
            used++;
        }
    if (used == 0) return EINVAL_DATA; /* rans.rs:252-256 */
    /* second pass with the budget captured before the loop, rans.rs:263-271 */
    uint64_t initial_remaining = remaining;
    for (int i = 0; i < 256; i++) {
        if (f[i] > 0 && remaining > 0) {
            uint32_t additional = (uint32_t)(((uint64_t)f[i] * initial_remaining) / (uint64_t)total_freq);
            uint32_t to_add = additional < remaining ? additional : remaining;
            norm[i] += to_add;
            remaining -= to_add;
        }
    }
    /* third pass, rans.rs:274-296 */
    while (remaining > 0) {
        uint32_t max_freq = 0;
        int max_idx = 0;
        for (int i = 0; i < 256; i++)
            if (f[i] > max_freq && norm[i] < TOTFREQ / 4) {
                max_freq = f[i];
                max_idx = i;
            }
        if (max_freq == 0) {
            for (int i = 0; i < 256; i++)
                if (f[i] > 0) {
                    max_idx = i;
                    break;
                }
        }
        norm[max_idx] += 1;
        remaining -= 1;
    }
    return OK;
}

/* Rans64Encoder::new, rans.rs:208-235 (sum is a wrapping u32 sum). */
int or_rans_table_build(const uint32_t raw[256], or_rans_table *t) {
    uint32_t total = 0;
    for (int i = 0; i < 256; i++) total += raw[i];
    memset(t, 0, sizeof(*t));
    if (total == 0) return OK; /* empty encoder, rans.rs:210-216 */
    int st = rans_normalize(raw, total, t->freq);
    if (st) return st;
    uint32_t cum = 0;
    for (int i = 0; i < 256; i++) { /* rans.rs:225-228 */
        t->start[i] = cum;
        cum += t->freq[i];
    }
    t->total_freq = TOTFREQ;
    return OK;
}

size_t or_rans_encode_bound(size_t n, uint32_t n_streams) {
    /* <= 2 renorm bytes per symbol (state in [2^16, 2^24)) + header */
    return 2 * n + 12 * (size_t)(n_streams ? n_streams : 1) + 16;
}

/* Rans64Encoder::encode_symbol, rans.rs:303-335. */
static int rans_encode_symbol(const or_rans_table *t, uint64_t *x, uint8_t sym, bvec *out) {
    uint32_t f = t->freq[sym];
    if (f == 0) return EINVAL_DATA; /* "Symbol {} not in frequency table" */
    uint64_t max_state = ((RANS64_L << 8) / TOTFREQ) * (uint64_t)f;
    while (*x >= max_state) {
        bv_push(out, (uint8_t)(*x & 0xFF));
        *x >>= 8;
    }
    uint64_t s = *x;
    *x = ((s / f) * TOTFREQ) + (s % f) + t->start[sym];
    return OK;
}

/* encode_single, rans.rs:354-366 */
static int rans_encode_single(const or_rans_table *t, const uint8_t *in, size_t n, bvec *out) {
    uint64_t x = RANS64_L;
    for (size_t i = n; i-- > 0;) {
        int st = rans_encode_symbol(t, &x, in[i], out);
        if (st) return st;
    }
    bv_u64(out, x);
    return OK;
}

/* Rans64Encoder::encode, rans.rs:338-420 (runtime N). */
int or_rans_encode(const or_rans_table *t, uint32_t N, const uint8_t *in, size_t n, uint8_t *out,
                   size_t *out_len) {
    bvec o = {0};
    int st = OK;
    if (n == 0) { /* rans.rs:339-344 */
        bv_u64(&o, RANS64_L);
    } else if (N <= 1 || n < N) { /* rans.rs:346-347, :373-376 */
        st = rans_encode_single(t, in, n, &o);
    } else {
        uint64_t *states = (uint64_t *)malloc(sizeof(uint64_t) * N);
        bvec *outs = (bvec *)calloc(N, sizeof(bvec));
        for (uint32_t s = 0; s < N && st == OK; s++) {
            states[s] = RANS64_L;
            size_t cnt = (n - s - 1) / N + 1; /* indices s, s+N, ... < n (rans.rs:388-391) */
            for (size_t k = cnt; k-- > 0;) { /* reverse order, rans.rs:394-399 */
                st = rans_encode_symbol(t, &states[s], in[s + k * N], &outs[s]);
                if (st) break;
            }
        }
        if (st == OK) {
            for (uint32_t s = 0; s < N; s++) bv_u64(&o, states[s]);        /* rans.rs:405-407 */
            for (uint32_t s = 0; s < N; s++) bv_u32(&o, (uint32_t)outs[s].n); /* rans.rs:410-412 */
            for (uint32_t s = 0; s < N; s++) bv_put(&o, outs[s].p, outs[s].n); /* :415-417 */
        }
        for (uint32_t s = 0; s < N; s++) free(outs[s].p);
        free(outs);
        free(states);
    }
    if (st == OK) {
        memcpy(out, o.p, o.n);
        *out_len = o.n;
    }
    free(o.p);
    return st;
}

typedef struct {
    uint8_t tbl[TOTFREQ];
    const or_rans_table *t;
} rans_dec;

/* Rans64Decoder::new, rans.rs:449-468 */
static void rans_dec_init(rans_dec *d, const or_rans_table *t) {
    memset(d->tbl, 0, sizeof(d->tbl));
    d->t = t;
    for (int s = 0; s < 256; s++)
        for (uint32_t i = 0; i < t->freq[s]; i++)
            if (t->start[s] + i < TOTFREQ) d->tbl[t->start[s] + i] = (uint8_t)s;
}

/* decode_symbol, rans.rs:472-507 */
static int rans_decode_symbol(const rans_dec *d, uint64_t *x, const uint8_t *in, size_t *pos,
                              uint8_t *sym) {
    while (*x < RANS64_L) {
        if (*pos == 0) return EINVAL_DATA; /* "Insufficient data for decoding" */
        *pos -= 1;
        *x = (*x << 8) | in[*pos];
    }
    uint32_t slot = (uint32_t)(*x % TOTFREQ);
    uint8_t s = d->tbl[slot];
    uint64_t f = d->t->freq[s], st = d->t->start[s], v = *x;
    *x = f * (v / TOTFREQ) + (v % TOTFREQ) - st;
    *sym = s;
    return OK;
}

/* decode_single, rans.rs:523-552 */
static int rans_decode_single(const rans_dec *d, const uint8_t *in, size_t len, uint8_t *out,
                              size_t n) {
    if (len < 8) return EINVAL_DATA; /* "rANS data too short" */
    uint64_t x = rd_u64(in + len - 8);
    size_t pos = len - 8;
    for (size_t i = 0; i < n; i++) {
        int st = rans_decode_symbol(d, &x, in, &pos, &out[i]);
        if (st) return st;
    }
    return OK;
}

/* Rans64Decoder::decode, rans.rs:510-651 */
int or_rans_decode(const or_rans_table *t, uint32_t N, const uint8_t *in, size_t len, uint8_t *out,
                   size_t n) {
    if (n == 0) return OK; /* rans.rs:511-513 */
    rans_dec *d = (rans_dec *)malloc(sizeof(rans_dec));
    rans_dec_init(d, t);
    int st = OK;
    if (N <= 1 || n < N) { /* rans.rs:515-516, :558-561 */
        st = rans_decode_single(d, in, len, out, n);
        free(d);
        return st;
    }
    size_t hdr = (size_t)N * 12; /* rans.rs:563-568 */
    if (len < hdr) {
        free(d);
        return EINVAL_DATA;
    }
    uint64_t total = 0;
    for (uint32_t s = 0; s < N; s++) total += rd_u32(in + (size_t)N * 8 + 4 * (size_t)s);
    if (hdr + total > len) { /* rans.rs:601-610 */
        free(d);
        return EINVAL_DATA;
    }
    size_t off = hdr;
    for (uint32_t s = 0; s < N && st == OK; s++) {
        uint64_t x = rd_u64(in + 8 * (size_t)s);
        size_t L = rd_u32(in + (size_t)N * 8 + 4 * (size_t)s);
        const uint8_t *sd = in + off;
        size_t pos = L; /* read backwards from the stream end, rans.rs:624-626 */
        for (size_t i = s; i < n; i += N) {
            st = rans_decode_symbol(d, &x, sd, &pos, &out[i]);
            if (st) break;
        }
        off += L;
    }
    free(d);
    return st;
}

/* ------------------------------------------------------------------------ */
/* Data-structure mirror of encode_parallel / decode_parallel (rans.rs:369-420, */
/* :555-651), for bench.py's single-thread CPU baseline only: the reference's  */
/* per-stream Vec<usize> index vectors (8 B per input byte, :385-391 and       */
/* :629-633), per-stream Vec<u8> outputs grown by push, and the final Vec      */
/* built by extend. Rust's RawVec growth (doubling, minimum capacity 8 for     */
/* u8 and 4 for usize) is followed. Same bytes as or_rans_encode/decode.       */
/* ------------------------------------------------------------------------ */
typedef struct {
    size_t *p;
    size_t n, cap;
} ivec;

static void iv_push(ivec *v, size_t x) {
    if (v->n == v->cap) {
        size_t c = v->cap ? 2 * v->cap : 4;
        v->p = (size_t *)realloc(v->p, c * sizeof(size_t));
        v->cap = c;
    }
    v->p[v->n++] = x;
}

static void rv_push(bvec *v, uint8_t b) { /* Vec<u8>::push: doubling from 8 */
    if (v->n == v->cap) {
        size_t c = v->cap ? 2 * v->cap : 8;
        v->p = (uint8_t *)realloc(v->p, c);
        v->cap = c;
    }
    v->p[v->n++] = b;
}

int or_rans_encode_mirror(const or_rans_table *t, uint32_t N, const uint8_t *in, size_t n, uint8_t *out,
                          size_t *out_len) {
    if (n == 0 || N <= 1 || n < N) return or_rans_encode(t, N, in, n, out, out_len);
    uint64_t *states = (uint64_t *)malloc(sizeof(uint64_t) * N); /* vec![Rans64State::new(); N] */
    bvec *outputs = (bvec *)calloc(N, sizeof(bvec));              /* vec![Vec::new(); N] */
    ivec *idx = (ivec *)calloc(N, sizeof(ivec));                  /* stream_indices */
    for (uint32_t s = 0; s < N; s++) states[s] = RANS64_L;
    for (size_t i = 0; i < n; i++) iv_push(&idx[i % N], i); /* rans.rs:388-391 */
    int st = OK;
    for (uint32_t s = 0; s < N && st == OK; s++) { /* rans.rs:394-399 */
        for (size_t k = idx[s].n; k-- > 0;) {
            const uint8_t sym = in[idx[s].p[k]];
            const uint32_t f = t->freq[sym];
            if (f == 0) {
                st = EINVAL_DATA;
                break;
            }
            const uint64_t max_state = ((RANS64_L << 8) / TOTFREQ) * (uint64_t)f; /* rans.rs:319-323 */
            while (states[s] >= max_state) {
                rv_push(&outputs[s], (uint8_t)(states[s] & 0xFF));
                states[s] >>= 8;
            }
            const uint64_t x = states[s];
            states[s] = ((x / f) * TOTFREQ) + (x % f) + t->start[sym]; /* rans.rs:326-332 */
        }
    }
    if (st == OK) {
        bvec o = {0}; /* final_output: Vec::new() + extend_from_slice */
        for (uint32_t s = 0; s < N; s++) bv_u64(&o, states[s]);
        for (uint32_t s = 0; s < N; s++) bv_u32(&o, (uint32_t)outputs[s].n);
        for (uint32_t s = 0; s < N; s++) bv_put(&o, outputs[s].p, outputs[s].n);
        memcpy(out, o.p, o.n);
        *out_len = o.n;
        free(o.p);
    }
    for (uint32_t s = 0; s < N; s++) {
        free(outputs[s].p);
        free(idx[s].p);
    }
    free(outputs);
    free(idx);
    free(states);
    return st;
}

int or_rans_decode_mirror(const or_rans_table *t, uint32_t N, const uint8_t *in, size_t len, uint8_t *out,
                          size_t n) {
    if (n == 0 || N <= 1 || n < N) return or_rans_decode(t, N, in, len, out, n);
    const size_t hdr = (size_t)N * 12;
    if (len < hdr) return EINVAL_DATA;
    rans_dec *d = (rans_dec *)malloc(sizeof(rans_dec)); /* Rans64Decoder::new */
    rans_dec_init(d, t);
    uint64_t *states = (uint64_t *)malloc(sizeof(uint64_t) * N);
    size_t *lens = (size_t *)malloc(sizeof(size_t) * N);
    const uint8_t **data = (const uint8_t **)malloc(sizeof(uint8_t *) * N);
    size_t *positions = (size_t *)malloc(sizeof(size_t) * N);
    size_t total = 0, pos = 0;
    for (uint32_t s = 0; s < N; s++, pos += 8) states[s] = rd_u64(in + pos); /* rans.rs:571-588 */
    for (uint32_t s = 0; s < N; s++, pos += 4) {                              /* rans.rs:592-606 */
        lens[s] = rd_u32(in + pos);
        total += lens[s];
    }
    int st = OK;
    if (pos + total > len) st = EINVAL_DATA; /* rans.rs:608-610 */
    if (st == OK) {
        for (uint32_t s = 0; s < N; s++) { /* rans.rs:613-617 */
            data[s] = in + pos;
            pos += lens[s];
            positions[s] = lens[s]; /* rans.rs:624-626 */
        }
        memset(out, 0, n);             /* vec![0u8; output_length] */
        ivec *idx = (ivec *)calloc(N, sizeof(ivec));
        for (size_t i = 0; i < n; i++) iv_push(&idx[i % N], i); /* rans.rs:629-633 */
        for (uint32_t s = 0; s < N && st == OK; s++) {       /* rans.rs:636-648 */
            for (size_t k = 0; k < idx[s].n; k++) {
                uint8_t sym;
                st = rans_decode_symbol(d, &states[s], data[s], &positions[s], &sym);
                if (st) break;
                out[idx[s].p[k]] = sym;
            }
        }
        for (uint32_t s = 0; s < N; s++) free(idx[s].p);
        free(idx);
    }
    free(positions);
    free(data);
    free(lens);
    free(states);
    free(d);
    return st;
}

/* ======================================================================== */
/* FSE -- src/entropy/fse.rs                                                  */
/* ======================================================================== */
#define FSE_MODE_SINGLE 0xF5   /* fse.rs:15 */
#define FSE_MODE_PARALLEL 0xF6 /* fse.rs:17 */
#define FSE_TF_SHIFT 12        /* fse.rs:425 */

void or_fse_config_default(or_fse_config *c) { /* fse.rs:245-263 */
    c->table_log = 12;
    c->compression_level = 3;
    c->max_table_size = 64 * 1024;
    c->parallel_blocks = 0;
    c->block_size = 64 * 1024;
    c->adaptive = 1;
}

/* FseConfig::validate, fse.rs:317-348 (max_symbol is fixed at 255 here). */
static int fse_validate(const or_fse_config *c) {
    if (c->table_log < 5 || c->table_log > 15) return EINVAL_DATA;
    if (c->compression_level < 1 || c->compression_level > 22) return EINVAL_DATA;
    if ((1ull << c->table_log) > c->max_table_size) return EINVAL_DATA;
    return OK;
}

/* FseTable::normalize_frequencies_exact, fse.rs:513-580 */
int or_fse_normalize_exact(const uint32_t f[256], uint32_t table_size, uint32_t norm[256]) {
    uint64_t total = 0;
    uint32_t count = 0;
    for (int i = 0; i < 256; i++) {
        total += f[i];
        count += f[i] > 0;
    }
    if (total == 0) return EINVAL_DATA;
    if (count > table_size) return EINVAL_DATA;
    uint64_t assigned = 0;
    memset(norm, 0, 256 * sizeof(uint32_t));
    for (int i = 0; i < 256; i++)
        if (f[i] > 0) {
            uint32_t scaled = (uint32_t)(((uint64_t)f[i] * table_size) / total);
            norm[i] = scaled > 1 ? scaled : 1;
            assigned += norm[i];
        }
    if (assigned > table_size) {
        uint64_t excess = assigned - table_size;
        while (excess > 0) {
            int max_idx = 0;
            uint32_t max_val = 0;
            for (int i = 0; i < 256; i++)
                if (norm[i] > max_val) {
                    max_val = norm[i];
                    max_idx = i;
                }
            uint64_t take = excess < (uint64_t)(max_val - 1) ? excess : (uint64_t)(max_val - 1);
            norm[max_idx] -= (uint32_t)take;
            excess -= take;
        }
    } else if (assigned < table_size) {
        int max_idx = 0;
        uint32_t max_val = 0;
        for (int i = 0; i < 256; i++)
            if (f[i] > max_val) {
                max_val = f[i];
                max_idx = i;
            }
        norm[max_idx] += (uint32_t)(table_size - assigned);
    }
    return OK;
}

typedef struct {
    uint64_t rcp_freq;
    uint16_t freq, bias, cmpl_freq;
    uint8_t rcp_shift;
} fse_enc_sym; /* fse.rs:352-359 */

typedef struct {
    uint32_t freq[256]; /* normalised frequencies (header content) */
    fse_enc_sym enc[256];
    uint16_t dstart[256], dfreq[256];
    uint8_t alias[4096];
    uint8_t max_symbol;
} fse_table;

/* FseTable::init_enc_symbol, fse.rs:583-615 */
static void fse_init_enc_symbol(fse_enc_sym *s, uint32_t start, uint32_t freq, uint32_t scale_bits) {
    s->freq = (uint16_t)freq;
    s->cmpl_freq = (uint16_t)((1u << scale_bits) - freq);
    if (freq < 2) {
        s->rcp_freq = ~0ull;
        s->rcp_shift = 0;
        s->bias = (uint16_t)(start + (1u << scale_bits) - 1);
    } else {
        uint32_t shift = 0;
        while (freq > (1u << shift)) shift++;
        uint64_t x0 = freq - 1;
        uint64_t x1 = 1ull << (shift + 31);
        uint64_t t1 = x1 / freq;
        uint64_t x0e = x0 + ((x1 % freq) << 32);
        uint64_t t0 = x0e / freq;
        s->rcp_freq = t0 + (t1 << 32);
        s->rcp_shift = (uint8_t)(shift - 1);
        s->bias = (uint16_t)start;
    }
}

/* FseTable::mul_hi, fse.rs:618-628 -- the middle sum wraps in release builds. */
uint64_t or_fse_mul_hi(uint64_t a, uint64_t b) {
    uint64_t a_lo = a & 0xFFFFFFFFull, a_hi = a >> 32;
    uint64_t b_lo = b & 0xFFFFFFFFull, b_hi = b >> 32;
    uint64_t x0 = b_lo * a_lo;
    uint64_t x1 = (b_lo * a_hi) + (b_hi * a_lo) + (x0 >> 32);
    return (b_hi * a_hi) + (x1 >> 32);
}

/* FseTable::new, fse.rs:411-500 (config already validated by the caller). */
static int fse_table_new(const uint32_t freqs[256], fse_table *t) {
    int max_symbol = -1;
    for (int i = 255; i >= 0; i--)
        if (freqs[i] > 0) {
            max_symbol = i;
            break;
        }
    if (max_symbol < 0) return EINVAL_DATA; /* "No symbols found in frequency table" */
    int st = or_fse_normalize_exact(freqs, 4096, t->freq);
    if (st) return st;
    memset(t->enc, 0, sizeof(t->enc));
    memset(t->dstart, 0, sizeof(t->dstart));
    memset(t->dfreq, 0, sizeof(t->dfreq));
    memset(t->alias, 0, sizeof(t->alias));
    uint32_t pos = 0;
    for (int s = 0; s <= max_symbol; s++) {
        uint32_t f = t->freq[s];
        if (!f) continue;
        fse_init_enc_symbol(&t->enc[s], pos, f, FSE_TF_SHIFT);
        t->dstart[s] = (uint16_t)pos;
        t->dfreq[s] = (uint16_t)f;
        for (uint32_t i = 0; i < f; i++) t->alias[pos + i] = (uint8_t)s;
        pos += f;
    }
    t->max_symbol = (uint8_t)max_symbol;
    return OK;
}

/* compress_single_internal, fse.rs:887-966 */
static int fse_compress_single(const fse_table *t, const uint8_t *d, size_t n, bvec *o) {
    if (n < 100) { /* raw marker, fse.rs:892-904 */
        bv_u32(o, (uint32_t)n);
        bv_push(o, 0xFF);
        bv_put(o, d, n);
        return OK;
    }
    bv_u32(o, (uint32_t)n);
    bv_push(o, FSE_TF_SHIFT); /* table.table_log is always TF_SHIFT (fse.rs:491) */
    uint16_t nsym = 0;
    for (int s = 0; s < 256; s++)
        if (t->freq[s] > 0 && s <= t->max_symbol) nsym++;
    bv_push(o, (uint8_t)nsym);
    bv_push(o, (uint8_t)(nsym >> 8));
    for (int s = 0; s < 256; s++)
        if (t->freq[s] > 0 && s <= t->max_symbol) {
            bv_push(o, (uint8_t)s);
            bv_u32(o, t->freq[s]);
        }
    uint64_t x = 1; /* fse.rs:931 */
    for (size_t i = n; i-- > 0;) {
        const fse_enc_sym *e = &t->enc[d[i]];
        uint32_t f = e->freq;
        /* renormalize_encode, fse.rs:680-700 */
        uint64_t x_max = ((65536ull >> FSE_TF_SHIFT) << 32) * (uint64_t)f;
        if (x >= x_max) {
            bv_u32(o, (uint32_t)x);
            x >>= 32;
        }
        if (f == 0) return EINVAL_DATA; /* encode_symbol None, fse.rs:946-953 */
        uint64_t q = or_fse_mul_hi(x, e->rcp_freq) >> e->rcp_shift; /* fse.rs:639 */
        x = x + (uint64_t)e->bias + q * (uint64_t)e->cmpl_freq;   /* fse.rs:642 */
    }
    bv_u64(o, x);
    return OK;
}

size_t or_fse_compress_bound(size_t n, const or_fse_config *c) {
    size_t bs = c->block_size ? c->block_size : 1;
    size_t nblocks = n / bs + 2;
    /* per block: 4+1+2+5*256 header, <=4 bytes per 16 bits of expansion... words <= n/2+4 */
    return n + n / 2 + nblocks * (4 + 1 + 2 + 5 * 256 + 8 + 4 + 16) + 64;
}

/* FseEncoder::compress, fse.rs:854-884; compress_parallel fse.rs:970-1023;
 * merge_compressed_blocks fse.rs:1026-1044. */
int or_fse_compress(const or_fse_config *c, const uint8_t *in, size_t n, uint8_t *out,
                    size_t *out_len) {
    return or_fse_compress_freqs(c, NULL, in, n, out, out_len);
}

int or_fse_compress_freqs(const or_fse_config *c, const uint32_t *freqs, const uint8_t *in, size_t n,
                          uint8_t *out, size_t *out_len) {
    int st = fse_validate(c); /* FseEncoder::new, fse.rs:773-786 */
    if (st) return st;
    if (n == 0) {
        *out_len = 0;
        return OK;
    }
    uint32_t hist[256] = {0};
    if (freqs) memcpy(hist, freqs, sizeof(hist));
    else
        for (size_t i = 0; i < n; i++) hist[in[i]]++; /* analyze_frequencies fse.rs:796-851 */
    fse_table *t = (fse_table *)malloc(sizeof(fse_table));
    st = fse_table_new(hist, t);
    if (st) {
        free(t);
        return st;
    }
    bvec o = {0};
    if (c->parallel_blocks != 0 && c->block_size > 0 && n > c->block_size * 2) {
        size_t bs = c->block_size;
        size_t nchunks = (n + bs - 1) / bs;
        if (nchunks <= 1 || c->parallel_blocks <= 1) {
            st = fse_compress_single(t, in, n, &o); /* no mode byte (reference quirk, fse.rs:975-977) */
        } else {
            bvec *bodies = (bvec *)calloc(nchunks, sizeof(bvec));
            for (size_t b = 0; b < nchunks && st == OK; b++) {
                size_t len = (b + 1) * bs <= n ? bs : n - b * bs;
                st = fse_compress_single(t, in + b * bs, len, &bodies[b]);
            }
            if (st == OK) {
                bv_push(&o, FSE_MODE_PARALLEL);
                bv_u32(&o, (uint32_t)nchunks);
                for (size_t b = 0; b < nchunks; b++) bv_u32(&o, (uint32_t)bodies[b].n);
                for (size_t b = 0; b < nchunks; b++) bv_put(&o, bodies[b].p, bodies[b].n);
            }
            for (size_t b = 0; b < nchunks; b++) free(bodies[b].p);
            free(bodies);
        }
    } else {
        bv_push(&o, FSE_MODE_SINGLE);
        st = fse_compress_single(t, in, n, &o);
    }
    free(t);
    if (st == OK) {
        memcpy(out, o.p, o.n);
        *out_len = o.n;
    }
    free(o.p);
    return st;
}

/* FseTable::renormalize_decode, fse.rs:704-735: after a decoded symbol, while
   fewer than 4 bytes are left one byte is read, else one u32 LE word; the
   state never drops below 1. (The reference's `pos + 4 <= len` guard always
   holds once pos >= 4, so the word is always read.) Returns the new state. */
uint64_t or_fse_renormalize_decode(uint64_t x, const uint8_t *in, size_t len, size_t *pos) {
    if (x < 65536 && *pos > 0) {
        if (*pos >= 4) {
            *pos -= 4;
            x <<= 32;
            if (*pos + 4 <= len) x |= rd_u32(in + *pos); /* fse.rs:722-726: no word read past the input */
        } else {
            *pos -= 1;
            if (*pos >= len) return 0; /* input[*pos] out of bounds: the reference panics (fse.rs:729) */
            x = (x << 8) | in[*pos];
        }
    }
    return x < 1 ? 1 : x;
}

/* decompress_single, fse.rs:1151-1281. Appends to o. */
static int fse_decompress_single(const uint8_t *data, size_t len, bvec *o, size_t out_cap) {
    if (len == 0) return OK;
    if (len < 5) return EINVAL_DATA;
    size_t pos = 0;
    size_t orig = rd_u32(data);
    pos += 4;
    if (orig == 0) return OK;
    uint8_t table_log = data[pos++];
    if (table_log == 0xFF) {
        if (pos + orig > len) return EINVAL_DATA;
        if (o->n + orig > out_cap) return EINVAL_DATA;
        bv_put(o, data + pos, orig);
        return OK;
    }
    if (table_log < 5 || table_log > 15) return EINVAL_DATA;
    if (pos + 2 > len) return EINVAL_DATA;
    size_t nsym = (size_t)data[pos] | ((size_t)data[pos + 1] << 8);
    pos += 2;
    uint32_t freqs[256] = {0};
    for (size_t i = 0; i < nsym; i++) {
        if (pos + 5 > len) return EINVAL_DATA;
        uint8_t s = data[pos];
        freqs[s] = rd_u32(data + pos + 1);
        pos += 5;
    }
    fse_table *t = (fse_table *)malloc(sizeof(fse_table));
    int st = fse_table_new(freqs, t); /* decoder config validated (defaults) */
    if (st) {
        free(t);
        return st;
    }
    if (len < pos + 8) {
        free(t);
        return EINVAL_DATA; /* "Missing final state" */
    }
    size_t state_start = len - 8;
    uint64_t x = rd_u64(data + state_start);
    if (x == 0) x = 1; /* fse.rs:1247-1249 */
    const uint8_t *cd = data + pos;
    size_t bp = state_start - pos;
    if (o->n + orig > out_cap) {
        free(t);
        return EINVAL_DATA;
    }
    bv_reserve(o, o->n + orig);
    for (size_t i = 0; i < orig; i++) {
        /* decode_symbol, fse.rs:664-676 */
        uint32_t lo = (uint32_t)(x & 4095);
        uint8_t s = t->alias[lo];
        x = (uint64_t)t->dfreq[s] * (x >> 12) + lo - t->dstart[s];
        o->p[o->n++] = s;
        x = or_fse_renormalize_decode(x, cd, state_start - pos, &bp);
    }
    free(t);
    return OK;
}

/* FseDecoder::decompress, fse.rs:1105-1148; decompress_parallel fse.rs:1284-1312. */
int or_fse_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap, size_t *out_len) {
    *out_len = 0;
    if (n == 0) return OK;
    uint8_t mode = in[0];
    const uint8_t *body = in + 1;
    size_t blen = n - 1;
    bvec o = {0};
    int st = OK;
    if (mode == FSE_MODE_SINGLE) {
        st = fse_decompress_single(body, blen, &o, out_cap);
    } else if (mode == FSE_MODE_PARALLEL) {
        if (blen < 4) return EINVAL_DATA;
        size_t nb = rd_u32(body);
        if (nb == 0) return EINVAL_DATA;
        if (nb > (blen - 4) / 4) return EINVAL_DATA;
        size_t pos = 4;
        size_t sizes_at = pos;
        pos += 4 * nb; /* block sizes are all present by the check above */
        for (size_t b = 0; b < nb && st == OK; b++) {
            size_t bs = rd_u32(body + sizes_at + 4 * b);
            if (pos + bs > blen) {
                st = EINVAL_DATA;
                break;
            }
            st = fse_decompress_single(body + pos, bs, &o, out_cap);
            pos += bs;
        }
    } else {
        return EINVAL_DATA; /* unknown mode byte */
    }
    if (st == OK) {
        if (o.n > out_cap) st = EINVAL_DATA;
        else {
            if (o.n) memcpy(out, o.p, o.n);
            *out_len = o.n;
        }
    }
    free(o.p);
    return st;
}

static size_t fse_single_size(const uint8_t *d, size_t len) {
    if (len < 5) return 0;
    return rd_u32(d);
}

int or_fse_decompressed_size(const uint8_t *in, size_t n, size_t *out_len) {
    *out_len = 0;
    if (n == 0) return OK;
    if (in[0] == FSE_MODE_SINGLE) {
        *out_len = fse_single_size(in + 1, n - 1);
        return OK;
    }
    if (in[0] != FSE_MODE_PARALLEL || n < 5) return EINVAL_DATA;
    size_t nb = rd_u32(in + 1);
    if (nb == 0 || nb > (n - 5) / 4) return EINVAL_DATA;
    size_t pos = 1 + 4 + 4 * nb, tot = 0;
    for (size_t b = 0; b < nb; b++) {
        size_t bs = rd_u32(in + 5 + 4 * b);
        if (pos + bs > n) return EINVAL_DATA;
        tot += fse_single_size(in + pos, bs);
        pos += bs;
    }
    *out_len = tot;
    return OK;
}

/* ======================================================================== */
/* Huffman O0 -- src/entropy/huffman/tree.rs, encoder.rs, decoder.rs        */
/* ======================================================================== */

/* Rust std BinaryHeap<Reverse<HuffmanNode>> emulation.
 * The element order is: a <= b  <=>  freq(a) <= freq(b)  (tree.rs:35-40 + Reverse),
 * so the heap pops the HIGHEST frequency first. */
typedef struct {
    int32_t data[1024];
    int32_t len;
    const uint32_t *freq; /* node frequencies */
} rheap;
static int rh_le(const rheap *h, int32_t a, int32_t b) { return h->freq[a] <= h->freq[b]; }
static int rh_sift_up(rheap *h, int start, int pos) {
    int32_t elem = h->data[pos];
    while (pos > start) {
        int parent = (pos - 1) / 2;
        if (rh_le(h, elem, h->data[parent])) break;
        h->data[pos] = h->data[parent];
        pos = parent;
    }
    h->data[pos] = elem;
    return pos;
}
static void rh_push(rheap *h, int32_t x) {
    int old = h->len;
    h->data[h->len++] = x;
    rh_sift_up(h, 0, old);
}
static void rh_sift_down_to_bottom(rheap *h, int pos) {
    int end = h->len, start = pos;
    int32_t elem = h->data[pos];
    int child = 2 * pos + 1;
    while (child <= (end >= 2 ? end - 2 : 0) && end >= 2) {
        if (rh_le(h, h->data[child], h->data[child + 1])) child += 1;
        h->data[pos] = h->data[child];
        pos = child;
        child = 2 * pos + 1;
    }
    if (child == end - 1) {
        h->data[pos] = h->data[child];
        pos = child;
    }
    h->data[pos] = elem;
    rh_sift_up(h, start, pos);
}
static int32_t rh_pop(rheap *h) {
    int32_t item = h->data[--h->len];
    if (h->len > 0) {
        int32_t t = h->data[0];
        h->data[0] = item;
        item = t;
        rh_sift_down_to_bottom(h, 0);
    }
    return item;
}

/* decode-tree builder helpers */
static int ht_new_node(or_huff_tree *t, int leaf, int sym) {
    int i = t->n_nodes++;
    t->node_leaf[i] = (uint8_t)leaf;
    t->node_sym[i] = (uint8_t)sym;
    t->node_child[i][0] = t->node_child[i][1] = -1;
    return i;
}

/* generate_codes, tree.rs:187-208 (left = 0, right = 1) over the build tree */
typedef struct {
    int32_t leaf_sym[512];
    int32_t left[512], right[512];
    uint32_t freq[512];
    int n;
} btree;
static void gen_codes(const btree *b, int node, uint64_t code, uint32_t len, or_huff_tree *t,
                      uint32_t *maxlen, int *overflow) {
    if (b->leaf_sym[node] >= 0) {
        if (len > *maxlen) *maxlen = len;
        int s = b->leaf_sym[node];
        t->code_len[s] = (uint8_t)(len > 255 ? 255 : len);
        t->code[s] = code;
        return;
    }
    if (len >= 64) *overflow = 1; /* codes longer than 64 bits cannot be stored; depth>64 path */
    gen_codes(b, b->left[node], code, len + 1, t, maxlen, overflow);
    gen_codes(b, b->right[node], len < 64 ? code | (1ull << len) : code, len + 1, t, maxlen,
              overflow);
}
static int copy_decode_tree(const btree *b, int node, or_huff_tree *t) {
    if (b->leaf_sym[node] >= 0) return ht_new_node(t, 1, b->leaf_sym[node]);
    int me = ht_new_node(t, 0, 0);
    int l = copy_decode_tree(b, b->left[node], t);
    int r = copy_decode_tree(b, b->right[node], t);
    t->node_child[me][0] = (int16_t)l;
    t->node_child[me][1] = (int16_t)r;
    return me;
}

/* insert_code_into_tree, tree.rs:359-469 (placeholder leaves: symbol 0, freq 0) */
static _Thread_local uint8_t ph[1024]; /* placeholder flag per node (per thread: the CPU baseline runs threads) */
static int insert_code(or_huff_tree *t, int node, uint8_t sym, uint64_t code, uint32_t len,
                       uint32_t at) {
    if (at == len) { /* empty code: replace node with a leaf */
        t->node_leaf[node] = 1;
        t->node_sym[node] = sym;
        ph[node] = 0;
        return OK;
    }
    if (t->node_leaf[node]) {
        if (!ph[node]) return EINVAL_DATA; /* "Code collision" */
        /* placeholder -> internal with two placeholder children */
        t->node_leaf[node] = 0;
        ph[node] = 0;
        int a = ht_new_node(t, 1, 0), b = ht_new_node(t, 1, 0);
        ph[a] = ph[b] = 1;
        t->node_child[node][0] = (int16_t)a;
        t->node_child[node][1] = (int16_t)b;
    }
    int bit = (int)((code >> at) & 1);
    return insert_code(t, t->node_child[node][bit], sym, code, len, at + 1);
}

/* from_frequencies_fixed_length, tree.rs:136-175 */
static int huff_fixed(const uint32_t freq[256], or_huff_tree *t) {
    memset(t->code_len, 0, sizeof(t->code_len));
    memset(t->code, 0, sizeof(t->code));
    t->n_nodes = 0;
    int rank = 0;
    for (int s = 0; s < 256; s++)
        if (freq[s] > 0) {
            t->code_len[s] = 8;
            t->code[s] = (uint64_t)rank; /* bits of rank, LSB first */
            rank++;
        }
    t->n_symbols = rank;
    t->max_code_length = 8;
    if (rank == 0) {
        t->kind = 0;
        return OK;
    }
    if (rank == 1) { /* build_decoding_tree_from_codes single-symbol case (tree.rs:325-335) */
        for (int s = 0; s < 256; s++)
            if (freq[s]) ht_new_node(t, 1, s);
        t->kind = 1;
        return OK;
    }
    /* root: internal with two placeholder leaves (tree.rs:338-348) */
    int root = ht_new_node(t, 0, 0);
    int a = ht_new_node(t, 1, 0), b = ht_new_node(t, 1, 0);
    memset(ph, 0, sizeof(ph));
    ph[a] = ph[b] = 1;
    t->node_child[root][0] = (int16_t)a;
    t->node_child[root][1] = (int16_t)b;
    for (int s = 0; s < 256; s++)
        if (t->code_len[s]) {
            int st = insert_code(t, root, (uint8_t)s, t->code[s], 8, 0);
            if (st) return st;
        }
    t->kind = 2;
    return OK;
}

/* HuffmanTree::from_frequencies, tree.rs:52-133 */
int or_huff_tree_build(const uint32_t freq[256], or_huff_tree *t) {
    memset(t, 0, sizeof(*t));
    btree *b = (btree *)calloc(1, sizeof(btree));
    rheap *h = (rheap *)calloc(1, sizeof(rheap));
    h->freq = b->freq;
    int count = 0;
    for (int s = 0; s < 256; s++)
        if (freq[s] > 0) { /* leaves pushed in byte order, tree.rs:59-67 */
            int id = b->n++;
            b->leaf_sym[id] = s;
            b->freq[id] = freq[s];
            b->left[id] = b->right[id] = -1;
            rh_push(h, id);
            count++;
        }
    t->n_symbols = count;
    int st = OK;
    if (count == 0) { /* tree.rs:69-75 */
        t->kind = 0;
    } else if (count == 1) { /* tree.rs:78-90: code [false] */
        int id = rh_pop(h);
        int s = b->leaf_sym[id];
        t->kind = 1;
        t->code_len[s] = 1;
        t->code[s] = 0;
        t->max_code_length = 1;
        ht_new_node(t, 1, s);
    } else {
        while (h->len > 1) { /* tree.rs:93-111 */
            int l = rh_pop(h);
            int r = rh_pop(h);
            int id = b->n++;
            b->leaf_sym[id] = -1;
            b->left[id] = l;
            b->right[id] = r;
            b->freq[id] = b->freq[l] + b->freq[r]; /* u32 add (wraps in release) */
            rh_push(h, id);
        }
        int root = rh_pop(h);
        uint32_t maxlen = 0;
        int overflow = 0;
        gen_codes(b, root, 0, 0, t, &maxlen, &overflow);
        if (maxlen > 64) { /* tree.rs:122-126 */
            st = huff_fixed(freq, t);
        } else {
            t->kind = 2;
            t->max_code_length = maxlen;
            copy_decode_tree(b, root, t);
        }
    }
    free(b);
    free(h);
    return st;
}

size_t or_huff_encode_bound(const or_huff_tree *t, const uint8_t *in, size_t n) {
    uint64_t bits = 0;
    for (size_t i = 0; i < n; i++) bits += t->code_len[in[i]];
    return (size_t)((bits + 7) / 8);
}

/* HuffmanEncoder::encode, encoder.rs:88-131 (codes concatenated, packed LSB-first) */
int or_huff_encode(const or_huff_tree *t, const uint8_t *in, size_t n, uint8_t *out,
                   size_t *out_len) {
    *out_len = 0;
    if (n == 0) return OK;
    uint64_t bitpos = 0;
    for (size_t i = 0; i < n; i++)
        if (t->code_len[in[i]] == 0) return EINVAL_DATA; /* "Symbol {} not in Huffman tree" */
    size_t nbytes = or_huff_encode_bound(t, in, n);
    memset(out, 0, nbytes);
    for (size_t i = 0; i < n; i++) {
        uint32_t L = t->code_len[in[i]];
        uint64_t c = t->code[in[i]];
        for (uint32_t j = 0; j < L; j++, bitpos++)
            if ((c >> j) & 1) out[bitpos >> 3] |= (uint8_t)(1u << (bitpos & 7));
    }
    *out_len = nbytes;
    return OK;
}

/* tree walk of decoder.rs:112-155 / interleaved.rs:1088-1128 (emit on the next bit). */
static size_t huff_walk(const or_huff_tree *t, const uint8_t *in, size_t in_len, uint8_t *out,
                        size_t n) {
    size_t r = 0;
    int cur = 0;
    for (size_t i = 0; i < in_len; i++) {
        uint8_t byte = in[i];
        for (int bp = 0; bp < 8; bp++) {
            if (r >= n) break;
            int bit = (byte >> bp) & 1;
            if (t->node_leaf[cur]) {
                out[r++] = t->node_sym[cur];
                cur = 0;
                if (!t->node_leaf[cur]) cur = t->node_child[cur][bit];
            } else {
                cur = t->node_child[cur][bit];
            }
        }
        if (r >= n) break;
    }
    if (t->node_leaf[cur] && r < n) out[r++] = t->node_sym[cur];
    return r;
}

/* HuffmanDecoder::decode, decoder.rs:90-165 */
/* HuffmanTree::serialize, tree.rs:226-262. The reference walks a HashMap;
 * this restatement writes the symbols in ascending order. out holds
 * 2 + 256 * 10 bytes. */
size_t or_huff_tree_serialize(const or_huff_tree *t, uint8_t *out) {
    size_t o = 2;
    unsigned count = 0;
    for (int s = 0; s < 256; s++) {
        const unsigned L = t->code_len[s];
        if (!L) continue;
        count++;
        out[o++] = (uint8_t)s;
        out[o++] = (uint8_t)L;
        uint8_t cur = 0;
        unsigned bi = 0;
        for (unsigned i = 0; i < L; i++) { /* pack LSB-first (tree.rs:239-256) */
            if ((t->code[s] >> i) & 1) cur |= (uint8_t)(1u << bi);
            if (++bi == 8) {
                out[o++] = cur;
                cur = 0;
                bi = 0;
            }
        }
        if (bi) out[o++] = cur;
    }
    out[0] = (uint8_t)count;
    out[1] = (uint8_t)(count >> 8);
    return o;
}

/* HuffmanTree::deserialize, tree.rs:265-306, and build_decoding_tree_from_codes,
 * tree.rs:311-356. `order` (256 symbols, or NULL = ascending) is the HashMap
 * iteration order the codes are inserted in. Codes over 64 bits are rejected
 * (they do not fit the 64-bit code words of this restatement). */
int or_huff_tree_deserialize(const uint8_t *in, size_t n, const int *order, or_huff_tree *t) {
    memset(t, 0, sizeof(*t));
    if (n < 2) return EINVAL_DATA; /* "Huffman tree data too short" */
    const unsigned count = (unsigned)in[0] | ((unsigned)in[1] << 8);
    uint8_t present[256] = {0};
    size_t o = 2;
    for (unsigned k = 0; k < count; k++) {
        if (o + 2 > n) return EINVAL_DATA; /* "Truncated Huffman tree data" */
        const uint8_t s = in[o], L = in[o + 1];
        o += 2;
        const size_t nb = ((size_t)L + 7) / 8;
        if (o + nb > n) return EINVAL_DATA; /* "Truncated Huffman code data" */
        if (L > 64) return EUNSUP;
        uint64_t c = 0;
        for (unsigned i = 0; i < L; i++) c |= (uint64_t)((in[o + i / 8] >> (i % 8)) & 1) << i;
        present[s] = 1; /* HashMap::insert: a repeated symbol overwrites */
        t->code_len[s] = L;
        t->code[s] = c;
        if (L > t->max_code_length) t->max_code_length = L;
        o += nb;
    }
    int nsym = 0, last = 0;
    for (int s = 0; s < 256; s++)
        if (present[s]) {
            nsym++;
            last = s;
        }
    t->n_symbols = nsym;
    if (nsym == 0) {
        t->kind = 0;
        return OK;
    }
    if (nsym == 1) {
        ht_new_node(t, 1, last);
        t->kind = 1;
        return OK;
    }
    int root = ht_new_node(t, 0, 0);
    int a = ht_new_node(t, 1, 0), b = ht_new_node(t, 1, 0);
    memset(ph, 0, sizeof(ph));
    ph[a] = ph[b] = 1;
    t->node_child[root][0] = (int16_t)a;
    t->node_child[root][1] = (int16_t)b;
    for (int k = 0; k < 256; k++) {
        const int s = order ? order[k] : k;
        if (!present[s]) continue;
        if (t->n_nodes + 2 * (int)t->code_len[s] + 2 > 1024) return EUNSUP;
        int st = insert_code(t, root, (uint8_t)s, t->code[s], t->code_len[s], 0);
        if (st) return st;
    }
    t->kind = 2;
    return OK;
}

int or_huff_decode(const or_huff_tree *t, const uint8_t *in, size_t in_len, uint8_t *out, size_t n,
                   size_t *out_len) {
    *out_len = 0;
    if (in_len == 0 || n == 0) return OK;         /* decoder.rs:91-93 */
    if (t->kind == 0) return EINVAL_DATA;         /* "Empty Huffman tree" */
    if (n / 64 > in_len || (n > in_len * 64)) return EINVAL_DATA; /* implausible, :100-107 */
    size_t r = huff_walk(t, in, in_len, out, n);
    if (r != n) return EINVAL_DATA; /* decoder.rs:157-163 */
    *out_len = r;
    return OK;
}

/* ======================================================================== */
/* Contextual Huffman -- src/entropy/huffman/interleaved.rs                  */
/* ======================================================================== */
struct or_ctx_huff {
    int order;          /* 0, 1, 2 */
    int ntrees;
    or_huff_tree *trees;
    int32_t map1[256];  /* Order-1 context -> tree index, -1 absent */
    int32_t *map2;      /* Order-2 context (65536) -> tree index, -1 absent */
};

static or_ctx_huff *ctx_alloc(int order, int ntrees) {
    or_ctx_huff *c = (or_ctx_huff *)calloc(1, sizeof(or_ctx_huff));
    c->order = order;
    c->ntrees = ntrees;
    c->trees = (or_huff_tree *)calloc(ntrees ? ntrees : 1, sizeof(or_huff_tree));
    for (int i = 0; i < 256; i++) c->map1[i] = -1;
    return c;
}

/* new_order0, interleaved.rs:103-115 */
static or_ctx_huff *ctx_new_o0(const uint8_t *d, size_t n, int *st) {
    uint32_t f[256] = {0};
    for (size_t i = 0; i < n; i++) f[d[i]]++;
    or_ctx_huff *c = ctx_alloc(0, 1);
    *st = or_huff_tree_build(f, &c->trees[0]);
    return c;
}

static void merged_freqs(const uint32_t *cf, const uint32_t *o0, uint32_t *m) {
    for (int s = 0; s < 256; s++) /* interleaved.rs:160-171 */
        m[s] = cf[s] > 0 ? cf[s] * 100 : (o0[s] > 0 ? o0[s] : 1);
}

/* new_order1, interleaved.rs:118-187 */
static or_ctx_huff *ctx_new_o1(const uint8_t *d, size_t n, int *st) {
    if (n < 2) return ctx_new_o0(d, n, st);
    uint32_t o0[256] = {0};
    for (size_t i = 0; i < n; i++) o0[d[i]]++;
    for (int s = 0; s < 256; s++)
        if (o0[s] == 0) o0[s] = 1;
    uint32_t *cf = (uint32_t *)calloc(256 * 256, sizeof(uint32_t));
    uint8_t seen[256] = {0};
    for (size_t i = 1; i < n; i++) {
        cf[d[i - 1] * 256 + d[i]]++;
        seen[d[i - 1]] = 1;
    }
    int nctx = 0;
    for (int c = 0; c < 256; c++) nctx += seen[c];
    or_ctx_huff *c = ctx_alloc(1, 1 + nctx);
    *st = or_huff_tree_build(o0, &c->trees[0]);
    int ti = 1;
    /* HashMap iteration order only affects tree indices, not codes */
    for (int ctx = 0; ctx < 256 && *st == OK; ctx++)
        if (seen[ctx]) {
            uint32_t m[256];
            merged_freqs(&cf[ctx * 256], o0, m);
            *st = or_huff_tree_build(m, &c->trees[ti]);
            c->map1[ctx] = ti++;
        }
    free(cf);
    return c;
}

/* new_order2, interleaved.rs:190-266. Context selection ties follow HashMap
 * order in the reference (nondeterministic); every merged tree holds all 256
 * symbols, so codes do not depend on which contexts were selected. Here ties
 * break by ascending context. */
static or_ctx_huff *ctx_new_o2(const uint8_t *d, size_t n, int *st) {
    if (n < 3) return ctx_new_o1(d, n, st);
    uint32_t o0[256] = {0};
    for (size_t i = 0; i < n; i++) o0[d[i]]++;
    for (int s = 0; s < 256; s++)
        if (o0[s] == 0) o0[s] = 1;
    uint32_t *tot = (uint32_t *)calloc(65536, sizeof(uint32_t));
    for (size_t i = 2; i < n; i++) tot[(d[i - 2] << 8) | d[i - 1]]++;
    int32_t *order = (int32_t *)malloc(65536 * sizeof(int32_t));
    int nctx = 0;
    for (int c = 0; c < 65536; c++)
        if (tot[c]) order[nctx++] = c;
    /* selection sort by descending total, ties by ascending context (the
     * reference's ties follow HashMap order); only the top 1024 are needed */
    int take = nctx < 1024 ? nctx : 1024;
    for (int i = 0; i < take; i++) {
        int best = i;
        for (int j = i + 1; j < nctx; j++)
            if (tot[order[j]] > tot[order[best]] ||
                (tot[order[j]] == tot[order[best]] && order[j] < order[best]))
                best = j;
        int32_t tmp = order[i];
        order[i] = order[best];
        order[best] = tmp;
    }
    or_ctx_huff *c = ctx_alloc(2, 1 + take);
    c->map2 = (int32_t *)malloc(65536 * sizeof(int32_t));
    for (int i = 0; i < 65536; i++) c->map2[i] = -1;
    *st = or_huff_tree_build(o0, &c->trees[0]);
    uint32_t *cf = (uint32_t *)calloc(256, sizeof(uint32_t));
    for (int k = 0; k < take && *st == OK; k++) {
        int ctx = order[k];
        memset(cf, 0, 256 * sizeof(uint32_t));
        for (size_t i = 2; i < n; i++)
            if (((d[i - 2] << 8) | d[i - 1]) == ctx) cf[d[i]]++;
        uint32_t m[256];
        merged_freqs(cf, o0, m);
        *st = or_huff_tree_build(m, &c->trees[1 + k]);
        c->map2[ctx] = 1 + k;
    }
    free(cf);
    free(order);
    free(tot);
    return c;
}

or_ctx_huff *or_ctx_new(const uint8_t *train, size_t n, int order, int *status) {
    int st = OK;
    or_ctx_huff *c = order == 0 ? ctx_new_o0(train, n, &st)
                     : order == 1 ? ctx_new_o1(train, n, &st)
                                  : ctx_new_o2(train, n, &st);
    *status = st;
    return c;
}
void or_ctx_free(or_ctx_huff *c) {
    if (!c) return;
    free(c->trees);
    free(c->map2);
    free(c);
}
int or_ctx_order(const or_ctx_huff *c) { return c->order; }

/* ContextualHuffmanEncoder::serialize, interleaved.rs:476-503. The reference
 * walks its context HashMap and numbers trees in HashMap order; here contexts
 * ascend, context k is listed with tree index k + 1, and the trees follow as
 * trees[0] then the contexts' trees in that order. */
static int ctx_tree_of(const or_ctx_huff *c, int ctx) {
    return c->order == 1 ? c->map1[ctx] : c->map2[ctx];
}
size_t or_ctx_serialize(const or_ctx_huff *c, uint8_t *out) {
    const int nctx_all = c->order == 0 ? 0 : (c->order == 1 ? 256 : 65536);
    uint32_t nctx = 0;
    for (int x = 0; x < nctx_all; x++)
        if (ctx_tree_of(c, x) >= 0) nctx++;
    size_t o = 0;
    out[o++] = (uint8_t)c->order;
    const uint32_t ntrees = 1 + nctx;
    for (int k = 0; k < 4; k++) out[o++] = (uint8_t)(ntrees >> (8 * k));
    for (int k = 0; k < 4; k++) out[o++] = (uint8_t)(nctx >> (8 * k));
    uint32_t idx = 1;
    for (int x = 0; x < nctx_all; x++) {
        if (ctx_tree_of(c, x) < 0) continue;
        for (int k = 0; k < 4; k++) out[o++] = (uint8_t)((uint32_t)x >> (8 * k));
        for (int k = 0; k < 4; k++) out[o++] = (uint8_t)(idx >> (8 * k));
        idx++;
    }
    uint8_t *buf = (uint8_t *)malloc(2 + 256 * 10);
    for (int x = -1; x < nctx_all; x++) {
        const int ti = x < 0 ? 0 : ctx_tree_of(c, x);
        if (ti < 0) continue;
        const size_t ts = or_huff_tree_serialize(&c->trees[ti], buf);
        for (int k = 0; k < 4; k++) out[o++] = (uint8_t)((uint32_t)ts >> (8 * k));
        memcpy(out + o, buf, ts);
        o += ts;
    }
    free(buf);
    return o;
}

static const or_huff_tree *ctx_tree(const or_ctx_huff *c, uint32_t context) {
    int32_t ti = -1;
    if (c->order == 1 && context < 256) ti = c->map1[context];
    if (c->order == 2 && context < 65536) ti = c->map2[context];
    return &c->trees[ti >= 0 ? ti : 0];
}

/* the per-symbol tree choice of encode(), interleaved.rs:269-392 */
static const or_huff_tree *enc_tree_for(const or_ctx_huff *c, const uint8_t *d, size_t i,
                                        int *use_fallback, uint8_t sym) {
    *use_fallback = 0;
    if (c->order == 0) return &c->trees[0];
    size_t warm = c->order == 1 ? 1 : 2;
    if (i < warm) return &c->trees[0];
    uint32_t ctx = c->order == 1 ? d[i - 1] : ((uint32_t)d[i - 2] << 8) | d[i - 1];
    int32_t ti = c->order == 1 ? c->map1[ctx] : c->map2[ctx];
    if (ti >= 0 && c->trees[ti].code_len[sym]) return &c->trees[ti];
    *use_fallback = 1;
    return &c->trees[0];
}

size_t or_ctx_encode_bound(const or_ctx_huff *c, const uint8_t *in, size_t n) {
    uint64_t bits = 0;
    for (size_t i = 0; i < n; i++) {
        int fb;
        bits += enc_tree_for(c, in, i, &fb, in[i])->code_len[in[i]];
    }
    return (size_t)((bits + 7) / 8) + 16 * 8 + 16;
}

int or_ctx_encode(const or_ctx_huff *c, const uint8_t *in, size_t n, uint8_t *out,
                  size_t *out_len) {
    *out_len = 0;
    if (n == 0) return OK;
    uint64_t bitpos = 0;
    size_t cap = or_ctx_encode_bound(c, in, n);
    memset(out, 0, cap);
    for (size_t i = 0; i < n; i++) {
        int fb;
        const or_huff_tree *t = enc_tree_for(c, in, i, &fb, in[i]);
        uint32_t L = t->code_len[in[i]];
        if (L == 0) return EINVAL_DATA;
        for (uint32_t j = 0; j < L; j++, bitpos++)
            if ((t->code[in[i]] >> j) & 1) out[bitpos >> 3] |= (uint8_t)(1u << (bitpos & 7));
    }
    *out_len = (size_t)((bitpos + 7) / 8);
    return OK;
}

/* fast symbol table entry, interleaved.rs:842-884 (codes truncated to 16 bits) */
static void fast_sym(const or_ctx_huff *c, int context, uint8_t sym, uint32_t *bits,
                     uint32_t *cnt) {
    const or_huff_tree *t = context == 256 ? &c->trees[0] : ctx_tree(c, (uint32_t)context);
    if (t->code_len[sym]) {
        uint32_t L = t->code_len[sym];
        *cnt = L < 16 ? L : 16;
        *bits = (uint32_t)(t->code[sym] & 0xFFFF);
    } else {
        *bits = 0;
        *cnt = 1;
    }
}

/* encode_with_interleaving / encode_xn, interleaved.rs:604-761 */
int or_ctx_encode_xn(const or_ctx_huff *c, int N, const uint8_t *in, size_t n, uint8_t *out,
                     size_t *out_len) {
    *out_len = 0;
    if (c->order != 1) return EINVAL_DATA; /* invalid_operation */
    if (n == 0) return OK;
    size_t starts[8], ends[8], pos[8];
    int ctxs[8];
    for (int k = 0; k < N; k++) {
        size_t sz = n / N + ((size_t)k < n % N ? 1 : 0);
        starts[k] = k == 0 ? 0 : ends[k - 1];
        ends[k] = starts[k] + sz;
        pos[k] = starts[k];
        ctxs[k] = 256;
    }
    uint64_t cur = 0;
    uint32_t nb = 0;
    size_t o = 0, done = 0;
    while (done < n) {
        for (int k = 0; k < N; k++) {
            if (pos[k] >= ends[k]) continue;
            uint8_t s = in[pos[k]];
            uint32_t bits, cnt;
            fast_sym(c, ctxs[k], s, &bits, &cnt);
            cur |= (uint64_t)bits << nb; /* BitStreamWriter::write, encoder.rs:44-56 */
            nb += cnt;
            while (nb >= 8) {
                out[o++] = (uint8_t)cur;
                cur >>= 8;
                nb -= 8;
            }
            ctxs[k] = s;
            pos[k]++;
            done++;
        }
    }
    if (nb > 0) out[o++] = (uint8_t)cur;
    *out_len = o;
    return OK;
}

/* BitStreamReader, decoder.rs:6-75 */
typedef struct {
    const uint8_t *d;
    size_t len, bp;
    uint64_t cur;
    uint32_t cnt;
} brd;
static void br_refill(brd *r) {
    while (r->cnt <= 56 && r->bp < r->len) {
        r->cur |= (uint64_t)r->d[r->bp] << r->cnt;
        r->cnt += 8;
        r->bp++;
    }
}

/* decode_one_symbol_tree, interleaved.rs:998-1034 */
static int dec_sym_tree(const or_huff_tree *t, brd *r, uint8_t *sym) {
    if (t->kind == 0) return EINVAL_DATA;
    int cur = 0;
    for (;;) {
        if (t->node_leaf[cur]) {
            *sym = t->node_sym[cur];
            return OK;
        }
        if (r->cnt == 0) {
            br_refill(r);
            if (r->cnt == 0) return EINVAL_DATA; /* "Unexpected end of stream" */
        }
        int bit = (int)(r->cur & 1);
        r->cur >>= 1;
        r->cnt -= 1;
        cur = t->node_child[cur][bit];
    }
}

/* build_decode_table entry for one 12-bit peek value, interleaved.rs:896-935 */
static void dec_table_entry(const or_huff_tree *t, uint32_t peek, uint8_t *sym, uint32_t *used) {
    *sym = 0;
    *used = 0;
    if (t->kind == 0) return;
    int cur = 0;
    uint32_t bits_used = 0;
    for (int bp = 0; bp < 12; bp++) {
        if (t->node_leaf[cur]) {
            *sym = t->node_sym[cur];
            *used = bits_used;
            return;
        }
        cur = t->node_child[cur][(peek >> bp) & 1];
        bits_used++;
    }
    if (t->node_leaf[cur]) {
        *sym = t->node_sym[cur];
        *used = bits_used;
    }
}

/* decode_one_symbol, interleaved.rs:953-995 */
static int dec_one(const or_ctx_huff *c, brd *r, int context, uint8_t *sym) {
    const or_huff_tree *t = context == 256 ? &c->trees[0] : ctx_tree(c, (uint32_t)context);
    if (r->cnt < 12) br_refill(r);
    if (r->cnt < 12) return dec_sym_tree(t, r, sym);
    uint32_t peek = (uint32_t)(r->cur & 0xFFF), used;
    uint8_t s;
    dec_table_entry(t, peek, &s, &used);
    if (used == 0) return dec_sym_tree(t, r, sym);
    if (r->cnt < used) return dec_sym_tree(t, r, sym);
    r->cur >>= used;
    r->cnt -= used;
    br_refill(r);
    *sym = s;
    return OK;
}

/* decode_with_interleaving / decode_xn, interleaved.rs:628-822 */
int or_ctx_decode_xn(const or_ctx_huff *c, int N, const uint8_t *in, size_t in_len, uint8_t *out,
                     size_t n, size_t *out_len) {
    *out_len = 0;
    if (c->order != 1) return EINVAL_DATA;
    if (in_len == 0) return OK; /* interleaved.rs:767-769 */
    brd r = {in, in_len, 0, 0, 0};
    br_refill(&r);
    size_t starts[8], ends[8], pos[8];
    int ctxs[8];
    for (int k = 0; k < N; k++) {
        size_t sz = n / N + ((size_t)k < n % N ? 1 : 0);
        starts[k] = k == 0 ? 0 : ends[k - 1];
        ends[k] = starts[k] + sz;
        pos[k] = starts[k];
        ctxs[k] = 256;
    }
    memset(out, 0, n);
    size_t done = 0;
    while (done < n) {
        for (int k = 0; k < N; k++) {
            if (pos[k] >= ends[k]) continue;
            uint8_t s;
            int st = dec_one(c, &r, ctxs[k], &s);
            if (st) return st;
            out[pos[k]] = s;
            ctxs[k] = s;
            pos[k]++;
            done++;
            if (done >= n) break;
        }
    }
    *out_len = n;
    return OK;
}

/* decode_next_symbol, interleaved.rs:1212-1251 */
static int dec_next(const or_huff_tree *t, const uint8_t *d, size_t len, size_t *bi, int *bp,
                    uint8_t *sym) {
    if (t->kind == 0) return EINVAL_DATA;
    int cur = 0;
    while (*bi < len) {
        uint8_t byte = d[*bi];
        while (*bp < 8) {
            int bit = (byte >> *bp) & 1;
            if (t->node_leaf[cur]) {
                *sym = t->node_sym[cur];
                return OK;
            }
            cur = t->node_child[cur][bit];
            *bp += 1;
        }
        *bp = 0;
        *bi += 1;
    }
    if (t->node_leaf[cur]) {
        *sym = t->node_sym[cur];
        return OK;
    }
    return EINVAL_DATA; /* "Incomplete symbol" */
}

/* ContextualHuffmanDecoder::decode, interleaved.rs:1050-1209 */
int or_ctx_decode(const or_ctx_huff *c, const uint8_t *in, size_t in_len, uint8_t *out, size_t n,
                  size_t *out_len) {
    *out_len = 0;
    if (in_len == 0 || n == 0) return OK;
    size_t r = 0;
    if (c->order == 0) {
        if (c->trees[0].kind == 0) return EINVAL_DATA;
        r = huff_walk(&c->trees[0], in, in_len, out, n);
    } else {
        size_t bi = 0;
        int bp = 0;
        uint8_t s;
        size_t warm = c->order == 1 ? 1 : (n < 2 ? n : 2);
        for (size_t k = 0; k < warm; k++) {
            if (dec_next(&c->trees[0], in, in_len, &bi, &bp, &s) == OK) out[r++] = s;
            else break;
        }
        /* (the reference would index an empty result here; such inputs cannot
         * reach this loop because a failed first decode exhausts the input) */
        while (r < n && bi < in_len && r >= (size_t)c->order) {
            uint32_t ctx = c->order == 1 ? out[r - 1] : ((uint32_t)out[r - 2] << 8) | out[r - 1];
            if (dec_next(ctx_tree(c, ctx), in, in_len, &bi, &bp, &s) == OK) out[r++] = s;
            else break;
        }
    }
    if (r != n) return EINVAL_DATA; /* "Decoded length {} != expected {}" */
    *out_len = r;
    return OK;
}

/* ======================================================================== */
/* record groups (bench.py's configs[4] CPU baseline)                        */
/* ======================================================================== */
/* Each of n_rec records of rec_len bytes at in + r*rec_len: Rans64Encoder::<X1>
 * encode (rans.rs:354-366) then decode (rans.rs:523-552) with the one shared
 * table, the round trip checked; the per-record codec RansBlobStore /
 * RansCompressor run (compression/mod.rs:456-517). One call per record group,
 * so a caller's threads do not meet on the interpreter lock per record.
 * *enc_total = the records' encoded bytes. -1 if any record fails to round-trip. */
int or_rans_x1_records(const or_rans_table *t, const uint8_t *in, size_t n_rec, size_t rec_len,
                       size_t *enc_total) {
    size_t cap = or_rans_encode_bound(rec_len, 1);
    uint8_t *enc = (uint8_t *)malloc(cap ? cap : 1), *dec = (uint8_t *)malloc(rec_len ? rec_len : 1);
    size_t tot = 0;
    int st = (enc && dec) ? OK : -2;
    for (size_t r = 0; st == OK && r < n_rec; r++) {
        const uint8_t *d = in + r * rec_len;
        size_t el = 0;
        st = or_rans_encode(t, 1, d, rec_len, enc, &el);
        if (st == OK) st = or_rans_decode(t, 1, enc, el, dec, rec_len);
        if (st == OK && memcmp(dec, d, rec_len) != 0) st = EINVAL_DATA;
        tot += el;
    }
    free(enc);
    free(dec);
    if (enc_total) *enc_total = tot;
    return st;
}

/* ======================================================================== */
/* inputs                                                                    */
/* ======================================================================== */
void or_gen_uniform(uint64_t seed, uint8_t *out, size_t n) { /* tests/fse_tests.rs:711-717 */
    uint64_t s = seed;
    for (size_t i = 0; i < n; i++) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        out[i] = (uint8_t)(s >> 32);
    }
}
