/*
 * zr_oracle.h -- CPU restatement of infinilabs/zipora src/entropy (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity oracle. It is linked/loaded ONLY by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg. The product
 * (zipora_amd/, libzipora_amd.so) never links or calls it.
 *
 * Parity pinning: the reference is Rust and no Rust toolchain exists in this
 * image, so the reference cannot be built or run here. This
 * restatement is pinned by the hand-derived known-answer vectors of SURVEY.md
 * Appendix B (B1..B14) and by the reference's own exact asserts
 * (rans.rs:734-809, huffman/tests.rs:8-29 and :630-705, decoder.rs:175-185,
 * tests/fse_tests.rs:822-830); see tests/test_oracle_kats.py.
 *
 * All buffers are caller-owned. Return codes mirror the reference's
 * Result<_, ZiporaError>: 0 = Ok, -1 = InvalidData/InvalidParameter.
 */
#ifndef ZR_ORACLE_H
#define ZR_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- rANS (src/entropy/rans.rs) ---- */
typedef struct {
    uint32_t freq[256];  /* normalised, sum 4096 (or all 0 when total_freq == 0) */
    uint32_t start[256];
    uint32_t total_freq; /* 4096, or 0 for the empty encoder (rans.rs:209-216) */
} or_rans_table;

/* Rans64Encoder::<P>::new (rans.rs:208-235). */
int or_rans_table_build(const uint32_t raw[256], or_rans_table *t);
/* Rans64Encoder::encode (rans.rs:338-420) with runtime P::N = n_streams.
 * out must hold or_rans_encode_bound(n, n_streams) bytes. */
size_t or_rans_encode_bound(size_t n, uint32_t n_streams);
int or_rans_encode(const or_rans_table *t, uint32_t n_streams, const uint8_t *in, size_t n,
                   uint8_t *out, size_t *out_len);
/* Rans64Decoder::decode (rans.rs:510-651). */
/* The same two calls with the reference's data structures (per-stream index
 * vectors, Vec growth) -- bench.py's single-thread CPU baseline. */
int or_rans_encode_mirror(const or_rans_table *t, uint32_t n_streams, const uint8_t *in, size_t n,
                          uint8_t *out, size_t *out_len);
int or_rans_decode_mirror(const or_rans_table *t, uint32_t n_streams, const uint8_t *in, size_t in_len,
                          uint8_t *out, size_t n);
int or_rans_decode(const or_rans_table *t, uint32_t n_streams, const uint8_t *in, size_t in_len,
                   uint8_t *out, size_t n);

/* ---- FSE (src/entropy/fse.rs) ---- */
typedef struct {
    uint32_t table_log;        /* 5..15 (validated; coding always uses 12) */
    int32_t compression_level; /* 1..22 */
    uint64_t max_table_size;
    uint64_t parallel_blocks;  /* 0 = None, k = Some(k) */
    uint64_t block_size;
    int32_t adaptive;          /* only affects table reuse, always recomputed here */
} or_fse_config;
void or_fse_config_default(or_fse_config *c);               /* fse.rs:245-263 */
int or_fse_normalize_exact(const uint32_t f[256], uint32_t table_size, uint32_t out[256]);
size_t or_fse_compress_bound(size_t n, const or_fse_config *c);
int or_fse_compress(const or_fse_config *c, const uint8_t *in, size_t n, uint8_t *out,
                    size_t *out_len);                        /* FseEncoder::compress fse.rs:854 */
/* compress with a caller-given raw frequency table: the static-table path
 * (adaptive=false reuses the first table, fse.rs:860-862) and dictionaries
 * (dictionary byte counts added, fse.rs:807-812). freqs == NULL: histogram of in. */
int or_fse_compress_freqs(const or_fse_config *c, const uint32_t *freqs, const uint8_t *in, size_t n,
                          uint8_t *out, size_t *out_len);
/* FseDecoder::decompress fse.rs:1105. out_cap bounds the output; *out_len = produced. */
int or_fse_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap, size_t *out_len);
/* Decoded length of a stream without decoding (host-side sizing helper). */
int or_fse_decompressed_size(const uint8_t *in, size_t n, size_t *out_len);
/* The portable mul_hi of fse.rs:618-628 (wrapping middle sum). */
uint64_t or_fse_mul_hi(uint64_t a, uint64_t b);
/* FseTable::renormalize_decode, fse.rs:704-735 (pos moves down; returns the state;
 * a word position past len shifts without a read, as fse.rs:722; returns 0
 * where the reference's one-byte read would index past the input and panic) */
uint64_t or_fse_renormalize_decode(uint64_t x, const uint8_t *in, size_t len, size_t *pos);

/* ---- Huffman O0 (src/entropy/huffman/{tree,encoder,decoder}.rs) ---- */
typedef struct {
    int32_t kind;          /* 0 empty, 1 single leaf, 2 tree */
    int32_t n_symbols;
    uint32_t max_code_length;
    uint8_t code_len[256]; /* 0 = symbol not in tree */
    uint64_t code[256];    /* code bits, bit i = i-th emitted bit (LSB-first) */
    /* decode tree: node 0 is the root; node i: is_leaf, symbol, child[0/1] */
    int32_t n_nodes;
    uint8_t node_leaf[1024];
    uint8_t node_sym[1024];
    int16_t node_child[1024][2];
} or_huff_tree;
int or_huff_tree_build(const uint32_t freq[256], or_huff_tree *t); /* tree.rs:52-133 */
size_t or_huff_encode_bound(const or_huff_tree *t, const uint8_t *in, size_t n);
int or_huff_encode(const or_huff_tree *t, const uint8_t *in, size_t n, uint8_t *out,
                   size_t *out_len);                                /* encoder.rs:88-131 */
int or_huff_decode(const or_huff_tree *t, const uint8_t *in, size_t in_len, uint8_t *out,
                   size_t n, size_t *out_len);                      /* decoder.rs:90-165 */

size_t or_huff_tree_serialize(const or_huff_tree *t, uint8_t *out);          /* tree.rs:226-262 */
int or_huff_tree_deserialize(const uint8_t *in, size_t n, const int *order,
                             or_huff_tree *t);                             /* tree.rs:265-356 */

/* ---- Contextual Huffman O1/O2 (src/entropy/huffman/interleaved.rs) ---- */
typedef struct or_ctx_huff or_ctx_huff;
or_ctx_huff *or_ctx_new(const uint8_t *train, size_t n, int order, int *status);
void or_ctx_free(or_ctx_huff *c);
int or_ctx_order(const or_ctx_huff *c);
/* ContextualHuffmanEncoder::serialize (interleaved.rs:476-503), canonical order;
 * out holds 9 + 8 * 65536 + 65537 * (4 + 2562) bytes at most */
size_t or_ctx_serialize(const or_ctx_huff *c, uint8_t *out);
size_t or_ctx_encode_bound(const or_ctx_huff *c, const uint8_t *in, size_t n);
int or_ctx_encode(const or_ctx_huff *c, const uint8_t *in, size_t n, uint8_t *out, size_t *out_len);
int or_ctx_encode_xn(const or_ctx_huff *c, int nway, const uint8_t *in, size_t n, uint8_t *out,
                     size_t *out_len);
int or_ctx_decode(const or_ctx_huff *c, const uint8_t *in, size_t in_len, uint8_t *out, size_t n,
                  size_t *out_len);
int or_ctx_decode_xn(const or_ctx_huff *c, int nway, const uint8_t *in, size_t in_len, uint8_t *out,
                     size_t n, size_t *out_len);

/* ---- record groups: x1 encode+decode of n_rec records of rec_len bytes with
 * one table, round trip checked; *enc_total = encoded bytes (bench CPU leg) ---- */
int or_rans_x1_records(const or_rans_table *t, const uint8_t *in, size_t n_rec, size_t rec_len,
                       size_t *enc_total);

/* ---- deterministic inputs ---- */
void or_gen_uniform(uint64_t seed, uint8_t *out, size_t n); /* tests/fse_tests.rs:711-717 */

#ifdef __cplusplus
}
#endif
#endif
