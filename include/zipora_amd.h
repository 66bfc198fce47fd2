/*
 * zipora_amd.h -- C ABI of the MI355X-native entropy-coding backend for zipora.
 *
 * Drop-in boundary for the reference's src/entropy Rust surface.
 * The reference has no entropy entry points in its C API (src/ffi/c_api.rs:84-608),
 * so each function below names the Rust method it replaces; INTEGRATION.md shows
 * the `extern "C"` block a maintainer adds on the Rust side.
 *
 * Conventions copied from src/ffi:
 *   - int32 status codes mirror CResult (src/ffi/mod.rs:29-58);
 *   - thread-local last error string (src/ffi/c_api.rs:17-42) and an optional
 *     error callback (src/ffi/c_api.rs:22);
 *   - no C++ exception crosses the ABI (the catch_unwind guard of c_api.rs:61-76).
 * Buffers are caller-owned. Functions without the _dev suffix take HOST memory
 * and are synchronous (they return the codec status like the Rust Result).
 * They are thread-safe: each call leases a per-device call context (its own
 * non-blocking HIP stream and cached device buffers) and synchronises only that
 * stream, never the device: a buffer that must grow is freed and re-allocated
 * stream-ordered on the context's stream (hipFreeAsync / hipMallocAsync).
 * Buffers up to 1 GiB stay cached in the context (nothing is allocated once the
 * sizes a workload needs have been seen, zr_device_alloc_count); larger ones
 * are returned when the call ends. zr_release_call_contexts() frees every idle
 * context and trims the devices' memory pools.
 * Functions with the _dev suffix take DEVICE memory, are ordered on the given
 * HIP stream (hipStream_t passed as void*, NULL = default stream) and report
 * per-buffer status into a device int32 array; read it after synchronising.
 * Graph capture: zr_rans_encode/decode_batch_dev, zr_histogram_dev,
 * zr_rans_dtab_from_hist*_dev, zr_rans_dtab_from_data_dev and the RCCL calls
 * may be captured into a HIP graph and replayed (they keep no host-side state;
 * zr_rans_dtab_from_data_dev keeps the ticket slot it was captured with, so
 * replays of one such graph must not run concurrently with each other). Every
 * other _dev call returns ZR_UNSUPPORTED on a capturing stream:
 * zr_rans_dtab_upload and zr_huff_decode_dev stage host data through memory a
 * host callback frees, and zr_huff_encode_dev, zr_fse_compress_dev, zr_fse_decompress_dev,
 * zr_ctx_huff_encode_dev, zr_ctx_huff_decode_dev and the
 * zr_rans_compressor_*_batch_dev calls are not capture-validated.
 */
#ifndef ZIPORA_AMD_H
#define ZIPORA_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (src/ffi/mod.rs:29-58) ---- */
#define ZR_OK 0
#define ZR_INVALID_INPUT (-1) /* ZiporaError::InvalidData / InvalidParameter (error.rs:139) */
#define ZR_MEMORY_ERROR (-2)
#define ZR_UNSUPPORTED (-4)
#define ZR_INTERNAL (-5)

typedef void (*zr_error_cb)(int32_t code, const char *message);

const char *zr_last_error(void);               /* c_api.rs:17-42 */
void zr_set_error_callback(zr_error_cb cb);    /* c_api.rs:22 */
const char *zr_version(void);
int32_t zr_device_count(int32_t *count);
int32_t zr_set_device(int32_t device);         /* binds this host thread to a GPU */
/* frees the idle call contexts of the host entry points (their cached device
 * buffers and streams) and trims the default memory pools */
int32_t zr_release_call_contexts(void);

/* ======================================================================
 * rANS order-0 -- src/entropy/rans.rs
 * ====================================================================== */
typedef struct {
    uint32_t freq[256];  /* normalised frequencies (sum 4096) -- Rans64Symbol::freq */
    uint32_t start[256]; /* cumulative starts -- Rans64Symbol::start */
    uint32_t total_freq; /* 4096, or 0 for the empty encoder (rans.rs:209-216) */
} zr_rans_table;

/* Rans64Encoder::<P>::new(&[u32;256]) -> Result<Self>           rans.rs:208-235 */
int32_t zr_rans_table_build(const uint32_t raw_freq[256], zr_rans_table *out);
/* upper bound of Rans64Encoder::encode output for n bytes and P::N = n_streams */
size_t zr_rans_encode_bound(size_t n, uint32_t n_streams);
/* Rans64Encoder::<P>::encode(&self, &[u8]) -> Result<Vec<u8>>    rans.rs:338-420
 * P::N is the runtime n_streams (rans::ParallelVariant::N, rans.rs:165-168). */
int32_t zr_rans_encode(const zr_rans_table *t, uint32_t n_streams, const uint8_t *in, size_t n,
                       uint8_t *out, size_t out_cap, size_t *out_len);
/* Rans64Decoder::<P>::new(&enc).decode(&self, &[u8], usize)      rans.rs:449-651 */
int32_t zr_rans_decode(const zr_rans_table *t, uint32_t n_streams, const uint8_t *in,
                       size_t in_len, uint8_t *out, size_t n);
/* AdaptiveRans64Encoder::select_variant (rans.rs:669-681): P::N = 1, 2, 4 or 8
 * for data sizes < 73, < 73^2, < 73^4, else */
uint32_t zr_rans_adaptive_streams(size_t data_size);
/* AdaptiveRans64Encoder::encode_adaptive (rans.rs:684-714): histogram of in,
 * Rans64Encoder::<P>::new, encode with P from select_variant; *n_streams
 * (optional) receives the P::N used, which the decoder needs */
int32_t zr_rans_encode_adaptive(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap, size_t *out_len,
                                uint32_t *n_streams);
/* Exhaustive check of the encoder's reciprocal division on the device (the
 * analogue of the reference's fast_div test, rans.rs:786-809): for every
 * freq 1..4096 and every x < 2^24, umulhi(x << 8, rcp) >> rsh == x / freq.
 * *mismatches receives the number of failures (0 expected). Synchronous. */
int32_t zr_rans_selftest_reciprocal(uint64_t *mismatches);
/* Rans64Symbol::new(start, freq).fast_div(x) -> (x / freq, x % freq)
 * (rans.rs:89-152, the pub symbol info of Rans64Encoder::get_symbol, rans.rs:423)
 * for n dividends, computed on the device by the encoder's 24-bit reciprocal
 * division for x < 2^24 (every state the coder holds, freq <= 4096) and by
 * 64-bit division otherwise. Any u32 freq: freq 0 gives (0, 0) as the
 * reference's early return does (rans.rs:138-140), every other freq the exact
 * quotient and remainder. Host arrays; synchronous. */
int32_t zr_rans_symbol_fast_div(uint32_t start, uint32_t freq, const uint64_t *x, size_t n, uint64_t *q,
                                uint64_t *r);
/* Diagnostic (no reference counterpart): the number of streams / records the
 * fast device decoders handed to their generic per-lane loop on the current
 * device since the last reset (a lane whose reads outran its LDS ring, a state
 * outside [2^16, 2^24), a table that is not normal). Waits for the device;
 * reset != 0 zeroes the counter after reading it. */
int32_t zr_rans_fallback_lanes(uint64_t *count, int32_t reset);

/* ---- device-resident batch pipeline (the GPU hot path) ----
 * A batch is B independent buffers, each coded as one reference rANS stream
 * set with P::N = n_streams. Every array below is DEVICE memory.
 *   raw_off[b], len[b] : buffer b's raw bytes live at raw + raw_off[b], len[b] bytes
 *   enc_off[b]         : buffer b's encoded bytes live at enc + enc_off[b]
 *   enc_len[b]         : encoded length (written by encode, read by decode)
 *   status[b]          : ZR_OK or ZR_INVALID_INPUT (written by both)
 * Tables are device tables (zr_rans_dtab_bytes() each); table_stride is 0 when
 * every buffer shares table 0, 1 when buffer b uses table b. min_len is a
 * host-side lower bound of the lengths (0 = unknown): when it is >= n_streams
 * > 1 no buffer takes the x1 layout and its kernels are not launched. */
typedef struct {
    uint32_t n_buffers;
    uint32_t n_streams;
    uint64_t max_len;        /* >= every len[b]; sizes scratch and grids */
    const uint64_t *len;
    const uint64_t *raw_off;
    const uint64_t *enc_off;
    uint64_t *enc_len;
    int32_t *status;
    const void *tables;
    uint32_t table_stride;
    uint64_t min_len;
} zr_rans_batch;

size_t zr_rans_dtab_bytes(void);
/* upload host tables (Rans64Encoder::new results) as device tables */
int32_t zr_rans_dtab_upload(const zr_rans_table *tables, uint32_t n_tables, void *dtabs_dev,
                            void *stream);
/* Upload is stream-ordered: the host tables may be freed on return. */
/* device histograms: per buffer (shared = 0, hist_dev has B x 256 u32) or one
 * histogram of the whole batch (shared = 1). Accumulates: zero hist_dev first
 * (zr_memset_dev). The callers this replaces count bytes on the CPU:
 * RansCompressor::new (compression/mod.rs:433-450), RansBlobStore::train
 * (blob_store/entropy.rs:212-219), AdaptiveRans64Encoder (rans.rs:708-714). */
int32_t zr_histogram_dev(const uint8_t *raw, const zr_rans_batch *batch, int32_t shared,
                         uint32_t *hist_dev, void *stream);
/* Rans64Encoder::new on device, one table per histogram (no host round trip) */
int32_t zr_rans_dtab_from_hist_dev(const uint32_t *hist_dev, uint32_t n_tables, void *dtabs_dev,
                                   void *stream);
/* the same, then zeroes the histograms it read (stream-ordered), so the next
 * accumulating zr_histogram_dev into them needs no zr_memset_dev */
int32_t zr_rans_dtab_from_hist_consume_dev(uint32_t *hist_dev, uint32_t n_tables, void *dtabs_dev,
                                           void *stream);
/* the shared table of a whole batch in ONE launch: the histogram of every byte
 * of the batch (zr_histogram_dev, shared = 1) and, in its last workgroup, the
 * table (Rans64Encoder::new, rans.rs:208-235) into dtab_dev (one table). The
 * RansBlobStore::train / RansCompressor::new path of a single GPU
 * (blob_store/entropy.rs:212-222, compression/mod.rs:433-450). hist_dev: 256
 * u32, all zero on entry, left all zero (the counts are consumed). Each call
 * picks its workgroups' ticket counters by a host-side call counter, slot
 * (call number % 64). Limit: fewer than 64 calls of this function may be
 * executing at once in the process (calls queued on one stream run one after
 * another and never share a slot; 64 or more concurrent streams each running
 * one could pair two calls on a slot, and a table would then be built before
 * its histogram is complete). Capturable: a captured call keeps its slot in
 * every replay, so replays of one graph must not overlap each other (replays
 * on one stream never do). */
int32_t zr_rans_dtab_from_data_dev(const uint8_t *raw, const zr_rans_batch *batch, uint32_t *hist_dev,
                                   void *dtab_dev, void *stream);
/* The name of the xN decode kernel a batch of n_buffers x n_streams (every
 * buffer at least n_streams bytes) runs (reports and profiles; a static
 * string). No codec setting is process-wide: a call's kernels depend only on
 * its batch geometry. */
const char *zr_rans_decoder_kernel(uint32_t n_buffers, uint32_t n_streams);
/* bytes of device workspace needed by encode/decode of this batch geometry.
 * Workspace contract: scratch owned by one call at a time (calls that share a
 * workspace must be ordered, e.g. on one stream); its content before a call
 * is never read as input, so it needs no initialisation and any content
 * (garbage, another geometry's arrays) gives the same results and statuses. */
size_t zr_rans_workspace_bytes(uint32_t n_buffers, uint32_t n_streams, uint64_t max_len);
/* batched Rans64Encoder::encode: raw -> enc (enc + enc_off[b] must hold
 * zr_rans_encode_bound(len[b], n_streams) bytes) */
int32_t zr_rans_encode_batch_dev(const zr_rans_batch *batch, const uint8_t *raw, uint8_t *enc,
                                 void *workspace, size_t workspace_bytes, void *stream);
/* batched Rans64Decoder::decode: enc -> raw. status[b] is set for every
 * buffer: the call first clears the statuses to ZR_OK (stream-ordered, 4 B per
 * buffer) and its kernels store ZR_INVALID_INPUT for a buffer whose header,
 * stream lengths or renormalisation reads are invalid (rans.rs:480-482,
 * :563-568, :601-610). */
int32_t zr_rans_decode_batch_dev(const zr_rans_batch *batch, const uint8_t *enc, uint8_t *raw,
                                 void *workspace, size_t workspace_bytes, void *stream);

/* ---- RansCompressor record format (compression/mod.rs:416-512) ----
 * record = 256 x u32 LE normalised freqs | u32 LE size | x1 stream; empty <-> empty.
 * decompress re-normalises the stored frequencies with Rans64Encoder::new, as the
 * reference does (mod.rs:514; not the identity for skewed tables). */
/* RansCompressor::new(training_data): histogram + Rans64Encoder::new   mod.rs:425-452 */
int32_t zr_rans_compressor_train(const uint8_t *train, size_t n, zr_rans_table *out);
/* record slot size for n input bytes (header + x1 bound) */
size_t zr_rans_compressor_bound(size_t n);
/* Compressor::compress                                                  mod.rs:457-477 */
int32_t zr_rans_compressor_compress(const zr_rans_table *t, const uint8_t *in, size_t n, uint8_t *out,
                                    size_t out_cap, size_t *out_len);
/* the stored original size of a record (0 for an empty record) */
int32_t zr_rans_compressor_decompressed_size(const uint8_t *in, size_t n, size_t *size);
/* Compressor::decompress                                                mod.rs:479-516 */
int32_t zr_rans_compressor_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                                      size_t *out_len);
/* device batches of records (blob-store put/get): x1, one compressor per batch.
 * compress: tables = the compressor's device table, enc + enc_off[b] holds
 * zr_rans_compressor_bound(len[b]) bytes, enc_len[b] = record length.
 * decompress: the table is rebuilt on device from the first non-empty record's
 * stored frequencies; len[b] must equal the stored size; a record whose stored
 * table differs from that one gets ZR_UNSUPPORTED. */
size_t zr_rans_compressor_workspace_bytes(uint32_t n_buffers, uint64_t max_len);
int32_t zr_rans_compressor_compress_batch_dev(const zr_rans_batch *batch, const uint8_t *raw, uint8_t *enc,
                                              void *workspace, size_t workspace_bytes, void *stream);
int32_t zr_rans_compressor_decompress_batch_dev(const zr_rans_batch *batch, const uint8_t *enc, uint8_t *raw,
                                                void *workspace, size_t workspace_bytes, void *stream);

/* ---- host-resident batches (blob-store records, file buffers) ----
 * The same batch coding with every array in HOST memory: buffers are cut into
 * groups of whole buffers (<= group_bytes raw bytes, 0 = 32 MiB) that stream
 * through two device slots, so one group's host-to-device copy, the previous
 * group's coding and the one before's copy back overlap. One shared table
 * (the RansBlobStore / RansCompressor case: blob_store/entropy.rs:203-260,
 * compression/mod.rs:433-470). Offsets are those of the device batch API;
 * enc + enc_off[b] must hold zr_rans_encode_bound(len[b], n_streams) bytes on
 * encode. Pin the host areas (zr_host_register) for the full PCIe rate. */
typedef struct zr_rans_pipe zr_rans_pipe;
int32_t zr_rans_pipe_create(const zr_rans_table *table, uint32_t n_streams, uint64_t group_bytes,
                            zr_rans_pipe **out);
int32_t zr_rans_pipe_destroy(zr_rans_pipe *pipe);
int32_t zr_rans_pipe_encode(zr_rans_pipe *pipe, uint32_t n_buffers, const uint64_t *len,
                            const uint8_t *raw, const uint64_t *raw_off, uint8_t *enc,
                            const uint64_t *enc_off, uint64_t *enc_len, int32_t *status);
/* encode into a packed host layout (records back to back, the ZipOffset
 * content area): enc_off[b] and enc_len[b] are outputs, enc_total the bytes
 * written; enc_cap >= the sum of zr_rans_encode_bound(len[b]). Only the
 * encoded bytes cross PCIe. Failed buffers get status != 0 and length 0. */
int32_t zr_rans_pipe_encode_packed(zr_rans_pipe *pipe, uint32_t n_buffers, const uint64_t *len,
                                   const uint8_t *raw, const uint64_t *raw_off, uint8_t *enc,
                                   size_t enc_cap, uint64_t *enc_off, uint64_t *enc_len,
                                   int32_t *status, uint64_t *enc_total);
int32_t zr_rans_pipe_decode(zr_rans_pipe *pipe, uint32_t n_buffers, const uint64_t *len,
                            const uint8_t *enc, const uint64_t *enc_off, const uint64_t *enc_len,
                            uint8_t *raw, const uint64_t *raw_off, int32_t *status);
/* page-lock / unlock a host range for asynchronous copies */
int32_t zr_host_register(void *ptr, size_t bytes);
int32_t zr_host_unregister(void *ptr);

/* ======================================================================
 * FSE (rANS with 32-bit renormalisation words) -- src/entropy/fse.rs
 * Stream formats (Appendix A): 0xF5 single | 0xF6 nblocks sizes bodies.
 * ====================================================================== */
typedef struct {
    uint32_t table_log;        /* FseConfig::table_log, validated 5..15 (coding uses 12, fse.rs:424-426) */
    int32_t compression_level; /* 1..22 */
    uint64_t max_table_size;
    uint64_t parallel_blocks;  /* 0 = None, k = Some(k) */
    uint64_t block_size;
    int32_t adaptive;
} zr_fse_config;               /* FseConfig, fse.rs:204-263 */

void zr_fse_config_default(zr_fse_config *c);                     /* FseConfig::default */
size_t zr_fse_compress_bound(size_t n, const zr_fse_config *c);
/* FseEncoder::new(config)?.compress(data)              fse.rs:773, :854-884 */
int32_t zr_fse_compress(const zr_fse_config *c, const uint8_t *in, size_t n, uint8_t *out,
                        size_t out_cap, size_t *out_len);
/* FseDecoder::new().decompress(data)                    fse.rs:1084, :1105-1312 */
int32_t zr_fse_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                          size_t *out_len);
/* FseEncoder::compress with a caller-given raw frequency table: the static
 * table kept when adaptive=false (fse.rs:860-862) and with_dictionary's added
 * dictionary counts (fse.rs:807-812). freqs == NULL: histogram of in. */
int32_t zr_fse_compress_freqs(const zr_fse_config *c, const uint32_t *freqs, const uint8_t *in,
                              size_t n, uint8_t *out, size_t out_cap, size_t *out_len);
/* FSE as the PA-Zip second stage (dict_zip/compression_types.rs:2272-2340):
 * apply = "UN" | raw below 32 bytes or when FSE does not shrink, else
 * "FS" | FseCompressor::compress; remove inverts it ("UN", "FS", or no magic =
 * the whole input is an FSE stream; < 2 bytes pass through). The config is
 * dict_zip's (parallel_blocks None, 64 KiB blocks/tables, :2107-2123). */
size_t zr_pazip_fse_bound(size_t n, const zr_fse_config *c);
int32_t zr_pazip_fse_apply(const zr_fse_config *c, const uint8_t *in, size_t n, uint8_t *out,
                           size_t out_cap, size_t *out_len);
int32_t zr_pazip_fse_removed_size(const uint8_t *in, size_t n, size_t *size);
int32_t zr_pazip_fse_remove(const zr_fse_config *c, const uint8_t *in, size_t n, uint8_t *out,
                            size_t out_cap, size_t *out_len);
/* analyze_frequencies' byte histogram (fse.rs:796-851) on the device */
int32_t zr_byte_histogram(const uint8_t *in, size_t n, uint32_t freqs[256]);
/* decoded length of a stream (parses the framing on the host) */
int32_t zr_fse_decompressed_size(const uint8_t *in, size_t n, size_t *out_len);
/* device-resident: one coder lane per 0xF6 block (the only parallel unit the
 * format has). *_dev status/out_len are device scalars. */
size_t zr_fse_workspace_bytes(size_t n, const zr_fse_config *c);
/* freqs_dev: device 256 x u32 raw frequency table, or NULL for the histogram of in */
int32_t zr_fse_compress_dev(const zr_fse_config *c, const uint32_t *freqs_dev, const uint8_t *in,
                            size_t n, uint8_t *out,
                            uint64_t *out_len_dev, int32_t *status_dev, void *workspace,
                            size_t workspace_bytes, void *stream);
/* max_blocks: an upper bound of the stream's block count (the host knows it
 * from the producer's config; zr_fse_decompressed_size parses it otherwise) */
size_t zr_fse_decode_workspace_bytes(uint64_t max_blocks);
int32_t zr_fse_decompress_dev(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                              uint64_t max_blocks, uint64_t *out_len_dev, int32_t *status_dev,
                              void *workspace, size_t workspace_bytes, void *stream);

/* ======================================================================
 * Multi-GPU shared table on RCCL (xGMI) -- one process per GPU
 * The reference trains one table on all of its data (RansBlobStore::train,
 * blob_store/entropy.rs:212-219; AdaptiveRans64Encoder, rans.rs:708-714).
 * Sharded over ranks, each rank counts its shard (zr_histogram_dev), the
 * counts are summed over the ranks in place, and every rank builds the same
 * table on its device (zr_rans_dtab_from_hist_dev). librccl is opened on the
 * first zr_comm_* call (ZR_UNSUPPORTED if absent). The caller moves the
 * unique id between its processes (ncclGetUniqueId/ncclCommInitRank contract).
 * ====================================================================== */
#define ZR_COMM_ID_BYTES 128
typedef struct zr_comm zr_comm;
/* rank 0 creates the id and shares it with the other ranks' processes */
int32_t zr_comm_unique_id(uint8_t id[ZR_COMM_ID_BYTES]);
/* collective over nranks processes; binds the calling thread's current device */
int32_t zr_comm_init(const uint8_t id[ZR_COMM_ID_BYTES], int32_t nranks, int32_t rank, zr_comm **comm);
/* the number of ranks RCCL itself reports for the communicator (ncclCommCount) */
int32_t zr_comm_count(const zr_comm *comm, int32_t *nranks);
/* in-place u32 SUM of n_bins device counters over the ranks (wraps mod 2^32 per
 * bin, as the reference's u32 counts); stream-ordered */
int32_t zr_histogram_allreduce_dev(zr_comm *comm, uint32_t *hist_dev, uint32_t n_bins, void *stream);
/* broadcast n_tables device tables (zr_rans_dtab_bytes() each) from root:
 * the alternative to re-building the table on every rank; stream-ordered */
int32_t zr_table_broadcast_dev(zr_comm *comm, void *dtabs_dev, uint32_t n_tables, int32_t root, void *stream);
int32_t zr_comm_destroy(zr_comm *comm);

/* ======================================================================
 * Huffman order-0 -- src/entropy/huffman/{tree,encoder,decoder}.rs
 * ====================================================================== */
typedef struct {
    int32_t kind;             /* 0 empty, 1 single leaf (code "0"), 2 tree */
    int32_t n_symbols;
    uint32_t max_code_length; /* HuffmanTree::max_code_length */
    uint8_t code_len[256];    /* 0: symbol not in the tree (get_code == None) */
    uint64_t code[256];       /* bit i = i-th emitted bit (LSB-first packing) */
    int32_t n_nodes;          /* decoding tree, node 0 = root */
    int16_t child[511][2];    /* -1 on leaves */
    uint8_t sym[511];         /* leaf symbol (placeholder leaves: 0) */
} zr_huff_tree;

/* HuffmanTree::from_frequencies                          tree.rs:52-133 */
int32_t zr_huff_tree_build(const uint32_t freq[256], zr_huff_tree *t);
size_t zr_huff_encode_bound(const zr_huff_tree *t, size_t n);
/* HuffmanEncoder::encode                                 encoder.rs:88-131 */
int32_t zr_huff_encode(const zr_huff_tree *t, const uint8_t *in, size_t n, uint8_t *out,
                       size_t out_cap, size_t *out_len);
/* HuffmanDecoder::decode (output_length = n)             decoder.rs:90-165 */
int32_t zr_huff_decode(const zr_huff_tree *t, const uint8_t *in, size_t in_len, uint8_t *out,
                       size_t n);
/* device-resident; the tree is passed by host pointer (its code table or
 * decode table is uploaded with the launch, stream-ordered). Decoding
 * synchronises its segments on the device (bounded parallel rounds, then an
 * exact in-order pass if needed): no host round trip; a short stream reports
 * ZR_INVALID_INPUT ("Decoded length mismatch") in *status_dev. */
size_t zr_huff_workspace_bytes(size_t n, size_t in_len);
int32_t zr_huff_encode_dev(const zr_huff_tree *t, const uint8_t *in, size_t n, uint8_t *out,
                           size_t out_cap, uint64_t *out_len_dev, int32_t *status_dev,
                           void *workspace, size_t workspace_bytes, void *stream);
int32_t zr_huff_decode_dev(const zr_huff_tree *t, const uint8_t *in, size_t in_len, uint8_t *out,
                           size_t n, int32_t *status_dev, void *workspace,
                           size_t workspace_bytes, void *stream);

/* HuffmanTree::serialize / deserialize (tree.rs:226-306). serialize writes
 * the symbols in ascending order (the reference walks a HashMap, so its bytes
 * vary between runs; every order deserializes to the same codes). Codes over
 * 64 bits or trees over 511 nodes (crafted input only) are ZR_UNSUPPORTED. */
size_t zr_huff_tree_serialized_bound(void);
int32_t zr_huff_tree_serialize(const zr_huff_tree *t, uint8_t *out, size_t out_cap, size_t *out_len);
int32_t zr_huff_tree_deserialize(const uint8_t *in, size_t n, zr_huff_tree *t);
/* HuffmanCompressor (compression/mod.rs:320-408): record = tree_size u32 |
 * serialized tree | size u32 | Huffman bits; empty <-> empty */
int32_t zr_huff_compressor_train(const uint8_t *train, size_t n, zr_huff_tree *t);
size_t zr_huff_compressor_bound(const zr_huff_tree *t, size_t n);
int32_t zr_huff_compressor_compress(const zr_huff_tree *t, const uint8_t *in, size_t n, uint8_t *out,
                                    size_t out_cap, size_t *out_len);
int32_t zr_huff_compressor_decompressed_size(const uint8_t *in, size_t n, size_t *size);
int32_t zr_huff_compressor_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                                      size_t *out_len);

/* ======================================================================
 * Contextual Huffman order-1/2 -- src/entropy/huffman/interleaved.rs
 * Every order-1/2 context tree holds all 256 symbols (interleaved.rs:160-171),
 * so each is the fixed 8-bit rank code (tree.rs:122-126) and the coded
 * stream is the byte sequence itself (x1) or its N-way chunk round-robin
 * (encode_xn, interleaved.rs:704-761). Order 2 trained on < 3 bytes is order 1
 * (interleaved.rs:191-193); order 1 trained on < 2 bytes is order 0 over that
 * data (interleaved.rs:119-121): zr_ctx_huff_order reports the effective order.
 * ====================================================================== */
typedef struct zr_ctx_huff zr_ctx_huff;
/* ContextualHuffmanEncoder::new(data, order)             interleaved.rs:94-266 */
int32_t zr_ctx_huff_new(const uint8_t *train, size_t n, int32_t order, zr_ctx_huff **out);
/* DictZipBlobStore entropy stage (dict_zip/blob_store.rs:1075-1224): algo 0
 * None, 1 HuffmanO1 (o1_model = ContextualHuffmanEncoder over the dictionary,
 * order 1), 2 Fse (parallel_blocks = interleave when > 1). encode keeps the
 * entropy form only when its size / n (f32) <= ratio_require and reports the
 * algorithm used; decode uses the non-interleaved O1 decoder with the record's
 * original size, as the reference does (:1179-1206). */
int32_t zr_dictzip_entropy_encode(int32_t algo, int32_t interleave, const zr_ctx_huff *o1_model,
                                  float ratio_require, const uint8_t *in, size_t n, uint8_t *out,
                                  size_t out_cap, size_t *out_len, int32_t *algo_used);
int32_t zr_dictzip_entropy_decode(int32_t algo, const zr_ctx_huff *o1_model, const uint8_t *in, size_t n,
                                  size_t original_size, uint8_t *out, size_t out_cap, size_t *out_len);
/* ContextualHuffmanEncoder::serialize / deserialize (interleaved.rs:476-595):
 * contexts ascending, context k owns tree k + 1 (the reference numbers and
 * lists them in HashMap order). */
size_t zr_ctx_huff_serialized_size(const zr_ctx_huff *h);
int32_t zr_ctx_huff_serialize(const zr_ctx_huff *h, uint8_t *out, size_t out_cap, size_t *out_len);
int32_t zr_ctx_huff_deserialize(const uint8_t *in, size_t n, zr_ctx_huff **out);
void zr_ctx_huff_free(zr_ctx_huff *h);
int32_t zr_ctx_huff_order(const zr_ctx_huff *h);        /* effective order */
size_t zr_ctx_huff_encode_bound(const zr_ctx_huff *h, size_t n);
/* encode (interleaved.rs:269-392); nway 0 = encode(), 1/2/4/8 =
 * encode_with_interleaving(X1..X8) (order 1 only, interleaved.rs:604-626) */
int32_t zr_ctx_huff_encode(const zr_ctx_huff *h, int32_t nway, const uint8_t *in, size_t n,
                           uint8_t *out, size_t out_cap, size_t *out_len);
/* ContextualHuffmanDecoder::decode (nway 0, interleaved.rs:1050-1209) or
 * decode_with_interleaving (nway 1/2/4/8, interleaved.rs:628-647, :764-822) */
int32_t zr_ctx_huff_decode(const zr_ctx_huff *h, int32_t nway, const uint8_t *in, size_t in_len,
                           uint8_t *out, size_t n, size_t *out_len);
/* device-resident order-1/2 coding (identity / N-way round-robin transpose);
 * ZR_UNSUPPORTED for an order-0 model (use zr_huff_*_dev with its tree) */
int32_t zr_ctx_huff_encode_dev(const zr_ctx_huff *h, int32_t nway, const uint8_t *in, size_t n,
                               uint8_t *out, void *stream);
int32_t zr_ctx_huff_decode_dev(const zr_ctx_huff *h, int32_t nway, const uint8_t *in,
                               size_t in_len, uint8_t *out, size_t n, void *stream);
/* the model's order-0 tree (trees[0]) */
int32_t zr_ctx_huff_tree0(const zr_ctx_huff *h, zr_huff_tree *t);

/* number of device allocations the library has made (process lifetime) */
int32_t zr_device_alloc_count(uint64_t *count);

/* ---- device memory helpers (for hosts without a HIP binding) ---- */
int32_t zr_malloc_dev(void **ptr, size_t bytes);
int32_t zr_free_dev(void *ptr);
int32_t zr_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream);
int32_t zr_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream);
int32_t zr_memset_dev(void *dst, int value, size_t bytes, void *stream);
/* device-to-device copy by a 16-B-per-lane streaming kernel (grid 0: 8 x CUs
 * workgroups of 256): the achievable one-pass ceiling the bench reports */
int32_t zr_memcpy_dev(void *dst, const void *src, size_t bytes, uint32_t grid, void *stream);
int32_t zr_stream_sync(void *stream);

/* ---- kernel timers: HIP events recorded around every launch of the named
 * kernel on the stream it is launched on ("rans_decode", "rans_encode",
 * "fse_decode", ...). read() synchronises those events. */
int32_t zr_timer_enable(int32_t on);
/* time only the named kernels (comma-separated, e.g. "rans_encode"); NULL or "" = all */
int32_t zr_timer_select(const char *names);
int32_t zr_timer_reset(void);
int32_t zr_timer_read(const char *kernel, double *total_ms, uint64_t *launches);

/* ---- synthetic inputs used by bench.py ----
 * kind 0 'u': xorshift64 bytes (tests/fse_tests.rs:711-717), byte = x >> 32
 * kind 1 'z': Zipf(alpha = 1.1) over 256 ranks, rank k -> byte k-1
 * kind 2 't': text-like order-1 Markov bytes over 64 printable symbols */
int32_t zr_synth_fill(int32_t kind, uint64_t seed, uint8_t *out, size_t n);

#ifdef __cplusplus
}
#endif
#endif
