// zr_huff.hip -- Huffman order-0 (src/entropy/huffman/{tree,encoder,decoder}.rs)
// and contextual order-1/2 (interleaved.rs) on MI355X / gfx950.
//
// Tree construction (H1) is host code: <= 256 leaves, a Rust BinaryHeap
// emulation. The coding is on the GPU:
//   encode (H2): code-length reduction -> block scan -> bit scatter with
//     atomicOr into a word image -> byte copy-out;
//   decode (H3): the stream is cut into fixed bit segments; every segment is
//     decoded from a guessed code boundary and the guesses are repaired by
//     propagating each segment's end into the next one until no start moves
//     (Huffman codes self-synchronise within a few codes); then a count scan
//     and a final decode pass that writes the symbols. Tables are 8-bit
//     multi-level LUTs built on the host from the decoding tree.
//   order 1/2 (H4-H6): every context tree holds all 256 symbols, so codes are
//     the fixed 8-bit rank codes == the byte itself; encode/decode are a
//     vectorised copy (x1) or the N-way chunk round-robin transpose.
#include <algorithm>
#include <cstring>
#include <vector>

#include "zr_internal.h"

namespace zr {

// ------------------------------------------------------------------ H1 (host)
namespace {
struct BNode {
    uint32_t freq;
    int32_t sym;  // -1 internal
    int32_t l, r;
};

// std::collections::BinaryHeap (max-heap over `Reverse(node)`; the node order
// of tree.rs:29-40 makes the element with the HIGHEST frequency the max).
struct RustHeap {
    std::vector<int32_t> d;
    const std::vector<BNode> *nodes;
    bool le(int32_t a, int32_t b) const { return (*nodes)[a].freq <= (*nodes)[b].freq; }
    size_t sift_up(size_t start, size_t pos) {
        const int32_t e = d[pos];
        while (pos > start) {
            const size_t parent = (pos - 1) / 2;
            if (le(e, d[parent])) break;
            d[pos] = d[parent];
            pos = parent;
        }
        d[pos] = e;
        return pos;
    }
    void push(int32_t x) {
        d.push_back(x);
        sift_up(0, d.size() - 1);
    }
    void sift_down_to_bottom(size_t pos) {
        const size_t end = d.size(), start = pos;
        const int32_t e = d[pos];
        size_t child = 2 * pos + 1;
        while (end >= 2 && child <= end - 2) {
            if (le(d[child], d[child + 1])) child += 1;
            d[pos] = d[child];
            pos = child;
            child = 2 * pos + 1;
        }
        if (child == end - 1) {
            d[pos] = d[child];
            pos = child;
        }
        d[pos] = e;
        sift_up(start, pos);
    }
    int32_t pop() {
        int32_t item = d.back();
        d.pop_back();
        if (!d.empty()) {
            std::swap(item, d[0]);
            sift_down_to_bottom(0);
        }
        return item;
    }
};

int new_node(zr_huff_tree *t, int sym) {
    const int i = t->n_nodes++;
    t->child[i][0] = t->child[i][1] = -1;
    t->sym[i] = (uint8_t)(sym < 0 ? 0 : sym);
    return i;
}

// from_frequencies_fixed_length (tree.rs:136-175) + build_decoding_tree_from_codes
// (tree.rs:311-350) + insert_code_into_tree (tree.rs:359-469).
int32_t fixed_tree(const uint32_t freq[256], zr_huff_tree *t) {
    memset(t->code_len, 0, sizeof(t->code_len));
    memset(t->code, 0, sizeof(t->code));
    t->n_nodes = 0;
    int rank = 0;
    for (int s = 0; s < 256; s++)
        if (freq[s]) {
            t->code_len[s] = 8;
            t->code[s] = (uint64_t)rank++;  // rank bits, LSB first
        }
    t->n_symbols = rank;
    t->max_code_length = 8;
    t->kind = 2;
    // the decoding tree of a complete set of distinct 8-bit codes: internal
    // nodes down to depth 8, leaves carry their code's symbol; codes that no
    // symbol owns end in placeholder leaves (symbol 0)
    std::vector<int> placeholder;
    auto mk = [&](int sym, bool ph) {
        const int i = new_node(t, sym);
        placeholder.resize(t->n_nodes);
        placeholder[i] = ph ? 1 : 0;
        return i;
    };
    const int root = mk(0, false);
    t->child[root][0] = (int16_t)mk(0, true);
    t->child[root][1] = (int16_t)mk(0, true);
    for (int s = 0; s < 256; s++) {
        if (!t->code_len[s]) continue;
        int node = root;
        for (int b = 0; b < 8; b++) {
            const int bit = (int)((t->code[s] >> b) & 1);
            int c = t->child[node][bit];
            if (b == 7) {
                if (!placeholder[c]) return set_error(ZR_INVALID_INPUT, "Code collision");
                placeholder[c] = 0;
                t->sym[c] = (uint8_t)s;
                break;
            }
            if (t->child[c][0] < 0) {  // leaf: placeholder -> internal with two placeholders
                if (!placeholder[c]) return set_error(ZR_INVALID_INPUT, "Code collision");
                placeholder[c] = 0;
                const int a = mk(0, true), z = mk(0, true);
                t->child[c][0] = (int16_t)a;
                t->child[c][1] = (int16_t)z;
            }
            node = c;
        }
    }
    return ZR_OK;
}
}  // namespace

int32_t huff_build(const uint32_t freq[256], zr_huff_tree *t) {
    memset(t, 0, sizeof(*t));
    std::vector<BNode> nodes;
    nodes.reserve(512);
    RustHeap h;
    h.nodes = &nodes;
    for (int s = 0; s < 256; s++)
        if (freq[s]) {  // leaves pushed in byte order (tree.rs:59-67)
            nodes.push_back({freq[s], s, -1, -1});
            h.push((int32_t)nodes.size() - 1);
        }
    const int count = (int)nodes.size();
    t->n_symbols = count;
    if (count == 0) {  // tree.rs:69-75
        t->kind = 0;
        return ZR_OK;
    }
    if (count == 1) {  // tree.rs:78-90: the code is [false]
        const int s = nodes[h.pop()].sym;
        t->kind = 1;
        t->code_len[s] = 1;
        t->code[s] = 0;
        t->max_code_length = 1;
        new_node(t, s);
        return ZR_OK;
    }
    while (h.d.size() > 1) {  // tree.rs:93-111
        const int32_t l = h.pop(), r = h.pop();
        nodes.push_back({nodes[l].freq + nodes[r].freq, -1, l, r});  // u32 add wraps (release)
        h.push((int32_t)nodes.size() - 1);
    }
    const int32_t root = h.pop();
    // generate_codes (tree.rs:187-208): left = 0, right = 1; depth-first with
    // an explicit stack (a chain tree is up to 255 deep)
    uint32_t maxlen = 0;
    struct Fr {
        int32_t n;
        uint32_t len;
        uint64_t code;
    };
    std::vector<Fr> st;
    st.push_back({root, 0, 0});
    while (!st.empty()) {
        const Fr f = st.back();
        st.pop_back();
        const BNode &b = nodes[f.n];
        if (b.sym >= 0) {
            maxlen = std::max(maxlen, f.len);
            t->code_len[b.sym] = (uint8_t)std::min<uint32_t>(f.len, 255);
            t->code[b.sym] = f.code;
            continue;
        }
        st.push_back({b.r, f.len + 1, f.len < 64 ? (f.code | (1ull << f.len)) : f.code});
        st.push_back({b.l, f.len + 1, f.code});
    }
    if (maxlen > 64) return fixed_tree(freq, t);  // tree.rs:122-126
    t->kind = 2;
    t->max_code_length = maxlen;
    // decoding tree = the build tree, preorder numbered from the root
    std::vector<std::pair<int32_t, int32_t>> work;  // (build node, parent slot)
    work.push_back({root, -1});
    while (!work.empty()) {
        const auto w = work.back();
        work.pop_back();
        const BNode &b = nodes[w.first];
        const int me = new_node(t, b.sym);
        if (w.second >= 0) t->child[w.second >> 1][w.second & 1] = (int16_t)me;
        if (b.sym < 0) {
            work.push_back({b.r, me * 2 + 1});
            work.push_back({b.l, me * 2 + 0});
        }
    }
    return ZR_OK;
}

// multi-level 8-bit decode LUT: table k has 256 entries for the node it
// starts at; entry = leaf: 1<<31 | bits << 8 | sym ; else next table index
// (8 bits consumed).
static void huff_lut(const zr_huff_tree *t, std::vector<uint32_t> &lut) {
    lut.clear();
    std::vector<int> tab_node{0}, node_tab(t->n_nodes, -1);
    node_tab[0] = 0;
    for (size_t k = 0; k < tab_node.size(); k++) {
        const int start = tab_node[k];
        lut.resize((k + 1) * 256);
        for (uint32_t v = 0; v < 256; v++) {
            int cur = start;
            uint32_t used = 0, e = 0;
            bool leaf = false;
            while (used < 8) {
                cur = t->child[cur][(v >> used) & 1];
                used++;
                if (t->child[cur][0] < 0) {
                    leaf = true;
                    break;
                }
            }
            if (leaf) {
                e = 0x80000000u | (used << 8) | t->sym[cur];
            } else {
                if (node_tab[cur] < 0) {
                    node_tab[cur] = (int)tab_node.size();
                    tab_node.push_back(cur);
                }
                e = (uint32_t)node_tab[cur];
            }
            lut[k * 256 + v] = e;
        }
    }
}

// ------------------------------------------------------------------ H2 (GPU)
constexpr uint32_t HE_SYM = 16;                 // symbols per thread
constexpr uint32_t HE_BLK = 256 * HE_SYM;       // symbols per workgroup

struct HuffCodes {
    uint64_t code[256];
    uint32_t len[256];
};

__device__ __forceinline__ uint64_t blk_excl_scan_u64(uint64_t v, unsigned long long *sh, uint64_t *total) {
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

// the code table travels as a by-value kernel argument (3 KiB of kernarg)
__global__ __launch_bounds__(256) void k_huff_enc_len(const uint8_t *in, uint64_t n, const HuffCodes hc,
                                                      uint64_t *blocksum, int32_t *status) {
    __shared__ uint32_t s_len[256];
    __shared__ unsigned long long sh[4];
    s_len[threadIdx.x] = hc.len[threadIdx.x];
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * HE_BLK + (uint64_t)threadIdx.x * HE_SYM;
    uint64_t bits = 0;
    bool miss = false;
    for (uint32_t k = 0; k < HE_SYM; k++) {
        const uint64_t i = base + k;
        if (i < n) {
            const uint32_t L = s_len[in[i]];
            miss |= L == 0;
            bits += L;
        }
    }
    if (miss) *status = ZR_INVALID_INPUT;  // "Symbol {} not in Huffman tree" (encoder.rs:96-101)
    uint64_t tot;
    blk_excl_scan_u64(bits, sh, &tot);
    if (threadIdx.x == 0) blocksum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_huff_scan(uint64_t *v, uint64_t nb, uint64_t *total_bits,
                                                   uint64_t *out_len, const int32_t *status) {
    __shared__ unsigned long long sh[4];
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nb; base += 256) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t x = i < nb ? v[i] : 0;
        uint64_t tot;
        const uint64_t ex = blk_excl_scan_u64(x, sh, &tot);
        if (i < nb) v[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        if (total_bits) *total_bits = carry;
        if (out_len) *out_len = (status && *status) ? 0 : (carry + 7) / 8;
    }
}

__device__ __forceinline__ void put_bits32(uint32_t *W, uint64_t p, uint32_t v, uint32_t L) {
    // v holds L <= 32 bits; OR them in at bit position p (LSB-first)
    if (L == 0) return;
    const uint64_t w = p >> 5;
    const uint32_t sh = (uint32_t)(p & 31);
    atomicOr(&W[w], v << sh);
    if (sh + L > 32) atomicOr(&W[w + 1], v >> (32 - sh));
}

__global__ __launch_bounds__(256) void k_huff_enc_write(const uint8_t *in, uint64_t n, const HuffCodes hc,
                                                        const uint64_t *blockoff, uint32_t *W,
                                                        const int32_t *status) {
    __shared__ uint32_t s_len[256];
    __shared__ uint64_t s_code[256];
    __shared__ unsigned long long sh[4];
    s_len[threadIdx.x] = hc.len[threadIdx.x];
    s_code[threadIdx.x] = hc.code[threadIdx.x];
    __syncthreads();
    if (*status) return;  // uniform: written only by the previous kernel
    const uint64_t base = (uint64_t)blockIdx.x * HE_BLK + (uint64_t)threadIdx.x * HE_SYM;
    uint8_t syms[HE_SYM];
    uint64_t bits = 0;
    for (uint32_t k = 0; k < HE_SYM; k++) {
        const uint64_t i = base + k;
        syms[k] = i < n ? in[i] : 0;
        bits += i < n ? s_len[syms[k]] : 0;
    }
    uint64_t p = blockoff[blockIdx.x] + blk_excl_scan_u64(bits, sh, nullptr);
    // gather into a 64-bit accumulator; emit whole 32-bit words
    uint64_t acc = 0;
    uint32_t na = 0;
    const uint32_t lead = (uint32_t)(p & 31);  // first partial word is shared with the left neighbour
    uint64_t wp = p - lead;                     // bit position of acc's bit 0
    acc = 0;
    na = lead;
    for (uint32_t k = 0; k < HE_SYM; k++) {
        if (base + k >= n) break;
        const uint32_t L = s_len[syms[k]];
        const uint64_t c = s_code[syms[k]];
        uint32_t done = 0;
        while (done < L) {
            const uint32_t take = min(L - done, 32u);
            const uint64_t part = (c >> done) & ((take == 32) ? 0xFFFFFFFFull : ((1ull << take) - 1));
            acc |= part << na;
            na += take;
            done += take;
            if (na >= 32) {
                atomicOr(&W[wp >> 5], (uint32_t)acc);
                acc >>= 32;
                na -= 32;
                wp += 32;
            }
        }
    }
    if (na > 0) atomicOr(&W[wp >> 5], (uint32_t)acc);
}

__global__ void k_copy_bytes(const uint8_t *src, uint8_t *dst, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

__global__ void k_copy_dev_len(const uint8_t *src, uint8_t *dst, const uint64_t *len, const int32_t *status) {
    if (*status) return;
    const uint64_t n = *len;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// ------------------------------------------------------------------ H3 (GPU)
constexpr uint64_t HD_SEG = 4096;  // bits per segment (>= the 64-bit longest code)

struct HuffDecArgs {
    const uint32_t *W;  // stream as little-endian words (+ two zero words of padding)
    uint64_t B;         // stream bits
    uint64_t nseg;
    const uint32_t *lut;
    uint64_t *start, *end;
    uint64_t *cnt;      // codes per segment, then their exclusive scan
    uint8_t *dirty;
    uint32_t *changed;
    uint8_t *out;
    uint64_t n;
};

__device__ __forceinline__ uint32_t peek8(const uint32_t *W, uint64_t p) {
    const uint64_t w = p >> 5;
    const uint64_t v = ((uint64_t)W[w + 1] << 32) | W[w];
    return (uint32_t)(v >> (p & 31)) & 0xFF;
}

// decode codes from p while p < lim; a code must complete within B.
// Returns the number of codes; *pe = position after the last code (or B when
// the stream ends inside a code).
template <bool WRITE>
__device__ uint64_t seg_decode(const HuffDecArgs &a, uint64_t p, uint64_t lim, uint64_t *pe, uint64_t obase) {
    uint64_t c = 0;
    while (p < lim) {
        uint32_t tab = 0;
        uint64_t q = p;
        uint32_t e;
        for (;;) {
            e = a.lut[tab * 256 + peek8(a.W, q)];
            if (e & 0x80000000u) {
                q += (e >> 8) & 0xFF;
                break;
            }
            q += 8;
            tab = e;
            if (q >= a.B) break;  // ran off the end inside a code
        }
        if (!(e & 0x80000000u) || q > a.B) {  // incomplete final code
            *pe = a.B;
            return c;
        }
        if (WRITE) {
            const uint64_t o = obase + c;
            if (o < a.n) a.out[o] = (uint8_t)e;
        }
        c++;
        p = q;
    }
    *pe = p;
    return c;
}

// Segment synchronisation runs entirely on the device (no host round trip):
// round r re-decodes the dirty segments, then moves every start to the end of
// the previous segment and records in changed[r] whether any start moved.
// Round r > 0 does nothing once round r-1 changed nothing (converged).
// k (non-zero): every code of the tree is k bits long, so the code boundaries
// are exactly the multiples of k and the first guess is already right (a
// fixed-length code never resynchronises from a wrong guess).
__global__ __launch_bounds__(256) void k_huff_init(HuffDecArgs a, uint32_t nflags, uint32_t k) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t < a.nseg) {
        a.start[t] = k ? (t * HD_SEG + k - 1) / k * k : t * HD_SEG;  // the guessed boundaries
        a.dirty[t] = 1;
    }
    if (t < nflags) a.changed[t] = 0;
}

__global__ __launch_bounds__(256) void k_huff_seg(HuffDecArgs a, uint32_t round) {
    if (round > 0 && a.changed[round - 1] == 0) return;
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= a.nseg || !a.dirty[t]) return;
    const uint64_t lim = min((t + 1) * HD_SEG, a.B);
    uint64_t pe;
    a.cnt[t] = seg_decode<false>(a, a.start[t], lim, &pe, 0);
    a.end[t] = pe;
    a.dirty[t] = 0;
}

__global__ __launch_bounds__(256) void k_huff_fix(HuffDecArgs a, uint32_t round) {
    if (round > 0 && a.changed[round - 1] == 0) return;
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t == 0 || t >= a.nseg) return;
    const uint64_t s = a.end[t - 1];
    if (s != a.start[t]) {
        a.start[t] = s;
        a.dirty[t] = 1;
        a.changed[round] = 1;
    }
}

// After the parallel rounds, if the last round still moved a start (a code set
// whose wrong guesses do not resynchronise, e.g. a deserialized tree of
// fixed-length codes of a length that does not divide the segment), the exact
// starts come from a parallel resolve instead of an in-order walk:
//   1. k_huff_map: for every segment t and every entry offset e < L (L = the
//      longest code; the true start of t is the first code boundary >= t*SEG,
//      so it is t*SEG + e for one such e) decode the segment and record the
//      exit offset into segment t+1 (ME_END: the stream ended), nseg x L
//      independent segment decodes;
//   2. k_huff_compose: one workgroup composes those maps by a Hillis-Steele
//      scan (log2 nseg levels), so C_t = f_t o ... o f_0 and segment t+1
//      starts at (t+1)*SEG + C_t(0); starts that differ are marked dirty and
//      one more k_huff_seg pass decodes them.
// Both return at once when the rounds converged (the usual case).
constexpr uint8_t ME_END = 0xFF;
__global__ __launch_bounds__(256) void k_huff_map(HuffDecArgs a, uint32_t last, uint32_t L, uint8_t *map) {
    if (a.changed[last] == 0) return;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.nseg * L) return;
    const uint64_t t = i / L, e = i % L;
    const uint64_t p = t * HD_SEG + e;
    uint8_t r = ME_END;
    if (p < a.B) {
        uint64_t pe;
        seg_decode<false>(a, p, min((t + 1) * HD_SEG, a.B), &pe, 0);
        if (pe < a.B) r = (uint8_t)(pe - (t + 1) * HD_SEG);  // < L: a code started below the limit
    }
    map[i] = r;
}

__global__ __launch_bounds__(1024) void k_huff_compose(HuffDecArgs a, uint32_t last, uint32_t L, uint8_t *m0,
                                                       uint8_t *m1) {
    if (a.changed[last] == 0) return;
    const uint64_t tot = a.nseg * L;
    uint8_t *src = m0, *dst = m1;
    for (uint64_t d = 1; d < a.nseg; d <<= 1) {
        for (uint64_t i = threadIdx.x; i < tot; i += 1024) {
            const uint64_t t = i / L, e = i % L;
            uint8_t v = src[i];
            if (t >= d) {  // C_t o C_{t-d}: first the lower segments' composite
                const uint8_t u = src[(t - d) * L + e];
                v = u == ME_END ? ME_END : src[t * L + u];
            }
            dst[i] = v;
        }
        __threadfence_block();
        __syncthreads();
        uint8_t *x = src;
        src = dst;
        dst = x;
    }
    for (uint64_t t = threadIdx.x; t < a.nseg; t += 1024) {
        uint64_t st = 0;
        if (t > 0) {
            const uint8_t o = src[(t - 1) * L];  // C_{t-1}(0)
            st = o == ME_END ? a.B : t * HD_SEG + o;
        }
        if (st != a.start[t]) {
            a.start[t] = st;
            a.dirty[t] = 1;
        }
    }
}

// fewer complete codes than requested (decoder.rs:157-163)
__global__ void k_huff_check(const uint64_t *total, uint64_t n, int32_t *status) {
    if (threadIdx.x == 0 && *total < n) *status = ZR_INVALID_INPUT;
}

__global__ __launch_bounds__(256) void k_huff_write(HuffDecArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= a.nseg) return;
    const uint64_t o = a.cnt[t];
    if (o >= a.n) return;
    const uint64_t lim = min((t + 1) * HD_SEG, a.B);
    uint64_t pe;
    seg_decode<true>(a, a.start[t], lim, &pe, o);
}

__global__ void k_fill(uint8_t *out, uint64_t n, uint8_t v) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = v;
}

// ------------------------------------------------------------ H5/H6 (GPU)
// x1: 16-byte vector copy. xN: out[i*N + k] = in[start_k + i] (the round
// robin of encode_xn, interleaved.rs:704-761), inverse for decode.
__global__ __launch_bounds__(256) void k_copy16(const uint8_t *src, uint8_t *dst, uint64_t n) {
    const uint64_t nv = n >> 4;
    typedef unsigned v4 __attribute__((ext_vector_type(4)));
    const v4 *s4 = reinterpret_cast<const v4 *>(src);
    v4 *d4 = reinterpret_cast<v4 *>(dst);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
        const v4 v = __builtin_nontemporal_load(&s4[i]);
        __builtin_nontemporal_store(v, &d4[i]);
    }
    for (uint64_t i = (nv << 4) + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        dst[i] = src[i];
}

template <int N, bool ENC>
__global__ __launch_bounds__(256) void k_xn(const uint8_t *src, uint8_t *dst, uint64_t n) {
    const uint64_t q = n / N, r = n % N;
    const uint64_t rounds = q + (r ? 1 : 0);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rounds; i += stride) {
        const uint32_t kk = i < q ? N : (uint32_t)r;
        uint8_t v[N];
#pragma unroll
        for (int k = 0; k < N; k++) {
            const uint64_t sk = (uint64_t)k * q + min((uint64_t)k, r);
            if ((uint32_t)k < kk) {
                if (ENC) v[k] = src[sk + i];
                else dst[sk + i] = src[i * N + k];
            }
        }
        if (ENC) {
            if (kk == N && (((uintptr_t)(dst + i * N)) % N) == 0) {
                if constexpr (N == 8) {
                    uint2 w;
                    w.x = v[0] | (v[1] << 8) | (v[2] << 16) | ((uint32_t)v[3] << 24);
                    w.y = v[4] | (v[5] << 8) | (v[6] << 16) | ((uint32_t)v[7] << 24);
                    *reinterpret_cast<uint2 *>(dst + i * N) = w;
                } else if constexpr (N == 4) {
                    *reinterpret_cast<uint32_t *>(dst + i * N) =
                        v[0] | (v[1] << 8) | (v[2] << 16) | ((uint32_t)v[3] << 24);
                } else {
#pragma unroll
                    for (int k = 0; k < N; k++) dst[i * N + k] = v[k];
                }
            } else {
                for (uint32_t k = 0; k < kk; k++) dst[i * N + k] = v[k];
            }
        }
    }
}

static void launch_xn(int nway, bool enc, const uint8_t *src, uint8_t *dst, uint64_t n, hipStream_t s) {
    const uint64_t per = (n + nway - 1) / nway;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(per, 256), 65535));
#define ZR_XN(NW)                                                                      \
    if (nway == NW) {                                                                 \
        if (enc) hipLaunchKernelGGL((k_xn<NW, true>), dim3(grid), dim3(256), 0, s, src, dst, n); \
        else hipLaunchKernelGGL((k_xn<NW, false>), dim3(grid), dim3(256), 0, s, src, dst, n);   \
    }
    ZR_XN(2) ZR_XN(4) ZR_XN(8)
#undef ZR_XN
}

static void launch_copy(const uint8_t *src, uint8_t *dst, uint64_t n, hipStream_t s) {
    if (((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0) {
        const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(n >> 4, 256), 8192));
        hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(256), 0, s, src, dst, n);
    } else {
        const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(n, 256), 1u << 30));
        hipLaunchKernelGGL(k_copy_bytes, dim3(grid), dim3(256), 0, s, src, dst, n);
    }
}


// build_decoding_tree_from_codes (tree.rs:311-356) + insert_code_into_tree
// (tree.rs:359-469). Placeholder leaves (symbol 0, frequency 0) fill the
// branches no code takes. An empty remaining code replaces the node it reaches
// with a leaf (tree.rs:360-366), so for such inputs insertion order matters:
// the reference iterates a HashMap, here the order is ascending symbol.
int32_t tree_from_codes(const uint8_t present[256], const uint8_t len[256], const uint64_t code[256],
                        zr_huff_tree *t) {
    memset(t, 0, sizeof(*t));
    int count = 0, last = -1;
    uint32_t maxlen = 0;
    for (int s = 0; s < 256; s++)
        if (present[s]) {
            count++;
            last = s;
            maxlen = std::max<uint32_t>(maxlen, len[s]);
            t->code_len[s] = len[s];
            t->code[s] = code[s];
        }
    t->n_symbols = count;
    t->max_code_length = maxlen;
    if (count == 0) {  // tree.rs:315-317
        t->kind = 0;
        return ZR_OK;
    }
    if (count == 1) {  // tree.rs:320-334: a single leaf whatever its code
        t->kind = 1;
        new_node(t, last);
        return ZR_OK;
    }
    t->kind = 2;
    std::vector<uint8_t> ph;  // placeholder flag per node
    auto mk = [&](bool p) -> int {
        if (t->n_nodes >= 511) return -1;
        const int i = new_node(t, 0);
        ph.resize(t->n_nodes);
        ph[i] = p ? 1 : 0;
        return i;
    };
    const int root = mk(false);
    t->child[root][0] = (int16_t)mk(true);
    t->child[root][1] = (int16_t)mk(true);
    for (int s = 0; s < 256; s++) {
        if (!present[s]) continue;
        int node = root;
        for (uint32_t i = 0;; i++) {
            if (i == len[s]) {  // remaining code empty: this node becomes the symbol's leaf
                t->child[node][0] = t->child[node][1] = -1;
                t->sym[node] = (uint8_t)s;
                ph[node] = 0;
                break;
            }
            if (t->child[node][0] < 0) {  // a leaf on the path
                if (!ph[node]) return set_error(ZR_INVALID_INPUT, "Code collision: trying to overwrite existing symbol");
                const int a = mk(true), b = mk(true);  // placeholder -> internal node
                if (a < 0 || b < 0) return set_error(ZR_UNSUPPORTED, "Huffman tree exceeds 511 nodes");
                ph[node] = 0;
                t->child[node][0] = (int16_t)a;
                t->child[node][1] = (int16_t)b;
            }
            node = t->child[node][(code[s] >> i) & 1];
        }
    }
    return ZR_OK;
}

}  // namespace zr

using namespace zr;

struct zr_ctx_huff {
    int32_t order;              // effective order
    zr_huff_tree t0;            // order 0: the model; order 1/2: trees[0] (all 256 symbols)
    std::vector<uint32_t> ctx;  // order 1/2: the contexts that own a tree, ascending
};

extern "C" {

int32_t zr_huff_tree_build(const uint32_t freq[256], zr_huff_tree *t) {
    ZR_GUARD_BEGIN
    clear_error();
    return huff_build(freq, t);
    ZR_GUARD_END
}

size_t zr_huff_encode_bound(const zr_huff_tree *t, size_t n) {
    return (size_t)((n * (uint64_t)std::max<uint32_t>(t->max_code_length, 1) + 7) / 8) + 16;
}

size_t zr_huff_workspace_bytes(size_t n, size_t in_len) {
    const uint64_t nb = ceil_div(std::max<size_t>(n, 1), HE_BLK);
    const uint64_t enc = 4096 + round_up(sizeof(HuffCodes), 256) + round_up(8 * nb, 256) +
                         round_up((n * 64 + 7) / 8 + 64, 256);
    const uint64_t B = (uint64_t)in_len * 8;
    const uint64_t nseg = std::max<uint64_t>(1, ceil_div(B, HD_SEG));
    const uint64_t dec = 4096 + round_up(in_len + 64, 256) + 3 * round_up(8 * nseg, 256) + round_up(nseg, 256) +
                         round_up(4ull * 256 * 256, 256) + 2 * round_up(64 * nseg, 256);
    return (size_t)std::max(enc, dec);
}

int32_t zr_huff_encode_dev(const zr_huff_tree *t, const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                           uint64_t *out_len_dev, int32_t *status_dev, void *ws, size_t ws_bytes, void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (capturing((hipStream_t)stream))
        return set_error(ZR_UNSUPPORTED, "zr_huff_encode_dev on a capturing stream");
    hipStream_t s = (hipStream_t)stream;
    ZR_HIP(hipMemsetAsync(status_dev, 0, 4, s));
    if (n == 0) {  // encoder.rs:89-91
        ZR_HIP(hipMemsetAsync(out_len_dev, 0, 8, s));
        return ZR_OK;
    }
    if (ws_bytes < zr_huff_workspace_bytes(n, 0)) return set_error(ZR_INVALID_INPUT, "workspace too small");
    // the worst case: every symbol takes max_code_length bits
    if (out_cap < zr_huff_encode_bound(t, n) - 16) return set_error(ZR_INVALID_INPUT, "output capacity too small");
    uint8_t *w = reinterpret_cast<uint8_t *>(round_up((uintptr_t)ws, 256));
    HuffCodes hc;
    for (int i = 0; i < 256; i++) {
        hc.code[i] = t->code[i];
        hc.len[i] = t->code_len[i];
    }
    const uint64_t nb = ceil_div(n, HE_BLK);
    uint64_t *bsum = reinterpret_cast<uint64_t *>(w);
    w += round_up(8 * nb, 256);
    uint32_t *W = reinterpret_cast<uint32_t *>(w);
    const uint64_t maxbytes = (n * (uint64_t)std::max<uint32_t>(t->max_code_length, 1) + 7) / 8;
    const uint64_t wbytes = round_up(maxbytes + 8, 4);
    ZR_HIP(hipMemsetAsync(W, 0, wbytes, s));
    timer_begin("huff_encode", s);
    hipLaunchKernelGGL(k_huff_enc_len, dim3((uint32_t)nb), dim3(256), 0, s, in, (uint64_t)n, hc, bsum, status_dev);
    hipLaunchKernelGGL(k_huff_scan, dim3(1), dim3(256), 0, s, bsum, nb, (uint64_t *)nullptr, out_len_dev,
                       (const int32_t *)status_dev);
    hipLaunchKernelGGL(k_huff_enc_write, dim3((uint32_t)nb), dim3(256), 0, s, in, (uint64_t)n, hc,
                       (const uint64_t *)bsum, W, (const int32_t *)status_dev);
    hipLaunchKernelGGL(k_copy_dev_len, dim3(1024), dim3(256), 0, s, (const uint8_t *)W, out,
                       (const uint64_t *)out_len_dev, (const int32_t *)status_dev);
    timer_end("huff_encode", s);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_huff_decode_dev(const zr_huff_tree *t, const uint8_t *in, size_t in_len, uint8_t *out, size_t n,
                           int32_t *status_dev, void *ws, size_t ws_bytes, void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    hipStream_t s = (hipStream_t)stream;
    ZR_HIP(hipMemsetAsync(status_dev, 0, 4, s));
    if (in_len == 0 || n == 0) return ZR_OK;  // decoder.rs:91-93
    if (t->kind == 0) return set_error(ZR_INVALID_INPUT, "Empty Huffman tree");
    if (n / 64 > in_len || n > in_len * 64)  // decoder.rs:100-107
        return set_error(ZR_INVALID_INPUT, "Implausible output length");
    const uint64_t B = (uint64_t)in_len * 8;
    if (t->kind == 1) {
        // a single-leaf root emits one symbol per bit plus the final fix-up
        // (decoder.rs:112-155): n symbols need n <= B + 1
        if (n > B + 1) return set_error(ZR_INVALID_INPUT, "Decoded length mismatch");
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, s, out, (uint64_t)n, t->sym[0]);
        ZR_HIP(hipGetLastError());
        return ZR_OK;
    }
    if (ws_bytes < zr_huff_workspace_bytes(0, in_len)) return set_error(ZR_INVALID_INPUT, "workspace too small");
    if (capturing(s))  // the decode table is staged from host memory freed by a host callback
        return set_error(ZR_UNSUPPORTED, "zr_huff_decode_dev stages its decode table: not capturable");
    std::vector<uint32_t> lut;
    huff_lut(t, lut);
    if (lut.size() > 256 * 256) return set_error(ZR_INTERNAL, "decode table too large");
    uint8_t *w = reinterpret_cast<uint8_t *>(round_up((uintptr_t)ws, 256));
    uint32_t *flag = reinterpret_cast<uint32_t *>(w);
    w += 4096;
    uint8_t *stream_copy = w;
    w += round_up(in_len + 64, 256);
    const uint64_t nseg = ceil_div(B, HD_SEG);
    HuffDecArgs a;
    a.W = reinterpret_cast<const uint32_t *>(stream_copy);
    a.B = B;
    a.nseg = nseg;
    a.start = reinterpret_cast<uint64_t *>(w);
    w += round_up(8 * nseg, 256);
    a.end = reinterpret_cast<uint64_t *>(w);
    w += round_up(8 * nseg, 256);
    a.cnt = reinterpret_cast<uint64_t *>(w);
    w += round_up(8 * nseg, 256);
    a.dirty = w;
    w += round_up(nseg, 256);
    uint32_t *dlut = reinterpret_cast<uint32_t *>(w);
    w += round_up(4ull * 256 * 256, 256);
    uint8_t *map0 = w;  // the resolve's segment maps (nseg x L, L <= 64), ping-pong
    w += round_up(64 * nseg, 256);
    uint8_t *map1 = w;
    a.lut = dlut;
    a.changed = flag;
    a.out = out;
    a.n = n;
    ZR_HIP(hipMemsetAsync(stream_copy + in_len, 0, 64, s));
    launch_copy(in, stream_copy, in_len, s);
    // the decode table leaves from a heap copy that a stream-ordered host
    // callback frees once the copy has run (no host synchronisation here)
    auto *held = new std::vector<uint32_t>(std::move(lut));
    ZR_HIP(hipMemcpyAsync(dlut, held->data(), held->size() * 4, hipMemcpyHostToDevice, s));
    ZR_HIP(hipLaunchHostFunc(
        s, [](void *p) { delete static_cast<std::vector<uint32_t> *>(p); }, held));
    const uint32_t g = (uint32_t)ceil_div(nseg, 256);
    // chain codes resynchronise at their first 1 bit (every code but the
    // all-zero one ends in a 1, tree.rs:187-208), fixed-length codes are seeded
    // on their boundaries: both settle in round 0 or 1
    constexpr uint32_t ROUNDS = 4;
    uint32_t kfix = 0;
    {
        uint32_t lo = 64, hi = 0;
        for (int v = 0; v < 256; v++)
            if (t->code_len[v]) {
                lo = std::min<uint32_t>(lo, t->code_len[v]);
                hi = std::max<uint32_t>(hi, t->code_len[v]);
            }
        if (lo == hi) kfix = hi;
    }
    const uint32_t L = std::max<uint32_t>(1, std::min<uint32_t>(64, t->max_code_length));
    hipLaunchKernelGGL(k_huff_init, dim3(g), dim3(256), 0, s, a, ROUNDS, kfix);
    timer_begin("huff_decode", s);
    for (uint32_t r = 0; r < ROUNDS; r++) {
        hipLaunchKernelGGL(k_huff_seg, dim3(g), dim3(256), 0, s, a, r);
        hipLaunchKernelGGL(k_huff_fix, dim3(g), dim3(256), 0, s, a, r);
    }
    // the parallel resolve (no-ops when round ROUNDS-1 moved nothing), then the
    // re-decode of the segments it moved (k_huff_seg's round ROUNDS reads the
    // same flag)
    hipLaunchKernelGGL(k_huff_map, dim3((uint32_t)ceil_div(nseg * L, 256)), dim3(256), 0, s, a, ROUNDS - 1, L, map0);
    hipLaunchKernelGGL(k_huff_compose, dim3(1), dim3(1024), 0, s, a, ROUNDS - 1, L, map0, map1);
    hipLaunchKernelGGL(k_huff_seg, dim3(g), dim3(256), 0, s, a, ROUNDS);
    uint64_t *tot = reinterpret_cast<uint64_t *>(flag + 8);
    hipLaunchKernelGGL(k_huff_scan, dim3(1), dim3(256), 0, s, a.cnt, nseg, tot, (uint64_t *)nullptr,
                       (const int32_t *)nullptr);
    hipLaunchKernelGGL(k_huff_write, dim3(g), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_huff_check, dim3(1), dim3(64), 0, s, (const uint64_t *)tot, (uint64_t)n, status_dev);
    timer_end("huff_decode", s);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

// ---- host-memory entry points (synchronous, on a leased call context:
// zr_internal.h CallLease -- no allocation in steady state, stream-scoped sync)
int32_t zr_huff_encode(const zr_huff_tree *t, const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                       size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    *out_len = 0;
    if (n == 0) return ZR_OK;
    const size_t wsb = zr_huff_workspace_bytes(n, 0), cap = zr_huff_encode_bound(t, n);
    CallLease L;
    int32_t st = L.acquire();
    if (st) return st;
    void *din, *dout, *dws, *dm;
    if ((st = L.get(0, n, &din)) || (st = L.get(1, cap, &dout)) || (st = L.get(4, wsb, &dws)) ||
        (st = L.get(2, 64, &dm)))
        return st;
    hipStream_t s = L.stream();
    ZR_HIP(hipMemcpyAsync(din, in, n, hipMemcpyHostToDevice, s));
    uint64_t *olen = reinterpret_cast<uint64_t *>(dm);
    int32_t *dst = reinterpret_cast<int32_t *>(olen + 1);
    st = zr_huff_encode_dev(t, (const uint8_t *)din, n, (uint8_t *)dout, cap, olen, dst, dws, wsb, s);
    if (st) return st;
    uint64_t *meta = L.ctx()->meta;
    ZR_HIP(hipMemcpyAsync(meta, dm, 16, hipMemcpyDeviceToHost, s));
    if ((st = L.sync())) return st;
    if ((int32_t)meta[1]) return set_error(ZR_INVALID_INPUT, "Symbol not in Huffman tree");
    if (meta[0] > out_cap) return set_error(ZR_INVALID_INPUT, "output capacity too small");
    ZR_HIP(hipMemcpyAsync(out, dout, meta[0], hipMemcpyDeviceToHost, s));
    if ((st = L.sync())) return st;
    *out_len = meta[0];
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_huff_decode(const zr_huff_tree *t, const uint8_t *in, size_t in_len, uint8_t *out, size_t n) {
    ZR_GUARD_BEGIN
    clear_error();
    if (in_len == 0 || n == 0) return ZR_OK;
    const size_t wsb = zr_huff_workspace_bytes(0, in_len);
    CallLease L;
    int32_t st = L.acquire();
    if (st) return st;
    void *din, *dout, *dws, *dm;
    if ((st = L.get(0, in_len, &din)) || (st = L.get(1, n, &dout)) || (st = L.get(4, wsb, &dws)) ||
        (st = L.get(2, 64, &dm)))
        return st;
    hipStream_t s = L.stream();
    ZR_HIP(hipMemcpyAsync(din, in, in_len, hipMemcpyHostToDevice, s));
    st = zr_huff_decode_dev(t, (const uint8_t *)din, in_len, (uint8_t *)dout, n, (int32_t *)dm, dws, wsb, s);
    if (st) return st;
    uint64_t *meta = L.ctx()->meta;
    ZR_HIP(hipMemcpyAsync(meta, dm, 8, hipMemcpyDeviceToHost, s));
    if ((st = L.sync())) return st;
    if ((int32_t)meta[0] != 0) return set_error(ZR_INVALID_INPUT, "Decoded length mismatch");
    ZR_HIP(hipMemcpyAsync(out, dout, n, hipMemcpyDeviceToHost, s));
    return L.sync();
    ZR_GUARD_END
}

// order-1/2 host calls: the identity / transpose kernels on a leased context
static int32_t ctx_host_run(const zr_ctx_huff *h, int32_t nway, bool enc, const uint8_t *in, size_t in_len,
                            uint8_t *out, size_t n) {
    CallLease L;
    int32_t st = L.acquire();
    if (st) return st;
    void *din, *dout;
    if ((st = L.get(0, in_len, &din)) || (st = L.get(1, n, &dout))) return st;
    hipStream_t s = L.stream();
    ZR_HIP(hipMemcpyAsync(din, in, in_len, hipMemcpyHostToDevice, s));
    st = enc ? zr_ctx_huff_encode_dev(h, nway, (const uint8_t *)din, n, (uint8_t *)dout, s)
             : zr_ctx_huff_decode_dev(h, nway, (const uint8_t *)din, in_len, (uint8_t *)dout, n, s);
    if (st) return st;
    ZR_HIP(hipMemcpyAsync(out, dout, n, hipMemcpyDeviceToHost, s));
    return L.sync();
}

// ---------------------------------------------------------- contextual O1/O2
int32_t zr_ctx_huff_new(const uint8_t *train, size_t n, int32_t order, zr_ctx_huff **out) {
    ZR_GUARD_BEGIN
    clear_error();
    *out = nullptr;
    if (order < 0 || order > 2) return set_error(ZR_INVALID_INPUT, "order must be 0, 1 or 2");
    int32_t eff = order;
    if (eff == 2 && n < 3) eff = 1;  // interleaved.rs:191-193
    if (eff == 1 && n < 2) eff = 0;  // interleaved.rs:119-121
    zr_ctx_huff *h = new zr_ctx_huff();
    h->order = eff;
    uint32_t f[256] = {0};
    if (eff == 0) {
        // new_order0: HuffmanTree::from_data (tree.rs:178-184): the byte histogram
        if (n) {
            std::vector<uint32_t> hist(256, 0);
            for (size_t i = 0; i < n; i++) hist[train[i]]++;
            memcpy(f, hist.data(), sizeof(f));
        }
    } else {
        // order-0 frequencies with zeros raised to 1 (interleaved.rs:131-136):
        // all 256 symbols, so the tree is the fixed rank code (rank == byte)
        for (int s = 0; s < 256; s++) f[s] = 1;
    }
    int32_t st = huff_build(f, &h->t0);
    if (st) {
        delete h;
        return st;
    }
    if (eff == 1) {  // one tree per context seen before a symbol (interleaved.rs:140-185)
        uint8_t seen[256] = {};
        for (size_t i = 1; i < n; i++) seen[train[i - 1]] = 1;
        for (uint32_t c = 0; c < 256; c++)
            if (seen[c]) h->ctx.push_back(c);
    } else if (eff == 2) {
        // the 1024 contexts with the most symbols (interleaved.rs:213-232); the
        // reference breaks ties in HashMap order, here by ascending context
        std::vector<uint32_t> tot(65536, 0);
        for (size_t i = 2; i < n; i++) tot[((uint32_t)train[i - 2] << 8) | train[i - 1]]++;
        std::vector<uint32_t> all;
        for (uint32_t c = 0; c < 65536; c++)
            if (tot[c]) all.push_back(c);
        const size_t take = std::min<size_t>(1024, all.size());
        std::partial_sort(all.begin(), all.begin() + take, all.end(), [&](uint32_t x, uint32_t y) {
            return tot[x] != tot[y] ? tot[x] > tot[y] : x < y;
        });
        h->ctx.assign(all.begin(), all.begin() + take);
        std::sort(h->ctx.begin(), h->ctx.end());
    }
    *out = h;
    return ZR_OK;
    ZR_GUARD_END
}

void zr_ctx_huff_free(zr_ctx_huff *h) { delete h; }
int32_t zr_ctx_huff_order(const zr_ctx_huff *h) { return h->order; }

int32_t zr_ctx_huff_tree0(const zr_ctx_huff *h, zr_huff_tree *t) {
    *t = h->t0;
    return ZR_OK;
}

size_t zr_ctx_huff_encode_bound(const zr_ctx_huff *h, size_t n) {
    return h->order == 0 ? zr_huff_encode_bound(&h->t0, n) : n + 16;
}

int32_t zr_ctx_huff_encode_dev(const zr_ctx_huff *h, int32_t nway, const uint8_t *in, size_t n, uint8_t *out,
                               void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (capturing((hipStream_t)stream))
        return set_error(ZR_UNSUPPORTED, "zr_ctx_huff_encode_dev on a capturing stream");
    if (h->order == 0) return set_error(ZR_UNSUPPORTED, "order-0 model: use zr_huff_encode_dev");
    if (nway != 0 && nway != 1 && nway != 2 && nway != 4 && nway != 8)
        return set_error(ZR_INVALID_INPUT, "interleaving factor must be 1, 2, 4 or 8");
    if (nway != 0 && h->order != 1)  // interleaved.rs:609-613
        return set_error(ZR_INVALID_INPUT, "Interleaving only supported for Order-1 Huffman encoding");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) return ZR_OK;
    timer_begin("huff_o1_encode", s);
    if (nway <= 1) launch_copy(in, out, n, s);
    else launch_xn(nway, true, in, out, n, s);
    timer_end("huff_o1_encode", s);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_ctx_huff_decode_dev(const zr_ctx_huff *h, int32_t nway, const uint8_t *in, size_t in_len,
                               uint8_t *out, size_t n, void *stream) {
    ZR_GUARD_BEGIN
    clear_error();
    if (capturing((hipStream_t)stream))
        return set_error(ZR_UNSUPPORTED, "zr_ctx_huff_decode_dev on a capturing stream");
    if (h->order == 0) return set_error(ZR_UNSUPPORTED, "order-0 model: use zr_huff_decode_dev");
    if (nway != 0 && nway != 1 && nway != 2 && nway != 4 && nway != 8)
        return set_error(ZR_INVALID_INPUT, "interleaving factor must be 1, 2, 4 or 8");
    if (nway != 0 && h->order != 1)
        return set_error(ZR_INVALID_INPUT, "Interleaving only supported for Order-1 Huffman decoding");
    hipStream_t s = (hipStream_t)stream;
    if (in_len == 0 || n == 0) return ZR_OK;
    if (in_len < n) return set_error(ZR_INVALID_INPUT, "Unexpected end of stream");
    timer_begin("huff_o1_decode", s);
    if (nway <= 1) launch_copy(in, out, n, s);
    else launch_xn(nway, false, in, out, n, s);
    timer_end("huff_o1_decode", s);
    ZR_HIP(hipGetLastError());
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_ctx_huff_encode(const zr_ctx_huff *h, int32_t nway, const uint8_t *in, size_t n, uint8_t *out,
                           size_t out_cap, size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    *out_len = 0;
    if (h->order == 0) {
        if (nway != 0) return set_error(ZR_INVALID_INPUT, "Interleaving only supported for Order-1 Huffman encoding");
        return zr_huff_encode(&h->t0, in, n, out, out_cap, out_len);
    }
    if (nway != 0 && h->order != 1)
        return set_error(ZR_INVALID_INPUT, "Interleaving only supported for Order-1 Huffman encoding");
    if (n == 0) return ZR_OK;
    if (out_cap < n) return set_error(ZR_INVALID_INPUT, "output capacity too small");
    int32_t st = ctx_host_run(h, nway, true, in, n, out, n);
    if (st) return st;
    *out_len = n;
    return ZR_OK;
    ZR_GUARD_END
}

int32_t zr_ctx_huff_decode(const zr_ctx_huff *h, int32_t nway, const uint8_t *in, size_t in_len, uint8_t *out,
                           size_t n, size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    *out_len = 0;
    if (h->order == 0) {
        if (nway != 0) return set_error(ZR_INVALID_INPUT, "Interleaving only supported for Order-1 Huffman decoding");
        if (in_len == 0 || n == 0) return ZR_OK;
        // decode_order0 (interleaved.rs:1082-1130) is the same walk as
        // HuffmanDecoder::decode without the plausibility check, whose
        // rejections the walk's length check also makes
        if (h->t0.kind == 0) return set_error(ZR_INVALID_INPUT, "Empty Huffman tree");
        if (n > (uint64_t)in_len * 8 + 1) return set_error(ZR_INVALID_INPUT, "Decoded length mismatch");
        int32_t st = zr_huff_decode(&h->t0, in, in_len, out, n);
        if (st == ZR_OK) *out_len = n;
        return st;
    }
    if (nway != 0 && h->order != 1)
        return set_error(ZR_INVALID_INPUT, "Interleaving only supported for Order-1 Huffman decoding");
    if (in_len == 0 || n == 0) return ZR_OK;
    if (in_len < n) return set_error(ZR_INVALID_INPUT, "Decoded length mismatch");
    int32_t st = ctx_host_run(h, nway, false, in, in_len, out, n);
    if (st) return st;
    *out_len = n;
    return ZR_OK;
    ZR_GUARD_END
}

}  // extern "C"

extern "C" {

// ---- serialized trees and the HuffmanCompressor record

size_t zr_huff_tree_serialized_bound(void) { return 2 + 256 * (2 + 8); }

// HuffmanTree::serialize (tree.rs:226-262) with the symbols in ascending
// order: the reference walks a HashMap, so its order (and bytes) vary from
// run to run; any order deserializes to the same codes.
int32_t zr_huff_tree_serialize(const zr_huff_tree *t, uint8_t *out, size_t out_cap, size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!t || !out || !out_len) return set_error(ZR_INVALID_INPUT, "null argument");
    *out_len = 0;
    size_t need = 2;
    uint32_t count = 0;
    for (int s = 0; s < 256; s++)
        if (t->code_len[s]) {
            count++;
            need += 2 + (t->code_len[s] + 7) / 8;
        }
    if (need > out_cap) return set_error(ZR_INVALID_INPUT, "output buffer too small");
    size_t o = 0;
    out[o++] = (uint8_t)count;
    out[o++] = (uint8_t)(count >> 8);
    for (int s = 0; s < 256; s++) {
        const uint32_t L = t->code_len[s];
        if (!L) continue;
        out[o++] = (uint8_t)s;
        out[o++] = (uint8_t)L;
        for (uint32_t k = 0; k < (L + 7) / 8; k++) {
            const uint32_t bits = std::min<uint32_t>(8, L - 8 * k);
            out[o++] = (uint8_t)((t->code[s] >> (8 * k)) & ((1u << bits) - 1));
        }
    }
    *out_len = o;
    return ZR_OK;
    ZR_GUARD_END
}

// HuffmanTree::deserialize (tree.rs:265-306). Codes longer than 64 bits
// (never produced by serialize: longer chains take the fixed 8-bit tree) are
// ZR_UNSUPPORTED, as are crafted code sets needing more than 511 tree nodes.
int32_t zr_huff_tree_deserialize(const uint8_t *in, size_t n, zr_huff_tree *t) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!t || (!in && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    if (n < 2) return set_error(ZR_INVALID_INPUT, "Huffman tree data too short");
    const uint32_t count = (uint32_t)in[0] | ((uint32_t)in[1] << 8);
    uint8_t present[256] = {}, len[256] = {};
    uint64_t code[256] = {};
    size_t o = 2;
    for (uint32_t k = 0; k < count; k++) {
        if (o + 2 > n) return set_error(ZR_INVALID_INPUT, "Truncated Huffman tree data");
        const uint8_t s = in[o], L = in[o + 1];
        o += 2;
        const size_t nb = (L + 7) / 8;
        if (o + nb > n) return set_error(ZR_INVALID_INPUT, "Truncated Huffman code data");
        if (L > 64) return set_error(ZR_UNSUPPORTED, "Huffman code longer than 64 bits");
        uint64_t c = 0;
        for (size_t i = 0; i < L; i++) c |= (uint64_t)((in[o + i / 8] >> (i % 8)) & 1) << i;
        present[s] = 1;  // a repeated symbol overwrites (HashMap::insert)
        len[s] = L;
        code[s] = c;
        o += nb;
    }
    return tree_from_codes(present, len, code, t);
    ZR_GUARD_END
}

// HuffmanCompressor::new (compression/mod.rs:330-334): HuffmanEncoder::new(training_data)
int32_t zr_huff_compressor_train(const uint8_t *train, size_t n, zr_huff_tree *t) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!t || (!train && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    uint32_t f[256];
    int32_t st = zr_byte_histogram(train, n, f);
    if (st) return st;
    return huff_build(f, t);
    ZR_GUARD_END
}

size_t zr_huff_compressor_bound(const zr_huff_tree *t, size_t n) {
    return 8 + zr_huff_tree_serialized_bound() + zr_huff_encode_bound(t, n);
}

// Compressor::compress (mod.rs:345-369): tree_size u32 | tree | size u32 | bits
int32_t zr_huff_compressor_compress(const zr_huff_tree *t, const uint8_t *in, size_t n, uint8_t *out,
                                    size_t out_cap, size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!t || (!in && n) || !out_len || (!out && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *out_len = 0;
    if (n == 0) return ZR_OK;
    uint8_t tree[2 + 256 * 10];
    size_t ts = 0;
    int32_t st = zr_huff_tree_serialize(t, tree, sizeof(tree), &ts);
    if (st) return st;
    if (out_cap < 8 + ts) return set_error(ZR_INVALID_INPUT, "output buffer too small");
    size_t body = 0;
    if ((st = zr_huff_encode(t, in, n, out + 8 + ts, out_cap - 8 - ts, &body))) return st;
    for (int k = 0; k < 4; k++) out[k] = (uint8_t)(ts >> (8 * k));
    memcpy(out + 4, tree, ts);
    for (int k = 0; k < 4; k++) out[4 + ts + k] = (uint8_t)((uint32_t)n >> (8 * k));
    *out_len = 8 + ts + body;
    return ZR_OK;
    ZR_GUARD_END
}

static int32_t huff_record_parse(const uint8_t *in, size_t n, size_t *ts, size_t *size) {
    if (n < 8) return set_error(ZR_INVALID_INPUT, "Huffman compressed data too short");  // mod.rs:376-380
    *ts = (size_t)in[0] | ((size_t)in[1] << 8) | ((size_t)in[2] << 16) | ((size_t)in[3] << 24);
    if (n < 8 + *ts) return set_error(ZR_INVALID_INPUT, "Huffman compressed data truncated");  // :385-389
    const uint8_t *p = in + 4 + *ts;
    *size = (size_t)p[0] | ((size_t)p[1] << 8) | ((size_t)p[2] << 16) | ((size_t)p[3] << 24);
    return ZR_OK;
}

int32_t zr_huff_compressor_decompressed_size(const uint8_t *in, size_t n, size_t *size) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!size || (!in && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *size = 0;
    if (n == 0) return ZR_OK;
    size_t ts = 0;
    return huff_record_parse(in, n, &ts, size);
    ZR_GUARD_END
}

// Compressor::decompress (mod.rs:371-407): the record's own tree decodes it
int32_t zr_huff_compressor_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                                      size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!out_len || (!in && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *out_len = 0;
    if (n == 0) return ZR_OK;
    size_t ts = 0, size = 0;
    int32_t st = huff_record_parse(in, n, &ts, &size);
    if (st) return st;
    zr_huff_tree t;
    if ((st = zr_huff_tree_deserialize(in + 4, ts, &t))) return st;
    if (size > out_cap || (!out && size)) return set_error(ZR_INVALID_INPUT, "output buffer too small");
    if ((st = zr_huff_decode(&t, in + 8 + ts, n - 8 - ts, out, size))) return st;
    *out_len = size;
    return ZR_OK;
    ZR_GUARD_END
}

}  // extern "C"

extern "C" {

// ContextualHuffmanEncoder::serialize (interleaved.rs:476-503): order u8 |
// tree count u32 | context count u32 | (context u32, tree index u32)* |
// (tree size u32, HuffmanTree::serialize)*. The reference walks its context
// HashMap (and numbers trees in HashMap order); here contexts ascend and
// context k owns tree k + 1.
size_t zr_ctx_huff_serialized_size(const zr_ctx_huff *h) {
    uint8_t tmp[2 + 256 * 10];
    size_t ts = 0;
    if (!h || zr_huff_tree_serialize(&h->t0, tmp, sizeof(tmp), &ts)) return 0;
    return 9 + 8 * h->ctx.size() + (1 + h->ctx.size()) * (4 + ts);
}

int32_t zr_ctx_huff_serialize(const zr_ctx_huff *h, uint8_t *out, size_t out_cap, size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!h || !out || !out_len) return set_error(ZR_INVALID_INPUT, "null argument");
    *out_len = 0;
    uint8_t tree[2 + 256 * 10];
    size_t ts = 0;
    int32_t st = zr_huff_tree_serialize(&h->t0, tree, sizeof(tree), &ts);
    if (st) return st;
    const size_t need = 9 + 8 * h->ctx.size() + (1 + h->ctx.size()) * (4 + ts);
    if (need > out_cap) return set_error(ZR_INVALID_INPUT, "output buffer too small");
    size_t o = 0;
    auto put32 = [&](uint32_t v) {
        for (int k = 0; k < 4; k++) out[o++] = (uint8_t)(v >> (8 * k));
    };
    out[o++] = (uint8_t)h->order;
    put32((uint32_t)(1 + h->ctx.size()));
    put32((uint32_t)h->ctx.size());
    for (size_t k = 0; k < h->ctx.size(); k++) {
        put32(h->ctx[k]);
        put32((uint32_t)(k + 1));
    }
    // trees[0] and every context tree: all the same fixed 8-bit identity code for
    // order 1/2 (every merged table has all 256 symbols); order 0 has only trees[0]
    for (size_t k = 0; k < 1 + h->ctx.size(); k++) {
        put32((uint32_t)ts);
        memcpy(out + o, tree, ts);
        o += ts;
    }
    *out_len = o;
    return ZR_OK;
    ZR_GUARD_END
}

// ContextualHuffmanEncoder::deserialize (interleaved.rs:506-595). Order 1/2
// models must consist of fixed 8-bit identity trees, which is what every
// serialized order-1/2 model holds; anything else is ZR_UNSUPPORTED, as is a
// model without trees.
int32_t zr_ctx_huff_deserialize(const uint8_t *in, size_t n, zr_ctx_huff **out) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!out || (!in && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *out = nullptr;
    if (n == 0) return set_error(ZR_INVALID_INPUT, "Empty contextual Huffman data");
    const uint8_t order = in[0];
    if (order > 2) return set_error(ZR_INVALID_INPUT, "Invalid Huffman order");
    size_t o = 1;
    auto get32 = [&](uint32_t *v) {
        *v = (uint32_t)in[o] | ((uint32_t)in[o + 1] << 8) | ((uint32_t)in[o + 2] << 16) | ((uint32_t)in[o + 3] << 24);
        o += 4;
    };
    uint32_t ntrees, nctx;
    if (o + 4 > n) return set_error(ZR_INVALID_INPUT, "Truncated tree count");
    get32(&ntrees);
    if (o + 4 > n) return set_error(ZR_INVALID_INPUT, "Truncated context count");
    get32(&nctx);
    std::vector<uint32_t> ctx;
    for (uint32_t k = 0; k < nctx; k++) {
        if (o + 8 > n) return set_error(ZR_INVALID_INPUT, "Truncated context map");
        uint32_t c, idx;
        get32(&c);
        get32(&idx);
        ctx.push_back(c);
    }
    std::sort(ctx.begin(), ctx.end());
    ctx.erase(std::unique(ctx.begin(), ctx.end()), ctx.end());  // HashMap keys
    zr_ctx_huff *h = new zr_ctx_huff();
    h->order = order;
    h->ctx = ctx;
    auto fail = [&](int32_t st) {
        delete h;
        return st;
    };
    for (uint32_t k = 0; k < ntrees; k++) {
        uint32_t ts;
        if (o + 4 > n) return fail(set_error(ZR_INVALID_INPUT, "Truncated tree size"));
        get32(&ts);
        if (o + ts > n) return fail(set_error(ZR_INVALID_INPUT, "Truncated tree data"));
        zr_huff_tree t;
        int32_t st = zr_huff_tree_deserialize(in + o, ts, &t);
        if (st) return fail(st);
        o += ts;
        if (order != 0) {
            bool ident = t.kind == 2;
            for (int s = 0; s < 256 && ident; s++) ident = t.code_len[s] == 8 && t.code[s] == (uint64_t)s;
            if (!ident) return fail(set_error(ZR_UNSUPPORTED, "order-1/2 model with a non-identity tree"));
        }
        if (k == 0) h->t0 = t;
    }
    if (ntrees == 0) return fail(set_error(ZR_UNSUPPORTED, "contextual Huffman model without trees"));
    *out = h;
    return ZR_OK;
    ZR_GUARD_END
}


// ---- DictZipBlobStore entropy stage (dict_zip/blob_store.rs:1075-1224)
// algo: 0 None, 1 HuffmanO1 (model = ContextualHuffmanEncoder::new(dictionary,
// Order1)), 2 Fse. The encoded form is kept only when encoded/raw (as f32)
// <= ratio_require (check_compression_ratio, :1155-1161).
int32_t zr_dictzip_entropy_encode(int32_t algo, int32_t interleave, const zr_ctx_huff *o1_model,
                                  float ratio_require, const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                                  size_t *out_len, int32_t *algo_used) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!out_len || !algo_used || (!in && n) || (!out && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *out_len = 0;
    *algo_used = 0;
    auto raw = [&]() -> int32_t {
        if (n > out_cap) return set_error(ZR_INVALID_INPUT, "output buffer too small");
        if (n) memcpy(out, in, n);
        *out_len = n;
        *algo_used = 0;
        return ZR_OK;
    };
    if (algo == 0) return raw();
    std::vector<uint8_t> enc;
    size_t el = 0;
    int32_t st;
    if (algo == 1) {
        if (!o1_model) return set_error(ZR_INVALID_INPUT, "HuffmanO1 needs the dictionary's order-1 model");
        int nway;
        switch (interleave) {  // apply_huffman_o1_encoding (:1114-1124)
            case 0: case 1: nway = 1; break;
            case 2: nway = 2; break;
            case 4: nway = 4; break;
            case 8: nway = 8; break;
            default: return set_error(ZR_INVALID_INPUT, "Invalid interleaving factor");
        }
        enc.resize(zr_ctx_huff_encode_bound(o1_model, n) + 16);
        st = zr_ctx_huff_encode(o1_model, nway, in, n, enc.data(), enc.size(), &el);
    } else if (algo == 2) {  // apply_fse_encoding (:1128-1152)
        zr_fse_config c;
        zr_fse_config_default(&c);
        c.parallel_blocks = interleave > 1 ? (uint64_t)interleave : 0;
        enc.resize(zr_fse_compress_bound(n, &c));
        st = zr_fse_compress(&c, in, n, enc.data(), enc.size(), &el);
    } else {
        return set_error(ZR_INVALID_INPUT, "unknown entropy algorithm");
    }
    if (st) return st;
    if (n == 0 || !((float)el / (float)n <= ratio_require)) return raw();
    if (el > out_cap) return set_error(ZR_INVALID_INPUT, "output buffer too small");
    memcpy(out, enc.data(), el);
    *out_len = el;
    *algo_used = algo;
    return ZR_OK;
    ZR_GUARD_END
}

// decode_entropy (:1164-1224). HuffmanO1 decodes with the non-interleaved
// decoder and the record's original size, whatever the encode interleaving
// was (:1179-1206) -- reproduced as is.
int32_t zr_dictzip_entropy_decode(int32_t algo, const zr_ctx_huff *o1_model, const uint8_t *in, size_t n,
                                  size_t original_size, uint8_t *out, size_t out_cap, size_t *out_len) {
    ZR_GUARD_BEGIN
    clear_error();
    if (!out_len || (!in && n)) return set_error(ZR_INVALID_INPUT, "null argument");
    *out_len = 0;
    if (algo == 0) {
        if (n > out_cap || (!out && n)) return set_error(ZR_INVALID_INPUT, "output buffer too small");
        if (n) memcpy(out, in, n);
        *out_len = n;
        return ZR_OK;
    }
    if (algo == 1) {
        if (!o1_model) return set_error(ZR_INVALID_INPUT, "HuffmanO1 needs the dictionary's order-1 model");
        if (original_size > out_cap || (!out && original_size))
            return set_error(ZR_INVALID_INPUT, "output buffer too small");
        return zr_ctx_huff_decode(o1_model, 0, in, n, out, original_size, out_len);
    }
    if (algo == 2) return zr_fse_decompress(in, n, out, out_cap, out_len);
    return set_error(ZR_INVALID_INPUT, "unknown entropy algorithm");
    ZR_GUARD_END
}

}  // extern "C"
