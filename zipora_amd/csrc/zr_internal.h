// zr_internal.h -- shared definitions of the MI355X entropy backend (product code).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stddef.h>
#include <string>

#include "../../include/zipora_amd.h"

// ---------------------------------------------------------------------------
// error plumbing (src/ffi/c_api.rs:17-76 conventions)
// ---------------------------------------------------------------------------
namespace zr {
int32_t set_error(int32_t code, const std::string &msg);
// compute units of the current device (cached per device)
uint32_t cu_count();
// the stream is being captured into a HIP graph
inline bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}
void clear_error();
// fill `bytes` bytes at device address p with the byte `value`, stream-ordered,
// by a kernel (zr_rans.hip): the memsets of the capturable calls. A
// hipMemsetAsync of 64 B or more captured into a HIP graph writes other data
// (address-like words) on the graph's second and later replays on this ROCm
// (tools/graph_memset_probe.py, profiles/r06_graph_memset_probe.log); a kernel
// node replays as captured.
void fill_dev(void *p, int value, size_t bytes, hipStream_t s);

#define ZR_HIP(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return ::zr::set_error(ZR_INTERNAL, std::string("HIP error: ") +              \
                                                    hipGetErrorString(e_) + " at " #expr); \
    } while (0)

#define ZR_GUARD_BEGIN try {
#define ZR_GUARD_END                                                   \
    }                                                                  \
    catch (const std::bad_alloc &) {                                   \
        return ::zr::set_error(ZR_MEMORY_ERROR, "out of host memory"); \
    }                                                                  \
    catch (...) {                                                      \
        return ::zr::set_error(ZR_INTERNAL, "internal exception");     \
    }

// ---------------------------------------------------------------------------
// rANS constants (src/entropy/rans.rs:14-16)
// ---------------------------------------------------------------------------
constexpr uint32_t RANS_L = 1u << 16;
constexpr uint32_t TF_SHIFT = 12;
constexpr uint32_t TOTFREQ = 1u << TF_SHIFT;
// top bit of an encoder block byte sum: a symbol of the block is not in the table
constexpr uint64_t BS_ERR = 1ull << 63;

// Device table: everything the encode and decode kernels need for one
// normalised frequency table. 16-byte aligned, copied into LDS per workgroup.
enum : uint32_t { DT_NORMAL = 0, DT_SINGLE = 1, DT_EMPTY = 2 };
struct alignas(16) RansDTab {
    uint32_t kind;      // DT_NORMAL: every freq <= 4095; DT_SINGLE: one symbol owns 4096; DT_EMPTY
    uint32_t status;    // ZR_OK, or ZR_INVALID_INPUT if normalisation failed
    uint32_t pad[2];
    uint32_t freq[256];
    uint32_t start[256];
    // encode: q = umulhi(x << 8, rcp) >> rsh == x / freq for every x < 2^24
    // (Granlund-Montgomery with N = 24, l = ceil(log2 freq), rcp = ceil(2^(24+l)/freq))
    uint32_t rcp[256];
    uint32_t rsh[256];
    // decode: slot -> sym | (slot - start) << 8 | freq << 20   (freq <= 4095 when DT_NORMAL)
    uint32_t slot[TOTFREQ];
};

// Encoder division x / freq for x < 2^24 (rans.rs:331 with the state in
// [2^16, 2^24)): q = umulhi(x << 8, rcp) >> rsh, Granlund-Montgomery with
// N = 24, l = ceil(log2 freq), rcp = ceil(2^(24+l) / freq). Shared by the
// device table build (k_tab), the host table build and the exhaustive
// self-test (zr_rans_selftest_reciprocal).
__host__ __device__ inline uint32_t enc_rsh(uint32_t f) { return f <= 1 ? 0u : 32u - (uint32_t)__builtin_clz(f - 1); }
__host__ __device__ inline uint32_t enc_rcp(uint32_t f) {
    return f ? (uint32_t)(((1ull << (24 + enc_rsh(f))) + f - 1) / f) : 0u;
}
// enc_rcp without a 64-bit division (device table builds)
// floor(num / d) for d >= 1 and num < 2^50: the f64 reciprocal (v_rcp_f64 and
// one Newton step, relative error ~2^-51) and the product's rounding put
// trunc(num * r) within one of the floor while num / d < 2^50, and the
// remainder's sign and size correct it by one (no IEEE division sequence on
// the chain). Beyond that bound the error can exceed one: not exact. Callers
// stay far below it (the table build: num < 2^44; enc_rcp_fast: num < 2^37).
__device__ inline uint64_t floor_div_u64(uint64_t num, uint32_t d) {
    const double dd = (double)d;
    double r = __builtin_amdgcn_rcp(dd);
    r = __builtin_fma(__builtin_fma(-dd, r, 1.0), r, r);
    uint64_t q = (uint64_t)((double)num * r);
    const int64_t rem = (int64_t)(num - q * d);
    q += rem >= (int64_t)d ? 1 : 0;
    q -= rem < 0 ? 1 : 0;
    return q;
}
__device__ inline uint32_t enc_rcp_fast(uint32_t f) {
    if (!f) return 0u;
    return (uint32_t)floor_div_u64((1ull << (24 + enc_rsh(f))) + f - 1, f);
}
__host__ __device__ inline uint32_t enc_div(uint32_t x, uint32_t rcp, uint32_t rsh) {
    return (uint32_t)(((uint64_t)(x << 8) * rcp) >> 32) >> rsh;
}

// host-side Rans64Encoder::new restatement (used by zr_rans_table_build and dtab upload)
int32_t rans_normalize_host(const uint32_t raw[256], zr_rans_table *out);
void rans_dtab_from_table(const zr_rans_table *t, RansDTab *d);

// per-batch workspace carve (device pointers)
struct RansWork {
    uint32_t *st_state;   // [B*N]
    uint32_t *st_len;     // [B*N]
    uint32_t *st_off;     // [B*N] (256-lane encoder) byte offset of each stream in its 256-stream block
    uint64_t *blocksum;   // [B*nblk]
    uint64_t *blockoff;   // [B*nblk]
    uint8_t *scratch;     // [B*R]
    uint64_t region;      // R: scratch bytes per buffer
    uint32_t cap;         // scratch bytes per stream (xN mode), a multiple of 16
    uint32_t nblk;
    // xN scratch layout. il = 1 (short streams): the IL_SPAN (zr_rans.hip, 64)
    // streams of a group s & ~(IL_SPAN - 1) share IL_SPAN * cap bytes, 16-B quad q
    // of stream s at ((q * IL_SPAN + s % IL_SPAN) * 16) (the encoder's burst stores
    // coalesce across lanes into 1 KiB runs). il = 0: stream s owns cap contiguous
    // bytes at s * cap
    uint32_t il;
};
size_t rans_workspace_bytes(uint32_t B, uint32_t N, uint64_t max_len);
int32_t rans_carve(uint32_t B, uint32_t N, uint64_t max_len, void *ws, size_t bytes, RansWork *w);

// HIP-event timing of named kernels (zr_timer_* in the C ABI).
// launch_timed: one kernel launch whose own begin/end the dispatch records in
// a pair of HIP events (hipExtLaunchKernelGGL). No marker packets enter the
// stream: a separate hipEventRecord costs the MI355X queue about 5 us of idle
// per event, 40 us per headline step with four timed kernels.
// timer_begin/timer_end bracket a multi-kernel range with recorded events.
struct TimerPair {
    hipEvent_t a, b;
};
TimerPair timer_pair(const char *name);  // {nullptr, nullptr} while timers are off
template <typename F, typename... Args>
inline void launch_timed(const char *name, F kernel, dim3 grid, dim3 block, uint32_t shmem, hipStream_t s,
                         Args... args) {
    const TimerPair t = timer_pair(name);
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, t.a, t.b, 0u, args...);
}
void timer_begin(const char *name, hipStream_t s);
void timer_end(const char *name, hipStream_t s);

inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
inline uint64_t round_up(uint64_t a, uint64_t b) { return ceil_div(a, b) * b; }

// Every device allocation the library makes goes through dev_alloc, which
// counts it (zr_device_alloc_count): the synchronous host entry points must
// reach a steady state with no allocation per call.
hipError_t dev_alloc(void **p, size_t bytes);

// ---------------------------------------------------------------------------
// Call contexts of the synchronous host-memory entry points (zr_rans_encode,
// zr_fse_compress, zr_huff_decode, ...): a non-blocking HIP stream plus device
// buffers grown on demand and kept. A call leases a context from a per-device
// pool and returns it, so concurrent host threads never share one, the only
// synchronisation is on the context's own stream (never the device), and once
// the sizes have been seen a call allocates nothing.
// ---------------------------------------------------------------------------
struct CallCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    enum { NBUF = 6 };
    void *buf[NBUF] = {};
    size_t cap[NBUF] = {};
    // host-side staging that must outlive the asynchronous copies of a call
    alignas(16) uint64_t meta[16] = {};
    std::string host_stage;
};

class CallLease {
   public:
    CallLease() = default;
    CallLease(const CallLease &) = delete;
    CallLease &operator=(const CallLease &) = delete;
    ~CallLease();  // drains the stream, returns the context to the pool
    int32_t acquire();
    // device buffer `slot` with at least `bytes` bytes (grown, never shrunk)
    int32_t get(int slot, size_t bytes, void **p);
    hipStream_t stream() const { return c_->stream; }
    CallCtx *ctx() { return c_; }
    int32_t sync();

   private:
    CallCtx *c_ = nullptr;
};
}  // namespace zr
