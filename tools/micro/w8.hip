// Microbenchmark: the rANS decode tile loop at 4 and 8 waves per SIMD, with the
// ring refilled three ways. Synthetic lock-step streams: a uniform table
// (f = 16 for every symbol), so every step consumes exactly one byte.
//   MODE 0: no refills (ring bytes stale): the floor of step + window + stores
//   MODE 2: LDS-DMA (global_load_lds_dwordx4) 16-B chunks, ring [4 rows][64 lanes][16 B]
//           per wave, chunk boundaries relative to each stream's end (unaligned sources)
//   MODE 5: as 2, chunks 16-B aligned in absolute addresses (rows differ per lane:
//           up to four DMA instructions per boundary, one per row)
//   MODE 3: VGPR staging (global_load_dwordx4), landed at the next boundary by four
//           ds_write_b32 into a [16 dword rows][1024 lanes] ring
// Build: hipcc --offload-arch=gfx950 -O3 w8.hip -o w8 ; run: ./w8
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr uint32_t FW = 1024, TT = 16, YB = 1u << 20;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void *base) {
    const uint64_t p = (uint64_t)base;
    const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)p) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(p >> 32)) << 32);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(u), 0, 0x7FFFFFFF, 0x00020000);
}

template <int MODE, int W, int BS = 0, int T8 = 0>
__global__ __launch_bounds__(FW, W) void kdec(const uint8_t *__restrict__ enc, uint8_t *__restrict__ raw,
                                               const uint32_t *__restrict__ tabg, uint32_t N, uint32_t S) {
    // T8 (MODE 0 only): 8-byte entries {f | sym << 24, bias} (32 KiB) and an 8-row ring
    constexpr uint32_t TABW = T8 ? 8192 : 4096, RROWS = T8 ? 8 : 16;
    __shared__ __attribute__((aligned(16))) uint32_t lds[TABW + RROWS * FW];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (T8) {
        for (uint32_t i = tid; i < 4096; i += FW) {
            const uint32_t e = tabg[i];
            lds[2 * i] = (e >> 20) | (e << 24);
            lds[2 * i + 1] = (e >> 8) & 0xFFF;
        }
    } else {
        for (uint32_t i = tid; i < 4096; i += FW) lds[i] = tabg[i];
    }
    const uint32_t s = blockIdx.x * FW + tid;
    const uint32_t end = 64 + (s + 1) * S;  // stream s: enc[64 + s*S, 64 + (s+1)*S)
    uint32_t x = ((s * 2654435761u) & 0xFFFFFFu) | 0x10000u;
    char *const ringb = reinterpret_cast<char *>(lds + TABW);
    constexpr bool DMA = MODE == 2 || MODE == 5 || MODE == 6 || MODE == 7, REL = MODE != 5;
    // DMA modes: the wave's ring, 4 rows of 1 KiB; lane slot lane * 16
    char *const wring = ringb + wv * 4096;
    const uint32_t lb = (uint32_t)(uintptr_t)(wring) + lane * 16;  // (LDS byte address)
    // coordinate of the position: REL: y = P - end + YB; else the absolute byte P
    const uint32_t cofs = REL ? YB - end : 0u;
    uint32_t p8 = (end + cofs) << 3;
    uint32_t ylo;  // lowest byte requested (coordinate), chunk-aligned
    const uintptr_t gb = (uintptr_t)enc - (int64_t)(int32_t)cofs;  // coordinate -> address
    v4u stg = {0, 0, 0, 0};
    bool pnd = false;  // MODE 3: a chunk in the staging registers
    auto dma_row = [&](uint32_t y0, bool m) __attribute__((always_inline)) {
        // y0: chunk base coordinate (16-aligned); row (y0 >> 4) & 3
        const uint32_t r = (y0 >> 4) & 3;
        // MODE 6: the same instruction stream, sources in a 512 KiB L2-resident region
        // (lane-distinct lines): timing only
        const uintptr_t gsrc = MODE == 6 ? (uintptr_t)enc + ((tid * 128 + (y0 & 0x70)) & 0x7FFFF) : gb + y0;
        for (uint32_t rr = 0; rr < 4; rr++) {
            const bool mm = m && r == rr;
            if (__builtin_amdgcn_ballot_w64(mm)) {
                if (mm)
                    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(gsrc),
                                                     reinterpret_cast<void *>(wring + rr * 1024), 16, 0, 0);
            }
        }
    };
    if constexpr (DMA) {
        const uint32_t ytop = ((end + cofs - 1) & ~15u) + 16;
        ylo = ytop - 64;
        for (uint32_t k = 0; k < 4; k++) dma_row(ylo + 16 * k, true);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (MODE == 3) {
        const uint32_t ytop = ((end - 1) & ~15u) + 16;
        ylo = ytop - 64;
        for (uint32_t k = 0; k < 4; k++) {
            const v4u c = *reinterpret_cast<const v4u *>(enc + ylo + 16 * k);
            const uint32_t r0 = ((ylo + 16 * k) >> 2) & 15;
            uint32_t *p = reinterpret_cast<uint32_t *>(ringb) + tid;
            p[((r0 + 0) & 15) * FW] = c.x; p[((r0 + 1) & 15) * FW] = c.y;
            p[((r0 + 2) & 15) * FW] = c.z; p[((r0 + 3) & 15) * FW] = c.w;
        }
    } else {
        ylo = 0;
    }
    __syncthreads();
    auto readD = [&](uint32_t q8) -> uint32_t __attribute__((always_inline)) {
        if constexpr (DMA) {
            const uint32_t yd = q8 >> 3;
            const uint32_t a1 = (((yd >> 4) & 3) << 10) | (yd & 12) | lb;
            const uint32_t y0 = yd - 4;
            const uint32_t a0 = (((y0 >> 4) & 3) << 10) | (y0 & 12) | lb;
            const uint32_t d1 = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>(a1);
            const uint32_t d0 = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>(a0);
            return __builtin_amdgcn_alignbit(d1, d0, q8);
        } else {
            constexpr uint32_t RM = (RROWS - 1) << 12;
            const uint32_t o1 = (q8 << 7) & RM, o0 = (o1 - 4096u) & RM;
            const char *base = ringb + tid * 4;
            return __builtin_amdgcn_alignbit(*reinterpret_cast<const uint32_t *>(base + o1),
                                             *reinterpret_cast<const uint32_t *>(base + o0), q8);
        }
    };
    auto step = [&](uint32_t D, uint32_t &hi, uint32_t &lo, uint32_t &sft) -> uint32_t __attribute__((always_inline)) {
        sft = __builtin_clz(x) & 24;
        const uint64_t t = ((((uint64_t)x) << 32) | D) << sft;
        hi = (uint32_t)(t >> 32);
        lo = (uint32_t)t;
        if (T8) {
            typedef uint32_t v2u_ __attribute__((ext_vector_type(2)));
            const v2u_ e2 = *reinterpret_cast<const v2u_ *>(reinterpret_cast<const char *>(lds) + ((hi >> 5) & 0x7FF8));
            x = __umul24(e2.x, hi >> 20) + e2.y;
            return e2.x >> 24;
        }
        const uint32_t ent = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(lds) + ((hi >> 6) & 0x3FFC));
        x = __umul24(ent >> 20, hi >> 20) + ((ent >> 8) & 0xFFF);
        return ent;
    };
    uint8_t *outb = raw + blockIdx.x * FW;
    const uint32_t voff_pk = (tid & ~3u) + (tid & 3u) * N;
    const uint32_t psel1 = (tid & 2) ? 0x03020706u : 0x05040100u;
    const uint32_t psel2 = (tid & 1) ? 0x03070105u : 0x06020400u;
    const uintptr_t dummy = (uintptr_t)tabg + 64 * wv;
    const uint32_t ntile = S / TT;
    for (uint32_t t = 0; t < ntile; t++) {
        if (MODE != 0 && t >= 1) {
            // the refill of boundary t - 1; younger: tile t-1's 4 stores
            asm volatile("s_waitcnt vmcnt(4)" : "+v"(stg)::"memory");
            if (MODE == 3 && pnd) {
                // land: rows of [ylo, ylo + 16) (ylo already lowered at issue)
                const uint32_t r0 = (ylo >> 2) & 15;
                uint32_t *p = reinterpret_cast<uint32_t *>(ringb) + tid;
                p[((r0 + 0) & 15) * FW] = stg.x; p[((r0 + 1) & 15) * FW] = stg.y;
                p[((r0 + 2) & 15) * FW] = stg.z; p[((r0 + 3) & 15) * FW] = stg.w;
            }
        }
        if (MODE != 0) {
            const uint32_t y = p8 >> 3;
            const bool issue = (int32_t)(y - ylo) < 48;
            if constexpr (MODE == 7) {
                // timing only: 64 B (4 chunks of one half line) every 4th boundary
                if ((t & 3) == 0) {
                    ylo -= 64;
                    for (uint32_t k = 0; k < 4; k++) dma_row(ylo + 16 * k, true);
                }
            } else if constexpr (DMA) {
                if (issue) ylo -= 16;
                dma_row(ylo, issue);
            } else {
                if (issue) ylo -= 16;
                pnd = issue;
                const uintptr_t g = issue ? (uintptr_t)enc + ylo : dummy;
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(stg) : "v"(g) : "memory");
            }
        }
        uint32_t D = readD(p8);
        const __amdgpu_buffer_rsrc_t orsrc = rsrc(outb + (uint64_t)t * TT * N);
        uint32_t row = 0, pk0 = 0;
#pragma unroll
        for (int j = 0; j < (int)TT / 2; j++) {
            uint32_t hA, lA, sA, hB, lB, sB;
            const uint32_t eA = step(D, hA, lA, sA);
            const uint32_t eB = step(__builtin_amdgcn_alignbyte(hA, lA, 1), hB, lB, sB);
            uint32_t used;
            asm("v_add3_u32 %0, %1, %2, -16" : "=v"(used) : "v"(sA), "v"(sB));
            p8 -= used;
            if (j + 1 < (int)TT / 2) D = readD(p8);
            if (BS) {
                const __amdgpu_buffer_rsrc_t br = orsrc;
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)eA, br, tid, row, 0);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)eB, br, tid, row + N, 0);
            } else if ((j & 1) == 0) {
                pk0 = __builtin_amdgcn_perm(eB, eA, 0x0c0c0400u);
            } else {
                uint32_t q = __builtin_amdgcn_perm(eB, eA, 0x04000c0cu) | pk0;
                uint32_t xx = (uint32_t)__builtin_amdgcn_mov_dpp((int)q, 0x4E, 0xF, 0xF, false);
                q = __builtin_amdgcn_perm(xx, q, psel1);
                xx = (uint32_t)__builtin_amdgcn_mov_dpp((int)q, 0xB1, 0xF, 0xF, false);
                q = __builtin_amdgcn_perm(xx, q, psel2);
                __builtin_amdgcn_raw_buffer_store_b32(q, orsrc, voff_pk, row - 2 * N, 0);
            }
            row += 2 * N;
        }
    }
}

// host reference of one stream (the same synthetic format), for checking
static void ref_stream(const std::vector<uint8_t> &enc, const std::vector<uint32_t> &tab, uint32_t s, uint32_t S,
                       std::vector<uint8_t> &out) {
    uint64_t X = ((s * 2654435761u) & 0xFFFFFFu) | 0x10000u;
    uint64_t pos = 64 + (uint64_t)(s + 1) * S;
    out.resize(S);
    for (uint32_t k = 0; k < S; k++) {
        while (X < (1u << 16)) X = (X << 8) | enc[--pos];
        const uint32_t slot = X & 4095, e = tab[slot];
        X = (uint64_t)(e >> 20) * (X >> 12) + ((e >> 8) & 0xFFF);
        out[k] = (uint8_t)e;
    }
}

template <int MODE, int W, int BS = 0, int T8 = 0>
void run(const char *name, const uint8_t *enc, uint8_t *raw, const uint32_t *tab, const std::vector<uint8_t> &henc,
         const std::vector<uint32_t> &htab) {
    const uint32_t N = 256u * 256u * W, S = (1u << 28) / N;
    auto k = kdec<MODE, W, BS, T8>;
    hipMemset(raw, 0, 1u << 28);
    const size_t dyn = W == 4 ? 16384 : 0;
    if (T8 && W == 8) { /* 32 KiB table + 32 KiB ring: two per CU */ }  // W = 4: one workgroup per CU (LDS > 80 KiB)
    hipLaunchKernelGGL(k, dim3(N / FW), dim3(FW), dyn, 0, enc, raw, tab, N, S);
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) { printf("%s: %s\n", name, hipGetErrorString(e)); exit(1); }
    // check a few streams
    int bad = 0;
    if (MODE != 0 && MODE != 6 && MODE != 7) {
        std::vector<uint8_t> o(1u << 28);
        hipMemcpy(o.data(), raw, 1u << 28, hipMemcpyDeviceToHost);
        std::vector<uint8_t> r;
        for (uint32_t s : {0u, 1u, 63u, 1000u, N / 2 + 7, N - 1}) {
            ref_stream(henc, htab, s, S, r);
            for (uint32_t kk = 0; kk < S; kk++) bad += o[(size_t)kk * N + s] != r[kk];
        }
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    float best = 1e9;
    for (int rep = 0; rep < 5; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, dim3(N / FW), dim3(FW), dyn, 0, enc, raw, tab, N, S);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double bytes = 2.0 * (1u << 28) + 12.0 * N;
    printf("%-34s waves/SIMD=%d N=2^%d steps=%4u: %7.1f us  %5.1f ns/step  %.2f TB/s  frac %.3f  mismatches %d\n", name, W,
           __builtin_ctz(N), S, best * 1e3, best * 1e6 / S, bytes / best / 1e9, bytes / best / 1e9 / 8.0, bad);
}

int main(int argc, char **argv) {
    const size_t EN = (1u << 28) + 4096;
    std::vector<uint8_t> henc(EN);
    uint64_t r = 0x9E3779B97F4A7C15ull;
    for (auto &b : henc) { r ^= r << 13; r ^= r >> 7; r ^= r << 17; b = (uint8_t)(r >> 32); }
    std::vector<uint32_t> htab(4096);
    for (uint32_t i = 0; i < 4096; i++) htab[i] = (i >> 4) | ((i & 15) << 8) | (16u << 20);
    uint8_t *enc, *raw; uint32_t *tab;
    hipMalloc(&enc, EN); hipMalloc(&raw, 1u << 28); hipMalloc(&tab, 4096 * 4);
    hipMemcpy(enc, henc.data(), EN, hipMemcpyHostToDevice);
    hipMemcpy(tab, htab.data(), 4096 * 4, hipMemcpyHostToDevice);
    const int which = argc > 1 ? atoi(argv[1]) : -1;
    if (which < 0 || which == 0) {
        run<0, 4>("no refill", enc, raw, tab, henc, htab); run<0, 8>("no refill", enc, raw, tab, henc, htab);
        run<0, 8, 1>("no refill, byte stores", enc, raw, tab, henc, htab);
        run<0, 8, 0, 1>("no refill, 8-B entries", enc, raw, tab, henc, htab);
        run<0, 8, 1, 1>("no refill, 8-B entries, byte st", enc, raw, tab, henc, htab);
    }
    if (which < 0 || which == 3) { run<3, 4>("VGPR staging, dword rows", enc, raw, tab, henc, htab); run<3, 8>("VGPR staging, dword rows", enc, raw, tab, henc, htab); }
    if (which < 0 || which == 2) { run<2, 4>("DMA x4, stream-relative chunks", enc, raw, tab, henc, htab); run<2, 8>("DMA x4, stream-relative chunks", enc, raw, tab, henc, htab); }
    if (which < 0 || which == 6) { run<6, 4>("DMA x4, L2-resident sources", enc, raw, tab, henc, htab); run<6, 8>("DMA x4, L2-resident sources", enc, raw, tab, henc, htab); }
    if (which < 0 || which == 7) { run<7, 4>("DMA x4, 64 B per 64 steps", enc, raw, tab, henc, htab); run<7, 8>("DMA x4, 64 B per 64 steps", enc, raw, tab, henc, htab); }
    if (which < 0 || which == 5) { run<5, 4>("DMA x4, aligned chunks", enc, raw, tab, henc, htab); run<5, 8>("DMA x4, aligned chunks", enc, raw, tab, henc, htab); }
    return 0;
}
