// Calibrates rocprofv3's FETCH_SIZE for the access shapes of the rANS decoders
// (MI355X_MICROARCH.md: FETCH_SIZE counts a wide coalesced streaming read at
// half its bytes; other shapes are uncalibrated). Each kernel reads a known
// number of bytes from a 1 GiB buffer (beyond the 256 MiB Infinity Cache), once:
//   k_stream : 16 B per lane, lanes contiguous (the guide's calibrated shape)
//   k_seg64  : one lane per 768-B region, its 64-B segments top-down, one
//              segment (4 x 16-B loads of the lane) per round, the regions of
//              adjacent lanes adjacent: the record decoder's refill shape
//   k_seg128 : the same with a whole 128-B line (8 loads) per round
// Run under rocprofv3 --pmc FETCH_SIZE (and TCC_EA0_RDREQ_sum /
// TCC_EA0_RDREQ_32B_sum in a pass of their own) and compare with the bytes
// printed. Build: hipcc -O3 --offload-arch=gfx950 fetch_cal.hip -o fetch_cal
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr uint64_t NBYTES = 1ull << 30;
constexpr uint32_t REG = 768;  // bytes per lane region

__global__ __launch_bounds__(256) void k_stream(const v4u *q, uint64_t units, uint32_t *out) {
    uint32_t acc = 0;
    const uint64_t T = (uint64_t)gridDim.x * 256;
    for (uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x; u < units; u += T) {
        const v4u v = q[u];
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// lanes: regions in flight at once (persistent: each lane walks regions
// lane, lane + lanes, ...); SEG: bytes per round (64 or 128)
template <uint32_t SEG>
__global__ __launch_bounds__(1024) void k_seg(const uint8_t *p, uint64_t nreg, uint32_t *out) {
    uint32_t acc = 0;
    const uint64_t lanes = (uint64_t)gridDim.x * 1024;
    for (uint64_t r = (uint64_t)blockIdx.x * 1024 + threadIdx.x; r < nreg; r += lanes) {
        const uint8_t *base = p + r * REG;
        for (int s = REG / SEG - 1; s >= 0; s--) {
            const v4u *q = reinterpret_cast<const v4u *>(base + s * SEG);
            v4u v[SEG / 16];
#pragma unroll
            for (uint32_t k = 0; k < SEG / 16; k++) v[k] = q[k];
#pragma unroll
            for (uint32_t k = 0; k < SEG / 16; k++) acc ^= v[k].x + v[k].y + v[k].z + v[k].w;
            // some work per round, as a decoder's 64 steps per segment
#pragma unroll 1
            for (int i = 0; i < 64; i++) acc = acc * 1664525u + 1013904223u;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    void *d, *o;
    if (hipMalloc(&d, NBYTES) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    hipMemset(d, 1, NBYTES);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const uint64_t nreg = NBYTES / REG;
    auto timed = [&](const char *name, uint64_t bytes, auto launch) {
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-9s bytes %12llu  %8.1f us  %5.2f TB/s\n", name, (unsigned long long)bytes, 1e3 * ms,
               bytes / (ms * 1e-3) / 1e12);
    };
    for (int rep = 0; rep < 2; rep++) {
        timed("stream", NBYTES, [&]() { k_stream<<<4096, 256>>>((const v4u *)d, NBYTES / 16, (uint32_t *)o); });
        timed("seg64", nreg * REG, [&]() { k_seg<64><<<256, 1024>>>((const uint8_t *)d, nreg, (uint32_t *)o); });
        timed("seg128", nreg * REG, [&]() { k_seg<128><<<256, 1024>>>((const uint8_t *)d, nreg, (uint32_t *)o); });
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
