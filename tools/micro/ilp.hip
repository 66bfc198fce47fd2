// Microbenchmark: decode-step chains per lane (ILP) at a fixed 1024 chains per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define ITERS 1024

template <int C, int LDSREAD>
__global__ void k(const uint32_t *tab_g, uint32_t *out, uint64_t *cyc, uint32_t seed) {
    __shared__ uint32_t tab[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) tab[i] = tab_g[i];
    __syncthreads();
    uint32_t x[C], D[C];
#pragma unroll
    for (int c = 0; c < C; c++) {
        x[c] = ((seed + (threadIdx.x * C + c) * 7919u) & 0xFFFFFF) | 0x10000;
        D[c] = x[c] * 2654435761u;
    }
#pragma unroll 8
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < C; c++) {
            const uint32_t sft = __builtin_clz(x[c] | 16) & 24;
            const uint64_t t = ((((uint64_t)x[c]) << 32) | D[c]) << sft;
            const uint32_t hi = (uint32_t)(t >> 32);
            uint32_t ent;
            if (LDSREAD)
                ent = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(tab) + ((hi >> 6) & 0x3FFC));
            else
                ent = hi * 0x9E3779B9u;
            x[c] = __umul24(ent >> 20, hi >> 20) + ((ent >> 8) & 0xFFF);
            D[c] = (uint32_t)t ^ ent;
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < C; c++) acc ^= x[c] ^ D[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int C, int LDSREAD>
void run(const char *name, uint32_t *tab, uint32_t *out, uint64_t *cyc) {
    const int threads = 1024 / C;
    hipLaunchKernelGGL((k<C, LDSREAD>), dim3(256), dim3(threads), 0, 0, tab, out, cyc, 1);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    float best = 1e9;
    for (int r = 0; r < 3; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k<C, LDSREAD>), dim3(256), dim3(threads), 0, 0, tab, out, cyc, 777 + r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        best = std::min(best, ms);
    }
    printf("%-22s chains/lane=%d waves/CU=%2d : %.1f us for %d steps x 1024 chains/CU (%.1f ns/step)\n",
           name, C, 16 / C, best * 1e3, ITERS, best * 1e6 / ITERS);
}

int main() {
    uint32_t *tab, *out; uint64_t *cyc;
    hipMalloc(&tab, 4096 * 4); hipMalloc(&out, 1 << 24); hipMalloc(&cyc, 1 << 20);
    std::vector<uint32_t> h(4096);
    for (int i = 0; i < 4096; i++) h[i] = (((i * 2654435761u) >> 8) & 0x000FFF00u) | ((uint32_t)(16 + (i & 7)) << 20) | (i & 0xFF);
    hipMemcpy(tab, h.data(), 4096 * 4, hipMemcpyHostToDevice);
    run<1, 1>("step+LDS", tab, out, cyc);
    run<2, 1>("step+LDS", tab, out, cyc);
    run<4, 1>("step+LDS", tab, out, cyc);
    run<8, 1>("step+LDS", tab, out, cyc);
    run<1, 0>("step, no LDS", tab, out, cyc);
    run<2, 0>("step, no LDS", tab, out, cyc);
    run<4, 0>("step, no LDS", tab, out, cyc);
    return 0;
}
