// Microbenchmark: cycles per dependent step of the rANS decode chain on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 chain.hip -o chain ; run: ./chain
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define ITERS 1024

template <int MODE>
__global__ void k(const uint32_t *tab_g, uint32_t *out, uint64_t *cyc, uint32_t seed) {
    __shared__ uint32_t tab[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) tab[i] = tab_g[i];
    __syncthreads();
    uint32_t x = seed + threadIdx.x * 7919u;
    x = (x & 0xFFFFFF) | 0x10000;
    uint32_t D = x * 2654435761u;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < ITERS; i++) {
        if (MODE == 0) {  // dependent v_add
            x = x + D;
        } else if (MODE == 1) {  // dependent 64-bit shift
            uint64_t t = (((uint64_t)x) << 32 | D) << (x & 24);
            x = (uint32_t)(t >> 32);
        } else if (MODE == 2) {  // dependent LDS read
            x = tab[x & 4095];
        } else if (MODE == 3) {  // full step: ffbh,and,lshl64,lshr,and,ds_read,lshr,bfe,mad
            const uint32_t sft = __builtin_clz(x | 16) & 24;
            const uint64_t t = ((((uint64_t)x) << 32) | D) << sft;
            const uint32_t hi = (uint32_t)(t >> 32);
            const uint32_t ent = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(tab) + ((hi >> 6) & 0x3FFC));
            x = __umul24(ent >> 20, hi >> 20) + ((ent >> 8) & 0xFFF);
            D = (uint32_t)t ^ ent;
        } else if (MODE == 4) {  // step without LDS
            const uint32_t sft = __builtin_clz(x | 16) & 24;
            const uint64_t t = ((((uint64_t)x) << 32) | D) << sft;
            const uint32_t hi = (uint32_t)(t >> 32);
            const uint32_t ent = hi * 0x9E3779B9u;
            x = __umul24(ent >> 20, hi >> 20) + ((ent >> 8) & 0xFFF);
            D = (uint32_t)t ^ ent;
        } else if (MODE == 5) {  // dependent ffbh+and
            x = (__builtin_clz(x | 1) & 24) + D;
        } else if (MODE == 6) {  // dependent mad24
            x = __umul24(x, D) + D;
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x ^ D;
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <int MODE>
void run(const char *name, int threads, int blocks, uint32_t *tab, uint32_t *out, uint64_t *cyc) {
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, tab, out, cyc, 12345);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, tab, out, cyc, 777);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    int nw = blocks * threads / 64;
    std::vector<uint64_t> c(nw);
    hipMemcpy(c.data(), cyc, nw * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (auto v : c) avg += v; avg /= nw;
    printf("%-28s threads/wg=%4d wgs=%4d waves/SIMD=%d : %.1f memtime-ticks/iter  kernel %.3f ms (%.1f ns/iter)\n",
           name, threads, blocks, threads / 256 * (blocks >= 256 ? blocks / 256 : 1), avg / ITERS, ms, ms * 1e6 / ITERS);
}

int main() {
    uint32_t *tab, *out; uint64_t *cyc;
    hipMalloc(&tab, 4096 * 4); hipMalloc(&out, 1 << 24); hipMalloc(&cyc, 1 << 20);
    std::vector<uint32_t> h(4096);
    for (int i = 0; i < 4096; i++) h[i] = (i * 2654435761u) & 0xFFFFFFFF | 0x00100000u;
    for (int i = 0; i < 4096; i++) h[i] = (h[i] & ~0xFFF00000u) | ((uint32_t)(16 + (i & 7)) << 20);
    hipMemcpy(tab, h.data(), 4096 * 4, hipMemcpyHostToDevice);
    for (int thr : {256, 1024}) {
        run<0>("dep v_add", thr, 256, tab, out, cyc);
        run<1>("dep lshl_b64", thr, 256, tab, out, cyc);
        run<2>("dep ds_read_b32", thr, 256, tab, out, cyc);
        run<5>("dep ffbh+and+add", thr, 256, tab, out, cyc);
        run<6>("dep mad24", thr, 256, tab, out, cyc);
        run<3>("full step", thr, 256, tab, out, cyc);
        run<4>("full step no LDS", thr, 256, tab, out, cyc);
    }
    run<3>("full step 2048thr(2wg)", 1024, 512, tab, out, cyc);
    return 0;
}
