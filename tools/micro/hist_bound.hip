// What bounds a byte histogram pass over 256 MiB (k_hist's loop): the same
// grid-stride 16-B loads (a) counted into 32 bank-spread LDS copies with one
// ds_add per byte, as k_hist does, (b) with a plain LDS store per byte
// instead of the atomic, (c) only summed in registers (the load ceiling),
// (d) one plain LDS store per 4 bytes.
// Build: hipcc -O3 --offload-arch=gfx950 hist_bound.hip -o hist_bound
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void k(const v4u *q, uint64_t units, uint32_t *out) {
    __shared__ uint32_t h[256 * 32];
    for (int i = threadIdx.x; i < 256 * 32; i += 256) h[i] = 0;
    __syncthreads();
    const uint32_t cp = threadIdx.x & 31;
    uint32_t acc = 0;
    auto add4 = [&](uint32_t w) {
        for (int j = 0; j < 4; j++) {
            const uint32_t b = (w >> (8 * j)) & 0xFF;
            if (MODE == 0) atomicAdd(&h[(b << 5) + cp], 1u);
            else if (MODE == 1) h[(b << 5) + cp] = w;
            else if (MODE == 3 && j == 0) h[(b << 5) + cp] = w;  // one store per 4 bytes
            else acc += b;
        }
    };
    const uint64_t T = (uint64_t)gridDim.x * 256;
    for (uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x; u < units; u += 2 * T) {
        const v4u a = __builtin_nontemporal_load(q + u);
        const v4u c = u + T < units ? __builtin_nontemporal_load(q + u + T) : v4u{0, 0, 0, 0};
        add4(a.x); add4(a.y); add4(a.z); add4(a.w);
        add4(c.x); add4(c.y); add4(c.z); add4(c.w);
    }
    __syncthreads();
    if (MODE == 2) {
        atomicAdd(&out[threadIdx.x], acc);  // keeps the loads
    } else {
        uint32_t s = 0;
        for (int k2 = 0; k2 < 32; k2++) s += h[(threadIdx.x << 5) + ((k2 + threadIdx.x) & 31)];
        atomicAdd(&out[threadIdx.x], s);
    }
}

int main() {
    const uint64_t n = 256ull << 20, units = n / 16;
    std::vector<uint8_t> host(n);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < n; i++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        host[i] = (uint8_t)x;
    }
    void *d, *o;
    hipMalloc(&d, n);
    hipMalloc(&o, 256 * 4);
    hipMemcpy(d, host.data(), n, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[4] = {"lds atomic per byte (k_hist)", "plain lds store per byte", "loads only (sum)",
                            "plain lds store per 4 bytes"};
    for (int grid : {1024, 2048, 4096}) {
        for (int m = 0; m < 4; m++) {
            auto launch = [&]() {
                if (m == 0) k<0><<<grid, 256>>>((const v4u *)d, units, (uint32_t *)o);
                if (m == 1) k<1><<<grid, 256>>>((const v4u *)d, units, (uint32_t *)o);
                if (m == 2) k<2><<<grid, 256>>>((const v4u *)d, units, (uint32_t *)o);
                if (m == 3) k<3><<<grid, 256>>>((const v4u *)d, units, (uint32_t *)o);
            };
            for (int w = 0; w < 3; w++) launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            const int R = 20;
            for (int r = 0; r < R; r++) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = 1e3 * ms / R;
            printf("grid %5d  %-30s %8.1f us  %6.2f TB/s\n", grid, names[m], us, n / (us * 1e-6) / 1e12);
        }
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    return 0;
}
