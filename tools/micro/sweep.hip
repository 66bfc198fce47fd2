// Microbenchmark: read bandwidth of a 256 MiB device buffer by access order.
//   mode 0: each wave reads its own contiguous 64 KiB chunk (k_hist's items),
//           eight 16-B loads per lane in flight, rounds of 8 KiB per wave
//   mode 1: the whole grid sweeps the buffer in order: wave-load k of wave w
//           reads the 1 KiB unit k * W + w (W = waves in the grid)
// Each lane XOR-folds what it reads (one store per lane at the end), so the
// kernel is bound by the reads alone. Prints GB/s per mode and grid.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void k(const v4u *in, uint64_t units, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4, w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    uint32_t acc = 0;
    if (MODE == 0) {
        const uint64_t per = units / W;  // units of 1 KiB per wave (64 for 4096 waves)
        const v4u *p = in + (w * per) * 64 + lane;
        for (uint64_t u = 0; u < per; u += 8) {
            v4u v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) v[k] = __builtin_nontemporal_load(p + (u + k) * 64);
#pragma unroll
            for (int k = 0; k < 8; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        }
    } else {
        for (uint64_t u = w; u < units; u += 8 * W) {
            v4u v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint64_t uu = u + k * W;
                v[k] = uu < units ? __builtin_nontemporal_load(in + uu * 64 + lane) : v4u{0, 0, 0, 0};
            }
#pragma unroll
            for (int k = 0; k < 8; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        }
    }
    out[w * 64 + lane] = acc;
}

int main() {
    const size_t bytes = 256ull << 20, units = bytes >> 10;
    v4u *in;
    uint32_t *out;
    hipMalloc(&in, bytes);
    hipMalloc(&out, 64ull << 20);
    hipMemset(in, 1, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grids[] = {1024, 2048, 4096};
    for (int mode = 0; mode < 2; mode++) {
        for (int g : grids) {
            if (mode == 0 && (units % ((size_t)g * 4 * 8))) continue;
            auto kern = mode ? k<1> : k<0>;
            for (int r = 0; r < 3; r++) hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, in, units, out);
            hipEventRecord(a, 0);
            const int reps = 20;
            for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, in, units, out);
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            printf("mode %d grid %5d: %.4f ms  %.1f GB/s\n", mode, g, ms / reps, bytes / (ms / reps * 1e-3) / 1e9);
        }
    }
    hipFree(in);
    hipFree(out);
    return 0;
}
