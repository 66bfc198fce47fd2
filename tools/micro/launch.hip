// Microbenchmark: kernel duration vs in-kernel span for big-LDS 1024-thread
// workgroups, with and without 256 MiB of output stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int MODE, int LDSW>
__global__ __launch_bounds__(1024) void k(uint8_t *out, uint64_t *rec, uint32_t N, uint32_t steps) {
    __shared__ uint32_t lds[LDSW];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    uint32_t v = lds[(threadIdx.x * 7) & 1023];
    uint8_t *o = out + (size_t)(blockIdx.x / 4) * (4u << 20) + (blockIdx.x % 4) * 1024;
    if (MODE == 1) {  // byte stores, row pattern k*N + s
        for (uint32_t k = 0; k < steps; k++) { o[(size_t)k * N + threadIdx.x] = (uint8_t)(v + k); }
    } else if (MODE == 2) {  // 16-B stores, contiguous per workgroup
        uint4 *o4 = reinterpret_cast<uint4 *>(out + (size_t)blockIdx.x * (1u << 20));
        for (uint32_t k = 0; k < 64; k++) o4[k * 1024 + threadIdx.x] = make_uint4(v, k, v, k);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { rec[2 * blockIdx.x] = t0; rec[2 * blockIdx.x + 1] = t1; }
}

template <int MODE, int LDSW>
void run(const char *name, uint8_t *out, uint64_t *rec, int reps = 3) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int r = 0; r < reps; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k<MODE, LDSW>), dim3(256), dim3(1024), 0, 0, out, rec, 4096u, 1024u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        std::vector<uint64_t> h(512);
        hipMemcpy(h.data(), rec, 4096, hipMemcpyDeviceToHost);
        uint64_t mn = ~0ull, mx = 0;
        for (int i = 0; i < 256; i++) { mn = std::min(mn, h[2 * i]); mx = std::max(mx, h[2 * i + 1]); }
        printf("%-34s event %.1f us, in-kernel span %.1f us\n", name, ms * 1e3, (mx - mn) / 100.0);
    }
}

int main() {
    uint8_t *out; uint64_t *rec;
    hipMalloc(&out, 512u << 20); hipMalloc(&rec, 4096);
    run<0, 1024>("empty, 4 KiB LDS", out, rec);
    run<0, 37888>("empty, 148 KiB LDS", out, rec);
    run<1, 37888>("byte rows 256 MiB, 148 KiB LDS", out, rec);
    run<1, 1024>("byte rows 256 MiB, 4 KiB LDS", out, rec);
    run<2, 37888>("x4 stores 256 MiB, 148 KiB LDS", out, rec);
    return 0;
}
