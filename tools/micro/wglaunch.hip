// Microbenchmark: the cost of a workgroup's life at the compaction's shape
// (256 lanes, 19.6 KiB LDS, 8 workgroups per CU, 16384 workgroups): empty, with
// its LDS, with one dependent global load round trip + barrier, with two.
// Build: hipcc --offload-arch=gfx950 -O3 wglaunch.hip -o wglaunch
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k(const uint32_t *in, uint32_t *out) {
    __shared__ uint32_t lds[MODE >= 1 ? 5000 : 1];
    uint32_t v = threadIdx.x;
    if (MODE >= 2) {
        v = in[(blockIdx.x * 64 + (threadIdx.x & 63)) & 0xFFFFF];
        lds[threadIdx.x] = v;
        __syncthreads();
        v = lds[(threadIdx.x + 1) & 255];
    }
    if (MODE >= 3) {
        v = in[(v * 64 + blockIdx.x) & 0xFFFFF];
        lds[threadIdx.x + 256] = v;
        __syncthreads();
        v += lds[256 + ((threadIdx.x + 1) & 255)];
    }
    if (MODE == 1) lds[threadIdx.x] = v, __syncthreads(), v = lds[255 - threadIdx.x];
    if (threadIdx.x < 64) out[blockIdx.x * 64 + threadIdx.x] = v;
}

template <int MODE>
void run(const char *name, const uint32_t *in, uint32_t *out, int nwg) {
    hipLaunchKernelGGL((k<MODE>), dim3(nwg), dim3(256), 0, 0, in, out);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k<MODE>), dim3(nwg), dim3(256), 0, 0, in, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = best < ms ? best : ms;
    }
    printf("%-28s %6d workgroups: %8.2f us\n", name, nwg, best * 1e3);
}

int main() {
    uint32_t *in, *out;
    hipMalloc(&in, 4 << 20);
    hipMalloc(&out, 64 << 20);
    hipMemset(in, 0, 4 << 20);
    for (int nwg : {2048, 16384, 65536}) {
        run<0>("empty", in, out, nwg);
        run<1>("20 KiB LDS + barrier", in, out, nwg);
        run<2>("+ 1 load round trip", in, out, nwg);
        run<3>("+ 2 dependent round trips", in, out, nwg);
    }
    return 0;
}
