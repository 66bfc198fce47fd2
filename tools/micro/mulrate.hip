// Microbenchmark: issue cost of integer multiplies on gfx950 (one wave per
// SIMD and four), 8 independent chains per lane so latency is hidden.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096

template <int OP>
__global__ void k(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
#pragma unroll
    for (int c = 0; c < 8; c++) a[c] = seed * (threadIdx.x + 1) + c * 7919u;
    const uint32_t b = seed | 0x10001;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < 8; c++) {
            if (OP == 0) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 1) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 2) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 4) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 5) {
                uint64_t t;
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(t) : "v"(a[c]), "v"(b) : "vcc");
                a[c] = (uint32_t)t;
            }
            if (OP == 6) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(*reinterpret_cast<uint64_t *>(&a[c & ~1])) : "v"(b));
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) acc ^= a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
void run(const char *name, uint32_t *out, int wps) {
    // 256 workgroups x (64 * wps) threads: wps waves per CU... one workgroup per CU
    const int threads = 64 * wps;
    hipLaunchKernelGGL((k<OP>), dim3(256), dim3(threads), 0, 0, out, 1u);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    float best = 1e9;
    for (int r = 0; r < 3; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k<OP>), dim3(256), dim3(threads), 0, 0, out, 3u + r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        best = best < ms ? best : ms;
    }
    // cycles per instruction per SIMD at ~2.4 GHz: waves per SIMD = wps / 4 (wps >= 4)
    const double instr_per_simd = (double)ITERS * 8 * (wps >= 4 ? wps / 4 : 1);
    printf("%-18s waves/CU=%2d : %.1f us, %.2f ns per instruction per SIMD (%.1f cycles at 2.4 GHz)\n", name, wps,
           best * 1e3, best * 1e6 / instr_per_simd, best * 1e6 / instr_per_simd * 2.4);
}

int main() {
    uint32_t *out;
    hipMalloc(&out, 256 * 1024 * 4);
    for (int wps : {4, 16}) {
        run<3>("v_add_u32", out, wps);
        run<2>("v_mul_u32_u24", out, wps);
        run<1>("v_mul_hi_u32_u24", out, wps);
        run<0>("v_mul_hi_u32", out, wps);
        run<4>("v_mul_lo_u32", out, wps);
        run<5>("v_mad_u64_u32", out, wps);
        run<6>("v_lshlrev_b64", out, wps);
    }
    return 0;
}
