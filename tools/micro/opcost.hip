// Microbenchmark: issue cost per SIMD of the VALU instructions of the rANS
// decode step on gfx950, at 4 and 8 waves per SIMD, 8 independent chains per
// lane (latency hidden). Reported: cycles per wave-instruction per SIMD at the
// clock the run measures with s_memtime (cycles / instruction).
// Build: hipcc --offload-arch=gfx950 -O3 opcost.hip -o opcost ; run: ./opcost
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define ITERS 2048

template <int OP>
__global__ __launch_bounds__(1024) void k(uint32_t *out, uint64_t *cyc, uint32_t seed) {
    __shared__ uint32_t tab[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) tab[i] = i * 2654435761u;
    __syncthreads();
    uint32_t a[8];
#pragma unroll
    for (int c = 0; c < 8; c++) a[c] = seed * (threadIdx.x + 1) + c * 7919u;
    const uint32_t b = seed | 0x10001;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < 8; c++) {
            if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 1) asm volatile("v_ffbh_u32 %0, %0" : "+v"(a[c]));
            if (OP == 2) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(*reinterpret_cast<uint64_t *>(&a[c & ~1])) : "v"(b));
            if (OP == 3) asm volatile("v_alignbit_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 4) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(a[c]) : "v"(b));
            if (OP == 5) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 6) asm volatile("v_bfe_u32 %0, %0, 8, 12" : "+v"(a[c]));
            if (OP == 7) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 8) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 9) asm volatile("v_add3_u32 %0, %0, %1, -16" : "+v"(a[c]) : "v"(b));
            if (OP == 10) asm volatile("v_lshrrev_b32 %0, 6, %0" : "+v"(a[c]));
            if (OP == 11) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "+v"(a[c]));
            if (OP == 12) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 13) {  // dependent pairs on a 4 KiB LDS table (random reads)
                const uint32_t v = tab[a[c] & 4095];
                a[c] = v ^ (a[c] >> 3);
            }
            if (OP == 14) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 15) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[c]) : "v"(b));
            if (OP == 16) asm volatile("v_and_b32 %0, 0x7ff8, %0" : "+v"(a[c]));
            if (OP == 17) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a[c]) : "s"(b));
            if (OP == 18) {  // a VOP3 and a VOP2 alternating
                if (c & 1) asm volatile("v_alignbit_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
                else asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            }
            if (OP == 19) {  // one VOP3 per three VOP2
                if ((c & 3) == 0) asm volatile("v_alignbit_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
                else asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            }
            if (OP == 20) asm volatile("v_add_u32 %0, 0x1000, %0" : "+v"(a[c]));
            if (OP == 21) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 22) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 23) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a[c]) : "v"(b));
            if (OP == 24) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 25) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 26) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 27) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 28) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a[c]));
            if (OP == 29) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 30) asm volatile("v_cmp_lt_u32_e64 s[40:41], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(a[c]) : "v"(b) : "s40", "s41");
            if (OP == 31) asm volatile("v_cmp_lt_u32_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[c]) : "v"(b) : "vcc");
            if (OP == 32) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 33) asm volatile("v_med3_u32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if (OP == 34) asm volatile("v_lshrrev_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD" : "+v"(a[c]) : "v"(b));
            if (OP == 35) asm volatile("v_sub_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, 0, vcc" : "+v"(a[c]) : "v"(b) : "vcc");
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) acc ^= a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char *name, uint32_t *out, uint64_t *cyc, int wps) {
    // wps waves per SIMD: 256 * wps / 4 workgroups of 1024 threads (16 waves: 4 per SIMD)
    const int blocks = 256 * wps / 4;
    hipLaunchKernelGGL((k<OP>), dim3(blocks), dim3(1024), 0, 0, out, cyc, 1u);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e9;
    for (int r = 0; r < 3; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k<OP>), dim3(blocks), dim3(1024), 0, 0, out, cyc, 3u + r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = best < ms ? best : ms;
    }
    uint64_t c0 = 0;
    hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);
    const double instr_per_simd = (double)ITERS * 8 * wps;
    // s_memtime ticks at the shader clock: cycles per instruction per SIMD from workgroup 0's span
    printf("%-16s waves/SIMD=%d : %8.1f us  %.2f cyc/instr/SIMD (memtime)  %.2f at 2.4 GHz\n", name, wps, best * 1e3,
           (double)c0 / (ITERS * 8 * wps), best * 1e6 / instr_per_simd * 2.4);
}

int main() {
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, 1 << 26);
    hipMalloc(&cyc, 1 << 16);
    for (int w : {4}) {
        run<25>("v_mul_hi_u32", out, cyc, w);
        run<26>("v_mul_lo_u32", out, cyc, w);
        run<27>("v_mul_f32", out, cyc, w);
        run<28>("v_cvt_f32_u32", out, cyc, w);
        run<29>("v_mul_hi_u32_u24", out, cyc, w);
        run<30>("cmp_e64+cndmask (2)", out, cyc, w);
        run<31>("cmp_e32+cndmask (2)", out, cyc, w);
        run<32>("v_max_u32", out, cyc, w);
        run<33>("v_med3_u32", out, cyc, w);
        run<34>("lshrrev_sdwa", out, cyc, w);
        run<35>("sub_co+addc (2)", out, cyc, w);
        run<7>("v_mad_u32_u24", out, cyc, w);
        run<6>("v_bfe_u32", out, cyc, w);
        run<0>("v_add_u32", out, cyc, w);
    }
    if (getenv("OPCOST_ALL") == nullptr) return 0;
    for (int w : {8}) {
        run<16>("v_and literal", out, cyc, w);
        run<17>("v_and sgpr", out, cyc, w);
        run<20>("v_add literal", out, cyc, w);
        run<21>("v_xor", out, cyc, w);
        run<22>("v_sub", out, cyc, w);
        run<23>("v_lshlrev vgpr", out, cyc, w);
        run<24>("v_or3", out, cyc, w);
        run<18>("alignbit|add 1:1", out, cyc, w);
        run<19>("alignbit|add 1:3", out, cyc, w);
    }
    for (int w : {4, 8}) {
        run<0>("v_add_u32", out, cyc, w);
        run<1>("v_ffbh_u32", out, cyc, w);
        run<2>("v_lshlrev_b64", out, cyc, w);
        run<3>("v_alignbit_b32", out, cyc, w);
        run<4>("v_alignbyte_b32", out, cyc, w);
        run<5>("v_perm_b32", out, cyc, w);
        run<6>("v_bfe_u32", out, cyc, w);
        run<7>("v_mad_u32_u24", out, cyc, w);
        run<14>("v_mul_u32_u24", out, cyc, w);
        run<8>("v_and_or_b32", out, cyc, w);
        run<9>("v_add3_u32", out, cyc, w);
        run<10>("v_lshrrev_b32", out, cyc, w);
        run<12>("v_lshl_or_b32", out, cyc, w);
        run<11>("v_mov_dpp", out, cyc, w);
        run<15>("v_cndmask_b32", out, cyc, w);
        run<13>("ds_read_b32 rnd", out, cyc, w);
    }
    return 0;
}
