// Does the LDS take unaligned 16-byte / 4-byte accesses (SH_MEM_CONFIG alignment
// mode)? Each lane writes 16 known bytes at byte offset 32*lane + (lane % 16)
// (a 32-B slot per lane, so no two lanes' 16 bytes overlap)
// with one ds_write_b128, then reads them back with a ds_read_b128 and with four
// ds_read_b32 at the same unaligned offsets; the host compares byte by byte.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
typedef unsigned v4u __attribute__((ext_vector_type(4)));

__global__ void k(uint32_t *out, uint64_t *cyc) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[64 * 32 + 64];
    const uint32_t l = threadIdx.x;
    for (uint32_t i = l; i < sizeof(lds); i += 64) lds[i] = 0xEE;
    __syncthreads();
    const uint32_t off = 32 * l + (l % 16);
    const uint32_t addr = (uint32_t)(uintptr_t)(lds + off);  // LDS address (local aperture offset)
    v4u v = {0x03020100u + l * 0x04040404u, 0x07060504u + l, 0x0B0A0908u + l, 0x0F0E0D0Cu + l};
    asm volatile("ds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(addr), "v"(v) : "memory");
    __syncthreads();
    v4u r;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr) : "memory");
    uint32_t r1;
    asm volatile("ds_read_b32 %0, %1 offset:4\n\ts_waitcnt lgkmcnt(0)" : "=v"(r1) : "v"(addr) : "memory");
    out[l * 8 + 0] = r.x; out[l * 8 + 1] = r.y; out[l * 8 + 2] = r.z; out[l * 8 + 3] = r.w;
    out[l * 8 + 4] = r1;
    // bytes as seen by byte reads (the ground truth of what the write stored)
    uint32_t b0 = 0, b1 = 0;
    for (int i = 0; i < 4; i++) b0 |= (uint32_t)lds[off + i] << (8 * i);
    for (int i = 0; i < 4; i++) b1 |= (uint32_t)lds[off + 4 + i] << (8 * i);
    out[l * 8 + 5] = b0; out[l * 8 + 6] = b1;
    out[l * 8 + 7] = v.x;
}

int main() {
    uint32_t *d;
    hipMalloc(&d, 64 * 8 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, nullptr);
    uint32_t h[64 * 8];
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 1; }
    int bad128 = 0, bad32 = 0, badw = 0;
    for (int l = 0; l < 64; l++) {
        const uint32_t *o = h + l * 8;
        const uint32_t vx = 0x03020100u + l * 0x04040404u, vy = 0x07060504u + l;
        if (o[5] != vx || o[6] != vy) badw++;          // the write landed at the unaligned offset
        if (o[0] != vx || o[1] != vy) bad128++;        // the b128 read returns it
        if (o[4] != vy) bad32++;                       // an unaligned b32 read returns bytes 4..7
        if (l < 4) printf("lane %d off %d: write %08x %08x | b128 %08x %08x | b32 %08x | expect %08x %08x\n", l,
                          32 * l + l % 16, o[5], o[6], o[0], o[1], o[4], vx, vy);
    }
    printf("unaligned LDS: write mismatches %d, b128 read mismatches %d, b32 read mismatches %d (of 64 lanes)\n",
           badw, bad128, bad32);
    return 0;
}
