// LDS-DMA placement test: global_load_lds_dword into [row][lane] dword rows of a
// 148 KiB LDS image, with the builtin's immediate offset folded into the LDS base.
// ./glds <mode>: 1 rows < 64 KiB, offset 0; 2 rows < 64 KiB, offsets; 3 all 33 rows (v3 pattern)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

constexpr int FW = 1024, RR = 32;
template <int I>
__device__ __forceinline__ void dma(const uint32_t *g, uint32_t *row) {
    __builtin_amdgcn_global_load_lds(g, row - I, 4, 4 * I, 0);
}

__global__ __launch_bounds__(FW) void k(const uint32_t *src, uint32_t *out, int mode) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4096 + (RR + 1) * FW];
    for (int i = threadIdx.x; i < 4096 + (RR + 1) * FW; i += FW) lds[i] = 0xDEADBEEFu;
    __syncthreads();
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t *ring = lds + 4096;
    uint32_t *wring = ring + 64 * wv;
    const uint32_t *g = src + 16 * threadIdx.x;  // lane's 64-B segment: dword i = 1000*tid + i
    if (mode == 1) {
        dma<0>(g, wring + 1 * FW);
    } else if (mode == 2) {
        dma<0>(g, wring + 1 * FW); dma<1>(g, wring + 2 * FW); dma<2>(g, wring + 3 * FW); dma<3>(g, wring + 4 * FW);
    } else {
        uint32_t *r = wring + 17 * FW;
        dma<0>(g, r + 0 * FW); dma<1>(g, r + 1 * FW); dma<2>(g, r + 2 * FW); dma<3>(g, r + 3 * FW);
        dma<4>(g, r + 4 * FW); dma<5>(g, r + 5 * FW); dma<6>(g, r + 6 * FW); dma<7>(g, r + 7 * FW);
        dma<8>(g, r + 8 * FW); dma<9>(g, r + 9 * FW); dma<10>(g, r + 10 * FW); dma<11>(g, r + 11 * FW);
        dma<12>(g, r + 12 * FW); dma<13>(g, r + 13 * FW); dma<14>(g, r + 14 * FW); dma<15>(g, r + 15 * FW);
        dma<15>(g, wring);
        r = wring + 1 * FW;
        dma<0>(g, r + 0 * FW); dma<1>(g, r + 1 * FW); dma<2>(g, r + 2 * FW); dma<3>(g, r + 3 * FW);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 4096 + (RR + 1) * FW; i += FW) out[i] = lds[i];
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 1;
    const int NW = 4096 + (RR + 1) * FW;
    uint32_t *src, *out;
    hipMalloc(&src, 16 * FW * 4); hipMalloc(&out, NW * 4);
    std::vector<uint32_t> h(16 * FW);
    for (int t = 0; t < FW; t++) for (int i = 0; i < 16; i++) h[16 * t + i] = 1000 * t + i;
    hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(FW), 0, 0, src, out, mode);
    hipError_t e = hipDeviceSynchronize();
    printf("mode %d: %s\n", mode, hipGetErrorString(e));
    if (e != hipSuccess) return 1;
    std::vector<uint32_t> o(NW);
    hipMemcpy(o.data(), out, NW * 4, hipMemcpyDeviceToHost);
    auto at = [&](int row, int t) { return o[4096 + row * FW + t]; };
    int bad = 0;
    auto expect = [&](int row, int i) {
        for (int t = 0; t < FW; t++)
            if (at(row, t) != (uint32_t)(1000 * t + i)) { if (bad++ < 5) printf("  row %d lane %d: got %u want %u\n", row, t, at(row, t), 1000 * t + i); }
    };
    if (mode == 1) expect(1, 0);
    else if (mode == 2) for (int i = 0; i < 4; i++) expect(1 + i, i);
    else { for (int i = 0; i < 16; i++) expect(17 + i, i); expect(0, 15); for (int i = 0; i < 4; i++) expect(1 + i, i); }
    int clob = 0;
    for (int j = 0; j < 4096; j++) clob += o[j] != 0xDEADBEEFu;
    printf("mode %d: %s (%d wrong), table area clobbered: %d\n", mode, bad ? "WRONG" : "ok", bad, clob);
    return bad ? 2 : 0;
}
