// Microbenchmark: the table build (tab_build, Rans64Encoder::new on the device)
// as k_tab runs it, one 256-lane workgroup, on the bench's histogram shape
// (256 symbols, ~2^20 each, uniform) and on a skewed one; per-phase times from a
// copy of zr_rans.hip compiled with ZR_TAB_STAMPS (s_memtime at each phase).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I../../zipora_amd/csrc
//          -DZR_TAB_STAMPS tabcost.hip -o tabcost -L../../zipora_amd -lzipora_amd
#include "../../zipora_amd/csrc/zr_rans.hip"
#include <cstdio>
#include <vector>

int main() {
    using namespace zr;
    uint32_t *hist;
    RansDTab *tab;
    uint64_t *st;
    hipMalloc(&hist, 1024);
    hipMalloc(&tab, sizeof(RansDTab));
    hipMalloc(&st, 64 * 8);
    for (int kind = 0; kind < 2; kind++) {
        std::vector<uint32_t> h(256);
        for (int v = 0; v < 256; v++) h[v] = kind == 0 ? 1048576 + (v * 7919 % 2001) - 1000 : (uint32_t)(268435456.0 / (1 + v) / 6.1);
        hipMemcpy(hist, h.data(), 1024, hipMemcpyHostToDevice);
        hipMemset(st, 0, 64 * 8);
        float best = 1e9;
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int r = 0; r < 20; r++) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_tab_stamped, dim3(1), dim3(256), 0, 0, hist, tab, st);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = best < ms ? best : ms;
        }
        uint64_t s[64];
        hipMemcpy(s, st, 64 * 8, hipMemcpyDeviceToHost);
        printf("%s: launch+kernel best %.2f us; phases (s_memtime ticks from start):", kind ? "skewed" : "uniform", best * 1e3);
        for (int i = 1; i < 12 && s[i]; i++) printf(" %llu", (unsigned long long)(s[i] - s[0]));
        printf("\n");
    }
    return 0;
}
