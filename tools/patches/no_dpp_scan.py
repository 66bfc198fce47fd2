# the __shfl (ds_bpermute) wave scans and sums (rounds 1-5) instead of DPP
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
i = s.index("__device__ __forceinline__ unsigned long long wave_incl_scan(unsigned long long v) {")
j = s.index("}\n", s.index("return (unsigned long long)a +", i)) + 2
s = s[:i] + """__device__ __forceinline__ unsigned long long wave_incl_scan(unsigned long long v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        unsigned long long t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}
""" + s[j:]
i = s.index("__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {")
j = s.index("}\n", s.index("<< 48);", i)) + 2
s = s[:i] + """__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor((unsigned long long)v, d, 64);
    return v;
}
""" + s[j:]
open(p, "w").write(s)
