// Counter-based dropout keep mask over channels-last rows, shared by the row kernels
// (bnrows.hip, resnorm.hip): keep(r, c) is a hash of (seed, site, r, c), so a backward
// regenerates the forward's mask instead of storing it.  Channels are hashed in pairs
// (one 32-bit hash, two 16-bit halves); a half >= thresh = round(p * 65536) keeps.
#pragma once
#include "common.h"

namespace rowdrop {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// 24-bit multiplies (v_mul_u32_u24 issues at the full VALU rate)
__device__ __forceinline__ uint32_t mix24(uint32_t x) {
    x ^= x >> 16;
    x = __umul24(x, 0x7feb35u) ^ (x >> 24);
    x ^= x >> 15;
    x = __umul24(x, 0x846ca7u) ^ (x >> 24);
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t seed_mix(const int64_t* seed, uint32_t site) {
    const uint64_t s = (uint64_t)*seed;
    return mix32((uint32_t)s ^ mix32((uint32_t)(s >> 32) + site * 0x9E3779B9u));
}
__device__ __forceinline__ uint32_t row_base(uint32_t seedmix, long long r) {
    return mix32(seedmix ^ ((uint32_t)r * 0xC2B2AE35u));
}
// keep decisions of channels c..c+7 of row r (c a multiple of 8)
__device__ __forceinline__ void keep8(uint32_t rowbase, int c, uint32_t thresh, bool* keep) {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        const uint32_t h = mix24(rowbase + (uint32_t)((c + j) >> 1) * 0x27D4EB2Fu);
        keep[j] = (h & 0xffffu) >= thresh;
        keep[j + 1] = (h >> 16) >= thresh;
    }
}
inline uint32_t thresh(float p) {
    return p > 0.f ? (uint32_t)fminf(rintf(p * 65536.0f), 65535.0f) : 0u;
}

}  // namespace rowdrop
