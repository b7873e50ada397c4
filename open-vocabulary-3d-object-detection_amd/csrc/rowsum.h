// Row reductions over 32 lanes (a 256-channel row at 8 channels a lane) for the LayerNorm row
// kernels (resnorm.hip, lngemm.hip).  The xor butterfly in ascending order (1, 2, 4, 8, 16)
// on VALU lane moves: quad permutes for 1 and 2, the 8- / 16-lane mirrors for 4 and 8 (equal
// to the xor partner once the value is uniform over the smaller group), v_permlane16_swap for
// 16.  Every lane ends with the same sum (IEEE addition is commutative); the moves cost a few
// cycles each where a ds_bpermute / ds_swizzle round trip through the LDS pipe costs ~100.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>


template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF,
                                                              0xF, true));
}

__device__ __forceinline__ float row_sum32_lanes(float v) {
    v += dpp_mov<0xB1>(v);    // quad_perm(1, 0, 3, 2): lane ^ 1
    v += dpp_mov<0x4E>(v);    // quad_perm(2, 3, 0, 1): lane ^ 2
    v += dpp_mov<0x141>(v);   // row_half_mirror: the other quad of the 8
    v += dpp_mov<0x140>(v);   // row_mirror: the other 8 of the 16
    const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, v),
                                                    __builtin_bit_cast(uint32_t, v), false, false);
    return __builtin_bit_cast(float, (uint32_t)r[0]) + __builtin_bit_cast(float, (uint32_t)r[1]);
}
