// Shared helpers for the ov3d HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ov3d.h"

#define OV3D_LAUNCH_CHECK()                              \
    do {                                                 \
        hipError_t e_ = hipGetLastError();               \
        if (e_ != hipSuccess) return OV3D_ELAUNCH;       \
    } while (0)

static inline hipStream_t ov3d_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline int ov3d_cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// Wave64 lane mask of lanes strictly below this one.
__device__ __forceinline__ unsigned long long lanemask_lt() {
    const unsigned lane = threadIdx.x & 63u;
    return lane == 0 ? 0ull : (~0ull >> (64u - lane));
}

// host: reserve 2 stamp words per wave of the next launch while stamps are armed (attn.hip
// ov3d_stamps_arm); kind 0 / 1 / 2 attention fwd / dQ / dK-dV, 3 gemm256; null when disarmed,
// below the armed min_work, or out of space
unsigned long long* ov3d_stamp_take(int kind, long long work, long long waves);

// In-kernel launch stamps (measurement only: bench.py's in-step timing of the roofline kernel).
// Lane 0 of every wave writes the wall clock (100 MHz) at entry (end = 0) and exit (end = 1)
// into its own 2-word slot of a buffer that nothing else in the kernel reads; st == null: off.
__device__ __forceinline__ void ov3d_stamp(unsigned long long* st, int end) {
    if (st && (threadIdx.x & 63) == 0) {
        const long long wg = blockIdx.x + (long long)gridDim.x * (blockIdx.y + (long long)gridDim.y * blockIdx.z);
        st[2 * (wg * (blockDim.x >> 6) + (threadIdx.x >> 6)) + end] = wall_clock64();
    }
}
