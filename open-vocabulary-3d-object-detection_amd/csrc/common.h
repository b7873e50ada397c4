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
