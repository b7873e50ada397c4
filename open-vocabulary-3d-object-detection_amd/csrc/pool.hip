// Max over the nsample neighbours of a set-abstraction layer's output rows (the
// F.max_pool2d(kernel [1, nsample]) of pointnet2 PointnetSAModuleVotes, reference
// models/model_3detr.py:353-362 / 385-391), for the SA modules the fused MFMA kernels do not
// take (the masked encoder's interim SA: 256 features + xyz in, gradient to the features).
//
// Rows are channels-last bf16 (P*S, C): pooled row p is the max over rows p*S .. p*S+S-1.
// Forward: a thread per (p, 8-channel run) reads the S rows' 16-byte runs, keeps the max and
// the FIRST row that holds it (max_pool2d's window order), writes the pooled run and the
// arg rows (uint8).  Backward: a thread per (p, 8-channel run) writes the S rows of the
// dense (P*S, C) gradient: the pooled gradient on the arg row, zero elsewhere (each row
// is written exactly once: no atomics, no zero-fill pass).
// BN form (ov3d_nbr_max_bnrelu_fwd): the rows are the LAST layer's pre-BatchNorm outputs y and
// the pooled values are z = bf16(relu(y * scale + shift)) (the ov3d_rows_bn_apply arithmetic,
// training BN without dropout), so z is never stored; its backward is the pooled-gradient mode
// of ov3d_rows_bn_bwd (csrc/bnrows.hip), which rebuilds this dense gradient row by row.
#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint8_t u8x8 __attribute__((ext_vector_type(8)));

__global__ void __launch_bounds__(256) nbr_max_fwd_kernel(const bf16* __restrict__ y, long long P,
                                                          int S, int C, bf16* __restrict__ out,
                                                          uint8_t* __restrict__ arg) {
    const int runs = C / 8;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= P * runs) return;
    const long long p = t / runs;
    const int c0 = (int)(t - p * runs) * 8;
    const bf16* src = y + p * S * C + c0;
    float m[8];
    u8x8 a;
    {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(src);
#pragma unroll
        for (int j = 0; j < 8; ++j) { m[j] = (float)v[j]; a[j] = 0; }
    }
    for (int s = 1; s < S; ++s) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(src + (size_t)s * C);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float f = (float)v[j];
            // strictly greater keeps the first maximum; a NaN wins like max_pool2d's
            const bool take = f > m[j] || (f != f && m[j] == m[j]);
            m[j] = take ? f : m[j];
            a[j] = take ? (uint8_t)s : a[j];
        }
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)m[j];
    *reinterpret_cast<bf16x8*>(out + p * C + c0) = o;
    *reinterpret_cast<u8x8*>(arg + p * C + c0) = a;
}

// z = bf16(relu(y * scale + shift)) per element, then the first maximum over the S rows; four
// rows' loads in flight at a time (one 16-byte load per row and thread otherwise serialises)
__global__ void __launch_bounds__(256) nbr_max_bnrelu_fwd_kernel(
    const bf16* __restrict__ y, long long P, int S, int C, const float* __restrict__ scale,
    const float* __restrict__ shift, bf16* __restrict__ out, uint8_t* __restrict__ arg) {
    const int runs = C / 8;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= P * runs) return;
    const long long p = t / runs;
    const int c0 = (int)(t - p * runs) * 8;
    const bf16* src = y + p * S * C + c0;
    float sc[8], sh[8];
    {
        const float4 a0 = *reinterpret_cast<const float4*>(scale + c0), a1 = *reinterpret_cast<const float4*>(scale + c0 + 4);
        const float4 b0 = *reinterpret_cast<const float4*>(shift + c0), b1 = *reinterpret_cast<const float4*>(shift + c0 + 4);
        sc[0] = a0.x; sc[1] = a0.y; sc[2] = a0.z; sc[3] = a0.w; sc[4] = a1.x; sc[5] = a1.y; sc[6] = a1.z; sc[7] = a1.w;
        sh[0] = b0.x; sh[1] = b0.y; sh[2] = b0.z; sh[3] = b0.w; sh[4] = b1.x; sh[5] = b1.y; sh[6] = b1.z; sh[7] = b1.w;
    }
    float m[8];
    u8x8 a;
#pragma unroll
    for (int j = 0; j < 8; ++j) { m[j] = -1.f; a[j] = 0; }   // every z >= 0: row 0 always takes
    auto take = [&](const bf16x8& v, int s) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float z = (float)(bf16)fmaxf(fmaf((float)v[j], sc[j], sh[j]), 0.f);
            const bool tk = z > m[j];   // strictly greater keeps the first maximum (z is never NaN)
            m[j] = tk ? z : m[j];
            a[j] = tk ? (uint8_t)s : a[j];
        }
    };
    int s = 0;
    for (; s + 4 <= S; s += 4) {
        bf16x8 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const bf16x8*>(src + (size_t)(s + u) * C);
#pragma unroll
        for (int u = 0; u < 4; ++u) take(v[u], s + u);
    }
    for (; s < S; ++s) take(*reinterpret_cast<const bf16x8*>(src + (size_t)s * C), s);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)m[j];
    *reinterpret_cast<bf16x8*>(out + p * C + c0) = o;
    *reinterpret_cast<u8x8*>(arg + p * C + c0) = a;
}

__global__ void __launch_bounds__(256) nbr_max_bwd_kernel(const bf16* __restrict__ g,
                                                          const uint8_t* __restrict__ arg,
                                                          long long P, int S, int C,
                                                          bf16* __restrict__ dy) {
    const int runs = C / 8;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= P * runs) return;
    const long long p = t / runs;
    const int c0 = (int)(t - p * runs) * 8;
    const bf16x8 gv = *reinterpret_cast<const bf16x8*>(g + p * C + c0);
    const u8x8 a = *reinterpret_cast<const u8x8*>(arg + p * C + c0);
    bf16* dst = dy + p * S * C + c0;
    for (int s = 0; s < S; ++s) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = a[j] == s ? gv[j] : (bf16)0.f;
        *reinterpret_cast<bf16x8*>(dst + (size_t)s * C) = o;
    }
}

}  // namespace

extern "C" int ov3d_nbr_max_fwd(const void* y, long long P, int S, int C, void* out,
                                uint8_t* arg, void* stream) {
    if (!y || !out || !arg || P < 0 || S <= 0 || S > 256 || C <= 0 || C % 8) return OV3D_EINVAL;
    if (P == 0) return OV3D_OK;
    const long long n = P * (C / 8);
    hipLaunchKernelGGL(nbr_max_fwd_kernel, dim3(ov3d_cdiv(n, 256)), dim3(256), 0,
                       ov3d_stream(stream), (const bf16*)y, P, S, C, (bf16*)out, arg);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_nbr_max_bwd(const void* g, const uint8_t* arg, long long P, int S, int C,
                                void* dy, void* stream) {
    if (!g || !arg || !dy || P < 0 || S <= 0 || S > 256 || C <= 0 || C % 8) return OV3D_EINVAL;
    if (P == 0) return OV3D_OK;
    const long long n = P * (C / 8);
    hipLaunchKernelGGL(nbr_max_bwd_kernel, dim3(ov3d_cdiv(n, 256)), dim3(256), 0,
                       ov3d_stream(stream), (const bf16*)g, arg, P, S, C, (bf16*)dy);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_nbr_max_bnrelu_fwd(const void* y, long long P, int S, int C, const float* scale,
                                       const float* shift, void* out, uint8_t* arg, void* stream) {
    if (!y || !out || !arg || !scale || !shift || P < 0 || S <= 0 || S > 256 || C <= 0 || C % 8 ||
        ((uintptr_t)y | (uintptr_t)out | (uintptr_t)scale | (uintptr_t)shift) % 16 || (uintptr_t)arg % 8)
        return OV3D_EINVAL;
    if (P == 0) return OV3D_OK;
    const long long n = P * (C / 8);
    hipLaunchKernelGGL(nbr_max_bnrelu_fwd_kernel, dim3(ov3d_cdiv(n, 256)), dim3(256), 0,
                       ov3d_stream(stream), (const bf16*)y, P, S, C, scale, shift, (bf16*)out, arg);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
