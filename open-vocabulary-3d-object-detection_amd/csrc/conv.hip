// 3x3 convolution operand staging for the RegionCLIP backbone and res5 (SURVEY §8a
// row a15): NHWC im2col, so that every 3x3 convolution is one hipBLASLt GEMM
// (rows = output pixels, K = 9*Cin ordered (ky, kx, ci), i.e. the channels-last
// weight (Cout, 3, 3, Cin) viewed as (Cout, 9*Cin)).  The caller stages a chunk of
// ROIs/images at a time, sized to stay resident in the 256 MB Infinity Cache
// between this write and the GEMM's read.
//
// One thread moves one 16-byte run of channels (8 bf16 / 4 fp32) of one tap of one
// output pixel; consecutive threads walk the channels, then the taps, so both the
// load (a channel run of a neighbouring input pixel) and the store (the row of the
// column matrix) are coalesced.  Out-of-image taps and the K padding are zeros.
#include "common.h"

namespace {

struct alignas(16) V16 {
    uint32_t w[4];
};

__global__ void __launch_bounds__(256) im2col_vec_kernel(
    const V16* __restrict__ in, int H, int W, int CV, int stride, int Ho, int Wo, int KV, long long rows,
    V16* __restrict__ out) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= rows * KV) return;
    const int kv = (int)(t % KV);
    const long long m = t / KV;
    V16 v = {{0u, 0u, 0u, 0u}};
    if (kv < 9 * CV) {
        const int tap = kv / CV, cv = kv - tap * CV;
        const int ox = (int)(m % Wo);
        const long long q = m / Wo;
        const int oy = (int)(q % Ho);
        const long long n = q / Ho;
        const int iy = oy * stride - 1 + tap / 3, ix = ox * stride - 1 + tap % 3;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) v = in[((n * H + iy) * W + ix) * CV + cv];
    }
    out[t] = v;
}

template <typename T>
__global__ void __launch_bounds__(256) im2col_scalar_kernel(
    const T* __restrict__ in, int H, int W, int C, int stride, int Ho, int Wo, int K, long long rows,
    T* __restrict__ out) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= rows * K) return;
    const int k = (int)(t % K);
    const long long m = t / K;
    T v = (T)0;
    if (k < 9 * C) {
        const int tap = k / C, c = k - tap * C;
        const int ox = (int)(m % Wo);
        const long long q = m / Wo;
        const int oy = (int)(q % Ho);
        const long long n = q / Ho;
        const int iy = oy * stride - 1 + tap / 3, ix = ox * stride - 1 + tap % 3;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) v = in[((n * H + iy) * W + ix) * C + c];
    }
    out[t] = v;
}

}  // namespace

extern "C" int ov3d_im2col3x3(const void* in, int elem_bytes, int N, int H, int W, int C, int stride,
                              int Kpad, void* out, void* stream) {
    if (!in || !out || N <= 0 || H <= 0 || W <= 0 || C <= 0 || (stride != 1 && stride != 2) ||
        Kpad < 9 * C || (elem_bytes != 2 && elem_bytes != 4))
        return OV3D_EINVAL;
    const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
    const long long rows = (long long)N * Ho * Wo;
    hipStream_t s = ov3d_stream(stream);
    const int per16 = 16 / elem_bytes;
    if ((C % per16) == 0 && (Kpad % per16) == 0) {
        const long long total = rows * (Kpad / per16);
        if (total > 0x7fffffffLL * 256) return OV3D_EINVAL;
        im2col_vec_kernel<<<ov3d_cdiv(total, 256), 256, 0, s>>>(
            (const V16*)in, H, W, C / per16, stride, Ho, Wo, Kpad / per16, rows, (V16*)out);
    } else {
        const long long total = rows * Kpad;
        if (total > 0x7fffffffLL * 256) return OV3D_EINVAL;
        if (elem_bytes == 2)
            im2col_scalar_kernel<uint16_t><<<ov3d_cdiv(total, 256), 256, 0, s>>>(
                (const uint16_t*)in, H, W, C, stride, Ho, Wo, Kpad, rows, (uint16_t*)out);
        else
            im2col_scalar_kernel<uint32_t><<<ov3d_cdiv(total, 256), 256, 0, s>>>(
                (const uint32_t*)in, H, W, C, stride, Ho, Wo, Kpad, rows, (uint32_t*)out);
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
