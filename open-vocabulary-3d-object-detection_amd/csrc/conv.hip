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

#include <hip/hip_bf16.h>

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

// The same with 32-bit index arithmetic (rows * KV < 2^31: every chunk the caller stages);
// the 64-bit divisions of the general form cost more VALU than the 16-byte move itself.
template <bool NT>
__global__ void __launch_bounds__(256) im2col_vec32_kernel(
    const V16* __restrict__ in, int H, int W, int CV, int stride, int Ho, int Wo, int KV, int total,
    V16* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int m = t / KV, kv = t - m * KV;
    V16 v = {{0u, 0u, 0u, 0u}};
    if (kv < 9 * CV) {
        const int tap = kv / CV, cv = kv - tap * CV;
        const int q = m / Wo, ox = m - q * Wo;
        const int n = q / Ho, oy = q - n * Ho;
        const int ky = tap / 3, kx = tap - ky * 3;
        const int iy = oy * stride - 1 + ky, ix = ox * stride - 1 + kx;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W)
            v = in[((long long)(n * H + iy) * W + ix) * CV + cv];
    }
    if (NT) {
        uint32_t* o = out[t].w;
#pragma unroll
        for (int e = 0; e < 4; ++e) __builtin_nontemporal_store(v.w[e], o + e);
    } else {
        out[t] = v;
    }
}

// y = act(y + bias + residual) in place on (rows, cols) rows of 16-byte runs: the 1x1
// convolution closing a bottleneck block after a plain GEMM (one pass instead of copying the
// residual into the GEMM's C, then a bias add and a ReLU pass).
template <typename T>
__device__ __forceinline__ float to_f(T v);
template <>
__device__ __forceinline__ float to_f<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f<__hip_bfloat16>(__hip_bfloat16 v) { return __bfloat162float(v); }

template <typename T>
__global__ void __launch_bounds__(256) bias_residual_act_kernel(
    T* __restrict__ y, const T* __restrict__ bias, const T* __restrict__ res, int cv_per_row,
    long long total, int relu) {
    constexpr int E = 16 / sizeof(T);
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int c0 = (int)(t % cv_per_row) * E;
    V16 a = reinterpret_cast<const V16*>(y)[t];
    const V16 r = reinterpret_cast<const V16*>(res)[t];
    const V16 b = *reinterpret_cast<const V16*>(bias + c0);
    const T* av = reinterpret_cast<const T*>(&a);
    const T* rv = reinterpret_cast<const T*>(&r);
    const T* bv = reinterpret_cast<const T*>(&b);
    V16 o;
    T* ov = reinterpret_cast<T*>(&o);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        // (conv + bias) + identity in fp32, rounded once (BN's shift folded into the bias)
        float v = (to_f(av[e]) + to_f(bv[e])) + to_f(rv[e]);
        if (relu) v = fmaxf(v, 0.f);
        ov[e] = (T)v;
    }
    reinterpret_cast<V16*>(y)[t] = o;
}

// 2x2 / stride-2 average pool on NHWC (the anti-aliasing pool of the ModifiedResNet's strided
// blocks and stem): one thread per 16-byte channel run of one output pixel, fp32 sum in
// torch's NHWC order (((0 + x00) + x01) + x10) + x11, then / 4, one rounding.
template <typename T>
__global__ void __launch_bounds__(256) avgpool2_kernel(
    const T* __restrict__ in, int H, int W, int CV, int Ho, int Wo, int total, T* __restrict__ out) {
    constexpr int E = 16 / sizeof(T);
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int m = t / CV, cv = t - m * CV;
    const int q = m / Wo, ox = m - q * Wo;
    const int n = q / Ho, oy = q - n * Ho;
    const V16* src = reinterpret_cast<const V16*>(in);
    const long long r0 = ((long long)(n * H + 2 * oy) * W + 2 * ox) * CV + cv;
    const long long rstride = (long long)W * CV;
    const V16 v00 = src[r0], v01 = src[r0 + CV], v10 = src[r0 + rstride], v11 = src[r0 + rstride + CV];
    const T* a = reinterpret_cast<const T*>(&v00);
    const T* b = reinterpret_cast<const T*>(&v01);
    const T* c = reinterpret_cast<const T*>(&v10);
    const T* d = reinterpret_cast<const T*>(&v11);
    V16 o;
    T* ov = reinterpret_cast<T*>(&o);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        float sum = 0.f;
        sum += to_f(a[e]);
        sum += to_f(b[e]);
        sum += to_f(c[e]);
        sum += to_f(d[e]);
        ov[e] = (T)(sum / 4.f);
    }
    reinterpret_cast<V16*>(out)[t] = o;
}

// Token rows of CLIP's AttentionPool2d in one pass: t[r, 0] = mean_j x[r, j] + pos[0] and
// t[r, 1 + j] = x[r, j] + pos[1 + j]; one thread per 16-byte channel run of one ROI, fp32 mean
// (token order) rounded to T before the position add, as mean().to(T) + pos does.
template <typename T>
__global__ void __launch_bounds__(256) attnpool_tokens_kernel(
    const T* __restrict__ x, int ntok, int CV, int total, const T* __restrict__ pos,
    T* __restrict__ t) {
    constexpr int E = 16 / sizeof(T);
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= total) return;
    const int r = g / CV, cv = g - r * CV;
    const V16* xs = reinterpret_cast<const V16*>(x) + (long long)r * ntok * CV + cv;
    const V16* ps = reinterpret_cast<const V16*>(pos) + cv;
    V16* ts = reinterpret_cast<V16*>(t) + (long long)r * (ntok + 1) * CV + cv;
    float sum[E];
#pragma unroll
    for (int e = 0; e < E; ++e) sum[e] = 0.f;
    for (int j = 0; j < ntok; ++j) {
        const V16 a = xs[(long long)j * CV];
        const V16 p = ps[(long long)(j + 1) * CV];
        const T* av = reinterpret_cast<const T*>(&a);
        const T* pv = reinterpret_cast<const T*>(&p);
        V16 o;
        T* ov = reinterpret_cast<T*>(&o);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            sum[e] += to_f(av[e]);
            ov[e] = (T)(to_f(av[e]) + to_f(pv[e]));
        }
        ts[(long long)(j + 1) * CV] = o;
    }
    const V16 p0 = ps[0];
    const T* pv = reinterpret_cast<const T*>(&p0);
    V16 o;
    T* ov = reinterpret_cast<T*>(&o);
#pragma unroll
    for (int e = 0; e < E; ++e) ov[e] = (T)(to_f((T)(sum[e] / (float)ntok)) + to_f(pv[e]));
    ts[0] = o;
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
        if (total <= 0x7fffffffLL && (long long)N * H * W * (C / per16) <= 0x7fffffffLL)
        {
            // columns larger than the 256 MB Infinity Cache go to HBM with non-temporal stores
            // (whole-conv staging: C5 step 67.7 -> 66.7-67.0 ms); smaller chunks stay cached
            if (total * 16 > (256LL << 20))
                im2col_vec32_kernel<true><<<ov3d_cdiv(total, 256), 256, 0, s>>>(
                    (const V16*)in, H, W, C / per16, stride, Ho, Wo, Kpad / per16, (int)total, (V16*)out);
            else
                im2col_vec32_kernel<false><<<ov3d_cdiv(total, 256), 256, 0, s>>>(
                    (const V16*)in, H, W, C / per16, stride, Ho, Wo, Kpad / per16, (int)total, (V16*)out);
        }
        else
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

extern "C" int ov3d_bias_residual_act(void* y, int elem_bytes, long long rows, int cols,
                                      const void* bias, const void* residual, int relu,
                                      void* stream) {
    if (!y || !bias || !residual || rows < 0 || cols <= 0 || (elem_bytes != 2 && elem_bytes != 4))
        return OV3D_EINVAL;
    const int per16 = 16 / elem_bytes;
    if (cols % per16 || ((uintptr_t)y | (uintptr_t)bias | (uintptr_t)residual) & 15) return OV3D_EINVAL;
    const long long total = rows * (cols / per16);
    if (total == 0) return OV3D_OK;
    if (total > 0x7fffffffLL * 256) return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    if (elem_bytes == 2)
        bias_residual_act_kernel<__hip_bfloat16><<<ov3d_cdiv(total, 256), 256, 0, s>>>(
            (__hip_bfloat16*)y, (const __hip_bfloat16*)bias, (const __hip_bfloat16*)residual,
            cols / per16, total, relu);
    else
        bias_residual_act_kernel<float><<<ov3d_cdiv(total, 256), 256, 0, s>>>(
            (float*)y, (const float*)bias, (const float*)residual, cols / per16, total, relu);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_avgpool2_nhwc(const void* in, int elem_bytes, int N, int H, int W, int C, void* out,
                                  void* stream) {
    if (!in || !out || N < 0 || H < 2 || W < 2 || C <= 0 || (elem_bytes != 2 && elem_bytes != 4))
        return OV3D_EINVAL;
    const int per16 = 16 / elem_bytes;
    if (C % per16 || ((uintptr_t)in | (uintptr_t)out) & 15) return OV3D_EINVAL;
    const int Ho = H / 2, Wo = W / 2, CV = C / per16;
    const long long total = (long long)N * Ho * Wo * CV;
    if (total == 0) return OV3D_OK;
    if (total > 0x7fffffffLL || (long long)N * H * W * CV > 0x7fffffffLL) return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    if (elem_bytes == 2)
        avgpool2_kernel<__hip_bfloat16><<<ov3d_cdiv(total, 256), 256, 0, s>>>(
            (const __hip_bfloat16*)in, H, W, CV, Ho, Wo, (int)total, (__hip_bfloat16*)out);
    else
        avgpool2_kernel<float><<<ov3d_cdiv(total, 256), 256, 0, s>>>(
            (const float*)in, H, W, CV, Ho, Wo, (int)total, (float*)out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_attnpool_tokens(const void* x, int elem_bytes, int R, int ntok, int C,
                                    const void* pos, void* t, void* stream) {
    if (!x || !pos || !t || R < 0 || ntok <= 0 || C <= 0 || (elem_bytes != 2 && elem_bytes != 4))
        return OV3D_EINVAL;
    const int per16 = 16 / elem_bytes;
    if (C % per16 || ((uintptr_t)x | (uintptr_t)pos | (uintptr_t)t) & 15) return OV3D_EINVAL;
    const long long total = (long long)R * (C / per16);
    if (total == 0) return OV3D_OK;
    if (total > 0x7fffffffLL) return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    if (elem_bytes == 2)
        attnpool_tokens_kernel<__hip_bfloat16><<<ov3d_cdiv(total, 256), 256, 0, s>>>(
            (const __hip_bfloat16*)x, ntok, C / per16, (int)total, (const __hip_bfloat16*)pos,
            (__hip_bfloat16*)t);
    else
        attnpool_tokens_kernel<float><<<ov3d_cdiv(total, 256), 256, 0, s>>>(
            (const float*)x, ntok, C / per16, (int)total, (const float*)pos, (float*)t);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
