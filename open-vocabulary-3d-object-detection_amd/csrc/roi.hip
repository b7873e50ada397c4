// RegionCLIP ROI-feature path: image preprocessing and
// ROIAlignV2 for CLIPFastRCNN.inference as called at criterion.py:397.
//
// Layout: every feature map is channels-last (NHWC) so that one ROI sample is a
// contiguous run of C values: a thread owns 8 (bf16) or 4 (fp32) consecutive
// channels of one output bin, so a wave covers a 1 KB run of channels of that bin
// and the four bilinear corners of each sample are four coalesced row segments.
// The output (R, P, P, C) is the row layout the res5 GEMMs consume directly.
//
// Arithmetic restates torchvision/detectron2 roi_align_forward_kernel_impl
// (aligned=True, adaptive sampling_ratio=0) operation by operation (file built
// with -ffp-contract=off), so fp32 results are bit-identical to
// oracle/ov3d_oracle.c:ov3d_roi_align_cpu.
#include "common.h"

namespace {

typedef __bf16 bf16;

template <typename T>
__device__ __forceinline__ float ld(const T* p) { return (float)*p; }

// One output bin's sampling geometry (roi_align_forward_kernel_impl prologue).
struct Bin {
    float y0, x0, bh, bw;  // roi_start + p*bin_size, bin sizes
    int gh, gw;            // roi_bin_grid
    float count;
};

__device__ __forceinline__ Bin bin_geometry(const float* box, float scale, int aligned, int P,
                                            int ph, int pw, int sampling_ratio) {
    const float offset = aligned ? 0.5f : 0.f;
    const float sw = box[0] * scale - offset;
    const float sh = box[1] * scale - offset;
    const float ew = box[2] * scale - offset;
    const float eh = box[3] * scale - offset;
    float rw = ew - sw, rh = eh - sh;
    if (!aligned) {
        rw = fmaxf(rw, 1.f);
        rh = fmaxf(rh, 1.f);
    }
    Bin b;
    b.bh = rh / (float)P;
    b.bw = rw / (float)P;
    b.gh = sampling_ratio > 0 ? sampling_ratio : (int)ceilf(rh / (float)P);
    b.gw = sampling_ratio > 0 ? sampling_ratio : (int)ceilf(rw / (float)P);
    b.count = (float)max(b.gh * b.gw, 1);
    b.y0 = sh + (float)ph * b.bh;
    b.x0 = sw + (float)pw * b.bw;
    return b;
}

// bilinear_interpolate (torchvision roi_align_kernel.cu) on VEC channels at once.
template <typename T, int VEC>
__device__ __forceinline__ void bilinear_acc(const T* __restrict__ f, int H, int W, int C, float y,
                                             float x, float* acc) {
    if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) return;  // adds 0
    if (y <= 0) y = 0;
    if (x <= 0) x = 0;
    int yl = (int)y, xl = (int)x, yh, xh;
    if (yl >= H - 1) {
        yh = yl = H - 1;
        y = (float)yl;
    } else {
        yh = yl + 1;
    }
    if (xl >= W - 1) {
        xh = xl = W - 1;
        x = (float)xl;
    } else {
        xh = xl + 1;
    }
    const float ly = y - (float)yl, lx = x - (float)xl;
    const float hy = 1.f - ly, hx = 1.f - lx;
    const float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
    // one 16-byte load per corner (VEC * sizeof(T) == 16, channel runs 16-byte aligned)
    const uint4 u1 = *reinterpret_cast<const uint4*>(f + ((size_t)yl * W + xl) * C);
    const uint4 u2 = *reinterpret_cast<const uint4*>(f + ((size_t)yl * W + xh) * C);
    const uint4 u3 = *reinterpret_cast<const uint4*>(f + ((size_t)yh * W + xl) * C);
    const uint4 u4 = *reinterpret_cast<const uint4*>(f + ((size_t)yh * W + xh) * C);
    const T* p1 = reinterpret_cast<const T*>(&u1);
    const T* p2 = reinterpret_cast<const T*>(&u2);
    const T* p3 = reinterpret_cast<const T*>(&u3);
    const T* p4 = reinterpret_cast<const T*>(&u4);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        const float v = w1 * ld(p1 + j) + w2 * ld(p2 + j) + w3 * ld(p3 + j) + w4 * ld(p4 + j);
        acc[j] += v;
    }
}

// One thread per (roi, ph, pw, channel vector); channel vector fastest.
// IDX: the index type of the thread -> (roi, ph, pw, cv) split (int when the grid fits: the
// 64-bit divisions cost more than the bin's arithmetic).
template <typename T, int VEC, typename IDX>
__global__ void __launch_bounds__(256) roi_align_kernel(
    const T* __restrict__ feat, int H, int W, int C, const float* __restrict__ boxes, int R,
    int per_image, int nimages, float scale, int P, int sampling_ratio, int aligned,
    T* __restrict__ out) {
    static_assert(VEC * sizeof(T) == 16, "one 16-byte channel run per thread");
    const int CV = C / VEC;
    const IDX total = (IDX)R * P * P * CV;
    const IDX t = (IDX)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int cv = (int)(t % CV);
    IDX q = t / CV;
    const int pw = (int)(q % P);
    q /= P;
    const int ph = (int)(q % P);
    const int r = (int)(q / P);
    const int img = (r / per_image) % nimages;
    const Bin b = bin_geometry(boxes + 4 * (size_t)r, scale, aligned, P, ph, pw, sampling_ratio);
    const T* f = feat + (size_t)img * H * W * C + cv * VEC;
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
    for (int iy = 0; iy < b.gh; ++iy) {
        const float y = b.y0 + (float)(iy + .5f) * b.bh / (float)b.gh;
        for (int ix = 0; ix < b.gw; ++ix) {
            const float x = b.x0 + (float)(ix + .5f) * b.bw / (float)b.gw;
            bilinear_acc<T, VEC>(f, H, W, C, y, x, acc);
        }
    }
    uint4 ov;
    T* oe = reinterpret_cast<T*>(&ov);
#pragma unroll
    for (int j = 0; j < VEC; ++j) oe[j] = (T)(acc[j] / b.count);
    *reinterpret_cast<uint4*>(out + (((size_t)r * P + ph) * P + pw) * C + cv * VEC) = ov;
}

// The same bins, a 2x2 block of them per thread, plus their 2x2 average pool (the res5 identity
// path's nn.AvgPool2d(2) over the ROIAlign output, torch's arithmetic as ov3d_avgpool2_nhwc:
// fp32 (((0 + b00) + b01) + b10) + b11 of the rounded bins, / 4) written beside them, so the
// pool does not read the (R, P, P, C) output back.  P even, 32-bit indices.
template <typename T, int VEC>
__global__ void __launch_bounds__(256) roi_align_pool2_kernel(
    const T* __restrict__ feat, int H, int W, int C, const float* __restrict__ boxes, int R,
    int per_image, int nimages, float scale, int P, int sampling_ratio, int aligned,
    T* __restrict__ out, T* __restrict__ pooled) {
    static_assert(VEC * sizeof(T) == 16, "one 16-byte channel run per thread");
    const int CV = C / VEC, P2 = P / 2;
    const int total = R * P2 * P2 * CV;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int cv = t % CV;
    int q = t / CV;
    const int pw2 = q % P2;
    q /= P2;
    const int ph2 = q % P2;
    const int r = q / P2;
    const int img = (r / per_image) % nimages;
    const T* f = feat + (size_t)img * H * W * C + cv * VEC;
    float psum[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) psum[j] = 0.f;
    for (int dy = 0; dy < 2; ++dy) {
        for (int dx = 0; dx < 2; ++dx) {
            const int ph = 2 * ph2 + dy, pw = 2 * pw2 + dx;
            const Bin b = bin_geometry(boxes + 4 * (size_t)r, scale, aligned, P, ph, pw, sampling_ratio);
            float acc[VEC];
#pragma unroll
            for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
            for (int iy = 0; iy < b.gh; ++iy) {
                const float y = b.y0 + (float)(iy + .5f) * b.bh / (float)b.gh;
                for (int ix = 0; ix < b.gw; ++ix) {
                    const float x = b.x0 + (float)(ix + .5f) * b.bw / (float)b.gw;
                    bilinear_acc<T, VEC>(f, H, W, C, y, x, acc);
                }
            }
            uint4 ov;
            T* oe = reinterpret_cast<T*>(&ov);
#pragma unroll
            for (int j = 0; j < VEC; ++j) {
                oe[j] = (T)(acc[j] / b.count);
                psum[j] += (float)oe[j];
            }
            *reinterpret_cast<uint4*>(out + (((size_t)r * P + ph) * P + pw) * C + cv * VEC) = ov;
        }
    }
    uint4 pv;
    T* pe = reinterpret_cast<T*>(&pv);
#pragma unroll
    for (int j = 0; j < VEC; ++j) pe[j] = (T)(psum[j] / 4.f);
    *reinterpret_cast<uint4*>(pooled + (((size_t)r * P2 + ph2) * P2 + pw2) * C + cv * VEC) = pv;
}

// CLIPFastRCNN.preprocess_image + ImageList.from_tensors: the (H_b, W_b, 3) view of
// each padded 1-D image buffer (criterion.py:371-375), (v * (1/div) - mean) / std per
// channel, zero-padded to (Hp, Wp), written NHWC.
template <typename T>
__global__ void __launch_bounds__(256) clip_preprocess_kernel(
    const float* __restrict__ images, long long img_stride, const int* __restrict__ heights,
    const int* __restrict__ widths, int B, int Hp, int Wp, float div, float m0, float m1, float m2,
    float s0, float s1, float s2, T* __restrict__ out) {
    const long long total = (long long)B * Hp * Wp;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int x = (int)(t % Wp);
    const int y = (int)((t / Wp) % Hp);
    const int b = (int)(t / ((long long)Wp * Hp));
    const int h = heights[b], w = widths[b];
    T* o = out + t * 3;
    if (y >= h || x >= w) {
        o[0] = (T)0.f;
        o[1] = (T)0.f;
        o[2] = (T)0.f;
        return;
    }
    const float* src = images + (size_t)b * img_stride + ((size_t)y * w + x) * 3;
    const float m[3] = {m0, m1, m2}, s[3] = {s0, s1, s2};
    // `x / 255.0` with a Python scalar is evaluated by torch as x * (1 / 255) in float
    // (div_true_kernel's CPU-scalar path); the std division is a true division.
    const float inv = 1.f / div;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float v = src[c];
        if (div != 1.f) v = v * inv;
        o[c] = (T)((v - m[c]) / s[c]);
    }
}

}  // namespace

extern "C" int ov3d_roi_align_fwd(const void* feat, int is_bf16, int N, int H, int W, int C,
                                  const float* boxes, int R, int per_image, int nimages,
                                  float spatial_scale, int pooled, int sampling_ratio, int aligned,
                                  void* out, void* stream) {
    if (!feat || !boxes || !out || N <= 0 || H <= 0 || W <= 0 || C <= 0 || R < 0 || pooled <= 0 ||
        per_image <= 0 || nimages <= 0 || nimages > N)
        return OV3D_EINVAL;
    if (R == 0) return OV3D_OK;
    const int vec = is_bf16 ? 8 : 4;
    if (C % vec) return OV3D_EINVAL;
    const long long total = (long long)R * pooled * pooled * (C / vec);
    if (total > 0x7fffffffLL * 256) return OV3D_EINVAL;
    const int blocks = ov3d_cdiv(total, 256);
    hipStream_t s = ov3d_stream(stream);
    if ((uintptr_t)feat & 15 || (uintptr_t)out & 15) return OV3D_EINVAL;
    const bool small = total + 256 <= 0x7fffffffLL;
    if (is_bf16 && small)
        roi_align_kernel<bf16, 8, int><<<blocks, 256, 0, s>>>(
            (const bf16*)feat, H, W, C, boxes, R, per_image, nimages, spatial_scale, pooled,
            sampling_ratio, aligned, (bf16*)out);
    else if (is_bf16)
        roi_align_kernel<bf16, 8, long long><<<blocks, 256, 0, s>>>(
            (const bf16*)feat, H, W, C, boxes, R, per_image, nimages, spatial_scale, pooled,
            sampling_ratio, aligned, (bf16*)out);
    else if (small)
        roi_align_kernel<float, 4, int><<<blocks, 256, 0, s>>>(
            (const float*)feat, H, W, C, boxes, R, per_image, nimages, spatial_scale, pooled,
            sampling_ratio, aligned, (float*)out);
    else
        roi_align_kernel<float, 4, long long><<<blocks, 256, 0, s>>>(
            (const float*)feat, H, W, C, boxes, R, per_image, nimages, spatial_scale, pooled,
            sampling_ratio, aligned, (float*)out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_roi_align_pool2_fwd(const void* feat, int is_bf16, int N, int H, int W, int C,
                                        const float* boxes, int R, int per_image, int nimages,
                                        float spatial_scale, int pooled, int sampling_ratio,
                                        int aligned, void* out, void* pooled_out, void* stream) {
    if (!feat || !boxes || !out || !pooled_out || N <= 0 || H <= 0 || W <= 0 || C <= 0 || R < 0 ||
        pooled <= 0 || (pooled & 1) || per_image <= 0 || nimages <= 0 || nimages > N)
        return OV3D_EINVAL;
    if (R == 0) return OV3D_OK;
    const int vec = is_bf16 ? 8 : 4;
    if (C % vec || ((uintptr_t)feat | (uintptr_t)out | (uintptr_t)pooled_out) & 15) return OV3D_EINVAL;
    const long long total = (long long)R * (pooled / 2) * (pooled / 2) * (C / vec);
    if (total + 256 > 0x7fffffffLL || (long long)R * pooled * pooled * C > (1LL << 40))
        return OV3D_EINVAL;
    const int blocks = ov3d_cdiv(total, 256);
    hipStream_t s = ov3d_stream(stream);
    if (is_bf16)
        roi_align_pool2_kernel<bf16, 8><<<blocks, 256, 0, s>>>(
            (const bf16*)feat, H, W, C, boxes, R, per_image, nimages, spatial_scale, pooled,
            sampling_ratio, aligned, (bf16*)out, (bf16*)pooled_out);
    else
        roi_align_pool2_kernel<float, 4><<<blocks, 256, 0, s>>>(
            (const float*)feat, H, W, C, boxes, R, per_image, nimages, spatial_scale, pooled,
            sampling_ratio, aligned, (float*)out, (float*)pooled_out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_clip_preprocess(const float* images, long long img_stride,
                                    const int32_t* heights, const int32_t* widths, int B, int Hp,
                                    int Wp, float div, float m0, float m1, float m2, float s0,
                                    float s1, float s2, int out_bf16, void* out, void* stream) {
    if (!images || !heights || !widths || !out || B <= 0 || Hp <= 0 || Wp <= 0 || div == 0.f)
        return OV3D_EINVAL;
    const long long total = (long long)B * Hp * Wp;
    const int blocks = ov3d_cdiv(total, 256);
    hipStream_t s = ov3d_stream(stream);
    if (out_bf16)
        clip_preprocess_kernel<bf16><<<blocks, 256, 0, s>>>(images, img_stride, heights, widths, B,
                                                            Hp, Wp, div, m0, m1, m2, s0, s1, s2,
                                                            (bf16*)out);
    else
        clip_preprocess_kernel<float><<<blocks, 256, 0, s>>>(images, img_stride, heights, widths,
                                                             B, Hp, Wp, div, m0, m1, m2, s0, s1,
                                                             s2, (float*)out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
