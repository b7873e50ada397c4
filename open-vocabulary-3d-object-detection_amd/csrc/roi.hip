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
#include <stdlib.h>

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

// bilinear_acc on 8 bf16 channels with the four corner runs from fetch(y, x) (uint4): the same
// expression, order and rounding as bilinear_acc<bf16, 8>
template <typename F>
__device__ __forceinline__ void bilinear_acc_src(int H, int W, float y, float x, float* acc, F fetch) {
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
    const uint4 u1 = fetch(yl, xl), u2 = fetch(yl, xh), u3 = fetch(yh, xl), u4 = fetch(yh, xh);
    const bf16* p1 = reinterpret_cast<const bf16*>(&u1);
    const bf16* p2 = reinterpret_cast<const bf16*>(&u2);
    const bf16* p3 = reinterpret_cast<const bf16*>(&u3);
    const bf16* p4 = reinterpret_cast<const bf16*>(&u4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v = w1 * (float)p1[j] + w2 * (float)p2[j] + w3 * (float)p3[j] + w4 * (float)p4[j];
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
// affine (grid % 8 == 0, R % per_image == 0, (R / per_image) % nimages == 0): image-affine XCD
// order.  Workgroup b runs on XCD b % 8 (the dispatcher's round robin; an assumption for speed
// only, any placement is correct): work item L = (b >> 3) + (b & 7) * (grid / 8), items ordered
// image-major, so each XCD's L2 serves the ROIs of one image (a 45 x 33 x 1280 bf16 res4 map is
// 3.8 MB) instead of all of them (the gathers of a whole-map ROI re-read its image ~75 times).
template <typename T, int VEC>
__global__ void __launch_bounds__(256) roi_align_pool2_kernel(
    const T* __restrict__ feat, int H, int W, int C, const float* __restrict__ boxes, int R,
    int per_image, int nimages, float scale, int P, int sampling_ratio, int aligned,
    T* __restrict__ out, T* __restrict__ pooled, int affine) {
    static_assert(VEC * sizeof(T) == 16, "one 16-byte channel run per thread");
    const int CV = C / VEC, P2 = P / 2;
    const int total = R * P2 * P2 * CV;
    const int b = affine ? (blockIdx.x >> 3) + (blockIdx.x & 7) * (gridDim.x >> 3) : blockIdx.x;
    const int t = b * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int cv = t % CV;
    int q = t / CV;
    const int pw2 = q % P2;
    q /= P2;
    const int ph2 = q % P2;
    int r = q / P2;
    if (affine) {   // image-major rank -> ROI: image i owns runs i, i + nimages, ...
        const int per_img_rois = R / nimages, i = r / per_img_rois, rem = r - i * per_img_rois;
        const int k = rem / per_image;
        r = (i + k * nimages) * per_image + (rem - k * per_image);
    }
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

// The same output as roi_align_pool2_kernel (bf16), with the feature window in LDS.  With boxes
// spanning most of the map (the C5 step: median ROI 45 x 33 of a 45 x 33 res4 map, 4.8 samples
// per bin) every output channel run gathers ~77 corner runs, and the global form ran at the
// L2's rate (3.7 ms for 4096 ROIs, profiles/r05_c5_trace_steady_v2.json).  Here a workgroup
// owns LGROUP consecutive ROIs of one image (a run of per_image ROIs shares its image) and a
// 32-channel slice: the union of their sample windows (rows / columns each bilinear corner can
// touch) is loaded into LDS once, 64 bytes per pixel, and every corner run is read from there.
// Arithmetic, order and rounding are roi_align_pool2_kernel's (bilinear_acc's expression per
// sample, fp32, one rounding per bin), so the outputs are bit-identical.  A window larger than
// LMAXPX pixels (or a non-finite box) leaves the workgroup on the global corner reads.
// Workgroup w covers work item L = (w >> 3) + (w & 7) * (grid / 8) (grid % 8 == 0): the two
// 32-channel slices that share the output's 128-byte lines run on one XCD, next to each other.
constexpr int LGROUP = 16;
constexpr int LCH = 32;                // channels per slice (4 runs of 8)
constexpr int LMAXPX = 1536;           // 96 KB of window

__device__ __forceinline__ void win_rows(float start, float size, int n, int& lo, int& hi) {
    // samples lie in [start, start + size]; a corner is floor(s) or floor(s) + 1, clamped
    lo = (int)floorf(start) - 1;
    hi = (int)floorf(start + size) + 2;
    lo = min(max(lo, 0), n - 1);
    hi = min(max(hi, 0), n - 1);
}

__global__ void __launch_bounds__(512) roi_align_pool2_lds_kernel(
    const bf16* __restrict__ feat, int H, int W, int C, const float* __restrict__ boxes, int R,
    int per_image, int nimages, float scale, int P, int sampling_ratio, int aligned, int nwork,
    bf16* __restrict__ out, bf16* __restrict__ pooled) {
    __shared__ __attribute__((aligned(16))) uint4 win[LMAXPX * (LCH / 8)];
    __shared__ int wbox[4];
    const int tid = threadIdx.x;
    const int L = (blockIdx.x >> 3) + (blockIdx.x & 7) * (gridDim.x >> 3);
    if (L >= nwork) return;
    const int nslice = C / LCH;
    const int slice = L % nslice, g = L / nslice;
    const int gpr = (per_image + LGROUP - 1) / LGROUP;
    const int run = g / gpr, r0 = run * per_image + (g - run * gpr) * LGROUP;
    const int nr = min(LGROUP, min(run * per_image + per_image, R) - r0);
    const int img = run % nimages;
    const float offset = aligned ? 0.5f : 0.f;
    if (tid == 0) {
        int y0 = H, y1 = -1, x0 = W, x1 = -1;
        bool ok = true;
        for (int i = 0; i < nr; ++i) {
            const float* b = boxes + 4 * (size_t)(r0 + i);
            const float sw = b[0] * scale - offset, sh = b[1] * scale - offset;
            float rw = b[2] * scale - offset - sw, rh = b[3] * scale - offset - sh;
            if (!aligned) { rw = fmaxf(rw, 1.f); rh = fmaxf(rh, 1.f); }
            if (!(__builtin_isfinite(sw) && __builtin_isfinite(sh) && __builtin_isfinite(rw) &&
                  __builtin_isfinite(rh)) || fabsf(sw) > 1e6f || fabsf(sh) > 1e6f || fabsf(rw) > 1e6f ||
                fabsf(rh) > 1e6f) {
                ok = false;
                break;
            }
            int lo, hi;
            win_rows(sh, rh, H, lo, hi);
            y0 = min(y0, lo); y1 = max(y1, hi);
            win_rows(sw, rw, W, lo, hi);
            x0 = min(x0, lo); x1 = max(x1, hi);
        }
        if (!ok || (long long)(y1 - y0 + 1) * (x1 - x0 + 1) > LMAXPX) y1 = -1;   // global path
        wbox[0] = y0; wbox[1] = y1; wbox[2] = x0; wbox[3] = x1;
    }
    __syncthreads();
    const int y0 = wbox[0], y1 = wbox[1], x0 = wbox[2], x1 = wbox[3];
    const bool lds = y1 >= y0;
    const int ww = x1 - x0 + 1;
    const bf16* const fimg = feat + (size_t)img * H * W * C + slice * LCH;
    if (lds) {
        const int npx = (y1 - y0 + 1) * ww;
        for (int i = tid; i < npx * (LCH / 8); i += 512) {
            const int p = i >> 2, v = i & 3;
            const int py = p / ww, px = p - py * ww;
            win[i] = *reinterpret_cast<const uint4*>(fimg + ((size_t)(y0 + py) * W + x0 + px) * C + 8 * v);
        }
        __syncthreads();
    }
    const int P2 = P / 2, nblk = P2 * P2;
    const int nitems = nr * nblk * (LCH / 8);
    for (int it = tid; it < nitems; it += 512) {
        const int v = it & 3, q = it >> 2;
        const int ri = q / nblk, blk = q - ri * nblk;
        const int ph2 = blk / P2, pw2 = blk - ph2 * P2;
        const int r = r0 + ri;
        const int cofs = slice * LCH + 8 * v;
        float psum[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) psum[j] = 0.f;
        for (int dy = 0; dy < 2; ++dy) {
            for (int dx = 0; dx < 2; ++dx) {
                const int ph = 2 * ph2 + dy, pw = 2 * pw2 + dx;
                const Bin b = bin_geometry(boxes + 4 * (size_t)r, scale, aligned, P, ph, pw, sampling_ratio);
                float acc[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[j] = 0.f;
                for (int iy = 0; iy < b.gh; ++iy) {
                    const float y = b.y0 + (float)(iy + .5f) * b.bh / (float)b.gh;
                    for (int ix = 0; ix < b.gw; ++ix) {
                        const float x = b.x0 + (float)(ix + .5f) * b.bw / (float)b.gw;
                        if (lds)
                            bilinear_acc_src(H, W, y, x, acc, [&](int yy, int xx) {
                                return win[((yy - y0) * ww + (xx - x0)) * 4 + v];
                            });
                        else
                            bilinear_acc_src(H, W, y, x, acc, [&](int yy, int xx) {
                                return *reinterpret_cast<const uint4*>(fimg + ((size_t)yy * W + xx) * C + 8 * v);
                            });
                    }
                }
                uint4 ov;
                bf16* oe = reinterpret_cast<bf16*>(&ov);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    oe[j] = (bf16)(acc[j] / b.count);
                    psum[j] += (float)oe[j];
                }
                *reinterpret_cast<uint4*>(out + (((size_t)r * P + ph) * P + pw) * C + cofs) = ov;
            }
        }
        uint4 pv;
        bf16* pe = reinterpret_cast<bf16*>(&pv);
#pragma unroll
        for (int j = 0; j < 8; ++j) pe[j] = (bf16)(psum[j] / 4.f);
        *reinterpret_cast<uint4*>(pooled + (((size_t)r * P2 + ph2) * P2 + pw2) * C + cofs) = pv;
    }
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
    // the LDS-window form is opt-in (OV3D_ROI_LDS=1, read per call): at the C5 shape it ran
    // 5.1 ms against the global form's 3.7 ms (one 512-thread workgroup per CU behind a 96 KB
    // window leaves two waves per SIMD to hide the corner reads' LDS latency)
    const int lds_env = getenv("OV3D_ROI_LDS") ? atoi(getenv("OV3D_ROI_LDS")) : 0;
    if (is_bf16 && lds_env && C % LCH == 0) {
        const long long groups = (long long)((R + per_image - 1) / per_image) *
                                 ((per_image + LGROUP - 1) / LGROUP);
        const long long nwork = groups * (C / LCH);
        if (nwork > 0x7fffffffLL - 8) return OV3D_EINVAL;
        const int grid = (int)((nwork + 7) / 8 * 8);
        roi_align_pool2_lds_kernel<<<grid, 512, 0, s>>>(
            (const bf16*)feat, H, W, C, boxes, R, per_image, nimages, spatial_scale, pooled,
            sampling_ratio, aligned, (int)nwork, (bf16*)out, (bf16*)pooled_out);
    } else {
        // image-affine XCD order, opt-in (OV3D_ROI_AFFINE=1; read per call): measured no gain at C5
        // (51.2 vs 50.9 ms median, profiles/r05_c5_roi_affine_ab.json)
        const int aff_env = getenv("OV3D_ROI_AFFINE") ? atoi(getenv("OV3D_ROI_AFFINE")) : 0;
        const int affine = aff_env && R % per_image == 0 && (R / per_image) % nimages == 0 &&
                           (long long)(blocks + 7) / 8 * 8 * 256 <= 0x7fffffffLL;
        const int grid = affine ? (blocks + 7) / 8 * 8 : blocks;
        if (is_bf16)
            roi_align_pool2_kernel<bf16, 8><<<grid, 256, 0, s>>>(
                (const bf16*)feat, H, W, C, boxes, R, per_image, nimages, spatial_scale, pooled,
                sampling_ratio, aligned, (bf16*)out, (bf16*)pooled_out, affine);
        else
            roi_align_pool2_kernel<float, 4><<<grid, 256, 0, s>>>(
                (const float*)feat, H, W, C, boxes, R, per_image, nimages, spatial_scale, pooled,
                sampling_ratio, aligned, (float*)out, (float*)pooled_out, affine);
    }
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
