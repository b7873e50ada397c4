// Greedy 3D NMS (float64), batched over scenes, gfx950.
//
// Replaces utils/nms.py:79-162 (nms_3d_faster, nms_3d_faster_samecls) as called
// once per scene on the host by utils/ap_calculator.py:153-190.
// One workgroup per scene:
//   1. rank sort by (score desc, index desc) -- the order of a stable ascending
//      argsort read from the back, i.e. the reference's pick order;
//   2. every thread builds one row of the K x K upper-triangular suppression
//      bitmask in LDS: bit (r,c) = IoU(order[r], order[c]) > thr (same class);
//      the IoU is evaluated exactly as the numpy reference does, picker first:
//      inter / ((area[i] + area[j]) - inter), no contraction;
//   3. one wave walks the rows in order, keeping a row iff its bit is not yet
//      removed and OR-ing its mask into the removed set (64-bit words on lanes).
// The result equals the reference greedy loop because the reference removes
// exactly the boxes whose overlap with an earlier pick exceeds thr.
#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr int kMaxK = 512;
constexpr int kWords = kMaxK / 64;
constexpr int kThreads = 512;

__device__ __forceinline__ double np_max(double a, double b) {
    return (isnan(a) || isnan(b)) ? __longlong_as_double(0x7ff8000000000000ll) : (a > b ? a : b);
}
__device__ __forceinline__ double np_min(double a, double b) {
    return (isnan(a) || isnan(b)) ? __longlong_as_double(0x7ff8000000000000ll) : (a < b ? a : b);
}

__global__ __launch_bounds__(kThreads) void nms3d_kernel(const double* __restrict__ boxes,
                                                         const uint8_t* __restrict__ valid, int K,
                                                         int stride, double thr, int old_type,
                                                         int samecls, uint8_t* __restrict__ keep) {
    __shared__ double s_box[kMaxK][8];  // x1,y1,z1,x2,y2,z2,area,cls
    __shared__ double s_score[kMaxK];
    __shared__ unsigned char s_valid[kMaxK];
    __shared__ int s_order[kMaxK];
    __shared__ unsigned long long s_mask[kMaxK][kWords];
    __shared__ int s_nvalid;
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const double* bx = boxes + (size_t)b * K * stride;
    if (tid == 0) s_nvalid = 0;
    for (int i = tid; i < K; i += kThreads) {
        const double* p = bx + (size_t)i * stride;
        for (int a = 0; a < 6; ++a) s_box[i][a] = p[a];
        s_box[i][6] = (p[3] - p[0]) * (p[4] - p[1]) * (p[5] - p[2]);
        s_box[i][7] = samecls ? p[7] : 0.0;
        s_score[i] = p[6];
        s_valid[i] = valid ? (valid[(size_t)b * K + i] != 0) : 1;
        keep[(size_t)b * K + i] = 0;
    }
    __syncthreads();
    // 1. rank among valid boxes
    for (int i = tid; i < K; i += kThreads) {
        if (!s_valid[i]) continue;
        const double si = s_score[i];
        int r = 0;
        for (int j = 0; j < K; ++j) {
            if (!s_valid[j]) continue;
            const double sj = s_score[j];
            r += (sj > si) || (sj == si && j > i);
        }
        s_order[r] = i;
        atomicAdd(&s_nvalid, 1);
    }
    __syncthreads();
    const int nv = s_nvalid;
    const int nw = (nv + 63) / 64;
    // 2. suppression rows
    for (int r = tid; r < nv; r += kThreads) {
        const int i = s_order[r];
        const double ax1 = s_box[i][0], ay1 = s_box[i][1], az1 = s_box[i][2];
        const double ax2 = s_box[i][3], ay2 = s_box[i][4], az2 = s_box[i][5];
        const double area_i = s_box[i][6], cls_i = s_box[i][7];
        for (int w = 0; w < nw; ++w) {
            unsigned long long bits = 0ull;
            for (int q = 0; q < 64; ++q) {
                const int c = w * 64 + q;
                if (c <= r || c >= nv) continue;
                const int j = s_order[c];
                const double xx1 = np_max(ax1, s_box[j][0]), yy1 = np_max(ay1, s_box[j][1]),
                             zz1 = np_max(az1, s_box[j][2]);
                const double xx2 = np_min(ax2, s_box[j][3]), yy2 = np_min(ay2, s_box[j][4]),
                             zz2 = np_min(az2, s_box[j][5]);
                const double l = np_max(0.0, xx2 - xx1), wd = np_max(0.0, yy2 - yy1),
                             h = np_max(0.0, zz2 - zz1);
                double o;
                if (old_type) {
                    o = (l * wd * h) / s_box[j][6];
                } else {
                    const double inter = l * wd * h;
                    o = inter / (area_i + s_box[j][6] - inter);
                }
                if (samecls) o = o * (double)(cls_i == s_box[j][7]);
                if (o > thr) bits |= 1ull << q;
            }
            s_mask[r][w] = bits;
        }
    }
    __syncthreads();
    // 3. serial greedy walk by wave 0; lane w < nw holds removed-word w
    if (tid < 64) {
        unsigned long long removed = 0ull;
        for (int r = 0; r < nv; ++r) {
            const unsigned long long word = __shfl(removed, r >> 6);
            if ((word >> (r & 63)) & 1ull) continue;
            if (tid == 0) keep[(size_t)b * K + s_order[r]] = 1;
            if (tid < nw) removed |= s_mask[r][tid];
        }
    }
}

__global__ __launch_bounds__(256) void nms_boxes_kernel(const float* __restrict__ corners,
                                                        const float* __restrict__ obj,
                                                        const int64_t* __restrict__ cls, int total,
                                                        double* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const float* c = corners + (size_t)t * 24;
    float mn[3] = {c[0], c[1], c[2]}, mx[3] = {c[0], c[1], c[2]};
    for (int v = 1; v < 8; ++v)
        for (int a = 0; a < 3; ++a) {
            const float x = c[v * 3 + a];
            mn[a] = x < mn[a] ? x : mn[a];
            mx[a] = x > mx[a] ? x : mx[a];
        }
    double* o = out + (size_t)t * 8;
    o[0] = mn[0]; o[1] = mn[1]; o[2] = mn[2];
    o[3] = mx[0]; o[4] = mx[1]; o[5] = mx[2];
    o[6] = (double)obj[t];
    o[7] = cls ? (double)cls[t] : 0.0;
}

}  // namespace

extern "C" int ov3d_nms3d(const double* boxes, const uint8_t* valid, int B, int K, int stride,
                          double thr, int old_type, int samecls, uint8_t* keep_out, void* stream) {
    if (B < 0 || K < 0 || K > kMaxK || stride < 7 || (samecls && stride < 8) || !boxes || !keep_out)
        return OV3D_EINVAL;
    if (B == 0 || K == 0) return OV3D_OK;
    hipLaunchKernelGGL(nms3d_kernel, dim3(B), dim3(kThreads), 0, ov3d_stream(stream), boxes, valid,
                       K, stride, thr, old_type, samecls, keep_out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_nms_boxes_from_corners(const float* corners, const float* obj,
                                           const int64_t* cls, int B, int K, double* boxes_out,
                                           void* stream) {
    if (B < 0 || K < 0 || !corners || !obj || !boxes_out) return OV3D_EINVAL;
    const int total = B * K;
    if (total == 0) return OV3D_OK;
    hipLaunchKernelGGL(nms_boxes_kernel, dim3(ov3d_cdiv(total, 256)), dim3(256), 0,
                       ov3d_stream(stream), corners, obj, cls, total, boxes_out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
