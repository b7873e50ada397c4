// Detection evaluation on the device.
//
// Replaces the CPU evaluation of utils/ap_calculator.py and utils/eval_det.py:
//   ov3d_box_points_count : remove_empty_box (ap_calculator.py:70-84) — points of the scene
//                           inside each predicted box's convex hull (box_util.py:22-31,
//                           scipy Delaunay.find_simplex), after flip_axis_to_depth
//   ov3d_box3d_iou_eval   : box3d_iou (box_util.py:116-141) of every (prediction, GT) pair
//                           of a scene: Sutherland-Hodgman clip of the bird's-eye rectangles
//                           (polygon_clip, box_util.py:34-80) in double, the Python
//                           evaluation order, no contraction; the clipped polygon's area by
//                           the shoelace formula where the reference asks Qhull
//                           (ConvexHull(...).volume, box_util.py:88-97)
//   ov3d_ap_match         : eval_det_cls's TP / FP walk (eval_det.py:104-131) for every
//                           (scene, class): detections by descending confidence, each GT
//                           matched once
//   ov3d_ap_curve         : cumulative precision / recall and voc_ap (eval_det.py:20-52,
//                           133-146) per class from the globally sorted TP flags
#include <float.h>

#include "common.h"

namespace {

// ---------------------------------------------------------------------------
// point-in-hull counts.  The hull facets of the box's 8 corners are the planes through 3
// corners with the other 5 on one side (exactly the convex hull, also for corners that
// float32 rounding left slightly non-coplanar); a point is inside when it is on the inner
// side of every facet (boundary: Qhull's find_simplex tolerance is not reproduced).
constexpr int kBoxesPerWG = 8;
constexpr int kMaxFacets = 56;   // C(8, 3)
constexpr int kCountThreads = 256;

__global__ __launch_bounds__(kCountThreads) void box_points_count_kernel(
    const float* __restrict__ pts, long long pt_sb, long long pt_sn, int N,
    const float* __restrict__ corners, int K, int32_t* __restrict__ counts) {
    const int b = blockIdx.y;
    const int k0 = blockIdx.x * kBoxesPerWG;
    __shared__ double s_pl[kBoxesPerWG][kMaxFacets][4];
    __shared__ int s_nf[kBoxesPerWG];
    __shared__ double s_bb[kBoxesPerWG][6];
    __shared__ int s_cnt[kBoxesPerWG];
    if (threadIdx.x < kBoxesPerWG) {
        const int q = threadIdx.x;
        const int k = k0 + q;
        int nf = 0;
        s_cnt[q] = 0;
        if (k < K) {
            // flip_axis_to_depth (ap_calculator.py:23-27) in float32: (x, z, -y)
            double P[8][3];
            const float* c = corners + ((long long)b * K + k) * 24;
            for (int v = 0; v < 8; ++v) {
                P[v][0] = (double)c[v * 3 + 0];
                P[v][1] = (double)c[v * 3 + 2];
                P[v][2] = (double)(-1.0f * c[v * 3 + 1]);
            }
            double lo[3] = {P[0][0], P[0][1], P[0][2]}, hi[3] = {P[0][0], P[0][1], P[0][2]};
            for (int v = 1; v < 8; ++v)
                for (int a = 0; a < 3; ++a) { lo[a] = fmin(lo[a], P[v][a]); hi[a] = fmax(hi[a], P[v][a]); }
            for (int a = 0; a < 3; ++a) { s_bb[q][a] = lo[a]; s_bb[q][3 + a] = hi[a]; }
            for (int i = 0; i < 8; ++i)
                for (int j = i + 1; j < 8; ++j)
                    for (int l = j + 1; l < 8; ++l) {
                        const double u[3] = {P[j][0] - P[i][0], P[j][1] - P[i][1], P[j][2] - P[i][2]};
                        const double w[3] = {P[l][0] - P[i][0], P[l][1] - P[i][1], P[l][2] - P[i][2]};
                        double n[3] = {u[1] * w[2] - u[2] * w[1], u[2] * w[0] - u[0] * w[2],
                                       u[0] * w[1] - u[1] * w[0]};
                        if (n[0] == 0.0 && n[1] == 0.0 && n[2] == 0.0) continue;
                        bool pos = false, neg = false;
                        for (int m = 0; m < 8; ++m) {
                            if (m == i || m == j || m == l) continue;
                            const double s = n[0] * (P[m][0] - P[i][0]) + n[1] * (P[m][1] - P[i][1]) +
                                             n[2] * (P[m][2] - P[i][2]);
                            pos |= s > 0.0;
                            neg |= s < 0.0;
                        }
                        if (pos && neg) continue;
                        if (pos) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }   // outward normal
                        if (!pos && !neg) continue;                               // all coplanar
                        s_pl[q][nf][0] = n[0];
                        s_pl[q][nf][1] = n[1];
                        s_pl[q][nf][2] = n[2];
                        s_pl[q][nf][3] = n[0] * P[i][0] + n[1] * P[i][1] + n[2] * P[i][2];
                        ++nf;
                    }
        }
        s_nf[q] = nf;
    }
    __syncthreads();
    int cnt[kBoxesPerWG];
#pragma unroll
    for (int q = 0; q < kBoxesPerWG; ++q) cnt[q] = 0;
    const float* P0 = pts + (long long)b * pt_sb;
    for (int i = threadIdx.x; i < N; i += kCountThreads) {
        const float* p = P0 + (long long)i * pt_sn;
        const double x = p[0], y = p[1], z = p[2];
#pragma unroll
        for (int q = 0; q < kBoxesPerWG; ++q) {
            if (s_nf[q] == 0) continue;
            if (x < s_bb[q][0] || y < s_bb[q][1] || z < s_bb[q][2] || x > s_bb[q][3] ||
                y > s_bb[q][4] || z > s_bb[q][5])
                continue;
            bool in = true;
            for (int f = 0; f < s_nf[q] && in; ++f)
                in = s_pl[q][f][0] * x + s_pl[q][f][1] * y + s_pl[q][f][2] * z <= s_pl[q][f][3];
            cnt[q] += in;
        }
    }
#pragma unroll
    for (int q = 0; q < kBoxesPerWG; ++q) {
        int v = cnt[q];
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(&s_cnt[q], v);
    }
    __syncthreads();
    if (threadIdx.x < kBoxesPerWG && k0 + (int)threadIdx.x < K)
        counts[(long long)b * K + k0 + threadIdx.x] = s_cnt[threadIdx.x];
}

// ---------------------------------------------------------------------------
// box3d_iou: rect = corners 3, 2, 1, 0 in (x, z) (box_util.py:128-129)
struct Pt { double x, y; };

__device__ __forceinline__ bool sh_inside(Pt p, Pt c1, Pt c2) {
    return (c2.x - c1.x) * (p.y - c1.y) > (c2.y - c1.y) * (p.x - c1.x);
}

__device__ __forceinline__ Pt sh_intersect(Pt c1, Pt c2, Pt s, Pt e) {
    const double dc0 = c1.x - c2.x, dc1 = c1.y - c2.y;
    const double dp0 = s.x - e.x, dp1 = s.y - e.y;
    const double n1 = c1.x * c2.y - c1.y * c2.x;
    const double n2 = s.x * e.y - s.y * e.x;
    const double n3 = 1.0 / (dc0 * dp1 - dc1 * dp0);
    return Pt{(n1 * dp0 - n2 * dc0) * n3, (n1 * dp1 - n2 * dc1) * n3};
}

// area of polygon_clip(rect1, rect2) (0 when the clip empties: the reference's None)
__device__ double clip_area(const Pt* r1, const Pt* r2) {
    Pt out[16], in[16];
    int n_out = 4;
    for (int i = 0; i < 4; ++i) out[i] = r1[i];
    Pt c1 = r2[3];
    for (int ci = 0; ci < 4; ++ci) {
        const Pt c2 = r2[ci];
        const int n_in = n_out;
        for (int i = 0; i < n_in; ++i) in[i] = out[i];
        n_out = 0;
        Pt s = in[n_in - 1];
        for (int i = 0; i < n_in; ++i) {
            const Pt e = in[i];
            if (sh_inside(e, c1, c2)) {
                if (!sh_inside(s, c1, c2)) out[n_out++] = sh_intersect(c1, c2, s, e);
                out[n_out++] = e;
            } else if (sh_inside(s, c1, c2)) {
                out[n_out++] = sh_intersect(c1, c2, s, e);
            }
            s = e;
        }
        c1 = c2;
        if (n_out == 0) return 0.0;
    }
    double a = 0.0;
    for (int i = 0; i < n_out; ++i) {
        const Pt p = out[i], q = out[(i + 1) % n_out];
        a += p.x * q.y - q.x * p.y;
    }
    return 0.5 * fabs(a);
}

__device__ __forceinline__ double box_vol(const float* c) {
    double e[3];
    const int pairs[3][2] = {{0, 1}, {1, 2}, {0, 4}};
    for (int q = 0; q < 3; ++q) {
        const double dx = (double)c[pairs[q][0] * 3] - (double)c[pairs[q][1] * 3];
        const double dy = (double)c[pairs[q][0] * 3 + 1] - (double)c[pairs[q][1] * 3 + 1];
        const double dz = (double)c[pairs[q][0] * 3 + 2] - (double)c[pairs[q][1] * 3 + 2];
        e[q] = sqrt(dx * dx + dy * dy + dz * dz);
    }
    return e[0] * e[1] * e[2];
}

__global__ void box3d_iou_kernel(const float* __restrict__ pred, const uint8_t* __restrict__ pvalid,
                                 const float* __restrict__ gt, const uint8_t* __restrict__ gvalid,
                                 int S, int K, int G, double* __restrict__ iou) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)S * K * G) return;
    const int g = (int)(t % G);
    const long long sk = t / G;
    const int s = (int)(sk / K);
    double v = 0.0;
    if (pvalid[sk] && gvalid[(long long)s * G + g]) {
        const float* c1 = pred + sk * 24;
        const float* c2 = gt + ((long long)s * G + g) * 24;
        Pt r1[4], r2[4];
        for (int i = 0; i < 4; ++i) {
            r1[i] = Pt{(double)c1[(3 - i) * 3], (double)c1[(3 - i) * 3 + 2]};
            r2[i] = Pt{(double)c2[(3 - i) * 3], (double)c2[(3 - i) * 3 + 2]};
        }
        const double inter = clip_area(r1, r2);
        const double ymax = fmin((double)c1[1], (double)c2[1]);
        const double ymin = fmax((double)c1[13], (double)c2[13]);
        const double inter_vol = inter * fmax(0.0, ymax - ymin);
        v = inter_vol / (box_vol(c1) + box_vol(c2) - inter_vol);
    }
    iou[t] = v;
}

// ---------------------------------------------------------------------------
// TP / FP of every detection, per (scene, class): detections of the class in that scene in
// descending score (ties: lower box index first), each matched to the first GT of the class
// with the largest IoU; a hit (IoU > thresh) on an unmatched GT is a TP and marks it.
__global__ void ap_match_kernel(const double* __restrict__ iou, const float* __restrict__ scores,
                                const int64_t* __restrict__ gt_cls,
                                const uint8_t* __restrict__ gvalid, int S, int K, int G, int C,
                                double thresh, uint8_t* __restrict__ tp) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)S * C) return;
    const int s = (int)(t / C), c = (int)(t % C);
    const float* sc = scores + (long long)s * K * C + c;
    unsigned long long done[4] = {0, 0, 0, 0};   // K <= 256 processed flags
    unsigned long long det = 0;                  // G <= 64 matched flags
    for (;;) {
        int best = -1;
        float bs = -INFINITY;
        for (int k = 0; k < K; ++k) {
            if ((done[k >> 6] >> (k & 63)) & 1ull) continue;
            const float v = sc[(long long)k * C];
            if (v > bs) { bs = v; best = k; }
        }
        if (best < 0) break;
        done[best >> 6] |= 1ull << (best & 63);
        double ovmax = -INFINITY;
        int jmax = -1;
        for (int g = 0; g < G; ++g) {
            if (!gvalid[(long long)s * G + g] || gt_cls[(long long)s * G + g] != c) continue;
            const double v = iou[((long long)s * K + best) * G + g];
            if (v > ovmax) { ovmax = v; jmax = g; }
        }
        uint8_t hit = 0;
        if (ovmax > thresh && !((det >> jmax) & 1ull)) {
            hit = 1;
            det |= 1ull << jmax;
        }
        tp[((long long)s * K + best) * C + c] = hit;
    }
}

// ---------------------------------------------------------------------------
// voc_ap per class (one workgroup each) from TP flags in global descending-score order:
//   prec_d = tp_d / (d + 1), rec_d = tp_d / npos; the area under the precision envelope
//   only changes at TP positions: ap = sum_k (rec_k - rec_{k-1}) * max_{k' >= k} prec_k'.
constexpr int kCurveThreads = 1024;

__global__ __launch_bounds__(kCurveThreads) void ap_curve_kernel(
    const uint8_t* __restrict__ tp_sorted, long long M, const int32_t* __restrict__ nvalid,
    const int32_t* __restrict__ npos, int32_t* __restrict__ tp_pos, long long tp_cap,
    double* __restrict__ ap, double* __restrict__ rec_last) {
    const int c = blockIdx.x;
    const uint8_t* f = tp_sorted + (long long)c * M;
    int32_t* pos = tp_pos + (long long)c * tp_cap;
    const int n = nvalid[c];
    const int np = npos[c];
    __shared__ int s_w[kCurveThreads / 64];
    __shared__ int s_base;
    if (threadIdx.x == 0) s_base = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // (1) positions of the TPs, in order
    for (int c0 = 0; c0 < n; c0 += kCurveThreads) {
        const int d = c0 + threadIdx.x;
        const bool hit = d < n && f[d];
        const unsigned long long m = __ballot(hit);
        if (lane == 0) s_w[w] = __popcll(m);
        __syncthreads();
        int p = s_base + __popcll(m & lanemask_lt());
        for (int q = 0; q < w; ++q) p += s_w[q];
        if (hit && p < tp_cap) pos[p] = d;
        __syncthreads();
        if (threadIdx.x == 0) {
            int tot = 0;
            for (int q = 0; q < kCurveThreads / 64; ++q) tot += s_w[q];
            s_base += tot;
        }
        __syncthreads();
    }
    // (2) suffix max of precision over TP positions + the sum (one thread: T <= #GT)
    if (threadIdx.x == 0) {
        const int T = min(s_base, (int)tp_cap);
        double sum = 0.0, env = 0.0;
        for (int k = T - 1; k >= 0; --k) {
            const double prec = (double)(k + 1) / fmax((double)(pos[k] + 1), DBL_EPSILON);
            env = fmax(env, prec);
            const double r1 = np > 0 ? (double)(k + 1) / (double)np : 0.0;
            const double r0 = np > 0 ? (double)k / (double)np : 0.0;
            sum += (r1 - r0) * env;
        }
        ap[c] = sum;
        rec_last[c] = (n > 0 && np > 0) ? (double)T / (double)np : 0.0;
    }
}

}  // namespace

extern "C" int ov3d_box_points_count(const float* pts, long long pt_sb, long long pt_sn, int N,
                                     const float* corners, int B, int K, int32_t* counts,
                                     void* stream) {
    if (!pts || !corners || !counts || B < 0 || K < 0 || N < 0 || pt_sn < 3) return OV3D_EINVAL;
    if (B == 0 || K == 0) return OV3D_OK;
    hipLaunchKernelGGL(box_points_count_kernel, dim3((K + kBoxesPerWG - 1) / kBoxesPerWG, B),
                       dim3(kCountThreads), 0, ov3d_stream(stream), pts, pt_sb, pt_sn, N, corners,
                       K, counts);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_box3d_iou_eval(const float* pred, const uint8_t* pvalid, const float* gt,
                                   const uint8_t* gvalid, int S, int K, int G, double* iou,
                                   void* stream) {
    if (!pred || !pvalid || !gt || !gvalid || !iou || S < 0 || K < 0 || G < 0) return OV3D_EINVAL;
    const long long n = (long long)S * K * G;
    if (n == 0) return OV3D_OK;
    hipLaunchKernelGGL(box3d_iou_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       ov3d_stream(stream), pred, pvalid, gt, gvalid, S, K, G, iou);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_ap_match(const double* iou, const float* scores, const int64_t* gt_cls,
                             const uint8_t* gvalid, int S, int K, int G, int C, double thresh,
                             uint8_t* tp, void* stream) {
    if (!iou || !scores || !gt_cls || !gvalid || !tp || S < 0 || K < 0 || K > 256 || G < 0 ||
        G > 64 || C <= 0)
        return OV3D_EINVAL;
    const long long n = (long long)S * C;
    if (n == 0 || K == 0) return OV3D_OK;
    hipLaunchKernelGGL(ap_match_kernel, dim3((unsigned)((n + 127) / 128)), dim3(128), 0,
                       ov3d_stream(stream), iou, scores, gt_cls, gvalid, S, K, G, C, thresh, tp);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_ap_curve(const uint8_t* tp_sorted, long long M, const int32_t* nvalid,
                             const int32_t* npos, int C, int32_t* tp_pos, long long tp_cap,
                             double* ap, double* rec_last, void* stream) {
    if (!tp_sorted || !nvalid || !npos || !tp_pos || !ap || !rec_last || C < 0 || M < 0 ||
        tp_cap <= 0)
        return OV3D_EINVAL;
    if (C == 0) return OV3D_OK;
    hipLaunchKernelGGL(ap_curve_kernel, dim3(C), dim3(kCurveThreads), 0, ov3d_stream(stream),
                       tp_sorted, M, nvalid, npos, tp_pos, tp_cap, ap, rec_last);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
