// 3D generalized IoU between predicted and GT boxes (corners, up = -Y), gfx950.
//
// Replaces utils/box_util.py:717-737 and both of its dispatch targets:
//   * generalized_box3d_iou_cython (box_util.py:624-714) whose rotated
//     intersection is utils/box_intersection.pyx:166-198 -- Sutherland-Hodgman
//     evaluated on untyped Python floats (double), vertices rounded to float32,
//     float32 shoelace; K2 = rect2.shape[2] (= 4) bug reproduced behind k2_bug;
//   * generalized_box3d_iou_tensor (box_util.py:517-618): same algorithm on
//     float32 scalars for every k2 < nums.
// One thread per (b, k1, k2) pair; the reference runs the intersection on the
// CPU after a device->host copy (box_util.py:684-694), here everything stays in
// HBM and the result feeds the matcher cost directly.
// Float contract (no contraction, IEEE div/sqrt) matches oracle/ov3d_oracle.c.
#include "common.h"

#pragma clang fp contract(off)

namespace {

template <typename T>
struct P2 {
    T x, y;
};

template <typename T>
__device__ __forceinline__ int clip_poly(const P2<T>* subj, const P2<T>* clip, P2<T>* res) {
    P2<T> in[10], cur[10];
    int nout = 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) cur[i] = subj[i];
    P2<T> cp1 = clip[3];
    for (int ci = 0; ci < 4; ++ci) {
        const P2<T> cp2 = clip[ci];
        const int nin = nout;
        for (int i = 0; i < nin; ++i) in[i] = cur[i];
        nout = 0;
        if (nin == 0) break;
        P2<T> s = in[nin - 1];
        for (int ii = 0; ii < nin; ++ii) {
            const P2<T> e = in[ii];
            const bool e_in = (cp2.x - cp1.x) * (e.y - cp1.y) > (cp2.y - cp1.y) * (e.x - cp1.x);
            const bool s_in = (cp2.x - cp1.x) * (s.y - cp1.y) > (cp2.y - cp1.y) * (s.x - cp1.x);
            if (e_in || s_in) {
                if (e_in != s_in) {
                    const T dc0 = cp1.x - cp2.x, dc1 = cp1.y - cp2.y;
                    const T dp0 = s.x - e.x, dp1 = s.y - e.y;
                    const T n1 = cp1.x * cp2.y - cp1.y * cp2.x;
                    const T n2 = s.x * e.y - s.y * e.x;
                    const T n3 = T(1) / (dc0 * dp1 - dc1 * dp0);
                    P2<T> q;
                    q.x = (n1 * dp0 - n2 * dc0) * n3;
                    q.y = (n1 * dp1 - n2 * dc1) * n3;
                    if (nout < 10) cur[nout++] = q;
                }
                if (e_in && nout < 10) cur[nout++] = e;
            }
            s = e;
        }
        cp1 = cp2;
        if (nout == 0) break;
    }
    for (int i = 0; i < nout; ++i) res[i] = cur[i];
    return nout;
}

__device__ __forceinline__ float shoelace(const float* xs, const float* ys, int n) {
    float s1 = 0.f, s2 = 0.f;
    for (int i = 0; i < n; ++i) {
        const int im = (i == 0) ? n - 1 : i - 1;
        s1 = s1 + xs[i] * ys[im];
        s2 = s2 + ys[i] * xs[im];
    }
    return 0.5f * fabsf(s1 - s2);
}

__device__ __forceinline__ float edge_len(const float* c, int a, int b) {
    const float d0 = c[a * 3] - c[b * 3], d1 = c[a * 3 + 1] - c[b * 3 + 1],
                d2 = c[a * 3 + 2] - c[b * 3 + 2];
    return sqrtf(fmaxf(d0 * d0 + d1 * d1 + d2 * d2, 1e-6f));
}

__device__ __forceinline__ float box_vol(const float* c) {
    return edge_len(c, 0, 1) * edge_len(c, 1, 2) * edge_len(c, 0, 4);
}

__device__ __forceinline__ void minmax_flip(const float* c, float* mn, float* mx) {
#pragma unroll
    for (int a = 0; a < 3; ++a) { mn[a] = INFINITY; mx[a] = -INFINITY; }
#pragma unroll
    for (int v = 0; v < 8; ++v)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float val = c[v * 3 + a];
            if (a == 1) val = -val;
            mn[a] = val < mn[a] ? val : mn[a];
            mx[a] = val > mx[a] ? val : mx[a];
        }
}

__global__ __launch_bounds__(256) void giou_kernel(const float* __restrict__ corners1,
                                                   const float* __restrict__ corners2,
                                                   const int32_t* __restrict__ nums, int B, int K1,
                                                   int K2, int mode, int rotated_host,
                                                   const int32_t* __restrict__ rotated_dev,
                                                   int k2_bug, float* __restrict__ out) {
    const int rotated = rotated_dev ? (*rotated_dev != 0) : rotated_host;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)B * K1 * K2) return;
    const int k2 = (int)(t % K2);
    const long long bk1 = t / K2;
    const int b = (int)(bk1 / K1);
    const int nk = nums ? nums[b] : K2;
    float c1[24], c2[24];
    const float* g1 = corners1 + bk1 * 24;
    const float* g2 = corners2 + ((long long)b * K2 + k2) * 24;
#pragma unroll
    for (int i = 0; i < 24; ++i) { c1[i] = g1[i]; c2[i] = g2[i]; }
    const float EPS = 1e-8f;

    const float ymax = fminf(c1[1], c2[1]);
    const float ymin = fmaxf(c1[4 * 3 + 1], c2[4 * 3 + 1]);
    const float height = fmaxf(ymax - ymin, 0.f);
    // rect[i] = (corner[3-i].x, corner[3-i].z); lt = rect[1] = corner 2, rb = rect[3] = corner 0
    const float ltx = fmaxf(c1[2 * 3], c2[2 * 3]), ltz = fmaxf(c1[2 * 3 + 2], c2[2 * 3 + 2]);
    const float rbx = fminf(c1[0], c2[0]), rbz = fminf(c1[2], c2[2]);
    float non_rot = fmaxf(rbx - ltx, 0.f) * fmaxf(rbz - ltz, 0.f);
    if (k2 >= nk) non_rot = 0.f;

    float mn1[3], mx1[3], mn2[3], mx2[3];
    minmax_flip(c1, mn1, mx1);
    minmax_flip(c2, mn2, mx2);
    const float enc = fabsf(fmaxf(mx1[0], mx2[0]) - fminf(mn1[0], mn2[0])) *
                      fabsf(fminf(mn1[1], mn2[1]) - fmaxf(mx1[1], mx2[1])) *
                      fabsf(fmaxf(mx1[2], mx2[2]) - fminf(mn1[2], mn2[2]));
    const float v1 = fmaxf(box_vol(c1), EPS);
    const float v2 = fmaxf(box_vol(c2), EPS);
    const float sum_vols = v1 + v2;
    const float good = (enc > 2e-8f && sum_vols > 4e-8f) ? 1.f : 0.f;

    float inter_area;
    if (rotated) {
        inter_area = 0.f;
        int limit = nk;
        if (mode == OV3D_GIOU_CYTHON && k2_bug && limit > 4) limit = 4;
        if (k2 < limit && non_rot != 0.f) {
            float xs[10], ys[10];
            int n;
            if (mode == OV3D_GIOU_CYTHON) {
                P2<double> s[4], c[4], r[10];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    s[i].x = c1[(3 - i) * 3]; s[i].y = c1[(3 - i) * 3 + 2];
                    c[i].x = c2[(3 - i) * 3]; c[i].y = c2[(3 - i) * 3 + 2];
                }
                n = clip_poly<double>(s, c, r);
                for (int i = 0; i < n; ++i) { xs[i] = (float)r[i].x; ys[i] = (float)r[i].y; }
            } else {
                P2<float> s[4], c[4], r[10];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    s[i].x = c1[(3 - i) * 3]; s[i].y = c1[(3 - i) * 3 + 2];
                    c[i].x = c2[(3 - i) * 3]; c[i].y = c2[(3 - i) * 3 + 2];
                }
                n = clip_poly<float>(s, c, r);
                for (int i = 0; i < n; ++i) { xs[i] = r[i].x; ys[i] = r[i].y; }
            }
            if (n > 0) inter_area = shoelace(xs, ys, n);
        }
    } else {
        inter_area = non_rot;
    }
    const float inter_vol = inter_area * height;
    const float uni = fmaxf(sum_vols - inter_vol, EPS);
    const float iou = inter_vol / uni;
    const float second = -(1.f - uni / enc);
    float g = (iou + second) * good;
    if (k2 >= nk) g = g * 0.f;
    out[t] = g;
}

// d/dcorners1 of the axis-aligned GIoU (torch autograd semantics of
// box_util.py:517-618 with rotated_boxes=False): binary min/max split ties 1/2,
// reductions over corners route to the first extremal corner, clamp passes
// where input >= bound, abs uses sign().  One thread per (b,k1), loop over k2.
__device__ __forceinline__ void bin_min_grad(float a, float b, float g, float& ga) {
    ga += (a < b) ? g : ((a == b) ? 0.5f * g : 0.f);
}
__device__ __forceinline__ void bin_max_grad(float a, float b, float g, float& ga) {
    ga += (a > b) ? g : ((a == b) ? 0.5f * g : 0.f);
}
__device__ __forceinline__ float sgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

// The rotated intersection area, differentiated: clip_poly<float> (the forward's arithmetic,
// box_util.py:387-440 on float32 tensors) with each stage's vertices and their parents
// recorded, the shoelace area (:591-596, |.| and the 0.5), then reverse mode back through the
// stages: a vertex kept as is passes its gradient to its parent; an intersection point
// q(cp1, cp2, s, e) (helper_computeIntersection, :387-396) sends J^T g to s and e (the clip
// edge is the GT box: constant).  Stage 0 is rect1 = corners (3, 2, 1, 0) (x, z).
struct ClipTrace {
    P2<float> v[5][10];
    int8_t pa[5][10], pb[5][10];   // stage s >= 1: parents in stage s - 1 (pb < 0: kept vertex)
    int n[5];
    int last;                      // final stage
};

__device__ __noinline__ float rot_area_grad(const float* c1, const float* c2, float g_area,
                                            float* gc) {
    ClipTrace T;
    P2<float> clip[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        T.v[0][i].x = c1[(3 - i) * 3]; T.v[0][i].y = c1[(3 - i) * 3 + 2];
        clip[i].x = c2[(3 - i) * 3]; clip[i].y = c2[(3 - i) * 3 + 2];
    }
    T.n[0] = 4;
    T.last = 0;
    P2<float> cp1 = clip[3];
    for (int ci = 0; ci < 4; ++ci) {
        const P2<float> cp2 = clip[ci];
        const int nin = T.n[ci];
        int nout = 0;
        if (nin == 0) break;
        int si = nin - 1;
        for (int ii = 0; ii < nin; ++ii) {
            const P2<float> s = T.v[ci][si], e = T.v[ci][ii];
            const bool e_in = (cp2.x - cp1.x) * (e.y - cp1.y) > (cp2.y - cp1.y) * (e.x - cp1.x);
            const bool s_in = (cp2.x - cp1.x) * (s.y - cp1.y) > (cp2.y - cp1.y) * (s.x - cp1.x);
            if (e_in || s_in) {
                if (e_in != s_in) {
                    const float dc0 = cp1.x - cp2.x, dc1 = cp1.y - cp2.y;
                    const float dp0 = s.x - e.x, dp1 = s.y - e.y;
                    const float n1 = cp1.x * cp2.y - cp1.y * cp2.x;
                    const float n2 = s.x * e.y - s.y * e.x;
                    const float n3 = 1.f / (dc0 * dp1 - dc1 * dp0);
                    if (nout < 10) {
                        T.v[ci + 1][nout].x = (n1 * dp0 - n2 * dc0) * n3;
                        T.v[ci + 1][nout].y = (n1 * dp1 - n2 * dc1) * n3;
                        T.pa[ci + 1][nout] = (int8_t)si;
                        T.pb[ci + 1][nout] = (int8_t)ii;
                        ++nout;
                    }
                }
                if (e_in && nout < 10) {
                    T.v[ci + 1][nout] = e;
                    T.pa[ci + 1][nout] = (int8_t)ii;
                    T.pb[ci + 1][nout] = (int8_t)-1;
                    ++nout;
                }
            }
            si = ii;
        }
        T.n[ci + 1] = nout;
        T.last = ci + 1;
        cp1 = cp2;
        if (nout == 0) break;
    }
    const int L = T.last, n = T.n[L];
    if (n == 0) return 0.f;
    float s1 = 0.f, s2 = 0.f;
    for (int i = 0; i < n; ++i) {
        const int im = (i == 0) ? n - 1 : i - 1;
        s1 = s1 + T.v[L][i].x * T.v[L][im].y;
        s2 = s2 + T.v[L][i].y * T.v[L][im].x;
    }
    const float S = s1 - s2;
    const float area = 0.5f * fabsf(S);
    if (g_area == 0.f) return area;
    // d area / d S = 0.5 sign(S); dS/dx_k = y_{k-1} - y_{k+1}, dS/dy_k = x_{k+1} - x_{k-1}
    const float gS = 0.5f * g_area * sgn(S);
    P2<float> g[5][10];
    for (int st = 0; st <= L; ++st)
        for (int i = 0; i < 10; ++i) g[st][i].x = g[st][i].y = 0.f;
    for (int k = 0; k < n; ++k) {
        const int km = (k == 0) ? n - 1 : k - 1, kp = (k + 1 == n) ? 0 : k + 1;
        g[L][k].x = gS * (T.v[L][km].y - T.v[L][kp].y);
        g[L][k].y = gS * (T.v[L][kp].x - T.v[L][km].x);
    }
    for (int st = L; st >= 1; --st) {
        const int ci = st - 1;
        const P2<float> cp2 = clip[ci], cp1 = clip[(ci + 3) & 3];
        const float dc0 = cp1.x - cp2.x, dc1 = cp1.y - cp2.y;
        const float n1 = cp1.x * cp2.y - cp1.y * cp2.x;
        for (int i = 0; i < T.n[st]; ++i) {
            const P2<float> gq = g[st][i];
            const int a = T.pa[st][i], bb = T.pb[st][i];
            if (bb < 0) {
                g[ci][a].x += gq.x;
                g[ci][a].y += gq.y;
                continue;
            }
            const P2<float> sv = T.v[ci][a], ev = T.v[ci][bb];
            const float dp0 = sv.x - ev.x, dp1 = sv.y - ev.y;
            const float n2 = sv.x * ev.y - sv.y * ev.x;
            const float n3 = 1.f / (dc0 * dp1 - dc1 * dp0);
            const float A = n1 * dp0 - n2 * dc0, Bq = n1 * dp1 - n2 * dc1;
            const float gA = gq.x * n3, gB = gq.y * n3;
            const float gden = -(n3 * n3) * (gq.x * A + gq.y * Bq);
            const float gdp0 = gA * n1 - gden * dc1, gdp1 = gB * n1 + gden * dc0;
            const float gn2 = -(gA * dc0 + gB * dc1);
            g[ci][a].x += gdp0 + gn2 * ev.y;
            g[ci][a].y += gdp1 - gn2 * ev.x;
            g[ci][bb].x += -gdp0 - gn2 * sv.y;
            g[ci][bb].y += -gdp1 + gn2 * sv.x;
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        gc[(3 - i) * 3] += g[0][i].x;
        gc[(3 - i) * 3 + 2] += g[0][i].y;
    }
    return area;
}

__global__ __launch_bounds__(128) void giou_bwd_kernel(
    const float* __restrict__ corners1, const float* __restrict__ corners2,
    const int32_t* __restrict__ nums, int B, int K1, int K2, int rotated_host,
    const int32_t* __restrict__ rotated_dev, const float* __restrict__ gout,
    float* __restrict__ gc1_out) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)B * K1) return;
    const bool rotated = rotated_dev ? (*rotated_dev != 0) : (rotated_host != 0);
    const int b = (int)(t / K1);
    const int nk = nums ? nums[b] : K2;
    float c1[24], gc[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) { c1[i] = corners1[t * 24 + i]; gc[i] = 0.f; }
    const float EPS = 1e-8f;
    // box-1 invariants
    float mn1[3], mx1[3];
    int amn1[3], amx1[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) { mn1[a] = INFINITY; mx1[a] = -INFINITY; amn1[a] = 0; amx1[a] = 0; }
#pragma unroll
    for (int v = 0; v < 8; ++v)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float val = c1[v * 3 + a];
            if (a == 1) val = -val;
            if (val < mn1[a]) { mn1[a] = val; amn1[a] = v; }
            if (val > mx1[a]) { mx1[a] = val; amx1[a] = v; }
        }
    const int ep[3][2] = {{0, 1}, {1, 2}, {0, 4}};
    float sq[3], len[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        const int a = ep[e][0], bb = ep[e][1];
        const float d0 = c1[a * 3] - c1[bb * 3], d1 = c1[a * 3 + 1] - c1[bb * 3 + 1],
                    d2 = c1[a * 3 + 2] - c1[bb * 3 + 2];
        sq[e] = d0 * d0 + d1 * d1 + d2 * d2;
        len[e] = sqrtf(fmaxf(sq[e], 1e-6f));
    }
    const float vraw1 = len[0] * len[1] * len[2];
    const float v1 = fmaxf(vraw1, EPS);
    float gv1 = 0.f;  // accumulated dL/dv1

    for (int k2 = 0; k2 < K2 && k2 < nk; ++k2) {
        const float G = gout[t * K2 + k2];
        if (G == 0.f) continue;
        const float* c2 = corners2 + ((long long)b * K2 + k2) * 24;
        const float ymax = fminf(c1[1], c2[1]);
        const float ymin = fmaxf(c1[13], c2[13]);
        const float hraw = ymax - ymin;
        const float height = fmaxf(hraw, 0.f);
        const float ltx = fmaxf(c1[6], c2[6]), ltz = fmaxf(c1[8], c2[8]);
        const float rbx = fminf(c1[0], c2[0]), rbz = fminf(c1[2], c2[2]);
        const float wxr = rbx - ltx, wzr = rbz - ltz;
        const float wx = fmaxf(wxr, 0.f), wz = fmaxf(wzr, 0.f);
        const float non_rot = wx * wz;
        // rotated: the clipped polygon's area where the axis-aligned overlap is nonzero
        // (box_util.py:583-585), its gradient taken once gI is known (below)
        float inter_area = non_rot;
        if (rotated) inter_area = non_rot != 0.f ? rot_area_grad(c1, c2, 0.f, gc) : 0.f;
        float mn2[3], mx2[3];
        minmax_flip(c2, mn2, mx2);
        const float X = fmaxf(mx1[0], mx2[0]) - fminf(mn1[0], mn2[0]);
        const float Y = fminf(mn1[1], mn2[1]) - fmaxf(mx1[1], mx2[1]);
        const float Z = fmaxf(mx1[2], mx2[2]) - fminf(mn1[2], mn2[2]);
        const float enc = fabsf(X) * fabsf(Y) * fabsf(Z);
        const float v2 = fmaxf(box_vol(c2), EPS);
        const float sum_vols = v1 + v2;
        const bool good = (enc > 2e-8f && sum_vols > 4e-8f);
        if (!good) continue;  // g * 0: no gradient (NaN-free by construction of good)
        const float I = inter_area * height;
        const float uraw = sum_vols - I;
        const float U = fmaxf(uraw, EPS);
        const float mU = (uraw >= EPS) ? 1.f : 0.f;
        const float A = -I / (U * U) + 1.f / enc;
        const float gI = G * (1.f / U - mU * A);
        gv1 += G * mU * A;
        const float genc = G * (-U / (enc * enc));
        // I = inter_area * height
        const float gnon = gI * height, gh = gI * inter_area;
        // height = clamp(ymax - ymin, 0)
        if (hraw >= 0.f) {
            bin_min_grad(c1[1], c2[1], gh, gc[1]);
            float tmp = 0.f;
            bin_max_grad(c1[13], c2[13], gh, tmp);
            gc[13] -= tmp;
        }
        if (rotated) {   // through the clip (non_rot only selects the pairs)
            if (non_rot != 0.f) rot_area_grad(c1, c2, gnon, gc);
        }
        // non_rot = wx * wz
        const float gwx = rotated ? 0.f : gnon * wz, gwz = rotated ? 0.f : gnon * wx;
        if (!rotated && wxr >= 0.f) {
            bin_min_grad(c1[0], c2[0], gwx, gc[0]);
            float tmp = 0.f;
            bin_max_grad(c1[6], c2[6], gwx, tmp);
            gc[6] -= tmp;
        }
        if (!rotated && wzr >= 0.f) {
            bin_min_grad(c1[2], c2[2], gwz, gc[2]);
            float tmp = 0.f;
            bin_max_grad(c1[8], c2[8], gwz, tmp);
            gc[8] -= tmp;
        }
        // enc = |X||Y||Z|
        const float gX = genc * fabsf(Y) * fabsf(Z) * sgn(X);
        const float gY = genc * fabsf(X) * fabsf(Z) * sgn(Y);
        const float gZ = genc * fabsf(X) * fabsf(Y) * sgn(Z);
        {   // X = max(mx1x, mx2x) - min(mn1x, mn2x)
            float g1 = 0.f, g2 = 0.f;
            bin_max_grad(mx1[0], mx2[0], gX, g1);
            bin_min_grad(mn1[0], mn2[0], gX, g2);
            gc[amx1[0] * 3] += g1;
            gc[amn1[0] * 3] -= g2;
        }
        {   // Y = min(mn1y', mn2y') - max(mx1y', mx2y'), y' = -y
            float g1 = 0.f, g2 = 0.f;
            bin_min_grad(mn1[1], mn2[1], gY, g1);
            bin_max_grad(mx1[1], mx2[1], gY, g2);
            gc[amn1[1] * 3 + 1] -= g1;
            gc[amx1[1] * 3 + 1] += g2;
        }
        {   // Z
            float g1 = 0.f, g2 = 0.f;
            bin_max_grad(mx1[2], mx2[2], gZ, g1);
            bin_min_grad(mn1[2], mn2[2], gZ, g2);
            gc[amx1[2] * 3 + 2] += g1;
            gc[amn1[2] * 3 + 2] -= g2;
        }
    }
    // v1 = clamp(len0*len1*len2, EPS)
    if (vraw1 >= EPS && gv1 != 0.f) {
        const float gl[3] = {gv1 * len[1] * len[2], gv1 * len[0] * len[2], gv1 * len[0] * len[1]};
#pragma unroll
        for (int e = 0; e < 3; ++e) {
            if (sq[e] < 1e-6f) continue;
            const float gs = gl[e] * 0.5f / len[e];
            const int a = ep[e][0], bb = ep[e][1];
#pragma unroll
            for (int ax = 0; ax < 3; ++ax) {
                const float d = c1[a * 3 + ax] - c1[bb * 3 + ax];
                gc[a * 3 + ax] += 2.f * d * gs;
                gc[bb * 3 + ax] -= 2.f * d * gs;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 24; ++i) gc1_out[t * 24 + i] = gc[i];
}

}  // namespace

extern "C" int ov3d_giou3d(const float* corners1, const float* corners2, const int32_t* nums, int B,
                           int K1, int K2, int mode, int rotated, const int32_t* rotated_dev,
                           int k2_bug, float* out, void* stream) {
    if (B < 0 || K1 < 0 || K2 < 0 || !corners1 || !corners2 || !out) return OV3D_EINVAL;
    if (mode != OV3D_GIOU_CYTHON && mode != OV3D_GIOU_TENSOR) return OV3D_EINVAL;
    const long long total = (long long)B * K1 * K2;
    if (total == 0) return OV3D_OK;
    hipLaunchKernelGGL(giou_kernel, dim3(ov3d_cdiv(total, 256)), dim3(256), 0, ov3d_stream(stream),
                       corners1, corners2, nums, B, K1, K2, mode, rotated, rotated_dev, k2_bug, out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_giou3d_bwd(const float* corners1, const float* corners2, const int32_t* nums,
                               int B, int K1, int K2, int rotated, const int32_t* rotated_dev,
                               const float* grad_out, float* grad_corners1, void* stream) {
    if (B < 0 || K1 < 0 || K2 < 0 || !corners1 || !corners2 || !grad_out || !grad_corners1)
        return OV3D_EINVAL;
    const long long total = (long long)B * K1;
    if (total == 0) return OV3D_OK;
    hipLaunchKernelGGL(giou_bwd_kernel, dim3(ov3d_cdiv(total, 128)), dim3(128), 0,
                       ov3d_stream(stream), corners1, corners2, nums, B, K1, K2, rotated,
                       rotated_dev, grad_out, grad_corners1);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_giou3d_bwd_aligned(const float* corners1, const float* corners2,
                                       const int32_t* nums, int B, int K1, int K2,
                                       const float* grad_out, float* grad_corners1, void* stream) {
    return ov3d_giou3d_bwd(corners1, corners2, nums, B, K1, K2, 0, nullptr, grad_out,
                           grad_corners1, stream);
}
