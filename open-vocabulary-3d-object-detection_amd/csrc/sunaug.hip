// SUN RGB-D training-data pipeline on the device.
//
// Replaces SunrgbdDetectionDataset.__getitem__ (datasets/sunrgbd.py:256-462) with
// augment=True / False, use_color=False, use_height=False: the support-class box
// filter (:268-270), flip / rotation / scale (:309-352), RandomCuboid
// (utils/random_cuboid.py:38-98), the label build (:356-400), random_sampling
// (utils/pc_util.py:24-32) and the normalisations (:402-460).
//
// Every random draw comes from the host (the numpy RandomState calls of the
// reference, in the reference's order: sunaug.py builds that plan); these kernels
// apply it.  Arithmetic follows the numpy evaluation of the reference operation by
// operation, in the type numpy uses (T = the raw points' dtype, float or double):
//   np.dot(points, R^T)     -> dgemm: acc = +0, then fma(a_k, b_k, acc) for k = 0..2, f64
//   f32 array op f64 array  -> computed in f64, stored to the f32 array (one rounding)
//   f32 array op python float -> f32
// so the outputs are bit-identical to the reference's (tests/test_sunaug_*.py), up to
// numpy's float32 SIMD cos/sin in get_3d_box_batch_np (corners, <= 2 ulp).
//
// Layout: raw scenes resident in HBM, (S, raw_stride, raw_c) points of type T and
// (S, k_stride, 8) float64 boxes; a batch is a list of scene indices.
#include <float.h>

#include "common.h"

namespace {

constexpr int kAugThreads = 256;
constexpr int kScanThreads = 1024;
constexpr double kPi = 3.141592653589793;  // np.pi

template <typename T>
__device__ __forceinline__ double dpt(const T v) { return (double)v; }

// one element of a BLAS dgemm with K = 3 (np.dot / np.matmul of the reference): the
// accumulator starts at +0 and takes one fma per k (the sign of an exact zero follows)
__device__ __forceinline__ double dgemm3(double a0, double b0, double a1, double b1, double a2,
                                         double b2) {
    return fma(a2, b2, fma(a1, b1, fma(a0, b0, 0.0)));
}

// numpy remainder for float64 (npy_divmod): sign of the divisor, -0 -> +0 of divisor
__device__ __forceinline__ double np_mod(double a, double b) {
    double m = fmod(a, b);
    if (m != 0.0) {
        if ((b < 0.0) != (m < 0.0)) m += b;
    } else {
        m = copysign(0.0, b);
    }
    return m;
}

// ---------------------------------------------------------------------------
// (1) points: flip, rotation about z, scale.  Per-block partial min / max of the
//     augmented xyz (RandomCuboid's range_xyz, random_cuboid.py:39-41).
//     params (B, 8) f64: [flip, rot_angle, cos, sin, scale, 0, 0, 0]
template <typename T>
__global__ __launch_bounds__(kAugThreads) void aug_points_kernel(
    const T* __restrict__ raw, long long raw_stride, int raw_c, const int32_t* __restrict__ sidx,
    const int32_t* __restrict__ npts, int n_max, const double* __restrict__ params, int augment,
    T* __restrict__ out, T* __restrict__ part) {
    const int b = blockIdx.y;
    const int n = npts[b];
    const T* src = raw + (long long)sidx[b] * raw_stride * raw_c;
    T* dst = out + (long long)b * n_max * 3;
    const double* P = params + b * 8;
    const bool flip = P[0] != 0.0;
    const double c = P[2], s = P[3], sc = P[4];
    T lo[3] = {(T)INFINITY, (T)INFINITY, (T)INFINITY}, hi[3] = {-(T)INFINITY, -(T)INFINITY, -(T)INFINITY};
    const int i = blockIdx.x * kAugThreads + threadIdx.x;
    if (i < n) {
        T x = src[(long long)i * raw_c], y = src[(long long)i * raw_c + 1], z = src[(long long)i * raw_c + 2];
        if (augment) {
            if (flip) x = -x;                                   // -1 * pc[:, 0]
            // np.dot(pc[:, 0:3], rotz^T) in f64, R = [[c,-s,0],[s,c,0],[0,0,1]]
            const double dx = dpt(x), dy = dpt(y), dz = dpt(z);
            const T rx = (T)dgemm3(dx, c, dy, -s, dz, 0.0);
            const T ry = (T)dgemm3(dx, s, dy, c, dz, 0.0);
            const T rz = (T)dgemm3(dx, 0.0, dy, 0.0, dz, 1.0);
            // pc[:, 0:3] *= scale_ratio (f64 array): computed in f64, stored as T
            x = (T)(dpt(rx) * sc);
            y = (T)(dpt(ry) * sc);
            z = (T)(dpt(rz) * sc);
        }
        dst[(long long)i * 3] = x;
        dst[(long long)i * 3 + 1] = y;
        dst[(long long)i * 3 + 2] = z;
        lo[0] = x; lo[1] = y; lo[2] = z;
        hi[0] = x; hi[1] = y; hi[2] = z;
    }
    __shared__ T s_red[6][kAugThreads / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        for (int off = 32; off >= 1; off >>= 1) {
            lo[a] = fmin(lo[a], (T)__shfl_xor(lo[a], off));
            hi[a] = fmax(hi[a], (T)__shfl_xor(hi[a], off));
        }
        if (lane == 0) { s_red[a][w] = lo[a]; s_red[3 + a][w] = hi[a]; }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int a = threadIdx.x;
        T v = s_red[a][0];
        for (int q = 1; q < kAugThreads / 64; ++q) v = a < 3 ? fmin(v, s_red[a][q]) : fmax(v, s_red[a][q]);
        part[((long long)b * gridDim.x + blockIdx.x) * 6 + a] = v;
    }
}

template <typename T>
__device__ __forceinline__ void scene_range(const T* __restrict__ part, int b, int nparts, T lo[3],
                                            T hi[3]) {
    for (int a = 0; a < 3; ++a) { lo[a] = (T)INFINITY; hi[a] = -(T)INFINITY; }
    for (int q = 0; q < nparts; ++q) {
        const T* p = part + ((long long)b * nparts + q) * 6;
        for (int a = 0; a < 3; ++a) { lo[a] = fmin(lo[a], p[a]); hi[a] = fmax(hi[a], p[3 + a]); }
    }
}

// ---------------------------------------------------------------------------
// (2) boxes: train-split support-class filter (sunrgbd.py:266-268, np.isin on the
//     class column) of the first ngt boxes -- the GT boxes; boxes past them are the
//     use_pbox pseudo boxes, appended after the filter (sunrgbd.py:269-271) and never
//     filtered -- then the same flip / rotation / scale (sunrgbd.py:302-343).
//     One workgroup per scene; order-preserving compaction.
__global__ __launch_bounds__(kAugThreads) void aug_boxes_kernel(
    const double* __restrict__ raw, long long k_stride, const int32_t* __restrict__ sidx,
    const int32_t* __restrict__ nbox, const int32_t* __restrict__ ngt, int k_max,
    const double* __restrict__ params, int augment, const double* __restrict__ support,
    int n_support, double* __restrict__ out, int32_t* __restrict__ out_n) {
    const int b = blockIdx.x;
    const int k = nbox[b];
    const int kf = ngt ? ngt[b] : k;     // boxes the support filter applies to
    const double* src = raw + (long long)sidx[b] * k_stride * 8;
    double* dst = out + (long long)b * k_max * 8;
    const double* P = params + b * 8;
    __shared__ int s_base;
    __shared__ int s_wcnt[kAugThreads / 64];
    if (threadIdx.x == 0) s_base = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int c0 = 0; c0 < k; c0 += kAugThreads) {
        const int i = c0 + threadIdx.x;
        bool keep = i < k;
        if (keep && n_support > 0 && i < kf) {
            const double cls = src[(long long)i * 8 + 7];
            bool hit = false;
            for (int q = 0; q < n_support; ++q) hit |= cls == support[q];
            keep = hit;
        }
        const unsigned long long m = __ballot(keep);
        if (lane == 0) s_wcnt[w] = __popcll(m);
        __syncthreads();
        int pos = s_base + __popcll(m & lanemask_lt());
        for (int q = 0; q < w; ++q) pos += s_wcnt[q];
        if (keep && pos < k_max) {
            double bx[8];
            for (int a = 0; a < 8; ++a) bx[a] = src[(long long)i * 8 + a];
            if (augment) {
                if (P[0] != 0.0) { bx[0] = -1.0 * bx[0]; bx[6] = kPi - bx[6]; }
                const double c = P[2], s = P[3];
                const double x = bx[0], y = bx[1], z = bx[2];
                bx[0] = dgemm3(x, c, y, -s, z, 0.0);
                bx[1] = dgemm3(x, s, y, c, z, 0.0);
                bx[2] = dgemm3(x, 0.0, y, 0.0, z, 1.0);
                bx[6] -= P[1];
                for (int a = 0; a < 6; ++a) bx[a] *= P[4];
            }
            for (int a = 0; a < 8; ++a) dst[(long long)pos * 8 + a] = bx[a];
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int t = 0;
            for (int q = 0; q < kAugThreads / 64; ++q) t += s_wcnt[q];
            s_base += t;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) out_n[b] = min(s_base, k_max);
}

// crop bounds of one attempt (random_cuboid.py:55-60), all in f64 as numpy does
template <typename T>
__device__ __forceinline__ void crop_bounds(const T* __restrict__ pts, const T lo[3], const T hi[3],
                                            const double* __restrict__ att, double mn[3],
                                            double mx[3]) {
    const long long ci = (long long)att[3];
    for (int a = 0; a < 3; ++a) {
        const T range = hi[a] - lo[a];                      // np.max - np.min (T)
        const double nr = dpt(range) * att[a] / 2.0;         // range_xyz * crop_range / 2.0
        const double ctr = dpt(pts[ci * 3 + a]);
        mx[a] = ctr + nr;
        mn[a] = ctr - nr;
    }
}

template <typename T>
__device__ __forceinline__ bool in_crop(const T* __restrict__ p, const double mn[3], const double mx[3]) {
    const double x = dpt(p[0]), y = dpt(p[1]), z = dpt(p[2]);
    return x <= mx[0] && y <= mx[1] && z <= mx[2] && x >= mn[0] && y >= mn[1] && z >= mn[2];
}

// ---------------------------------------------------------------------------
// (3) RandomCuboid: every attempt of every scene at once, one workgroup each.
//     attempts (B, A, 4) f64 = crop_range xyz + sampled centre index (-1: the attempt
//     failed check_aspect and drew no centre).  Writes per attempt the point count, the
//     crop's point min / max (T) and the accept flag (count >= min_points and, when the
//     boxes sum to > 0, at least one box centre inside the crop's point bbox).
template <typename T>
__global__ __launch_bounds__(kScanThreads) void cuboid_eval_kernel(
    const T* __restrict__ pts, int n_max, const int32_t* __restrict__ npts, const T* __restrict__ part,
    int nparts, const double* __restrict__ attempts, int A, int min_points,
    const double* __restrict__ boxes, const int32_t* __restrict__ nbox, int k_max,
    int32_t* __restrict__ counts, T* __restrict__ crop_mm, int32_t* __restrict__ accept) {
    const int t = blockIdx.x, b = blockIdx.y;
    const double* att = attempts + ((long long)b * A + t) * 4;
    const long long o = (long long)b * A + t;
    if (att[3] < 0.0) {
        if (threadIdx.x == 0) { counts[o] = 0; accept[o] = 0; }
        return;
    }
    const int n = npts[b];
    const T* P = pts + (long long)b * n_max * 3;
    T lo[3], hi[3];
    scene_range(part, b, nparts, lo, hi);
    double mn[3], mx[3];
    crop_bounds(P, lo, hi, att, mn, mx);
    int cnt = 0;
    T plo[3] = {(T)INFINITY, (T)INFINITY, (T)INFINITY}, phi[3] = {-(T)INFINITY, -(T)INFINITY, -(T)INFINITY};
    for (int i = threadIdx.x; i < n; i += kScanThreads) {
        const T* p = P + (long long)i * 3;
        if (in_crop(p, mn, mx)) {
            ++cnt;
            for (int a = 0; a < 3; ++a) { plo[a] = fmin(plo[a], p[a]); phi[a] = fmax(phi[a], p[a]); }
        }
    }
    __shared__ int s_cnt[kScanThreads / 64];
    __shared__ T s_mm[6][kScanThreads / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int off = 32; off >= 1; off >>= 1) {
        cnt += __shfl_xor(cnt, off);
        for (int a = 0; a < 3; ++a) {
            plo[a] = fmin(plo[a], (T)__shfl_xor(plo[a], off));
            phi[a] = fmax(phi[a], (T)__shfl_xor(phi[a], off));
        }
    }
    if (lane == 0) {
        s_cnt[w] = cnt;
        for (int a = 0; a < 3; ++a) { s_mm[a][w] = plo[a]; s_mm[3 + a][w] = phi[a]; }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int total = 0;
        T m[6];
        for (int a = 0; a < 3; ++a) { m[a] = (T)INFINITY; m[3 + a] = -(T)INFINITY; }
        for (int q = 0; q < kScanThreads / 64; ++q) {
            total += s_cnt[q];
            for (int a = 0; a < 3; ++a) { m[a] = fmin(m[a], s_mm[a][q]); m[3 + a] = fmax(m[3 + a], s_mm[3 + a][q]); }
        }
        for (int a = 0; a < 6; ++a) crop_mm[o * 6 + a] = m[a];
        counts[o] = total;
        int ok = total >= min_points;
        if (ok) {
            // box filter policy "center" (random_cuboid.py:72-88)
            const int k = nbox[b];
            const double* bx = boxes + (long long)b * k_max * 8;
            double sum = 0.0;
            for (int i = 0; i < k * 8; ++i) sum += bx[i];
            if (sum > 0.0) {
                int kept = 0;
                for (int i = 0; i < k; ++i) {
                    bool in = true;
                    for (int a = 0; a < 3; ++a)
                        in = in && bx[i * 8 + a] >= dpt(m[a]) && bx[i * 8 + a] <= dpt(m[3 + a]);
                    kept += in;
                }
                ok = kept > 0;
            }
        }
        accept[o] = ok;
    }
}

// first accepted attempt per scene (or -1: the fallback keeps every point), and the
// number of points random_sampling draws from.  sel (B, 2) int32.
__global__ void cuboid_select_kernel(const int32_t* __restrict__ counts,
                                     const int32_t* __restrict__ accept, int A,
                                     const int32_t* __restrict__ npts, int B,
                                     int32_t* __restrict__ sel) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    int t = -1;
    for (int q = 0; q < A && t < 0; ++q)
        if (accept[(long long)b * A + q]) t = q;
    sel[2 * b] = t;
    sel[2 * b + 1] = t < 0 ? npts[b] : counts[(long long)b * A + t];
}

// ---------------------------------------------------------------------------
// (4) order-preserving compaction of the selected crop: crop_idx[b, j] = the j-th
//     in-crop point (new_point_cloud = point_cloud[new_pointidx], random_cuboid.py:65).
template <typename T>
__global__ __launch_bounds__(kScanThreads) void crop_compact_kernel(
    const T* __restrict__ pts, int n_max, const int32_t* __restrict__ npts, const T* __restrict__ part,
    int nparts, const double* __restrict__ attempts, int A, const int32_t* __restrict__ sel,
    int32_t* __restrict__ crop_idx) {
    const int b = blockIdx.x;
    const int n = npts[b];
    const int t = sel[2 * b];
    const T* P = pts + (long long)b * n_max * 3;
    int32_t* dst = crop_idx + (long long)b * n_max;
    double mn[3], mx[3];
    if (t >= 0) {
        T lo[3], hi[3];
        scene_range(part, b, nparts, lo, hi);
        crop_bounds(P, lo, hi, attempts + ((long long)b * A + t) * 4, mn, mx);
    }
    __shared__ int s_wcnt[kScanThreads / 64];
    __shared__ int s_base;
    if (threadIdx.x == 0) s_base = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int c0 = 0; c0 < n; c0 += kScanThreads) {
        const int i = c0 + threadIdx.x;
        const bool keep = i < n && (t < 0 || in_crop(P + (long long)i * 3, mn, mx));
        const unsigned long long m = __ballot(keep);
        if (lane == 0) s_wcnt[w] = __popcll(m);
        __syncthreads();
        int pos = s_base + __popcll(m & lanemask_lt());
        for (int q = 0; q < w; ++q) pos += s_wcnt[q];
        if (keep) dst[pos] = i;
        __syncthreads();
        if (threadIdx.x == 0) {
            int tot = 0;
            for (int q = 0; q < kScanThreads / 64; ++q) tot += s_wcnt[q];
            s_base += tot;
        }
        __syncthreads();
    }
}

// (5) random_sampling gather: out[b, i] = float(points[crop_idx[choices[b, i]]]); per-block
//     min / max of the sampled points (point_cloud_dims_min / max, sunrgbd.py:402-403).
template <typename T>
__global__ __launch_bounds__(kAugThreads) void sample_gather_kernel(
    const T* __restrict__ pts, int n_max, const int32_t* __restrict__ crop_idx,
    const int64_t* __restrict__ choices, int num_points, float* __restrict__ out,
    T* __restrict__ dpart) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * kAugThreads + threadIdx.x;
    T lo[3] = {(T)INFINITY, (T)INFINITY, (T)INFINITY}, hi[3] = {-(T)INFINITY, -(T)INFINITY, -(T)INFINITY};
    if (i < num_points) {
        const long long j = choices[(long long)b * num_points + i];
        const int src = crop_idx[(long long)b * n_max + j];
        const T* p = pts + ((long long)b * n_max + src) * 3;
        for (int a = 0; a < 3; ++a) {
            out[((long long)b * num_points + i) * 3 + a] = (float)p[a];
            lo[a] = p[a];
            hi[a] = p[a];
        }
    }
    __shared__ T s_red[6][kAugThreads / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int a = 0; a < 3; ++a) {
        for (int off = 32; off >= 1; off >>= 1) {
            lo[a] = fmin(lo[a], (T)__shfl_xor(lo[a], off));
            hi[a] = fmax(hi[a], (T)__shfl_xor(hi[a], off));
        }
        if (lane == 0) { s_red[a][w] = lo[a]; s_red[3 + a][w] = hi[a]; }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int a = threadIdx.x;
        T v = s_red[a][0];
        for (int q = 1; q < kAugThreads / 64; ++q) v = a < 3 ? fmin(v, s_red[a][q]) : fmax(v, s_red[a][q]);
        dpart[((long long)b * gridDim.x + blockIdx.x) * 6 + a] = v;
    }
}

// ---------------------------------------------------------------------------
// (6) labels (sunrgbd.py:356-460), one workgroup of max_num_obj threads per scene.
template <typename T>
__global__ void labels_kernel(ov3d_sun_labels_args a) {
    const int b = blockIdx.x;
    const int i = threadIdx.x;
    const int G = a.max_num_obj;
    const int k = a.nbox[b];
    const double* bx = a.boxes + (long long)b * a.k_max * 8;
    // RandomCuboid's box filter of the selected attempt (or none: fallback / augment off)
    const int t = a.sel ? a.sel[2 * b] : -1;
    __shared__ int s_keep[256];
    __shared__ double s_sum;
    if (i == 0) {
        double sum = 0.0;
        for (int q = 0; q < k * 8; ++q) sum += bx[q];
        s_sum = sum;
    }
    __syncthreads();
    const T* cmm = (const T*)a.crop_mm;
    for (int q = i; q < k; q += blockDim.x) {
        bool keep = true;
        if (t >= 0 && s_sum > 0.0) {
            const T* m = cmm + ((long long)b * a.num_attempts + t) * 6;
            for (int c = 0; c < 3; ++c) keep = keep && bx[q * 8 + c] >= dpt(m[c]) && bx[q * 8 + c] <= dpt(m[3 + c]);
        }
        s_keep[q] = keep;
    }
    __syncthreads();
    // i-th kept box (order-preserving), if any
    int src = -1, seen = 0;
    for (int q = 0; q < k && src < 0; ++q) {
        if (s_keep[q]) {
            if (seen == i) src = q;
            ++seen;
        }
    }
    // point_cloud_dims_min / max from the sampled points' partials
    const T* dp = (const T*)a.dims_part;
    T dmin[3] = {(T)INFINITY, (T)INFINITY, (T)INFINITY}, dmax[3] = {-(T)INFINITY, -(T)INFINITY, -(T)INFINITY};
    for (int q = 0; q < a.n_dims_part; ++q) {
        const T* p = dp + ((long long)b * a.n_dims_part + q) * 6;
        for (int c = 0; c < 3; ++c) { dmin[c] = fmin(dmin[c], p[c]); dmax[c] = fmax(dmax[c], p[3 + c]); }
    }
    if (i < 3) {
        ((T*)a.dims_min)[b * 3 + i] = dmin[i];
        ((T*)a.dims_max)[b * 3 + i] = dmax[i];
    }
    if (i >= G) return;
    const long long o = (long long)b * G + i;
    const bool present = src >= 0;
    // per-box label values (zeros for padded slots, as the reference's np.zeros)
    float raw_size[3] = {0.f, 0.f, 0.f};
    float center[3] = {0.f, 0.f, 0.f};
    int64_t ang_cls = 0, sem = 0;
    float ang_res = 0.f;
    if (present) {
        const double* B8 = bx + (long long)src * 8;
        sem = (int64_t)B8[7];
        for (int c = 0; c < 3; ++c) raw_size[c] = (float)(B8[3 + c] * 2.0);
        // angle2class (sunrgbd.py:102-120)
        const double two_pi = 2.0 * kPi;
        const double per = two_pi / (double)a.num_angle_bin;
        const double ang = np_mod(B8[6], two_pi);
        const double shifted = np_mod(ang + per / 2.0, two_pi);
        const int cid = (int)(shifted / per);
        ang_cls = cid;
        ang_res = (float)(shifted - ((double)cid * per + per / 2.0));
        // my_compute_box_3d (sunrgbd.py:153-165) -> axis-aligned box centre
        const double h = -1.0 * B8[6];
        const double c = cos(h), s = sin(h);
        const double l = B8[3], w = B8[4], hh = B8[5];
        const double xc[8] = {-l, l, l, -l, -l, l, l, -l};
        const double yc[8] = {w, w, -w, -w, w, w, -w, -w};
        const double zc[8] = {hh, hh, hh, hh, -hh, -hh, -hh, -hh};
        double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int q = 0; q < 8; ++q) {
            // np.dot(R, vstack(...)) (dgemm, R = rotz(-heading)) then += center
            const double v[3] = {dgemm3(c, xc[q], -s, yc[q], 0.0, zc[q]) + B8[0],
                                 dgemm3(s, xc[q], c, yc[q], 0.0, zc[q]) + B8[1],
                                 dgemm3(0.0, xc[q], 0.0, yc[q], 1.0, zc[q]) + B8[2]};
            for (int d = 0; d < 3; ++d) { mn[d] = fmin(mn[d], v[d]); mx[d] = fmax(mx[d], v[d]); }
        }
        for (int d = 0; d < 3; ++d) center[d] = (float)((mn[d] + mx[d]) / 2.0);
    }
    // normalisations with the sampled points' range (sunrgbd.py:405-425)
    float size_n[3], center_n[3];
    for (int c = 0; c < 3; ++c) {
        const T mult = dmax[c] - dmin[c];
        const T inv = (T)1.0 / mult;                             // 1.0 / mult_factor
        size_n[c] = (float)((T)raw_size[c] * inv);              // scale_points
        const T src_diff = dmax[c] - dmin[c];
        const T v = (((T)center[c] - dmin[c]) * (T)1.0f) / src_diff + (T)0.0f;  // shift_scale_points
        center_n[c] = (float)((double)v * (present ? 1.0 : 0.0));       // * target_bboxes_mask
    }
    // class2angle_batch (sunrgbd.py:131-138), int64 class * python float + f32 residual
    const double per = 2.0 * kPi / (double)a.num_angle_bin;
    double ang = (double)ang_cls * per + (double)ang_res;
    if (ang > kPi) ang = ang - 2.0 * kPi;
    const float angf = (float)ang;
    // get_3d_box_batch_np(raw_sizes, raw_angles.astype(f32), flip_axis_to_camera_np(centers))
    const float cx = center[0], cy = -center[2], cz = center[1];
    const double cc = (double)cosf(angf), ss = (double)sinf(angf);
    const double L = (double)(raw_size[0] / 2), W = (double)(raw_size[1] / 2), H = (double)(raw_size[2] / 2);
    const double px[8] = {L, L, -L, -L, L, L, -L, -L};
    const double py[8] = {H, H, H, H, -H, -H, -H, -H};
    const double pz[8] = {W, -W, -W, W, W, -W, -W, W};
    float* cor = a.corners + o * 24;
    for (int q = 0; q < 8; ++q) {
        // corners @ R^T, R = roty = [[c,0,s],[0,1,0],[-s,0,c]] (dgemm order), += center
        const double vx = dgemm3(px[q], cc, py[q], 0.0, pz[q], ss);
        const double vy = dgemm3(px[q], 0.0, py[q], 1.0, pz[q], 0.0);
        const double vz = dgemm3(px[q], -ss, py[q], 0.0, pz[q], cc);
        cor[q * 3 + 0] = (float)(vx + (double)cx);
        cor[q * 3 + 1] = (float)(vy + (double)cy);
        cor[q * 3 + 2] = (float)(vz + (double)cz);
    }
    for (int c = 0; c < 3; ++c) {
        a.centers[o * 3 + c] = center[c];
        a.centers_normalized[o * 3 + c] = center_n[c];
        a.sizes[o * 3 + c] = raw_size[c];
        a.sizes_normalized[o * 3 + c] = size_n[c];
    }
    a.sem_cls[o] = sem;
    a.present[o] = present ? 1.f : 0.f;
    a.angles[o] = angf;
    a.angle_cls[o] = ang_cls;
    a.angle_res[o] = ang_res;
}

}  // namespace

extern "C" int ov3d_sun_aug_points(const void* raw, int pc_f64, long long raw_stride, int raw_c,
                                   const int32_t* scene_idx, const int32_t* npts, int B, int n_max,
                                   const double* params, int augment, void* out, void* range_part,
                                   void* stream) {
    if (!raw || !scene_idx || !npts || !params || !out || !range_part || B < 0 || n_max <= 0 ||
        raw_c < 3 || raw_stride < n_max)
        return OV3D_EINVAL;
    if (B == 0) return OV3D_OK;
    const dim3 grid(ov3d_sun_range_parts(n_max), B);
    hipStream_t s = ov3d_stream(stream);
    if (pc_f64)
        hipLaunchKernelGGL(aug_points_kernel<double>, grid, dim3(kAugThreads), 0, s, (const double*)raw,
                           raw_stride, raw_c, scene_idx, npts, n_max, params, augment, (double*)out,
                           (double*)range_part);
    else
        hipLaunchKernelGGL(aug_points_kernel<float>, grid, dim3(kAugThreads), 0, s, (const float*)raw,
                           raw_stride, raw_c, scene_idx, npts, n_max, params, augment, (float*)out,
                           (float*)range_part);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_sun_range_parts(int n) { return (n + kAugThreads - 1) / kAugThreads; }

extern "C" int ov3d_sun_aug_boxes(const double* raw, long long k_stride, const int32_t* scene_idx,
                                  const int32_t* nbox, const int32_t* ngt, int B, int k_max,
                                  const double* params, int augment, const double* support,
                                  int n_support, double* out, int32_t* out_n, void* stream) {
    if (!raw || !scene_idx || !nbox || !params || !out || !out_n || B < 0 || k_max <= 0 ||
        k_stride <= 0 || n_support < 0 || (n_support > 0 && !support))
        return OV3D_EINVAL;
    if (B == 0) return OV3D_OK;
    hipLaunchKernelGGL(aug_boxes_kernel, dim3(B), dim3(kAugThreads), 0, ov3d_stream(stream), raw,
                       k_stride, scene_idx, nbox, ngt, k_max, params, augment, support, n_support,
                       out, out_n);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_sun_cuboid_eval(const void* pts, int pc_f64, int n_max, const int32_t* npts,
                                    const void* range_part, const double* attempts, int B, int A,
                                    int min_points, const double* boxes, const int32_t* nbox,
                                    int k_max, int32_t* counts, void* crop_mm, int32_t* accept,
                                    int32_t* sel, void* stream) {
    if (!pts || !npts || !range_part || !attempts || !boxes || !nbox || !counts || !crop_mm ||
        !accept || !sel || B < 0 || A <= 0 || n_max <= 0)
        return OV3D_EINVAL;
    if (B == 0) return OV3D_OK;
    hipStream_t s = ov3d_stream(stream);
    const int np = ov3d_sun_range_parts(n_max);
    if (pc_f64)
        hipLaunchKernelGGL(cuboid_eval_kernel<double>, dim3(A, B), dim3(kScanThreads), 0, s,
                           (const double*)pts, n_max, npts, (const double*)range_part, np, attempts, A,
                           min_points, boxes, nbox, k_max, counts, (double*)crop_mm, accept);
    else
        hipLaunchKernelGGL(cuboid_eval_kernel<float>, dim3(A, B), dim3(kScanThreads), 0, s,
                           (const float*)pts, n_max, npts, (const float*)range_part, np, attempts, A,
                           min_points, boxes, nbox, k_max, counts, (float*)crop_mm, accept);
    hipLaunchKernelGGL(cuboid_select_kernel, dim3((B + 63) / 64), dim3(64), 0, s, counts, accept, A,
                       npts, B, sel);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_sun_crop_sample(const void* pts, int pc_f64, int n_max, const int32_t* npts,
                                    const void* range_part, const double* attempts, int B, int A,
                                    const int32_t* sel, const int64_t* choices, int num_points,
                                    int32_t* crop_idx, float* out, void* dims_part, void* stream) {
    if (!pts || !npts || !range_part || !attempts || !sel || !choices || !crop_idx || !out ||
        !dims_part || B < 0 || A <= 0 || n_max <= 0 || num_points <= 0)
        return OV3D_EINVAL;
    if (B == 0) return OV3D_OK;
    hipStream_t s = ov3d_stream(stream);
    const int np = ov3d_sun_range_parts(n_max);
    const dim3 g2(ov3d_sun_range_parts(num_points), B);
    if (pc_f64) {
        hipLaunchKernelGGL(crop_compact_kernel<double>, dim3(B), dim3(kScanThreads), 0, s,
                           (const double*)pts, n_max, npts, (const double*)range_part, np, attempts, A,
                           sel, crop_idx);
        hipLaunchKernelGGL(sample_gather_kernel<double>, g2, dim3(kAugThreads), 0, s,
                           (const double*)pts, n_max, crop_idx, choices, num_points, out,
                           (double*)dims_part);
    } else {
        hipLaunchKernelGGL(crop_compact_kernel<float>, dim3(B), dim3(kScanThreads), 0, s,
                           (const float*)pts, n_max, npts, (const float*)range_part, np, attempts, A,
                           sel, crop_idx);
        hipLaunchKernelGGL(sample_gather_kernel<float>, g2, dim3(kAugThreads), 0, s,
                           (const float*)pts, n_max, crop_idx, choices, num_points, out,
                           (float*)dims_part);
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_sun_labels(const ov3d_sun_labels_args* args, int pc_f64, void* stream) {
    if (!args || args->B < 0 || args->max_num_obj <= 0 || args->max_num_obj > 256 ||
        args->k_max > 256 || args->num_angle_bin <= 0 || !args->boxes || !args->nbox ||
        !args->dims_part || !args->dims_min || !args->dims_max || !args->corners)
        return OV3D_EINVAL;
    if (args->sel && !args->crop_mm) return OV3D_EINVAL;
    if (args->B == 0) return OV3D_OK;
    const int threads = ((max(args->max_num_obj, 3) + 63) / 64) * 64;
    if (pc_f64)
        hipLaunchKernelGGL(labels_kernel<double>, dim3(args->B), dim3(threads), 0,
                           ov3d_stream(stream), *args);
    else
        hipLaunchKernelGGL(labels_kernel<float>, dim3(args->B), dim3(threads), 0,
                           ov3d_stream(stream), *args);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
