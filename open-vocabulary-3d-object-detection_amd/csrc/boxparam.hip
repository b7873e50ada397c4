// Box parametrisation of the 3DETR heads for all decoder layers, one launch each way.
//
// Reference: models/model_3detr.py BoxProcessor (19-69) + get_box_predictions (217-315),
// utils/pc_util.py shift_scale_points / scale_points, datasets/sunrgbd.py
// box_parametrization_to_corners -> utils/box_util.py flip_axis_to_camera_tensor +
// get_3d_box_batch_tensor:
//   center_offset = sigmoid(c) - 0.5;   center_u = query_xyz + center_offset
//   center_n      = (center_u - dmin) / (dmax - dmin)
//   size_n        = sigmoid(s);          size_u = size_n * max(dmax - dmin, 0.1)
//   angle_res     = angle_res_n * (pi / NB)
//   angle         = (2 pi / NB) * argmax(angle_logits) + angle_res[argmax]; angle > pi: - 2 pi
//                   (NB == 1: 0)
//   corners       = R_y(angle) (+-l/2, +-h/2, +-w/2) + flip(center_u)
//   sem_prob, objectness = softmax(logits)[:T-1], 1 - softmax(logits)[T-1]   (no grad)
// evaluated with the same fp32 operations as the torch expressions (models/model_3detr.py,
// box_util.py in this package; no FMA contraction).  Proposal (l, b, q) is row
// (l*B + b)*Q + q; the raw head outputs are row r of a (R, ld) matrix:
// [center 3 | size 3 | angle logits NB | angle residual NB] (heads.py out_s).
// Backward: one thread per proposal writes the gradient of its raw row from the gradients
// of every output (each may be absent), including the corner gradient (GIoU loss).
#include "common.h"

#include <math.h>

namespace {

constexpr int kThreads = 256;
constexpr float kPi = 3.14159265358979323846f;

__constant__ float kSX[8] = {1, 1, -1, -1, 1, 1, -1, -1};
__constant__ float kSY[8] = {1, 1, 1, 1, -1, -1, -1, -1};
__constant__ float kSZ[8] = {1, -1, -1, 1, 1, -1, -1, 1};

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

struct BoxArgs {
    long long R;
    int B, Q, NB, T;
    const float* raw; long long ld;
    const float* qxyz; const float* dmin; const float* dmax;
    const float* logits;
    float per_cls;      // (float)(2 pi / NB)
    float res_scale;    // (float)(pi / NB)
    float two_pi;       // (float)(2 pi)
    float pi_f;         // (float)pi
};

// the angle bin (first maximum) and the continuous angle of one row
__device__ __forceinline__ int angle_of(const BoxArgs& a, const float* r, float& angle) {
    if (a.NB == 1) {
        angle = 0.f;
        return 0;
    }
    const float* lg = r + 6;
    int cls = 0;
    float mx = lg[0];
    for (int t = 1; t < a.NB; ++t)
        if (lg[t] > mx) { mx = lg[t]; cls = t; }
    const float res = r[6 + a.NB + cls] * a.res_scale;
    const float ang = (float)cls * a.per_cls + res;
    angle = ang > a.pi_f ? ang - a.two_pi : ang;
    return cls;
}

__global__ void __launch_bounds__(kThreads) box_param_fwd_kernel(
    BoxArgs a, float* center_n, float* center_u, float* size_n, float* size_u, float* alog,
    float* ares_n, float* ares, float* angle_out, float* corners, float* sem_prob,
    float* obj_prob) {
    // blockIdx.y = part: 0 centre / size / angle / corners, 1 angle logits and residuals,
    // 2 class probabilities (a thread per proposal and part: the serial per-proposal chain
    // on 32 workgroups was latency-bound)
    const long long row = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (row >= a.R) return;
    const int part = blockIdx.y;
    const long long bq = row % ((long long)a.B * a.Q);
    const int b = (int)(bq / a.Q);
    const float* r = a.raw + row * a.ld;
    if (part == 2) {
        if (!a.logits) return;
        const float* x = a.logits + row * a.T;
        float mx = x[0];
        for (int t = 1; t < a.T; ++t) mx = fmaxf(mx, x[t]);
        float sum = 0.f;
        for (int t = 0; t < a.T; ++t) sum += expf(x[t] - mx);
        for (int t = 0; t < a.T - 1; ++t) sem_prob[row * (a.T - 1) + t] = expf(x[t] - mx) / sum;
        obj_prob[row] = 1.f - expf(x[a.T - 1] - mx) / sum;
        return;
    }
    if (part == 1) {
        for (int t = 0; t < a.NB; ++t) {
            alog[row * a.NB + t] = r[6 + t];
            const float rn = r[6 + a.NB + t];
            ares_n[row * a.NB + t] = rn;
            ares[row * a.NB + t] = rn * a.res_scale;
        }
        return;
    }
    float cu[3], su[3];
    for (int j = 0; j < 3; ++j) {
        const float lo = a.dmin[b * 3 + j], hi = a.dmax[b * 3 + j];
        const float off = sigm(r[j]) - 0.5f;
        cu[j] = a.qxyz[bq * 3 + j] + off;
        center_u[row * 3 + j] = cu[j];
        center_n[row * 3 + j] = ((cu[j] - lo) * 1.f) / (hi - lo) + 0.f;
        const float sn = sigm(r[3 + j]);
        size_n[row * 3 + j] = sn;
        su[j] = sn * fmaxf(hi - lo, 0.1f);
        size_u[row * 3 + j] = su[j];
    }
    float ang;
    angle_of(a, r, ang);
    angle_out[row] = ang;
    // corners: size (l, w, h) = su, center in camera axes (x, -z, y)
    const float l = su[0] / 2.f, w = su[1] / 2.f, h = su[2] / 2.f;
    const float c = cosf(ang), s = sinf(ang);
    const float cx = cu[0], cy = -cu[2], cz = cu[1];
    for (int k = 0; k < 8; ++k) {
        const float lx = l * kSX[k], ly = h * kSY[k], lz = w * kSZ[k];
        float* o = corners + (row * 8 + k) * 3;
        o[0] = (lx * c + lz * s) + cx;
        o[1] = ly + cy;
        o[2] = (lz * c - lx * s) + cz;
    }
}

struct BoxGrads {
    const float *center_n, *center_u, *size_n, *size_u, *alog, *ares_n, *ares, *angle, *corners;
};

__global__ void __launch_bounds__(kThreads) box_param_bwd_kernel(BoxArgs a, BoxGrads g,
                                                                 float* draw, long long ldd) {
    const long long row = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (row >= a.R) return;
    const long long bq = row % ((long long)a.B * a.Q);
    const int b = (int)(bq / a.Q);
    const float* r = a.raw + row * a.ld;
    float* d = draw + row * ldd;
    float sig_c[3], sig_s[3], dcu[3] = {0, 0, 0}, dsu[3] = {0, 0, 0}, scale[3];
    for (int j = 0; j < 3; ++j) {
        sig_c[j] = sigm(r[j]);
        sig_s[j] = sigm(r[3 + j]);
        const float lo = a.dmin[b * 3 + j], hi = a.dmax[b * 3 + j];
        scale[j] = fmaxf(hi - lo, 0.1f);
        if (g.center_n) dcu[j] += g.center_n[row * 3 + j] / (hi - lo);
        if (g.center_u) dcu[j] += g.center_u[row * 3 + j];
        if (g.size_u) dsu[j] += g.size_u[row * 3 + j];
    }
    float dang = g.angle ? g.angle[row] : 0.f;
    if (g.corners) {
        float ang;
        angle_of(a, r, ang);
        float su[3];
        for (int j = 0; j < 3; ++j) su[j] = sig_s[j] * scale[j];
        const float l = su[0] / 2.f, w = su[1] / 2.f;
        const float c = cosf(ang), s = sinf(ang);
        float dl = 0.f, dw = 0.f, dh = 0.f, dcx = 0.f, dcy = 0.f, dcz = 0.f;
        for (int k = 0; k < 8; ++k) {
            const float* go = g.corners + (row * 8 + k) * 3;
            const float lx = l * kSX[k], lz = w * kSZ[k];
            // x = lx c + lz s + cx ; y = ly + cy ; z = lz c - lx s + cz
            const float dlx = go[0] * c - go[2] * s;
            const float dlz = go[0] * s + go[2] * c;
            dl += dlx * kSX[k];
            dw += dlz * kSZ[k];
            dh += go[1] * kSY[k];
            dang += go[0] * (lz * c - lx * s) + go[2] * (-lz * s - lx * c);
            dcx += go[0];
            dcy += go[1];
            dcz += go[2];
        }
        dsu[0] += dl / 2.f;
        dsu[1] += dw / 2.f;
        dsu[2] += dh / 2.f;
        // camera center (x, -z, y) <- center_u
        dcu[0] += dcx;
        dcu[2] -= dcy;
        dcu[1] += dcz;
    }
    for (int j = 0; j < 3; ++j) {
        // sigmoid backward: grad * (1 - y) * y
        d[j] = dcu[j] * (1.f - sig_c[j]) * sig_c[j];
        float dsn = g.size_n ? g.size_n[row * 3 + j] : 0.f;
        dsn += dsu[j] * scale[j];
        d[3 + j] = dsn * (1.f - sig_s[j]) * sig_s[j];
    }
    int cls = -1;
    if (a.NB > 1 && dang != 0.f) {
        float ang;
        cls = angle_of(a, r, ang);
    }
    for (int t = 0; t < a.NB; ++t) {
        d[6 + t] = g.alog ? g.alog[row * a.NB + t] : 0.f;
        float dr = g.ares_n ? g.ares_n[row * a.NB + t] : 0.f;
        float dres = g.ares ? g.ares[row * a.NB + t] : 0.f;
        if (t == cls) dres += dang;
        d[6 + a.NB + t] = dr + dres * a.res_scale;
    }
}

BoxArgs make(long long R, int B, int Q, int NB, int T, const float* raw, long long ld,
             const float* qxyz, const float* dmin, const float* dmax, const float* logits) {
    BoxArgs a;
    a.R = R; a.B = B; a.Q = Q; a.NB = NB; a.T = T;
    a.raw = raw; a.ld = ld; a.qxyz = qxyz; a.dmin = dmin; a.dmax = dmax; a.logits = logits;
    a.per_cls = (float)(2.0 * 3.14159265358979323846 / NB);
    a.res_scale = (float)(3.14159265358979323846 / NB);
    a.two_pi = (float)(2.0 * 3.14159265358979323846);
    a.pi_f = kPi;
    return a;
}

bool args_ok(long long R, int B, int Q, int NB, const float* raw, long long ld, const float* qxyz,
             const float* dmin, const float* dmax) {
    return R > 0 && B > 0 && Q > 0 && NB >= 1 && R % ((long long)B * Q) == 0 && raw &&
           ld >= 6 + 2 * NB && qxyz && dmin && dmax;
}

}  // namespace

extern "C" int ov3d_box_param_fwd(long long R, int B, int Q, int NB, int T, const float* raw,
                                  long long ld, const float* qxyz, const float* dmin,
                                  const float* dmax, const float* logits, float* center_n,
                                  float* center_u, float* size_n, float* size_u, float* alog,
                                  float* ares_n, float* ares, float* angle, float* corners,
                                  float* sem_prob, float* obj_prob, void* stream) {
    if (!args_ok(R, B, Q, NB, raw, ld, qxyz, dmin, dmax) || !center_n || !center_u || !size_n ||
        !size_u || !alog || !ares_n || !ares || !angle || !corners ||
        (logits && (T < 2 || !sem_prob || !obj_prob)))
        return OV3D_EINVAL;
    const BoxArgs a = make(R, B, Q, NB, T, raw, ld, qxyz, dmin, dmax, logits);
    box_param_fwd_kernel<<<dim3(ov3d_cdiv(R, kThreads), 3), kThreads, 0, ov3d_stream(stream)>>>(
        a, center_n, center_u, size_n, size_u, alog, ares_n, ares, angle, corners, sem_prob,
        obj_prob);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_box_param_bwd(long long R, int B, int Q, int NB, const float* raw,
                                  long long ld, const float* qxyz, const float* dmin,
                                  const float* dmax, const float* g_center_n,
                                  const float* g_center_u, const float* g_size_n,
                                  const float* g_size_u, const float* g_alog, const float* g_ares_n,
                                  const float* g_ares, const float* g_angle, const float* g_corners,
                                  float* draw, long long ldd, void* stream) {
    if (!args_ok(R, B, Q, NB, raw, ld, qxyz, dmin, dmax) || !draw || ldd < 6 + 2 * NB)
        return OV3D_EINVAL;
    const BoxArgs a = make(R, B, Q, NB, 0, raw, ld, qxyz, dmin, dmax, nullptr);
    const BoxGrads g{g_center_n, g_center_u, g_size_n, g_size_u, g_alog, g_ares_n, g_ares, g_angle,
                     g_corners};
    box_param_bwd_kernel<<<ov3d_cdiv(R, kThreads), kThreads, 0, ov3d_stream(stream)>>>(a, g, draw,
                                                                                      ldd);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

// ---- Fourier position embedding (models/position_embedding.py:89-118) ----
// x = xyz (normalised to [0, 1] by the scene range when dmin != NULL) * 2 pi;
// p = x @ gauss_B (3 x d); out = [sin p | cos p]   (B, N, 2d) fp32, one thread per (point, j);
// seq_first: rows in (N, B) order instead (the transformer's sequence-first layout)
namespace {
__global__ void __launch_bounds__(256) fourier_pe_kernel(const float* __restrict__ xyz, long long BN,
                                                        int B, int N, const float* __restrict__ dmin,
                                                        const float* __restrict__ dmax,
                                                        const float* __restrict__ gb, int ldb,
                                                        int d, float two_pi, int seq_first,
                                                        float* __restrict__ out) {
    // 32-bit index arithmetic (the host checks BN * d < 2^31): the 64-bit divisions were
    // most of the kernel's instructions
    const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t >= (int)(BN * d)) return;
    const int pt = t / d;
    const int j = t - pt * d;
    const int b = pt / N;
    const long long orow = seq_first ? (long long)(pt - b * N) * B + b : (long long)pt;
    float x[3];
    for (int i = 0; i < 3; ++i) {
        float v = xyz[(long long)pt * 3 + i];
        if (dmin) v = ((v - dmin[b * 3 + i]) * 1.f) / (dmax[b * 3 + i] - dmin[b * 3 + i]) + 0.f;
        x[i] = v * two_pi;
    }
    const float p = fmaf(x[2], gb[2 * ldb + j], fmaf(x[1], gb[ldb + j], x[0] * gb[j]));
    out[orow * 2 * d + j] = sinf(p);
    out[orow * 2 * d + d + j] = cosf(p);
}
}  // namespace

extern "C" int ov3d_fourier_pe(const float* xyz, int B, int N, const float* dmin, const float* dmax,
                               const float* gauss_b, int ldb, int d, int seq_first, float* out,
                               void* stream) {
    if (!xyz || !gauss_b || !out || B <= 0 || N <= 0 || d <= 0 || ldb < d || (!dmin != !dmax))
        return OV3D_EINVAL;
    const long long n = (long long)B * N * d;
    if (n >= (1LL << 31)) return OV3D_EINVAL;
    fourier_pe_kernel<<<ov3d_cdiv(n, 256), 256, 0, ov3d_stream(stream)>>>(
        xyz, (long long)B * N, B, N, dmin, dmax, gauss_b, ldb, d, (float)(2.0 * 3.14159265358979323846),
        seq_first, out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
