// 3DETR set-criterion losses for every decoder layer: one launch forward, one backward.
//
// Reference: criterion.py SetCriterion — loss_sem_cls (143-178: weighted cross-entropy,
// unmatched proposals labelled background), loss_angle (180-246: cross-entropy on the
// matched GT bin + Huber(delta 1) on the residual of that bin, normalised by pi/nbins),
// loss_center (248-272: L1 of the matched centre, the gathered cdist(p=1)), loss_size
// (298-337: L1 over the 3 normalised sizes), loss_giou (274-296: 1 - GIoU of the match),
// loss_cardinality (121-130, logged), the weighting of 402-419 and the layer sum of
// 425-442 (final layer first, then the auxiliary layers).
//
// Rows: proposal (l, b, q) is row (l*B + b)*Q + q of every (L*B*Q, n) operand, read
// through a row stride so column slices of a wider head output need no copy.
//
// Forward: one workgroup per decoder layer accumulates that layer's sums in fp64 and
// writes the unweighted per-layer terms; the last workgroup to finish (ticket counter,
// reset by that workgroup) forms the (L, 8) table of weighted dict values in the
// reference's key order and the total in the reference's summation order
// (criterion.py:415-419: per layer 0 + w_k0*l_k0 + w_k1*l_k1 ...; layers summed
// final, aux 0, aux 1, ...), in fp32 like the torch expression.
// Backward: one thread per proposal writes its rows of every gradient.
#include "common.h"

#include <math.h>

namespace {

constexpr int kThreads = 256;
constexpr int kCols = OV3D_LOSS_NCOLS;   // sem, angle_cls, angle_reg, center, size, giou, 2d, card
constexpr int kRaw = kCols + 1;          // + the layer's sum of class weights (sem denominator)

__device__ __forceinline__ int clampi(long long v, int hi) {
    return v < 0 ? 0 : (v > hi ? hi : (int)v);
}

__device__ __forceinline__ float huber(float e) {
    // reference utils/misc.py:25-36 with delta = 1: 0.5*q^2 + (a - q), q = min(a, 1)
    const float a = fabsf(e);
    const float q = fminf(a, 1.f);
    return 0.5f * (q * q) + (a - q);
}

__device__ __forceinline__ float sgnf(float x) { return (float)((x > 0.f) - (x < 0.f)); }

// position of computation layer l in the reference's (final, aux 0, aux 1, ...) order
__device__ __forceinline__ int dict_pos(const ov3d_set_loss_desc& d, int l) {
    return d.final_last ? (l == d.L - 1 ? 0 : l + 1) : l;
}
__device__ __forceinline__ int layer_at(const ov3d_set_loss_desc& d, int i) {
    return d.final_last ? (i == 0 ? d.L - 1 : i - 1) : i;
}
// row of (layer l, proposal p of the layer) in the matcher's outputs: computation order, or
// the reference's problem order (final layer first) when match_ref_order
__device__ __forceinline__ long long match_row(const ov3d_set_loss_desc& d, int l, int p) {
    const int lm = d.match_ref_order ? dict_pos(d, l) : l;
    return (long long)lm * d.B * d.Q + p;
}

// max, index of the first maximum and sum of exp(x - max) over n values
__device__ __forceinline__ void softmax_stats(const float* x, int n, float& mx, int& am, float& s) {
    mx = x[0];
    am = 0;
    for (int t = 1; t < n; ++t)
        if (x[t] > mx) { mx = x[t]; am = t; }
    s = 0.f;
    for (int t = 0; t < n; ++t) s += expf(x[t] - mx);
}

__device__ __forceinline__ double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// the loss terms of proposal p of computation layer l into acc (sem num, sem den, angle cls,
// angle reg, center, size, giou) and the scene's count of non-background argmax (cnt, LDS)
__device__ __forceinline__ void proposal_terms(const ov3d_set_loss_desc& d, int l, int p, int P,
                                               double* acc, int* cnt) {
    const int b = p / d.Q;
    const long long row = (long long)l * P + p;
    const long long mrow = match_row(d, l, p);
    const float m = d.matched[mrow];
    const int g = clampi(d.inds[mrow], d.G - 1);
    const long long bg = (long long)b * d.G + g;

    const float* x = d.logits + row * d.ld_logits;
    float mx, s;
    int am;
    softmax_stats(x, d.T, mx, am, s);
    if (am != d.T - 1) atomicAdd(&cnt[b], 1);
    if (d.flags & OV3D_LOSS_SEM) {
        const int lab = (m == 0.f) ? d.T - 1 : clampi(d.gt_sem[bg], d.T - 1);
        const float nll = logf(s) - (x[lab] - mx);
        const float wt = d.cls_weights[lab];
        acc[0] += (double)(nll * wt);
        acc[1] += (double)wt;
    }
    {
        const float* a = d.angle_logits + row * d.ld_angle_logits;
        float ma, sa;
        int ia;
        softmax_stats(a, d.NB, ma, ia, sa);
        const int gl = clampi(d.gt_angle_cls[bg], d.NB - 1);
        acc[2] += (double)((logf(sa) - (a[gl] - ma)) * m);
        const float gr = d.gt_angle_res[bg] * d.res_scale;
        const float e = d.angle_res[row * d.ld_angle_res + gl] - gr;
        acc[3] += (double)(huber(e) * m);
    }
    if (d.flags & OV3D_LOSS_CENTER) {
        const float* c = d.center + row * d.ld_center;
        const float* gc = d.gt_center + bg * 3;
        const float cl = (fabsf(c[0] - gc[0]) + fabsf(c[1] - gc[1])) + fabsf(c[2] - gc[2]);
        acc[4] += (double)(cl * m);
    }
    if (d.flags & OV3D_LOSS_SIZE) {
        const float* z = d.size + row * d.ld_size;
        const float* gz = d.gt_size + bg * 3;
        const float sl = (fabsf(z[0] - gz[0]) + fabsf(z[1] - gz[1])) + fabsf(z[2] - gz[2]);
        acc[5] += (double)(sl * m);
    }
    if (d.flags & OV3D_LOSS_GIOU) {
        acc[6] += (double)((1.f - d.gious[row * d.G + g]) * m);
    }
}

// one layer's raw loss row (criterion.py:274-311 terms, normalised as the reference)
__device__ __forceinline__ void layer_raw(const ov3d_set_loss_desc& d, int l, const double* t,
                                          float card_sum, float* raw) {
    const float nb = *d.num_boxes;
    float* r = raw + (long long)l * kRaw;
    r[0] = (d.flags & OV3D_LOSS_SEM) ? (float)t[0] / (float)t[1] : 0.f;
    r[1] = (float)t[2] / nb;
    r[2] = (float)t[3] / nb;
    r[3] = (d.flags & OV3D_LOSS_CENTER) ? (float)t[4] / nb : 0.f;
    r[4] = (d.flags & OV3D_LOSS_SIZE) ? (float)t[5] / nb : 0.f;
    r[5] = (d.flags & OV3D_LOSS_GIOU) ? (float)t[6] / nb : 0.f;
    r[6] = (d.flags & OV3D_LOSS_ALIGN) ? d.align[l] : 0.f;
    r[7] = card_sum / (float)d.B;
    r[8] = (float)t[1];
}

// the dict table and the total from every layer's raw row (one thread)
__device__ __forceinline__ void finalize_total(const ov3d_set_loss_desc& d, const float* raw,
                                               float* dict_out, float* total) {
    float tot = 0.f;
    for (int i = 0; i < d.L; ++i) {
        const float* r = raw + (long long)layer_at(d, i) * kRaw;
        for (int k = 0; k < kCols; ++k) dict_out[i * kCols + k] = r[k] * d.dict_w[k];
        float ll = 0.f;
        for (int j = 0; j < d.n_total; ++j) {
            const int k = d.total_order[j];
            ll = (j == 0) ? r[k] * d.dict_w[k] : ll + r[k] * d.dict_w[k];
        }
        tot = (i == 0) ? ll : tot + ll;
    }
    if (d.match_status) {   // a matching that scipy would have refused poisons the total
        int bad = 0;
        for (int p = 0; p < d.n_status; ++p) bad |= d.match_status[p];
        if (bad) tot = __int_as_float(0x7fc00000);
    }
    *total = tot;
}

__global__ void __launch_bounds__(kThreads) set_loss_fwd_kernel(ov3d_set_loss_desc d, float* raw,
                                                                 int* ticket, float* dict_out,
                                                                 float* total) {
    const int l = blockIdx.x;
    const int P = d.B * d.Q;
    __shared__ int cnt[OV3D_LOSS_MAX_B];
    __shared__ double red[kThreads / 64][7];
    __shared__ int is_last;
    for (int b = threadIdx.x; b < d.B; b += kThreads) cnt[b] = 0;
    __syncthreads();

    double acc[7] = {0, 0, 0, 0, 0, 0, 0};   // sem num, sem den, acls, areg, center, size, giou
    for (int p = threadIdx.x; p < P; p += kThreads) proposal_terms(d, l, p, P, acc, cnt);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const double v = wave_sum(acc[k]);
        if (lane == 0) red[w][k] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t[7];
        for (int k = 0; k < 7; ++k) {
            t[k] = 0;
            for (int j = 0; j < kThreads / 64; ++j) t[k] += red[j][k];
        }
        float card = 0.f;
        for (int b = 0; b < d.B; ++b) card += fabsf((float)cnt[b] - (float)d.nactual[b]);
        layer_raw(d, l, t, card, raw);
        __threadfence();
        is_last = (atomicAdd(ticket, 1) == d.L - 1);
    }
    __syncthreads();
    if (!is_last || threadIdx.x != 0) return;
    __threadfence();
    finalize_total(d, raw, dict_out, total);
    *ticket = 0;
}

// Split form (ov3d_set_loss_fwd_split): a workgroup per (chunk of kThreads proposals, layer),
// one proposal per thread (the per-layer form runs 4 proposals per thread through two
// softmaxes each on 8 workgroups: latency-bound).  Each workgroup writes its chunk's 7 sums
// and per-scene argmax counts; the last one to finish adds each layer's chunks in chunk
// order (deterministic) and finalises as the per-layer form.
__global__ void __launch_bounds__(kThreads) set_loss_fwd_split_kernel(
    ov3d_set_loss_desc d, float* raw, int* ticket, float* dict_out, float* total,
    double* __restrict__ part) {
    const int S = gridDim.x, sidx = blockIdx.x, l = blockIdx.y;
    const int P = d.B * d.Q, W = 7 + d.B;
    __shared__ int cnt[OV3D_LOSS_MAX_B];
    __shared__ double red[kThreads / 64][7];
    __shared__ int is_last;
    for (int b = threadIdx.x; b < d.B; b += kThreads) cnt[b] = 0;
    __syncthreads();
    double acc[7] = {0, 0, 0, 0, 0, 0, 0};
    const int p = sidx * kThreads + threadIdx.x;
    if (p < P) proposal_terms(d, l, p, P, acc, cnt);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const double v = wave_sum(acc[k]);
        if (lane == 0) red[w][k] = v;
    }
    __syncthreads();
    double* mine = part + ((size_t)l * S + sidx) * W;
    if (threadIdx.x < 7) {
        double t = 0;
        for (int j = 0; j < kThreads / 64; ++j) t += red[j][threadIdx.x];
        mine[threadIdx.x] = t;
    }
    for (int b = threadIdx.x; b < d.B; b += kThreads) mine[7 + b] = (double)cnt[b];
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) is_last = (atomicAdd(ticket, 1) == d.L * S - 1);
    __syncthreads();
    if (!is_last) return;
    __threadfence();
    for (int ll = threadIdx.x; ll < d.L; ll += kThreads) {
        double t[7] = {0, 0, 0, 0, 0, 0, 0};
        const double* pl = part + (size_t)ll * S * W;
        for (int c = 0; c < S; ++c)
            for (int k = 0; k < 7; ++k) t[k] += pl[(size_t)c * W + k];
        float card = 0.f;
        for (int b = 0; b < d.B; ++b) {
            double n = 0;
            for (int c = 0; c < S; ++c) n += pl[(size_t)c * W + 7 + b];
            card += fabsf((float)n - (float)d.nactual[b]);
        }
        layer_raw(d, ll, t, card, raw);
    }
    __threadfence();
    __syncthreads();
    if (threadIdx.x != 0) return;
    finalize_total(d, raw, dict_out, total);
    *ticket = 0;
}

__global__ void __launch_bounds__(kThreads) set_loss_bwd_kernel(
    ov3d_set_loss_desc d, const float* raw, const float* d_dict, const float* d_total,
    float* g_logits, float* g_alog, float* g_ares, float* g_center, float* g_size, float* g_gious,
    float* g_align) {
    const int P = d.B * d.Q;
    const long long row = (long long)blockIdx.x * kThreads + threadIdx.x;
    const float dt = d_total ? *d_total : 0.f;
    if (blockIdx.x == 0 && threadIdx.x < d.L && g_align) {
        const int l = threadIdx.x;
        const float dd = d_dict ? d_dict[dict_pos(d, l) * kCols + 6] : 0.f;
        g_align[l] = d.dict_w[6] * dd + d.total_w[6] * dt;
    }
    if (row >= (long long)d.L * P) return;
    const int l = (int)(row / P);
    const int b = (int)((row % P) / d.Q);
    const int i = dict_pos(d, l);
    float c[6];
#pragma unroll
    for (int k = 0; k < 6; ++k)
        c[k] = d.dict_w[k] * (d_dict ? d_dict[i * kCols + k] : 0.f) + d.total_w[k] * dt;
    const float nb = *d.num_boxes;
    const long long mrow = match_row(d, l, (int)(row % P));
    const float m = d.matched[mrow];
    const int g = clampi(d.inds[mrow], d.G - 1);
    const long long bg = (long long)b * d.G + g;

    if (g_logits) {
        const float* x = d.logits + row * d.ld_logits;
        float* gx = g_logits + row * d.T;
        float mx, s;
        int am;
        softmax_stats(x, d.T, mx, am, s);
        const int lab = (m == 0.f) ? d.T - 1 : clampi(d.gt_sem[bg], d.T - 1);
        const float den = raw[(long long)l * kRaw + 8];
        const float gn = (c[0] / den) * d.cls_weights[lab];
        const float inv = 1.f / s;
        for (int t = 0; t < d.T; ++t)
            gx[t] = gn * (expf(x[t] - mx) * inv - (t == lab ? 1.f : 0.f));
    }
    const float* a = d.angle_logits + row * d.ld_angle_logits;
    const int gl = clampi(d.gt_angle_cls[bg], d.NB - 1);
    if (g_alog) {
        float ma, sa;
        int ia;
        softmax_stats(a, d.NB, ma, ia, sa);
        const float gce = (c[1] / nb) * m;
        const float inv = 1.f / sa;
        float* ga = g_alog + row * d.NB;
        for (int t = 0; t < d.NB; ++t) ga[t] = gce * (expf(a[t] - ma) * inv - (t == gl ? 1.f : 0.f));
    }
    if (g_ares) {
        const float gr = d.gt_angle_res[bg] * d.res_scale;
        const float e = d.angle_res[row * d.ld_angle_res + gl] - gr;
        const float gh = (c[2] / nb) * m * (sgnf(e) * fminf(fabsf(e), 1.f));
        float* ga = g_ares + row * d.NB;
        for (int t = 0; t < d.NB; ++t) ga[t] = (t == gl) ? gh : 0.f;
    }
    if (g_center) {
        const float* cc = d.center + row * d.ld_center;
        const float* gc = d.gt_center + bg * 3;
        const float gk = (c[3] / nb) * m;
        for (int j = 0; j < 3; ++j) g_center[row * 3 + j] = gk * sgnf(cc[j] - gc[j]);
    }
    if (g_size) {
        const float* z = d.size + row * d.ld_size;
        const float* gz = d.gt_size + bg * 3;
        const float gk = (c[4] / nb) * m;
        for (int j = 0; j < 3; ++j) g_size[row * 3 + j] = gk * sgnf(z[j] - gz[j]);
    }
    if (g_gious) {
        const float gk = -(c[5] / nb) * m;
        float* gg = g_gious + row * d.G;
        for (int j = 0; j < d.G; ++j) gg[j] = (j == g) ? gk : 0.f;
    }
}

// ---- 16 lanes per proposal row (the forward split and the backward): the two softmaxes'
// statistics as lane-parallel reductions, the gradient rows written by consecutive lanes.  One
// thread per row took 35 us (forward) and 26 us (backward) per SUN step on 32 workgroups: every
// lane walked its own row serially, every load and store touching 64 rows.
constexpr int kGrp = 16;                       // lanes per row
constexpr int kRowsPerWG = kThreads / kGrp;    // 16 rows per workgroup
constexpr int kGrpMaxN = 2 * kGrp;             // softmax widths served (T, NB)
constexpr int kTailMaxL = 32;                  // layers the parallel tail serves

// group_softmax_stats == softmax_stats for n <= 32 values spread over the row's 16 lanes (lane
// j: values j and j + 16): the same maximum and first argmax; the sum in a fixed tree order
__device__ __forceinline__ void group_softmax_stats(const float* x, int n, int j, float& mx,
                                                    int& am, float& s) {
    const float v0 = j < n ? x[j] : -INFINITY;
    const float v1 = j + kGrp < n ? x[j + kGrp] : -INFINITY;
    float m = v0;
    int i = j;
    if (v1 > m) {
        m = v1;
        i = j + kGrp;
    }
#pragma unroll
    for (int o = kGrp / 2; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, kGrp);
        const int i2 = __shfl_xor(i, o, kGrp);
        if (m2 > m || (m2 == m && i2 < i)) {
            m = m2;
            i = i2;
        }
    }
    float e = (j < n ? expf(v0 - m) : 0.f) + (j + kGrp < n ? expf(v1 - m) : 0.f);
#pragma unroll
    for (int o = kGrp / 2; o > 0; o >>= 1) e += __shfl_xor(e, o, kGrp);
    mx = m;
    am = i;
    s = e;
}

// proposal_terms with the two softmaxes over the row's lanes (every lane of the row calls it;
// lane 0 accumulates)
__device__ __forceinline__ void proposal_terms_grp(const ov3d_set_loss_desc& d, int l, int p, int P,
                                                   int j, double* acc, int* cnt) {
    const int b = p / d.Q;
    const long long row = (long long)l * P + p;
    const long long mrow = match_row(d, l, p);
    const float m = d.matched[mrow];
    const int g = clampi(d.inds[mrow], d.G - 1);
    const long long bg = (long long)b * d.G + g;
    const float* x = d.logits + row * d.ld_logits;
    float mx, s;
    int am;
    group_softmax_stats(x, d.T, j, mx, am, s);
    const float* a = d.angle_logits + row * d.ld_angle_logits;
    float ma, sa;
    int ia;
    group_softmax_stats(a, d.NB, j, ma, ia, sa);
    if (j != 0) return;
    if (am != d.T - 1) atomicAdd(&cnt[b], 1);
    if (d.flags & OV3D_LOSS_SEM) {
        const int lab = (m == 0.f) ? d.T - 1 : clampi(d.gt_sem[bg], d.T - 1);
        const float nll = logf(s) - (x[lab] - mx);
        const float wt = d.cls_weights[lab];
        acc[0] += (double)(nll * wt);
        acc[1] += (double)wt;
    }
    {
        const int gl = clampi(d.gt_angle_cls[bg], d.NB - 1);
        acc[2] += (double)((logf(sa) - (a[gl] - ma)) * m);
        const float gr = d.gt_angle_res[bg] * d.res_scale;
        const float e = d.angle_res[row * d.ld_angle_res + gl] - gr;
        acc[3] += (double)(huber(e) * m);
    }
    if (d.flags & OV3D_LOSS_CENTER) {
        const float* c = d.center + row * d.ld_center;
        const float* gc = d.gt_center + bg * 3;
        const float cl = (fabsf(c[0] - gc[0]) + fabsf(c[1] - gc[1])) + fabsf(c[2] - gc[2]);
        acc[4] += (double)(cl * m);
    }
    if (d.flags & OV3D_LOSS_SIZE) {
        const float* z = d.size + row * d.ld_size;
        const float* gz = d.gt_size + bg * 3;
        const float sl = (fabsf(z[0] - gz[0]) + fabsf(z[1] - gz[1])) + fabsf(z[2] - gz[2]);
        acc[5] += (double)(sl * m);
    }
    if (d.flags & OV3D_LOSS_GIOU) acc[6] += (double)((1.f - d.gious[row * d.G + g]) * m);
}

// the split forward on 16-row workgroups: chunk partials only.  No last-workgroup ticket: its
// device-scope fence per workgroup (512 of them) took the launch from 35 to 79 us; the sums
// and the finalise are a second, one-workgroup launch (set_loss_tail_kernel)
__global__ void __launch_bounds__(kThreads) set_loss_fwd_grp_kernel(
    ov3d_set_loss_desc d, double* __restrict__ part) {
    const int S = gridDim.x, sidx = blockIdx.x, l = blockIdx.y;
    const int P = d.B * d.Q, W = 7 + d.B;
    __shared__ int cnt[OV3D_LOSS_MAX_B];
    __shared__ double gred[kRowsPerWG][7];
    for (int b = threadIdx.x; b < d.B; b += kThreads) cnt[b] = 0;
    __syncthreads();
    double acc[7] = {0, 0, 0, 0, 0, 0, 0};
    const int j = threadIdx.x & (kGrp - 1);
    const int p = sidx * kRowsPerWG + threadIdx.x / kGrp;
    if (p < P) proposal_terms_grp(d, l, p, P, j, acc, cnt);
    // the groups' sums (lane 0 of each) through LDS, not double wave shuffles
    if (j == 0) {
#pragma unroll
        for (int k = 0; k < 7; ++k) gred[threadIdx.x / kGrp][k] = acc[k];
    }
    __syncthreads();
    double* mine = part + ((size_t)l * S + sidx) * W;
    if (threadIdx.x < 7) {
        double t = 0;
        for (int q = 0; q < kRowsPerWG; ++q) t += gred[q][threadIdx.x];
        mine[threadIdx.x] = t;
    }
    for (int b = threadIdx.x; b < d.B; b += kThreads) mine[7 + b] = (double)cnt[b];
}

// every (layer, column) summed over the S chunks by one wave (lane c, c + 64, ... then a fixed
// lane tree: deterministic; a thread per pair walking the chunks serially waited one load
// round trip per chunk, 34 us); then the per-layer rows and the total (one workgroup, after
// the partials' launch)
__global__ void __launch_bounds__(kThreads) set_loss_tail_kernel(
    ov3d_set_loss_desc d, int S, const double* __restrict__ part, float* raw, float* dict_out,
    float* total) {
    const int W = 7 + d.B;
    __shared__ double tot[kTailMaxL][7 + OV3D_LOSS_MAX_B];
    // a thread per (layer, column), chunks in chunk order, 16 loads in flight at a time (one
    // load per chunk step waited a round trip each; a wave tree of double shuffles per pair
    // was as slow: ~12 ds_bpermute per pair, back to back)
    const int LW = d.L * W;
    for (int pc = threadIdx.x; pc < LW; pc += kThreads) {
        const int ll = pc / W, k = pc - ll * W;
        const double* pl = part + (size_t)ll * S * W + k;
        double t = 0;
        int c = 0;
        for (; c + 16 <= S; c += 16) {
            double x[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) x[u] = pl[(size_t)(c + u) * W];
#pragma unroll
            for (int u = 0; u < 16; ++u) t += x[u];
        }
        for (; c < S; ++c) t += pl[(size_t)c * W];
        tot[ll][k] = t;
    }
    __syncthreads();
    // the rows in LDS, then every output from there: finalize_total's loads of raw behind its
    // own stores to dict_out (possible aliases) ran as ~130 serial round trips
    __shared__ float sraw[kTailMaxL][kRaw];
    for (int ll = threadIdx.x; ll < d.L; ll += kThreads) {
        double t[7];
        for (int k = 0; k < 7; ++k) t[k] = tot[ll][k];
        float card = 0.f;
        for (int b = 0; b < d.B; ++b) card += fabsf((float)tot[ll][7 + b] - (float)d.nactual[b]);
        layer_raw(d, ll, t, card, &sraw[0][0]);
    }
    int bad = 0;
    if (d.match_status)
        for (int q = threadIdx.x; q < d.n_status; q += kThreads) bad |= d.match_status[q];
    bad = __syncthreads_or(bad);
    for (int q = threadIdx.x; q < d.L * kRaw; q += kThreads) raw[q] = (&sraw[0][0])[q];
    for (int q = threadIdx.x; q < d.L * kCols; q += kThreads) {
        const int i = q / kCols, k = q - i * kCols;
        dict_out[q] = sraw[layer_at(d, i)][k] * d.dict_w[k];
    }
    if (threadIdx.x != 0) return;
    float tt = 0.f;   // finalize_total's order
    for (int i = 0; i < d.L; ++i) {
        const float* r = sraw[layer_at(d, i)];
        float ll = 0.f;
        for (int j = 0; j < d.n_total; ++j) {
            const int k = d.total_order[j];
            ll = (j == 0) ? r[k] * d.dict_w[k] : ll + r[k] * d.dict_w[k];
        }
        tt = (i == 0) ? ll : tt + ll;
    }
    *total = bad ? __int_as_float(0x7fc00000) : tt;   // a refused matching poisons the total
}

__global__ void __launch_bounds__(kThreads) set_loss_bwd_grp_kernel(
    ov3d_set_loss_desc d, const float* raw, const float* d_dict, const float* d_total,
    float* g_logits, float* g_alog, float* g_ares, float* g_center, float* g_size, float* g_gious,
    float* g_align) {
    const int P = d.B * d.Q;
    const int j = threadIdx.x & (kGrp - 1);
    const long long row = (long long)blockIdx.x * kRowsPerWG + threadIdx.x / kGrp;
    const float dt = d_total ? *d_total : 0.f;
    if (blockIdx.x == 0 && threadIdx.x < d.L && g_align) {
        const int l = threadIdx.x;
        const float dd = d_dict ? d_dict[dict_pos(d, l) * kCols + 6] : 0.f;
        g_align[l] = d.dict_w[6] * dd + d.total_w[6] * dt;
    }
    if (row >= (long long)d.L * P) return;   // the whole row's group
    const int l = (int)(row / P);
    const int b = (int)((row % P) / d.Q);
    const int i = dict_pos(d, l);
    float c[6];
#pragma unroll
    for (int k = 0; k < 6; ++k)
        c[k] = d.dict_w[k] * (d_dict ? d_dict[i * kCols + k] : 0.f) + d.total_w[k] * dt;
    const float nb = *d.num_boxes;
    const long long mrow = match_row(d, l, (int)(row % P));
    const float m = d.matched[mrow];
    const int g = clampi(d.inds[mrow], d.G - 1);
    const long long bg = (long long)b * d.G + g;
    if (g_logits) {
        const float* x = d.logits + row * d.ld_logits;
        float* gx = g_logits + row * d.T;
        float mx, s;
        int am;
        group_softmax_stats(x, d.T, j, mx, am, s);
        const int lab = (m == 0.f) ? d.T - 1 : clampi(d.gt_sem[bg], d.T - 1);
        const float den = raw[(long long)l * kRaw + 8];
        const float gn = (c[0] / den) * d.cls_weights[lab];
        const float inv = 1.f / s;
        for (int t = j; t < d.T; t += kGrp)
            gx[t] = gn * (expf(x[t] - mx) * inv - (t == lab ? 1.f : 0.f));
    }
    const float* a = d.angle_logits + row * d.ld_angle_logits;
    const int gl = clampi(d.gt_angle_cls[bg], d.NB - 1);
    if (g_alog) {
        float ma, sa;
        int ia;
        group_softmax_stats(a, d.NB, j, ma, ia, sa);
        const float gce = (c[1] / nb) * m;
        const float inv = 1.f / sa;
        float* ga = g_alog + row * d.NB;
        for (int t = j; t < d.NB; t += kGrp)
            ga[t] = gce * (expf(a[t] - ma) * inv - (t == gl ? 1.f : 0.f));
    }
    if (g_ares) {
        const float gr = d.gt_angle_res[bg] * d.res_scale;
        const float e = d.angle_res[row * d.ld_angle_res + gl] - gr;
        const float gh = (c[2] / nb) * m * (sgnf(e) * fminf(fabsf(e), 1.f));
        float* ga = g_ares + row * d.NB;
        for (int t = j; t < d.NB; t += kGrp) ga[t] = (t == gl) ? gh : 0.f;
    }
    if (g_center && j < 3) {
        const float* cc = d.center + row * d.ld_center;
        const float* gc = d.gt_center + bg * 3;
        g_center[row * 3 + j] = ((c[3] / nb) * m) * sgnf(cc[j] - gc[j]);
    }
    if (g_size && j < 3) {
        const float* z = d.size + row * d.ld_size;
        const float* gz = d.gt_size + bg * 3;
        g_size[row * 3 + j] = ((c[4] / nb) * m) * sgnf(z[j] - gz[j]);
    }
    if (g_gious) {
        const float gk = -(c[5] / nb) * m;
        float* gg = g_gious + row * d.G;
        for (int t = j; t < d.G; t += kGrp) gg[t] = (t == g) ? gk : 0.f;
    }
}

int check_desc(const ov3d_set_loss_desc* d) {
    if (!d || d->L <= 0 || d->B <= 0 || d->Q <= 0 || d->G <= 0 || d->T < 1 || d->NB < 1 ||
        d->B > OV3D_LOSS_MAX_B || !d->logits || !d->angle_logits || !d->angle_res || !d->inds ||
        !d->matched || !d->gt_angle_cls || !d->gt_angle_res || !d->nactual || !d->num_boxes ||
        d->ld_logits < d->T || d->ld_angle_logits < d->NB || d->ld_angle_res < d->NB ||
        d->n_total < 0 || d->n_total > kCols)
        return OV3D_EINVAL;
    if ((d->flags & OV3D_LOSS_SEM) && (!d->gt_sem || !d->cls_weights)) return OV3D_EINVAL;
    if ((d->flags & OV3D_LOSS_CENTER) && (!d->center || !d->gt_center || d->ld_center < 3))
        return OV3D_EINVAL;
    if ((d->flags & OV3D_LOSS_SIZE) && (!d->size || !d->gt_size || d->ld_size < 3))
        return OV3D_EINVAL;
    if ((d->flags & OV3D_LOSS_GIOU) && !d->gious) return OV3D_EINVAL;
    if ((d->flags & OV3D_LOSS_ALIGN) && !d->align) return OV3D_EINVAL;
    for (int j = 0; j < d->n_total; ++j)
        if (d->total_order[j] < 0 || d->total_order[j] >= kCols - 1) return OV3D_EINVAL;
    return OV3D_OK;
}

}  // namespace

// the 16-lanes-per-row kernels serve softmax widths up to 32 and up to 32 layers
static bool grp_ok(const ov3d_set_loss_desc& d) {
    return d.T <= kGrpMaxN && d.NB <= kGrpMaxN && d.L <= kTailMaxL;
}

extern "C" long long ov3d_set_loss_desc_size(void) { return (long long)sizeof(ov3d_set_loss_desc); }

extern "C" int ov3d_set_loss_fwd(const ov3d_set_loss_desc* desc, float* raw, int* ticket,
                                 float* dict_out, float* total, void* stream) {
    if (check_desc(desc) != OV3D_OK || !raw || !ticket || !dict_out || !total) return OV3D_EINVAL;
    set_loss_fwd_kernel<<<desc->L, kThreads, 0, ov3d_stream(stream)>>>(*desc, raw, ticket, dict_out,
                                                                       total);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

/* doubles of scratch ov3d_set_loss_fwd_split needs */
extern "C" long long ov3d_set_loss_fwd_parts(int L, int B, int Q) {
    if (L <= 0 || B <= 0 || Q <= 0) return 0;
    // the 16-row chunks of the grouped kernel (more than the 256-row chunks of the other)
    return (long long)L * ((B * Q + kRowsPerWG - 1) / kRowsPerWG) * (7 + B);
}

extern "C" int ov3d_set_loss_fwd_split(const ov3d_set_loss_desc* desc, float* raw, int* ticket,
                                       float* dict_out, float* total, double* parts, void* stream) {
    if (check_desc(desc) != OV3D_OK || !raw || !ticket || !dict_out || !total || !parts)
        return OV3D_EINVAL;
    if (grp_ok(*desc)) {
        const int S = (desc->B * desc->Q + kRowsPerWG - 1) / kRowsPerWG;
        set_loss_fwd_grp_kernel<<<dim3(S, desc->L), kThreads, 0, ov3d_stream(stream)>>>(*desc, parts);
        OV3D_LAUNCH_CHECK();
        set_loss_tail_kernel<<<1, kThreads, 0, ov3d_stream(stream)>>>(*desc, S, parts, raw, dict_out,
                                                                      total);
        OV3D_LAUNCH_CHECK();
        return OV3D_OK;
    }
    const int S = (desc->B * desc->Q + kThreads - 1) / kThreads;
    set_loss_fwd_split_kernel<<<dim3(S, desc->L), kThreads, 0, ov3d_stream(stream)>>>(
        *desc, raw, ticket, dict_out, total, parts);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_set_loss_bwd(const ov3d_set_loss_desc* desc, const float* raw,
                                 const float* d_dict, const float* d_total, float* g_logits,
                                 float* g_angle_logits, float* g_angle_res, float* g_center,
                                 float* g_size, float* g_gious, float* g_align, void* stream) {
    if (check_desc(desc) != OV3D_OK || !raw || desc->L > kThreads) return OV3D_EINVAL;
    const ov3d_set_loss_desc& d = *desc;
    if ((g_logits && !(d.flags & OV3D_LOSS_SEM)) || (g_center && !(d.flags & OV3D_LOSS_CENTER)) ||
        (g_size && !(d.flags & OV3D_LOSS_SIZE)) || (g_gious && !(d.flags & OV3D_LOSS_GIOU)) ||
        (g_align && !(d.flags & OV3D_LOSS_ALIGN)))
        return OV3D_EINVAL;
    const long long rows = (long long)d.L * d.B * d.Q;
    if (grp_ok(d)) {
        set_loss_bwd_grp_kernel<<<ov3d_cdiv(rows, kRowsPerWG), kThreads, 0, ov3d_stream(stream)>>>(
            d, raw, d_dict, d_total, g_logits, g_angle_logits, g_angle_res, g_center, g_size,
            g_gious, g_align);
        OV3D_LAUNCH_CHECK();
        return OV3D_OK;
    }
    set_loss_bwd_kernel<<<ov3d_cdiv(rows, kThreads), kThreads, 0, ov3d_stream(stream)>>>(
        d, raw, d_dict, d_total, g_logits, g_angle_logits, g_angle_res, g_center, g_size, g_gious,
        g_align);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

// ---- Hungarian matcher cost and target counts (criterion.py:33-92, 346-360, 425) ----
namespace {

// cost[p, q, g] = w_cls * (-prob[p, q, label[b, g]]) + w_obj * (-obj[p, q])
//               + w_center * |center[p, q] - gt_center[b, g]|_1 + w_giou * (-giou[p, q, g]),
// b = p % B (the L*B problems stack the B scenes L times); one thread per (p, q, g)
__global__ void __launch_bounds__(256) matcher_cost_kernel(
    long long total, int B, int Q, int G, int C, int L, int final_last,
    const float* __restrict__ prob, long long ldp,
    const float* __restrict__ obj, const float* __restrict__ center, const float* __restrict__ gious,
    const float* __restrict__ gt_center, const int64_t* __restrict__ gt_label, float w_cls,
    float w_obj, float w_center, float w_giou, float* __restrict__ cost) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int g = (int)(t % G);
    const long long pq = t / G;
    const long long p = pq / Q;
    const int b = (int)(p % B);
    const int lab = clampi(gt_label[(long long)b * G + g], C - 1);
    const float* c = center + pq * 3;
    const float* gc = gt_center + ((long long)b * G + g) * 3;
    const float dist = (fabsf(c[0] - gc[0]) + fabsf(c[1] - gc[1])) + fabsf(c[2] - gc[2]);
    const float v = ((w_cls * (-prob[pq * ldp + lab]) + w_obj * (-obj[pq])) + w_center * dist) +
                    w_giou * (-gious[t]);
    // problem p = l*B + b goes to the reference's problem order (final layer first:
    // criterion.py:431-444) when final_last, i.e. layer l -> position (l + 1) % L
    const long long l = p / B;
    const long long lo = final_last ? (l + 1) % L : l;
    cost[((lo * B + b) * Q + (pq % Q)) * G + g] = v;
}

// per scene: nactual = (int64)(sum present), int32 copies repeated L times, the replica's
// box count, the clamped num_boxes (single process) and the rotated flag (any angle > 0)
__global__ void __launch_bounds__(256) targets_prep_kernel(int B, int G, int L,
                                                          const float* __restrict__ present,
                                                          const float* __restrict__ angles,
                                                          int64_t* nact64, int32_t* nact32_rep,
                                                          int64_t* total, float* num_boxes,
                                                          int32_t* rotated) {
    // a wave per scene (lanes over its boxes: the box flags are 0 / 1, so the float count is
    // exact in any order), the four waves' totals through LDS.  A thread per scene and one
    // thread adding 256 LDS slots took 9.9 us.
    __shared__ long long cnt[4];
    __shared__ int rot[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    long long my = 0;
    int r = 0;
    for (int b = wave; b < B; b += 4) {
        float s = 0.f;
        int rb = 0;
        for (int g = lane; g < G; g += 64) {
            s += present[(long long)b * G + g];
            rb |= angles[(long long)b * G + g] > 0.f;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            s += __shfl_xor(s, o);
            rb |= __shfl_xor(rb, o);
        }
        const long long n = (long long)s;
        if (lane == 0) nact64[b] = n;
        for (int l = lane; l < L; l += 64) nact32_rep[(long long)l * B + b] = (int32_t)n;
        my += n;
        r |= rb;
    }
    if (lane == 0) {
        cnt[wave] = my;
        rot[wave] = r;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const long long t = (cnt[0] + cnt[1]) + (cnt[2] + cnt[3]);
        *total = t;
        if (num_boxes) *num_boxes = fmaxf((float)t, 1.f);
        *rotated = rot[0] | rot[1] | rot[2] | rot[3];
    }
}

}  // namespace

extern "C" int ov3d_matcher_cost(int P, int B, int Q, int G, int C, int final_last,
                                 const float* prob, long long ldp, const float* obj,
                                 const float* center,
                                 const float* gious, const float* gt_center,
                                 const int64_t* gt_label, float w_cls, float w_obj, float w_center,
                                 float w_giou, float* cost, void* stream) {
    if (P <= 0 || B <= 0 || P % B || Q <= 0 || G <= 0 || C <= 0 || ldp < C || !prob || !obj ||
        !center || !gious || !gt_center || !gt_label || !cost)
        return OV3D_EINVAL;
    const long long total = (long long)P * Q * G;
    matcher_cost_kernel<<<ov3d_cdiv(total, 256), 256, 0, ov3d_stream(stream)>>>(
        total, B, Q, G, C, P / B, final_last, prob, ldp, obj, center, gious, gt_center, gt_label,
        w_cls, w_obj,
        w_center, w_giou, cost);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_targets_prep(int B, int G, int L, const float* present, const float* angles,
                                 int64_t* nact64, int32_t* nact32_rep, int64_t* total,
                                 float* num_boxes, int32_t* rotated, void* stream) {
    if (B <= 0 || G <= 0 || L <= 0 || !present || !angles || !nact64 || !nact32_rep || !total ||
        !rotated)
        return OV3D_EINVAL;
    targets_prep_kernel<<<1, 256, 0, ov3d_stream(stream)>>>(B, G, L, present, angles, nact64,
                                                            nact32_rep, total, num_boxes, rotated);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
