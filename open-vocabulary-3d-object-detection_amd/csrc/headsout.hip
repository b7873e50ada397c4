// Output layers of the five 3DETR prediction heads plus the query <-> text alignment, in one
// launch each way.
//
// Reference: models/model_3detr.py:_build_heads / get_box_predictions -- each head's last
// Conv1d(256, n_out) (visual_embed_head n_out = 640, center 3, size 3, angle_cls / angle_residual
// num_angle_bin) on the decoder-feature rows, then sem_cls_head = Linear(640, T, bias=False)
// holding the frozen text embedding (model_3detr.py:152-154, 237-238) on the visual embedding.
// heads.py feeds the rows z2 (R, 5*256) bf16: columns [0, 256) are the visual head's hidden
// features, [256 (1+i), 256 (2+i)) those of box head i.
//
// Forward (heads_out_fwd_kernel): six workgroups of 4 waves per 32 rows (see "Column groups"
// below).  Each 32-channel output tile is one MFMA 32x32x16 chain over K = 256 (A = weight rows,
// B = the 32 rows, so a lane owns a row and 16 of the tile's channels): the visual head's 20
// tiles (one per wave of five workgroups) and one tile per box head (n_out <= 32, rows past
// n_out read as zero).  The visual tiles' epilogue writes the fp32 embedding and, with the
// group's 128 text columns staged in LDS, the fp32 partial logits of the lane's row over its
// channels (the alignment GEMM never re-reads the embedding from HBM); a second launch adds
// the groups' partials.  Logits are written in the caller's layout: row-major (R, T), or with
// Q > 0 the reference's transposed layout (quirk Q8: element (lb, q, t) of the (L*B, Q, T)
// result at lb*Q*T + t*Q + q).
//
// Backward (heads_out_bwd_kernel): per 32 rows, five workgroups for the visual embedding's gradient
// plus the alignment's contribution, g_v + g_logits . text, rounded once to bf16 (the operand
// of the dgrad GEMM and the deferred weight gradient) and one for the box heads' output
// gradients in bf16 and the box heads' input gradient dz2[:, 256 (1+i) + c] = sum_j g_i[j] W_i[j, c]
// (n_out <= 32 terms, fp32) into its columns of the caller's dz2.
#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int RB = 32;          // rows per workgroup
constexpr int KH = 256;         // hidden width of every head
constexpr int MAXT = 32;        // text rows (classes) the fused alignment supports
constexpr int MAXS = 4;         // box heads
constexpr int NV = 640;         // visual embedding width (clip_embed_length)

struct HeadsOutArgs {
    const bf16* z;              // (R, ldz) bf16
    long long ldz;
    int R;
    const bf16* wv;             // (Nv, 256) bf16 visual output weight
    const float* bv;            // (Nv) fp32
    int Nv;
    const float* text;          // (T, Nv) fp32, or null (no alignment)
    int T;
    int lq;                     // logits layout: 0 row-major, else the Q of quirk Q8
    float* out_v;               // (R, Nv) fp32
    float* logits;              // (R, T) fp32
    int ns;                     // box heads
    const bf16* ws[MAXS];       // (n_i, 256) bf16
    const float* bs[MAXS];      // (n_i) fp32
    int n[MAXS];
    int kcol[MAXS];             // input column of head i (256 (1+i))
    int ocol[MAXS];             // output column of head i in out_s
    float* out_s;               // (R, Ns) fp32
    int Ns;
};

// element i (0..3, wave-uniform) of a kernel-argument array without a dynamic index (which
// would copy the argument struct into scratch)
template <class T>
__device__ __forceinline__ T pick4(const T (&v)[MAXS], int i) {
    return i == 0 ? v[0] : i == 1 ? v[1] : i == 2 ? v[2] : v[3];
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// one 32-channel tile of rows z (this lane: row r, operand k-half h): acc[e] = channel
// 8 (e / 4) + 4 h + e % 4 of the tile
__device__ __forceinline__ f32x16 tile_gemm(const bf16* __restrict__ w, int nrows, const bf16x8* zf,
                                            int r, int h) {
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    const bool live = r < nrows;
    const bf16* wr = w + (size_t)(live ? r : 0) * KH + 8 * h;
    bf16x8 wf[KH / 16];
#pragma unroll
    for (int s = 0; s < KH / 16; ++s) {
        wf[s] = *reinterpret_cast<const bf16x8*>(wr + 16 * s);
        if (!live) {
#pragma unroll
            for (int j = 0; j < 8; ++j) wf[s][j] = (bf16)0.f;
        }
    }
#pragma unroll
    for (int s = 0; s < KH / 16; ++s) acc = mfma(wf[s], zf[s], acc);
    return acc;
}

// Column groups of the forward (round 3): the visual head's 20 output tiles split over NGV = 5
// workgroups per 32-row block (one tile per wave), the four box heads in a sixth (one head per
// wave), so a 32-row block is 6 workgroups of single-tile waves instead of one workgroup walking
// 5 + 1 tiles per wave with the whole text embedding staged (74 us for 8192 rows, latency-bound).
// Each visual workgroup stages the block's z rows once in LDS and its 128 text columns, and
// writes the alignment's partial logits over those 128 channels; ov3d_heads_logits_sum adds the
// NGV partials in group order.
constexpr int NGV = NV / 128;   // visual column groups
constexpr int ZLD = KH + 8;     // padded LDS row of the staged z block (bf16)

// TMAX: the text rows rounded up (8, 16, 24 or 32); rows T..TMAX-1 of the LDS image are zero,
// so the logit loops are branch-free and their LDS reads batch
template <int TMAX>
__global__ void __launch_bounds__(256) heads_out_fwd_kernel(HeadsOutArgs a, float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) bf16 zS[RB * ZLD];       // the block's z rows
    __shared__ __attribute__((aligned(16))) float textS[TMAX * 128];  // (TMAX, 128 channels)
    __shared__ float red[4][RB][TMAX + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int row0 = blockIdx.x * RB;
    const int row = row0 + r;
    const int grp = blockIdx.y;
    const bool visual = grp < NGV;
    if (!visual && wave >= a.ns) return;
    const bool align = visual && a.text != nullptr;
    const int zcol = visual ? 0 : pick4(a.kcol, wave);
    bf16x8 zf[KH / 16];
    if (visual) {
        // z rows [row0, row0 + 32), columns [0, 256): 1024 16-byte chunks, 4 per thread
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int ch = tid + 256 * u, rr = ch >> 5, kc = (ch & 31) * 8;
            const int rowc = min(row0 + rr, a.R - 1);
            *reinterpret_cast<bf16x8*>(&zS[rr * ZLD + kc]) =
                *reinterpret_cast<const bf16x8*>(a.z + (size_t)rowc * a.ldz + kc);
        }
        if (align)
            for (int i = tid; i < TMAX * 32; i += 256) {   // (TMAX, 128) float4 chunks
                const int t = i >> 5, c4 = i & 31;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (t < a.T) v = *reinterpret_cast<const float4*>(a.text + (size_t)t * a.Nv + grp * 128 + 4 * c4);
                reinterpret_cast<float4*>(textS)[i] = v;
            }
        __syncthreads();
#pragma unroll
        for (int s2 = 0; s2 < KH / 16; ++s2) zf[s2] = *reinterpret_cast<const bf16x8*>(&zS[r * ZLD + 16 * s2 + 8 * h]);
    } else {
        const int rowc = min(row, a.R - 1);
        const bf16* zr = a.z + (size_t)rowc * a.ldz + zcol + 8 * h;
#pragma unroll
        for (int s2 = 0; s2 < KH / 16; ++s2) zf[s2] = *reinterpret_cast<const bf16x8*>(zr + 16 * s2);
    }
    if (visual) {
        const int ct = grp * 4 + wave;   // output tile: channels [32 ct, 32 ct + 32)
        const f32x16 acc = tile_gemm(a.wv + (size_t)ct * 32 * KH, 32, zf, r, h);
        float v[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int ch = 32 * ct + 8 * g + 4 * h;
            const float4 b4 = *reinterpret_cast<const float4*>(a.bv + ch);
            v[4 * g] = acc[4 * g] + b4.x;
            v[4 * g + 1] = acc[4 * g + 1] + b4.y;
            v[4 * g + 2] = acc[4 * g + 2] + b4.z;
            v[4 * g + 3] = acc[4 * g + 3] + b4.w;
            // (staging the group's 32 x 128 outputs in LDS for whole-row stores measured slower:
            // 36.5 -> 39.2 us, the extra 17 KB of LDS costs occupancy)
            if (row < a.R)
                *reinterpret_cast<float4*>(a.out_v + (size_t)row * a.Nv + ch) =
                    make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
        }
        if (align) {
#pragma unroll
            for (int t = 0; t < TMAX; ++t) {
                float lg = 0.f;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int cl = 32 * wave + 8 * g + 4 * h;   // channel within the group
                    const float4 tx = *reinterpret_cast<const float4*>(textS + t * 128 + cl);
                    lg = fmaf(v[4 * g], tx.x, fmaf(v[4 * g + 1], tx.y,
                         fmaf(v[4 * g + 2], tx.z, fmaf(v[4 * g + 3], tx.w, lg))));
                }
                lg += __shfl_xor(lg, 32);
                if (h == 0) red[wave][r][t] = lg;
            }
            __syncthreads();
            // the group's partial logits (R, T) at part[grp], rows of this block
            for (int i = tid; i < RB * a.T; i += 256) {
                const int rr = i / a.T, t = i - rr * a.T;
                if (row0 + rr >= a.R) continue;
                part[((size_t)grp * a.R + row0 + rr) * a.T + t] =
                    (red[0][rr][t] + red[1][rr][t]) + (red[2][rr][t] + red[3][rr][t]);
            }
        }
        return;
    }
    // box head `wave`: one tile
    const int n = pick4(a.n, wave);
    const f32x16 acc = tile_gemm(pick4(a.ws, wave), n, zf, r, h);
    if (row < a.R) {
        float* o = a.out_s + (size_t)row * a.Ns + pick4(a.ocol, wave);
        const float* bsw = pick4(a.bs, wave);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int c = 8 * (e >> 2) + 4 * h + (e & 3);
            if (c < n) o[c] = acc[e] + bsw[c];
        }
    }
}

// logits = the NGV groups' partials added in group order, written in the caller's layout
__global__ void __launch_bounds__(256) heads_logits_sum_kernel(const float* __restrict__ part, int R,
                                                              int T, int lq, float* __restrict__ logits) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long long)R * T) return;
    const int row = (int)(i / T), t = (int)(i - (long long)row * T);
    float s = part[i];
#pragma unroll
    for (int g = 1; g < NGV; ++g) s += part[(size_t)g * R * T + i];
    long long at = i;
    if (lq > 0) {
        const int lb = row / lq, q = row - lb * lq;
        at = ((long long)lb * T + t) * lq + q;
    }
    logits[at] = s;
}

struct HeadsOutBwdArgs {
    const float* gv;            // (R, Nv) fp32 gradient of the visual embedding
    const float* glog;          // logits gradient (layout of the forward) or null
    const float* text;          // (T, Nv)
    int R, Nv, T, lq;
    const float* gs;            // (R, Ns) fp32 gradient of the box heads' outputs
    int Ns, ns;
    const bf16* ws[MAXS];
    int n[MAXS];
    int kcol[MAXS];
    int ocol[MAXS];
    bf16* gvb;                  // (R, Nv) bf16
    bf16* gsb;                  // (R, Ns) bf16
    bf16* dz;                   // (R, lddz) bf16: box head i's input gradient at column kcol[i]
    long long lddz;
};

// Column groups as in the forward: NGV workgroups per 32-row block for the visual gradient
// (thread: 4 of the group's 128 columns x 4 rows, its text columns in registers, the rows'
// logit gradients from LDS, broadcast), one per box head (its output gradient in bf16 and its
// input gradient, weights from LDS).
template <int TMAX>
__global__ void __launch_bounds__(256) heads_out_bwd_kernel(HeadsOutBwdArgs a) {
    __shared__ float gl[RB * TMAX];                  // (32 rows, TMAX), zero past T
    __shared__ float gsS[RB * 32];                   // the head's bf16-rounded output gradients
    __shared__ __attribute__((aligned(16))) bf16 wS[32 * KH];   // the head's weights (n, 256)
    const int tid = threadIdx.x;
    const int row0 = blockIdx.x * RB;
    const int nrows = min(RB, a.R - row0);
    const int grp = blockIdx.y;
    if (grp < NGV) {
        const bool align = a.glog != nullptr;
        const int c4 = tid & 31, rq = tid >> 5;
        const int col = grp * 128 + 4 * c4;
        float4 tx[TMAX];
#pragma unroll
        for (int t = 0; t < TMAX; ++t) {
            const int tc = t < a.T ? t : 0;
            const float4 x = align ? *reinterpret_cast<const float4*>(a.text + (size_t)tc * NV + col)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
            const float z = t < a.T ? 1.f : 0.f;
            tx[t] = make_float4(x.x * z, x.y * z, x.z * z, x.w * z);
        }
        for (int i = tid; i < RB * TMAX; i += 256) {
            const int rr = i / TMAX, t = i - rr * TMAX;
            const int row = row0 + rr;
            float g = 0.f;
            if (align && rr < nrows && t < a.T) {
                long long at;
                if (a.lq <= 0) {
                    at = (long long)row * a.T + t;
                } else {
                    const int lb = row / a.lq, q = row - lb * a.lq;
                    at = ((long long)lb * a.T + t) * a.lq + q;
                }
                g = a.glog[at];
            }
            gl[i] = g;
        }
        float4 gvr[4];   // (gv null: the embedding itself has no consumer, only the logits)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int rr = min(rq * 4 + k, nrows - 1);
            gvr[k] = a.gv ? *reinterpret_cast<const float4*>(a.gv + (size_t)(row0 + rr) * NV + col)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int rr = rq * 4 + k;
            if (rr >= nrows) break;
            float4 g = gvr[k];
#pragma unroll
            for (int t4 = 0; t4 < TMAX / 4; ++t4) {
                const float4 w = *reinterpret_cast<const float4*>(gl + rr * TMAX + 4 * t4);
                const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float4 x = tx[4 * t4 + u];
                    g.x = fmaf(wv[u], x.x, g.x);
                    g.y = fmaf(wv[u], x.y, g.y);
                    g.z = fmaf(wv[u], x.z, g.z);
                    g.w = fmaf(wv[u], x.w, g.w);
                }
            }
            bf16x4 o;
            o[0] = (bf16)g.x;
            o[1] = (bf16)g.y;
            o[2] = (bf16)g.z;
            o[3] = (bf16)g.w;
            *reinterpret_cast<bf16x4*>(a.gvb + (size_t)(row0 + rr) * NV + col) = o;
        }
        return;
    }
    // box head hi = grp - NGV (one workgroup per head): its output gradient in bf16 and its
    // input gradient dz[:, kcol + c] = sum_j bf16(g[j]) W[j, c]
    const int hi = grp - NGV;
    if (hi >= a.ns) return;
    const int n = pick4(a.n, hi), oc = pick4(a.ocol, hi);
    {
        const int n8 = n * KH / 8;
        const float4* src = reinterpret_cast<const float4*>(pick4(a.ws, hi));
        for (int i = tid; i < n8; i += 256) reinterpret_cast<float4*>(wS)[i] = src[i];
    }
    for (int i = tid; i < nrows * n; i += 256) {
        const int rr = i / n, j = i - rr * n;
        const bf16 v = (bf16)a.gs[(size_t)(row0 + rr) * a.Ns + oc + j];
        a.gsb[(size_t)(row0 + rr) * a.Ns + oc + j] = v;
        gsS[rr * 32 + j] = (float)v;
    }
    __syncthreads();
    for (int i = tid; i < nrows * (KH / 4); i += 256) {
        const int cc = i % (KH / 4), rr = i / (KH / 4);
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        const bf16* w = wS + 4 * cc;
        const float* gr = gsS + rr * 32;
        int j = 0;
        for (; j + 4 <= n; j += 4) {
            bf16x4 wv[4];
            float gj[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                wv[u] = *reinterpret_cast<const bf16x4*>(w + (size_t)(j + u) * KH);
                gj[u] = gr[j + u];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[q] = fmaf(gj[u], (float)wv[u][q], acc[q]);
        }
        for (; j < n; ++j) {
            const bf16x4 wv = *reinterpret_cast<const bf16x4*>(w + (size_t)j * KH);
            const float gj = gr[j];
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] = fmaf(gj, (float)wv[q], acc[q]);
        }
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (bf16)acc[q];
        *reinterpret_cast<bf16x4*>(a.dz + (size_t)(row0 + rr) * a.lddz + pick4(a.kcol, hi) + 4 * cc) = o;
    }
}

int tmax_of(int T) { return T <= 8 ? 8 : T <= 16 ? 16 : T <= 24 ? 24 : 32; }

bool common_ok(int R, int Nv, int T, int ns, const int* n) {
    if (R <= 0 || Nv != NV || T < 0 || T > MAXT || ns < 0 || ns > MAXS) return false;
    for (int i = 0; i < ns; ++i)
        if (n[i] <= 0 || n[i] > 32) return false;
    return true;
}

}  // namespace

extern "C" int ov3d_heads_out_max_text(void) { return MAXT; }

extern "C" int ov3d_heads_out_fwd(const void* z, long long ldz, int R, const void* wv, const float* bv,
                                  int Nv, const float* text, int T, int lq, float* out_v,
                                  float* logits, int ns, const void* const* ws,
                                  const float* const* bs, const int* n, const int* kcol,
                                  const int* ocol, float* out_s, int Ns, float* work, void* stream) {
    if (!z || !wv || !bv || !out_v || !common_ok(R, Nv, text ? T : 0, ns, n) ||
        (text && (!logits || T <= 0 || !work)) || (ns > 0 && (!ws || !bs || !kcol || !ocol || !out_s)))
        return OV3D_EINVAL;
    HeadsOutArgs a = {};
    a.z = static_cast<const bf16*>(z);
    a.ldz = ldz;
    a.R = R;
    a.wv = static_cast<const bf16*>(wv);
    a.bv = bv;
    a.Nv = Nv;
    a.text = text;
    a.T = text ? T : 0;
    a.lq = lq;
    a.out_v = out_v;
    a.logits = logits;
    a.ns = ns;
    for (int i = 0; i < ns; ++i) {
        if (!ws[i] || !bs[i] || kcol[i] < 0 || kcol[i] + KH > ldz || ocol[i] < 0 || ocol[i] + n[i] > Ns)
            return OV3D_EINVAL;
        a.ws[i] = static_cast<const bf16*>(ws[i]);
        a.bs[i] = bs[i];
        a.n[i] = n[i];
        a.kcol[i] = kcol[i];
        a.ocol[i] = ocol[i];
    }
    if (KH > ldz) return OV3D_EINVAL;
    a.out_s = out_s;
    a.Ns = Ns;
    const int tm = tmax_of(a.T);
    const dim3 grid((unsigned)((R + RB - 1) / RB), NGV + 1);
    hipStream_t st = ov3d_stream(stream);
    switch (tm) {
        case 8: hipLaunchKernelGGL(heads_out_fwd_kernel<8>, grid, dim3(256), 0, st, a, work); break;
        case 16: hipLaunchKernelGGL(heads_out_fwd_kernel<16>, grid, dim3(256), 0, st, a, work); break;
        case 24: hipLaunchKernelGGL(heads_out_fwd_kernel<24>, grid, dim3(256), 0, st, a, work); break;
        default: hipLaunchKernelGGL(heads_out_fwd_kernel<32>, grid, dim3(256), 0, st, a, work); break;
    }
    OV3D_LAUNCH_CHECK();
    if (a.T) {
        hipLaunchKernelGGL(heads_logits_sum_kernel, dim3(ov3d_cdiv((long long)R * a.T, 256)), dim3(256), 0,
                           st, work, R, a.T, a.lq, logits);
        OV3D_LAUNCH_CHECK();
    }
    return OV3D_OK;
}

/* floats of the forward's workspace (the column groups' partial logits) */
extern "C" long long ov3d_heads_out_workspace(int R, int T) {
    return R > 0 && T > 0 ? (long long)NGV * R * T : 0;
}

extern "C" int ov3d_heads_out_bwd(const float* gv, const float* glog, const float* text, int R, int Nv,
                                  int T, int lq, const float* gs, int Ns, int ns,
                                  const void* const* ws, const int* n, const int* kcol,
                                  const int* ocol, void* gvb, void* gsb, void* dz, long long lddz,
                                  void* stream) {
    if (!gvb || !common_ok(R, Nv, glog ? T : 0, ns, n) || (glog && (!text || T <= 0)) ||
        (ns > 0 && (!gs || !gsb || !dz || !ws || !kcol || !ocol)) || Ns > MAXS * 32)
        return OV3D_EINVAL;
    HeadsOutBwdArgs a = {};
    a.gv = gv;
    a.glog = glog;
    a.text = text;
    a.R = R;
    a.Nv = Nv;
    a.T = glog ? T : 0;
    a.lq = lq;
    a.gs = gs;
    a.Ns = ns > 0 ? Ns : 0;
    a.ns = ns;
    for (int i = 0; i < ns; ++i) {
        if (!ws[i] || kcol[i] < 0 || kcol[i] + KH > lddz || ocol[i] < 0 || ocol[i] + n[i] > Ns)
            return OV3D_EINVAL;
        a.ws[i] = static_cast<const bf16*>(ws[i]);
        a.n[i] = n[i];
        a.kcol[i] = kcol[i];
        a.ocol[i] = ocol[i];
    }
    a.gvb = static_cast<bf16*>(gvb);
    a.gsb = static_cast<bf16*>(gsb);
    a.dz = static_cast<bf16*>(dz);
    a.lddz = lddz;
    const int tm = tmax_of(a.T);
    const dim3 grid((unsigned)((R + RB - 1) / RB), NGV + ns);
    hipStream_t st = ov3d_stream(stream);
    switch (tm) {
        case 8: hipLaunchKernelGGL(heads_out_bwd_kernel<8>, grid, dim3(256), 0, st, a); break;
        case 16: hipLaunchKernelGGL(heads_out_bwd_kernel<16>, grid, dim3(256), 0, st, a); break;
        case 24: hipLaunchKernelGGL(heads_out_bwd_kernel<24>, grid, dim3(256), 0, st, a); break;
        default: hipLaunchKernelGGL(heads_out_bwd_kernel<32>, grid, dim3(256), 0, st, a); break;
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
