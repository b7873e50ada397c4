// LayerNorm boundary + the adjacent row GEMM in ONE launch each way, for the decoder's short
// row blocks (models/transformer.py TransformerDecoderLayer.forward_pre 355-379: every
// sub-layer ends with `tgt = tgt + dropout(branch)`, the next starts with `norm(tgt)` and
// feeds it straight into a linear layer — the self-attention in-projection, the cross
// attention's query projection, the FFN's linear1).
//
// Forward (ov3d_lngemm_fwd): the resnorm_fwd row pass (csrc/resnorm.hip) as the PROLOGUE of
// the next GEMM:
//     s   = src + dropout(y);  xa = bf16(LN(s) * ga + ba);  xap = bf16(xa_f32 + pos);  xb
//     out_i = epi(xsel_i W_i^T + b_i)        (xsel = xa or xap per problem; epi: none or
//                                             dropout(relu(.)) with the rowdrop.h hash)
// Backward (ov3d_lngemm_bwd): the resnorm_bwd row pass as the PROLOGUE of the input gradient
// of the branch's last linear (the output projection / FFN linear2, y = x W^T + b):
//     g = ds + rstd * (dxh - mean(dxh) - xh * mean(dxh xh));   dy = dropout(g)
//     dx = epi(dy W)                          (epi: none or the FFN activation mask)
// Both are the resnorm launch and the rows-GEMM launch (csrc/rowsgemm.hip) of the unfused
// path with the row pass recomputed per column tile: one ~2.5 us launch boundary less per
// sub-layer boundary and direction (3 + 3 per decoder layer).  The arithmetic is the unfused
// kernels' in the same order (row sums over the same 32-lane shuffles, the GEMM's K in four
// 64-deep quarters summed (q0 + q1) + (q2 + q3) as rowsgemm's four waves), so the outputs
// equal the two-launch path's.
//
// Layout: a workgroup = 16 rows x BN output columns (BN = 64, or 128 for the 768-wide
// in-projection), 8 waves.  The row pass runs on all 512 threads (32 lanes a row, 8 channels a
// lane, one row a thread: the pass is VALU latency, so it is spread as thin as the rows allow)
// and leaves the GEMM's A operand as a bf16 image of the 16 rows in LDS; W's BN rows are loaded
// whole (coalesced) into LDS.  The waves split the output columns in 32-wide slices and K in
// quarters (BN = 64) or halves (BN = 128) exactly as rowsgemm's waves split K; the quarter sums
// meet in LDS in rowsgemm's order.  The 32x32x16 MFMA's 32 row lanes carry the 16 rows twice
// (half of its work is discarded: the launch is latency-bound, not MFMA-bound).  The column
// tile t == 0 workgroups also store the row pass's outputs (s, mean, rstd, xa, xap, xb /
// dsrc, dy, dpos and the LayerNorm column partials in resnorm_bwd's per-8-row layout).
#include "common.h"
#include "rowdrop.h"
#include "rowsum.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int C = 256;            // model width: the LayerNorm rows and the GEMMs' K / N
constexpr int RB = 16;            // rows per workgroup
constexpr int NT = 512;           // threads (8 waves)
constexpr int LDX = C + 8;        // LDS row of the row / W images (bf16): 528 bytes
constexpr int MAXP = 2;
constexpr int BNB = 64;           // backward: output columns per workgroup
// backward LDS strides (round 6; every read conflict-free under the MI355X lane groups, the
// padded forward strides left 3.9 conflict cycles per LDS instruction, tools/lds_banks_dy9.py):
constexpr int LDXB = C + 4;       // dy rows: 130 dwords (16 rows of a read on distinct bank pairs)
constexpr int LDWB = 32;          // W slice rows unpadded: 4 rows of a transposed read on 4 16-bank windows
constexpr int LDRB = RB + 4;      // partial products [column][row]: 20 dwords
constexpr int CRB = C + 32;       // LayerNorm column terms: 4 pad dwords per 32 columns
__device__ __forceinline__ int redix(int row, int col) { return row * CRB + col + 4 * (col >> 5); }
enum { EPI_NONE = 0, EPI_RELU_DROP = 1, EPI_MASK = 2 };

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x4 tr16(const bf16* p) {
    s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
    return __builtin_bit_cast(bf16x4, r);
}
__device__ __forceinline__ void st8f(float* p, long long off, const float* v) {
    *reinterpret_cast<float4*>(p + off) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + off + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ bf16x8 pack8(const float* v) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
    return o;
}
// raw 8-channel row pieces: loaded early (every load of a row pass in flight at once),
// converted at their use
struct Raw8 {
    uint4 a, b;
};
// Loads are never predicated: a load under a branch makes the wait-count pass drain every
// load in flight at the join, i.e. one memory round trip per optional operand and row.  An
// absent operand reads this zero block instead (at the lane's channel offset) and its value
// is discarded by a select.
__device__ __attribute__((aligned(16))) unsigned char g_zero[4096];
template <typename T>
__device__ __forceinline__ const T* orz(const T* p) {
    return p ? p : reinterpret_cast<const T*>(g_zero);
}
__device__ __forceinline__ Raw8 ldraw(const void* p, int is_bf16, long long off) {
    const char* b = (const char*)p + off * (is_bf16 ? 2 : 4);
    Raw8 r;
    r.a = *reinterpret_cast<const uint4*>(b);
    r.b = *reinterpret_cast<const uint4*>(b + (is_bf16 ? 0 : 16));
    return r;
}
__device__ __forceinline__ void cvt8(const Raw8& r, int is_bf16, float* v) {
    if (is_bf16) {
        const bf16x8 x = __builtin_bit_cast(bf16x8, r.a);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
    } else {
        const float4 a = __builtin_bit_cast(float4, r.a), b = __builtin_bit_cast(float4, r.b);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
}
__device__ __forceinline__ float row_sum32(float v) { return row_sum32_lanes(v); }

// ---------------------------------------------------------------- forward
struct LnProb {
    const bf16* W; long long ldw;   // (N, C) rows (nn.Linear weight rows)
    const bf16* bias;
    bf16* out; long long ldo;
    int N; int sel;                 // sel 0: xa, 1: xap
};
struct LnFwdArgs {
    int R;
    const void* src; int src_bf16;
    const bf16* y;
    const void* pos; int pos_bf16;
    uint32_t thresh; float keep_scale; const int64_t* seed; uint32_t site;
    const float *ga, *ba, *gb, *bb;
    float eps;
    float* s; float* mean; float* rstd;
    bf16* xa; bf16* xap; void* xb; int xb_bf16;
    long long xb_inner, xb_s0, xb_s1;
    LnProb p[MAXP];
    int tiles[MAXP + 1];
    int np;
    int epi; uint32_t thresh2; float keep_scale2; const int64_t* seed2; uint32_t site2;
    unsigned long long* stamp;   // measurement only (tools/lngemm_probe.py): phase clocks
};

template <int EPI, int BN, int RBT>
__global__ void __launch_bounds__(NT) lngemm_fwd_kernel(LnFwdArgs a) {
    constexpr int NR = RBT / 16;   // rows a thread in the row pass
    constexpr int LDQ = RBT + 1;   // fp32 partial-product rows
    constexpr int NCS = BN / 32;   // 32-column slices
    constexpr int NKG = 8 / NCS;   // K groups: 4 quarters (BN 64) or 2 halves (BN 128)
    constexpr int WL = BN / 16;    // W row-pair loads per wave
    __shared__ __attribute__((aligned(16))) bf16 img[2][RBT * LDX];  // xa / xap rows
    __shared__ __attribute__((aligned(16))) bf16 wimg[BN * LDX];     // W rows nb .. nb+BN-1
    __shared__ float red[NKG][BN * LDQ];                              // per K group products
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
    unsigned long long* const stp = a.stamp
        ? a.stamp + 8 * ((blockIdx.y * gridDim.x + blockIdx.x) * 8 + w) : nullptr;
    if (stp && lane == 0) stp[0] = __builtin_amdgcn_s_memtime();
    const int m0 = blockIdx.x * RBT;
    const int t = blockIdx.y;
    const int pi = (a.np > 1 && t >= a.tiles[1]) ? 1 : 0;
    const bf16* const W = pi ? a.p[1].W : a.p[0].W;
    const long long ldw = pi ? a.p[1].ldw : a.p[0].ldw;
    const bf16* const bias = pi ? a.p[1].bias : a.p[0].bias;
    bf16* const out = pi ? a.p[1].out : a.p[0].out;
    const long long ldo = pi ? a.p[1].ldo : a.p[0].ldo;
    const int sel = pi ? a.p[1].sel : a.p[0].sel;
    const int nb = (t - a.tiles[pi]) * BN;
    const bool writer = t == 0;

    // W rows (two whole 512-byte rows a load) in flight first
    bf16x8 wr[WL];
#pragma unroll
    for (int i = 0; i < WL; ++i)
        wr[i] = *reinterpret_cast<const bf16x8*>(
            W + (size_t)(nb + w * (BN / 8) + 2 * i + (lane >> 5)) * ldw + 8 * (lane & 31));
    // the epilogue's 4 columns (columns nb + 4 cg .., rows em + k * NT / (BN / 4))
    const int cg = tid % (BN / 4);
    const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(bias ? bias + nb + 4 * cg : orz(bias));

    // ---- the resnorm_fwd row pass: NR rows a thread (rows tid / 32 + 16 it), 32 lanes a row
    const int c = (tid & 31) * 8, lr0 = tid >> 5;
    float ga[8], ba[8], gb[8], bb[8];
    {
        const float* gbp = orz(a.gb);
        const float* bbp = orz(a.bb);
        const float4 g0 = *reinterpret_cast<const float4*>(a.ga + c), g1 = *reinterpret_cast<const float4*>(a.ga + c + 4);
        const float4 b0 = *reinterpret_cast<const float4*>(a.ba + c), b1 = *reinterpret_cast<const float4*>(a.ba + c + 4);
        const float4 g2 = *reinterpret_cast<const float4*>(gbp + c), g3 = *reinterpret_cast<const float4*>(gbp + c + 4);
        const float4 b2 = *reinterpret_cast<const float4*>(bbp + c), b3 = *reinterpret_cast<const float4*>(bbp + c + 4);
        ga[0] = g0.x; ga[1] = g0.y; ga[2] = g0.z; ga[3] = g0.w; ga[4] = g1.x; ga[5] = g1.y; ga[6] = g1.z; ga[7] = g1.w;
        ba[0] = b0.x; ba[1] = b0.y; ba[2] = b0.z; ba[3] = b0.w; ba[4] = b1.x; ba[5] = b1.y; ba[6] = b1.z; ba[7] = b1.w;
        gb[0] = g2.x; gb[1] = g2.y; gb[2] = g2.z; gb[3] = g2.w; gb[4] = g3.x; gb[5] = g3.y; gb[6] = g3.z; gb[7] = g3.w;
        bb[0] = b2.x; bb[1] = b2.y; bb[2] = b2.z; bb[3] = b2.w; bb[4] = b3.x; bb[5] = b3.y; bb[6] = b3.z; bb[7] = b3.w;
    }
    const uint32_t smix = rowdrop::seed_mix(a.seed ? a.seed : reinterpret_cast<const int64_t*>(g_zero), a.site);
    Raw8 rsr[NR], rpr[NR];
    uint4 ryr[NR];
#pragma unroll
    for (int it = 0; it < NR; ++it) {
        const long long off = (long long)(m0 + lr0 + 16 * it) * C + c;
        rsr[it] = ldraw(orz(a.src), a.src_bf16, a.src ? off : c);
        ryr[it] = *reinterpret_cast<const uint4*>(orz(a.y) + (a.y ? off : c));
        rpr[it] = ldraw(orz(a.pos), a.pos_bf16, a.pos ? off : c);
    }
    // W into LDS (waits for the W loads only: they went out first)
#pragma unroll
    for (int i = 0; i < WL; ++i)
        *reinterpret_cast<bf16x8*>(&wimg[(w * (BN / 8) + 2 * i + (lane >> 5)) * LDX + 8 * (lane & 31)]) = wr[i];
    if (stp && lane == 0) stp[5] = __builtin_amdgcn_s_memtime();

    // the row arithmetic without branches (absent operands read zeros; selects keep the
    // two-launch path's operations: no add of an absent y)
    float sr[NR][8], xbr[NR][8], mur[NR], rsr_[NR];
#pragma unroll
    for (int it = 0; it < NR; ++it) {
        const int lr = lr0 + 16 * it;
        const long long row = m0 + lr;
        float s[8], pv[8], y[8];
        cvt8(rsr[it], a.src_bf16, s);
        cvt8(rpr[it], a.pos_bf16, pv);
        const bf16x8 yv = __builtin_bit_cast(bf16x8, ryr[it]);
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = (float)yv[j];
        bool keep[8];
        rowdrop::keep8(rowdrop::row_base(smix, row), c, a.thresh, keep);   // all kept at p = 0
        const bool has_y = a.y != nullptr;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float d = (float)(bf16)(y[j] * a.keep_scale);   // = y at p = 0
            const float sn = s[j] + (keep[j] ? d : 0.f);
            s[j] = has_y ? sn : s[j];
        }
        float tt = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) tt += s[j];
        const float mu = row_sum32(tt) / (float)C;
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) q += (s[j] - mu) * (s[j] - mu);
        const float rs = rsqrtf(row_sum32(q) / (float)C + a.eps);
        float xh[8], o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) xh[j] = (s[j] - mu) * rs;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = xh[j] * ga[j] + ba[j];
        *reinterpret_cast<bf16x8*>(&img[0][lr * LDX + c]) = pack8(o);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += pv[j];
        *reinterpret_cast<bf16x8*>(&img[1][lr * LDX + c]) = pack8(o);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            xbr[it][j] = xh[j] * gb[j] + bb[j];
            sr[it][j] = s[j];
        }
        mur[it] = mu;
        rsr_[it] = rs;
    }
    if (stp && lane == 0) stp[6] = __builtin_amdgcn_s_memtime();
    if (writer) {   // the row pass's own outputs (column tile 0 only)
#pragma unroll
        for (int it = 0; it < NR; ++it) {
            const long long row = m0 + lr0 + 16 * it;
            const long long off = row * C + c;
            st8f(a.s, off, sr[it]);
            if (c == 0) {
                a.mean[row] = mur[it];
                a.rstd[row] = rsr_[it];
            }
            if (a.xb) {
                const int ri = (int)row, xi = (int)a.xb_inner;
                const long long ob = xi ? (long long)(ri / xi) * a.xb_s0 + (long long)(ri % xi) * a.xb_s1 + c : off;
                if (a.xb_bf16) *reinterpret_cast<bf16x8*>((bf16*)a.xb + ob) = pack8(xbr[it]);
                else st8f((float*)a.xb, ob, xbr[it]);
            }
        }
    }
    if (stp && lane == 0) stp[7] = __builtin_amdgcn_s_memtime();
    if (stp && lane == 0) stp[1] = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (stp && lane == 0) stp[2] = __builtin_amdgcn_s_memtime();
    if (writer) {   // xa / xap rows from the images, 16 bytes a lane
#pragma unroll
        for (int it = 0; it < NR; ++it) {
            const int lr = lr0 + 16 * it;
            const long long off = (long long)(m0 + lr) * C + c;
            if (a.xa) *reinterpret_cast<bf16x8*>(a.xa + off) = *reinterpret_cast<const bf16x8*>(&img[0][lr * LDX + c]);
            if (a.xap) *reinterpret_cast<bf16x8*>(a.xap + off) = *reinterpret_cast<const bf16x8*>(&img[1][lr * LDX + c]);
        }
    }

    // ---- the product: wave = (column slice cs, K group kg); quarter chains in rowsgemm's
    // k order, a half's two quarters summed (q0 + q1) / (q2 + q3) here, the rest in LDS
    {
        const int cs = w % NCS, kg = w / NCS;
        const bf16* im = &img[sel][(r & (RBT - 1)) * LDX + 8 * h];
        const bf16* wm = &wimg[(32 * cs + r) * LDX + 8 * h];
        constexpr int NQ = 4 / NKG;   // quarters per wave
        f32x16 acc[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[q][v] = 0.f;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int ks = 4 * (kg * NQ + q) + s4;
                acc[q] = mfma(*reinterpret_cast<const bf16x8*>(wm + 16 * ks),
                              *reinterpret_cast<const bf16x8*>(im + 16 * ks), acc[q]);
            }
        if (r < RBT) {
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int n = 32 * cs + 8 * (v >> 2) + 4 * h + (v & 3);
                red[kg][n * LDQ + r] = NQ == 2 ? acc[0][v] + acc[NQ - 1][v] : acc[0][v];
            }
        }
    }
    if (stp && lane == 0) stp[3] = __builtin_amdgcn_s_memtime();
    __syncthreads();
#pragma unroll
    for (int e0 = tid; e0 < RBT * BN / 4; e0 += NT) {
        const int em = e0 / (BN / 4);
        const long long orow = m0 + em;
        const int col = nb + 4 * cg;
        bool keep[4] = {true, true, true, true};
        if (EPI == EPI_RELU_DROP) {
            const uint32_t rb2 = rowdrop::row_base(
                rowdrop::seed_mix(a.seed2 ? a.seed2 : reinterpret_cast<const int64_t*>(g_zero), a.site2), orow);
#pragma unroll
            for (int j = 0; j < 4; j += 2) {
                const uint32_t hs = rowdrop::mix24(rb2 + (uint32_t)((col + j) >> 1) * 0x27D4EB2Fu);
                keep[j] = (hs & 0xffffu) >= a.thresh2;
                keep[j + 1] = (hs >> 16) >= a.thresh2;
            }
        }
        const bool has_bias = bias != nullptr;
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int n = 4 * cg + e;
            const float t0 = NKG == 4
                ? (red[0][n * LDQ + em] + red[1 % NKG][n * LDQ + em]) +
                  (red[2 % NKG][n * LDQ + em] + red[3 % NKG][n * LDQ + em])
                : red[0][n * LDQ + em] + red[1 % NKG][n * LDQ + em];
            const float tt = has_bias ? t0 + (float)b4[e] : t0;
            const bf16 yv = (bf16)tt;
            if (EPI == EPI_RELU_DROP) {
                const float rr = fmaxf((float)yv, 0.f);
                // all kept at p = 0, and rr * 1 == rr: the unmasked relu of the two-launch path
                o[e] = keep[e] ? (bf16)(rr * a.keep_scale2) : (bf16)0.f;
            } else {
                o[e] = yv;
            }
        }
        *reinterpret_cast<bf16x4*>(out + orow * ldo + col) = o;
    }
    if (stp && lane == 0) stp[4] = __builtin_amdgcn_s_memtime();
}

// ---------------------------------------------------------------- backward
struct LnBwdArgs {
    int R;
    const float* s; const float* mean; const float* rstd;
    const float* ds;
    const bf16* dxa; const bf16* dxap; const void* dxb; int dxb_bf16;
    long long dxb_inner, dxb_s0, dxb_s1;
    const float *ga, *gb;
    uint32_t thresh; float keep_scale; const int64_t* seed; uint32_t site;
    float* dsrc; bf16* dy; void* dpos; int dpos_bf16;
    float* partials; int accumulate;
    const bf16* W; long long ldw;   // (C, N) rows: the branch linear's (out, in) weight
    bf16* dx; long long lddx;
    int N;
    int epi; float keep_scale2; const bf16* H; long long ldh;
};

template <int EPI>
__global__ void __launch_bounds__(NT) lngemm_bwd_kernel(LnBwdArgs a) {
    __shared__ __attribute__((aligned(16))) bf16 img[RB * LDXB];       // dy rows
    __shared__ __attribute__((aligned(16))) bf16 wsm[2][C * LDWB];     // W (k, 32 columns) x 2
    __shared__ __attribute__((aligned(16))) float red[4][RB * CRB];    // LayerNorm column terms
    __shared__ float pr[4][BNB * LDRB];                                // per K quarter products
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.x * RB;
    const bool writer = blockIdx.y == 0;
    const int nb = blockIdx.y * BNB;
    const int cs = w & 1, kq = w >> 1;   // the wave's 32-column slice and K quarter

    // the wave's W sub-tile (rows 64 kq .. +63, columns nb + 32 cs ..) in flight first:
    // 16 rows a load, 4 lanes a row
    bf16x8 wr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        wr[i] = *reinterpret_cast<const bf16x8*>(a.W + (size_t)(64 * kq + 16 * i + (lane >> 2)) * a.ldw +
                                                 nb + 32 * cs + 8 * (lane & 3));

    // ---- the resnorm_bwd row pass (csrc/resnorm.hip bwd_row): one row a thread
    const int c = (tid & 31) * 8, lr = tid >> 5;
    const long long row = m0 + lr;
    const long long off = row * C + c;
    const uint32_t sm = rowdrop::seed_mix(a.seed ? a.seed : reinterpret_cast<const int64_t*>(g_zero), a.site);
    float ga[8], gb[8];
    {
        const float* gap = orz(a.ga);
        const float* gbp = orz(a.dxb ? a.gb : nullptr);
        const float4 g0 = *reinterpret_cast<const float4*>(gap + c), g1 = *reinterpret_cast<const float4*>(gap + c + 4);
        const float4 g2 = *reinterpret_cast<const float4*>(gbp + c), g3 = *reinterpret_cast<const float4*>(gbp + c + 4);
        ga[0] = g0.x; ga[1] = g0.y; ga[2] = g0.z; ga[3] = g0.w; ga[4] = g1.x; ga[5] = g1.y; ga[6] = g1.z; ga[7] = g1.w;
        gb[0] = g2.x; gb[1] = g2.y; gb[2] = g2.z; gb[3] = g2.w; gb[4] = g3.x; gb[5] = g3.y; gb[6] = g3.z; gb[7] = g3.w;
    }
    const bool acc_pos = writer && a.dpos && a.dxap && (a.accumulate & 1);
    const Raw8 rds = ldraw(orz(a.ds), 0, a.ds ? off : c);
    const Raw8 rsv = ldraw(a.s, 0, off);
    const float mu = a.mean[row], rs = a.rstd[row];
    const uint4 rda = *reinterpret_cast<const uint4*>(orz(a.dxa) + (a.dxa ? off : c));
    const uint4 rdap = *reinterpret_cast<const uint4*>(orz(a.dxap) + (a.dxap ? off : c));
    const int ri = (int)row, xi = (int)a.dxb_inner;
    const long long ob = !a.dxb ? c : xi
        ? (long long)(ri / xi) * a.dxb_s0 + (long long)(ri % xi) * a.dxb_s1 + c : off;
    const Raw8 rdb = ldraw(orz(a.dxb), a.dxb_bf16, ob);
    const Raw8 rold = ldraw(acc_pos ? a.dpos : (const void*)g_zero, a.dpos_bf16, acc_pos ? off : c);
    // the epilogue's activation values (EPI_MASK), fetched with the rest
    // the epilogue's row / 4-column group: consecutive lanes take consecutive rows of a column
    // group (the partial-product reads conflict-free; the 8-byte stores hit 16 rows)
    const int em = tid % RB, cg = tid / RB;
    const bool eact = tid < RB * BNB / 4;
    bf16x4 hv;
    if (EPI == EPI_MASK)
        hv = *reinterpret_cast<const bf16x4*>(a.H + (long long)(m0 + (eact ? em : 0)) * a.ldh + nb + 4 * (eact ? cg : 0));
#pragma unroll
    for (int i = 0; i < 4; ++i)
        *reinterpret_cast<bf16x8*>(&wsm[cs][(64 * kq + 16 * i + (lane >> 2)) * LDWB + 8 * (lane & 3)]) = wr[i];

    float g[8], sv[8], da[8], db[8], tv[8];
    cvt8(rds, 0, g);                 // zeros without ds
    cvt8(rsv, 0, sv);
    {
        const bf16x8 x = __builtin_bit_cast(bf16x8, rda), xp = __builtin_bit_cast(bf16x8, rdap);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            tv[j] = (float)xp[j];
            da[j] = (float)x[j];
        }
    }
    const bool has_ap = a.dxap != nullptr;
#pragma unroll
    for (int j = 0; j < 8; ++j) da[j] = has_ap ? da[j] + tv[j] : da[j];
    cvt8(rdb, a.dxb_bf16, db);       // zeros without dxb
    float xh[8], dxh[8], s1 = 0.f, s2 = 0.f;
    float t0[8], t1[8], t2[8], t3[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        xh[j] = (sv[j] - mu) * rs;
        dxh[j] = da[j] * ga[j] + db[j] * gb[j];
        s1 += dxh[j];
        s2 += dxh[j] * xh[j];
        t0[j] = 0.f + da[j] * xh[j];
        t1[j] = 0.f + da[j];
        t2[j] = 0.f + db[j] * xh[j];
        t3[j] = 0.f + db[j];
    }
    {   // 16-byte stores (the padded offset is a multiple of 4 floats)
        const int ro = redix(lr, c);
        float4* const r0 = reinterpret_cast<float4*>(&red[0][ro]);
        float4* const r1 = reinterpret_cast<float4*>(&red[1][ro]);
        float4* const r2 = reinterpret_cast<float4*>(&red[2][ro]);
        float4* const r3 = reinterpret_cast<float4*>(&red[3][ro]);
        r0[0] = make_float4(t0[0], t0[1], t0[2], t0[3]); r0[1] = make_float4(t0[4], t0[5], t0[6], t0[7]);
        r1[0] = make_float4(t1[0], t1[1], t1[2], t1[3]); r1[1] = make_float4(t1[4], t1[5], t1[6], t1[7]);
        r2[0] = make_float4(t2[0], t2[1], t2[2], t2[3]); r2[1] = make_float4(t2[4], t2[5], t2[6], t2[7]);
        r3[0] = make_float4(t3[0], t3[1], t3[2], t3[3]); r3[1] = make_float4(t3[4], t3[5], t3[6], t3[7]);
    }
    s1 = row_sum32(s1) / (float)C;
    s2 = row_sum32(s2) / (float)C;
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] += rs * (dxh[j] - s1 - xh[j] * s2);
    bool keep[8];
    rowdrop::keep8(rowdrop::row_base(sm, row), c, a.thresh, keep);   // all kept at p = 0
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = keep[j] ? g[j] * a.keep_scale : 0.f;   // g * 1 at p = 0
    const bf16x8 dv = pack8(d);
    *reinterpret_cast<bf16x4*>(&img[lr * LDXB + c]) = bf16x4{dv[0], dv[1], dv[2], dv[3]};
    *reinterpret_cast<bf16x4*>(&img[lr * LDXB + c + 4]) = bf16x4{dv[4], dv[5], dv[6], dv[7]};
    if (writer) {
        if (a.dsrc) st8f(a.dsrc, off, g);
        *reinterpret_cast<bf16x8*>(a.dy + off) = dv;
        if (a.dpos && has_ap) {
            float u[8], old[8];
            cvt8(rold, a.dpos_bf16, old);
#pragma unroll
            for (int j = 0; j < 8; ++j) u[j] = acc_pos ? old[j] + tv[j] : tv[j];
            if (a.dpos_bf16) *reinterpret_cast<bf16x8*>((bf16*)a.dpos + off) = pack8(u);
            else st8f((float*)a.dpos, off, u);
        }
    }
    __syncthreads();
    if (writer) {
        // the two 8-row blocks' LayerNorm column partials, summed over their rows in order
        // (resnorm_bwd_kernel<32, 1>: one block = 8 rows)
#pragma unroll
        for (int i = 0; i < 2 * 4 * C / NT; ++i) {
            const int e = tid + NT * i, blk = e / (4 * C), rem = e - blk * 4 * C;
            const int k = rem / C, col = rem - k * C;
            float tt = 0.f;
#pragma unroll
            for (int p = 0; p < 8; ++p) tt += red[k][redix(8 * blk + p, col)];
            a.partials[(long long)(m0 / 8 + blk) * 4 * C + rem] = tt;
        }
    }

    // ---- dx = dy W: A = the dy image (rowsgemm's trans_b = 0 k order), W read transposed
    {
        const bf16* ar = &img[(r & 15) * LDXB];
        const bf16* ws = wsm[cs];
        const int gq = lane >> 4, i16 = lane & 15;
        const int d0 = 16 * (gq & 1) + 4 * (i16 & 3);
        f32x16 acc;
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[v] = 0.f;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const int ks = 4 * kq + s4;
            const bf16x4 lo = *reinterpret_cast<const bf16x4*>(ar + 16 * ks + 4 * h);
            const bf16x4 hi = *reinterpret_cast<const bf16x4*>(ar + 16 * ks + 8 + 4 * h);
            const bf16x8 av = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            const int k0 = 16 * ks + 4 * (gq >> 1) + (i16 >> 2);
            const bf16x4 wl = tr16(ws + k0 * LDWB + d0);
            const bf16x4 wh = tr16(ws + (k0 + 8) * LDWB + d0);
            const bf16x8 bv = bf16x8{wl[0], wl[1], wl[2], wl[3], wh[0], wh[1], wh[2], wh[3]};
            acc = mfma(bv, av, acc);
        }
        if (r < RB) {
#pragma unroll
            for (int v = 0; v < 16; ++v)
                pr[kq][(32 * cs + 8 * (v >> 2) + 4 * h + (v & 3)) * LDRB + r] = acc[v];
        }
    }
    __syncthreads();
    if (eact) {
        const long long orow = m0 + em;
        const int col = nb + 4 * cg;
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int n = 4 * cg + e;
            const float tt = (pr[0][n * LDRB + em] + pr[1][n * LDRB + em]) +
                             (pr[2][n * LDRB + em] + pr[3][n * LDRB + em]);
            const bf16 yv = (bf16)tt;
            if (EPI == EPI_MASK)
                o[e] = (float)hv[e] > 0.f ? (bf16)((float)yv * a.keep_scale2) : (bf16)0.f;
            else
                o[e] = yv;
        }
        *reinterpret_cast<bf16x4*>(a.dx + orow * a.lddx + col) = o;
    }
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

unsigned long long* g_stamp = nullptr;   // ov3d_lngemm_stamps_arm

}  // namespace

extern "C" int ov3d_lngemm_supported(int R, int C_, int N) {
    return R > 0 && R % RB == 0 && C_ == C && N > 0 && N % 128 == 0;
}

extern "C" int ov3d_lngemm_fwd(int R, const void* src, int src_bf16, const void* y, float dropout_p,
                               const int64_t* seed, int site, const float* ga, const float* ba,
                               const void* pos, int pos_bf16, const float* gb, const float* bb,
                               float eps, float* s, float* mean, float* rstd, void* xa, void* xap,
                               void* xb, int xb_bf16, long long xb_inner, long long xb_s0,
                               long long xb_s1, int nprob, const ov3d_lngemm_problem* probs,
                               int epilogue, float dropout_p2, const int64_t* seed2, int site2,
                               void* stream) {
    if (R <= 0 || R % RB || nprob < 1 || nprob > MAXP || !probs || !s || !mean || !rstd || !ga ||
        !ba || dropout_p < 0.f || dropout_p >= 1.f || (dropout_p > 0.f && (!seed || !y)) ||
        dropout_p2 < 0.f || dropout_p2 >= 1.f || (epilogue != EPI_NONE && epilogue != EPI_RELU_DROP) ||
        (epilogue == EPI_RELU_DROP && dropout_p2 > 0.f && !seed2))
        return OV3D_EINVAL;
    if (!al16(s) || (src && !al16(src)) || (y && !al16(y)) || (pos && !al16(pos)) ||
        (xa && !al16(xa)) || (xap && !al16(xap)) || ((uintptr_t)ga | (uintptr_t)ba) % 16)
        return OV3D_EINVAL;
    if (xb && (!gb || !bb || ((uintptr_t)gb | (uintptr_t)bb) % 16 || !al16(xb))) return OV3D_EINVAL;
    if (xb_inner < 0 || (xb_inner > 0 && (xb_s0 < C || xb_s1 < C || xb_s0 % 8 || xb_s1 % 8)))
        return OV3D_EINVAL;
    LnFwdArgs a{};
    a.R = R; a.src = src; a.src_bf16 = src_bf16; a.y = (const bf16*)y; a.pos = pos;
    a.pos_bf16 = pos_bf16; a.thresh = rowdrop::thresh(dropout_p);
    a.keep_scale = 1.f / (1.f - dropout_p); a.seed = seed; a.site = (uint32_t)site;
    a.ga = ga; a.ba = ba; a.gb = gb; a.bb = bb; a.eps = eps; a.s = s; a.mean = mean; a.rstd = rstd;
    a.xa = (bf16*)xa; a.xap = (bf16*)xap; a.xb = xb; a.xb_bf16 = xb_bf16;
    a.xb_inner = xb_inner; a.xb_s0 = xb_s0; a.xb_s1 = xb_s1;
    a.np = nprob;
    a.tiles[0] = 0;
    int ntot = 0;
    for (int i = 0; i < nprob; ++i) {
        const ov3d_lngemm_problem& q = probs[i];
        if (!q.W || !q.out || q.N <= 0 || q.N % 128 || q.ldw < C || q.ldw % 8 || !al16(q.W) ||
            (uintptr_t)q.out % 8 || q.ldo < q.N || q.ldo % 4 || (q.bias && (uintptr_t)q.bias % 8) ||
            (q.sel != 0 && q.sel != 1) || (q.sel == 1 && !pos))
            return OV3D_EINVAL;
        a.p[i] = LnProb{(const bf16*)q.W, q.ldw, (const bf16*)q.bias, (bf16*)q.out, q.ldo, q.N, q.sel};
        ntot += q.N;
    }
    // the 768-wide in-projection: 128-column tiles over 32 rows (fewer row-pass repeats, one
    // workgroup a CU); else 64 x 16 (256 workgroups for the decoder's 1024 rows)
    const int bn = ntot <= 256 ? 64 : 128;
    const int rbt = (bn == 128 && R % 32 == 0) ? 32 : 16;
    for (int i = 0; i < nprob; ++i) a.tiles[i + 1] = a.tiles[i] + probs[i].N / bn;
    a.epi = epilogue; a.thresh2 = rowdrop::thresh(dropout_p2);
    a.keep_scale2 = 1.f / (1.f - dropout_p2); a.seed2 = seed2; a.site2 = (uint32_t)site2;
    a.stamp = g_stamp;
    const dim3 grid(R / rbt, a.tiles[nprob]);
    hipStream_t st = ov3d_stream(stream);
    if (bn == 64) {
        if (epilogue == EPI_RELU_DROP) lngemm_fwd_kernel<EPI_RELU_DROP, 64, 16><<<grid, NT, 0, st>>>(a);
        else lngemm_fwd_kernel<EPI_NONE, 64, 16><<<grid, NT, 0, st>>>(a);
    } else if (rbt == 32) {
        if (epilogue == EPI_RELU_DROP) lngemm_fwd_kernel<EPI_RELU_DROP, 128, 32><<<grid, NT, 0, st>>>(a);
        else lngemm_fwd_kernel<EPI_NONE, 128, 32><<<grid, NT, 0, st>>>(a);
    } else {
        if (epilogue == EPI_RELU_DROP) lngemm_fwd_kernel<EPI_RELU_DROP, 128, 16><<<grid, NT, 0, st>>>(a);
        else lngemm_fwd_kernel<EPI_NONE, 128, 16><<<grid, NT, 0, st>>>(a);
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

// Measurement only: forward launches after this stamp 5 phase clocks per wave into buf
// (8 words a wave, (tile * row blocks + row block) * 8 + wave); null disarms.
extern "C" int ov3d_lngemm_stamps_arm(void* buf) {
    g_stamp = (unsigned long long*)buf;
    return OV3D_OK;
}

extern "C" int ov3d_lngemm_bwd_parts(int R) { return R > 0 && R % RB == 0 ? R / 8 : 0; }

extern "C" int ov3d_lngemm_bwd(int R, const float* s, const float* mean, const float* rstd,
                               const float* ds, const void* dxa, const void* dxap, const void* dxb,
                               int dxb_bf16, long long dxb_inner, long long dxb_s0,
                               long long dxb_s1, const float* ga, const float* gb, float dropout_p,
                               const int64_t* seed, int site, float* dsrc, void* dy, void* dpos,
                               int dpos_bf16, float* partials, int accumulate, const void* W,
                               long long ldw, int N, int epilogue, float dropout_p2, const void* H,
                               long long ldh, void* dx, long long lddx, void* stream) {
    if (R <= 0 || R % RB || !s || !mean || !rstd || !dy || !partials || !W || !dx || N <= 0 ||
        N % BNB || ldw < N || ldw % 8 || lddx < N || lddx % 4 || dropout_p < 0.f ||
        dropout_p >= 1.f || (dropout_p > 0.f && !seed) || dropout_p2 < 0.f || dropout_p2 >= 1.f ||
        (epilogue != EPI_NONE && epilogue != EPI_MASK))
        return OV3D_EINVAL;
    if (!(dxa || dxap || dxb)) return OV3D_EINVAL;
    if ((dxa || dxap) && (!ga || (uintptr_t)ga % 16)) return OV3D_EINVAL;
    if (dxb && (!gb || (uintptr_t)gb % 16)) return OV3D_EINVAL;
    if (dpos && !dxap) return OV3D_EINVAL;
    if (epilogue == EPI_MASK && (!H || (uintptr_t)H % 8 || ldh < N || ldh % 4)) return OV3D_EINVAL;
    if (!al16(s) || !al16(dy) || !al16(W) || (uintptr_t)dx % 8 || (ds && !al16(ds)) ||
        (dxa && !al16(dxa)) || (dxap && !al16(dxap)) || (dsrc && !al16(dsrc)) ||
        (dpos && !al16(dpos)) || (dxb && !dxb_inner && !al16(dxb)))
        return OV3D_EINVAL;
    if (dxb_inner < 0 || (dxb_inner > 0 && (dxb_s0 < C || dxb_s1 < C || dxb_s0 % 8 || dxb_s1 % 8)))
        return OV3D_EINVAL;
    LnBwdArgs a{};
    a.R = R; a.s = s; a.mean = mean; a.rstd = rstd; a.ds = ds; a.dxa = (const bf16*)dxa;
    a.dxap = (const bf16*)dxap; a.dxb = dxb; a.dxb_bf16 = dxb_bf16; a.dxb_inner = dxb_inner;
    a.dxb_s0 = dxb_s0; a.dxb_s1 = dxb_s1; a.ga = ga; a.gb = gb;
    a.thresh = rowdrop::thresh(dropout_p); a.keep_scale = 1.f / (1.f - dropout_p); a.seed = seed;
    a.site = (uint32_t)site; a.dsrc = dsrc; a.dy = (bf16*)dy; a.dpos = dpos; a.dpos_bf16 = dpos_bf16;
    a.partials = partials; a.accumulate = accumulate; a.W = (const bf16*)W; a.ldw = ldw;
    a.dx = (bf16*)dx; a.lddx = lddx; a.N = N; a.epi = epilogue;
    a.keep_scale2 = 1.f / (1.f - dropout_p2); a.H = (const bf16*)H; a.ldh = ldh;
    const dim3 grid(R / RB, N / BNB);
    hipStream_t st = ov3d_stream(stream);
    if (epilogue == EPI_MASK) lngemm_bwd_kernel<EPI_MASK><<<grid, NT, 0, st>>>(a);
    else lngemm_bwd_kernel<EPI_NONE><<<grid, NT, 0, st>>>(a);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
