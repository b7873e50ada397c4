// CLIP AttentionPool2d of the RegionCLIP ROI path, first query only (SURVEY §8a row a15:
// clip.inference at criterion.py:397 -> CLIPRes5ROIHeads -> upstream CLIP AttentionPool2d
// .forward, whose x[0] is the only output used), after the reassociation of
// regionclip._pool_tokens: a[r, h] = Wk_h^T q[r, h] is formed by the caller, so the keys and
// values of the 82 tokens are never projected.
//
// Token rows (never stored): t[r, 0] = t0[r] (ov3d_attnpool_mean: bf16(mean_j x[r, j]) + pos[0]),
// t[r, 1 + j] = bf16(x[r, j] + pos[1 + j]) from the res5 rows x (R, ntok, C).  Per ROI and head:
//   s[h, j] = bf16(a[r, h, :] . t[r, j, :])            fp32 sums (the bmm of _pool_tokens)
//   p[h, :] = bf16(softmax(s[h, :]))                      fp32
//   y[h, r, :] = bf16(sum_j p[h, j] t[r, j, :])           fp32 sums (the second bmm)
// in ONE launch: one 256-thread workgroup per ROI streams its rows twice in 64-channel chunks
// (s over the channels, then y chunk by chunk), t rebuilt in LDS both times; nothing of size
// R * (ntok + 1) * C reaches HBM (the token rows were 1.7 GB per C5 step, written once and read
// by two library bmm's).
//
// Matrix cores: v_mfma_f32_16x16x32_bf16.  s: A = a rows (h), B = t rows (j), both row reads of
// row-major LDS images; y^T = t^T p^T: A = t^T read with ds_read_b64_tr_b16 from the same
// row-major t image, B = p rows.  The y chunk goes out through LDS as whole 128-byte runs.
#include <math.h>

#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int TP = 96;     // token rows (ntok + 1 <= TP), padded with zeros
constexpr int HP = 48;     // head rows (H <= HP), padded with zeros
constexpr int CK = 64;     // channels per chunk
constexpr int LDT = 72;    // bf16 row stride of the t / a / y images (144 B)
constexpr int LDP = 104;   // bf16 row stride of the p image (208 B)
constexpr int LDS_S = 100; // f32 row stride of the score image

struct PoolArgs {
    const bf16* x;     // (R, ntok, C) res5 rows
    const bf16* t0;    // (R, C) mean-token rows (pos[0] added)
    const bf16* pos;   // (ntok + 1, C)
    const bf16* a;     // element (r, h, c) at a[h * sa_h + r * sa_r + c]
    long long sa_h, sa_r;
    bf16* y;           // (H, R, C)
    int R, ntok, C, H;
};

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x4 tr16(const bf16* p) {
    s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
    return __builtin_bit_cast(bf16x4, r);
}

// bf16(x + p) element-wise on one 16-byte run (fp32 add, one rounding: x + pos of the token rows)
__device__ __forceinline__ uint4 add_bf16x8(uint4 xa, uint4 pa) {
    const bf16x8 xv = __builtin_bit_cast(bf16x8, xa), pv = __builtin_bit_cast(bf16x8, pa);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)((float)xv[e] + (float)pv[e]);
    return __builtin_bit_cast(uint4, o);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// One chunk's global loads, held in registers while the previous chunk computes.  Thread
// (g = tid >> 3, v = tid & 7): token rows j = g, g + 32, g + 64 (j < ntok) and the 16-byte run v
// of the chunk; thread g == 31 also the t0 run (its third token slot, j = 95, is never a token);
// with A: head rows g and g + 32 (< H).
struct Stage {
    uint4 x[3], p[3], t0, a[2];
};

template <bool A>
__device__ __forceinline__ void load_chunk(const PoolArgs& P, int r, int c0, int g, int v, Stage& s) {
    const size_t cv = (size_t)c0 + 8 * v;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int j = g + 32 * k;
        if (j < P.ntok) {
            s.x[k] = *reinterpret_cast<const uint4*>(P.x + ((size_t)r * P.ntok + j) * P.C + cv);
            s.p[k] = *reinterpret_cast<const uint4*>(P.pos + (size_t)(1 + j) * P.C + cv);
        }
    }
    if (g == 31) s.t0 = *reinterpret_cast<const uint4*>(P.t0 + (size_t)r * P.C + cv);
    if (A) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int h = g + 32 * k;
            if (h < P.H) s.a[k] = *reinterpret_cast<const uint4*>(P.a + h * P.sa_h + r * P.sa_r + cv);
        }
    }
}

template <bool A>
__device__ __forceinline__ void store_chunk(const PoolArgs& P, int g, int v, const Stage& s, bf16* tS,
                                            bf16* aS) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int j = g + 32 * k;
        if (j < P.ntok) *reinterpret_cast<uint4*>(tS + (1 + j) * LDT + 8 * v) = add_bf16x8(s.x[k], s.p[k]);
    }
    if (g == 31) *reinterpret_cast<uint4*>(tS + 8 * v) = s.t0;
    if (A) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int h = g + 32 * k;
            if (h < P.H) *reinterpret_cast<uint4*>(aS + h * LDT + 8 * v) = s.a[k];
        }
    }
}

__global__ void __launch_bounds__(256) attnpool_fused_kernel(PoolArgs P) {
    __shared__ __attribute__((aligned(16))) bf16 tS[TP * LDT];
    __shared__ __attribute__((aligned(16))) bf16 aS[HP * LDT];   // a chunk; the y chunk in pass 2
    __shared__ __attribute__((aligned(16))) float sS[HP * LDS_S];
    __shared__ __attribute__((aligned(16))) bf16 pS[HP * LDP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = tid >> 3, v = tid & 7;
    const int li = lane & 15, G = lane >> 4;
    const int r = blockIdx.x;
    const int T = P.ntok + 1, nC = P.C / CK;

    // zero padding: token rows >= T, head rows >= H (never written below)
    for (int i = tid; i < (TP - T) * (LDT / 8); i += 256)
        *reinterpret_cast<uint4*>(tS + (T + i / (LDT / 8)) * LDT + 8 * (i % (LDT / 8))) = make_uint4(0, 0, 0, 0);
    for (int i = tid; i < (HP - P.H) * (LDT / 8); i += 256)
        *reinterpret_cast<uint4*>(aS + (P.H + i / (LDT / 8)) * LDT + 8 * (i % (LDT / 8))) = make_uint4(0, 0, 0, 0);
    for (int i = tid; i < HP * LDP / 8; i += 256) reinterpret_cast<uint4*>(pS)[i] = make_uint4(0, 0, 0, 0);

    // ---- pass 1: s = a t^T over the channel chunks.  Wave w: tiles i = w + 4n < 18 of the
    // 3 (heads) x 6 (tokens) 16 x 16 tiles
    f32x4 acc[5];
#pragma unroll
    for (int n = 0; n < 5; ++n) acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
    Stage st;
    load_chunk<true>(P, r, 0, g, v, st);
    for (int cc = 0; cc < nC; ++cc) {
        __syncthreads();   // previous chunk's MFMA reads done (and the padding zeroed)
        store_chunk<true>(P, g, v, st, tS, aS);
        __syncthreads();
        if (cc + 1 < nC) load_chunk<true>(P, r, (cc + 1) * CK, g, v, st);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int n = 0; n < 5; ++n) {
                const int i = wave + 4 * n;
                if (i < 18) {
                    const int mt = i / 6, jt = i - 6 * (i / 6);
                    const bf16x8 fa = *reinterpret_cast<const bf16x8*>(aS + (16 * mt + li) * LDT + 32 * ks + 8 * G);
                    const bf16x8 fb = *reinterpret_cast<const bf16x8*>(tS + (16 * jt + li) * LDT + 32 * ks + 8 * G);
                    acc[n] = mfma16(fa, fb, acc[n]);
                }
            }
        }
    }
    // scores as the bmm leaves them: bf16, then fp32 for the softmax
#pragma unroll
    for (int n = 0; n < 5; ++n) {
        const int i = wave + 4 * n;
        if (i < 18) {
            const int mt = i / 6, jt = i - 6 * (i / 6);
#pragma unroll
            for (int e = 0; e < 4; ++e)
                sS[(16 * mt + 4 * G + e) * LDS_S + 16 * jt + li] = (float)(bf16)acc[n][e];
        }
    }
    __syncthreads();
    // ---- softmax over the T tokens of each head row: wave w takes rows w, w + 4, ...; lane
    // holds tokens lane and lane + 64
    for (int h = wave; h < P.H; h += 4) {
        const float v0 = lane < T ? sS[h * LDS_S + lane] : -INFINITY;
        const float v1 = lane + 64 < T ? sS[h * LDS_S + lane + 64] : -INFINITY;
        const float m = wave_max(fmaxf(v0, v1));
        const float e0 = lane < T ? expf(v0 - m) : 0.f;
        const float e1 = lane + 64 < T ? expf(v1 - m) : 0.f;
        const float sum = wave_sum(e0 + e1);
        pS[h * LDP + lane] = (bf16)(e0 / sum);
        if (lane + 64 < TP) pS[h * LDP + lane + 64] = (bf16)(e1 / sum);
    }
    // ---- pass 2: y^T = t^T p^T chunk by chunk.  Wave w: channels 16w .. 16w + 15 of the chunk,
    // the 3 head tiles, k over the 96 token rows (3 steps of 32)
    bf16* const yS = aS;   // [HP][LDT] bf16: the chunk's y rows
    load_chunk<false>(P, r, 0, g, v, st);
    for (int cc = 0; cc < nC; ++cc) {
        const int c0 = cc * CK;
        __syncthreads();   // pass 1 / the previous chunk done with tS; softmax done with sS
        store_chunk<false>(P, g, v, st, tS, nullptr);
        __syncthreads();
        if (cc + 1 < nC) load_chunk<false>(P, r, c0 + CK, g, v, st);
        f32x4 o[3];
#pragma unroll
        for (int ht = 0; ht < 3; ++ht) o[ht] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
            // t^T operand: lane (G, li) gets t[32ks + 8G + q][16w + li], q = 0..7; lane 4q' + p'
            // of the 16-lane group addresses row 32ks + 8G + q', columns 16w + 4p' .. + 3
            const bf16* ta = tS + (32 * ks + 8 * G + (li >> 2)) * LDT + 16 * wave + 4 * (li & 3);
            const bf16x4 lo = tr16(ta), hi = tr16(ta + 4 * LDT);
            bf16x8 fa;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                fa[e] = lo[e];
                fa[4 + e] = hi[e];
            }
#pragma unroll
            for (int ht = 0; ht < 3; ++ht) {
                const bf16x8 fb = *reinterpret_cast<const bf16x8*>(pS + (16 * ht + li) * LDP + 32 * ks + 8 * G);
                o[ht] = mfma16(fa, fb, o[ht]);
            }
        }
        // D[c][h]: lane holds head 16ht + li, channels 16w + 4G .. + 3
#pragma unroll
        for (int ht = 0; ht < 3; ++ht) {
            bf16x4 w4;
#pragma unroll
            for (int e = 0; e < 4; ++e) w4[e] = (bf16)o[ht][e];
            *reinterpret_cast<bf16x4*>(yS + (16 * ht + li) * LDT + 16 * wave + 4 * G) = w4;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int h = g + 32 * k;
            if (h < P.H)
                *reinterpret_cast<uint4*>(P.y + ((size_t)h * P.R + r) * P.C + c0 + 8 * v) =
                    *reinterpret_cast<const uint4*>(yS + h * LDT + 8 * v);
        }
    }
}

// t0[r] = bf16(bf16(mean_j x[r, j]) + pos[0]): fp32 sum in token order, as attnpool_tokens_kernel
// (csrc/conv.hip) forms t[r, 0]; one thread per 16-byte channel run of one ROI
__global__ void __launch_bounds__(256) attnpool_mean_kernel(const bf16* __restrict__ x, int ntok, int CV,
                                                            int total, const bf16* __restrict__ pos,
                                                            bf16* __restrict__ t0) {
    const int gi = blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= total) return;
    const int r = gi / CV, cv = gi - r * CV;
    const uint4* xs = reinterpret_cast<const uint4*>(x) + (size_t)r * ntok * CV + cv;
    float sum[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) sum[e] = 0.f;
    for (int j = 0; j < ntok; ++j) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, xs[(size_t)j * CV]);
#pragma unroll
        for (int e = 0; e < 8; ++e) sum[e] += (float)a[e];
    }
    const bf16x8 p0 = __builtin_bit_cast(bf16x8, reinterpret_cast<const uint4*>(pos)[cv]);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)((float)(bf16)(sum[e] / (float)ntok) + (float)p0[e]);
    reinterpret_cast<uint4*>(t0)[(size_t)r * CV + cv] = __builtin_bit_cast(uint4, o);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int ov3d_attnpool_mean(const void* x, int R, int ntok, int C, const void* pos, void* t0,
                                  void* stream) {
    if (!x || !pos || !t0 || R < 0 || ntok <= 0 || C <= 0 || C % 8 || !aligned16(x) || !aligned16(pos) ||
        !aligned16(t0))
        return OV3D_EINVAL;
    const long long total = (long long)R * (C / 8);
    if (total == 0) return OV3D_OK;
    if (total > 0x7fffffffLL) return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    attnpool_mean_kernel<<<ov3d_cdiv(total, 256), 256, 0, s>>>((const bf16*)x, ntok, C / 8, (int)total,
                                                               (const bf16*)pos, (bf16*)t0);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_attnpool_fused_supported(int ntok, int C, int H) {
    return ntok >= 1 && ntok + 1 <= TP && C >= CK && C % CK == 0 && H >= 1 && H <= HP;
}

extern "C" int ov3d_attnpool_fused(const void* x, const void* t0, const void* pos, const void* a,
                                   long long sa_h, long long sa_r, int R, int ntok, int C, int H,
                                   void* y, void* stream) {
    if (!x || !t0 || !pos || !a || !y || R < 0 || !ov3d_attnpool_fused_supported(ntok, C, H) ||
        sa_h % 8 || sa_r % 8 || sa_h < 0 || sa_r < 0 || !aligned16(x) || !aligned16(t0) ||
        !aligned16(pos) || !aligned16(a) || !aligned16(y))
        return OV3D_EINVAL;
    if (R == 0) return OV3D_OK;
    PoolArgs P{(const bf16*)x, (const bf16*)t0, (const bf16*)pos, (const bf16*)a, sa_h, sa_r,
               (bf16*)y, R, ntok, C, H};
    hipStream_t s = ov3d_stream(stream);
    attnpool_fused_kernel<<<R, 256, 0, s>>>(P);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
