// Training BatchNorm1d + ReLU + Dropout over channels-last rows, for the GenericMLP
// prediction heads of 3DETR (models/helpers.py:45-112 as built by
// models/model_3detr.py:_build_heads: Conv1d -> BatchNorm1d -> ReLU -> Dropout(0.3), x2)
// with the five heads evaluated side by side as one (R, 5*256) channel set.
//
// Tensor addressing (every operand): channel c of row r lives at
//   base + (c / cb) * bstride + r * ld + (c % cb)
// so one kernel reads a row-major (R, C) tensor (cb = C, bstride = 0) or the per-head
// blocks of a batched GEMM output (cb = 256, ld = 256, bstride = R*256).  A thread owns
// 8 adjacent channels (one 16-byte bf16 run) of a row.
//
//   ov3d_rows_bn_stats  : fp64 partials (nparts, 2, C) of sum x and sum x^2
//   (ov3d_reduce_partials + ov3d_bn_finalize of sa_mlp.hip turn them into scale/shift)
//   ov3d_rows_bn_apply  : z = dropout(relu(x*scale + shift)) -> bf16
//   ov3d_rows_bn_bwd    : dt = dz * keep/(1-p) * [x*scale+shift > 0];
//                         pass 0: partials of sum dt and sum dt*xhat; pass 1: dx = cA dt + cB x + cC
// Dropout keep(r, c) is a counter-based hash of (seed, site, r, c): the backward
// regenerates the mask instead of storing it.
#include "common.h"
#include "rowdrop.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct RowsLayout {
    long long ld, bstride;
    int cb;
};

__device__ __forceinline__ long long addr(const RowsLayout& L, long long r, int c) {
    return (long long)(c / L.cb) * L.bstride + r * L.ld + (c % L.cb);
}

using rowdrop::keep8;
using rowdrop::mix32;
using rowdrop::row_base;

// rows-per-thread phase layout: TP threads per row (one per 8-channel run), RP rows at once
struct Phase {
    int tp, rp, ph, c;
    bool active;
};
__device__ __forceinline__ Phase phase(int C) {
    Phase p;
    const int runs = C / 8;
    p.tp = runs < 256 ? runs : 256;
    p.rp = 256 / p.tp;
    p.ph = threadIdx.x / p.tp;
    p.c = (threadIdx.x % p.tp) * 8;
    p.active = p.ph < p.rp;
    return p;
}

template <typename T>
__device__ __forceinline__ void load8(const T* base, const RowsLayout& L, long long r, int c, float* v);
template <>
__device__ __forceinline__ void load8<bf16>(const bf16* base, const RowsLayout& L, long long r, int c,
                                            float* v) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(base + addr(L, r, c));
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
}
template <>
__device__ __forceinline__ void load8<float>(const float* base, const RowsLayout& L, long long r,
                                             int c, float* v) {
    const float4 a = *reinterpret_cast<const float4*>(base + addr(L, r, c));
    const float4 b = *reinterpret_cast<const float4*>(base + addr(L, r, c) + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// reduce the two per-thread accumulators over the RP row phases of the block and write
// the block's fp64 partials (sum over its rows) for channels cbase .. cbase + 8*TP
__device__ void block_partials(const Phase& p, int C, int cbase, float (*acc)[8],
                               double* partials) {
    __shared__ float red[2][2048];
    const int W = p.tp * 8;
    __syncthreads();
    if (p.active)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            red[0][p.ph * W + p.c + j] = acc[0][j];
            red[1][p.ph * W + p.c + j] = acc[1][j];
        }
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * W; i += blockDim.x) {
        const int v = i / W, cc = i - v * W;
        if (cbase + cc < C) {
            double t = 0.0;
            for (int k = 0; k < p.rp; ++k) t += (double)red[v][k * W + cc];
            partials[((size_t)blockIdx.x * 2 + v) * C + cbase + cc] = t;
        }
    }
}

template <typename T>
__global__ void __launch_bounds__(256) rows_bn_stats_kernel(const T* __restrict__ x, RowsLayout L,
                                                            long long R, int C,
                                                            double* __restrict__ partials) {
    const Phase p = phase(C);
    for (int cbase = 0; cbase < C; cbase += p.tp * 8) {
        const int c = cbase + p.c;
        float acc[2][8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[0][j] = acc[1][j] = 0.f;
        if (p.active && c < C) {
            // 4 rows' loads in flight per round (the loop is latency-bound otherwise: 32 rows
            // per block at 8192 rows); the per-lane summation order is the row order, as before
            const long long step = (long long)gridDim.x * p.rp;
            long long r = (long long)blockIdx.x * p.rp + p.ph;
            for (; r + 3 * step < R; r += 4 * step) {
                float v[4][8];
#pragma unroll
                for (int u = 0; u < 4; ++u) load8<T>(x, L, r + u * step, c, v[u]);
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        acc[0][j] += v[u][j];
                        acc[1][j] = fmaf(v[u][j], v[u][j], acc[1][j]);
                    }
            }
            for (; r < R; r += step) {
                float v[8];
                load8<T>(x, L, r, c, v);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    acc[0][j] += v[j];
                    acc[1][j] = fmaf(v[j], v[j], acc[1][j]);
                }
            }
        }
        block_partials(p, C, cbase, acc, partials);
    }
}

// Element passes: a thread owns one 8-channel run (its per-channel coefficients loaded once and
// its layout offset computed once) and RPT rows of it, the rows' loads in flight together; the
// grid covers R in (256 / runs) * RPT-row slabs.  (One run per thread per launch cost ~60 %
// more than the HBM floor at 2^18 x 256: ten coefficient loads, three runtime divisions of the
// layout and 64-bit index math for each 16 bytes of data.)
constexpr int RPT = 4;

__device__ __forceinline__ long long coff(const RowsLayout& L, int c) {
    return (long long)(c / L.cb) * L.bstride + (c % L.cb);
}

template <typename T>
__device__ __forceinline__ void load8o(const T* base, long long off, float* v);
template <>
__device__ __forceinline__ void load8o<bf16>(const bf16* base, long long off, float* v) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(base + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
}
template <>
__device__ __forceinline__ void load8o<float>(const float* base, long long off, float* v) {
    const float4 a = *reinterpret_cast<const float4*>(base + off);
    const float4 b = *reinterpret_cast<const float4*>(base + off + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void ld8f(const float* p, float* v) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// the run / rows of this thread: rows r0 + k * rstep (k < RPT), channel c
struct Slab {
    int c;
    long long r0, rstep;
    bool active;
};
__device__ __forceinline__ Slab slab(int C) {
    Slab q;
    const int runs = C / 8;
    const int tpr = runs < 256 ? runs : 256;       // threads per row
    const int rpb = 256 / tpr;                      // rows per block pass
    const int ph = threadIdx.x / tpr;
    const int chunks = (runs + tpr - 1) / tpr;      // C > 2048: several thread rows per row
    const int chunk = blockIdx.x % chunks;
    const long long blk = blockIdx.x / chunks;
    q.c = (chunk * tpr + threadIdx.x % tpr) * 8;
    q.r0 = blk * (long long)rpb * RPT + ph;
    q.rstep = rpb;
    q.active = ph < rpb && q.c < C;
    return q;
}
__host__ __device__ inline long long slab_blocks(long long R, int C) {
    const int runs = C / 8;
    const int tpr = runs < 256 ? runs : 256;
    const int rpb = 256 / tpr;
    return ((R + (long long)rpb * RPT - 1) / ((long long)rpb * RPT)) * ((runs + tpr - 1) / tpr);
}

template <typename T>
__global__ void __launch_bounds__(256) rows_bn_apply_kernel(
    const T* __restrict__ x, RowsLayout L, long long R, int C, const float* __restrict__ scale,
    const float* __restrict__ shift, uint32_t thresh, float keep_scale, const int64_t* seed,
    uint32_t site, bf16* __restrict__ out, RowsLayout LO) {
    const Slab q = slab(C);
    if (!q.active) return;
    const int c = q.c;
    float sc[8], sh[8];
    ld8f(scale + c, sc);
    ld8f(shift + c, sh);
    const long long ox = coff(L, c), oo = coff(LO, c);
    uint32_t sm = 0;
    if (thresh) {
        const uint64_t s = (uint64_t)*seed;
        sm = mix32((uint32_t)s ^ mix32((uint32_t)(s >> 32) + site * 0x9E3779B9u));
    }
    float v[RPT][8];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const long long r = q.r0 + k * q.rstep;
        if (r < R) load8o<T>(x, ox + r * L.ld, v[k]);
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const long long r = q.r0 + k * q.rstep;
        if (r >= R) break;
        bool keep[8];
        if (thresh) keep8(row_base(sm, r), c, thresh, keep);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float z = fmaxf(fmaf(v[k][j], sc[j], sh[j]), 0.f);
            if (thresh) z = keep[j] ? z * keep_scale : 0.f;
            o[j] = (bf16)z;
        }
        *reinterpret_cast<bf16x8*>(out + oo + r * LO.ld) = o;
    }
}

// the dz run (row r, channels c .. c+7): read, or (POOLED) rebuilt from the neighbour max-pool's
// pooled gradient g (P, C) and arg rows (P, C) uint8 -- row r = p * S + s takes g[p] where
// arg[p] == s, else 0 (exactly the dense gradient ov3d_nbr_max_bwd would have written)
typedef uint8_t u8x8 __attribute__((ext_vector_type(8)));
template <bool POOLED>
__device__ __forceinline__ void load_dz(const bf16* dz, const RowsLayout& LZ, long long r, int c,
                                        const uint8_t* parg, int pS, int C, float* v) {
    if constexpr (!POOLED) {
        load8<bf16>(dz, LZ, r, c, v);
    } else {
        const long long p = r / pS;
        const int s = (int)(r - p * pS);
        float g[8];
        load8<bf16>(dz, LZ, p, c, g);
        const u8x8 a = *reinterpret_cast<const u8x8*>(parg + p * C + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = a[j] == s ? g[j] : 0.f;
    }
}

template <int PASS, typename T, bool POOLED = false>
__global__ void __launch_bounds__(256) rows_bn_bwd_kernel(
    const bf16* __restrict__ dz, RowsLayout LZ, const T* __restrict__ x, RowsLayout LX, long long R,
    int C, const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ cA,
    const float* __restrict__ cB, const float* __restrict__ cC, uint32_t thresh, float keep_scale,
    const int64_t* seed, uint32_t site, double* __restrict__ partials, bf16* __restrict__ dx,
    RowsLayout LD, const uint8_t* __restrict__ parg = nullptr, int pS = 1) {
    uint32_t sm = 0;
    if (thresh) {
        const uint64_t s = (uint64_t)*seed;
        sm = mix32((uint32_t)s ^ mix32((uint32_t)(s >> 32) + site * 0x9E3779B9u));
    }
    if (PASS == 1) {
        const Slab q = slab(C);
        if (!q.active) return;
        const int c = q.c;
        float sc[8], sh[8], a[8], b[8], cc[8];
        ld8f(scale + c, sc);
        ld8f(shift + c, sh);
        ld8f(cA + c, a);
        ld8f(cB + c, b);
        ld8f(cC + c, cc);
        const long long ox = coff(LX, c), oz = coff(LZ, c), od = coff(LD, c);
        float xv[RPT][8], zv[RPT][8];
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const long long r = q.r0 + k * q.rstep;
            if (r < R) {
                load8o<T>(x, ox + r * LX.ld, xv[k]);
                if constexpr (POOLED) load_dz<true>(dz, LZ, r, c, parg, pS, C, zv[k]);
                else load8o<bf16>(dz, oz + r * LZ.ld, zv[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const long long r = q.r0 + k * q.rstep;
            if (r >= R) break;
            bool keep[8];
            if (thresh) keep8(row_base(sm, r), c, thresh, keep);
            bf16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float dt = fmaf(xv[k][j], sc[j], sh[j]) > 0.f ? zv[k][j] : 0.f;
                if (thresh) dt = keep[j] ? dt * keep_scale : 0.f;
                o[j] = (bf16)fmaf(a[j], dt, fmaf(b[j], xv[k][j], cc[j]));
            }
            *reinterpret_cast<bf16x8*>(dx + od + r * LD.ld) = o;
        }
        return;
    }
    const Phase p = phase(C);
    for (int cbase = 0; cbase < C; cbase += p.tp * 8) {
        const int c = cbase + p.c;
        float acc[2][8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[0][j] = acc[1][j] = 0.f;
        if (p.active && c < C) {
            float sc[8], sh[8], mu[8], is[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                sc[j] = scale[c + j]; sh[j] = shift[c + j]; mu[j] = mean[c + j]; is[j] = invstd[c + j];
            }
            auto row = [&](long long r, const float* xv, const float* zv) {
                bool keep[8];
                if (thresh) keep8(row_base(sm, r), c, thresh, keep);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    float dt = fmaf(xv[j], sc[j], sh[j]) > 0.f ? zv[j] : 0.f;
                    if (thresh) dt = keep[j] ? dt * keep_scale : 0.f;
                    acc[0][j] += dt;
                    acc[1][j] = fmaf(dt, (xv[j] - mu[j]) * is[j], acc[1][j]);
                }
            };
            // 4 rows' loads in flight per round (latency-bound loop otherwise: the heads' 1280
            // channels leave one row per block and step; 2 rows measured 14.9 us); row order kept
            const long long step = (long long)gridDim.x * p.rp;
            long long r = (long long)blockIdx.x * p.rp + p.ph;
            for (; r + 3 * step < R; r += 4 * step) {
                float xv[4][8], zv[4][8];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    load8<T>(x, LX, r + u * step, c, xv[u]);
                    load_dz<POOLED>(dz, LZ, r + u * step, c, parg, pS, C, zv[u]);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) row(r + u * step, xv[u], zv[u]);
            }
            for (; r < R; r += step) {
                float xv[8], zv[8];
                load8<T>(x, LX, r, c, xv);
                load_dz<POOLED>(dz, LZ, r, c, parg, pS, C, zv);
                row(r, xv, zv);
            }
        }
        block_partials(p, C, cbase, acc, partials);
    }
}

uint32_t drop_thresh(float p) { return rowdrop::thresh(p); }

bool layout_ok(const RowsLayout& L, int C) {
    return L.cb > 0 && L.cb % 8 == 0 && C % L.cb == 0 && L.ld >= L.cb && L.ld % 8 == 0 &&
           L.bstride % 8 == 0;
}

}  // namespace

extern "C" int ov3d_rows_bn_stats(const void* x, int is_bf16, long long ld, long long bstride,
                                  int cb, long long R, int C, double* partials, int nparts,
                                  void* stream) {
    RowsLayout L{ld, bstride, cb};
    if (!x || !partials || R <= 0 || C <= 0 || C % 8 || nparts <= 0 || !layout_ok(L, C))
        return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    if (is_bf16)
        rows_bn_stats_kernel<bf16><<<nparts, 256, 0, s>>>((const bf16*)x, L, R, C, partials);
    else
        rows_bn_stats_kernel<float><<<nparts, 256, 0, s>>>((const float*)x, L, R, C, partials);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_rows_bn_apply(const void* x, int is_bf16, long long ld, long long bstride, int cb,
                                  long long R, int C, const float* scale, const float* shift,
                                  float dropout_p, const int64_t* seed, int site, void* out,
                                  long long ldo, long long bstride_o, int cbo, void* stream) {
    RowsLayout L{ld, bstride, cb}, LO{ldo, bstride_o, cbo};
    if (!x || !scale || !shift || !out || R <= 0 || C <= 0 || C % 8 || !layout_ok(L, C) ||
        !layout_ok(LO, C) || dropout_p < 0.f || dropout_p >= 1.f || (dropout_p > 0.f && !seed))
        return OV3D_EINVAL;
    const long long nb = slab_blocks(R, C);
    hipStream_t s = ov3d_stream(stream);
    const uint32_t th = drop_thresh(dropout_p);
    const float ks = 1.f / (1.f - dropout_p);
    if (is_bf16)
        rows_bn_apply_kernel<bf16><<<(unsigned)nb, 256, 0, s>>>(
            (const bf16*)x, L, R, C, scale, shift, th, ks, seed, (uint32_t)site, (bf16*)out, LO);
    else
        rows_bn_apply_kernel<float><<<(unsigned)nb, 256, 0, s>>>(
            (const float*)x, L, R, C, scale, shift, th, ks, seed, (uint32_t)site, (bf16*)out, LO);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_rows_bn_bwd(int pass, const void* dz, long long ldz, long long bstride_z, int cbz,
                                const void* x, int x_bf16, long long ldx, long long bstride_x,
                                int cbx, long long R, int C, const float* scale, const float* shift,
                                const float* mean, const float* invstd, const float* cA,
                                const float* cB, const float* cC, float dropout_p,
                                const int64_t* seed, int site, double* partials, int nparts,
                                void* dx, long long ldd, long long bstride_d, int cbd,
                                void* stream) {
    RowsLayout LZ{ldz, bstride_z, cbz}, LX{ldx, bstride_x, cbx}, LD{ldd, bstride_d, cbd};
    if (!dz || !x || R <= 0 || C <= 0 || C % 8 || !layout_ok(LZ, C) || !layout_ok(LX, C) ||
        dropout_p < 0.f || dropout_p >= 1.f || (dropout_p > 0.f && !seed) || (pass != 0 && pass != 1))
        return OV3D_EINVAL;
    if (pass == 0 && (!partials || nparts <= 0 || !mean || !invstd)) return OV3D_EINVAL;
    if (pass == 1 && (!dx || !cA || !cB || !cC || !layout_ok(LD, C))) return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    const uint32_t th = drop_thresh(dropout_p);
    const float ks = 1.f / (1.f - dropout_p);
    if (pass == 0) {
        if (x_bf16)
            rows_bn_bwd_kernel<0, bf16><<<nparts, 256, 0, s>>>(
                (const bf16*)dz, LZ, (const bf16*)x, LX, R, C, scale, shift, mean, invstd, cA, cB,
                cC, th, ks, seed, (uint32_t)site, partials, (bf16*)dx, LD);
        else
            rows_bn_bwd_kernel<0, float><<<nparts, 256, 0, s>>>(
                (const bf16*)dz, LZ, (const float*)x, LX, R, C, scale, shift, mean, invstd, cA, cB,
                cC, th, ks, seed, (uint32_t)site, partials, (bf16*)dx, LD);
    } else {
        const long long nb = slab_blocks(R, C);
        if (x_bf16)
            rows_bn_bwd_kernel<1, bf16><<<(unsigned)nb, 256, 0, s>>>(
                (const bf16*)dz, LZ, (const bf16*)x, LX, R, C, scale, shift, mean, invstd, cA, cB,
                cC, th, ks, seed, (uint32_t)site, partials, (bf16*)dx, LD);
        else
            rows_bn_bwd_kernel<1, float><<<(unsigned)nb, 256, 0, s>>>(
                (const bf16*)dz, LZ, (const float*)x, LX, R, C, scale, shift, mean, invstd, cA, cB,
                cC, th, ks, seed, (uint32_t)site, partials, (bf16*)dx, LD);
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_rows_bn_bwd_pooled(int pass, const void* g, const uint8_t* arg, int S,
                                       const void* x, long long R, int C, const float* scale,
                                       const float* shift, const float* mean, const float* invstd,
                                       const float* cA, const float* cB, const float* cC,
                                       double* partials, int nparts, void* dx, void* stream) {
    // row-major bf16 (P * S, C) rows x, (P, C) pooled gradient g and arg; no dropout (the SA
    // layers' BatchNorm + ReLU)
    RowsLayout L{C, 0, C};
    if (!g || !arg || !x || S <= 0 || S > 256 || R <= 0 || R % S || C <= 0 || C % 8 ||
        ((uintptr_t)g | (uintptr_t)x) % 16 || (uintptr_t)arg % 8 || (pass != 0 && pass != 1))
        return OV3D_EINVAL;
    if (pass == 0 && (!partials || nparts <= 0 || !mean || !invstd || !scale || !shift))
        return OV3D_EINVAL;
    if (pass == 1 && (!dx || !cA || !cB || !cC || !scale || !shift || (uintptr_t)dx % 16))
        return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    if (pass == 0)
        rows_bn_bwd_kernel<0, bf16, true><<<nparts, 256, 0, s>>>(
            (const bf16*)g, L, (const bf16*)x, L, R, C, scale, shift, mean, invstd, cA, cB, cC, 0u,
            1.f, nullptr, 0u, partials, (bf16*)dx, L, arg, S);
    else
        rows_bn_bwd_kernel<1, bf16, true><<<(unsigned)slab_blocks(R, C), 256, 0, s>>>(
            (const bf16*)g, L, (const bf16*)x, L, R, C, scale, shift, mean, invstd, cA, cB, cC, 0u,
            1.f, nullptr, 0u, partials, (bf16*)dx, L, arg, S);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
