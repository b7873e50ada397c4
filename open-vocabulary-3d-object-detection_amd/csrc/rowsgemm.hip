// Short row-block GEMMs with the bias epilogue: the 3DETR decoder's linear layers (M = Q*B =
// 1024 rows of 256 / 512 features, models/transformer.py:355-379 forward_pre) forward and
// input-gradient, where a library GEMM's time is its pipeline latency, not its work.
//
//   trans_b = 1 (nn.Linear forward): C (M x N) = A (M x K) W^T + bias, W (N x K) row-major
//   trans_b = 0 (input gradient):    C (M x N) = A (M x K) W,          W (K x N) row-major
//
// bf16 operands, fp32 accumulation, bf16 output (bias added in fp32 before the rounding, as
// the hipBLASLt bias epilogue does).  One workgroup = 4 waves = one 32 x 32 output tile;
// the K range is split over the 4 waves (one v_mfma_f32_32x32x16_bf16 chain each) and the
// partial tiles are summed through LDS in a fixed order.  Every operand load of a wave is
// issued before its first MFMA: one memory round trip per launch.
//   trans_b = 1: both operands are K-contiguous rows, loaded straight into the MFMA
//                fragment layout (lane = row / column, 8 consecutive k).
//   trans_b = 0: the W tile (k rows x 32 columns) goes through LDS and is read transposed
//                with ds_read_b64_tr_b16 (k order 8(j>>2) + 4h + (j&3) inside a 16-k step;
//                A's fragment is loaded in the same k order).
// Epilogues (ov3d_rows_gemm_act) fuse the FFN activation of the transformer layers
// (models/transformer.py:276-278, 375-377: linear1 -> ReLU -> dropout):
//   EPI_RELU_DROP: out = dropout(relu(bf16(acc + bias)))   (the rowdrop.h keep hash, as
//                  ov3d_relu_dropout_fwd: identical output)
//   EPI_MASK:      out = h > 0 ? bf16(bf16(acc) / (1 - p)) : 0   (the input gradient of
//                  linear2 through that activation, as ov3d_relu_dropout_bwd)
#include "common.h"
#include "rowdrop.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4;
constexpr int kTile = 32;
constexpr int kMaxSteps = 16;   // 16-k MFMA steps per wave: K <= 4 * 16 * 16 = 1024
constexpr int LDW = 40;         // LDS row of the (k, 32 columns) W tile, bf16 elements (80 B)
enum { EPI_NONE = 0, EPI_RELU_DROP = 1, EPI_MASK = 2 };

struct GemmArgs {
    const bf16* A; long long lda;
    const bf16* W; long long ldw;
    const bf16* bias;
    bf16* C; long long ldc;
    int M, N, K;
    int epi; uint32_t thresh; float keep_scale; const int64_t* seed; uint32_t site;
    const bf16* H; long long ldh;   // EPI_MASK: the activation output
};

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x4 tr16(const bf16* p) {
    s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(p));
    return __builtin_bit_cast(bf16x4, r);
}

// One 32 x 32 output tile (m0, n0) of problem a; K = 4 waves x 16 x `steps` (<= STEPS).
template <int TB, int STEPS>
__device__ __forceinline__ void gemm_tile(const GemmArgs& a, int m0, int n0, int steps,
                                          float (*red)[kTile][kTile + 1], bf16* Ws) {
    const int KW = 16 * steps;   // k per wave
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int kq = w * KW;
    const int row = min(m0 + r, a.M - 1);
    const bf16* ap = a.A + (size_t)row * a.lda + kq;
    bf16x8 av[STEPS], bv[STEPS];
    if (TB) {
        const bf16* wp = a.W + (size_t)(n0 + r) * a.ldw + kq + 8 * h;
#pragma unroll
        for (int s = 0; s < STEPS; ++s) {
            if (s < steps) {
                av[s] = *reinterpret_cast<const bf16x8*>(ap + 16 * s + 8 * h);
                bv[s] = *reinterpret_cast<const bf16x8*>(wp + 16 * s);
            }
        }
        // every load in flight before the first MFMA (the scheduler would otherwise pair
        // each load with its MFMA and serialise the memory latency)
        __builtin_amdgcn_sched_barrier(0);
    } else {
        // W rows kq .. kq+KW-1, columns n0 .. n0+31: 4 lanes x 16 B per row, 16 rows a pass
        bf16* ws = Ws + w * 16 * STEPS * LDW;
        bf16x8 wr[STEPS];
#pragma unroll
        for (int s = 0; s < STEPS; ++s)
            if (s < steps)
                wr[s] = *reinterpret_cast<const bf16x8*>(a.W + (size_t)(kq + 16 * s + (lane >> 2)) * a.ldw +
                                                         n0 + 8 * (lane & 3));
#pragma unroll
        for (int s = 0; s < STEPS; ++s) {
            if (s < steps) {
                const bf16x4 lo = *reinterpret_cast<const bf16x4*>(ap + 16 * s + 4 * h);
                const bf16x4 hi = *reinterpret_cast<const bf16x4*>(ap + 16 * s + 8 + 4 * h);
                av[s] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < STEPS; ++s)
            if (s < steps)
                *reinterpret_cast<bf16x8*>(ws + (16 * s + (lane >> 2)) * LDW + 8 * (lane & 3)) = wr[s];
        __syncthreads();
        const int g = lane >> 4, i = lane & 15;
        const int d0 = 16 * (g & 1) + 4 * (i & 3);
#pragma unroll
        for (int s = 0; s < STEPS; ++s) {
            if (s < steps) {
                const int k0 = 16 * s + 4 * (g >> 1) + (i >> 2);
                const bf16x4 lo = tr16(ws + k0 * LDW + d0);
                const bf16x4 hi = tr16(ws + (k0 + 8) * LDW + d0);
                bv[s] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            }
        }
    }
    // S^T-style product: acc lane (col = r, rows (v&3) + 8(v>>2) + 4h) = C[m0 + row][n0 + r]
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.f;
#pragma unroll
    for (int s = 0; s < STEPS; ++s)
        if (s < steps) acc = mfma(av[s], bv[s], acc);
#pragma unroll
    for (int v = 0; v < 16; ++v) red[w][(v & 3) + 8 * (v >> 2) + 4 * h][r] = acc[v];
    __syncthreads();
    const int orow = threadIdx.x >> 3, oc = (threadIdx.x & 7) * 4;
    const int gr = m0 + orow, gc = n0 + oc;
    if (gr >= a.M) return;
    bool keep[4] = {true, true, true, true};
    if (a.epi == EPI_RELU_DROP && a.thresh) {
        // rowdrop.h: one hash per channel pair of row gr
        const uint32_t rb = rowdrop::row_base(rowdrop::seed_mix(a.seed, a.site), gr);
#pragma unroll
        for (int j = 0; j < 4; j += 2) {
            const uint32_t hs = rowdrop::mix24(rb + (uint32_t)((gc + j) >> 1) * 0x27D4EB2Fu);
            keep[j] = (hs & 0xffffu) >= a.thresh;
            keep[j + 1] = (hs >> 16) >= a.thresh;
        }
    }
    bf16x4 hv;
    if (a.epi == EPI_MASK) hv = *reinterpret_cast<const bf16x4*>(a.H + (size_t)gr * a.ldh + gc);
    bf16x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        float t = (red[0][orow][oc + q] + red[1][orow][oc + q]) +
                  (red[2][orow][oc + q] + red[3][orow][oc + q]);
        if (a.bias) t += (float)a.bias[gc + q];
        const bf16 y = (bf16)t;
        if (a.epi == EPI_RELU_DROP) {
            const float rr = fmaxf((float)y, 0.f);
            o[q] = a.thresh ? (keep[q] ? (bf16)(rr * a.keep_scale) : (bf16)0.f) : (bf16)rr;
        } else if (a.epi == EPI_MASK) {
            o[q] = (float)hv[q] > 0.f ? (bf16)((float)y * a.keep_scale) : (bf16)0.f;
        } else {
            o[q] = y;
        }
    }
    *reinterpret_cast<bf16x4*>(a.C + (size_t)gr * a.ldc + gc) = o;
}

template <int TB, int STEPS>
__global__ void __launch_bounds__(256) rows_gemm_kernel(GemmArgs a) {
    __shared__ float red[kWaves][kTile][kTile + 1];
    __shared__ __attribute__((aligned(16))) bf16 Ws[TB ? 1 : kWaves * 16 * STEPS * LDW];
    gemm_tile<TB, STEPS>(a, blockIdx.x * kTile, blockIdx.y * kTile, STEPS, red, Ws);
}

// Several problems over the same rows in one launch (the in-projection blocks of one
// attention, gemm._InProj): blockIdx.y enumerates the 32-column tiles of all problems.
constexpr int kGroupProbs = 4;
struct GemmGroup {
    GemmArgs p[kGroupProbs];
    int tiles[kGroupProbs + 1];
    int n;
};

template <int TB, int STEPS>
__global__ void __launch_bounds__(256) rows_gemm_group_kernel(GemmGroup g) {
    __shared__ float red[kWaves][kTile][kTile + 1];
    __shared__ __attribute__((aligned(16))) bf16 Ws[TB ? 1 : kWaves * 16 * STEPS * LDW];
    const int t = blockIdx.y;
    int i = 0;
    while (i + 1 < g.n && t >= g.tiles[i + 1]) ++i;
    const GemmArgs& a = g.p[i];
    gemm_tile<TB, STEPS>(a, blockIdx.x * kTile, (t - g.tiles[i]) * kTile, a.K / (16 * kWaves), red,
                         Ws);
}

template <int TB>
int launch(const GemmArgs& a, hipStream_t s) {
    const dim3 grid(ov3d_cdiv(a.M, kTile), a.N / kTile);
    switch (a.K / (16 * kWaves)) {
#define OV3D_RG(S) \
    case S: rows_gemm_kernel<TB, S><<<grid, 256, 0, s>>>(a); break;
        OV3D_RG(1) OV3D_RG(2) OV3D_RG(3) OV3D_RG(4) OV3D_RG(5) OV3D_RG(6) OV3D_RG(7) OV3D_RG(8)
        OV3D_RG(9) OV3D_RG(10) OV3D_RG(11) OV3D_RG(12) OV3D_RG(13) OV3D_RG(14) OV3D_RG(15)
        OV3D_RG(16)
#undef OV3D_RG
        default: return OV3D_EINVAL;
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

}  // namespace

extern "C" int ov3d_rows_gemm_supported(int M, int N, int K) {
    return M > 0 && N > 0 && N % kTile == 0 && K > 0 && K % (16 * kWaves) == 0 &&
           K / (16 * kWaves) <= kMaxSteps;
}

extern "C" int ov3d_rows_gemm_act(int M, int N, int K, const void* A, long long lda, const void* W,
                                  long long ldw, int trans_b, const void* bias, int epilogue,
                                  float dropout_p, const int64_t* seed, int site, const void* H,
                                  long long ldh, void* C, long long ldc, void* stream) {
    if (!ov3d_rows_gemm_supported(M, N, K) || !A || !W || !C) return OV3D_EINVAL;
    // 16-byte operand loads, 8-byte output stores
    if (((uintptr_t)A | (uintptr_t)W) % 16 || (uintptr_t)C % 8 || (bias && (uintptr_t)bias % 2) ||
        lda % 8 || ldw % 8 || ldc % 4 || lda < K || ldc < N || ldw < (trans_b ? K : N))
        return OV3D_EINVAL;
    if (epilogue < EPI_NONE || epilogue > EPI_MASK || dropout_p < 0.f || dropout_p >= 1.f)
        return OV3D_EINVAL;
    if (epilogue == EPI_RELU_DROP && dropout_p > 0.f && !seed) return OV3D_EINVAL;
    if (epilogue == EPI_MASK && (!H || (uintptr_t)H % 8 || ldh % 4 || ldh < N)) return OV3D_EINVAL;
    GemmArgs a{(const bf16*)A, lda, (const bf16*)W, ldw, (const bf16*)bias, (bf16*)C, ldc, M, N, K,
               epilogue, epilogue == EPI_RELU_DROP ? rowdrop::thresh(dropout_p) : 0u,
               1.f / (1.f - dropout_p), seed, (uint32_t)site, (const bf16*)H, ldh};
    hipStream_t s = ov3d_stream(stream);
    return trans_b ? launch<1>(a, s) : launch<0>(a, s);
}

extern "C" int ov3d_rows_gemm(int M, int N, int K, const void* A, long long lda, const void* W,
                              long long ldw, int trans_b, const void* bias, void* C, long long ldc,
                              void* stream) {
    return ov3d_rows_gemm_act(M, N, K, A, lda, W, ldw, trans_b, bias, EPI_NONE, 0.f, nullptr, 0,
                              nullptr, 0, C, ldc, stream);
}

namespace {
template <int TB>
int launch_group(const GemmGroup& g, int M, int steps, hipStream_t s) {
    const dim3 grid(ov3d_cdiv(M, kTile), g.tiles[g.n]);
    switch (steps <= 4 ? 4 : steps <= 8 ? 8 : steps <= 12 ? 12 : 16) {
        case 4: rows_gemm_group_kernel<TB, 4><<<grid, 256, 0, s>>>(g); break;
        case 8: rows_gemm_group_kernel<TB, 8><<<grid, 256, 0, s>>>(g); break;
        case 12: rows_gemm_group_kernel<TB, 12><<<grid, 256, 0, s>>>(g); break;
        default: rows_gemm_group_kernel<TB, 16><<<grid, 256, 0, s>>>(g); break;
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
}  // namespace

extern "C" int ov3d_rows_gemm_group(int M, int n, const ov3d_rows_gemm_problem* probs, int trans_b,
                                    void* stream) {
    if (M <= 0 || n <= 0 || n > kGroupProbs || !probs) return OV3D_EINVAL;
    GemmGroup g;
    g.n = n;
    g.tiles[0] = 0;
    int steps = 1;
    for (int i = 0; i < n; ++i) {
        const ov3d_rows_gemm_problem& q = probs[i];
        if (!ov3d_rows_gemm_supported(M, q.N, q.K) || !q.A || !q.W || !q.C) return OV3D_EINVAL;
        if (((uintptr_t)q.A | (uintptr_t)q.W) % 16 || (uintptr_t)q.C % 8 ||
            (q.bias && (uintptr_t)q.bias % 2) || q.lda % 8 || q.ldw % 8 || q.ldc % 4 ||
            q.lda < q.K || q.ldc < q.N || q.ldw < (trans_b ? q.K : q.N))
            return OV3D_EINVAL;
        g.p[i] = GemmArgs{(const bf16*)q.A, q.lda, (const bf16*)q.W, q.ldw, (const bf16*)q.bias,
                          (bf16*)q.C, q.ldc, M, q.N, q.K, EPI_NONE, 0u, 1.f, nullptr, 0u,
                          nullptr, 0};
        g.tiles[i + 1] = g.tiles[i] + q.N / kTile;
        steps = max(steps, q.K / (16 * kWaves));
    }
    hipStream_t s = ov3d_stream(stream);
    return trans_b ? launch_group<1>(g, M, steps, s) : launch_group<0>(g, M, steps, s);
}
