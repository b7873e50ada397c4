// Long row-block GEMMs: the 3DETR encoder's linear layers (M = B * 2048 = 16384 rows of
// 128 / 256 / 768 features, models/transformer.py:262-278 TransformerEncoderLayer
// forward_pre: in-projection, out-projection, linear1, linear2) forward and input gradient,
// where the library GEMM (hipBLASLt, 15-17 us per call whatever N) runs far below both the
// HBM and the MFMA roofline for K <= 256.
//
//   trans_b = 1 (nn.Linear forward): C (M x N) = A (M x K) W^T + bias, W (N x K) row-major
//   trans_b = 0 (input gradient):    C (M x N) = A (M x K) W,          W (K x N) row-major
//
// bf16 operands, fp32 accumulation, bf16 output (bias added in fp32 before the rounding).
// One workgroup = 4 waves = a 128-row x 128-column output tile; wave w owns rows 32w..32w+31
// and all 128 columns (4 MFMA 32x32x16 accumulators).  The K range goes in chunks of
// BK = 256 (128, 64 when K is not a multiple), all of a chunk's loads issued before the first
// wait (K <= 256: one memory round trip per workgroup):
//   * the W chunk (128 columns x BK) is staged in LDS once per workgroup and shared by the
//     4 waves (W is re-read from L2 once per 128 rows, not once per 32);
//   * a wave's A fragments come straight from global memory into the MFMA layout (each row
//     is read by exactly one wave);
//   * trans_b = 1: the W chunk is stored [n][k] and read with ds_read_b128 (k-contiguous);
//     trans_b = 0: stored [k][n] and read transposed with ds_read_b64_tr_b16; A's fragment
//     is then loaded in the same k order (16s + 8(j>>2) + 4h + (j&3)).
// Accumulator element v of lane l is C[32w + 8(v>>2) + 4(l>>5) + (v&3)][32ct + (l&31)].
#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128;
constexpr int KALIGN = 64;      // K granularity (the chunk depth BK is 64, 128 or 256)

struct TileArgs {
    const bf16* A;
    long long lda;
    const bf16* W;
    long long ldw;
    const bf16* bias;
    bf16* C;
    long long ldc;
    int M, N, K;
};

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x4 tr16(const bf16* p) {
    s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
    return __builtin_bit_cast(bf16x4, r);
}

template <int TB, int BK>
__global__ __launch_bounds__(256, 2) void tile_gemm_kernel(TileArgs p) {
    constexpr int LDW1 = BK + 8;    // trans_b = 1: Ws[n][k]
    constexpr int LDW0 = BN + 8;    // trans_b = 0: Ws[k][n], 272-byte rows
    constexpr int WSZ = TB ? BN * LDW1 : BK * LDW0;
    constexpr int NW = BN * BK / 8 / 256;   // 16-byte W pieces per thread per chunk
    constexpr int KS = BK / 16;             // k-steps per chunk
    __shared__ __attribute__((aligned(16))) bf16 Ws[WSZ];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r32 = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const int row = min(m0 + 32 * wave + r32, p.M - 1);   // rows past M load the last row
    const bf16* arow = p.A + (size_t)row * p.lda;

    f32x16 acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[ct][i] = 0.f;

    for (int kc = 0; kc < p.K; kc += BK) {
        // every load of the chunk is issued before the first wait: one memory round trip
        bf16x8 wr[NW], af[KS];
#pragma unroll
        for (int c = 0; c < NW; ++c) {
            const int idx = tid + 256 * c;
            if (TB)   // row n = idx / (BK/8), k piece idx % (BK/8)
                wr[c] = *reinterpret_cast<const bf16x8*>(p.W + (size_t)(n0 + idx / (BK / 8)) * p.ldw + kc +
                                                         8 * (idx % (BK / 8)));
            else      // row k = idx >> 4, n piece idx & 15
                wr[c] = *reinterpret_cast<const bf16x8*>(p.W + (size_t)(kc + (idx >> 4)) * p.ldw + n0 +
                                                         8 * (idx & 15));
        }
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (TB) {
                af[s] = *reinterpret_cast<const bf16x8*>(arow + kc + 16 * s + 8 * h);
            } else {
                const bf16x4 lo = *reinterpret_cast<const bf16x4*>(arow + kc + 16 * s + 4 * h);
                const bf16x4 hi = *reinterpret_cast<const bf16x4*>(arow + kc + 16 * s + 8 + 4 * h);
                af[s] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            }
        }
        if (kc) __syncthreads();   // the previous chunk's LDS reads are done
#pragma unroll
        for (int c = 0; c < NW; ++c) {
            const int idx = tid + 256 * c;
            if (TB)
                *reinterpret_cast<bf16x8*>(&Ws[(idx / (BK / 8)) * LDW1 + 8 * (idx % (BK / 8))]) = wr[c];
            else
                *reinterpret_cast<bf16x8*>(&Ws[(idx >> 4) * LDW0 + 8 * (idx & 15)]) = wr[c];
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            bf16x8 bfr[4];
#pragma unroll
            for (int ct = 0; ct < 4; ++ct) {
                if (TB) {
                    bfr[ct] = *reinterpret_cast<const bf16x8*>(&Ws[(32 * ct + r32) * LDW1 + 16 * s + 8 * h]);
                } else {
                    const int g = lane >> 4, i = lane & 15;
                    const int d0 = 32 * ct + 16 * (g & 1) + 4 * (i & 3);
                    const int k0 = 16 * s + 4 * (g >> 1) + (i >> 2);
                    const bf16x4 lo = tr16(&Ws[k0 * LDW0 + d0]);
                    const bf16x4 hi = tr16(&Ws[(k0 + 8) * LDW0 + d0]);
                    bfr[ct] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
            }
#pragma unroll
            for (int ct = 0; ct < 4; ++ct) acc[ct] = mfma(af[s], bfr[ct], acc[ct]);
        }
    }

    // epilogue: bias in fp32, one bf16 rounding; lanes of a row write 32 adjacent columns
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
        const int n = n0 + 32 * ct + r32;
        const float bv = p.bias ? (float)p.bias[n] : 0.f;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int m = m0 + 32 * wave + 8 * (v >> 2) + 4 * h + (v & 3);
            if (m < p.M) p.C[(size_t)m * p.ldc + n] = (bf16)(acc[ct][v] + bv);
        }
    }
}

template <int TB>
void launch(const TileArgs& a, hipStream_t s) {
    const dim3 grid(ov3d_cdiv(a.M, BM), a.N / BN);
    if (a.K % 256 == 0)
        tile_gemm_kernel<TB, 256><<<grid, 256, 0, s>>>(a);
    else if (a.K % 128 == 0)
        tile_gemm_kernel<TB, 128><<<grid, 256, 0, s>>>(a);
    else
        tile_gemm_kernel<TB, 64><<<grid, 256, 0, s>>>(a);
}

}  // namespace

extern "C" int ov3d_tile_gemm_supported(int M, int N, int K) {
    return M > 0 && N > 0 && N % BN == 0 && K > 0 && K % KALIGN == 0;
}

extern "C" int ov3d_tile_gemm(int M, int N, int K, const void* A, long long lda, const void* W,
                              long long ldw, int trans_b, const void* bias, void* C, long long ldc,
                              void* stream) {
    if (!ov3d_tile_gemm_supported(M, N, K) || !A || !W || !C) return OV3D_EINVAL;
    // 16-byte W / A loads (8-byte A pieces for trans_b = 0), 2-byte output stores
    if (((uintptr_t)A | (uintptr_t)W) % 16 || (uintptr_t)C % 2 || (bias && (uintptr_t)bias % 2) ||
        lda % 8 || ldw % 8 || lda < K || ldc < N || ldw < (trans_b ? K : N))
        return OV3D_EINVAL;
    if ((long long)M > (1LL << 31) / 2) return OV3D_EINVAL;
    TileArgs a{(const bf16*)A, lda, (const bf16*)W, ldw, (const bf16*)bias, (bf16*)C, ldc, M, N, K};
    hipStream_t s = ov3d_stream(stream);
    if (trans_b)
        launch<1>(a, s);
    else
        launch<0>(a, s);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
