// Long row-block GEMMs: the 3DETR encoder's linear layers (M = B * 2048 = 16384 rows of
// 128 / 256 / 768 features, models/transformer.py:262-278 TransformerEncoderLayer
// forward_pre: in-projection, out-projection, linear1, linear2) forward and input gradient,
// the decoder's memory K/V projections (N = 8 layers x 256) and the heads' 8192-row layers.
//
//   trans_b = 1 (nn.Linear forward): C (M x N) = A (M x K) W^T + bias, W (N x K) row-major
//   trans_b = 0 (input gradient):    C (M x N) = A (M x K) W,          W (K x N) row-major
//
// bf16 operands, fp32 accumulation, bf16 output (bias added in fp32 before the one rounding).
// These shapes are HBM-bound (K <= 256: 2 flop per byte of A), so the kernel is laid out for
// the memory path, not for MFMA reuse:
//   * one workgroup = 4 waves = a BM x 128 output tile (BM = 128, or 64 when the grid would
//     otherwise not put two workgroups on every CU); waves 2 x 2, each (BM/2) x 64;
//   * K in 64-deep chunks; both operand chunks staged in LDS (double buffer), the next
//     chunk's 16-byte global loads in flight while the current one is multiplied;
//   * XCD-aware tile order: the column tiles of one row block run on one XCD (consecutive
//     slots of the same hardware queue), so A comes from HBM into that XCD's L2 once;
//   * the MFMA takes the W fragment as its first operand: a lane holds one output row and
//     4 consecutive columns per 4 accumulators, packed to bf16 into an LDS image of the
//     tile, which the workgroup stores as whole 256-byte row pieces (16 bytes a lane).
// trans_b = 1: W chunk stored [n][k], read with ds_read_b128; trans_b = 0: stored [k][n],
// read transposed with ds_read_b64_tr_b16 (k order 16s + 8(j>>2) + 4h + (j&3), and A's
// fragment is read in that order: two 8-byte pieces).
// Epilogues (ov3d_tile_gemm_act, as ov3d_rows_gemm_act for the short row blocks) fuse the
// encoder FFN's activation (models/transformer.py:276-278: linear1 -> ReLU -> dropout):
//   EPI_RELU_DROP: out = dropout(relu(bf16(acc + bias)))   (the rowdrop.h keep hash)
//   EPI_MASK:      out = h > 0 ? bf16(bf16(acc) / (1 - p)) : 0   (linear2's input gradient
//                  through that activation, h = the activation output)
#include "common.h"
#include "rowdrop.h"

#include <stdlib.h>

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int BN = 128, BK = 64;
constexpr int KALIGN = BK;
enum { EPI_NONE = 0, EPI_RELU_DROP = 1, EPI_MASK = 2 };

struct TileArgs {
    const bf16* A;
    long long lda;
    const bf16* W;
    long long ldw;
    const bf16* bias;
    bf16* C;
    long long ldc;
    int M, N, K;
    int epi; uint32_t thresh; float keep_scale; const int64_t* seed; uint32_t site;
    const bf16* H; long long ldh;   // EPI_MASK: the activation output
    // a second product summed into the same accumulators (ov3d_tile_gemm2): K chunks past
    // K come from (A2, W2), K2 deep; K2 = 0 for one product
    const bf16* A2; long long lda2;
    const bf16* W2; long long ldw2;
    int K2;
    // batched products (ov3d_tile_gemm_batched): grid.y = batch, element strides per batch
    long long sA, sW, sC;
};

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x4 tr16(const bf16* p) {
    s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
    return __builtin_bit_cast(bf16x4, r);
}

template <int TB, int BM>
struct Tile {
    // LDS images (bf16 elements): A [m][k] (trans_b = 0: 136-byte rows so the two 8-byte
    // fragment reads of a half-wave hit 64 distinct banks; 144-byte rows for the b128 reads),
    // W [n][k] (trans_b = 1) or [k][n] (trans_b = 0)
    static constexpr int LDA = TB ? BK + 8 : BK + 4;
    static constexpr int LDW = TB ? BK + 8 : BN + 8;
    static constexpr int ASZ = BM * LDA;
    static constexpr int WSZ = TB ? BN * LDW : BK * LDW;
    static constexpr int BUF = ASZ + WSZ;
    static constexpr int LDC = BN + 8;               // epilogue image, 272-byte rows
    static constexpr int NA = BM * BK / 8 / 256;     // 16-byte A pieces per thread per chunk
    static constexpr int NW = BN * BK / 8 / 256;     // 16-byte W pieces per thread per chunk
    static constexpr int MT = BM / 64;               // 32-row MFMA tiles per wave
    static constexpr int SMEM = 2 * BUF > BM * LDC ? 2 * BUF : BM * LDC;
    static_assert(NA >= 1 && NW >= 1 && MT >= 1, "tile shape");
    static_assert(SMEM * 2 <= 80 * 1024, "two workgroups per CU");
};

template <int TB, int BM>
__global__ __launch_bounds__(256, 2) void tile_gemm_kernel(TileArgs p) {
    using T = Tile<TB, BM>;
    __shared__ __attribute__((aligned(16))) bf16 smem[T::SMEM];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r32 = lane & 31, h = lane >> 5;
    const int wm = wave >> 1, wn = wave & 1;

    // XCD-aware order: hardware workgroup b runs on XCD b % 8; logical tile L (row block
    // L / nct, column tile L % nct) goes to XCD L / (ntiles / 8)
    const int nct = p.N / BN, ntiles = nct * ((p.M + BM - 1) / BM);
    const int b = blockIdx.x;
    const int L = (ntiles & 7) ? b : (b & 7) * (ntiles >> 3) + (b >> 3);
    const int m0 = (L / nct) * BM, n0 = (L % nct) * BN;
    const bf16* const Ab = p.A + blockIdx.y * p.sA;
    const bf16* const Wb = p.W + blockIdx.y * p.sW;
    bf16* const Cb = p.C + blockIdx.y * p.sC;

    f32x16 acc[T::MT][2];
#pragma unroll
    for (int mt = 0; mt < T::MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[mt][nt][i] = 0.f;

    bf16x8 ra[T::NA], rw[T::NW];
    auto load = [&](int kc) {
        const bool second = kc >= p.K;   // uniform
        const bf16* Ap = second ? p.A2 : Ab;
        const bf16* Wp = second ? p.W2 : Wb;
        const long long lda = second ? p.lda2 : p.lda, ldw = second ? p.ldw2 : p.ldw;
        if (second) kc -= p.K;
#pragma unroll
        for (int j = 0; j < T::NA; ++j) {
            const int idx = tid + 256 * j, r = idx >> 3, pc = idx & 7;
            const int row = min(m0 + r, p.M - 1);   // rows past M load the last row
            ra[j] = *reinterpret_cast<const bf16x8*>(Ap + (size_t)row * lda + kc + 8 * pc);
        }
#pragma unroll
        for (int j = 0; j < T::NW; ++j) {
            const int idx = tid + 256 * j;
            if (TB)
                rw[j] = *reinterpret_cast<const bf16x8*>(Wp + (size_t)(n0 + (idx >> 3)) * ldw + kc +
                                                         8 * (idx & 7));
            else
                rw[j] = *reinterpret_cast<const bf16x8*>(Wp + (size_t)(kc + (idx >> 4)) * ldw + n0 +
                                                         8 * (idx & 15));
        }
    };
    auto store = [&](int buf) {
        bf16* As = smem + buf * T::BUF;
        bf16* Ws = As + T::ASZ;
#pragma unroll
        for (int j = 0; j < T::NA; ++j) {
            const int idx = tid + 256 * j, r = idx >> 3, pc = idx & 7;
            if (TB) {
                *reinterpret_cast<bf16x8*>(&As[r * T::LDA + 8 * pc]) = ra[j];
            } else {   // 136-byte rows: 8-byte aligned only
                *reinterpret_cast<bf16x4*>(&As[r * T::LDA + 8 * pc]) =
                    bf16x4{ra[j][0], ra[j][1], ra[j][2], ra[j][3]};
                *reinterpret_cast<bf16x4*>(&As[r * T::LDA + 8 * pc + 4]) =
                    bf16x4{ra[j][4], ra[j][5], ra[j][6], ra[j][7]};
            }
        }
#pragma unroll
        for (int j = 0; j < T::NW; ++j) {
            const int idx = tid + 256 * j;
            if (TB)
                *reinterpret_cast<bf16x8*>(&Ws[(idx >> 3) * T::LDW + 8 * (idx & 7)]) = rw[j];
            else
                *reinterpret_cast<bf16x8*>(&Ws[(idx >> 4) * T::LDW + 8 * (idx & 15)]) = rw[j];
        }
    };
    auto compute = [&](int buf) {
        const bf16* As = smem + buf * T::BUF;
        const bf16* Ws = As + T::ASZ;
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
            bf16x8 af[T::MT], wf[2];
#pragma unroll
            for (int mt = 0; mt < T::MT; ++mt) {
                const bf16* ar = As + (wm * (BM / 2) + 32 * mt + r32) * T::LDA + 16 * s;
                if (TB) {
                    af[mt] = *reinterpret_cast<const bf16x8*>(ar + 8 * h);
                } else {
                    const bf16x4 lo = *reinterpret_cast<const bf16x4*>(ar + 4 * h);
                    const bf16x4 hi = *reinterpret_cast<const bf16x4*>(ar + 8 + 4 * h);
                    af[mt] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
            }
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                if (TB) {
                    wf[nt] = *reinterpret_cast<const bf16x8*>(
                        &Ws[(wn * 64 + 32 * nt + r32) * T::LDW + 16 * s + 8 * h]);
                } else {
                    const int g = lane >> 4, i = lane & 15;
                    const int d0 = wn * 64 + 32 * nt + 16 * (g & 1) + 4 * (i & 3);
                    const int k0 = 16 * s + 4 * (g >> 1) + (i >> 2);
                    const bf16x4 lo = tr16(&Ws[k0 * T::LDW + d0]);
                    const bf16x4 hi = tr16(&Ws[(k0 + 8) * T::LDW + d0]);
                    wf[nt] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
            }
#pragma unroll
            for (int mt = 0; mt < T::MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma(wf[nt], af[mt], acc[mt][nt]);
        }
    };

    const int nk = (p.K + p.K2) / BK;
    load(0);
    store(0);
    __syncthreads();
    for (int c = 0; c < nk; ++c) {
        if (c + 1 < nk) load((c + 1) * BK);   // in flight under this chunk's MFMAs
        compute(c & 1);
        if (c + 1 < nk) store((c + 1) & 1);   // that buffer was last read before the previous barrier
        __syncthreads();
    }

    // epilogue: acc[mt][nt][v] of lane l is C[row r32][col 8(v>>2) + 4h + (v&3)] of the
    // wave's (mt, nt) 32 x 32 tile; bias in fp32, one bf16 rounding, through the LDS image
    bf16* Cs = smem;
    const uint32_t smix = (p.epi == EPI_RELU_DROP && p.thresh) ? rowdrop::seed_mix(p.seed, p.site) : 0u;
    uint32_t rbase[T::MT];
#pragma unroll
    for (int mt = 0; mt < T::MT; ++mt)
        rbase[mt] = smix ? rowdrop::row_base(smix, m0 + wm * (BM / 2) + 32 * mt + r32) : 0u;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int col = wn * 64 + 32 * nt + 8 * g + 4 * h;
            float bv[4] = {0.f, 0.f, 0.f, 0.f};
            if (p.bias) {
                const bf16x4 bb = *reinterpret_cast<const bf16x4*>(p.bias + n0 + col);
#pragma unroll
                for (int q = 0; q < 4; ++q) bv[q] = (float)bb[q];
            }
#pragma unroll
            for (int mt = 0; mt < T::MT; ++mt) {
                const int row = wm * (BM / 2) + 32 * mt + r32;
                bf16x4 o;
#pragma unroll
                for (int q = 0; q < 4; ++q) o[q] = (bf16)(acc[mt][nt][4 * g + q] + bv[q]);
                if (p.epi == EPI_RELU_DROP) {
                    bool keep[4] = {true, true, true, true};
                    if (smix) {   // one hash per channel pair (rowdrop.h keep8's pairs)
#pragma unroll
                        for (int j = 0; j < 4; j += 2) {
                            const uint32_t hs =
                                rowdrop::mix24(rbase[mt] + (uint32_t)((n0 + col + j) >> 1) * 0x27D4EB2Fu);
                            keep[j] = (hs & 0xffffu) >= p.thresh;
                            keep[j + 1] = (hs >> 16) >= p.thresh;
                        }
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float rr = fmaxf((float)o[q], 0.f);
                        o[q] = smix ? (keep[q] ? (bf16)(rr * p.keep_scale) : (bf16)0.f) : (bf16)rr;
                    }
                } else if (p.epi == EPI_MASK) {
                    const int gr = min(m0 + row, p.M - 1);
                    const bf16x4 hv = *reinterpret_cast<const bf16x4*>(p.H + (size_t)gr * p.ldh + n0 + col);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        o[q] = (float)hv[q] > 0.f ? (bf16)((float)o[q] * p.keep_scale) : (bf16)0.f;
                }
                *reinterpret_cast<bf16x4*>(&Cs[row * T::LDC + col]) = o;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < BM * BN / 8 / 256; ++j) {
        const int idx = tid + 256 * j, r = idx >> 4, pc = idx & 15;
        if (m0 + r < p.M)
            *reinterpret_cast<bf16x8*>(Cb + (size_t)(m0 + r) * p.ldc + n0 + 8 * pc) =
                *reinterpret_cast<const bf16x8*>(&Cs[r * T::LDC + 8 * pc]);
    }
}

// BM = 128 unless that leaves fewer than two workgroups per CU (OV3D_TILE_GEMM_BM overrides)
int pick_bm(int M, int N) {
    const char* e = getenv("OV3D_TILE_GEMM_BM");
    if (e) return atoi(e) == 64 ? 64 : 128;
    return (long long)ov3d_cdiv(M, 128) * (N / BN) >= 512 ? 128 : 64;
}

template <int TB>
void launch(const TileArgs& a, hipStream_t s, int batch = 1) {
    if (pick_bm(a.M, a.N * batch) == 128)
        tile_gemm_kernel<TB, 128><<<dim3(ov3d_cdiv(a.M, 128) * (a.N / BN), batch), 256, 0, s>>>(a);
    else
        tile_gemm_kernel<TB, 64><<<dim3(ov3d_cdiv(a.M, 64) * (a.N / BN), batch), 256, 0, s>>>(a);
}

}  // namespace

extern "C" int ov3d_tile_gemm_supported(int M, int N, int K) {
    return M > 0 && N > 0 && N % BN == 0 && K > 0 && K % KALIGN == 0;
}

extern "C" int ov3d_tile_gemm_act(int M, int N, int K, const void* A, long long lda, const void* W,
                                  long long ldw, int trans_b, const void* bias, int epilogue,
                                  float dropout_p, const int64_t* seed, int site, const void* H,
                                  long long ldh, void* C, long long ldc, void* stream) {
    if (!ov3d_tile_gemm_supported(M, N, K) || !A || !W || !C) return OV3D_EINVAL;
    if (epilogue < EPI_NONE || epilogue > EPI_MASK || dropout_p < 0.f || dropout_p >= 1.f)
        return OV3D_EINVAL;
    if (epilogue == EPI_RELU_DROP && dropout_p > 0.f && !seed) return OV3D_EINVAL;
    if (epilogue == EPI_MASK && (!H || (uintptr_t)H % 8 || ldh % 4 || ldh < N)) return OV3D_EINVAL;
    // 16-byte A / W / C pieces, 8-byte bias pieces
    if (((uintptr_t)A | (uintptr_t)W | (uintptr_t)C) % 16 || (bias && (uintptr_t)bias % 8) ||
        lda % 8 || ldw % 8 || ldc % 8 || lda < K || ldc < N || ldw < (trans_b ? K : N))
        return OV3D_EINVAL;
    if ((long long)M * (N / BN) > (1LL << 31) / 2 || (long long)M > (1LL << 31) / 2)
        return OV3D_EINVAL;
    TileArgs a{(const bf16*)A, lda, (const bf16*)W, ldw, (const bf16*)bias, (bf16*)C, ldc, M, N, K,
               epilogue, epilogue == EPI_RELU_DROP ? rowdrop::thresh(dropout_p) : 0u,
               1.f / (1.f - dropout_p), seed, (uint32_t)site, (const bf16*)H, ldh,
               nullptr, 0, nullptr, 0, 0, 0, 0, 0};
    hipStream_t s = ov3d_stream(stream);
    if (trans_b)
        launch<1>(a, s);
    else
        launch<0>(a, s);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_tile_gemm(int M, int N, int K, const void* A, long long lda, const void* W,
                              long long ldw, int trans_b, const void* bias, void* C, long long ldc,
                              void* stream) {
    return ov3d_tile_gemm_act(M, N, K, A, lda, W, ldw, trans_b, bias, EPI_NONE, 0.f, nullptr, 0,
                              nullptr, 0, C, ldc, stream);
}

extern "C" int ov3d_tile_gemm2(int M, int N, int K1, const void* A1, long long lda1, const void* W1,
                               long long ldw1, int K2, const void* A2, long long lda2,
                               const void* W2, long long ldw2, int trans_b, void* C, long long ldc,
                               void* stream) {
    if (!ov3d_tile_gemm_supported(M, N, K1) || !ov3d_tile_gemm_supported(M, N, K2) || !A1 || !W1 ||
        !A2 || !W2 || !C)
        return OV3D_EINVAL;
    if (((uintptr_t)A1 | (uintptr_t)W1 | (uintptr_t)A2 | (uintptr_t)W2 | (uintptr_t)C) % 16 ||
        lda1 % 8 || ldw1 % 8 || lda2 % 8 || ldw2 % 8 || ldc % 8 || lda1 < K1 || lda2 < K2 ||
        ldc < N || ldw1 < (trans_b ? K1 : N) || ldw2 < (trans_b ? K2 : N))
        return OV3D_EINVAL;
    if ((long long)M * (N / BN) > (1LL << 31) / 2 || (long long)M > (1LL << 31) / 2 ||
        (long long)K1 + K2 > (1LL << 30))
        return OV3D_EINVAL;
    TileArgs a{(const bf16*)A1, lda1, (const bf16*)W1, ldw1, nullptr, (bf16*)C, ldc, M, N, K1,
               EPI_NONE, 0u, 1.f, nullptr, 0u, nullptr, 0,
               (const bf16*)A2, lda2, (const bf16*)W2, ldw2, K2, 0, 0, 0};
    hipStream_t s = ov3d_stream(stream);
    if (trans_b)
        launch<1>(a, s);
    else
        launch<0>(a, s);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_tile_gemm_batched(int batch, int M, int N, int K, const void* A, long long lda,
                                      long long sA, const void* W, long long ldw, long long sW,
                                      int trans_b, void* C, long long ldc, long long sC,
                                      void* stream) {
    if (!ov3d_tile_gemm_supported(M, N, K) || batch <= 0 || batch > 65535 || !A || !W || !C)
        return OV3D_EINVAL;
    if (((uintptr_t)A | (uintptr_t)W | (uintptr_t)C) % 16 || lda % 8 || ldw % 8 || ldc % 8 ||
        sA % 8 || sW % 8 || sC % 8 || lda < K || ldc < N || ldw < (trans_b ? K : N) || sA < 0 ||
        sW < 0 || sC < (long long)M * ldc)
        return OV3D_EINVAL;
    if ((long long)M * (N / BN) > (1LL << 31) / 2 || (long long)M > (1LL << 31) / 2)
        return OV3D_EINVAL;
    TileArgs a{(const bf16*)A, lda, (const bf16*)W, ldw, nullptr, (bf16*)C, ldc, M, N, K,
               EPI_NONE, 0u, 1.f, nullptr, 0u, nullptr, 0, nullptr, 0, nullptr, 0, 0, sA, sW, sC};
    hipStream_t s = ov3d_stream(stream);
    if (trans_b)
        launch<1>(a, s, batch);
    else
        launch<0>(a, s, batch);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
