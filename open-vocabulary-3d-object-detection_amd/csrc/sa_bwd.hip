// Backward of the last SA MLP layer (the pooled one, model_3detr.py:353-362 pre-encoder
// SharedMLP layer 3: 1x1 conv 128 -> 256, BN, ReLU, max over nsample) in ONE pass over the
// R = B*M*S rows, replacing the dy recompute kernel + a dW GEMM + a dgrad GEMM that each
// streamed the (R, 256) bf16 dy3 through HBM (sa_dy_fused_kernel):
//
//   per 64-row tile (persistent workgroups, W3 fragments in VGPRs for the whole launch):
//     z   = relu(a2*y2 + b2)            (layer 2's folded BN, bf16)   -> LDS
//     y3  = z W3^T                      (MFMA 32x32x16, recomputed)
//     dy3 = cA*g + cB*y3 + cC           (BN backward of the pooled layer; g = the pooled
//                                        gradient at its arg row)     -> LDS (bf16), stored
//                                        transposed [n][row] (8-byte LDS stores)
//     dz^T = W3^T dy3^T                 (MFMA, W3^T fragments: a lane holds 4 consecutive
//                                        channels of a row -> 8-byte stores) -> HBM (R, 128)
//     dW3 += dy3^T z                    (MFMA on ds_read_b64_tr_b16 reads of both LDS tiles,
//                                        accumulated over the workgroup's tiles)
//   dW3 partials per workgroup (fixed order), summed by the caller.
//   With `stats`: also the previous layer's ReLU + BN backward partial sums over the rows,
//   sum dt and sum dt * xhat2 per channel, dt = (a2*y2 + b2 > 0) * bf16(dz) (the pass 0 of
//   bn_relu_bwd_kernel, whose read of dz and y2 it replaces).
// dy3 and z are never stored: the forward no longer writes z (2^20 x 128 bf16) either.
#include <stdlib.h>

#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 64;      // rows per tile (one centroid at S = 64, two at S = 32)
constexpr int kThreads = 256;  // 4 waves

struct DyFusedArgs {
    const bf16* yprev;     // (R, K) layer-2 output y2
    const float* scale;    // (K) layer-2 folded BN a2
    const float* shift;    // (K) b2
    const bf16* W;         // (N, K) W3
    int R, S;
    const float* gsel;     // (P, N) pooled gradient after the ReLU mask
    const uint8_t* isel;   // (P, N) row of the pooled value within its centroid
    const float* ysel;     // (P, N) the pooled y3 value (the forward's, at the isel row)
    const float* cA;       // (N) dy3 = cA*g + cB*y3 + cC
    const float* cB;
    const float* cC;
    bf16* dz;              // (R, K) gradient of z (layer-2 activation output)
    float* dwpart;         // (gridDim.x, N, K) dW3 partial per workgroup
    const float* mean;     // (K) layer-2 batch mean / invstd (with stats)
    const float* invstd;
    double* stats;         // (gridDim.x, 2, K) or null
};

#ifdef OV3D_SA_PROBE
// diagnostic build only (tools/sa_probe.py): per-wave s_memtime totals of the tile phases
__device__ unsigned long long* g_sa_probe;
#define PROBE_DECL unsigned long long pr_t = __builtin_amdgcn_s_memtime(), pr_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PROBE(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); pr_acc[i] += t_ - pr_t; pr_t = t_; } while (0)
#define PROBE_END do { if ((threadIdx.x & 63) == 0 && g_sa_probe) { \
    unsigned long long* o_ = g_sa_probe + ((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8; \
    for (int i_ = 0; i_ < 8; ++i_) o_[i_] = pr_acc[i_]; } } while (0)
#else
#define PROBE_DECL
#define PROBE(i) do { } while (0)
#define PROBE_END do { } while (0)
#endif

// buffer resource word 3 for gfx950 raw buffer loads (32-bit data format, no swizzle)
constexpr int kBufDword3 = 0x00020000;

// the lane index recomputed where it is used (volatile: not hoisted out of the loop, so no
// loop-invariant copy of it competes for registers)
__device__ __forceinline__ int lane_fresh() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x4 tr16(const bf16* p) {
    s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(p));
    return __builtin_bit_cast(bf16x4, r);
}

// MFMA operand whose lane index runs over the columns c0 .. c0+31 of a row-major LDS tile
// and whose 8 elements are rows 16s + 8(j>>2) + 4h + (j&3) (ds_read_b64_tr_b16; the two
// operands of one product use the same row order)
__device__ __forceinline__ bf16x8 col_operand(const bf16* T, int ld, int lane, int c0, int s) {
    const int g = lane >> 4, i = lane & 15;
    const int d0 = c0 + 16 * (g & 1) + 4 * (i & 3);
    const int k0 = 16 * s + 4 * (g >> 1) + (i >> 2);
    const bf16x4 lo = tr16(T + k0 * ld + d0);
    const bf16x4 hi = tr16(T + (k0 + 8) * ld + d0);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int K, int N, bool STATS>
__global__ __launch_bounds__(kThreads, 1) void sa_dy_fused_kernel(DyFusedArgs p) {
    constexpr int LDK = K + 8;        // padded LDS rows (bf16)
    constexpr int LDR = kTile + 8;    // DsT row: one channel n, the tile's 64 rows
    constexpr int NB = N / 128;       // y3: 32-column blocks per wave (a wave owns N/4 columns)
    constexpr int KS = K / 16;        // y3: k-steps
    constexpr int KB = K / 128;       // dz: 32-column blocks per wave (a wave owns K/4 columns)
    constexpr int NS = N / 16;        // dz: k-steps
    constexpr int WN = N / 128;       // dW: 32-row blocks per wave (a wave owns N/4 rows)
    constexpr int WK = K / 32;        // dW: 32-column blocks (all K)
    static_assert(N % 128 == 0 && K % 128 == 0, "tile shape");
    __shared__ __attribute__((aligned(16))) bf16 As[kTile * LDK];
    __shared__ __attribute__((aligned(16))) bf16 DsT[N * LDR];        // dy3 transposed
    __shared__ __attribute__((aligned(16))) bf16 Ys[STATS ? kTile * LDK : 8];   // raw y2 (stats)
    __shared__ float sc[K], sh[K], smu[K], sis[K];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r32 = lane & 31, h = lane >> 5;

    constexpr bool stats = STATS;
    for (int k = tid; k < K; k += kThreads) {
        sc[k] = p.scale[k];
        sh[k] = p.shift[k];
        smu[k] = stats ? p.mean[k] : 0.f;
        sis[k] = stats ? p.invstd[k] : 0.f;
    }
    // W3 fragments for y3 = z W3^T: lane row n, 8 consecutive k
    bf16x8 bfrag[NB][KS];
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) {
        const int n = wave * (N / 4) + cb * 32 + r32;
#pragma unroll
        for (int s = 0; s < KS; ++s)
            bfrag[cb][s] = *reinterpret_cast<const bf16x8*>(p.W + (size_t)n * K + 16 * s + 8 * h);
    }
    // W3^T fragments for dz^T = W3^T dy3^T: lane row k, 8 channels n in the row order of
    // col_operand (16s + 8(j>>2) + 4h + (j&3)); gathered once
    bf16x8 wt[KB][NS];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
        const int k = wave * (K / 4) + kb * 32 + r32;
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                wt[kb][s][j] = p.W[(size_t)(16 * s + 8 * (j >> 2) + 4 * h + (j & 3)) * K + k];
    }
    float cA[NB], cB[NB], cC[NB];
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) {
        const int n = wave * (N / 4) + cb * 32 + r32;
        cA[cb] = p.cA[n];
        cB[cb] = p.cB[n];
        cC[cb] = p.cC[n];
    }
    // stats: a lane's 16 channels kb*32 + 8g + 4h + j (g, j < 4), summed over its rows
    float st1[KB][STATS ? 16 : 1], st2[KB][STATS ? 16 : 1];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < (STATS ? 16 : 1); ++i) st1[kb][i] = st2[kb][i] = 0.f;
    f32x16 dw[WN][WK];
#pragma unroll
    for (int a = 0; a < WN; ++a)
#pragma unroll
        for (int b = 0; b < WK; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) dw[a][b][i] = 0.f;
    __syncthreads();

    const int ntiles = p.R / kTile;
    constexpr int CH = kTile * K / 8 / kThreads;
    static_assert(CH * kThreads * 8 == kTile * K, "tile chunks");
    bf16x8 pre[CH];
    auto fetch = [&](int tile) {
        const size_t row0 = (size_t)tile * kTile;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int ch = tid + c * kThreads;
            const int row = ch / (K / 8), kc = (ch % (K / 8)) * 8;
            pre[c] = *reinterpret_cast<const bf16x8*>(p.yprev + (row0 + row) * K + kc);
        }
    };
    if (blockIdx.x < ntiles) fetch(blockIdx.x);
    PROBE_DECL
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const size_t row0 = (size_t)tile * kTile;
        PROBE(0);
        // z = relu(a2*y2 + b2) of the prefetched rows -> LDS
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int ch = tid + c * kThreads;
            const int row = ch / (K / 8), kc = (ch % (K / 8)) * 8;
            bf16x8 z;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                z[j] = (bf16)fmaxf(fmaf(sc[kc + j], (float)pre[c][j], sh[kc + j]), 0.f);
            *reinterpret_cast<bf16x8*>(&As[row * LDK + kc]) = z;
            if constexpr (STATS) *reinterpret_cast<bf16x8*>(&Ys[row * LDK + kc]) = pre[c];
        }
        PROBE(1);
        __syncthreads();
        PROBE(2);
        if (tile + (int)gridDim.x < ntiles) fetch(tile + gridDim.x);   // in flight below

        // y3 = z W3^T, then dy3 -> LDS
        {
            f32x16 acc[2][NB];
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                for (int cb = 0; cb < NB; ++cb)
#pragma unroll
                    for (int i = 0; i < 16; ++i) acc[rb][cb][i] = 0.f;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
#pragma unroll
                for (int rb = 0; rb < 2; ++rb) {
                    const bf16x8 a = *reinterpret_cast<const bf16x8*>(&As[(rb * 32 + r32) * LDK + 16 * s + 8 * h]);
#pragma unroll
                    for (int cb = 0; cb < NB; ++cb) acc[rb][cb] = mfma(a, bfrag[cb][s], acc[rb][cb]);
                }
            }
#pragma unroll
            for (int cb = 0; cb < NB; ++cb) {
                const int n = wave * (N / 4) + cb * 32 + r32;
#pragma unroll
                for (int rb = 0; rb < 2; ++rb) {
                    const size_t pc = (p.S == 64 ? (size_t)tile : (size_t)tile * 2 + rb) * N + n;
                    const int sel = p.isel[pc] + (p.S == 64 ? 0 : 32 * rb);
                    const float g = p.gsel[pc];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {   // rows rb*32 + 8q + 4h + (0..3)
                        bf16x4 d4;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int row = rb * 32 + 8 * q + 4 * h + j;
                            const float y = (float)(bf16)acc[rb][cb][4 * q + j];
                            const float gi = row == sel ? g : 0.f;
                            d4[j] = (bf16)fmaf(cA[cb], gi, fmaf(cB[cb], y, cC[cb]));
                        }
                        *reinterpret_cast<bf16x4*>(&DsT[n * LDR + rb * 32 + 8 * q + 4 * h]) = d4;
                    }
                }
            }
        }
        PROBE(3);
        __syncthreads();
        PROBE(4);

        // dz^T = W3^T dy3^T -> HBM: lane = row rb*32 + r32, channels kbase + 8g + 4h + (0..3)
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            const int kbase = wave * (K / 4) + kb * 32;
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
                f32x16 acc;
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
                for (int s = 0; s < NS; ++s)
                    acc = mfma(wt[kb][s], col_operand(DsT, LDR, lane, rb * 32, s), acc);
                const int row = rb * 32 + r32;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int k = kbase + 8 * g + 4 * h;
                    bf16x4 o;
#pragma unroll
                    for (int j = 0; j < 4; ++j) o[j] = (bf16)acc[4 * g + j];
                    *reinterpret_cast<bf16x4*>(p.dz + (row0 + row) * K + k) = o;
                    if constexpr (STATS) {   // bn_relu_bwd pass 0 on the stored values
                        const bf16x4 y4 = *reinterpret_cast<const bf16x4*>(&Ys[row * LDK + k]);
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float yy = (float)y4[j];
                            const float dt = fmaf(sc[k + j], yy, sh[k + j]) > 0.f ? (float)o[j] : 0.f;
                            st1[kb][4 * g + j] += dt;
                            st2[kb][4 * g + j] = fmaf(dt, (yy - smu[k + j]) * sis[k + j],
                                                      st2[kb][4 * g + j]);
                        }
                    }
                }
            }
        }
        PROBE(5);
        // dW3 += dy3^T z over this tile's rows
#pragma unroll
        for (int s = 0; s < kTile / 16; ++s) {
            bf16x8 bz[WK];
#pragma unroll
            for (int b = 0; b < WK; ++b) bz[b] = col_operand(As, LDK, lane, 32 * b, s);
#pragma unroll
            for (int a = 0; a < WN; ++a) {
                // dy3^T rows of channel n, rows in col_operand's order
                const bf16* dn = DsT + (wave * (N / 4) + 32 * a + r32) * LDR + 16 * s + 4 * h;
                const bf16x4 lo = *reinterpret_cast<const bf16x4*>(dn);
                const bf16x4 hi = *reinterpret_cast<const bf16x4*>(dn + 8);
                const bf16x8 ad = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
                for (int b = 0; b < WK; ++b) dw[a][b] = mfma(ad, bz[b], dw[a][b]);
            }
        }
        PROBE(6);
        __syncthreads();   // As / Ds are rewritten by the next tile
        PROBE(7);
    }
    PROBE_END;
    if constexpr (STATS) {   // sum each channel over the 32 lanes (rows) of its lane half
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                double s1 = (double)st1[kb][i], s2 = (double)st2[kb][i];
#pragma unroll
                for (int o = 16; o > 0; o >>= 1) {
                    s1 += __shfl_xor(s1, o, 64);
                    s2 += __shfl_xor(s2, o, 64);
                }
                if (r32 == 0) {
                    const int k = wave * (K / 4) + kb * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
                    p.stats[(size_t)blockIdx.x * 2 * K + k] = s1;
                    p.stats[(size_t)blockIdx.x * 2 * K + K + k] = s2;
                }
            }
    }
    // this workgroup's dW3 partial: element (a, b, i) = dW[n][k],
    // n = wave*(N/4) + 32a + (i&3) + 8(i>>2) + 4h, k = 32b + r32
    float* out = p.dwpart + (size_t)blockIdx.x * N * K;
#pragma unroll
    for (int a = 0; a < WN; ++a)
#pragma unroll
        for (int b = 0; b < WK; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int n = wave * (N / 4) + 32 * a + (i & 3) + 8 * (i >> 2) + 4 * h;
                out[(size_t)n * K + 32 * b + r32] = dw[a][b][i];
            }
}

// sa_dy9's LDS images.  Rows / lines are unpadded and XOR-swizzled in 16- or 8-byte pieces, so
// that every access below is free of bank conflicts (MI355X_MICROARCH.md §LDS lane groups;
// tools/lds_banks_dy9.py enumerates them):
//   As  (z: 64 rows x 128 k): 16-byte piece c of row r at c ^ zsw(r).  Read row-wise by the y3 A
//       operand (ds_read_b128, lanes = rows) and transposed by the dW3 B operand
//       (ds_read_b64_tr_b16 over 4 rows x 16 k): one image serves both (round 4's sa_dy8 kept two).
//   DsT (dy3^T: 256 lines x 64 rows): 8-byte piece c (4 rows) of line n at c ^ dsw(n).  Written
//       by the y3 epilogue (ds_write_b64, 16 consecutive lines per lane group), read transposed
//       by the dz A operand (4 lines x 16 rows) and by the dW3 A operand (ds_read_b64 over 32
//       consecutive lines).  Round 4's padded 34-dword lines left the dz reads 2-way conflicted.
__device__ __forceinline__ int dsw(int n) {
    return (((n >> 1) & 1) << 3) | (((n >> 3) & 1) << 2) | (((n >> 2) & 1) << 1) | ((n ^ (n >> 4)) & 1);
}
__device__ __forceinline__ int zsw(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// The round-4 8-wave kernel (sa_dy8) restructured so its three MFMA chains are fed two steps
// ahead.  sa_dy8 held, per lane,
// 16 channels x 2 statistics partials (32 VGPRs) next to the W3^T fragments (64) and the dW3
// accumulators (64): at the 256-VGPR cap every MFMA waited for the LDS read issued just before
// it.  Here the dz product is computed transposed, dz[row][k] = dy3 W3 with dy3 as the A
// operand: a lane holds ONE channel (kz = kbz + r32) of 16 rows, so the statistics partials are
// 2 registers and the channel's BN constants 4; the freed registers carry the operands ahead.
// The dz values are staged in LDS (Dz, 2-byte writes) and stored as 16-byte rows by the next
// tile's prologue.  dy3 is cB*y3 + cC everywhere but at the pooled row of each centroid, whose
// value comes from the pooled y3 (ysel, the forward's value at that row, which the recompute
// reproduces bit for bit): one 2-byte LDS write per lane over the 8-byte row stores.
// Same roles per wave and output layouts as sa_dy8; the statistics are summed over a lane's
// rows in a different order: fp32 over a tile's 16 rows, fp64 across tiles, lanes and
// workgroups (a lane sees 16x the rows sa_dy8's did: fp32 across tiles lost precision on the
// near-cancelling sum of dt).
template <int K, int N, bool STATS>
__global__ __launch_bounds__(512, 1) void sa_dy9_kernel(DyFusedArgs p) {
    constexpr int T8 = 512;
    constexpr int LDR = kTile;        // DsT line (swizzled, unpadded)
    constexpr int LDY = K + 32;       // Ys: ds_read_b64_tr_b16 column reads (80 dwords)
    constexpr int KS = K / 16;
    constexpr int NS = N / 16;
    constexpr int NWL = 6;            // dz k-steps whose W3 fragments are read from W3s, not held
    static_assert(K == 128 && N == 256, "8 waves: 32 y3 columns, 32 dz channels x 32 rows, 32 dW rows");
    __shared__ __attribute__((aligned(256))) bf16 As[kTile * K];
    __shared__ __attribute__((aligned(128))) bf16 DsT[N * LDR];
    __shared__ __attribute__((aligned(16))) bf16 Dz[kTile * K];
    __shared__ __attribute__((aligned(16))) bf16 Ys[STATS ? kTile * LDY : 8];
    __shared__ __attribute__((aligned(256))) bf16 W3s[N * K];   // swizzled as As (zsw of the row n)
    __shared__ float sc[K], sh[K];
    static_assert(sizeof(As) + sizeof(DsT) + sizeof(Dz) + sizeof(Ys) + sizeof(W3s) +
                  2 * K * sizeof(float) <= 160 * 1024, "LDS images exceed the CU's 160 KB");
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r32 = lane & 31, h = lane >> 5;

    for (int k = tid; k < K; k += T8) {
        sc[k] = p.scale[k];
        sh[k] = p.shift[k];
    }
    for (int i = tid; i < N * K / 8; i += T8) {   // W3 (N, K) -> swizzled LDS rows
        const int n = i / (K / 8), c = i % (K / 8);
        *reinterpret_cast<bf16x8*>(&W3s[n * K + 8 * (c ^ zsw(n))]) = *reinterpret_cast<const bf16x8*>(p.W + (size_t)n * K + 8 * c);
    }
    const int kbz = (wave & 3) * 32, rbz = wave >> 2;   // dz: channel block, row block
    const int kz = kbz + r32;                           // dz: this lane's channel
    // W3 fragments (B operand of dz = dy3 W3): channel kz, n in col_operand's order; the first
    // NWL k-steps' come from W3s in the dz loop (registers for the operands read ahead)
    bf16x8 wt[NS];
#pragma unroll
    for (int s = NWL; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j)
            wt[s][j] = p.W[(size_t)(16 * s + 8 * (j >> 2) + 4 * h + (j & 3)) * K + kz];
    float zsc = 0.f, zsh = 0.f, zmu = 0.f, zis = 0.f;   // layer 2's BN of channel kz
    if constexpr (STATS) {
        zsc = p.scale[kz];
        zsh = p.shift[kz];
        zmu = p.mean[kz];
        zis = p.invstd[kz];
    }
    const int ny = wave * 32 + r32;   // y3 column / dW3 row of this lane
    const float cA = p.cA[ny], cB = p.cB[ny], cC = p.cC[ny];
    double st1 = 0.0, st2 = 0.0;   // fp32 over a tile's 16 rows, fp64 across tiles
    f32x16 dw[K / 32];
#pragma unroll
    for (int b = 0; b < K / 32; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) dw[b][i] = 0.f;

    // element offsets.  As, y3 A operand: row r32 (+32), piece 2s + h -> ya ^ 16s.
    const int zt = zsw(r32);
    const int ya = r32 * K + 8 * (h ^ zt);
    const int wy = ny * K + 8 * (h ^ zt);   // W3s, y3 B operand: row ny (zsw(ny) = zsw(r32))
    // As, dW3 B operand (col_operand's lane pattern): rows 16s + rl (+8), k = 32b + 16(g&1) +
    // 4(i&3); zsw(16s + rl) = zsw(rl), so (base ^ 32b) + 16K s.  The same pattern reads the
    // dz B operand from W3s (rows n = 16s + rl, k = kbz + ...): (base ^ kbz) + 16K s.
    const int g4 = lane >> 4, i16 = lane & 15;
    const int rl = 4 * (g4 >> 1) + (i16 >> 2);
    const int kq = 2 * (g4 & 1) + ((i16 >> 1) & 1);   // 16-byte piece within the 64-byte column run
    const int zl = zsw(rl), zh = zsw(rl + 8);
    const int xlo = rl * K + 32 * (zl >> 2) + 8 * (kq ^ (zl & 3)) + 4 * (i16 & 1);
    const int xhi = (rl + 8) * K + 32 * (zh >> 2) + 8 * (kq ^ (zh & 3)) + 4 * (i16 & 1);
    // DsT.  y3 stores / dW3 reads: line ny, piece c at 4 (c ^ dsw(ny)); the pieces 8rb + 2q + h
    // and 4s + h (+2) are oy ^ (32rb + 8q) and oy ^ 16s (^ 8).  dz reads: lines 16s + nl (+8),
    // pieces pc; dsw(16s + nl) = dsw(nl) ^ (s & 1): two bases per half and an immediate 1024 s.
    const int sgy = dsw(r32);
    const int oy = ny * LDR + 4 * (h ^ sgy);
    const int pc = rbz * 8 + 4 * (g4 & 1) + (i16 & 3);
    const int nl = 4 * (g4 >> 1) + (i16 >> 2);
    const int zl0 = nl * LDR + 4 * (pc ^ dsw(nl));
    const int zh0 = (nl + 8) * LDR + 4 * (pc ^ dsw(nl + 8));
    const bf16* zlo[2] = {DsT + zl0, DsT + (zl0 ^ 4)};
    const bf16* zhi[2] = {DsT + zh0, DsT + (zh0 ^ 4)};

    const int ntiles = p.R / kTile;
    constexpr int CH = kTile * K / 8 / T8;
    static_assert(CH * T8 * 8 == kTile * K, "tile chunks");
    bf16x8 pre[CH];
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.yprev, 0, (int)min((long long)p.R * K * 2, 0x7fffffffLL), kBufDword3);
    const __amdgpu_buffer_rsrc_t irs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.isel, 0, 0x7fffffff, kBufDword3);
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.gsel, 0, 0x7fffffff, kBufDword3);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.ysel, 0, 0x7fffffff, kBufDword3);
    auto fetch = [&](int tile) __attribute__((always_inline)) {
        const int soff = tile * kTile * K * 2;
        const int tf = (wv * 64 + lane_fresh()) * 16;
#pragma unroll
        for (int c = 0; c < CH; ++c)
            pre[c] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                    yrs, tf + c * T8 * 16, soff, 0));
    };
    // the pooled gradient, value and row of this lane's column, one tile ahead
    float gv_n[2] = {0.f, 0.f}, yv_n[2] = {0.f, 0.f};
    uint32_t sv_n[2] = {0u, 0u};
    auto fetch_g = [&](int tile) __attribute__((always_inline)) {
        const int nyf = wv * 32 + (lane_fresh() & 31);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const int pc0 = (p.S == 64 ? tile : tile * 2 + rb) * N;
            sv_n[rb] = __builtin_amdgcn_raw_buffer_load_b8(irs, nyf, pc0, 0);
            gv_n[rb] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(grs, nyf * 4, pc0 * 4, 0));
            yv_n[rb] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vrs, nyf * 4, pc0 * 4, 0));
        }
    };
    // a finished tile's dz rows (staged in Dz by its dz phase) -> HBM as 16-byte row pieces
    auto flush_dz = [&](size_t prow0) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int ch = tid + c * T8;
            const int row = ch / (K / 8), kc = (ch % (K / 8)) * 8;
            *reinterpret_cast<bf16x8*>(p.dz + (prow0 + row) * K + kc) =
                *reinterpret_cast<const bf16x8*>(&Dz[row * K + kc]);
        }
    };
    if (blockIdx.x < ntiles) {
        fetch(blockIdx.x);
        fetch_g(blockIdx.x);
    }
    __syncthreads();
    PROBE_DECL
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const size_t row0 = (size_t)tile * kTile;
        PROBE(0);
        if (tile != (int)blockIdx.x) flush_dz(row0 - (size_t)gridDim.x * kTile);
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int ch = tid + c * T8;
            const int row = ch / (K / 8), kc = (ch % (K / 8)) * 8;
            bf16x8 z;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                z[j] = (bf16)fmaxf(fmaf(sc[kc + j], (float)pre[c][j], sh[kc + j]), 0.f);
            *reinterpret_cast<bf16x8*>(&As[row * K + 8 * ((kc >> 3) ^ zsw(row))]) = z;
            if constexpr (STATS) *reinterpret_cast<bf16x8*>(&Ys[row * LDY + kc]) = pre[c];
        }
        const float gv[2] = {gv_n[0], gv_n[1]}, yv[2] = {yv_n[0], yv_n[1]};
        const int sv[2] = {(int)sv_n[0], (int)sv_n[1] + (p.S == 64 ? 0 : 32)};
        PROBE(1);
        __syncthreads();
        PROBE(2);
        if (tile + (int)gridDim.x < ntiles) {   // in flight below
            fetch_g(tile + gridDim.x);
            fetch(tile + gridDim.x);
        }

        // y3 = z W3^T for columns 32w.., then dy3 -> DsT; operands two k-steps ahead
        {
            bf16x8 bq[KS], a0q[KS], a1q[KS];
            auto ld = [&](int s) __attribute__((always_inline)) {
                bq[s] = *reinterpret_cast<const bf16x8*>(&W3s[wy ^ (16 * s)]);
                a0q[s] = *reinterpret_cast<const bf16x8*>(&As[ya ^ (16 * s)]);
                a1q[s] = *reinterpret_cast<const bf16x8*>(&As[(ya ^ (16 * s)) + 32 * K]);
            };
            f32x16 acc[2];
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[rb][i] = 0.f;
            ld(0);
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                if (s + 1 < KS) ld(s + 1);
                acc[0] = mfma(a0q[s], bq[s], acc[0]);
                acc[1] = mfma(a1q[s], bq[s], acc[1]);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {   // rows rb*32 + 8q + 4h + (0..3): piece 8rb + 2q + h
                    bf16x4 d4;
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        d4[j] = (bf16)fmaf(cB, (float)(bf16)acc[rb][4 * q + j], cC);
                    *reinterpret_cast<bf16x4*>(&DsT[oy ^ (32 * rb + 8 * q)]) = d4;
                }
            }
            // the pooled row of each centroid (one per tile at S = 64, per row block at 32)
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
                const int r = sv[rb];
                if ((rb == 0 || p.S == 32) && h == ((r >> 2) & 1))
                    DsT[ny * LDR + 4 * ((r >> 2) ^ sgy) + (r & 3)] = (bf16)fmaf(cA, gv[rb], fmaf(cB, yv[rb], cC));
            }
        }
        PROBE(3);
        __syncthreads();
        PROBE(4);

        // dz[row][k] = dy3 W3 for rows rbz*32.., channel kz: A = dy3 rows (transposed DsT reads).
        // Its epilogue (bf16 values to Dz, the layer-2 statistics) runs one element per dW3
        // MFMA below, in that chain's shadow (dW3 does not depend on dz).
        f32x16 acc;
        bf16x8 yq[2];   // layer 2's raw rows of this lane's channel (the statistics)
        {
            bf16x8 aq[NS];
            auto ld = [&](int s) __attribute__((always_inline)) {
                const bf16x4 lo = tr16(zlo[s & 1] + 16 * LDR * s);
                const bf16x4 hi = tr16(zhi[s & 1] + 16 * LDR * s);
                aq[s] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                if (s < NWL) {
                    const bf16x4 wl = tr16(W3s + (xlo ^ kbz) + 16 * K * s);
                    const bf16x4 wh = tr16(W3s + (xhi ^ kbz) + 16 * K * s);
                    wt[s] = bf16x8{wl[0], wl[1], wl[2], wl[3], wh[0], wh[1], wh[2], wh[3]};
                }
            };
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = 0.f;
            ld(0);
            ld(1);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                if (s + 2 < NS) ld(s + 2);
                acc = mfma(aq[s], wt[s], acc);
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (STATS) {
                yq[0] = col_operand(Ys, LDY, lane, kbz, 2 * rbz);
                yq[1] = col_operand(Ys, LDY, lane, kbz, 2 * rbz + 1);
            }
        }
        PROBE(5);

        // dW3 rows 32w.. += dy3^T z over this tile's rows; operands one product ahead; dz
        // element t (row rbz*32 + (t&3) + 8(t>>2) + 4h of channel kz) beside product t
        {
            bf16x8 adq[kTile / 16], bzq[kTile / 16 * (K / 32)];
            auto ld = [&](int t) __attribute__((always_inline)) {
                const int s = t >> 2, b = t & 3;
                if (b == 0) {
                    const bf16x4 lo = *reinterpret_cast<const bf16x4*>(&DsT[oy ^ (16 * s)]);
                    const bf16x4 hi = *reinterpret_cast<const bf16x4*>(&DsT[oy ^ 8 ^ (16 * s)]);
                    adq[s] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
                const bf16x4 lo = tr16(As + (xlo ^ (32 * b)) + 16 * K * s);
                const bf16x4 hi = tr16(As + (xhi ^ (32 * b)) + 16 * K * s);
                bzq[t] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            };
            constexpr int NT = kTile / 16 * (K / 32);
            static_assert(NT == 16, "one dz element per dW3 product");
            bf16* dzl = &Dz[(rbz * 32 + 4 * h) * K + kz];
            float t1 = 0.f, t2 = 0.f;
            ld(0);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                if (t + 1 < NT) ld(t + 1);
                dw[t & 3] = mfma(adq[t >> 2], bzq[t], dw[t & 3]);
                const bf16 o = (bf16)acc[t];
                dzl[((t & 3) + 8 * (t >> 2)) * K] = o;
                if constexpr (STATS) {   // bn_relu_bwd pass 0 on the stored value
                    const float yy = (float)yq[t >> 3][t & 7];
                    const float dt = fmaf(zsc, yy, zsh) > 0.f ? (float)o : 0.f;
                    t1 += dt;
                    t2 = fmaf(dt, (yy - zmu) * zis, t2);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (STATS) {
                st1 += (double)t1;
                st2 += (double)t2;
            }
        }
        PROBE(6);
        __syncthreads();   // As / DsT / Ys / Dz are rewritten / stored by the next tile
        PROBE(7);
    }
    PROBE_END;
    if (blockIdx.x < ntiles)   // the last tile's dz rows
        flush_dz((size_t)(blockIdx.x + (ntiles - 1 - blockIdx.x) / gridDim.x * gridDim.x) * kTile);
    if constexpr (STATS) {
        // channel kz: the two lane halves (rows 4h..), then row block 1 handed to row block 0
        const double s1 = st1 + __shfl_xor(st1, 32);
        const double s2 = st2 + __shfl_xor(st2, 32);
        double* xs = reinterpret_cast<double*>(DsT);
        if (rbz == 1 && h == 0) {
            xs[((wave & 3) * 32 + r32) * 2] = s1;
            xs[((wave & 3) * 32 + r32) * 2 + 1] = s2;
        }
        __syncthreads();
        if (rbz == 0 && h == 0) {
            p.stats[(size_t)blockIdx.x * 2 * K + kz] = s1 + xs[(wave * 32 + r32) * 2];
            p.stats[(size_t)blockIdx.x * 2 * K + K + kz] = s2 + xs[(wave * 32 + r32) * 2 + 1];
        }
    }
    // dW3 partial: element (b, i) = dW[n][k], n = 32w + (i&3) + 8(i>>2) + 4h, k = 32b + r32
    float* out = p.dwpart + (size_t)blockIdx.x * N * K;
#pragma unroll
    for (int b = 0; b < K / 32; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int n = wave * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
            out[(size_t)n * K + 32 * b + r32] = dw[b][i];
        }
}

// The middle layer's backward in one pass (sa_dy2_fused_kernel), after the pooled layer's
// (which produced dz2 and this layer's BN-backward coefficients cA2 / cB2 / cC2):
//   per 64-row tile:  z1 = relu(a1*y1 + b1) -> LDS (and raw y1 for the statistics)
//                     dy2 = cA2*dt + cB2*y2 + cC2, dt = (a2*y2 + b2 > 0) * dz2 -> LDS
//                     dz1^T = W2^T dy2^T (MFMA) -> HBM (R, K) bf16, 8-byte stores
//                     layer 1's ReLU + BN backward partials on the stored dz1
//                     dW2 += dy2^T z1 (MFMA on transposed LDS reads), per workgroup
// replacing the ReLU+BN apply pass (dy2 stored), a dW2 GEMM, a dgrad GEMM and the layer-1
// statistics pass.  K = 64 (layer-1 channels), N = 128 (layer-2 channels).
struct Dy2Args {
    const bf16* y1; const float* a1; const float* b1;    // (R, K), layer-1 folded BN
    const bf16* y2; const float* a2; const float* b2;    // (R, N), layer-2 folded BN
    const bf16* dz2;                                     // (R, N)
    const float* cA; const float* cB; const float* cC;   // (N) layer-2 BN backward
    const bf16* W;                                       // (N, K) W2
    const float* mean1; const float* invstd1;            // (K)
    int R;
    bf16* dz1;          // (R, K)
    float* dwpart;      // (gridDim.x, N, K)
    double* stats;      // (gridDim.x, 2, K)
    const float* x0;    // X0 variant (y1 == NULL): y1 = bf16(x0 W1^T) recomputed, (R, 3)
    const float* W1;    // (K, 3)
};

// sa_dy2_fused's LDS images (round 6), conflict-free for every access of the kernel under the
// MI355X lane-group rules (tools/lds_banks_dy9.py enumerates them):
//   Ds (dy2: 64 rows x 128 n, 256-byte rows): 16-byte piece c of row r at c ^ zsw(r).  Read
//      row-wise by the dz1 B operand (ds_read_b128, lanes = rows) and transposed by the dW2 A
//      operand (ds_read_b64_tr_b16 over 4 rows x 16 n).  Padded 272-byte rows were 4-way on the
//      transposed reads.
//   As (z1: 64 rows x 64 k, 128-byte rows): piece c of row r at c ^ asw(r) (rows r and r ^ 2 of
//      a transposed read share a 32-bank half: the XOR moves one to the other 16 banks).
//   Ys (raw y1, read by rows, 4 channels a lane): 66-dword rows, two rows per bank pair window.
__device__ __forceinline__ int asw(int r) { return ((r >> 1) & 1) << 2; }

template <int K, int N, bool X0>
__global__ __launch_bounds__(kThreads, 1) void sa_dy2_fused_kernel(Dy2Args p) {
    static_assert(K == 64 && N == 128, "4 waves = 2 x 2 dz tiles, 32 dW rows each");
    constexpr int LDY = K + 68;   // Ys row: 66 dwords
    __shared__ __attribute__((aligned(256))) bf16 As[kTile * K];   // z1, swizzled (asw)
    __shared__ __attribute__((aligned(16))) bf16 Ys[kTile * LDY];  // raw y1
    __shared__ __attribute__((aligned(256))) bf16 Ds[kTile * N];   // dy2, swizzled (zsw)
    __shared__ float a1s[K], b1s[K], mus[K], iss[K], a2s[N], b2s[N], cAs[N], cBs[N], cCs[N];
    __shared__ float w1s[X0 ? 3 * K : 1];
    __shared__ __attribute__((aligned(16))) float x0s[X0 ? 3 * kTile : 4];   // the tile's x0 rows
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r32 = lane & 31, h = lane >> 5;
    for (int k = tid; k < K; k += kThreads) {
        a1s[k] = p.a1[k];
        b1s[k] = p.b1[k];
        mus[k] = p.mean1[k];
        iss[k] = p.invstd1[k];
    }
    if constexpr (X0)
        for (int k = tid; k < 3 * K; k += kThreads) w1s[k] = p.W1[k];
    for (int n = tid; n < N; n += kThreads) {
        a2s[n] = p.a2[n];
        b2s[n] = p.b2[n];
        cAs[n] = p.cA[n];
        cBs[n] = p.cB[n];
        cCs[n] = p.cC[n];
    }
    // dz1^T tile of this wave: channels kbase .. +31, rows rb*32 .. +31
    const int kbase = (wave & 1) * 32, rb = wave >> 1;
    constexpr int NS = N / 16;
    bf16x8 wt[NS];   // W2^T: lane row k = kbase + r32, channels 16s + 8h + j
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) wt[s][j] = p.W[(size_t)(16 * s + 8 * h + j) * K + kbase + r32];
    f32x16 dw[2];    // dW2 rows wave*32 .. +31, columns 0..31 / 32..63
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) dw[b][i] = 0.f;
    float st1[16], st2[16];   // channels kbase + 8g + 4h + j of this lane's rows
#pragma unroll
    for (int i = 0; i < 16; ++i) st1[i] = st2[i] = 0.f;
    __syncthreads();

    // a thread's coefficients, invariant over the tiles (its chunks all start at the same
    // channel): from LDS once per launch, not per chunk and tile (the prologue's and the
    // epilogue's LDS reads were ~40 % of the kernel's LDS instructions)
    const int kc0 = (tid % (K / 8)) * 8, nc0 = (tid % (N / 8)) * 8;
    float ca1[8], cb1[8], ca2[8], cb2[8], cca[8], ccb[8], ccc[8], cw1[X0 ? 24 : 1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        ca1[j] = a1s[kc0 + j]; cb1[j] = b1s[kc0 + j];
        ca2[j] = a2s[nc0 + j]; cb2[j] = b2s[nc0 + j];
        cca[j] = cAs[nc0 + j]; ccb[j] = cBs[nc0 + j]; ccc[j] = cCs[nc0 + j];
    }
    if constexpr (X0)
#pragma unroll
        for (int j = 0; j < 24; ++j) cw1[j] = w1s[3 * kc0 + j];
    float ea1[16], eb1[16], emu[16], eis[16];   // the epilogue's 16 channels kbase + 8g + 4h + j
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int kk = kbase + 8 * (i >> 2) + 4 * h + (i & 3);
        ea1[i] = a1s[kk]; eb1[i] = b1s[kk]; emu[i] = mus[kk]; eis[i] = iss[kk];
    }
    const int ntiles = p.R / kTile;
    // swizzled element offsets.  dz1 B operand (Ds rows rb*32 + r32): zsw(r) depends on r & 15.
    const int zr = zsw(r32);
    // dW2 operands in col_operand's lane pattern (rows 16s + rl (+8), columns c0 + 16(g&1) +
    // 4(i&3)): piece cq of the 32-column run, 4 elements at eq; the swizzles do not depend on s
    const int g4 = lane >> 4, i16 = lane & 15;
    const int rl = 4 * (g4 >> 1) + (i16 >> 2);
    const int cq = 2 * (g4 & 1) + ((i16 & 3) >> 1), eq = 4 * (i16 & 1);
    const int dlo = rl * N + 8 * ((4 * wave + cq) ^ zsw(rl)) + eq;
    const int dhi = (rl + 8) * N + 8 * ((4 * wave + cq) ^ zsw(rl + 8)) + eq;
    const int alo = rl * K + 8 * (cq ^ asw(rl)) + eq;         // column run 32b: ^ 32b
    const int ahi = (rl + 8) * K + 8 * (cq ^ asw(rl + 8)) + eq;
    constexpr int C1 = kTile * K / 8 / kThreads;   // 16-byte chunks per thread: y1
    constexpr int C2 = kTile * N / 8 / kThreads;   // y2, dz2
    bf16x8 py1[X0 ? 1 : C1], py2[C2], pdz[C2];
    float4 px0 = make_float4(0.f, 0.f, 0.f, 0.f);   // X0: 16 bytes of the tile's 768 B of x0
    auto fetch = [&](int tile) {
        const size_t row0 = (size_t)tile * kTile;
        if constexpr (X0) {
            if (tid < 3 * kTile / 4) px0 = reinterpret_cast<const float4*>(p.x0 + row0 * 3)[tid];
        } else {
#pragma unroll
            for (int c = 0; c < C1; ++c) {
                const int ch = tid + c * kThreads, row = ch / (K / 8), kc = (ch % (K / 8)) * 8;
                py1[c] = *reinterpret_cast<const bf16x8*>(p.y1 + (row0 + row) * K + kc);
            }
        }
#pragma unroll
        for (int c = 0; c < C2; ++c) {
            const int ch = tid + c * kThreads, row = ch / (N / 8), nc = (ch % (N / 8)) * 8;
            py2[c] = *reinterpret_cast<const bf16x8*>(p.y2 + (row0 + row) * N + nc);
            pdz[c] = *reinterpret_cast<const bf16x8*>(p.dz2 + (row0 + row) * N + nc);
        }
    };
    if (blockIdx.x < ntiles) fetch(blockIdx.x);
    if constexpr (X0) {   // x0 of the first tile -> LDS (read in the first prologue)
        if (tid < 3 * kTile / 4) reinterpret_cast<float4*>(x0s)[tid] = px0;
        __syncthreads();
    }
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const size_t row0 = (size_t)tile * kTile;
#pragma unroll
        for (int c = 0; c < C1; ++c) {
            const int ch = tid + c * kThreads, row = ch / (K / 8), kc = kc0;
            bf16x8 y1v;
            if constexpr (X0) {
                const float* xr = &x0s[3 * row];
#pragma unroll
                for (int j = 0; j < 8; ++j) {   // sa_l1_kernel's value, bit for bit
                    const float* w = &cw1[3 * j];
                    y1v[j] = (bf16)fmaf(w[2], xr[2], fmaf(w[1], xr[1], w[0] * xr[0]));
                }
            } else {
                y1v = py1[c];
            }
            bf16x8 z;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                z[j] = (bf16)fmaxf(fmaf(ca1[j], (float)y1v[j], cb1[j]), 0.f);
            *reinterpret_cast<bf16x8*>(&As[row * K + 8 * ((kc >> 3) ^ asw(row))]) = z;
            *reinterpret_cast<bf16x4*>(&Ys[row * LDY + kc]) = bf16x4{y1v[0], y1v[1], y1v[2], y1v[3]};
            *reinterpret_cast<bf16x4*>(&Ys[row * LDY + kc + 4]) = bf16x4{y1v[4], y1v[5], y1v[6], y1v[7]};
        }
#pragma unroll
        for (int c = 0; c < C2; ++c) {   // bn_relu_bwd_kernel pass 1 arithmetic
            const int ch = tid + c * kThreads, row = ch / (N / 8), nc = nc0;
            bf16x8 d;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float yy = (float)py2[c][j];
                const float dt = fmaf(ca2[j], yy, cb2[j]) > 0.f ? (float)pdz[c][j] : 0.f;
                d[j] = (bf16)fmaf(cca[j], dt, fmaf(ccb[j], yy, ccc[j]));
            }
            *reinterpret_cast<bf16x8*>(&Ds[row * N + 8 * ((nc >> 3) ^ zsw(row))]) = d;
        }
        __syncthreads();
        if (tile + (int)gridDim.x < ntiles) fetch(tile + gridDim.x);   // in flight below

        // dz1^T = W2^T dy2^T: lane = row rb*32 + r32, channels kbase + 8g + 4h + (0..3)
        {
            f32x16 acc;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const bf16x8 b = *reinterpret_cast<const bf16x8*>(&Ds[(rb * 32 + r32) * N + 8 * ((2 * s + h) ^ zr)]);
                acc = mfma(wt[s], b, acc);
            }
            const int row = rb * 32 + r32;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int k = kbase + 8 * g + 4 * h;
                bf16x4 o;
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] = (bf16)acc[4 * g + j];
                *reinterpret_cast<bf16x4*>(p.dz1 + (row0 + row) * K + k) = o;
                const bf16x4 y4 = *reinterpret_cast<const bf16x4*>(&Ys[row * LDY + k]);
#pragma unroll
                for (int j = 0; j < 4; ++j) {   // bn_relu_bwd pass 0 of layer 1
                    const float yy = (float)y4[j];
                    const float dt = fmaf(ea1[4 * g + j], yy, eb1[4 * g + j]) > 0.f ? (float)o[j] : 0.f;
                    st1[4 * g + j] += dt;
                    st2[4 * g + j] = fmaf(dt, (yy - emu[4 * g + j]) * eis[4 * g + j], st2[4 * g + j]);
                }
            }
        }
        // dW2 += dy2^T z1 over the tile's rows
#pragma unroll
        for (int s = 0; s < kTile / 16; ++s) {
            const bf16x4 dl = tr16(Ds + dlo + 16 * N * s), dh = tr16(Ds + dhi + 16 * N * s);
            const bf16x8 ad = bf16x8{dl[0], dl[1], dl[2], dl[3], dh[0], dh[1], dh[2], dh[3]};
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const bf16x4 al = tr16(As + (alo ^ (32 * b)) + 16 * K * s);
                const bf16x4 ah = tr16(As + (ahi ^ (32 * b)) + 16 * K * s);
                dw[b] = mfma(ad, bf16x8{al[0], al[1], al[2], al[3], ah[0], ah[1], ah[2], ah[3]}, dw[b]);
            }
        }
        if constexpr (X0) {   // the next tile's x0 (its prologue reads it after the barrier)
            if (tid < 3 * kTile / 4 && tile + (int)gridDim.x < ntiles)
                reinterpret_cast<float4*>(x0s)[tid] = px0;
        }
        __syncthreads();   // As / Ys / Ds (and x0s) are rewritten by the next tile
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        double s1 = (double)st1[i], s2 = (double)st2[i];
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) {
            s1 += __shfl_xor(s1, o, 64);
            s2 += __shfl_xor(s2, o, 64);
        }
        if (r32 == 0) {
            const int k = kbase + 8 * (i >> 2) + 4 * h + (i & 3);
            // rows rb*32..: two waves (rb = 0, 1) per channel -> separate slots, summed below
            p.stats[((size_t)blockIdx.x * 2 + rb) * 2 * K + k] = s1;
            p.stats[((size_t)blockIdx.x * 2 + rb) * 2 * K + K + k] = s2;
        }
    }
    float* out = p.dwpart + (size_t)blockIdx.x * N * K;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int n = wave * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
            out[(size_t)n * K + 32 * b + r32] = dw[b][i];
        }
}

}  // namespace

extern "C" int ov3d_sa_dy_fused_supported(int K, int N) { return K == 128 && N == 256; }

#ifdef OV3D_SA_PROBE
extern "C" void ov3d_sa_probe_set(unsigned long long* dbg) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sa_probe), &dbg, sizeof(dbg));
}
#endif

extern "C" int ov3d_sa_dy_fused(const void* yprev, const float* scale, const float* shift,
                                const void* W, int R, int K, int N, int S, const float* gsel,
                                const uint8_t* isel, const float* ysel, const float* cA,
                                const float* cB, const float* cC, void* dz, float* dwpart,
                                const float* mean, const float* invstd, double* stats, int nwg,
                                void* stream) {
    if (!ov3d_sa_dy_fused_supported(K, N) || R <= 0 || R % kTile || (S != 32 && S != 64) ||
        !yprev || !scale || !shift || !W || !gsel || !isel || !ysel || !cA || !cB || !cC || !dz ||
        !dwpart || nwg <= 0 || (stats && (!mean || !invstd)))
        return OV3D_EINVAL;
    DyFusedArgs a{(const bf16*)yprev, scale, shift, (const bf16*)W, R, S, gsel, isel, ysel, cA, cB,
                  cC, (bf16*)dz, dwpart, mean, invstd, stats};
    // sa_dy9 addresses the previous layer's rows through a buffer resource with 32-bit tile
    // offsets (num_records clamped to 2^31 - 1 bytes): past that the loads would return zeros.
    // The 4-wave kernel indexes with 64-bit addresses, so larger inputs go there.
    if ((long long)R * K * 2 > 0x7fffffffLL) {
        if (stats)
            hipLaunchKernelGGL((sa_dy_fused_kernel<128, 256, true>), dim3(nwg), dim3(kThreads), 0,
                               ov3d_stream(stream), a);
        else
            hipLaunchKernelGGL((sa_dy_fused_kernel<128, 256, false>), dim3(nwg), dim3(kThreads), 0,
                               ov3d_stream(stream), a);
    } else if (stats) {
        hipLaunchKernelGGL((sa_dy9_kernel<128, 256, true>), dim3(nwg), dim3(512), 0,
                           ov3d_stream(stream), a);
    } else {
        hipLaunchKernelGGL((sa_dy9_kernel<128, 256, false>), dim3(nwg), dim3(512), 0,
                           ov3d_stream(stream), a);
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_sa_dy2_fused(const void* y1, const float* x0, const float* W1, const float* a1,
                                 const float* b1, const void* y2, const float* a2, const float* b2,
                                 const void* dz2, const float* cA, const float* cB, const float* cC,
                                 const void* W, const float* mean1, const float* invstd1, int R,
                                 int K, int N, void* dz1, float* dwpart, double* stats, int nwg,
                                 void* stream) {
    if (K != 64 || N != 128 || R <= 0 || R % kTile || (!y1 && !(x0 && W1)) || !a1 || !b1 || !y2 ||
        !a2 || !b2 || !dz2 || !cA || !cB || !cC || !W || !mean1 || !invstd1 || !dz1 || !dwpart ||
        !stats || nwg <= 0)
        return OV3D_EINVAL;
    Dy2Args a{(const bf16*)y1, a1, b1, (const bf16*)y2, a2, b2, (const bf16*)dz2, cA, cB, cC,
              (const bf16*)W, mean1, invstd1, R, (bf16*)dz1, dwpart, stats, x0, W1};
    if (y1)
        hipLaunchKernelGGL((sa_dy2_fused_kernel<64, 128, false>), dim3(nwg), dim3(kThreads), 0,
                           ov3d_stream(stream), a);
    else
        hipLaunchKernelGGL((sa_dy2_fused_kernel<64, 128, true>), dim3(nwg), dim3(kThreads), 0,
                           ov3d_stream(stream), a);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
