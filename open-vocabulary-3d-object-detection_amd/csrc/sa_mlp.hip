// Set-abstraction MLP of PointnetSAModuleVotes (model_3detr.py:353-362, the
// pre-encoder) fused for training on MFMA: 1x1 conv (no bias) -> BatchNorm
// (batch statistics) -> ReLU, three times, then max over the nsample rows of
// each centroid (pointnet2 SharedMLP + F.max_pool2d [1, nsample]).
//
// Layout: channels-last rows (R = B*M*S, C), one row per (centroid, neighbour);
// the S rows of a centroid are consecutive, a 64-row tile holds one centroid
// (S = 64) or two (S = 32).  Activations are bf16 in HBM, accumulation fp32.
//
// Forward, per layer k >= 2, ONE pass over the rows (sa_layer_kernel):
//   load y_{k-1} tile (bf16) -> z = relu(a*y + b) with the previous layer's BN
//   folded into (a, b) -> LDS -> MFMA 32x32x16 with W_k held in VGPRs for the
//   whole (persistent) workgroup -> epilogue:
//     MODE_STORE: y_k (bf16) + per-channel sum / sum of squares partials;
//     MODE_POOL : nothing per row: per centroid and channel the max and min of
//                 y_k and their rows (first occurrence) + the BN partials.
//     Because relu(a*y + b) is monotone in y (non-decreasing for a >= 0,
//     non-increasing for a < 0, also after rounding), max_s relu(a*y_s + b) ==
//     relu(a * (a >= 0 ? max_s y : min_s y) + b): the last layer's activations
//     are never written (2^20 x 256 values per step).
//     MODE_POOL1: MODE_POOL given the sign of the layer's BN weight (the sign of a = gamma *
//                 invstd, known before the statistics): a channel needs only one extreme,
//                 so y is negated where gamma < 0 and one max (value, first row) is kept;
//                 the sums of the negated values are negated back once (exact), the squares
//                 are unchanged: the same bits as MODE_POOL's chosen extreme and partials.
//     MODE_DY   : backward recompute of y_k fused with the BN backward:
//                 dy = cA*g + cB*y + cC, g = pooled gradient at the arg row.
// BN statistics are reduced per workgroup (fp32 per lane over its rows, fp64
// across lanes / workgroups) and finalised on the device.
#include <limits.h>

#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

// two fp32 -> two bf16 in one dword (one v_cvt_pk_bf16_f32), the first in the low half
__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}
// the two bf16 halves of a dword as fp32 (exact)
__device__ __forceinline__ f32x2 unpack_bf16(uint32_t u) {
    return f32x2{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
}

#ifdef OV3D_SA_PROBE
// diagnostic build only (tools/sa_probe.py fwd): per-wave s_memtime totals of the layer
// kernel's tile phases (MODE_POOL launches)
__device__ unsigned long long* g_sal_probe;
#define LPROBE_DECL unsigned long long pr_t = __builtin_amdgcn_s_memtime(), pr_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define LPROBE(i) do { if (MODE == MODE_POOL || MODE == MODE_POOL1) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); pr_acc[i] += t_ - pr_t; pr_t = t_; } } while (0)
#define LPROBE_END do { if ((MODE == MODE_POOL || MODE == MODE_POOL1) && (threadIdx.x & 63) == 0 && g_sal_probe) { \
    unsigned long long* o_ = g_sal_probe + ((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8; \
    for (int i_ = 0; i_ < 8; ++i_) o_[i_] = pr_acc[i_]; } } while (0)
#else
#define LPROBE_DECL
#define LPROBE(i) do { } while (0)
#define LPROBE_END do { } while (0)
#endif

constexpr int kTile = 64;      // rows per tile
constexpr int kThreads = 256;  // 4 waves
enum { MODE_STORE = 0, MODE_POOL = 1, MODE_DY = 2, MODE_POOL1 = 3 };

__device__ __forceinline__ float relu_bn(float a, float y, float b) { return fmaxf(fmaf(a, y, b), 0.f); }

// x of lane ^ 32 (h = lane >> 5): v_permlane32_swap exchanges the two 32-lane halves of its
// operands, A = [x_lo, x_lo], B = [x_hi, x_hi]: the partner is B in the low half, A in the high
__device__ __forceinline__ uint32_t xor32(uint32_t x, int h) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return h ? (uint32_t)r[0] : (uint32_t)r[1];
}

struct LayerArgs {
    const bf16* yprev;     // (R, K)
    const float* scale;    // (K) previous layer's folded BN: a
    const float* shift;    // (K) b
    const bf16* W;         // (N, K)
    int R, S;
    bf16* zout;            // (R, K) optional: relu(a*yprev+b) as used by the MFMA
    bf16* yout;            // MODE_STORE: (R, N)
    double* partials;      // (gridDim.x, 2, N): sum, sum of squares
    float* pmax;           // MODE_POOL: (P, N) per centroid max / min of y, rows
    float* pmin;
    uint8_t* imax;
    uint8_t* imin;
    const float* gsel;     // MODE_DY: (P, N) pooled gradient after the ReLU mask
    const uint8_t* isel;   // (P, N) row of the pooled value within its centroid
    const float* gamma;    // MODE_POOL1: (N) the layer's BN weight (its sign picks the extreme)
    const float* cA;       // (N) dy = cA*g + cB*y + cC
    const float* cB;
    const float* cC;
    bf16* dyout;           // (R, N)
    const float* x0;       // X0 variant: (R, 3) first-layer input, yprev = bf16(x0 W1^T)
    const float* W1;       // (K, 3) fp32 first-layer weight
};

// the first SA layer's output row element, recomputed instead of stored (sa_l1_kernel's
// formula: bit-identical values)
__device__ __forceinline__ float l1_value(const float* w, const float* x) {
    return (float)(bf16)fmaf(w[2], x[2], fmaf(w[1], x[1], w[0] * x[0]));
}

template <int K, int N, int MODE, bool X0 = false>
__global__ __launch_bounds__(kThreads, 2) void sa_layer_kernel(LayerArgs p) {
    constexpr int LDK = K + 8;          // padded LDS row (bf16): spreads rows over banks
    constexpr int NB = N / 128;         // 32-column blocks per wave
    constexpr int KS = K / 16;          // MFMA k-steps
    __shared__ __attribute__((aligned(16))) bf16 As[kTile * LDK];
    __shared__ float sc[K], sh[K];
    __shared__ float w1s[X0 ? 3 * K : 1];
    __shared__ __attribute__((aligned(16))) float x0s[X0 ? 3 * kTile : 4];   // the tile's x0 rows
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r32 = lane & 31, h = lane >> 5;

    for (int k = tid; k < K; k += kThreads) {
        sc[k] = p.scale[k];
        sh[k] = p.shift[k];
    }
    if constexpr (X0)
        for (int k = tid; k < 3 * K; k += kThreads) w1s[k] = p.W1[k];
    bf16x8 bfrag[NB][KS];
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) {
        const int n = wave * (N / 4) + cb * 32 + r32;
#pragma unroll
        for (int s = 0; s < KS; ++s)
            bfrag[cb][s] = *reinterpret_cast<const bf16x8*>(p.W + (size_t)n * K + 16 * s + 8 * h);
    }
    float ssum[NB], ssq[NB];
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) ssum[cb] = ssq[cb] = 0.f;
    // the pool modes sum a column's values in two interleaved fp32 chains (even / odd rows of
    // a lane: packed v_pk_add / v_pk_fma over the bf16 pairs), joined at the end
    f32x2 ssum2[NB], ssq2[NB];
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) ssum2[cb] = ssq2[cb] = f32x2{0.f, 0.f};
    uint32_t fm[NB];   // MODE_POOL1: sign mask of this lane's columns (gamma < 0: negated)
#pragma unroll
    for (int cb = 0; cb < NB; ++cb)
        fm[cb] = (MODE == MODE_POOL1 && p.gamma[wave * (N / 4) + cb * 32 + r32] < 0.f) ? 0x80000000u : 0u;
    float cA[NB], cB[NB], cC[NB];
    if constexpr (MODE == MODE_DY) {
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) {
            const int n = wave * (N / 4) + cb * 32 + r32;
            cA[cb] = p.cA[n];
            cB[cb] = p.cB[n];
            cC[cb] = p.cC[n];
        }
    }
    __syncthreads();

    const int ntiles = p.R / kTile;
    // software pipeline: the next tile's rows are loaded into registers while this tile's
    // MFMA phase and epilogue run (CH 16-byte chunks per thread)
    constexpr int CH = kTile * K / 8 / kThreads;
    static_assert(CH * kThreads * 8 == kTile * K, "tile chunks");
    // a thread's chunks all start at channel kc0 (kThreads % (K / 8) == 0): its 8 BN
    // coefficients are read from LDS once, not per chunk and tile
    static_assert(kThreads % (K / 8) == 0, "chunk channel fixed per thread");
    const int kc0 = (tid % (K / 8)) * 8;
    float scv[8], shv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        scv[j] = sc[kc0 + j];
        shv[j] = sh[kc0 + j];
    }
    bf16x8 pre[X0 ? 1 : CH];
    float4 prex = make_float4(0.f, 0.f, 0.f, 0.f);   // X0: 16 bytes of the tile's 768 B of x0
    auto fetch = [&](int tile) {
        const size_t row0 = (size_t)tile * kTile;
        if constexpr (X0) {
            if (tid < 3 * kTile / 4) prex = reinterpret_cast<const float4*>(p.x0 + row0 * 3)[tid];
        } else {
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const int ch = tid + c * kThreads;
                const int row = ch / (K / 8), kc = (ch % (K / 8)) * 8;
                pre[c] = *reinterpret_cast<const bf16x8*>(p.yprev + (row0 + row) * K + kc);
            }
        }
    };
    if (blockIdx.x < ntiles) fetch(blockIdx.x);
    if constexpr (X0) {   // x0 of the first tile -> LDS (read in the first prologue)
        if (tid < 3 * kTile / 4) reinterpret_cast<float4*>(x0s)[tid] = prex;
        __syncthreads();
    }
    LPROBE_DECL
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const size_t row0 = (size_t)tile * kTile;
        LPROBE(0);
        // prologue: previous layer's BN + ReLU of the prefetched rows, to bf16, into LDS
        // (and optionally HBM)
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int ch = tid + c * kThreads;
            const int row = ch / (K / 8), kc = (ch % (K / 8)) * 8;
            bf16x8 z;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float yv;
                if constexpr (X0) yv = l1_value(&w1s[3 * (kc + j)], &x0s[3 * row]);
                else yv = (float)pre[c][j];
                z[j] = (bf16)relu_bn(scv[j], yv, shv[j]);
            }
            *reinterpret_cast<bf16x8*>(&As[row * LDK + kc]) = z;
            if (p.zout) *reinterpret_cast<bf16x8*>(p.zout + (row0 + row) * K + kc) = z;
        }
        LPROBE(1);
        __syncthreads();
        LPROBE(2);
        if (tile + (int)gridDim.x < ntiles) fetch(tile + gridDim.x);   // in flight during the MFMAs
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
                for (int cb = 0; cb < NB; ++cb)
                    acc[rb][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bfrag[cb][s], acc[rb][cb], 0, 0, 0);
            }
        }
        if constexpr (X0) {   // the next tile's x0 (its prologue reads it after the barrier)
            if (tid < 3 * kTile / 4 && tile + (int)gridDim.x < ntiles)
                reinterpret_cast<float4*>(x0s)[tid] = prex;
        }
        LPROBE(3);
        __syncthreads();   // As (and x0s) are rewritten by the next tile's prologue
        LPROBE(4);

        // epilogue: element (rb, cb, i) is row rb*32 + (i&3) + 8*(i>>2) + 4h, column n
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) {
            const int n = wave * (N / 4) + cb * 32 + r32;
            if constexpr (MODE == MODE_STORE) {
#pragma unroll
                for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int row = rb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                        const bf16 yb = (bf16)acc[rb][cb][i];
                        p.yout[(row0 + row) * N + n] = yb;
                        const float f = (float)yb;
                        ssum[cb] += f;
                        ssq[cb] = fmaf(f, f, ssq[cb]);
                    }
            } else if constexpr (MODE == MODE_POOL) {
                float mx[2], mn[2];
                int imx[2], imn[2];
#pragma unroll
                for (int rb = 0; rb < 2; ++rb) {
                    mx[rb] = -__builtin_huge_valf();
                    mn[rb] = __builtin_huge_valf();
                    imx[rb] = imn[rb] = 0;
#pragma unroll
                    for (int i = 0; i < 16; i += 2) {    // rows increase with i (fixed h)
                        const f32x2 f2 = unpack_bf16(pack_bf16(acc[rb][cb][i], acc[rb][cb][i + 1]));
                        ssum2[cb] += f2;
                        ssq2[cb] = __builtin_elementwise_fma(f2, f2, ssq2[cb]);
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            const int row = rb * 32 + ((i + e) & 3) + 8 * ((i + e) >> 2) + 4 * h;
                            const float f = f2[e];
                            if (f > mx[rb]) { mx[rb] = f; imx[rb] = row; }
                            if (f < mn[rb]) { mn[rb] = f; imn[rb] = row; }
                        }
                    }
                    // combine the two lane halves (rows 4h..): value, then lower row (the
                    // partner lane's values by v_permlane32_swap, not a ds_bpermute round trip)
                    const float omx = __builtin_bit_cast(float, xor32(__builtin_bit_cast(uint32_t, mx[rb]), h));
                    const float omn = __builtin_bit_cast(float, xor32(__builtin_bit_cast(uint32_t, mn[rb]), h));
                    const int oimx = (int)xor32((uint32_t)imx[rb], h), oimn = (int)xor32((uint32_t)imn[rb], h);
                    if (omx > mx[rb] || (omx == mx[rb] && oimx < imx[rb])) { mx[rb] = omx; imx[rb] = oimx; }
                    if (omn < mn[rb] || (omn == mn[rb] && oimn < imn[rb])) { mn[rb] = omn; imn[rb] = oimn; }
                }
                if (h == 0) {
                    if (p.S == 64) {
                        const int c0 = mx[1] > mx[0] ? 1 : 0, c1 = mn[1] < mn[0] ? 1 : 0;
                        const size_t o = (size_t)tile * N + n;
                        p.pmax[o] = mx[c0];
                        p.imax[o] = (uint8_t)imx[c0];
                        p.pmin[o] = mn[c1];
                        p.imin[o] = (uint8_t)imn[c1];
                    } else {   // S == 32: one centroid per row block
#pragma unroll
                        for (int rb = 0; rb < 2; ++rb) {
                            const size_t o = ((size_t)tile * 2 + rb) * N + n;
                            p.pmax[o] = mx[rb];
                            p.imax[o] = (uint8_t)(imx[rb] - 32 * rb);
                            p.pmin[o] = mn[rb];
                            p.imin[o] = (uint8_t)(imn[rb] - 32 * rb);
                        }
                    }
                }
            } else if constexpr (MODE == MODE_POOL1) {
                // one integer max per row block, no compare / select chain: the flipped value's
                // bits made order-preserving as an int (t, low 16 bits zero: bf16 values), plus
                // 63 - row in the low bits, so ties go to the first row.  Two values per dword
                // (round 6): one v_cvt_pk_bf16_f32, one sign flip, the order-preserving map on
                // both 16-bit halves at once (v_pk_ashrrev_i16), the statistics as packed f32
                // ops, the two keys into one v_max3_i32 (9.4 -> ~6 vector ops per value)
                const uint32_t fm2 = fm[cb] | (fm[cb] >> 16);
                int key[2];
#pragma unroll
                for (int rb = 0; rb < 2; ++rb) {
                    key[rb] = INT_MIN;
#pragma unroll
                    for (int i = 0; i < 16; i += 2) {    // rows rb*32 + (i&3) + 8(i>>2) + 4h (+1)
                        const uint32_t u2 = pack_bf16(acc[rb][cb][i], acc[rb][cb][i + 1]) ^ fm2;
                        const f32x2 f2 = unpack_bf16(u2);
                        ssum2[cb] += f2;
                        ssq2[cb] = __builtin_elementwise_fma(f2, f2, ssq2[cb]);
                        const s16x2 sg = __builtin_bit_cast(s16x2, u2) >> (s16x2){15, 15};
                        const uint32_t t2 = u2 ^ (__builtin_bit_cast(uint32_t, sg) & 0x7fff7fffu);
                        // low bits 63 - row without the lane half's 4h: compile-time constants;
                        // all of a lane's rows share h, so it is subtracted after the max
                        const uint32_t c0 = 63 - rb * 32 - (i & 3) - 8 * (i >> 2);
                        const int k0 = (int)((t2 << 16) | c0);
                        const int k1 = (int)((t2 & 0xffff0000u) | (c0 - 1u));
                        key[rb] = max(key[rb], max(k0, k1));
                    }
                    key[rb] -= 4 * h;   // low bits >= 63 - 59 - 4 = 0: no borrow into the value
                    key[rb] = max(key[rb], (int)xor32((uint32_t)key[rb], h));
                }
                float mx[2];
                int imx[2];
#pragma unroll
                for (int rb = 0; rb < 2; ++rb) {
                    const int t = key[rb] & (int)0xffff0000;
                    mx[rb] = __builtin_bit_cast(float, (uint32_t)t ^ ((uint32_t)(t >> 31) & 0x7fff0000u));
                    imx[rb] = 63 - (key[rb] & 63);
                }
                if (h == 0) {
                    float* pv = fm[cb] ? p.pmin : p.pmax;
                    uint8_t* pi = fm[cb] ? p.imin : p.imax;
                    if (p.S == 64) {
                        const int c0 = key[1] > key[0] ? 1 : 0;
                        const size_t o = (size_t)tile * N + n;
                        pv[o] = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, mx[c0]) ^ fm[cb]);
                        pi[o] = (uint8_t)imx[c0];
                    } else {   // S == 32: one centroid per row block
#pragma unroll
                        for (int rb = 0; rb < 2; ++rb) {
                            const size_t o = ((size_t)tile * 2 + rb) * N + n;
                            pv[o] = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, mx[rb]) ^ fm[cb]);
                            pi[o] = (uint8_t)(imx[rb] - 32 * rb);
                        }
                    }
                }
            } else {   // MODE_DY
#pragma unroll
                for (int rb = 0; rb < 2; ++rb) {
                    const size_t pc = (p.S == 64 ? (size_t)tile : (size_t)tile * 2 + rb) * N + n;
                    const int sel = p.isel[pc] + (p.S == 64 ? 0 : 32 * rb);
                    const float g = p.gsel[pc];
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int row = rb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                        const float y = (float)(bf16)acc[rb][cb][i];
                        const float gi = row == sel ? g : 0.f;
                        const float dy = fmaf(cA[cb], gi, fmaf(cB[cb], y, cC[cb]));
                        p.dyout[(row0 + row) * N + n] = (bf16)dy;
                    }
                }
            }
        }
        LPROBE(5);
    }
    LPROBE_END;

    if constexpr (MODE != MODE_DY) {
        // per-column totals of this workgroup: both lane halves hold the same column
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) {
            if constexpr (MODE == MODE_POOL || MODE == MODE_POOL1) {
                ssum[cb] = ssum2[cb][0] + ssum2[cb][1];
                ssq[cb] = ssq2[cb][0] + ssq2[cb][1];
            }
            ssum[cb] = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, ssum[cb]) ^ fm[cb]);
            const double s = (double)ssum[cb] + (double)__shfl_xor(ssum[cb], 32);
            const double q = (double)ssq[cb] + (double)__shfl_xor(ssq[cb], 32);
            if (h == 0) {
                const int n = wave * (N / 4) + cb * 32 + r32;
                p.partials[(size_t)blockIdx.x * 2 * N + n] = s;
                p.partials[(size_t)blockIdx.x * 2 * N + N + n] = q;
            }
        }
    }
}

// First layer: Cin = CIN fp32 (grouped, normalised xyz; + 3 colour features for ScanNet
// with --use_color) -> C1 channels.
// Chunks of 256 rows: their inputs staged through LDS by coalesced loads, then thread t
// computes channel t % C1 of the rows t / C1, t / C1 + kThreads / C1, ...
// y1 == NULL: BN statistics only.
// y = x[0] w[0] + x[1] w[1] + ... in fmaf order: the Conv2d(1x1) of the first SA layer
template <int CIN>
__device__ __forceinline__ float l1_dot(const float* w, const float* x) {
    float y = w[0] * x[0];
#pragma unroll
    for (int k = 1; k < CIN; ++k) y = fmaf(w[k], x[k], y);
    return y;
}

template <int CIN>
__global__ __launch_bounds__(kThreads) void sa_l1_kernel(const float* __restrict__ x0,
                                                         const float* __restrict__ W1, int R, int C1,
                                                         bf16* __restrict__ y1,
                                                         double* __restrict__ partials) {
    __shared__ double red[2][kThreads];
    __shared__ float xs[kThreads * CIN];
    const int tid = threadIdx.x;
    const int c = tid % C1, ph = tid / C1, nph = kThreads / C1;
    float wr[CIN];
#pragma unroll
    for (int k = 0; k < CIN; ++k) wr[k] = W1[c * CIN + k];
    float s = 0.f, q = 0.f;
    const long long nchunk = ((long long)R + kThreads - 1) / kThreads;
    for (long long ck = blockIdx.x; ck < nchunk; ck += gridDim.x) {
        const long long r0 = ck * kThreads;
        const int nr = (int)min((long long)kThreads, (long long)R - r0);
        for (int i = tid; i < CIN * nr; i += kThreads) xs[i] = x0[r0 * CIN + i];
        __syncthreads();
        for (int rr = ph; rr < nr; rr += nph) {
            const float y = l1_dot<CIN>(wr, xs + rr * CIN);
            const bf16 yb = (bf16)y;
            if (y1) y1[(r0 + rr) * C1 + c] = yb;
            const float f = (float)yb;
            s += f;
            q = fmaf(f, f, q);
        }
        __syncthreads();
    }
    red[0][tid] = s;
    red[1][tid] = q;
    __syncthreads();
    if (tid < C1) {
        double ts = 0, tq = 0;
        for (int k = 0; k < nph; ++k) {
            ts += red[0][k * C1 + tid];
            tq += red[1][k * C1 + tid];
        }
        partials[(size_t)blockIdx.x * 2 * C1 + tid] = ts;
        partials[(size_t)blockIdx.x * 2 * C1 + C1 + tid] = tq;
    }
}

// (nparts, width) fp64 partials -> (width) totals, fixed summation order (deterministic).
// A 1024-thread block covers 8 columns x 128 partial lanes (pl): a lane sums rows pl,
// pl + 128, ... of up to two columns (ca, cb < 0: none) with 8 loads of each in flight, then
// a fixed two-level LDS reduction (16 lanes x 8, then 16).  (Was 32 columns x 32 lanes: one
// block per 32 columns left the C <= 256 BatchNorms latency-bound on 2-8 CUs.)  The results
// are valid in the pl == 0 lanes.
constexpr int kColW = 8, kColPL = 1024 / kColW;
__device__ __forceinline__ void column_totals2(const double* __restrict__ partials, int nparts,
                                               int width, int ca, int cb, int pl,
                                               double (*red)[2][kColW + 1], double& ta,
                                               double& tb) {
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bool va = ca >= 0 && ca < width, vb = cb >= 0 && cb < width;
    int w = pl;
    for (; w + 7 * kColPL < nparts; w += 8 * kColPL) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (va) a[u] += partials[(size_t)(w + u * kColPL) * width + ca];
            if (vb) b[u] += partials[(size_t)(w + u * kColPL) * width + cb];
        }
    }
    for (; w < nparts; w += kColPL) {
        if (va) a[0] += partials[(size_t)w * width + ca];
        if (vb) b[0] += partials[(size_t)w * width + cb];
    }
    const int col = threadIdx.x % kColW;
    __syncthreads();   // red may still be read by a previous round
    red[pl][0][col] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    red[pl][1][col] = ((b[0] + b[1]) + (b[2] + b[3])) + ((b[4] + b[5]) + (b[6] + b[7]));
    __syncthreads();
    double ra = 0, rb = 0;
    if (pl < 16) {
#pragma unroll
        for (int k = 0; k < kColPL / 16; ++k) {
            ra += red[pl + 16 * k][0][col];
            rb += red[pl + 16 * k][1][col];
        }
    }
    __syncthreads();
    if (pl < 16) {
        red[pl][0][col] = ra;
        red[pl][1][col] = rb;
    }
    __syncthreads();
    ta = tb = 0;
    if (pl == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            ta += red[k][0][col];
            tb += red[k][1][col];
        }
    }
}

// OutT float: the totals rounded once (a weight gradient consumed in fp32, no cast launch)
template <typename OutT>
__global__ __launch_bounds__(1024) void reduce_partials_kernel(const double* __restrict__ partials,
                                                               int nparts, int width,
                                                               OutT* __restrict__ totals) {
    __shared__ double red[kColPL][2][kColW + 1];
    const int c = blockIdx.x * kColW + (threadIdx.x % kColW), pl = threadIdx.x / kColW;
    double t, unused;
    column_totals2(partials, nparts, width, c, -1, pl, red, t, unused);
    if (pl == 0 && c < width) totals[c] = (OutT)t;
}

// f32 column sums of (nparts, width) partials (the SA backward's per-workgroup dW partials):
// 64 lanes x V columns per 512-thread block, the 8 waves take every 8th part with 8 loads in
// flight, then the waves' sums are added in a fixed order (deterministic; replaces a torch
// sum(0) whose few blocks each walked all parts)
template <int V>
__global__ __launch_bounds__(512) void colsum_f32_kernel(const float* __restrict__ parts,
                                                         int nparts, int width,
                                                         float* __restrict__ out) {
    typedef float fv __attribute__((ext_vector_type(V)));
    __shared__ fv red[8][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long c0 = ((long long)blockIdx.x * 64 + lane) * V;
    const bool ok = c0 < width;
    fv a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = (fv)0.f;
    int r = w;
    if (ok) {
        for (; r + 56 < nparts; r += 64) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                a[u] += *reinterpret_cast<const fv*>(parts + (size_t)(r + 8 * u) * width + c0);
        }
        for (; r < nparts; r += 8) a[0] += *reinterpret_cast<const fv*>(parts + (size_t)r * width + c0);
    }
    red[w][lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    __syncthreads();
    if (w == 0 && ok)
        *reinterpret_cast<fv*>(out + c0) = ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane])) +
                                           ((red[4][lane] + red[5][lane]) + (red[6][lane] + red[7][lane]));
}

// sum / sum of squares of channel c over `count` rows -> mean, invstd, scale, shift (and the
// running statistics)
__device__ __forceinline__ void bn_finalize_one(int c, double tsum, double tsq, double count,
                                                const float* gamma, const float* beta, float eps,
                                                float momentum, float* running_mean,
                                                float* running_var, float* mean_out,
                                                float* invstd_out, float* scale_out,
                                                float* shift_out) {
    const double mean = tsum / count;
    double var = tsq / count - mean * mean;
    var = var < 0 ? 0 : var;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    mean_out[c] = (float)mean;
    invstd_out[c] = invstd;
    const float a = g * invstd;
    scale_out[c] = a;
    shift_out[c] = b - (float)mean * a;
    if (running_mean) {
        const double unb = count > 1 ? var * count / (count - 1) : var;
        running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
        running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
    }
}

// Training BatchNorm from totals (sum, sum of squares) over `count` rows:
// mean, biased var -> invstd, folded scale/shift; running stats with momentum
// and the unbiased variance (torch.nn.functional.batch_norm semantics).
__global__ void bn_finalize_kernel(const double* __restrict__ totals, double count, int C,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float eps, float momentum, float* running_mean, float* running_var,
                                   float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                   float* __restrict__ scale_out, float* __restrict__ shift_out,
                                   long long* num_batches_tracked) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c == 0 && num_batches_tracked) *num_batches_tracked += 1;
    if (c >= C) return;
    bn_finalize_one(c, totals[c], totals[C + c], count, gamma, beta, eps, momentum, running_mean,
                    running_var, mean_out, invstd_out, scale_out, shift_out);
}


// pooled row p = b*M + m -> its output row: p itself, or m*B + b when the output is written
// sequence-first (seq_m = M > 0: the encoder's (M, B, C) input layout, no transpose pass)
__device__ __forceinline__ long long pool_out_row(long long p, int seq_m, long long nb) {
    return seq_m > 0 ? (p % seq_m) * nb + p / seq_m : p;
}

// Pool: out = relu(a * (a >= 0 ? max : min) + b); remembers the value and row used.
__global__ void sa_pool_fwd_kernel(const float* __restrict__ pmax, const float* __restrict__ pmin,
                                   const uint8_t* __restrict__ imax, const uint8_t* __restrict__ imin,
                                   const float* __restrict__ scale, const float* __restrict__ shift,
                                   long long PN, int N, int seq_m, long long nb,
                                   float* __restrict__ out, float* __restrict__ ysel,
                                   uint8_t* __restrict__ isel) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= PN) return;
    const int n = (int)(i % N);
    const float a = scale[n];
    const bool up = a >= 0.f;
    const float y = up ? pmax[i] : pmin[i];
    out[pool_out_row(i / N, seq_m, nb) * N + n] = relu_bn(a, y, shift[n]);
    ysel[i] = y;
    isel[i] = up ? imax[i] : imin[i];
}

// Pool backward: g = dout masked by the ReLU at the pooled row; partial sums of
// g and g * xhat per channel (the BN backward reductions; zero rows add nothing).
__global__ __launch_bounds__(kThreads) void sa_pool_bwd_kernel(
    const float* __restrict__ dout, const float* __restrict__ ysel, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ mean, const float* __restrict__ invstd,
    int P, int N, int seq_m, float* __restrict__ gsel, double* __restrict__ partials) {
    // thread: channel tid % N (N <= 256, 256 % N == 0), centroid phase tid / N
    __shared__ double red[2][kThreads];
    const int tid = threadIdx.x, n = tid % N, ph = tid / N, nph = kThreads / N;
    const float a = scale[n], b = shift[n], mu = mean[n], is = invstd[n];
    float s = 0.f, q = 0.f;
#pragma unroll 4
    for (long long pi = (long long)blockIdx.x * nph + ph; pi < P; pi += (long long)gridDim.x * nph) {
        const long long i = pi * N + n;
        const float y = ysel[i];
        const float g = fmaf(a, y, b) > 0.f
                            ? dout[pool_out_row(pi, seq_m, seq_m > 0 ? P / seq_m : 0) * N + n]
                            : 0.f;
        gsel[i] = g;
        s += g;
        q = fmaf(g, (y - mu) * is, q);
    }
    red[0][tid] = s;
    red[1][tid] = q;
    __syncthreads();
    if (tid < N) {
        double ts = 0, tq = 0;
        for (int k = 0; k < nph; ++k) {
            ts += red[0][k * N + tid];
            tq += red[1][k * N + tid];
        }
        partials[(size_t)blockIdx.x * 2 * N + tid] = ts;
        partials[(size_t)blockIdx.x * 2 * N + N + tid] = tq;
    }
}

// BN backward coefficients from totals (sum g, sum g*xhat) over `count` rows:
//   dx = gamma*invstd * (g - mean(g) - xhat * mean(g*xhat))  ==  cA*g + cB*y + cC
// (PyTorch batch_norm_backward, training), plus dgamma / dbeta.
__device__ __forceinline__ void bn_bwd_finalize_one(int c, double t1, double t2, double count,
                                                    const float* gamma, const float* mean,
                                                    const float* invstd, float* cA, float* cB,
                                                    float* cC, float* dgamma, float* dbeta) {
    const double m1 = t1 / count, m2 = t2 / count;
    const double is = invstd[c], g = gamma ? gamma[c] : 1.0, mu = mean[c];
    const double a = g * is;
    cA[c] = (float)a;
    cB[c] = (float)(-a * is * m2);
    cC[c] = (float)(-a * m1 + a * is * m2 * mu);
    if (dgamma) dgamma[c] = (float)t2;
    if (dbeta) dbeta[c] = (float)t1;
}

__global__ void bn_bwd_finalize_kernel(const double* __restrict__ totals, double count, int C,
                                       const float* __restrict__ gamma, const float* __restrict__ mean,
                                       const float* __restrict__ invstd, float* __restrict__ cA,
                                       float* __restrict__ cB, float* __restrict__ cC,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    bn_bwd_finalize_one(c, totals[c], totals[C + c], count, gamma, mean, invstd, cA, cB, cC, dgamma,
                        dbeta);
}

// Both reductions in one launch: column totals of the (nparts, 2C) partials for 32 channels
// per block (the reduce_partials_kernel order, so the totals are bit-identical), then the
// finalize of those channels.  Single-replica BatchNorm (no all-reduce in between).
__global__ __launch_bounds__(1024) void bn_stats_finalize_kernel(
    const double* __restrict__ partials, int nparts, int C, double count, const float* gamma,
    const float* beta, float eps, float momentum, float* running_mean, float* running_var,
    float* mean_out, float* invstd_out, float* scale_out, float* shift_out,
    long long* num_batches_tracked) {
    __shared__ double red[kColPL][2][kColW + 1];
    const int c = blockIdx.x * kColW + (threadIdx.x % kColW), pl = threadIdx.x / kColW;
    double tsum, tsq;
    column_totals2(partials, nparts, 2 * C, c < C ? c : -1, c < C ? C + c : -1, pl, red, tsum, tsq);
    if (blockIdx.x == 0 && threadIdx.x == 0 && num_batches_tracked) *num_batches_tracked += 1;
    if (pl == 0 && c < C)
        bn_finalize_one(c, tsum, tsq, count, gamma, beta, eps, momentum, running_mean, running_var,
                        mean_out, invstd_out, scale_out, shift_out);
}

__global__ __launch_bounds__(1024) void bn_bwd_stats_finalize_kernel(
    const double* __restrict__ partials, int nparts, int C, double count, const float* gamma,
    const float* mean, const float* invstd, float* cA, float* cB, float* cC, float* dgamma,
    float* dbeta) {
    __shared__ double red[kColPL][2][kColW + 1];
    const int c = blockIdx.x * kColW + (threadIdx.x % kColW), pl = threadIdx.x / kColW;
    double t1, t2;
    column_totals2(partials, nparts, 2 * C, c < C ? c : -1, c < C ? C + c : -1, pl, red, t1, t2);
    if (pl == 0 && c < C)
        bn_bwd_finalize_one(c, t1, t2, count, gamma, mean, invstd, cA, cB, cC, dgamma, dbeta);
}

// ReLU + BN backward over rows, C = 8 * (threads per row):
// pass 0 (stats): partial sums of dt and dt*xhat, dt = relu'(a*y+b) * dz;
// pass 1 (apply): dy = cA*dt + cB*y + cC stored as bf16;
// pass 2 (weight): dy of a first layer with Cin = CIN (3, or 6 with colour) is reduced
//                  against x0 into dW1 partials (nparts, C, CIN) and never stored.
template <int PASS, int CIN = 3>
__global__ __launch_bounds__(kThreads) void bn_relu_bwd_kernel(
    const bf16* __restrict__ dz, const bf16* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ cA, const float* __restrict__ cB, const float* __restrict__ cC,
    const float* __restrict__ x0, long long R, int C, double* __restrict__ partials,
    bf16* __restrict__ dyout, const float* __restrict__ W1) {
    const int tid = threadIdx.x;
    const int tpr = C / 8;                          // threads per row
    const int kc = (tid % tpr) * 8, ph = tid / tpr, nph = kThreads / tpr;
    // y == NULL (PASS 2): the first layer's y recomputed from x0 and W1 (l1_value)
    float w1r[PASS == 2 ? 24 : 1];
    if constexpr (PASS == 2) {
        if (!y)
#pragma unroll
            for (int q = 0; q < 24; ++q) w1r[q] = W1[kc * 3 + q];
    }
    float pa[8], pb[8], p0[8], p1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        pa[j] = scale[kc + j];
        pb[j] = shift[kc + j];
        if (PASS == 0) {
            p0[j] = mean[kc + j];
            p1[j] = invstd[kc + j];
        } else {
            p0[j] = cA[kc + j];
            p1[j] = cB[kc + j];
        }
    }
    float c2[8];
    if (PASS != 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) c2[j] = cC[kc + j];
    }
    float acc0[8], acc1[8], acc2[8];
    float accx[PASS == 2 && CIN > 3 ? CIN - 3 : 1][8];   // dW1 columns 3.. (colour)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        acc0[j] = acc1[j] = acc2[j] = 0.f;
#pragma unroll
        for (int k = 0; k < (PASS == 2 && CIN > 3 ? CIN - 3 : 1); ++k) accx[k][j] = 0.f;
    }
    // rows r, r + G, ...: four rows' loads are issued before any of them is used (the loop was
    // bound by one row's load latency per iteration: 52 us for the 2^20 x 64 layer-1 pass)
    auto row_body = [&](long long r, const bf16x8& vz, const float* xr, const bf16x8& vyl)
                        __attribute__((always_inline)) {
        bf16x8 vy = vyl;
        if (PASS == 2 && !y) {
#pragma unroll
            for (int j = 0; j < 8; ++j) vy[j] = (bf16)l1_value(&w1r[PASS == 2 ? 3 * j : 0], xr);
        }
        bf16x8 out;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float yy = (float)vy[j];
            const float dt = fmaf(pa[j], yy, pb[j]) > 0.f ? (float)vz[j] : 0.f;
            if (PASS == 0) {
                acc0[j] += dt;
                acc1[j] = fmaf(dt, (yy - p0[j]) * p1[j], acc1[j]);
            } else {
                const float d = fmaf(p0[j], dt, fmaf(p1[j], yy, c2[j]));
                if (PASS == 1) {
                    out[j] = (bf16)d;
                } else {
                    acc0[j] = fmaf(d, xr[0], acc0[j]);
                    acc1[j] = fmaf(d, xr[1], acc1[j]);
                    acc2[j] = fmaf(d, xr[2], acc2[j]);
                    if constexpr (PASS == 2 && CIN > 3) {
#pragma unroll
                        for (int k = 3; k < CIN; ++k) accx[k - 3][j] = fmaf(d, xr[k], accx[k - 3][j]);
                    }
                }
            }
        }
        if (PASS == 1) *reinterpret_cast<bf16x8*>(dyout + r * C + kc) = out;
    };
    constexpr int U = 4;
    constexpr int NX = PASS == 2 ? CIN : 1;
    const long long G = (long long)gridDim.x * nph;
    long long r = (long long)blockIdx.x * nph + ph;
    for (; r + (U - 1) * G < R; r += U * G) {
        bf16x8 vz[U], vy[U];
        float xr[U][NX];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long ru = r + u * G;
            vz[u] = *reinterpret_cast<const bf16x8*>(dz + ru * C + kc);
            if (PASS == 2) {
#pragma unroll
                for (int k = 0; k < NX; ++k) xr[u][k] = x0[ru * NX + k];
            }
            if (PASS != 2 || y) vy[u] = *reinterpret_cast<const bf16x8*>(y + ru * C + kc);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) row_body(r + u * G, vz[u], xr[u], vy[u]);
    }
    for (; r < R; r += G) {
        const bf16x8 vz = *reinterpret_cast<const bf16x8*>(dz + r * C + kc);
        float xr[NX];
        if (PASS == 2) {
#pragma unroll
            for (int k = 0; k < NX; ++k) xr[k] = x0[r * NX + k];
        }
        bf16x8 vy;
        if (PASS != 2 || y) vy = *reinterpret_cast<const bf16x8*>(y + r * C + kc);
        row_body(r, vz, xr, vy);
    }
    if (PASS == 1) return;
    // reduce over the row phases: LDS [value][phase * C + channel] (nph * C == 8 * kThreads)
    // (CIN > 3: the 3 + CIN - 3 values go through the LDS in rounds of at most 3)
    __shared__ double sred[PASS == 0 ? 2 : 3][8 * kThreads];
    constexpr int NV = PASS == 0 ? 2 : CIN;
#pragma unroll
    for (int v0 = 0; v0 < NV; v0 += 3) {
        if (v0) __syncthreads();   // the previous round's reads are done
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
            for (int u = 0; u < 3 && v0 + u < NV; ++u) {
                const int v = v0 + u;
                float a;
                if (v == 0) a = acc0[j];
                else if (v == 1) a = acc1[j];
                else if (v == 2) a = acc2[j];
                else a = accx[(v >= 3 ? v - 3 : 0) % (PASS == 2 && CIN > 3 ? CIN - 3 : 1)][j];
                sred[u][ph * C + kc + j] = a;
            }
        }
        __syncthreads();
        const int nv = NV - v0 < 3 ? NV - v0 : 3;
        for (int i = tid; i < nv * C; i += kThreads) {
            const int u = i / C, c = i % C;
            double t = 0;
            for (int k = 0; k < nph; ++k) t += sred[u][k * C + c];
            if (PASS == 0)
                partials[(size_t)blockIdx.x * 2 * C + u * C + c] = t;
            else   // (C, CIN) = dW1[c][k]
                partials[(size_t)blockIdx.x * CIN * C + c * CIN + v0 + u] = t;
        }
    }
}

int grid_for(long long work, int cap) {
    long long g = work < cap ? work : cap;
    return g < 1 ? 1 : (int)g;
}

}  // namespace

extern "C" int ov3d_sa_l1_fwd_cin(const float* x0, int cin, const float* W1, int R, int C1,
                                  void* y1, double* partials, int nparts, void* stream) {
    if (R < 0 || C1 <= 0 || C1 > kThreads || kThreads % C1 || nparts <= 0) return OV3D_EINVAL;
    if (!x0 || !W1 || !partials || (cin != 3 && cin != 6)) return OV3D_EINVAL;
    if (cin == 3)
        hipLaunchKernelGGL(sa_l1_kernel<3>, dim3(nparts), dim3(kThreads), 0, ov3d_stream(stream), x0,
                           W1, R, C1, reinterpret_cast<bf16*>(y1), partials);
    else
        hipLaunchKernelGGL(sa_l1_kernel<6>, dim3(nparts), dim3(kThreads), 0, ov3d_stream(stream), x0,
                           W1, R, C1, reinterpret_cast<bf16*>(y1), partials);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_sa_l1_fwd(const float* x0, const float* W1, int R, int C1, void* y1,
                              double* partials, int nparts, void* stream) {
    return ov3d_sa_l1_fwd_cin(x0, 3, W1, R, C1, y1, partials, nparts, stream);
}

template <int MODE>
static int launch_layer(const LayerArgs& a, int K, int N, int nparts, hipStream_t s) {
#define OV3D_SA_CASE(KK, NN)                                                                     \
    if (K == KK && N == NN) {                                                                    \
        hipLaunchKernelGGL((sa_layer_kernel<KK, NN, MODE>), dim3(nparts), dim3(kThreads), 0, s, a); \
        OV3D_LAUNCH_CHECK();                                                                     \
        return OV3D_OK;                                                                          \
    }
    OV3D_SA_CASE(64, 128)
    OV3D_SA_CASE(128, 256)
    OV3D_SA_CASE(128, 128)
#undef OV3D_SA_CASE
    return OV3D_EINVAL;
}

extern "C" int ov3d_sa_layer_supported(int K, int N) {
    return (K == 64 && N == 128) || (K == 128 && N == 256) || (K == 128 && N == 128);
}

extern "C" int ov3d_sa_layer_fwd(const void* yprev, const float* scale, const float* shift,
                                 const void* W, int R, int K, int N, void* zout, void* yout,
                                 double* partials, int nparts, void* stream) {
    if (R < 0 || R % kTile || !yprev || !scale || !shift || !W || !yout || !partials || nparts <= 0)
        return OV3D_EINVAL;
    LayerArgs a = {};
    a.yprev = reinterpret_cast<const bf16*>(yprev);
    a.scale = scale;
    a.shift = shift;
    a.W = reinterpret_cast<const bf16*>(W);
    a.R = R;
    a.S = kTile;
    a.zout = reinterpret_cast<bf16*>(zout);
    a.yout = reinterpret_cast<bf16*>(yout);
    a.partials = partials;
    return launch_layer<MODE_STORE>(a, K, N, nparts, ov3d_stream(stream));
}

extern "C" int ov3d_sa_layer_fwd_x0(const float* x0, const float* W1, const float* scale,
                                    const float* shift, const void* W, int R, int K, int N,
                                    void* yout, double* partials, int nparts, void* stream) {
    if (R < 0 || R % kTile || !x0 || !W1 || !scale || !shift || !W || !yout || !partials ||
        nparts <= 0 || K != 64 || N != 128)
        return OV3D_EINVAL;
    LayerArgs a = {};
    a.x0 = x0;
    a.W1 = W1;
    a.scale = scale;
    a.shift = shift;
    a.W = reinterpret_cast<const bf16*>(W);
    a.R = R;
    a.S = kTile;
    a.yout = reinterpret_cast<bf16*>(yout);
    a.partials = partials;
    hipLaunchKernelGGL((sa_layer_kernel<64, 128, MODE_STORE, true>), dim3(nparts), dim3(kThreads), 0,
                       ov3d_stream(stream), a);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

#ifdef OV3D_SA_PROBE
extern "C" void ov3d_sal_probe_set(unsigned long long* dbg) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sal_probe), &dbg, sizeof(dbg));
}
#endif

extern "C" int ov3d_sa_layer_pool_fwd(const void* yprev, const float* scale, const float* shift,
                                      const void* W, int R, int K, int N, int S, void* zout,
                                      float* pmax, float* pmin, uint8_t* imax, uint8_t* imin,
                                      const float* gamma, double* partials, int nparts,
                                      void* stream) {
    if (R < 0 || R % kTile || (S != 32 && S != 64) || !yprev || !scale || !shift || !W || !pmax ||
        !pmin || !imax || !imin || !partials || nparts <= 0)
        return OV3D_EINVAL;
    LayerArgs a = {};
    a.yprev = reinterpret_cast<const bf16*>(yprev);
    a.scale = scale;
    a.shift = shift;
    a.W = reinterpret_cast<const bf16*>(W);
    a.R = R;
    a.S = S;
    a.zout = reinterpret_cast<bf16*>(zout);
    a.partials = partials;
    a.pmax = pmax;
    a.pmin = pmin;
    a.imax = imax;
    a.imin = imin;
    a.gamma = gamma;
    if (gamma) return launch_layer<MODE_POOL1>(a, K, N, nparts, ov3d_stream(stream));
    return launch_layer<MODE_POOL>(a, K, N, nparts, ov3d_stream(stream));
}

extern "C" int ov3d_sa_layer_dy(const void* yprev, const float* scale, const float* shift,
                                const void* W, int R, int K, int N, int S, const float* gsel,
                                const uint8_t* isel, const float* cA, const float* cB,
                                const float* cC, void* dyout, int nparts, void* stream) {
    if (R < 0 || R % kTile || (S != 32 && S != 64) || !yprev || !scale || !shift || !W || !gsel ||
        !isel || !cA || !cB || !cC || !dyout || nparts <= 0)
        return OV3D_EINVAL;
    LayerArgs a = {};
    a.yprev = reinterpret_cast<const bf16*>(yprev);
    a.scale = scale;
    a.shift = shift;
    a.W = reinterpret_cast<const bf16*>(W);
    a.R = R;
    a.S = S;
    a.gsel = gsel;
    a.isel = isel;
    a.cA = cA;
    a.cB = cB;
    a.cC = cC;
    a.dyout = reinterpret_cast<bf16*>(dyout);
    return launch_layer<MODE_DY>(a, K, N, nparts, ov3d_stream(stream));
}

extern "C" int ov3d_reduce_partials(const double* partials, int nparts, int width, double* totals,
                                    void* stream) {
    if (nparts <= 0 || width <= 0 || !partials || !totals) return OV3D_EINVAL;
    hipLaunchKernelGGL(reduce_partials_kernel<double>, dim3(ov3d_cdiv(width, kColW)), dim3(1024), 0,
                       ov3d_stream(stream), partials, nparts, width, totals);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_reduce_partials_f32(const double* partials, int nparts, int width, float* totals,
                                        void* stream) {
    if (nparts <= 0 || width <= 0 || !partials || !totals) return OV3D_EINVAL;
    hipLaunchKernelGGL(reduce_partials_kernel<float>, dim3(ov3d_cdiv(width, kColW)), dim3(1024), 0,
                       ov3d_stream(stream), partials, nparts, width, totals);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_bn_finalize(const double* totals, double count, int C, const float* gamma,
                                const float* beta, float eps, float momentum, float* running_mean,
                                float* running_var, float* mean_out, float* invstd_out,
                                float* scale_out, float* shift_out, long long* num_batches_tracked,
                                void* stream) {
    if (C <= 0 || count <= 0 || !totals || !mean_out || !invstd_out || !scale_out || !shift_out)
        return OV3D_EINVAL;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(ov3d_cdiv(C, 256)), dim3(256), 0, ov3d_stream(stream),
                       totals, count, C, gamma, beta, eps, momentum, running_mean, running_var,
                       mean_out, invstd_out, scale_out, shift_out, num_batches_tracked);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_bn_stats_finalize(const double* partials, int nparts, int C, double count,
                                      const float* gamma, const float* beta, float eps,
                                      float momentum, float* running_mean, float* running_var,
                                      float* mean_out, float* invstd_out, float* scale_out,
                                      float* shift_out, long long* num_batches_tracked,
                                      void* stream) {
    if (C <= 0 || nparts <= 0 || count <= 0 || !partials || !mean_out || !invstd_out ||
        !scale_out || !shift_out)
        return OV3D_EINVAL;
    hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3(ov3d_cdiv(C, kColW)), dim3(1024), 0,
                       ov3d_stream(stream), partials, nparts, C, count, gamma, beta, eps, momentum,
                       running_mean, running_var, mean_out, invstd_out, scale_out, shift_out,
                       num_batches_tracked);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_bn_bwd_stats_finalize(const double* partials, int nparts, int C, double count,
                                          const float* gamma, const float* mean,
                                          const float* invstd, float* cA, float* cB, float* cC,
                                          float* dgamma, float* dbeta, void* stream) {
    if (C <= 0 || nparts <= 0 || count <= 0 || !partials || !mean || !invstd || !cA || !cB || !cC)
        return OV3D_EINVAL;
    hipLaunchKernelGGL(bn_bwd_stats_finalize_kernel, dim3(ov3d_cdiv(C, kColW)), dim3(1024), 0,
                       ov3d_stream(stream), partials, nparts, C, count, gamma, mean, invstd, cA, cB,
                       cC, dgamma, dbeta);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_colsum_f32(const float* parts, int nparts, int width, float* out,
                               void* stream) {
    if (nparts <= 0 || width <= 0 || !parts || !out) return OV3D_EINVAL;
    const bool al16 = reinterpret_cast<uintptr_t>(parts) % 16 == 0 &&
                      reinterpret_cast<uintptr_t>(out) % 16 == 0;
    const bool al8 = reinterpret_cast<uintptr_t>(parts) % 8 == 0 &&
                     reinterpret_cast<uintptr_t>(out) % 8 == 0;
    // widest vector that still gives >= 256 blocks (one per CU), when the width allows it
    const int v = (al16 && width % 4 == 0 && width >= 4 * 64 * 256) ? 4
                : (al8 && width % 2 == 0 && width >= 2 * 64 * 256) ? 2 : 1;
    hipStream_t s = ov3d_stream(stream);
    const int blocks = ov3d_cdiv(width, 64 * v);
    if (v == 4) hipLaunchKernelGGL(colsum_f32_kernel<4>, dim3(blocks), dim3(512), 0, s, parts, nparts, width, out);
    else if (v == 2) hipLaunchKernelGGL(colsum_f32_kernel<2>, dim3(blocks), dim3(512), 0, s, parts, nparts, width, out);
    else hipLaunchKernelGGL(colsum_f32_kernel<1>, dim3(blocks), dim3(512), 0, s, parts, nparts, width, out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_sa_pool_fwd(const float* pmax, const float* pmin, const uint8_t* imax,
                                const uint8_t* imin, const float* scale, const float* shift, int P,
                                int N, int seq_m, float* out, float* ysel, uint8_t* isel,
                                void* stream) {
    if (P < 0 || N <= 0 || seq_m < 0 || (seq_m > 0 && P % seq_m) || !pmax || !pmin || !imax ||
        !imin || !scale || !shift || !out || !ysel || !isel)
        return OV3D_EINVAL;
    const long long PN = (long long)P * N;
    if (PN == 0) return OV3D_OK;
    hipLaunchKernelGGL(sa_pool_fwd_kernel, dim3(ov3d_cdiv(PN, 256)), dim3(256), 0, ov3d_stream(stream),
                       pmax, pmin, imax, imin, scale, shift, PN, N, seq_m,
                       seq_m > 0 ? (long long)(P / seq_m) : 0LL, out, ysel, isel);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_sa_pool_bwd(const float* dout, const float* ysel, const float* scale,
                                const float* shift, const float* mean, const float* invstd, int P,
                                int N, int seq_m, float* gsel, double* partials, int nparts,
                                void* stream) {
    if (P < 0 || N <= 0 || N > kThreads || kThreads % N || nparts <= 0 || seq_m < 0 ||
        (seq_m > 0 && P % seq_m) || !dout || !ysel || !scale || !shift || !mean || !invstd ||
        !gsel || !partials)
        return OV3D_EINVAL;
    hipLaunchKernelGGL(sa_pool_bwd_kernel, dim3(nparts), dim3(kThreads), 0, ov3d_stream(stream), dout,
                       ysel, scale, shift, mean, invstd, P, N, seq_m, gsel, partials);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_bn_bwd_finalize(const double* totals, double count, int C, const float* gamma,
                                    const float* mean, const float* invstd, float* cA, float* cB,
                                    float* cC, float* dgamma, float* dbeta, void* stream) {
    if (C <= 0 || count <= 0 || !totals || !mean || !invstd || !cA || !cB || !cC) return OV3D_EINVAL;
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(ov3d_cdiv(C, 256)), dim3(256), 0,
                       ov3d_stream(stream), totals, count, C, gamma, mean, invstd, cA, cB, cC, dgamma,
                       dbeta);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_bn_relu_bwd_cin(int pass, const void* dz, const void* y, const float* scale,
                                    const float* shift, const float* mean, const float* invstd,
                                    const float* cA, const float* cB, const float* cC,
                                    const float* x0, int cin, int R, int C, double* partials,
                                    void* dyout, int nparts, const float* W1, void* stream) {
    if (R < 0 || C <= 0 || C % 8 || C / 8 > kThreads || kThreads % (C / 8) || C > 256 ||
        nparts <= 0 || !dz || !scale || !shift || (!y && !(pass == 2 && x0 && W1 && cin == 3)) ||
        (cin != 3 && cin != 6))
        return OV3D_EINVAL;
    const bf16* dzb = reinterpret_cast<const bf16*>(dz);
    const bf16* yb = reinterpret_cast<const bf16*>(y);
    hipStream_t s = ov3d_stream(stream);
    if (pass == 0) {
        if (!mean || !invstd || !partials) return OV3D_EINVAL;
        hipLaunchKernelGGL(bn_relu_bwd_kernel<0>, dim3(nparts), dim3(kThreads), 0, s, dzb, yb, scale,
                           shift, mean, invstd, cA, cB, cC, x0, (long long)R, C, partials,
                           (bf16*)nullptr, W1);
    } else if (pass == 1) {
        if (!cA || !cB || !cC || !dyout) return OV3D_EINVAL;
        hipLaunchKernelGGL(bn_relu_bwd_kernel<1>, dim3(nparts), dim3(kThreads), 0, s, dzb, yb, scale,
                           shift, mean, invstd, cA, cB, cC, x0, (long long)R, C, partials,
                           reinterpret_cast<bf16*>(dyout), W1);
    } else if (pass == 2) {
        if (!cA || !cB || !cC || !x0 || !partials) return OV3D_EINVAL;
        if (cin == 3)
            hipLaunchKernelGGL(bn_relu_bwd_kernel<2>, dim3(nparts), dim3(kThreads), 0, s, dzb, yb,
                               scale, shift, mean, invstd, cA, cB, cC, x0, (long long)R, C, partials,
                               (bf16*)nullptr, W1);
        else
            hipLaunchKernelGGL((bn_relu_bwd_kernel<2, 6>), dim3(nparts), dim3(kThreads), 0, s, dzb,
                               yb, scale, shift, mean, invstd, cA, cB, cC, x0, (long long)R, C,
                               partials, (bf16*)nullptr, W1);
    } else {
        return OV3D_EINVAL;
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_bn_relu_bwd(int pass, const void* dz, const void* y, const float* scale,
                                const float* shift, const float* mean, const float* invstd,
                                const float* cA, const float* cB, const float* cC, const float* x0,
                                int R, int C, double* partials, void* dyout, int nparts,
                                const float* W1, void* stream) {
    return ov3d_bn_relu_bwd_cin(pass, dz, y, scale, shift, mean, invstd, cA, cB, cC, x0, 3, R, C,
                                partials, dyout, nparts, W1, stream);
}
