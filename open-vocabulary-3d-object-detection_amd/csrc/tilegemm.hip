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

#include <type_traits>

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int BN = 128, BK = 64;
constexpr int KALIGN = BK;
constexpr int kMaxBiasN = 2048;
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

template <int TB, int BM, int NWV = 4>
struct Tile {
    static constexpr int NT_ = 64 * NWV;               // threads
    static constexpr int WM = NWV / 2;                 // wave rows (2 wave columns of 64)
    // LDS images (bf16 elements): A [m][k] (trans_b = 0: 136-byte rows so the two 8-byte
    // fragment reads of a half-wave hit 64 distinct banks; 144-byte rows for the b128 reads),
    // W [n][k] (trans_b = 1) or [k][n] (trans_b = 0, rows of BN + 32)
    static constexpr int LDA = TB ? BK + 8 : BK + 4;
    // trans_b = 0: 320-byte rows (80 dwords = 16 mod 64): the 4 rows x 8 column pieces of a
    // half-wave's ds_read_b64_tr_b16 land on 64 distinct banks (272-byte rows: 2-way)
    static constexpr int LDW = TB ? BK + 8 : BN + 32;
    static constexpr int ASZ = BM * LDA;
    static constexpr int WSZ = TB ? BN * LDW : BK * LDW;
    static constexpr int BUF = ASZ + WSZ;
    static constexpr int LDC = BN + 8;               // epilogue image, 272-byte rows
    static constexpr int NA = BM * BK / 8 / NT_;     // 16-byte A pieces per thread per chunk
    static constexpr int NW = BN * BK / 8 / NT_;     // 16-byte W pieces per thread per chunk
    static constexpr int MT = BM / WM / 32;          // 32-row MFMA tiles per wave
    static constexpr int NBIAS = kMaxBiasN;            // bias entries staged in LDS
    static constexpr int SMEM = 2 * BUF + BM * LDC + NBIAS;   // operands x 2, epilogue image, bias
    static_assert(NA >= 1 && NW >= 1 && MT >= 1, "tile shape");
    static_assert(SMEM * 2 <= 160 * 1024, "LDS");
};

template <int TB, int BM, int EPI, int NWV>
__global__ __launch_bounds__(64 * NWV, 2) void tile_gemm_kernel(TileArgs p) {
    using T = Tile<TB, BM, NWV>;
    constexpr int NTH = T::NT_;
    __shared__ __attribute__((aligned(16))) bf16 smem[T::SMEM];
    bf16* const Cs = smem + 2 * T::BUF;   // the epilogue image, its own region
    // the bias row, staged once (a global load at every tile end would drain the chunk loads
    // in flight: the wait counter is in order)
    bf16* const bias_s = Cs + BM * T::LDC;
    const bool has_bias = p.bias != nullptr;   // N <= NBIAS (host check)
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r32 = lane & 31, h = lane >> 5;
    const int wm = wave >> 1, wn = wave & 1;
    constexpr int WROWS = BM / T::WM;   // rows per wave

    // Persistent over tiles: workgroup b takes every G-th tile of its XCD's share.  Hardware
    // workgroup b runs on XCD b % 8; tile L (row block L / nct, column tile L % nct) belongs to
    // XCD L / (ntiles / 8), so the column tiles of a row block run on one XCD at about the same
    // time (A read from HBM into that XCD's L2 once).
    const int nct = p.N / BN, ntiles = nct * ((p.M + BM - 1) / BM);
    const int G = gridDim.x, b = blockIdx.x;
    const bool xcd = !(ntiles & 7) && !(G & 7);
    const int t0 = xcd ? (b & 7) * (ntiles >> 3) + (b >> 3) : b;
    const int tstep = xcd ? G >> 3 : G;
    const int tend = xcd ? ((b & 7) + 1) * (ntiles >> 3) : ntiles;
    const int mytiles = t0 < tend ? (tend - t0 + tstep - 1) / tstep : 0;
    const int nk = (p.K + p.K2) / BK;
    const int total = mytiles * nk;   // chunks of this workgroup, tile-major
    const bf16* const Ab = p.A + blockIdx.y * p.sA;
    const bf16* const Wb = p.W + blockIdx.y * p.sW;
    bf16* const Cb = p.C + blockIdx.y * p.sC;
    auto tile_of = [&](int t, int& m0, int& n0) __attribute__((always_inline)) {
        const int L = t0 + t * tstep;
        m0 = (L / nct) * BM;
        n0 = (L % nct) * BN;
    };

    f32x16 acc[T::MT][2];
    auto zero = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int mt = 0; mt < T::MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[mt][nt][i] = 0.f;
    };
    zero();

    // two register sets: chunks i+1 and i+2 are in flight while chunk i is multiplied (the
    // loop is unrolled by two so the set index is static).  Loads address as a uniform base
    // (the tile's row block / column block at this chunk's k) plus a per-thread 32-bit byte
    // offset fixed for the launch: no per-load address arithmetic.
    bf16x8 ra[2][T::NA], rw[2][T::NW];
    uint32_t offA[T::NA], offW[T::NW];
#pragma unroll
    for (int j = 0; j < T::NW; ++j) {
        const int idx = tid + NTH * j;
        offW[j] = TB ? (uint32_t)(((idx >> 3) * p.ldw + 8 * (idx & 7)) * 2)
                     : (uint32_t)(((idx >> 4) * p.ldw + 8 * (idx & 15)) * 2);
    }
    auto set_offA = [&](int lim) __attribute__((always_inline)) {   // rows past M: the last row
#pragma unroll
        for (int j = 0; j < T::NA; ++j) {
            const int idx = tid + NTH * j;
            offA[j] = (uint32_t)((min(idx >> 3, lim) * p.lda + 8 * (idx & 7)) * 2);
        }
    };
    set_offA(BM - 1);
    int lt = 0, lc = 0, lm0 = 0, ln0 = 0;   // tile / chunk / origin of the next load (uniform)
    auto load = [&](int set) __attribute__((always_inline)) {
        if (lc == 0) {
            tile_of(lt, lm0, ln0);
            if (lm0 + BM > p.M) set_offA(p.M - 1 - lm0);   // the last row block (ragged)
        }
        int kc = lc * BK;
        const bool second = kc >= p.K;   // uniform; (A2, W2) share A / W's strides
        if (second) kc -= p.K;
        const bf16* Ap = (second ? p.A2 : Ab) + (size_t)lm0 * p.lda + kc;
        const bf16* Wp = (second ? p.W2 : Wb) + (TB ? (size_t)ln0 * p.ldw + kc : (size_t)kc * p.ldw + ln0);
#pragma unroll
        for (int j = 0; j < T::NA; ++j)
            ra[set][j] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(Ap) + offA[j]);
#pragma unroll
        for (int j = 0; j < T::NW; ++j)
            rw[set][j] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(Wp) + offW[j]);
        if (++lc == nk) {
            lc = 0;
            ++lt;
        }
    };
    auto store = [&](int buf, int set) __attribute__((always_inline)) {
        bf16* As = smem + buf * T::BUF;
        bf16* Ws = As + T::ASZ;
#pragma unroll
        for (int j = 0; j < T::NA; ++j) {
            const int idx = tid + NTH * j, r = idx >> 3, pc = idx & 7;
            if (TB) {
                *reinterpret_cast<bf16x8*>(&As[r * T::LDA + 8 * pc]) = ra[set][j];
            } else {   // 136-byte rows: 8-byte aligned only
                const bf16x8 v = ra[set][j];
                *reinterpret_cast<bf16x4*>(&As[r * T::LDA + 8 * pc]) = bf16x4{v[0], v[1], v[2], v[3]};
                *reinterpret_cast<bf16x4*>(&As[r * T::LDA + 8 * pc + 4]) = bf16x4{v[4], v[5], v[6], v[7]};
            }
        }
#pragma unroll
        for (int j = 0; j < T::NW; ++j) {
            const int idx = tid + NTH * j;
            if (TB)
                *reinterpret_cast<bf16x8*>(&Ws[(idx >> 3) * T::LDW + 8 * (idx & 7)]) = rw[set][j];
            else
                *reinterpret_cast<bf16x8*>(&Ws[(idx >> 4) * T::LDW + 8 * (idx & 15)]) = rw[set][j];
        }
    };
    auto compute = [&](int buf) __attribute__((always_inline)) {
        const bf16* As = smem + buf * T::BUF;
        const bf16* Ws = As + T::ASZ;
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
            bf16x8 af[T::MT], wf[2];
#pragma unroll
            for (int mt = 0; mt < T::MT; ++mt) {
                const bf16* ar = As + (wm * WROWS + 32 * mt + r32) * T::LDA + 16 * s;
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

    // tile epilogue, part 1 (after the tile's last chunk): acc[mt][nt][v] of lane l is
    // C[row r32][col 8(v>>2) + 4h + (v&3)] of the wave's (mt, nt) 32 x 32 tile; bias in fp32,
    // the FFN activation, one bf16 rounding, into the LDS image
    const bool drop = EPI == EPI_RELU_DROP && p.thresh;   // uniform
    const uint32_t smix = drop ? rowdrop::seed_mix(p.seed, p.site) : 0u;
    auto finish = [&](int m0, int n0) __attribute__((always_inline)) {
        uint32_t rbase[T::MT];
#pragma unroll
        for (int mt = 0; mt < T::MT; ++mt)
            rbase[mt] = drop ? rowdrop::row_base(smix, m0 + wm * WROWS + 32 * mt + r32) : 0u;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int col = wn * 64 + 32 * nt + 8 * g + 4 * h;
                float bv[4] = {0.f, 0.f, 0.f, 0.f};
                if (has_bias) {
                    const bf16x4 bb = *reinterpret_cast<const bf16x4*>(bias_s + n0 + col);
#pragma unroll
                    for (int q = 0; q < 4; ++q) bv[q] = (float)bb[q];
                }
#pragma unroll
                for (int mt = 0; mt < T::MT; ++mt) {
                    const int row = wm * WROWS + 32 * mt + r32;
                    bf16x4 o;
#pragma unroll
                    for (int q = 0; q < 4; ++q) o[q] = (bf16)(acc[mt][nt][4 * g + q] + bv[q]);
                    if (EPI == EPI_RELU_DROP) {
                        bool keep[4] = {true, true, true, true};
                        if (drop) {   // one hash per channel pair (rowdrop.h keep8's pairs)
#pragma unroll
                            for (int j = 0; j < 4; j += 2) {
                                const uint32_t hs = rowdrop::mix24(
                                    rbase[mt] + (uint32_t)((n0 + col + j) >> 1) * 0x27D4EB2Fu);
                                keep[j] = (hs & 0xffffu) >= p.thresh;
                                keep[j + 1] = (hs >> 16) >= p.thresh;
                            }
                        }
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const float rr = fmaxf((float)o[q], 0.f);
                            o[q] = keep[q] ? (bf16)(rr * p.keep_scale) : (bf16)0.f;   // scale 1 at p = 0
                        }
                    } else if (EPI == EPI_MASK) {
                        const int gr = min(m0 + row, p.M - 1);
                        const bf16x4 hv =
                            *reinterpret_cast<const bf16x4*>(p.H + (size_t)gr * p.ldh + n0 + col);
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            o[q] = (float)hv[q] > 0.f ? (bf16)((float)o[q] * p.keep_scale) : (bf16)0.f;
                    }
                    *reinterpret_cast<bf16x4*>(&Cs[row * T::LDC + col]) = o;
                }
            }
        }
        zero();
    };
    // part 2 (after the next barrier): the image stored as whole row pieces, 16 bytes a lane
    auto flush = [&](int m0, int n0) __attribute__((always_inline)) {
        if (m0 + BM <= p.M) {   // uniform: no per-row guard on full tiles
#pragma unroll
            for (int j = 0; j < BM * BN / 8 / NTH; ++j) {
                const int idx = tid + NTH * j, r = idx >> 4, pc = idx & 15;
                *reinterpret_cast<bf16x8*>(Cb + (size_t)(m0 + r) * p.ldc + n0 + 8 * pc) =
                    *reinterpret_cast<const bf16x8*>(&Cs[r * T::LDC + 8 * pc]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < BM * BN / 8 / NTH; ++j) {
                const int idx = tid + NTH * j, r = idx >> 4, pc = idx & 15;
                if (m0 + r < p.M)
                    *reinterpret_cast<bf16x8*>(Cb + (size_t)(m0 + r) * p.ldc + n0 + 8 * pc) =
                        *reinterpret_cast<const bf16x8*>(&Cs[r * T::LDC + 8 * pc]);
            }
        }
    };

    if (total == 0) return;
    if (has_bias)
        for (int c = 4 * tid; c < p.N; c += 4 * NTH)
            *reinterpret_cast<bf16x4*>(bias_s + c) = *reinterpret_cast<const bf16x4*>(p.bias + c);
    load(0);
    if (total > 1) load(1);
    store(0, 0);
    __syncthreads();
    // step i: chunk i in LDS buffer i&1 and register set i&1 (free again), chunk i+1 in set
    // (i+1)&1; flush the previous tile's image if one is pending, issue chunk i+2 into set
    // i&1, multiply chunk i (finish the tile after its last chunk), move chunk i+1 to LDS
    // buffer (i+1)&1 (last read before the previous barrier).  The load / store flags are
    // compile-time so that the wait before the store leaves chunk i+2's loads in flight (a
    // conditional load makes the wait-count pass drain everything at the join).
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    int pend_m = -1, pend_n = 0;
    int ft = 0, fc = 0;   // tile / chunk of the multiply (uniform)
    auto step = [&](int i, auto set_c, auto ld_c, auto st_c) __attribute__((always_inline)) {
        constexpr int set = decltype(set_c)::value;
        if (pend_m >= 0) {
            flush(pend_m, pend_n);
            pend_m = -1;
        }
        if (decltype(ld_c)::value) load(set);
        compute(set);
        if (++fc == nk) {   // chunk i closes tile ft
            fc = 0;
            if (nk == 1) __syncthreads();   // this step's flush read the image
            tile_of(ft++, pend_m, pend_n);
            finish(pend_m, pend_n);
        }
        if (decltype(st_c)::value) store(set ^ 1, set ^ 1);
        __syncthreads();
    };
    int i = 0;
    for (; i + 3 < total; i += 2) {
        step(i, I0{}, I1{}, I1{});
        step(i + 1, I1{}, I1{}, I1{});
    }
    const int rem = total - i;   // 1, 2 or 3 chunks left, i even
    if (rem == 3) {
        step(i, I0{}, I1{}, I1{});
        step(i + 1, I1{}, I0{}, I1{});
        step(i + 2, I0{}, I0{}, I0{});
    } else if (rem == 2) {
        step(i, I0{}, I0{}, I1{});
        step(i + 1, I1{}, I0{}, I0{});
    } else {
        step(i, I0{}, I0{}, I0{});
    }
    flush(pend_m, pend_n);
}

// 128-row tiles with 8 waves (one workgroup per CU: operand buffers + image take 110 KB of
// LDS; a third fewer operand bytes per output than 64 x 128) when they alone fill the CUs on
// the encoder's 16384 rows with K >= 256; else 64-row tiles with 4 waves (two workgroups per
// CU).  Measured per shape (tools/gemm_time.py): N = 768 16.8 vs 17.8 us, K = 768 13.7 vs
// 15.0, K = 2048 28.0 vs 31.4; the 8192-row heads layers and K = 128 faster on 64 rows.
// OV3D_TILE_GEMM_BM=64 / 128 overrides.
int pick_bm(int M, int N, int K) {
    const char* e = getenv("OV3D_TILE_GEMM_BM");
    if (e) return atoi(e) == 128 ? 128 : 64;
    return (M >= 16384 && K >= 256 && (long long)ov3d_cdiv(M, 128) * (N / BN) >= 256) ? 128 : 64;
}

template <int TB, int BM, int NWV>
void launch_bm(const TileArgs& a, hipStream_t s, int batch) {
#define OV3D_TG(E) tile_gemm_kernel<TB, BM, E, NWV><<<dim3(G, batch), 64 * NWV, 0, s>>>(a)
    using T = Tile<TB, BM, NWV>;
    const int per_cu = (160 * 1024) / (T::SMEM * 2) >= 2 ? 2 : 1;   // workgroups per CU (LDS)
    const int ntiles = ov3d_cdiv(a.M, BM) * (a.N / BN);
    const char* e = getenv("OV3D_TILE_GEMM_G");   // grid cap (workgroups), default one CU fill
    const int slots = e && atoi(e) > 0 ? atoi(e) : 256 * per_cu;
    const int G = ntiles < slots ? ntiles : slots;
    if (a.epi == EPI_RELU_DROP)
        OV3D_TG(EPI_RELU_DROP);
    else if (a.epi == EPI_MASK)
        OV3D_TG(EPI_MASK);
    else
        OV3D_TG(EPI_NONE);
#undef OV3D_TG
}

template <int TB>
void launch(const TileArgs& a, hipStream_t s, int batch = 1) {
    if (pick_bm(a.M, a.N * batch, a.K + a.K2) == 128)
        launch_bm<TB, 128, 8>(a, s, batch);
    else
        launch_bm<TB, 64, 4>(a, s, batch);
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
    if (bias && N > kMaxBiasN) return OV3D_EINVAL;   // the bias row is staged in LDS
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
        lda1 % 8 || ldw1 % 8 || lda2 != lda1 || ldw2 != ldw1 || ldc % 8 || lda1 < K1 || lda2 < K2 ||
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
