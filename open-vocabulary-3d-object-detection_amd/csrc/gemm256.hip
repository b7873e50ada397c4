// Large bf16 GEMM on 256 x 256 output tiles, and the 3x3 convolution as an implicit GEMM on
// the same main loop, for the RegionCLIP ROI path (res5 of the RN50x4
// ModifiedResNet over all L*B*Q ROIs, clip.inference at criterion.py:397) and the 3DETR
// decoder's memory K / V projections (models/transformer.py:369-372):
//
//   C (M, N) = act(A (M, K) . B (N, K)^T + bias (N) [+ R (M, N)]),  bf16 in / out, fp32 sums
//
// A and B are row-major with K contiguous (activations rows x weight rows: the "NT" product
// of a linear layer / 1x1 convolution).  In the convolution form A is never materialised: row
// m of A is output pixel (n, y, x) of an NHWC input (nimg, H, W, C) and column k = (ky*3 +
// kx)*C + c reads input pixel (y + ky - 1, x + kx - 1), zero outside the image (pad 1,
// stride 1) -- the (Cout, 3, 3, C) channels-last weight viewed as (Cout, 9C) is B.
//
// Main loop (cdna_hip_programming.md §5, "The 256^2 8-phase template"):
//   * 512 threads = 8 waves, wave (wr, wc) = (wave >> 2, wave & 3) owns output rows
//     mi*128 + wr*64 + [0, 64) and columns ni*128 + wc*32 + [0, 32), mi, ni in {0, 1};
//   * K-steps of 64; each operand tile (256 x 64) is held as two halves (rows 0-127 / 128-255)
//     of 16 KB, two LDS buffers: 128 KB.  Halves are filled by LDS-DMA (buffer_load ... lds,
//     16 bytes a lane, lane-linear destination; the 16-byte chunks of a 128-byte row are
//     XOR-swizzled by (row >> 1) & 7 through the per-lane SOURCE offset, which makes the
//     16x16x32 fragment reads ds_read_b128 conflict-free);
//   * four phases per K-step, one C quadrant (64 x 32 per wave: 16 MFMAs 16x16x32) each:
//       P0: read B_lo + A_lo fragments -> Q(lo, lo)      P1: read B_hi -> Q(lo, hi)
//       P2: read A_hi                  -> Q(hi, hi)      P3: (no reads)  -> Q(hi, lo)
//     each phase issues ONE half-tile of LDS-DMA (2 instructions a thread) into the buffer
//     half whose last read is far enough behind: P0 A_hi(t+1), P1 B_lo(t+2), P2 A_lo(t+2),
//     P3 B_hi(t+2); one counted vmcnt(6) per K-step (P3) retires K-step t+1 and leaves three
//     half-tiles in flight across the barriers (raw s_barrier, never __syncthreads inside
//     the loop: its fence would drain the DMA);
//   * waves 4-7 (wr = 1) run one barrier behind waves 0-3: each SIMD holds one wave of each
//     group, so one computes while its partner reads and issues (the stagger of §5; every
//     restage respects the extra barrier: the 1-phase restage of B_lo is ordered by an
//     lgkmcnt(8) before P0's first barrier, the others are 2 phases behind their last read);
//   * XCD-aware tile order (consecutive tiles of one row panel on one XCD, bijective remap).
// Epilogue: per row half, the fp32 quadrants go through LDS ([128][260] f32), then every
// thread owns 8 consecutive columns of a row: + bias, + residual (fp32), ReLU, one rounding,
// one 16-byte store.
#include <stdlib.h>
#include <type_traits>

#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 64;
constexpr int HALF = 128 * BK * 2;   // bytes of one 128-row half of an operand K-step
constexpr int BUF = 4 * HALF;        // A_lo, A_hi, B_lo, B_hi
constexpr uint32_t OOB = 0x80000000u;   // buffer offset past num_records: the load returns 0

struct Gemm256Args {
    const bf16* A;     // dense: (M, K) rows, lda; conv: NHWC input (nimg, H, W, C)
    long long lda;
    const bf16* B;     // (N, K) rows, ldb
    long long ldb;
    const void* bias;  // (N) bf16 or f32, or null
    const bf16* R;     // residual (M, N), ldr, or null
    long long ldr;
    bf16* C;
    long long ldc;
    int M, N, K;
    int bias_f32, relu;
    int H, W, Cin;     // conv form
    int gm;            // row panels per group of the tile order
    int stagger;       // waves 4-7 one barrier behind (1) or in step (0)
    int delay;         // s_sleep rounds before the first tile of every other workgroup
    // nprob products of the same shape in the same launch, problem p at A + p sA, B + p sB,
    // bias + p sbias, C + p sC (elements); its tiles follow problem p - 1's in the tile order
    // (the decoder's K and V projections of the memory; the attention pool's per-head products)
    int nprob;
    long long sA, sB, sbias, sC;
    unsigned long long* stamp;   // in-kernel launch stamps (bench.py's C5 roofline) or null
};

__device__ __forceinline__ f32x4 mfma16(i32x4 a, i32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// ds_read_b128 as an asm statement: hipcc would otherwise treat the LDS read as aliasing the
// in-flight LDS-DMA and wait vmcnt(0) before it.  The result is unprotected until a wait
// statement names it (lgkm_wait*).
template <int OFF>
__device__ __forceinline__ i32x4 lds128(uint32_t addr) {
    i32x4 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF) : "memory");
    return r;
}

__device__ __forceinline__ void lgkm_wait12(i32x4 (&a)[8], i32x4 (&b)[4]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                   "+v"(a[6]), "+v"(a[7]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3])
                 :
                 : "memory");
}
__device__ __forceinline__ void lgkm_wait8(i32x4 (&a)[8]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                   "+v"(a[6]), "+v"(a[7])
                 :
                 : "memory");
}
__device__ __forceinline__ void lgkm_wait4(i32x4 (&b)[4]) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) : : "memory");
}

__device__ __forceinline__ void barrier() { __builtin_amdgcn_s_barrier(); }

// one quadrant: 4 x 2 tiles of 16 x 16, K = 64 (two 32-deep MFMA steps); B fragments as the
// A operand: each tile is C^T (the epilogue's row-contiguous layout)
__device__ __forceinline__ void mma_quad(f32x4 (&acc)[4][2], const i32x4 (&fa)[8], const i32x4 (&fb)[4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(fb[2 * j + kh], fa[2 * i + kh], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
}

// 8 A fragments of a half (rows wr*64 + 16 i + (lane & 15)), OFF = the half's byte offset
template <int OFF>
__device__ __forceinline__ void read_a(i32x4 (&fa)[8], uint32_t p0, uint32_t p1) {
    fa[0] = lds128<OFF + 0 * 2048>(p0);
    fa[1] = lds128<OFF + 0 * 2048>(p1);
    fa[2] = lds128<OFF + 1 * 2048>(p0);
    fa[3] = lds128<OFF + 1 * 2048>(p1);
    fa[4] = lds128<OFF + 2 * 2048>(p0);
    fa[5] = lds128<OFF + 2 * 2048>(p1);
    fa[6] = lds128<OFF + 3 * 2048>(p0);
    fa[7] = lds128<OFF + 3 * 2048>(p1);
}
template <int OFF>
__device__ __forceinline__ void read_b(i32x4 (&fb)[4], uint32_t p0, uint32_t p1) {
    fb[0] = lds128<OFF + 0 * 2048>(p0);
    fb[1] = lds128<OFF + 0 * 2048>(p1);
    fb[2] = lds128<OFF + 1 * 2048>(p0);
    fb[3] = lds128<OFF + 1 * 2048>(p1);
}

__device__ __forceinline__ void glds(__amdgpu_buffer_rsrc_t rs, char* lds, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const uint32_t n = bytes > 0x7fffffffLL ? 0x7fffffffu : (uint32_t)(bytes > 0 ? bytes : 0);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)n, 0x00020000);
}

template <bool CONV, bool TAIL>   // TAIL: K % 64 != 0 (its own instance: the checks cost registers)
__global__ void __launch_bounds__(512, 2) gemm256_kernel(Gemm256Args a) {
    __shared__ __attribute__((aligned(16))) char L[2 * BUF];
    // launch stamp (measurement only, a.stamp != null): each wave's entry clock waits in LDS and
    // both words leave in one vector store at the exit -- nothing stays live in registers across
    // the kernel (ov3d_stamp's entry store kept an address live: at the 256-VGPR cap that spilled)
    __shared__ unsigned long long s_t0[8];
    if ((threadIdx.x & 63) == 0) s_t0[threadIdx.x >> 6] = wall_clock64();
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int ntn = (a.N + 255) >> 8, ntm = (a.M + 255) >> 8;
    const int ptiles = ntm * ntn, tiles = ptiles * a.nprob;
    const int nk = (a.K + BK - 1) / BK;   // a K tail (K % 64 != 0, K % 8 == 0) reads zeros

    // ---- tile schedule.  Persistent (tiles > grid): the tiles of XCD x (blocks b, b % 8 == x)
    // are one contiguous range of the logical order, taken round robin by its workgroups, so
    // the tiles in flight on one XCD share A row panels and B column panels in its L2 (the
    // logical order walks groups of `gm` row panels, columns inside a group).  Otherwise one
    // tile per block through the same bijective XCD remap.
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7;
    int lt, lt_end, lt_step;
    const int cnt8 = nwg == tiles ? nwg : tiles;
    const int q8 = cnt8 >> 3, r8 = cnt8 & 7;
    auto xbeg_of = [&](int x) { return x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8; };
    {
        const int xbeg = xbeg_of(xcd);
        if (nwg == tiles) {
            lt = xbeg + (bid >> 3); lt_end = lt + 1; lt_step = 1;
        } else {   // nwg % 8 == 0 (host)
            lt = xbeg + (bid >> 3); lt_end = xbeg + q8 + (xcd < r8 ? 1 : 0); lt_step = nwg >> 3;
        }
    }
    // the current tile's problem: operand / output pointers (scalar selects)
    const bf16* pA = a.A;
    const bf16* pB = a.B;
    auto coords = [&](int t, int& m0, int& n0) {
        const int p = t / ptiles;
        t -= p * ptiles;
        pA = a.A + p * a.sA;
        pB = a.B + p * a.sB;
        const int per = a.gm * ntn, g = t / per, first = g * a.gm;
        const int gs = min(ntm - first, a.gm), rem = t - g * per;
        m0 = (first + rem % gs) * 256;
        n0 = (rem / gs) * 256;
    };

    // ---- LDS-DMA sources.  Wave w fills rows 16 w + 8 j + (lane >> 3) of each half (j = 0, 1),
    // physical chunk lane & 7 <- logical chunk (lane & 7) ^ ((row >> 1) & 7)
    const int lrow0 = 16 * wave + (lane >> 3);             // j = 0; j = 1: + 8
    const int lc0 = (lane & 7) ^ ((lane >> 4) & 7);        // (row >> 1) & 7 for j = 0
    const int lc1 = (lane & 7) ^ (((lane >> 4) + 4) & 7);  // for j = 1
    __amdgpu_buffer_rsrc_t rsA, rsB;
    uint32_t vA[4], vB[4];   // [half][j]
    // conv form: the row's pixel offset and the validity of its 9 taps
    uint32_t tapok[4] = {0, 0, 0, 0};
    auto setup = [&](int m0, int n0) {
        rsB = make_rsrc(pB + (long long)n0 * a.ldb, (long long)(a.N - n0) * a.ldb * 2);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                vB[2 * h + j] = (uint32_t)((128 * h + lrow0 + 8 * j) * a.ldb * 2) + 16u * (j ? lc1 : lc0);
        if constexpr (!CONV) {
            rsA = make_rsrc(pA + (long long)m0 * a.lda, (long long)(a.M - m0) * a.lda * 2);
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    vA[2 * h + j] = (uint32_t)((128 * h + lrow0 + 8 * j) * a.lda * 2) + 16u * (j ? lc1 : lc0);
        } else {
            const int HW = a.H * a.W;
            const int img0 = m0 / HW;
            rsA = make_rsrc(pA + (long long)img0 * HW * a.Cin, (long long)(a.M - img0 * HW) * a.Cin * 2);
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int m = m0 + 128 * h + lrow0 + 8 * j;
                    const int n = m / HW, rem = m - n * HW, y = rem / a.W, x = rem - y * a.W;
                    uint32_t ok = 0;
                    if (m < a.M) {
#pragma unroll
                        for (int t = 0; t < 9; ++t) {
                            const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
                            ok |= (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) ? (1u << t) : 0u;
                        }
                    }
                    tapok[2 * h + j] = ok;
                    vA[2 * h + j] = (uint32_t)(((n - img0) * HW + rem) * a.Cin * 2) + 16u * (j ? lc1 : lc0);
                }
        }
    };
    // per K-step A offsets of the conv form: tap (ky, kx) and channel block c0 of the step
    // (branch-free: an invalid tap's offset is OOB, the DMA then writes zeros)
    auto conv_voff = [&](int i, int t, uint32_t add) -> uint32_t {
        const uint32_t keep = 0u - ((tapok[i] >> t) & 1u);
        return ((vA[i] + add) & keep) | (OOB & ~keep);
    };

    // half h (0 A_lo, 1 A_hi, 2 B_lo, 3 B_hi) of K-step kt into LDS buffer kt & 1
    // the K tail: chunks at k >= K read zeros (OOB) in both operands of the last K-step
    auto ktail = [&](uint32_t v, int kt, int lc) -> uint32_t {
        return kt * BK + 8 * lc < a.K ? v : OOB;
    };
    auto stage = [&](int h, int kt, int ctap, int cc) {
        char* dst = L + (kt & 1) * BUF + h * HALF + 16 * wave * 128;
        const bool tail = TAIL && (kt + 1) * BK > a.K;   // wave-uniform
        if (h >= 2) {
            const uint32_t ko = (uint32_t)kt * (BK * 2);
            uint32_t v0 = vB[2 * (h - 2)] + ko, v1 = vB[2 * (h - 2) + 1] + ko;
            if (tail) { v0 = ktail(v0, kt, lc0); v1 = ktail(v1, kt, lc1); }
            glds(rsB, dst, v0);
            glds(rsB, dst + 8 * 128, v1);
        } else if constexpr (!CONV) {
            const uint32_t ko = (uint32_t)kt * (BK * 2);
            uint32_t v0 = vA[2 * h] + ko, v1 = vA[2 * h + 1] + ko;
            if (tail) { v0 = ktail(v0, kt, lc0); v1 = ktail(v1, kt, lc1); }
            glds(rsA, dst, v0);
            glds(rsA, dst + 8 * 128, v1);
        } else {
            const uint32_t add = (uint32_t)(((ctap / 3 - 1) * a.W + (ctap % 3 - 1)) * a.Cin * 2 + 2 * cc);
            glds(rsA, dst, conv_voff(2 * h, ctap, add));
            glds(rsA, dst + 8 * 128, conv_voff(2 * h + 1, ctap, add));
        }
    };
    // (tap, c0) of K-steps t+1 and t+2 in the conv form, advanced incrementally
    int tap1 = 0, c1 = 0, tap2 = 0, c2 = 0;
    auto adv = [&](int& t, int& c) {
        c += BK;
        if (c >= a.Cin) { c = 0; ++t; }
    };
    // the first two K-steps of a tile: K-step 0 whole, K-step 1 without A_hi (its P0 issues it)
    auto prologue = [&]() {
        stage(2, 0, 0, 0); stage(0, 0, 0, 0); stage(3, 0, 0, 0); stage(1, 0, 0, 0);
        tap1 = 0; c1 = 0;
        if constexpr (CONV) adv(tap1, c1);
        if (nk > 1) { stage(2, 1, tap1, c1); stage(0, 1, tap1, c1); stage(3, 1, tap1, c1); }
        tap2 = tap1; c2 = c1;
        if constexpr (CONV) adv(tap2, c2);
    };

    // ---- fragment read bases (bytes): row R = base + 16 i + (lane & 15), chunk q ^ ((R >> 1) & 7)
    const uint32_t lbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)L;
    const int fr = lane & 15, fq = lane >> 4, fs = (fr >> 1) & 7;
    const uint32_t pa0 = lbase + (uint32_t)((64 * wr + fr) * 128 + 16 * (fq ^ fs));
    const uint32_t pa1 = lbase + (uint32_t)((64 * wr + fr) * 128 + 16 * ((4 + fq) ^ fs));
    const uint32_t pb0 = lbase + (uint32_t)((32 * wc + fr) * 128 + 16 * (fq ^ fs));
    const uint32_t pb1 = lbase + (uint32_t)((32 * wc + fr) * 128 + 16 * ((4 + fq) ^ fs));

    // epilogue addressing: the MFMAs compute C^T tiles (B fragments as the A operand), so
    // accumulator register r of lane l is C[m = .. + (l & 15)][n = .. + 4 (l >> 4) + r]: four
    // consecutive columns of one row, one 8-byte store
    const bool has_r = a.R != nullptr;
    uint2 res[2][4][2];   // residual rows of one row half, [ni][i][j]
    auto load_res = [&](int mi, int m0, int n0) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int m = m0 + 128 * mi + 64 * wr + 16 * i + fr;
                    const int n = n0 + 128 * ni + 32 * wc + 16 * j + 4 * fq;
                    res[ni][i][j] = make_uint2(0u, 0u);
                    if (m < a.M && n < a.N)
                        res[ni][i][j] = *reinterpret_cast<const uint2*>(a.R + (long long)m * a.ldr + n);
                }
    };

    f32x4 acc[2][2][4][2];
    i32x4 fa[8], fb0[4], fb1[4];
    int m0, n0;
    // de-phase the workgroups: with equal tiles every CU would reach its epilogue (HBM-bound
    // stores / residual reads) at the same time and its main loop (MFMA-bound) at the same time
    if (a.delay && ((bid >> 3) & 1)) {
        for (int d = 0; d < a.delay; ++d) __builtin_amdgcn_s_sleep(127);
    }
    coords(lt, m0, n0);
    setup(m0, n0);
    prologue();
    bool first = true;
    while (lt < lt_end) {
        // K-step 0 landed (every wave's DMA: the barrier); K-step 1's three halves and the
        // previous tile's 32 epilogue stores may still be in flight
        if (first) {
            if (nk > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            if (nk > 1) asm volatile("s_waitcnt vmcnt(38)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        }
        first = false;
        barrier();
        if (a.stagger && wr == 1) barrier();   // stagger: waves 4-7 one barrier behind
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[x][y][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

        // a column tile with only its first 128 columns inside N (N = 640 = 2.5 tiles: the res5
        // 3x3 / 1x1 convolutions with 640 outputs): B_hi is all zeros, so the two quadrants
        // against it (P1, P2) are skipped -- their barriers and the A_hi read stay (tile-uniform)
        const bool bhalf = n0 + 128 >= a.N;
        auto kloop = [&](auto bh_) __attribute__((always_inline)) {
        constexpr bool BH = decltype(bh_)::value;
        for (int t = 0; t < nk; ++t) {
            const uint32_t bo = (uint32_t)(t & 1) * BUF;
            const uint32_t a0 = pa0 + bo, a1 = pa1 + bo, b0 = pb0 + bo, b1 = pb1 + bo;
            // P0: B_lo, A_lo -> Q(lo, lo); restage A_hi of K-step t+1
            read_b<2 * HALF>(fb0, b0, b1);
            read_a<0>(fa, a0, a1);
            asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");   // B_lo reads done: restaged in P1
            if (t + 1 < nk) stage(1, t + 1, tap1, c1);
            barrier();
            lgkm_wait12(fa, fb0);
            __builtin_amdgcn_sched_barrier(0);
            mma_quad(acc[0][0], fa, fb0);
            __builtin_amdgcn_sched_barrier(0);
            barrier();
            // P1: B_hi -> Q(lo, hi); restage B_lo of K-step t+2
            if (!BH) read_b<3 * HALF>(fb1, b0, b1);
            if (t + 2 < nk) stage(2, t + 2, tap2, c2);
            barrier();
            if (!BH) {
                lgkm_wait4(fb1);
                __builtin_amdgcn_sched_barrier(0);
                mma_quad(acc[0][1], fa, fb1);
                __builtin_amdgcn_sched_barrier(0);
            }
            barrier();
            // P2: A_hi -> Q(hi, hi); restage A_lo of K-step t+2
            read_a<HALF>(fa, a0, a1);
            if (t + 2 < nk) stage(0, t + 2, tap2, c2);
            barrier();
            lgkm_wait8(fa);
            if (!BH) {
                __builtin_amdgcn_sched_barrier(0);
                mma_quad(acc[1][1], fa, fb1);
                __builtin_amdgcn_sched_barrier(0);
            }
            barrier();
            // P3: -> Q(hi, lo); restage B_hi of K-step t+2; retire K-step t+1
            if (t + 2 < nk) {
                stage(3, t + 2, tap2, c2);
                asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            barrier();
            __builtin_amdgcn_sched_barrier(0);
            mma_quad(acc[1][0], fa, fb0);
            __builtin_amdgcn_sched_barrier(0);
            barrier();
            if constexpr (CONV) { tap1 = tap2; c1 = c2; adv(tap2, c2); }
        }
        };
        if (bhalf) kloop(std::true_type{});
        else kloop(std::false_type{});
        if (a.stagger && wr == 0) barrier();   // close the stagger: every wave is past its last LDS read

        // ---- epilogue of this tile, the next tile's first two K-steps in flight meanwhile
        const int em0 = m0, en0 = n0;
        const int ep = lt / ptiles;
        bf16* const eC = a.C + ep * a.sC;
        const void* const ebias = a.bias ? reinterpret_cast<const char*>(a.bias) + ep * a.sbias * (a.bias_f32 ? 4 : 2)
                                         : nullptr;
        if (has_r) load_res(0, em0, en0);
        float bias[2][2][4];
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int n = en0 + 128 * ni + 32 * wc + 16 * j + 4 * fq;
                f32x4 bv = {0.f, 0.f, 0.f, 0.f};
                if (ebias && n < a.N) {
                    if (a.bias_f32) {
                        bv = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(ebias) + n);
                    } else {
                        const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16*>(ebias) + n);
                        bv = f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                   __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) bias[ni][j][r] = bv[r];
            }
        lt += lt_step;
        if (lt < lt_end) {
            coords(lt, m0, n0);
            setup(m0, n0);
            prologue();
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
            if (mi == 1 && has_r) load_res(1, em0, en0);
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int m = em0 + 128 * mi + 64 * wr + 16 * i + fr;
                    uint2 pk[2];
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        float o[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r) o[r] = acc[mi][ni][i][j][r] + bias[ni][j][r];
                        if (has_r) {
                            const uint2 u = res[ni][i][j];
                            o[0] += __uint_as_float(u.x << 16);
                            o[1] += __uint_as_float(u.x & 0xffff0000u);
                            o[2] += __uint_as_float(u.y << 16);
                            o[3] += __uint_as_float(u.y & 0xffff0000u);
                        }
                        if (a.relu) {
#pragma unroll
                            for (int r = 0; r < 4; ++r) o[r] = fmaxf(o[r], 0.f);
                        }
                        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
                        const bf16x2 lo = {(bf16)o[0], (bf16)o[1]}, hi = {(bf16)o[2], (bf16)o[3]};
                        pk[j] = make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
                    }
                    // 16-row groups fq: j = 0 holds columns 4 fq .. +3, j = 1 holds 16 + 4 fq .. +3.
                    // Swapping the odd groups of j = 0 with the even groups of j = 1 leaves 8
                    // consecutive columns per lane (fq 0: 0-7, 1: 16-23, 2: 8-15, 3: 24-31): one
                    // 16-byte store instead of two 8-byte ones (store issue halves)
                    const auto sx = __builtin_amdgcn_permlane16_swap(pk[0].x, pk[1].x, false, false);
                    const auto sy = __builtin_amdgcn_permlane16_swap(pk[0].y, pk[1].y, false, false);
                    const int c = 4 * (fq & 1) * 4 + 8 * (fq >> 1);   // 0, 16, 8, 24
                    const int n = en0 + 128 * ni + 32 * wc + c;
                    if (m < a.M && n < a.N)
                        *reinterpret_cast<uint4*>(eC + (long long)m * a.ldc + n) =
                            make_uint4(sx[0], sy[0], sx[1], sy[1]);
                }
        }
    }
    if (a.stamp && lane == 0) {
        const long long slot = (long long)blockIdx.x * 8 + (tid >> 6);
        const unsigned long long t_exit = wall_clock64();
        *reinterpret_cast<ulonglong2*>(a.stamp + 2 * slot) = make_ulonglong2(s_t0[tid >> 6], t_exit);
    }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int launch(Gemm256Args a, bool conv, void* stream, bool one_tile = false) {
    const long long tiles = (long long)((a.M + 255) / 256) * ((a.N + 255) / 256) * a.nprob;
    if (tiles <= 0 || tiles > 0x7fffffffLL) return OV3D_EINVAL;
    // persistent grid: one 512-thread workgroup per CU (128 KB of LDS each)
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        cus &= ~7;
        if (cus <= 0) cus = 8;
    }
    static const int gm_env = getenv("OV3D_GEMM256_GM") ? atoi(getenv("OV3D_GEMM256_GM")) : 0;
    const int ntn = (a.N + 255) / 256;
    a.gm = gm_env > 0 ? gm_env : (ntn >= 8 ? 8 : 1);
    static const int st_env = getenv("OV3D_GEMM256_STAGGER") ? atoi(getenv("OV3D_GEMM256_STAGGER")) : 1;
    static const int dl_env = getenv("OV3D_GEMM256_DELAY") ? atoi(getenv("OV3D_GEMM256_DELAY")) : 0;
    a.stagger = st_env;
    a.delay = dl_env;
    // The two-problem launch (the decoder's memory K / V inside the SUN step) runs one tile per
    // workgroup: the step's side-stream FPS holds 8 CUs for milliseconds, and a persistent grid's
    // workgroups queued behind it took their whole tile ranges late (99 us in the step vs 57 us
    // alone, profiles/r05_trace_steady_v1.json); hardware dispatch hands single tiles to the free
    // CUs instead.  OV3D_GEMM256_PAIR_PERSIST=1 keeps the persistent grid.
    static const int pp_env = getenv("OV3D_GEMM256_PAIR_PERSIST") ? atoi(getenv("OV3D_GEMM256_PAIR_PERSIST")) : 0;
    one_tile = one_tile && !pp_env;
    const unsigned grid = (unsigned)(tiles <= cus || one_tile ? tiles : cus);
    // kind 3, work = the launch's flops (2 M N K per problem)
    a.stamp = ov3d_stamp_take(3, 2LL * a.M * a.N * a.K * a.nprob, (long long)grid * 8);
    if (conv)   // Cin % 64 == 0: no K tail
        hipLaunchKernelGGL((gemm256_kernel<true, false>), dim3(grid), dim3(512), 0, ov3d_stream(stream), a);
    else if (a.K % BK)
        hipLaunchKernelGGL((gemm256_kernel<false, true>), dim3(grid), dim3(512), 0, ov3d_stream(stream), a);
    else
        hipLaunchKernelGGL((gemm256_kernel<false, false>), dim3(grid), dim3(512), 0, ov3d_stream(stream), a);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

bool common_ok(const void* B, long long ldb, const void* bias, const void* R, long long ldr,
               const void* C, long long ldc, int M, int N, int K) {
    if (!B || !C || M <= 0 || N <= 0 || K <= 0 || K % 8 || N % 8 || ldc % 8 || ldb % 8 || ldb < K ||
        ldc < N || !aligned16(B) || !aligned16(C))
        return false;
    if (bias && !aligned16(bias)) return false;
    if (R && (ldr % 8 || ldr < N || !aligned16(R))) return false;
    // 32-bit buffer offsets: one tile's operand rows
    if (256LL * ldb * 2 + 2LL * K > 0x7fffffffLL) return false;
    return true;
}

}  // namespace

extern "C" int ov3d_gemm256(const void* A, long long lda, const void* B, long long ldb,
                            const void* bias, int bias_f32, const void* R, long long ldr, void* C,
                            long long ldc, int M, int N, int K, int relu, void* stream) {
    if (!A || lda % 8 || lda < K || !aligned16(A) || 256LL * lda * 2 + 2LL * K > 0x7fffffffLL ||
        !common_ok(B, ldb, bias, R, ldr, C, ldc, M, N, K))
        return OV3D_EINVAL;
    Gemm256Args a{(const bf16*)A, lda, (const bf16*)B, ldb, bias, (const bf16*)R, ldr, (bf16*)C, ldc,
                  M, N, K, bias_f32 ? 1 : 0, relu ? 1 : 0, 0, 0, 0, 1, 1, 0, 1, 0, 0, 0, 0};
    return launch(a, false, stream);
}

extern "C" int ov3d_conv3x3_gemm256(const void* X, int nimg, int H, int W, int Cin, const void* Wt,
                                    long long ldb, const void* bias, int bias_f32, const void* R,
                                    long long ldr, void* Y, long long ldc, int Cout, int relu,
                                    void* stream) {
    if (!X || nimg <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cin % BK || !aligned16(X))
        return OV3D_EINVAL;
    const long long M = (long long)nimg * H * W;
    // pixel offsets and the input extent read by one tile in 32-bit buffer arithmetic
    if (M > 0x7fffffffLL || (long long)(256 + 2 * W + 2 + (long long)H * W) * Cin * 2 > 0x7fffffffLL)
        return OV3D_EINVAL;
    const int K = 9 * Cin;
    if (!common_ok(Wt, ldb, bias, R, ldr, Y, ldc, (int)M, Cout, K)) return OV3D_EINVAL;
    Gemm256Args a{(const bf16*)X, 0, (const bf16*)Wt, ldb, bias, (const bf16*)R, ldr, (bf16*)Y, ldc,
                  (int)M, Cout, K, bias_f32 ? 1 : 0, relu ? 1 : 0, H, W, Cin, 1, 1, 0, 1, 0, 0, 0, 0};
    return launch(a, true, stream);
}

// element offset of q from p (both bf16 / f32 pointers of one address space)
static long long elem_diff(const void* q, const void* p, int esz) {
    return ((long long)(uintptr_t)q - (long long)(uintptr_t)p) / esz;
}

extern "C" int ov3d_gemm256_pair(const void* A, const void* A2, long long lda, const void* B,
                                 const void* B2, long long ldb, const void* bias, const void* bias2,
                                 int bias_f32, void* C, void* C2, long long ldc, int M, int N, int K,
                                 void* stream) {
    if (!A || !A2 || !B2 || !C2 || lda % 8 || lda < K || !aligned16(A) || !aligned16(A2) ||
        !aligned16(B2) || !aligned16(C2) || 256LL * lda * 2 + 2LL * K > 0x7fffffffLL ||
        (bias2 && !aligned16(bias2)) || (!bias) != (!bias2) ||
        !common_ok(B, ldb, bias, nullptr, 0, C, ldc, M, N, K))
        return OV3D_EINVAL;
    Gemm256Args a{(const bf16*)A, lda, (const bf16*)B, ldb, bias, nullptr, 0, (bf16*)C, ldc,
                  M, N, K, bias_f32 ? 1 : 0, 0, 0, 0, 0, 1, 1, 0, 2, elem_diff(A2, A, 2), elem_diff(B2, B, 2),
                  bias ? elem_diff(bias2, bias, bias_f32 ? 4 : 2) : 0, elem_diff(C2, C, 2)};
    return launch(a, false, stream, true);
}

extern "C" int ov3d_gemm256_batched(const void* A, long long lda, long long sA, const void* B,
                                    long long ldb, long long sB, const void* bias, long long sbias,
                                    int bias_f32, void* C, long long ldc, long long sC, int M, int N,
                                    int K, int nbatch, int relu, void* stream) {
    if (!A || nbatch <= 0 || lda % 8 || lda < K || !aligned16(A) || sA % 8 || sB % 8 || sC % 8 ||
        (bias && sbias % (bias_f32 ? 4 : 8)) || 256LL * lda * 2 + 2LL * K > 0x7fffffffLL ||
        !common_ok(B, ldb, bias, nullptr, 0, C, ldc, M, N, K))
        return OV3D_EINVAL;
    Gemm256Args a{(const bf16*)A, lda, (const bf16*)B, ldb, bias, nullptr, 0, (bf16*)C, ldc,
                  M, N, K, bias_f32 ? 1 : 0, relu ? 1 : 0, 0, 0, 0, 1, 1, 0, nbatch, sA, sB, sbias, sC};
    return launch(a, false, stream);
}
