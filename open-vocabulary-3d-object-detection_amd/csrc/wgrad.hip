// Weight + bias gradient of a row-major linear layer (y = x W^T + b over R rows):
//   dW (N, K) = dy^T x,   db (N) = sum_r dy[r, :]
// for every dense layer of the 3DETR step (encoder / decoder projections and FFNs,
// encoder->decoder projection, query projection, heads: models/transformer.py,
// models/helpers.py GenericMLP), where R (points, memory tokens, query slots: 1024 ..
// 16384) is long and N, K <= 768 are small.  Replaces a split-K batched GEMM + an fp32
// sum over the splits + a separate bias reduction (three launches, gemm.py) by one
// kernel:
//   * split-K over row chunks (grid.z), 128 x 128 output tile per workgroup (grid.x, .y),
//     4 waves of 64 x 64 (2 x 2 MFMA 32x32x16 tiles);
//   * both operands are column reads of row-major tiles (dy^T and x): staged in LDS
//     as loaded (coalesced 16-byte row segments) and read with ds_read_b64_tr_b16;
//   * db: the workgroups of output column tile 0 also sum the staged dy rows on the VALU;
//   * split partials (fp32, a few MB, L2/MALL-resident) are summed in split order by a
//     second, chip-wide launch (deterministic); R <= one chunk needs no second launch.
// The grouped launch (every deferred dW of a backward pass) uses 256 x 256 output tiles
// over 8 waves (64 x 128 each), staged by LDS-DMA: a row stage of a 128 x 128 tile moves 64 flop per loaded
// byte and the step's ~95 GFLOP of weight gradients were bound by the per-CU load path
// (~12 B/cycle); 256 x 256 halves the bytes per flop.  Its work is split stream-K style:
// the (problem, tile, 64-row stage) units of all problems, in order, are cut into one
// equal range per CU; a workgroup flushes its accumulators at every tile boundary, straight
// into dW when it owns the whole tile, else into a partial slot that the reduction launch
// adds in workgroup order (deterministic: the cut depends only on the problem list).
#include <type_traits>
#include <vector>

#include <stdlib.h>

#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int TN = 128, TK = 128;  // output tile (rows of dW = N, cols = K)
constexpr int RS = 32;             // rows of dy / x per LDS stage
constexpr int kGroupMax = 28;      // problems per 128 x 128 grouped launch (kernel argument space)
constexpr int LDT = TN + 32;       // padded LDS row (bf16): conflict-free tr16 reads

struct WgradArgs {
    const bf16* dy;
    const bf16* x;
    long long ldy, ldx;
    int R, N, K;
    float* dW;        // (N, K), leading dimension ldw
    long long ldw;
    float* db;        // (N) or null
    float* part;      // (nsplit, N, K) + (nsplit, N) split partials
    int nsplit, rows_per_split;
    int vec_dy, vec_x;  // 16-byte row segments are aligned (row strides % 8 == 0)
    // x = bf16(relu(x_stored * xs + xh)) per channel when xs != null (ov3d_wgrad_bn: the layer's
    // input is the previous layer's BatchNorm + ReLU, applied on load instead of stored)
    const float* xs;
    const float* xh;
};

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x4 tr16(const bf16* p) {
    s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
    return __builtin_bit_cast(bf16x4, r);
}

// operand fragment of a 32-column slice c0 of a [RS][LDT] tile for k-step ks (16 rows):
// lane (col = c0 + (lane & 31), half h) gets rows 16ks + 8h + j, j = 0..7
__device__ __forceinline__ bf16x8 col_frag(const bf16* T, int lane, int c0, int ks) {
    const int g = lane >> 4, i = lane & 15;
    const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
    const int row = 16 * ks + 8 * (g >> 1) + (i >> 2);
    const bf16x4 lo = tr16(T + row * LDT + col);
    const bf16x4 hi = tr16(T + (row + 4) * LDT + col);
    bf16x8 a;
    a[0] = lo[0]; a[1] = lo[1]; a[2] = lo[2]; a[3] = lo[3];
    a[4] = hi[0]; a[5] = hi[1]; a[6] = hi[2]; a[7] = hi[3];
    return a;
}

// ------------------------------------------------------------- 256 x 256 tiles, 8 waves
constexpr int TB = 256;            // output tile edge
constexpr int BK = 64;             // rows per LDS stage
constexpr int STG = BK * TB;       // bf16 elements of one operand's stage image

// LDS image of a stage: [BK rows][32 chunks of 8 bf16], rows unpadded (512 B) and the chunk
// index XOR-swizzled by 4 (row & 3), so the 4 rows a ds_read_b64_tr_b16 touches fall in 4
// different 16-bank groups.  Filled by global_load_lds (one wave-instruction = rows 2j, 2j+1
// lane-linear; the swizzle goes on the per-lane SOURCE address).
__device__ __forceinline__ int swz(int row, int col) {   // element offset of (row, col)
    return row * TB + ((((col >> 3) ^ (4 * (row & 3)))) << 3) + (col & 7);
}

// ds_read_b64_tr_b16 as an asm statement: hipcc's wait tracking treats every LDS read as
// possibly aliasing an in-flight LDS-DMA and would wait vmcnt(0) before it, draining the next
// stage's DMA before this stage is computed.  The asm result is not protected by the
// compiler: the caller passes every result through lgkm_wait6 (an s_waitcnt lgkmcnt(0) that
// takes them as in/out operands, so no use can be scheduled before the wait).
template <int OFF>
__device__ __forceinline__ s16x4 tr16_asm(uint32_t lds_byte_addr) {
    s16x4 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(lds_byte_addr), "i"(OFF) : "memory");
    return r;
}
__device__ __forceinline__ void lgkm_wait6(s16x4 (&v)[12]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]),
                   "+v"(v[6]), "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11])
                 :
                 : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// rows [rbeg, rend) (whole BK-row stages) of the 256 x 256 output tile (bx: N, by: K);
// 512 threads, wave (wn, wk) = (wave >> 1, wave & 1) owns rows 64 wn .. +64 of dW and
// columns 128 wk .. +128.  The tile sums go to dst (leading dimension ld, element
// (n - n0, k - k0) when `local`) and the bias column sums (tiles with by == 0) to bdst.
// Problems here have N, K % 8 == 0, 16-byte aligned rows and R % BK == 0 (sk_ok); the rest
// take the 128 x 128 register-staged group kernel.
template <typename A>   // WgradArgs or the stream-K launch's WgradSK
__device__ __forceinline__ void wgrad_seg256(const A& a, int bx, int by, int rbeg, int rend,
                                             float* dst, size_t ld, bool local, float* bdst,
                                             bf16* L) {
    // the wave index in a scalar register: every per-wave LDS / row base below stays scalar
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave >> 1, wk = wave & 1;
    const int n0 = bx * TB, k0 = by * TB;
    const bool do_bias = a.db != nullptr && by == 0;

    // stage image b: dy at L + 2b STG, x at L + (2b + 1) STG.  32 wave-instructions per
    // operand, 4 per wave: rows 2j, 2j+1 (j = 4 wave + q), lane -> row 2j + (lane >> 5),
    // physical chunk lane & 31, loading the logical chunk the swizzle puts there.  row & 3 =
    // 2q + (lane >> 5) (mod 4): the source column is lane-constant per q (a 32-bit lane
    // offset plus a wave-uniform row base).  Columns past N / K read a clamped in-row chunk:
    // they only feed dW rows / columns that are never stored (and the bias sum skips them).
    const int pc = lane & 31, hl = lane >> 5;
    uint32_t voffD[4], voffX[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int lc = pc ^ (4 * ((2 * q + hl) & 3));
        voffD[q] = (uint32_t)(hl * a.ldy + min(n0 + 8 * lc, a.N - 8)) * 2u;
        voffX[q] = (uint32_t)(hl * a.ldx + min(k0 + 8 * lc, a.K - 8)) * 2u;
    }
    // LDS-DMA needs whole in-range 16-byte row chunks; problems without them (the heads'
    // 3- and 12-wide outputs, unaligned rows, a stage past rend) load per element through
    // registers into the same image (wave-uniform branch)
    const bool dma = a.vec_dy && a.vec_x && (a.N % 8 == 0) && (a.K % 8 == 0);
    auto fill = [&](int b, int r0) {
        bf16* D = L + 2 * b * STG;
        bf16* X = D + STG;
        if (!dma || r0 + BK > rend) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {   // 64 rows x 32 chunks per operand, 4 per thread
                const int idx = tid + 512 * c, row = idx >> 5, ch = idx & 31;
                const int r = r0 + row, n = n0 + 8 * ch, k = k0 + 8 * ch;
                bf16x8 zd, zx;
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) zd[jj] = zx[jj] = (bf16)0.f;
                if (r < rend) {
                    const bf16* pd = a.dy + (size_t)r * a.ldy + n;
                    const bf16* px = a.x + (size_t)r * a.ldx + k;
                    if (a.vec_dy && n + 8 <= a.N) zd = *reinterpret_cast<const bf16x8*>(pd);
                    else
                        for (int jj = 0; jj < 8; ++jj) zd[jj] = n + jj < a.N ? pd[jj] : (bf16)0.f;
                    if (a.vec_x && k + 8 <= a.K) zx = *reinterpret_cast<const bf16x8*>(px);
                    else
                        for (int jj = 0; jj < 8; ++jj) zx[jj] = k + jj < a.K ? px[jj] : (bf16)0.f;
                }
                *reinterpret_cast<bf16x8*>(&D[swz(row, 8 * ch)]) = zd;
                *reinterpret_cast<bf16x8*>(&X[swz(row, 8 * ch)]) = zx;
            }
            return;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = 4 * wave + q, row0 = r0 + 2 * j;   // wave-uniform
            const char* gd = reinterpret_cast<const char*>(a.dy + (size_t)row0 * a.ldy) + voffD[q];
            const char* gx = reinterpret_cast<const char*>(a.x + (size_t)row0 * a.ldx) + voffX[q];
            __builtin_amdgcn_global_load_lds(gd, (__attribute__((address_space(3))) void*)(D + 2 * j * TB), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(gx, (__attribute__((address_space(3))) void*)(X + 2 * j * TB), 16, 0, 0);
        }
    };
    // column fragment (lane: column c0 + 16(g&1) + 4(i&3), rows 16 ks + 8(g>>1) + (i>>2) + {0,4})
    // of the swizzled image: row & 3 = i >> 2 for every k-step, so the swizzled byte offset
    // of a 32-column slice c0 is lane-constant; k-step and +4-row halves are immediates
    const int fg = lane >> 4, fi = lane & 15;
    auto foff = [&](int c0) {
        return (uint32_t)((8 * (fg >> 1) + (fi >> 2)) * TB +
                          (((c0 >> 3) ^ (4 * (fi >> 2))) + 2 * (fg & 1) + ((fi & 3) >> 1)) * 8 + 4 * (fi & 1)) * 2u;
    };
    const uint32_t lbase = lds_addr(L);
    uint32_t offD[2], offX[4];
#pragma unroll
    for (int t = 0; t < 2; ++t) offD[t] = lbase + foff(64 * wn + 32 * t);
#pragma unroll
    for (int t = 0; t < 4; ++t) offX[t] = lbase + STG * 2u + foff(128 * wk + 32 * t);

    f32x16 acc[2][4];
#pragma unroll
    for (int tn = 0; tn < 2; ++tn)
#pragma unroll
        for (int tk = 0; tk < 4; ++tk)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[tn][tk][i] = 0.f;
    float bsum[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bsum[j] = 0.f;
    const bool bias_cols = do_bias && n0 + 8 * (tid & 31) < a.N;

    auto kstep = [&](const uint32_t (&ad)[2], const uint32_t (&ax)[4], auto ksc) {
        constexpr int KS = decltype(ksc)::value;
        constexpr int O0 = 16 * KS * TB * 2, O1 = O0 + 4 * TB * 2;
        s16x4 v[12];   // halves: dy slices 0, 1 then x slices 0..3, (lo, hi) each
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            v[2 * t] = tr16_asm<O0>(ad[t]);
            v[2 * t + 1] = tr16_asm<O1>(ad[t]);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            v[4 + 2 * t] = tr16_asm<O0>(ax[t]);
            v[4 + 2 * t + 1] = tr16_asm<O1>(ax[t]);
        }
        lgkm_wait6(v);
        bf16x8 af[2], bfr[4];
#pragma unroll
        for (int t = 0; t < 2; ++t)
            af[t] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v[2 * t], v[2 * t + 1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int t = 0; t < 4; ++t)
            bfr[t] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v[4 + 2 * t], v[5 + 2 * t], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int tn = 0; tn < 2; ++tn)
#pragma unroll
            for (int tk = 0; tk < 4; ++tk) acc[tn][tk] = mfma(af[tn], bfr[tk], acc[tn][tk]);
    };
    auto compute = [&](int b) {
        const uint32_t sb = (uint32_t)b * 4u * STG;   // byte offset of stage b
        const uint32_t ad[2] = {offD[0] + sb, offD[1] + sb};
        const uint32_t ax[4] = {offX[0] + sb, offX[1] + sb, offX[2] + sb, offX[3] + sb};
        kstep(ad, ax, std::integral_constant<int, 0>());
        kstep(ad, ax, std::integral_constant<int, 1>());
        kstep(ad, ax, std::integral_constant<int, 2>());
        kstep(ad, ax, std::integral_constant<int, 3>());
        if (bias_cols) {   // thread: 8 adjacent columns (tid & 31) x rows (tid >> 5) + 16 rr
            const bf16* D = L + 2 * b * STG;
#pragma unroll
            for (int rr = 0; rr < BK / 16; ++rr) {
                const bf16x8 v = *reinterpret_cast<const bf16x8*>(&D[swz((tid >> 5) + 16 * rr, 8 * (tid & 31))]);
#pragma unroll
                for (int j = 0; j < 8; ++j) bsum[j] += (float)v[j];
            }
        }
    };

    // two LDS stages: the DMA of stage s+1 flies while stage s is computed; the barrier's
    // vmcnt(0) retires it (cdna_hip_programming.md section 5, glds vs register staging)
    __syncthreads();   // the previous segment's last reads of the images are done
    fill(0, rbeg);
    __syncthreads();
    int b = 0;
    for (int r = rbeg; r < rend; r += BK, b ^= 1) {
        if (r + BK < rend) fill(b ^ 1, r + BK);
        compute(b);
        __syncthreads();
    }

    // column sums: 16 row-threads per 8-column group -> LDS -> 256 values
    float* bred = reinterpret_cast<float*>(L);   // 512 x 8 floats, free after the loop
    static_assert(4 * STG * sizeof(bf16) >= 512 * 8 * sizeof(float), "column-sum staging overruns the stage images");
    if (do_bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bred[tid * 8 + j] = bsum[j];
    }
    __syncthreads();
    if (do_bias && tid < TB && n0 + tid < a.N) {
        const int cg = tid >> 3, j = tid & 7;
        float bcol = 0.f;   // column n0 + tid
        for (int rt = 0; rt < 16; ++rt) bcol += bred[(rt * 32 + cg) * 8 + j];
        bdst[local ? tid : n0 + tid] = bcol;
    }
    const int h = lane >> 5, cl = lane & 31;
#pragma unroll
    for (int tn = 0; tn < 2; ++tn)
#pragma unroll
        for (int tk = 0; tk < 4; ++tk) {
            const int k = k0 + 128 * wk + 32 * tk + cl;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int n = n0 + 64 * wn + 32 * tn + (i & 3) + 8 * (i >> 2) + 4 * h;
                if (n < a.N && k < a.K) {
                    if (local) dst[(size_t)(n - n0) * ld + (k - k0)] = acc[tn][tk][i];
                    else dst[(size_t)n * ld + k] = acc[tn][tk][i];
                }
            }
        }
}

// one 128 x 128 output tile (bx, by) of one row split
__device__ __forceinline__ void wgrad_body(const WgradArgs& a, int bx, int by, int split) {
    __shared__ __attribute__((aligned(16))) bf16 Ds[2][RS * LDT];
    __shared__ __attribute__((aligned(16))) bf16 Xs[2][RS * LDT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wn = wave >> 1, wk = wave & 1;
    const int n0 = bx * TN, k0 = by * TK;
    const int rbeg = split * a.rows_per_split;
    const int rend = min(a.R, rbeg + a.rows_per_split);
    // db: the workgroups of output column tile 0 also sum their dy stage tile over its
    // rows on the VALU (thread: 8 adjacent columns x 2 rows per stage)
    const bool do_bias = a.db != nullptr && by == 0;

    // ov3d_wgrad_bn: the thread's 8 x channels (k0 + 8 (tid & 15) ..) are the same in every
    // stage: their BN coefficients in registers (zeros past K: those columns are never stored)
    float xsc[8], xsh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xsc[j] = xsh[j] = 0.f;
    if (a.xs) {
        const int kx = k0 + 8 * (tid & 15);
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (kx + j < a.K) {
                xsc[j] = a.xs[kx + j];
                xsh[j] = a.xh[kx + j];
            }
    }
    // stage loader: RS rows x 16 chunks (16 B) per operand = 512 chunks, 2 per thread.
    // Two register sets: stage n+2 is in flight while stage n is computed and stage n+1
    // waits in the other set (a stage is only 4-6 MFMAs per wave, too short to cover a
    // global load).
    auto load = [&](bf16x8 (&dr)[2], bf16x8 (&xr)[2], int r0) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int idx = tid + 256 * c, row = r0 + (idx >> 4), ch = idx & 15;
            const int n = n0 + 8 * ch, k = k0 + 8 * ch;
            bf16x8 zd, zx;
#pragma unroll
            for (int j = 0; j < 8; ++j) zd[j] = zx[j] = (bf16)0.f;
            if (row < rend) {
                const bf16* pd = a.dy + (size_t)row * a.ldy + n;
                const bf16* px = a.x + (size_t)row * a.ldx + k;
                if (a.vec_dy && n + 8 <= a.N) zd = *reinterpret_cast<const bf16x8*>(pd);
                else
                    for (int j = 0; j < 8; ++j) zd[j] = n + j < a.N ? pd[j] : (bf16)0.f;
                if (a.vec_x && k + 8 <= a.K) zx = *reinterpret_cast<const bf16x8*>(px);
                else
                    for (int j = 0; j < 8; ++j) zx[j] = k + j < a.K ? px[j] : (bf16)0.f;
            }
            dr[c] = zd;
            xr[c] = zx;
        }
    };
    // ov3d_wgrad_bn: the BN + ReLU (ov3d_rows_bn_apply's arithmetic) here, when the stage's
    // registers have long landed (in the loader it would wait for every load at once); rows past
    // rend stay zero
    auto store = [&](const bf16x8 (&dr)[2], const bf16x8 (&xr)[2], int buf, int r0) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int idx = tid + 256 * c, row = idx >> 4, ch = idx & 15;
            bf16x8 xv = xr[c];
            if (a.xs && r0 + row < rend) {
#pragma unroll
                for (int j = 0; j < 8; ++j) xv[j] = (bf16)fmaxf(fmaf((float)xv[j], xsc[j], xsh[j]), 0.f);
            }
            *reinterpret_cast<bf16x8*>(&Ds[buf][row * LDT + 8 * ch]) = dr[c];
            *reinterpret_cast<bf16x8*>(&Xs[buf][row * LDT + 8 * ch]) = xv;
        }
    };

    f32x16 acc[2][2];
    float bsum[8];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[0][0][i] = acc[0][1][i] = acc[1][0][i] = acc[1][1][i] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) bsum[j] = 0.f;

    auto compute = [&](int buf) {
#pragma unroll
        for (int ks = 0; ks < RS / 16; ++ks) {
            bf16x8 af[2], bfr[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                af[t] = col_frag(Ds[buf], lane, 64 * wn + 32 * t, ks);
                bfr[t] = col_frag(Xs[buf], lane, 64 * wk + 32 * t, ks);
            }
#pragma unroll
            for (int tn = 0; tn < 2; ++tn)
#pragma unroll
                for (int tk = 0; tk < 2; ++tk) acc[tn][tk] = mfma(af[tn], bfr[tk], acc[tn][tk]);
        }
        if (do_bias) {
#pragma unroll
            for (int rr = 0; rr < RS / 16; ++rr) {
                const bf16x8 v = *reinterpret_cast<const bf16x8*>(
                    &Ds[buf][((tid >> 4) + 16 * rr) * LDT + 8 * (tid & 15)]);
#pragma unroll
                for (int j = 0; j < 8; ++j) bsum[j] += (float)v[j];
            }
        }
    };

    bf16x8 dA[2], xA[2], dB[2], xB[2];
    if (rbeg < rend) {
        load(dA, xA, rbeg);
        store(dA, xA, 0, rbeg);
        if (rbeg + RS < rend) load(dA, xA, rbeg + RS);
    }
    __syncthreads();
    for (int r = rbeg; r < rend;) {
        // LDS buffer 0 holds stage r, set A holds stage r + RS
        if (r + 2 * RS < rend) load(dB, xB, r + 2 * RS);
        compute(0);
        if (r + RS < rend) store(dA, xA, 1, r + RS);
        __syncthreads();
        r += RS;
        if (r >= rend) break;
        // LDS buffer 1 holds stage r, set B holds stage r + RS
        if (r + 2 * RS < rend) load(dA, xA, r + 2 * RS);
        compute(1);
        if (r + RS < rend) store(dB, xB, 0, r + RS);
        __syncthreads();
        r += RS;
    }

    // column sums of this split: 16 row-threads per 8-column group -> LDS -> 128 values
    float* bred = reinterpret_cast<float*>(&Xs[0][0]);   // 256 x 8 floats, free after the loop
    static_assert(sizeof(Xs) >= 256 * 8 * sizeof(float), "column-sum staging overruns Xs");
    if (do_bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bred[tid * 8 + j] = bsum[j];
    }
    __syncthreads();
    float bcol = 0.f;   // thread t < 128: column n0 + t
    if (do_bias && tid < TN) {
        const int cg = tid >> 3, j = tid & 7;
        for (int rt = 0; rt < 16; ++rt) bcol += bred[(rt * 16 + cg) * 8 + j];
    }
    // accumulator element i of lane: row (n) = (i&3) + 8(i>>2) + 4h, col (k) = lane & 31
    const int h = lane >> 5, cl = lane & 31;
    const size_t NK = (size_t)a.N * a.K;
    if (a.nsplit == 1) {
#pragma unroll
        for (int tn = 0; tn < 2; ++tn)
#pragma unroll
            for (int tk = 0; tk < 2; ++tk) {
                const int k = k0 + 64 * wk + 32 * tk + cl;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int n = n0 + 64 * wn + 32 * tn + (i & 3) + 8 * (i >> 2) + 4 * h;
                    if (n < a.N && k < a.K) a.dW[(size_t)n * a.ldw + k] = acc[tn][tk][i];
                }
            }
        if (do_bias && tid < TN && n0 + tid < a.N) a.db[n0 + tid] = bcol;
        return;
    }
    // split partials
    float* pw = a.part + (size_t)split * NK;
    float* pb = a.part + (size_t)a.nsplit * NK + (size_t)split * a.N;
#pragma unroll
    for (int tn = 0; tn < 2; ++tn)
#pragma unroll
        for (int tk = 0; tk < 2; ++tk) {
            const int k = k0 + 64 * wk + 32 * tk + cl;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int n = n0 + 64 * wn + 32 * tn + (i & 3) + 8 * (i >> 2) + 4 * h;
                if (n < a.N && k < a.K) pw[(size_t)n * a.K + k] = acc[tn][tk][i];
            }
        }
    if (do_bias && tid < TN && n0 + tid < a.N) pb[n0 + tid] = bcol;
}

// dW / db = sum of the split partials in split order (deterministic).  One thread per
// output element (coalesced across threads), 8 split loads in flight per thread.
__device__ __forceinline__ void wgrad_reduce_body(const WgradArgs& a, long long t) {
    const size_t NK = (size_t)a.N * a.K;
    const float* p;
    size_t stride;
    if (t < (long long)NK) {
        p = a.part + t;
        stride = NK;
    } else if (a.db != nullptr && t < (long long)NK + a.N) {
        p = a.part + (size_t)a.nsplit * NK + (t - NK);
        stride = a.N;
    } else {
        return;
    }
    float acc = 0.f;
    int sp = 0;
    for (; sp + 8 <= a.nsplit; sp += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[(size_t)(sp + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; sp < a.nsplit; ++sp) acc += p[(size_t)sp * stride];
    if (t < (long long)NK) {
        const int n = (int)(t / a.K), k = (int)(t - (long long)n * a.K);
        a.dW[(size_t)n * a.ldw + k] = acc;
    } else {
        a.db[t - NK] = acc;
    }
}

__global__ void __launch_bounds__(256, 2) wgrad_kernel(WgradArgs a) {
    wgrad_body(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

__global__ void __launch_bounds__(256) wgrad_reduce_kernel(WgradArgs a) {
    wgrad_reduce_body(a, (long long)blockIdx.x * blockDim.x + threadIdx.x);
}

// Grouped problems the stream-K kernel does not take (N or K % 8 != 0, unaligned rows,
// R % 64 != 0; the heads' 3- and 12-wide outputs): 128 x 128 tiles, fixed row splits,
// problem i owns workgroups [blk[i], blk[i+1]).
struct WgradGroup128 {
    WgradArgs p[kGroupMax];
    int blk[kGroupMax + 1];
    int red[kGroupMax + 1];   // reduce: workgroups [red[i], red[i+1]) of problem i
    int n;
};
static_assert(sizeof(WgradGroup128) <= 4000, "kernel argument space");

__global__ void __launch_bounds__(256, 2) wgrad_group128_kernel(WgradGroup128 g) {
    const int b = blockIdx.x;
    int i = 0;
    while (i + 1 < g.n && b >= g.blk[i + 1]) ++i;
    const WgradArgs& a = g.p[i];
    const int tn = (a.N + TN - 1) / TN, tk = (a.K + TK - 1) / TK;
    const int local = b - g.blk[i];
    wgrad_body(a, local % tn, (local / tn) % tk, local / (tn * tk));
}

__global__ void __launch_bounds__(256) wgrad_group128_reduce_kernel(WgradGroup128 g) {
    const int b = blockIdx.x;
    int i = 0;
    while (i + 1 < g.n && b >= g.red[i + 1]) ++i;
    if (b >= g.red[i + 1] || b < g.red[i]) return;
    wgrad_reduce_body(g.p[i], (long long)(b - g.red[i]) * blockDim.x + threadIdx.x);
}


// Several independent weight gradients in one launch (the deferred dW / db of a whole
// backward pass, gemm.py), stream-K over the units (problem, 256 x 256 tile, 64-row stage).
constexpr int kSlot = TB * TB + TB;   // floats of one partial slot: tile + bias columns
// a stream-K launch's problem: WgradArgs without the split fields, 32-bit strides (64 bytes),
// so 48 problems fit the argument space (28 with WgradArgs: the step's ~100 deferred weight
// gradients took 4 launches + 4 reductions)
struct WgradSK {
    const bf16* dy;
    const bf16* x;
    float* dW;
    float* db;
    int ldy, ldx, ldw;
    int R, N, K;
    int vec_dy, vec_x;
};
static_assert(sizeof(WgradSK) == 64, "compact stream-K problem");
constexpr int kSKMax = 48;   // problems per stream-K launch
struct WgradGroup {
    WgradSK p[kSKMax];
    long long ubeg[kSKMax + 1];   // first unit of problem i
    int sbeg[kSKMax + 1];         // first partial slot of problem i
    int tbeg[kSKMax + 1];         // first tile of problem i (reduction grid)
    int n, G;
    float* part;                  // partial slots, kSlot floats each
};
static_assert(sizeof(WgradGroup) <= 4000, "kernel argument space");

template <typename A>
__host__ __device__ inline int sk_tiles_n(const A& a) { return (a.N + TB - 1) / TB; }
template <typename A>
__host__ __device__ inline int sk_tiles(const A& a) { return sk_tiles_n(a) * ((a.K + TB - 1) / TB); }
template <typename A>
__host__ __device__ inline int sk_stages(const A& a) { return (a.R + BK - 1) / BK; }
// first unit of workgroup w / the workgroup owning unit u (ranges floor(U w / G))
__host__ __device__ inline long long sk_start(long long U, int G, int w) { return U * w / G; }
__host__ __device__ inline int sk_owner(long long U, int G, long long u) {
    return (int)(((u + 1) * G - 1) / U);
}
// slots used by tile t of problem i (0 when one workgroup owns the whole tile)
__host__ __device__ inline int sk_tile_slots(const WgradGroup& g, int i, int t, long long U) {
    const int st = sk_stages(g.p[i]);
    const long long uf = g.ubeg[i] + (long long)t * st, ul = uf + st - 1;
    const int wf = sk_owner(U, g.G, uf), wl = sk_owner(U, g.G, ul);
    return wf == wl ? 0 : wl - wf + 1;
}

__global__ void __launch_bounds__(512, 1) wgrad_group_kernel(WgradGroup g) {
    // all LDS in ONE array: dy / x images of the two stages
    __shared__ __attribute__((aligned(16))) bf16 L[4 * STG];
    const long long U = g.ubeg[g.n];
    const int w = blockIdx.x;
    long long u = sk_start(U, g.G, w);
    const long long u1 = sk_start(U, g.G, w + 1);
    int i = 0;
    while (u < u1) {
        while (u >= g.ubeg[i + 1]) ++i;
        const WgradSK& a = g.p[i];
        const int st = sk_stages(a), tn = sk_tiles_n(a);
        const long long local = u - g.ubeg[i];
        const int t = (int)(local / st), s0 = (int)(local - (long long)t * st);
        const int s1 = (int)min((long long)st, s0 + (u1 - u));
        const int rbeg = s0 * BK, rend = min(a.R, s1 * BK);
        const long long uf = g.ubeg[i] + (long long)t * st;
        const int wf = sk_owner(U, g.G, uf), wl = sk_owner(U, g.G, uf + st - 1);
        if (wf == wl) {
            wgrad_seg256(a, t % tn, t / tn, rbeg, rend, a.dW, a.ldw, false, a.db, L);
        } else {
            int slot = g.sbeg[i];
            for (int tt = 0; tt < t; ++tt) slot += sk_tile_slots(g, i, tt, U);
            float* ps = g.part + (size_t)(slot + (w - wf)) * kSlot;
            wgrad_seg256(a, t % tn, t / tn, rbeg, rend, ps, TB, true, ps + TB * TB, L);
        }
        u += s1 - s0;
    }
}

// split tiles: dW / db = the tile's partial slots summed in workgroup order.  Block b: tile
// b / 65 (all tiles of the launch), part b % 65 (64 x 1024 tile elements, then the bias)
__global__ void __launch_bounds__(256) wgrad_group_reduce_kernel(WgradGroup g) {
    const long long U = g.ubeg[g.n];
    const int gt = blockIdx.x / 65, sub = blockIdx.x - gt * 65;
    int i = 0;
    while (i + 1 < g.n && gt >= g.tbeg[i + 1]) ++i;
    const WgradSK& a = g.p[i];
    const int t = gt - g.tbeg[i];
    const int nsl = sk_tile_slots(g, i, t, U);
    if (nsl == 0) return;
    int slot = g.sbeg[i];
    for (int tt = 0; tt < t; ++tt) slot += sk_tile_slots(g, i, tt, U);
    const int tn = sk_tiles_n(a);
    const int n0 = (t % tn) * TB, k0 = (t / tn) * TB;
    const float* ps = g.part + (size_t)slot * kSlot;
    if (sub == 64) {
        const int c = threadIdx.x;
        if (a.db == nullptr || k0 != 0 || n0 + c >= a.N) return;
        float acc = 0.f;
        int sl = 0;
        for (; sl + 4 <= nsl; sl += 4) {   // four loads in flight, summed in slot order
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = ps[(size_t)(sl + u) * kSlot + TB * TB + c];
#pragma unroll
            for (int u = 0; u < 4; ++u) acc += v[u];
        }
        for (; sl < nsl; ++sl) acc += ps[(size_t)sl * kSlot + TB * TB + c];
        a.db[n0 + c] = acc;
        return;
    }
    const int e = sub * 1024 + threadIdx.x * 4;   // 4 adjacent columns of one tile row
    const int nl = e / TB, kl = e - nl * TB;
    if (n0 + nl >= a.N || k0 + kl >= a.K) return;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    auto add = [&](const float4& v) {
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
    };
    int sl = 0;
    for (; sl + 4 <= nsl; sl += 4) {   // four slots' loads in flight, summed in slot order
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(ps + (size_t)(sl + u) * kSlot + e);
#pragma unroll
        for (int u = 0; u < 4; ++u) add(v[u]);
    }
    for (; sl < nsl; ++sl) add(*reinterpret_cast<const float4*>(ps + (size_t)sl * kSlot + e));
    float* d = a.dW + (size_t)(n0 + nl) * a.ldw + k0 + kl;
    const float o[4] = {acc.x, acc.y, acc.z, acc.w};
    for (int j = 0; j < 4 && k0 + kl + j < a.K; ++j) d[j] = o[j];
}

}  // namespace

extern "C" long long ov3d_wgrad_workspace(int R, int N, int K, int nsplit) {
    if (nsplit <= 1) return 0;
    return (long long)nsplit * ((long long)N * K + N);
}

extern "C" int ov3d_wgrad_tiles(int N, int K) { return ((N + TN - 1) / TN) * ((K + TK - 1) / TK); }

/* output tiles of one problem in ov3d_wgrad_group (256 x 256 tiles) */
extern "C" int ov3d_wgrad_group_tiles(int N, int K) { return ((N + TB - 1) / TB) * ((K + TB - 1) / TB); }

static int make_args(WgradArgs& a, const void* dy, long long ldy, const void* x, long long ldx,
                     int R, int N, int K, float* dW, long long ldw, float* db, float* workspace,
                     int nsplit) {
    if (!dy || !x || !dW || R <= 0 || N <= 0 || K <= 0 || ldy < N || ldx < K || ldw < K ||
        nsplit <= 0)
        return OV3D_EINVAL;
    int rps = (R + nsplit - 1) / nsplit;
    rps = (rps + RS - 1) / RS * RS;
    nsplit = (R + rps - 1) / rps;
    if (nsplit > 1 && !workspace) return OV3D_EINVAL;
    a.dy = (const bf16*)dy;
    a.x = (const bf16*)x;
    a.ldy = ldy;
    a.ldx = ldx;
    a.R = R;
    a.N = N;
    a.K = K;
    a.dW = dW;
    a.ldw = ldw;
    a.db = db;
    a.part = workspace;
    a.nsplit = nsplit;
    a.rows_per_split = rps;
    a.vec_dy = (ldy % 8 == 0) && ((uintptr_t)dy % 16 == 0);
    a.vec_x = (ldx % 8 == 0) && ((uintptr_t)x % 16 == 0);
    a.xs = nullptr;
    a.xh = nullptr;
    return OV3D_OK;
}

namespace {
int wgrad_launch(const void* dy, long long ldy, const void* x, long long ldx, int R, int N, int K,
                 float* dW, long long ldw, float* db, float* workspace, int nsplit,
                 const float* xs, const float* xh, void* stream) {
    WgradArgs a;
    const int rc = make_args(a, dy, ldy, x, ldx, R, N, K, dW, ldw, db, workspace, nsplit);
    if (rc != OV3D_OK) return rc;
    if (xs || xh) {
        if (!xs || !xh || K % 8 || !a.vec_x) return OV3D_EINVAL;
        a.xs = xs;
        a.xh = xh;
    }
    nsplit = a.nsplit;
    dim3 grid((N + TN - 1) / TN, (K + TK - 1) / TK, nsplit);
    hipStream_t st = ov3d_stream(stream);
    wgrad_kernel<<<grid, 256, 0, st>>>(a);
    OV3D_LAUNCH_CHECK();
    if (nsplit > 1) {
        const long long threads = (long long)N * K + (db ? N : 0);
        wgrad_reduce_kernel<<<ov3d_cdiv(threads, 256), 256, 0, st>>>(a);
        OV3D_LAUNCH_CHECK();
    }
    return OV3D_OK;
}
}  // namespace

extern "C" int ov3d_wgrad(const void* dy, long long ldy, const void* x, long long ldx, int R, int N,
                          int K, float* dW, long long ldw, float* db, float* workspace,
                          int* counters, int nsplit, void* stream) {
    (void)counters;
    return wgrad_launch(dy, ldy, x, ldx, R, N, K, dW, ldw, db, workspace, nsplit, nullptr, nullptr,
                        stream);
}

extern "C" int ov3d_wgrad_bn(const void* dy, long long ldy, const void* x, long long ldx, int R,
                             int N, int K, const float* scale, const float* shift, float* dW,
                             long long ldw, float* db, float* workspace, int* counters, int nsplit,
                             void* stream) {
    (void)counters;
    if (!scale || !shift) return OV3D_EINVAL;
    return wgrad_launch(dy, ldy, x, ldx, R, N, K, dW, ldw, db, workspace, nsplit, scale, shift,
                        stream);
}

// stream-K plan of problems [first, first + g.n): units, slot and tile prefixes, grid
static int cu_count() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            cus = n;
        else
            cus = 256;
        // OV3D_WGRAD_WGS: workgroups of the stream-K launch (measurement knob; default one
        // per CU)
        if (const char* e = getenv("OV3D_WGRAD_WGS")) {
            const int v = atoi(e);
            if (v > 0) cus = v;
        }
    }
    return cus;
}

// problems per stream-K launch: kSKMax; OV3D_WGRAD_SK_MAX (1 .. kSKMax) for A/B runs (28: the
// round-5 split)
static int sk_max() {
    static int m = 0;
    if (!m) {
        m = kSKMax;
        if (const char* e = getenv("OV3D_WGRAD_SK_MAX")) {
            const int v = atoi(e);
            if (v >= 1 && v <= kSKMax) m = v;
        }
    }
    return m;
}

static bool sk_ok(const ov3d_wgrad_problem& q) {
    (void)q;   // every problem: the stream-K kernel loads unaligned / narrow rows per element
    return true;
}

// stream-K plan of the problems idx[first .. first + g.n): units, slot and tile prefixes, grid
static int plan_group(WgradGroup& g, const ov3d_wgrad_problem* probs, const int* idx, int first,
                      int n, long long& slots) {
    g.n = n - first < sk_max() ? n - first : sk_max();
    long long U = 0;
    int tiles = 0;
    for (int j = 0; j < g.n; ++j) {
        const ov3d_wgrad_problem& q = probs[idx[first + j]];
        WgradArgs f;
        const int rc = make_args(f, q.dy, q.ldy, q.x, q.ldx, q.R, q.N, q.K, q.dW, q.ldw, q.db,
                                 nullptr, 1);
        if (rc != OV3D_OK) return rc;
        if (f.ldy >= (1LL << 31) || f.ldx >= (1LL << 31) || f.ldw >= (1LL << 31)) return OV3D_EINVAL;
        g.p[j] = WgradSK{f.dy, f.x, f.dW, f.db, (int)f.ldy, (int)f.ldx, (int)f.ldw, f.R, f.N, f.K,
                         f.vec_dy, f.vec_x};
        g.ubeg[j] = U;
        g.tbeg[j] = tiles;
        U += (long long)sk_tiles(g.p[j]) * sk_stages(g.p[j]);
        tiles += sk_tiles(g.p[j]);
    }
    g.ubeg[g.n] = U;
    g.tbeg[g.n] = tiles;
    g.G = (int)(U < cu_count() ? U : cu_count());
    int sl = 0;
    for (int j = 0; j < g.n; ++j) {
        g.sbeg[j] = sl;
        for (int t = 0; t < sk_tiles(g.p[j]); ++t) sl += sk_tile_slots(g, j, t, U);
    }
    g.sbeg[g.n] = sl;
    slots = sl;
    return OV3D_OK;
}

// workspace floats: [stream-K partial slots of the largest launch | fallback split partials]
static long long group_space(const ov3d_wgrad_problem* probs, int n, long long* sk_part) {
    std::vector<int> sk;
    long long fb = 0;
    for (int i = 0; i < n; ++i) {
        if (sk_ok(probs[i])) sk.push_back(i);
        else fb += ov3d_wgrad_workspace(probs[i].R, probs[i].N, probs[i].K, probs[i].nsplit);
    }
    long long most = 0;
    for (int first = 0; first < (int)sk.size(); first += sk_max()) {
        WgradGroup g;
        long long slots = 0;
        if (plan_group(g, probs, sk.data(), first, (int)sk.size(), slots) != OV3D_OK) return -1;
        most = slots > most ? slots : most;
    }
    *sk_part = most * kSlot;
    return most * kSlot + fb;
}

/* floats of workspace for ov3d_wgrad_group (the launches of one call run in stream order) */
extern "C" long long ov3d_wgrad_group_workspace(const ov3d_wgrad_problem* probs, int n) {
    if (!probs || n <= 0) return 0;
    long long skp = 0;
    const long long w = group_space(probs, n, &skp);
    return w < 0 ? 0 : w;
}

extern "C" int ov3d_wgrad_group(const ov3d_wgrad_problem* probs, int n, float* workspace,
                                void* stream) {
    if (!probs || n <= 0) return OV3D_EINVAL;
    hipStream_t st = ov3d_stream(stream);
    long long skp = 0;
    const long long need = group_space(probs, n, &skp);
    if (need < 0) return OV3D_EINVAL;
    if (need > 0 && !workspace) return OV3D_EINVAL;
    std::vector<int> sk, fb;
    for (int i = 0; i < n; ++i) (sk_ok(probs[i]) ? sk : fb).push_back(i);
    for (int first = 0; first < (int)sk.size(); first += sk_max()) {
        WgradGroup g;
        long long slots = 0;
        const int rc = plan_group(g, probs, sk.data(), first, (int)sk.size(), slots);
        if (rc != OV3D_OK) return rc;
        g.part = workspace;
        if (g.G <= 0) continue;
        wgrad_group_kernel<<<g.G, 512, 0, st>>>(g);
        OV3D_LAUNCH_CHECK();
        if (slots > 0) {
            wgrad_group_reduce_kernel<<<g.tbeg[g.n] * 65, 256, 0, st>>>(g);
            OV3D_LAUNCH_CHECK();
        }
    }
    long long woff = skp;
    for (int first = 0; first < (int)fb.size(); first += kGroupMax) {
        WgradGroup128 g;
        g.n = (int)fb.size() - first < kGroupMax ? (int)fb.size() - first : kGroupMax;
        int blk = 0, red = 0;
        for (int j = 0; j < g.n; ++j) {
            const ov3d_wgrad_problem& q = probs[fb[first + j]];
            const long long ws = ov3d_wgrad_workspace(q.R, q.N, q.K, q.nsplit);
            const int rc = make_args(g.p[j], q.dy, q.ldy, q.x, q.ldx, q.R, q.N, q.K, q.dW, q.ldw,
                                     q.db, ws > 0 ? workspace + woff : nullptr, q.nsplit);
            if (rc != OV3D_OK) return rc;
            woff += ws;
            g.blk[j] = blk;
            g.red[j] = red;
            blk += ((q.N + TN - 1) / TN) * ((q.K + TK - 1) / TK) * g.p[j].nsplit;
            if (g.p[j].nsplit > 1)
                red += ov3d_cdiv((long long)q.N * q.K + (q.db ? q.N : 0), 256);
        }
        g.blk[g.n] = blk;
        g.red[g.n] = red;
        wgrad_group128_kernel<<<blk, 256, 0, st>>>(g);
        OV3D_LAUNCH_CHECK();
        if (red > 0) {
            wgrad_group128_reduce_kernel<<<red, 256, 0, st>>>(g);
            OV3D_LAUNCH_CHECK();
        }
    }
    return OV3D_OK;
}
