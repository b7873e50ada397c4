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
#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int TN = 128, TK = 128;  // output tile (rows of dW = N, cols = K)
constexpr int RS = 32;             // rows of dy / x per LDS stage
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
    auto store = [&](const bf16x8 (&dr)[2], const bf16x8 (&xr)[2], int buf) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int idx = tid + 256 * c, row = idx >> 4, ch = idx & 15;
            *reinterpret_cast<bf16x8*>(&Ds[buf][row * LDT + 8 * ch]) = dr[c];
            *reinterpret_cast<bf16x8*>(&Xs[buf][row * LDT + 8 * ch]) = xr[c];
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
        store(dA, xA, 0);
        if (rbeg + RS < rend) load(dA, xA, rbeg + RS);
    }
    __syncthreads();
    for (int r = rbeg; r < rend;) {
        // LDS buffer 0 holds stage r, set A holds stage r + RS
        if (r + 2 * RS < rend) load(dB, xB, r + 2 * RS);
        compute(0);
        if (r + RS < rend) store(dA, xA, 1);
        __syncthreads();
        r += RS;
        if (r >= rend) break;
        // LDS buffer 1 holds stage r, set B holds stage r + RS
        if (r + 2 * RS < rend) load(dA, xA, r + 2 * RS);
        compute(1);
        if (r + RS < rend) store(dB, xB, 0);
        __syncthreads();
        r += RS;
    }

    // column sums of this split: 16 row-threads per 8-column group -> LDS -> 128 values
    float* bred = reinterpret_cast<float*>(&Xs[0][0]);   // 256 x 8 floats, free after the loop
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

// Several independent weight gradients in one launch (the deferred dW / db of a whole
// backward pass, gemm.py): problem i owns workgroups [blk[i], blk[i+1]).
constexpr int kGroupMax = 28;
struct WgradGroup {
    WgradArgs p[kGroupMax];
    int blk[kGroupMax + 1];
    int red[kGroupMax + 1];   // reduce: workgroups [red[i], red[i+1]) of problem i
    int n;
};
static_assert(sizeof(WgradGroup) <= 4000, "kernel argument space");

__global__ void __launch_bounds__(256, 2) wgrad_group_kernel(WgradGroup g) {
    const int b = blockIdx.x;
    int i = 0;
    while (i + 1 < g.n && b >= g.blk[i + 1]) ++i;
    const WgradArgs& a = g.p[i];
    const int tn = (a.N + TN - 1) / TN, tk = (a.K + TK - 1) / TK;
    const int local = b - g.blk[i];
    wgrad_body(a, local % tn, (local / tn) % tk, local / (tn * tk));
}

__global__ void __launch_bounds__(256) wgrad_group_reduce_kernel(WgradGroup g) {
    const int b = blockIdx.x;
    int i = 0;
    while (i + 1 < g.n && b >= g.red[i + 1]) ++i;
    if (b >= g.red[i + 1] || b < g.red[i]) return;
    wgrad_reduce_body(g.p[i], (long long)(b - g.red[i]) * blockDim.x + threadIdx.x);
}

}  // namespace

extern "C" long long ov3d_wgrad_workspace(int R, int N, int K, int nsplit) {
    if (nsplit <= 1) return 0;
    return (long long)nsplit * ((long long)N * K + N);
}

extern "C" int ov3d_wgrad_tiles(int N, int K) { return ((N + TN - 1) / TN) * ((K + TK - 1) / TK); }

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
    return OV3D_OK;
}

extern "C" int ov3d_wgrad(const void* dy, long long ldy, const void* x, long long ldx, int R, int N,
                          int K, float* dW, long long ldw, float* db, float* workspace,
                          int* counters, int nsplit, void* stream) {
    (void)counters;
    WgradArgs a;
    const int rc = make_args(a, dy, ldy, x, ldx, R, N, K, dW, ldw, db, workspace, nsplit);
    if (rc != OV3D_OK) return rc;
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

extern "C" long long ov3d_wgrad_group_workspace(const ov3d_wgrad_problem* probs, int n) {
    long long w = 0;
    for (int i = 0; i < n; ++i) w += ov3d_wgrad_workspace(probs[i].R, probs[i].N, probs[i].K, probs[i].nsplit);
    return w;
}

extern "C" int ov3d_wgrad_group(const ov3d_wgrad_problem* probs, int n, float* workspace,
                                void* stream) {
    if (!probs || n <= 0) return OV3D_EINVAL;
    hipStream_t st = ov3d_stream(stream);
    long long woff = 0;
    for (int first = 0; first < n; first += kGroupMax) {
        WgradGroup g;
        g.n = n - first < kGroupMax ? n - first : kGroupMax;
        int blk = 0, red = 0;
        for (int j = 0; j < g.n; ++j) {
            const ov3d_wgrad_problem& q = probs[first + j];
            const long long ws = ov3d_wgrad_workspace(q.R, q.N, q.K, q.nsplit);
            const int rc = make_args(g.p[j], q.dy, q.ldy, q.x, q.ldx, q.R, q.N, q.K, q.dW, q.ldw,
                                     q.db, ws > 0 && workspace ? workspace + woff : nullptr,
                                     q.nsplit);
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
        wgrad_group_kernel<<<blk, 256, 0, st>>>(g);
        OV3D_LAUNCH_CHECK();
        if (red > 0) {
            wgrad_group_reduce_kernel<<<red, 256, 0, st>>>(g);
            OV3D_LAUNCH_CHECK();
        }
    }
    return OV3D_OK;
}
