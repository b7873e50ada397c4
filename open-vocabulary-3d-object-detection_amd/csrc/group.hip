// Ball query, grouping and gather for gfx950.
//
// Replaces the un-vendored third_party.pointnet2 ops used by
// PointnetSAModuleVotes / QueryAndGroup (models/model_3detr.py:355-361, 385-391):
// ball_query, grouping_operation (+ backward), gather_operation (+ backward).
//
// Ball query = one wave64 per 1-8 centroids.  Each lane owns 4 consecutive points of a
// 256-point chunk (3 x 16-B loads per lane, one coalesced 3 KiB wave read), four
// ballots give the in-radius masks, and popcounts of the masks below the lane give
// every hit its slot -- so the output is the first S in-radius indices in
// ascending order exactly as the upstream sequential scan produces them, and the
// wave stops at the first chunk that fills S slots.
#include "common.h"

namespace {

constexpr int kBQWavesPerBlock = 4;

template <bool ALIGNED>
__device__ __forceinline__ void load4(const float* __restrict__ p, int k0, int N, float (&x)[4],
                                      float (&y)[4], float (&z)[4]) {
    if (ALIGNED && k0 + 3 < N) {
        const float4* q = reinterpret_cast<const float4*>(p + 3 * (size_t)k0);
        const float4 a = q[0], b = q[1], c = q[2];
        x[0] = a.x; y[0] = a.y; z[0] = a.z;
        x[1] = a.w; y[1] = b.x; z[1] = b.y;
        x[2] = b.z; y[2] = b.w; z[2] = c.x;
        x[3] = c.y; y[3] = c.z; z[3] = c.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = k0 + j;
            if (k < N) { x[j] = p[3 * k]; y[j] = p[3 * k + 1]; z[j] = p[3 * k + 2]; }
            else { x[j] = 0.f; y[j] = 0.f; z[j] = 0.f; }
        }
    }
}

// CPW consecutive centroids of one scene per wave (M % CPW == 0; CPW = 1 is one wave per
// centroid): each 256-point chunk is loaded once and tested against all CPW centres.  The
// scan is VALU-bound (with few in-radius points per centroid nearly every wave scans the
// whole scene), so the distances run as packed-f32 pairs (v_pk_add / v_pk_mul / v_pk_fma:
// two points per lane and instruction, the same IEEE operations per element as
// fmaf(dz, dz, fmaf(dy, dy, dx * dx))), and points past N are padded far away
// (d2 = inf) instead of being masked.  A centroid whose S slots are full skips the tests;
// the wave stops when all CPW are full.
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <bool ALIGNED, int CPW>
__global__ __launch_bounds__(64 * kBQWavesPerBlock) void ball_query_kernel(
    const float* __restrict__ xyz, const float* __restrict__ new_xyz, int B, int N, int M, float r2,
    int S, int32_t* __restrict__ idx) {
    const int c0 = (blockIdx.x * kBQWavesPerBlock + (threadIdx.x >> 6)) * CPW;
    if (c0 >= B * M) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    const int b = c0 / M;      // the CPW centroids share the scene
    const float* __restrict__ p = xyz + (size_t)b * N * 3;
    float cx[CPW], cy[CPW], cz[CPW];
    int cnt[CPW], first[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        cx[c] = new_xyz[(size_t)(c0 + c) * 3];
        cy[c] = new_xyz[(size_t)(c0 + c) * 3 + 1];
        cz[c] = new_xyz[(size_t)(c0 + c) * 3 + 2];
        cnt[c] = 0;
        first[c] = 0;
    }
    const unsigned long long below = lanemask_lt();
    bool open = true;
    for (int base = 0; base < N && open; base += 256) {
        const int k0 = base + 4 * lane;
        float x[4], y[4], z[4];
        load4<ALIGNED>(p, k0, N, x, y, z);
        if (k0 + 3 >= N) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (k0 + j >= N) { x[j] = 3.0e38f; y[j] = 3.0e38f; z[j] = 3.0e38f; }
        }
        const f32x2 xa = {x[0], x[1]}, xb = {x[2], x[3]};
        const f32x2 ya = {y[0], y[1]}, yb = {y[2], y[3]};
        const f32x2 za = {z[0], z[1]}, zb = {z[2], z[3]};
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            if (cnt[c] >= S) continue;   // wave-uniform
            const f32x2 ccx = {cx[c], cx[c]}, ccy = {cy[c], cy[c]}, ccz = {cz[c], cz[c]};
            const f32x2 dxa = ccx - xa, dya = ccy - ya, dza = ccz - za;
            const f32x2 dxb = ccx - xb, dyb = ccy - yb, dzb = ccz - zb;
            const f32x2 da = __builtin_elementwise_fma(
                dza, dza, __builtin_elementwise_fma(dya, dya, dxa * dxa));
            const f32x2 db = __builtin_elementwise_fma(
                dzb, dzb, __builtin_elementwise_fma(dyb, dyb, dxb * dxb));
            const bool hit[4] = {da.x < r2, da.y < r2, db.x < r2, db.y < r2};
            if (__ballot(hit[0] | hit[1] | hit[2] | hit[3]) == 0) continue;
            unsigned long long m[4];
            int tot = 0, pre = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                m[j] = __ballot(hit[j]);
                tot += __popcll(m[j]);
                pre += __popcll(m[j] & below);
            }
            if (cnt[c] == 0) {
                int f = 0x7fffffff;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (m[j]) {
                        const int q = base + 4 * (__ffsll((long long)m[j]) - 1) + j;
                        f = q < f ? q : f;
                    }
                first[c] = f;
            }
            int32_t* __restrict__ out = idx + (size_t)(c0 + c) * S;
            int pos = cnt[c] + pre;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (hit[j]) {
                    if (pos < S) out[pos] = k0 + j;
                    ++pos;
                }
            }
            cnt[c] += tot;
        }
        open = false;
#pragma unroll
        for (int c = 0; c < CPW; ++c) open |= cnt[c] < S;
    }
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        int32_t* __restrict__ out = idx + (size_t)(c0 + c) * S;
        const int filled = cnt[c] < S ? cnt[c] : S;
        const int fill = cnt[c] > 0 ? first[c] : 0;
        for (int s = filled + lane; s < S; s += 64) out[s] = fill;
    }
}

// centroids per wave of the ball query (OV3D_BQ_CPW: 1, 2, 4, 8)
int bq_cpw() {
    static const int v = [] {
        const char* e = getenv("OV3D_BQ_CPW");
        const int c = e ? atoi(e) : 2;
        return (c == 1 || c == 2 || c == 4 || c == 8) ? c : 2;
    }();
    return v;
}

template <int CPW>
void launch_bq_multi(bool aligned, hipStream_t s, const float* xyz, const float* new_xyz, int B,
                     int N, int M, float r2, int S, int32_t* idx) {
    const int blocks = ov3d_cdiv((long long)B * M / CPW, kBQWavesPerBlock);
    if (aligned)
        hipLaunchKernelGGL((ball_query_kernel<true, CPW>), dim3(blocks),
                           dim3(64 * kBQWavesPerBlock), 0, s, xyz, new_xyz, B, N, M, r2, S, idx);
    else
        hipLaunchKernelGGL((ball_query_kernel<false, CPW>), dim3(blocks),
                           dim3(64 * kBQWavesPerBlock), 0, s, xyz, new_xyz, B, N, M, r2, S, idx);
}

// ---------------------------------------------------------------------------
// Cell-indexed ball query (ov3d_ball_query_cells): the same output as the scan above, from
// a uniform grid instead of a scan of the whole scene.
//
// Build (one 1024-thread workgroup per scene): bbox of the finite points, cube cells of side
// csz = max(1.001 r, extent / (kBQDim - 1)) (at most kBQDim^3 cells), a counting sort in LDS
// (16-bit counters, N < 65536), the cells' start offsets and the scene's points in cell order
// as float4 (x, y, z, index bits) into the workspace.
// Query (one wave per centroid): every point within r of the centroid lies in the 3 x 3 x 3
// cells around the centroid's cell (csz >= 1.001 r covers the rounding of d2 and of the cell
// coordinates), i.e. in 9 contiguous runs of 3 cells.  The wave tests those runs' points with
// the reference's d2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx)) < r^2 (dx = centre - point), keeps
// the hits' indices in LDS and outputs the S smallest in ascending order -- exactly the first S
// hits of the upstream index-order scan -- padded with the smallest (upstream: the first hit),
// or zeros without a hit.  A centroid with more than kBQCap hits in its runs falls back to the
// index-order scan on its wave (exact either way).
constexpr int kBQDim = 40;
constexpr int kBQCells = kBQDim * kBQDim * kBQDim;   // 64000 16-bit counters = 125 KiB LDS
constexpr int kBQCap = 1024;                          // hits kept per wave (4 KiB LDS)
constexpr int kBQParams = 8;                          // lo xyz, inv, dims xyz, pad (4-byte words)
// measured (tools/bq_time.py): B=8, M=2048, r=0.2, S=64: N=20000 scan 107 us, cells 50 (build,
// 8 workgroups) + 23 (query); N=40000 205 vs 106; B=8, N=2048, M=1024, r=0.4: scan 13-16 us,
// cells 13 + 8
constexpr int kBQCellsMinN = 8192;

struct BQLayout {
    float* params;      // [B][kBQParams]
    uint32_t* cstart;   // [B][kBQCells + 1]
    float4* pts;        // [B][N]
};

__host__ __device__ inline long long bq_ws_bytes(int B, int N) {
    return (long long)B * kBQParams * 4 + (long long)B * (kBQCells + 1) * 4 +
           (long long)B * N * 16 + 64;
}

__host__ __device__ inline BQLayout bq_layout(void* ws, int B, int N) {
    char* c = static_cast<char*>(ws);
    BQLayout l;
    l.params = reinterpret_cast<float*>(c);
    c += (long long)B * kBQParams * 4;
    l.cstart = reinterpret_cast<uint32_t*>(c);
    c += (long long)B * (kBQCells + 1) * 4;
    c = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(c) + 15) & ~uintptr_t(15));
    l.pts = reinterpret_cast<float4*>(c);
    return l;
}

__device__ __forceinline__ bool bq_finite(float x, float y, float z) {
    return fabsf(x) <= 3.0e38f && fabsf(y) <= 3.0e38f && fabsf(z) <= 3.0e38f;
}

// the point's cell coordinate on one axis (build and query evaluate the same expression)
__device__ __forceinline__ int bq_axis(float v, float lo, float inv, int dim) {
    const float f = floorf((v - lo) * inv);
    return f < 0.f ? -1 : (f >= (float)dim ? dim : (int)f);
}

__device__ __forceinline__ float bq_wave_fmin(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fminf(v, __shfl_xor(v, off));
    return v;
}
__device__ __forceinline__ float bq_wave_fmax(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}

// the scene's points as PPT register slots per thread (point k = tid + 1024 i), all loads in
// flight at once; PPT = 0: a loop over global memory per pass (N > 32768)
template <int PPT>
struct BQPoints {
    float x[PPT], y[PPT], z[PPT];
    __device__ __forceinline__ void load(const float* __restrict__ p, int N, int tid) {
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            const int k = tid + 1024 * i;
            x[i] = k < N ? p[3 * k] : NAN;
            y[i] = k < N ? p[3 * k + 1] : NAN;
            z[i] = k < N ? p[3 * k + 2] : NAN;
        }
    }
    template <class F>
    __device__ __forceinline__ void each(const float* __restrict__, int, int tid, F&& f) const {
#pragma unroll
        for (int i = 0; i < PPT; ++i) f(tid + 1024 * i, x[i], y[i], z[i]);
    }
};
template <>
struct BQPoints<0> {
    __device__ __forceinline__ void load(const float* __restrict__, int, int) {}
    template <class F>
    __device__ __forceinline__ void each(const float* __restrict__ p, int N, int tid, F&& f) const {
        for (int k = tid; k < N; k += 1024) f(k, p[3 * k], p[3 * k + 1], p[3 * k + 2]);
    }
};

template <int PPT>
__global__ __launch_bounds__(1024) void bq_cells_build_kernel(const float* __restrict__ xyz, int N,
                                                              float radius, BQLayout L) {
    __shared__ uint32_t s_cnt[kBQCells / 2];   // two 16-bit counters per word
    __shared__ float s_red[6][16];
    __shared__ uint32_t s_tot[16];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float* __restrict__ p = xyz + (size_t)b * N * 3;
    BQPoints<PPT> P;
    P.load(p, N, tid);
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    P.each(p, N, tid, [&](int, float x, float y, float z) {
        if (!bq_finite(x, y, z)) return;
        lo[0] = fminf(lo[0], x); lo[1] = fminf(lo[1], y); lo[2] = fminf(lo[2], z);
        hi[0] = fmaxf(hi[0], x); hi[1] = fmaxf(hi[1], y); hi[2] = fmaxf(hi[2], z);
    });
#pragma unroll
    for (int a = 0; a < 3; ++a) { lo[a] = bq_wave_fmin(lo[a]); hi[a] = bq_wave_fmax(hi[a]); }
    if (lane == 0)
#pragma unroll
        for (int a = 0; a < 3; ++a) { s_red[a][w] = lo[a]; s_red[3 + a][w] = hi[a]; }
    for (int i = tid; i < kBQCells / 2; i += 1024) s_cnt[i] = 0u;
    __syncthreads();
    float ext = 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float l = s_red[a][0], h = s_red[3 + a][0];
        for (int q = 1; q < 16; ++q) { l = fminf(l, s_red[a][q]); h = fmaxf(h, s_red[3 + a][q]); }
        if (!(l <= h)) { l = 0.f; h = 0.f; }   // no finite point
        lo[a] = l;
        hi[a] = h - l;                          // extent
        ext = fmaxf(ext, hi[a]);
    }
    const float csz = fmaxf(fmaxf(fabsf(radius) * 1.001f, ext / (float)(kBQDim - 1)), 1e-30f);
    const float inv = 1.f / csz;
    int dim[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) dim[a] = min((int)floorf(hi[a] * inv) + 1, kBQDim);
    const int ncell = dim[0] * dim[1] * dim[2];
    if (tid == 0) {
        float* prm = L.params + (size_t)b * kBQParams;
        prm[0] = lo[0]; prm[1] = lo[1]; prm[2] = lo[2]; prm[3] = inv;
        prm[4] = __int_as_float(dim[0]); prm[5] = __int_as_float(dim[1]);
        prm[6] = __int_as_float(dim[2]); prm[7] = 0.f;
    }
    auto cell = [&](float x, float y, float z) {
        return (min(bq_axis(z, lo[2], inv, dim[2]), dim[2] - 1) * dim[1] +
                min(bq_axis(y, lo[1], inv, dim[1]), dim[1] - 1)) * dim[0] +
               min(bq_axis(x, lo[0], inv, dim[0]), dim[0] - 1);
    };
    // counts (the old counter value is not kept: positions come from the second pass)
    P.each(p, N, tid, [&](int, float x, float y, float z) {
        if (!bq_finite(x, y, z)) return;
        const int c = cell(x, y, z);
        atomicAdd(&s_cnt[c >> 1], 1u << (16 * (c & 1)));
    });
    __syncthreads();
    // exclusive scan of the counters: 32 words (64 cells) per thread, in place, and the
    // starts (+ the end) into the workspace
    uint32_t* __restrict__ cs = L.cstart + (size_t)b * (kBQCells + 1);
    const int nw = (ncell + 1) >> 1;
    constexpr int WPT = kBQCells / 2 / 1024 + 1;   // 32 words
    const int w0 = tid * WPT;
    uint32_t sum = 0;
    for (int i = 0; i < WPT; ++i) {
        const int wi = w0 + i;
        if (wi < nw) { const uint32_t v = s_cnt[wi]; sum += (v & 0xffffu) + (v >> 16); }
    }
    uint32_t inc = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(inc, off);
        if (lane >= off) inc += o;
    }
    if (lane == 63) s_tot[w] = inc;
    __syncthreads();
    uint32_t run = inc - sum;
    for (int q = 0; q < w; ++q) run += s_tot[q];
    for (int i = 0; i < WPT; ++i) {
        const int wi = w0 + i;
        if (wi >= nw) break;
        const uint32_t v = s_cnt[wi];
        const uint32_t a0 = run, a1 = run + (v & 0xffffu);
        run = a1 + (v >> 16);
        s_cnt[wi] = a0 | (a1 << 16);
        if (2 * wi < ncell) cs[2 * wi] = a0;
        if (2 * wi + 1 < ncell) cs[2 * wi + 1] = a1;
    }
    if (tid == 1023) {
        uint32_t t = 0;
        for (int q = 0; q < 16; ++q) t += s_tot[q];
        cs[ncell] = t;
    }
    __syncthreads();
    // scatter: the counter of the point's cell hands out its position (16-bit adds never carry:
    // every running value stays below the scene's finite-point count < 65536)
    float4* __restrict__ dst = L.pts + (size_t)b * N;
    P.each(p, N, tid, [&](int k, float x, float y, float z) {
        if (!bq_finite(x, y, z)) return;
        const int c = cell(x, y, z);
        const uint32_t old = atomicAdd(&s_cnt[c >> 1], 1u << (16 * (c & 1)));
        const uint32_t pos = (old >> (16 * (c & 1))) & 0xffffu;
        dst[pos] = make_float4(x, y, z, __int_as_float(k));
    });
}

// ascending bitonic sort of one value per lane across the wave
__device__ __forceinline__ int wave_sort_asc(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const int o = __shfl_xor(v, j);
            const bool up = (lane & k) == 0;
            const bool low = (lane & j) == 0;
            v = (low == up) ? min(v, o) : max(v, o);
        }
    return v;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

constexpr int kBQQWaves = 4;

__global__ __launch_bounds__(64 * kBQQWaves) void bq_cells_query_kernel(
    const float* __restrict__ xyz, const float* __restrict__ new_xyz, int B, int N, int M, float r2,
    int S, BQLayout L, int32_t* __restrict__ idx) {
    __shared__ int s_hit[kBQQWaves][kBQCap];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int c0 = blockIdx.x * kBQQWaves + wv;
    if (c0 >= B * M) return;   // wave-uniform; no block barrier below
    const int b = c0 / M;
    int* __restrict__ hits = s_hit[wv];
    int32_t* __restrict__ out = idx + (size_t)c0 * S;
    const float cx = new_xyz[(size_t)c0 * 3], cy = new_xyz[(size_t)c0 * 3 + 1],
                cz = new_xyz[(size_t)c0 * 3 + 2];
    const float* __restrict__ prm = L.params + (size_t)b * kBQParams;
    const float lox = prm[0], loy = prm[1], loz = prm[2], inv = prm[3];
    const int dx = __float_as_int(prm[4]), dy = __float_as_int(prm[5]), dz = __float_as_int(prm[6]);
    const uint32_t* __restrict__ cs = L.cstart + (size_t)b * (kBQCells + 1);
    const float4* __restrict__ pts = L.pts + (size_t)b * N;
    // the 9 runs: lane r < 9 holds run r = (z, y) row, cells x-1 .. x+1 (clipped)
    int rbeg = 0, rlen = 0;
    if (bq_finite(cx, cy, cz)) {
        const int ix = bq_axis(cx, lox, inv, dx), iy = bq_axis(cy, loy, inv, dy),
                  iz = bq_axis(cz, loz, inv, dz);
        if (lane < 9) {
            const int yy = iy + lane % 3 - 1, zz = iz + lane / 3 - 1;
            const int x0 = max(ix - 1, 0), x1 = min(ix + 1, dx - 1);
            if (yy >= 0 && yy < dy && zz >= 0 && zz < dz && x0 <= x1) {
                const int row = (zz * dy + yy) * dx;
                rbeg = (int)cs[row + x0];
                rlen = (int)cs[row + x1 + 1] - rbeg;
            }
        }
    }
    // inclusive prefix of the run lengths over lanes 0..8
    int pre = rlen;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
        const int o = __shfl_up(pre, off);
        if (lane >= off) pre += o;
    }
    // wave-uniform run table: P[q] = end of run q in the flattened candidate list, OFF[q] =
    // its cell-order position minus its flattened start
    int P[9], OFF[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) {
        P[q] = __builtin_amdgcn_readlane(pre, q);
        OFF[q] = __builtin_amdgcn_readlane(rbeg, q) - P[q] + __builtin_amdgcn_readlane(rlen, q);
    }
    const int total = P[8];
    int cnt = 0;
    bool overflow = false;
    const unsigned long long below = lanemask_lt();
    for (int f0 = 0; f0 < total; f0 += 64) {
        const int f = f0 + lane;
        bool hit = false;
        int k = 0;
        if (f < total) {
            int off = OFF[0];
#pragma unroll
            for (int q = 0; q < 8; ++q) off = P[q] <= f ? OFF[q + 1] : off;
            const float4 v = pts[f + off];
            const float ddx = cx - v.x, ddy = cy - v.y, ddz = cz - v.z;
            const float d2 = fmaf(ddz, ddz, fmaf(ddy, ddy, ddx * ddx));
            hit = d2 < r2;
            k = __float_as_int(v.w);
        }
        const unsigned long long m = __ballot(hit);
        const int n = __popcll(m);
        if (cnt + n > kBQCap) { overflow = true; break; }
        if (hit) hits[cnt + __popcll(m & below)] = k;
        cnt += n;
    }
    if (overflow) {
        // index-order scan of the whole scene (the reference's loop), one point per lane
        int filled = 0, first = 0;
        for (int base = 0; base < N && filled < S; base += 64) {
            const int k = base + lane;
            bool hit = false;
            if (k < N) {
                const float ddx = cx - xyz[((size_t)b * N + k) * 3],
                            ddy = cy - xyz[((size_t)b * N + k) * 3 + 1],
                            ddz = cz - xyz[((size_t)b * N + k) * 3 + 2];
                hit = fmaf(ddz, ddz, fmaf(ddy, ddy, ddx * ddx)) < r2;
            }
            const unsigned long long m = __ballot(hit);
            if (!m) continue;
            if (filled == 0) first = base + __ffsll((long long)m) - 1;
            const int pos = filled + __popcll(m & below);
            if (hit && pos < S) out[pos] = k;
            filled += __popcll(m);
        }
        const int fill = filled > 0 ? first : 0;
        for (int s = (filled < S ? filled : S) + lane; s < S; s += 64) out[s] = fill;
        return;
    }
    if (cnt == 0) {
        for (int s = lane; s < S; s += 64) out[s] = 0;
        return;
    }
    int v;
    if (cnt <= 64) {
        v = lane < cnt ? hits[lane] : INT_MAX;
    } else {
        // the S-th smallest hit index t - 1: the least t with #(hits < t) >= S (indices are
        // distinct), by bisection over [0, N]
        int tlo = 0, thi = N;   // #(< tlo) < S <= #(< thi)
        while (thi - tlo > 1) {
            const int mid = (tlo + thi) >> 1;
            int c = 0;
            for (int i = lane; i < cnt; i += 64) c += hits[i] < mid ? 1 : 0;
            if (wave_sum(c) >= S) thi = mid; else tlo = mid;
        }
        // the S hits below thi, compacted in place to the front of the list: chunk i0's kept
        // values land in [base, base + n) with base + n <= i0 + 64, i.e. on entries this wave
        // has already read (its LDS operations retire in order)
        int base = 0;
        for (int i0 = 0; i0 < cnt; i0 += 64) {
            const int i = i0 + lane;
            const int h = i < cnt ? hits[i] : INT_MAX;
            const bool keep = h < thi;
            const unsigned long long m = __ballot(keep);
            if (keep) hits[base + __popcll(m & below)] = h;
            base += __popcll(m);
        }
        v = lane < S ? hits[lane] : INT_MAX;
    }
    v = wave_sort_asc(v);
    const int smallest = __shfl(v, 0);
    const int have = cnt < S ? cnt : S;
    for (int s = lane; s < S; s += 64) out[s] = s < have ? v : smallest;
}

// out (B,M,S,3+C) channels-last rows: thread per output element (row, channel);
// features addressed through (sb, sn, sc) element strides, so both the reference
// (B,C,N) layout and the encoder's seq-first (N,B,C) layout are read in place.
// I: the element-index type (uint32_t when B*M*S*(3+C) < 2^31: the three index divisions
// are 32-bit instead of 64-bit; the C4 pre-encoder's 6.3M-element launch 31.0 -> 29.2 us)
template <typename I>
__global__ __launch_bounds__(256) void group_fwd_kernel(
    const float* __restrict__ xyz, const float* __restrict__ new_xyz,
    const float* __restrict__ feats, long long sb, long long sn, long long sc,
    const int32_t* __restrict__ idx, int B, int C, int N, int M, int S, float radius,
    int normalize, float* __restrict__ out) {
    const I CW = (I)(3 + C);
    const I t = (I)blockIdx.x * (I)blockDim.x + (I)threadIdx.x;
    const I rows = (I)B * (I)M * (I)S;
    if (t >= rows * CW) return;
    const I row = t / CW;
    const int c = (int)(t - row * CW);
    const int b = (int)(row / ((I)M * (I)S));
    const int m = (int)((row / (I)S) % (I)M);
    const int k = idx[row];
    float v;
    if (c < 3) {
        v = xyz[((size_t)b * N + k) * 3 + c] - new_xyz[((size_t)b * M + m) * 3 + c];
        if (normalize) v = v / radius;
    } else {
        v = feats[b * sb + k * sn + (c - 3) * sc];
    }
    out[t] = v;
}

__global__ __launch_bounds__(256) void group_bwd_kernel(const float* __restrict__ gout,
                                                        const int32_t* __restrict__ idx, int B,
                                                        int C, int M, int S, long long sb,
                                                        long long sn, long long sc,
                                                        float* __restrict__ gfeat) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long rows = (long long)B * M * S;
    if (t >= rows * C) return;
    const long long row = t / C;
    const int c = (int)(t - row * C);
    const int b = (int)(row / ((long long)M * S));
    const int k = idx[row];
    atomicAdd(gfeat + b * sb + k * sn + c * sc, gout[row * (3 + C) + 3 + c]);
}

// (B,C,N),(B,M) -> (B,C,M): thread per output element
__global__ __launch_bounds__(256) void gather_fwd_kernel(const float* __restrict__ f,
                                                         const int32_t* __restrict__ idx, int B,
                                                         int C, int N, int M,
                                                         float* __restrict__ out) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)B * C * M) return;
    const int m = (int)(t % M);
    const long long bc = t / M;
    const int b = (int)(bc / C);
    out[t] = f[bc * N + idx[(size_t)b * M + m]];
}

__global__ __launch_bounds__(256) void gather_bwd_kernel(const float* __restrict__ g,
                                                         const int32_t* __restrict__ idx, int B,
                                                         int C, int N, int M,
                                                         float* __restrict__ gf) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)B * C * M) return;
    const int m = (int)(t % M);
    const long long bc = t / M;
    const int b = (int)(bc / C);
    atomicAdd(gf + bc * N + idx[(size_t)b * M + m], g[t]);
}

// ---- inverse of the ball-query index (CSR per source point), for a gather-form backward
// count: rows per (b, n) into cnt[b*N + n] (zeroed by the caller's launch below)
__global__ __launch_bounds__(256) void inv_count_kernel(const int32_t* __restrict__ idx, int N,
                                                        long long MS, long long total,
                                                        int32_t* __restrict__ cnt) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int b = (int)(t / MS);
    atomicAdd(cnt + (size_t)b * N + idx[t], 1);
}

// exclusive scan of n counts -> off[0..n] (one 1024-thread workgroup, sequential per thread);
// cur = off[0..n-1] (fill cursors)
__global__ __launch_bounds__(1024) void inv_scan_kernel(const int32_t* __restrict__ cnt, int n,
                                                        int32_t* __restrict__ off,
                                                        int32_t* __restrict__ cur) {
    __shared__ int32_t part[1024];
    const int tid = threadIdx.x;
    const int per = (n + 1023) / 1024;
    const int b0 = tid * per, b1 = min(n, b0 + per);
    int sum = 0;
    for (int i = b0; i < b1; ++i) sum += cnt[i];
    part[tid] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {   // Hillis-Steele inclusive scan of the parts
        const int v = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int run = part[tid] - sum;
    for (int i = b0; i < b1; ++i) {
        off[i] = run;
        cur[i] = run;
        run += cnt[i];
    }
    if (tid == 1023) off[n] = part[1023];
}

__global__ __launch_bounds__(256) void inv_fill_kernel(const int32_t* __restrict__ idx, int N,
                                                       long long MS, long long total,
                                                       int32_t* __restrict__ cur,
                                                       int32_t* __restrict__ rows) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int b = (int)(t / MS);
    const int pos = atomicAdd(cur + (size_t)b * N + idx[t], 1);
    rows[pos] = (int32_t)t;
}

// the fill's atomics hand out slots in an arbitrary order; the backward's fp32 sums follow the
// list order, so each list is put in ascending row order: the gradient is then the same bit for
// bit in every run.  One wave per list: the list (row ids are distinct) is staged in LDS and
// every entry goes to its rank (the number of smaller entries): len^2 / 64 LDS reads per lane,
// no dependent global round trips (a one-thread insertion sort over global memory took ~1 ms
// per ScanNet step on its longest lists, ~180 entries).  Lists longer than kSortLds (none at
// the reference's shapes) take the one-lane insertion sort.
constexpr int kSortLds = 1024;
__global__ __launch_bounds__(256) void inv_sort_kernel(const int32_t* __restrict__ off, long long n,
                                                       int32_t* __restrict__ rows) {
    __shared__ int32_t s[4][kSortLds];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long i = (long long)blockIdx.x * 4 + w;
    if (i >= n) return;   // whole waves only; no workgroup barrier below
    const int e0 = off[i], e1 = off[i + 1], len = e1 - e0;
    if (len <= 1) return;
    if (len > kSortLds) {
        if (lane == 0)
            for (int j = e0 + 1; j < e1; ++j) {
                const int32_t v = rows[j];
                int k = j - 1;
                while (k >= e0 && rows[k] > v) {
                    rows[k + 1] = rows[k];
                    --k;
                }
                rows[k + 1] = v;
            }
        return;
    }
    for (int j = lane; j < len; j += 64) s[w][j] = rows[e0 + j];
    // one wave's LDS accesses complete in order: its reads below see all its writes
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int j0 = 0; j0 < len; j0 += 64) {
        const int j = j0 + lane;
        const int32_t v = j < len ? s[w][j] : 0;
        int rank = 0;
        for (int u = 0; u < len; ++u) rank += s[w][u] < v;
        if (j < len) rows[e0 + rank] = v;
    }
}

// gather-form grouping backward: thread per (b, n, c), c fastest (a wave reads 64 channels of
// one grad row per list entry); every (b, n, c) written (0 when no row refers to n)
// The same rows as group_fwd_kernel in bf16 with a padded row stride ldo (a multiple of 8,
// columns 3 + C .. ldo - 1 zero): the SA MLP's first GEMM reads them directly with an aligned K
// (bf16 autocast rounds the fp32 rows to these values before the GEMM anyway).  One thread per
// 8 columns of a row: consecutive threads cover a row left to right (contiguous feature reads
// for channel-contiguous features), one 16-byte store each.
// VEC: channel-contiguous feature rows (sc = 1, C % 4 == 0, 16-byte aligned rows): the 8
// feature values of a chunk (channels c0 - 3 .. c0 + 4) from three aligned 16-byte loads
// instead of eight misaligned 4-byte ones (same values)
template <bool VEC>
__global__ __launch_bounds__(256) void group_rows_bf16_kernel(
    const float* __restrict__ xyz, const float* __restrict__ new_xyz,
    const float* __restrict__ feats, long long sb, long long sn, long long sc,
    const int32_t* __restrict__ idx, int B, int C, int N, int M, int S, float radius,
    int normalize, int ldo, __bf16* __restrict__ out) {
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    const int chunks = ldo >> 3;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long rows = (long long)B * M * S;
    if (t >= rows * chunks) return;
    const long long row = t / chunks;
    const int c0 = (int)(t - row * chunks) * 8;
    const int b = (int)(row / ((long long)M * S));
    const int m = (int)((row / S) % M);
    const int k = idx[row];
    const float* const f = feats ? feats + b * sb + k * sn : nullptr;
    float fv[12];   // VEC: features c0 - 4 .. c0 + 7 (zeros outside 0 .. C - 1)
    if constexpr (VEC) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int e = c0 - 4 + 4 * q;
            float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e >= 0 && e + 4 <= C) u = *reinterpret_cast<const float4*>(f + e);
            fv[4 * q] = u.x; fv[4 * q + 1] = u.y; fv[4 * q + 2] = u.z; fv[4 * q + 3] = u.w;
        }
    }
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        float x = 0.f;
        if (c < 3) {
            x = xyz[((size_t)b * N + k) * 3 + c] - new_xyz[((size_t)b * M + m) * 3 + c];
            if (normalize) x = x / radius;
        } else if (c < 3 + C) {
            if constexpr (VEC) x = fv[j + 1];   // channel c - 3 = (c0 - 4) + (j + 1)
            else x = f[(c - 3) * sc];
        }
        v[j] = (__bf16)x;
    }
    *reinterpret_cast<bf16x8*>(out + row * ldo + c0) = v;
}

// gather-form grouping backward (below) reading the feature columns 3 .. 3 + C of grad rows
// with row stride ldg (fp32 rows of group_fwd_kernel: ldg = 3 + C; bf16 rows of
// group_rows_bf16_kernel: ldg = its ldo)
template <typename GT>
__global__ __launch_bounds__(256) void group_bwd_csr_kernel(const GT* __restrict__ gout, long long ldg,
                                                            const int32_t* __restrict__ off,
                                                            const int32_t* __restrict__ rows, int B,
                                                            int C, int N, long long sb,
                                                            long long sn, long long sc,
                                                            float* __restrict__ gfeat) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)B * N * C) return;
    const int c = (int)(t % C);
    const long long bn = t / C;
    const int b = (int)(bn / N), n = (int)(bn - (long long)b * N);
    const int e0 = off[bn], e1 = off[bn + 1];
    float acc = 0.f;
    // 8 entries per round: their row ids, then their values, are independent loads (one
    // memory round trip each instead of two per entry)
    int e = e0;
    for (; e + 8 <= e1; e += 8) {
        int r[8];
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = rows[e + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = (float)gout[(size_t)r[u] * ldg + 3 + c];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    if (e < e1) {
        int r[8];
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = e + u < e1 ? rows[e + u] : -1;
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = r[u] >= 0 ? (float)gout[(size_t)r[u] * ldg + 3 + c] : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    gfeat[b * sb + n * sn + c * sc] = acc;
}

typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

// the same gather over bf16 rows with ldg % 8 == 0 and 16-byte aligned rows: a thread owns
// the 16-byte chunk q of each row it reads (columns 8q .. 8q+7 = channels 8q-3 .. 8q+4), one
// row id and one 16-byte load per entry instead of one of each per channel.  Each channel sums
// its entries in the scalar kernel's order (8 a round, a zero-padded tail round): bit-equal.
__global__ __launch_bounds__(256) void group_bwd_csr_vec_kernel(const __bf16* __restrict__ gout,
                                                                long long ldg,
                                                                const int32_t* __restrict__ off,
                                                                const int32_t* __restrict__ rows,
                                                                int B, int C, int N, int nq,
                                                                long long sb, long long sn,
                                                                long long sc,
                                                                float* __restrict__ gfeat) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)B * N * nq) return;
    const int q = (int)(t % nq);
    const long long bn = t / nq;
    const int b = (int)(bn / N), n = (int)(bn - (long long)b * N);
    const int e0 = off[bn], e1 = off[bn + 1];
    const __bf16* g = gout + 8 * q;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    int e = e0;
    for (; e + 8 <= e1; e += 8) {
        int r[8];
        bf16x8v v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = rows[e + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const bf16x8v*>(g + (size_t)r[u] * ldg);
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] += (float)v[u][j];
    }
    if (e < e1) {
        int r[8];
        bf16x8v v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = e + u < e1 ? rows[e + u] : -1;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (r[u] >= 0) {
                v[u] = *reinterpret_cast<const bf16x8v*>(g + (size_t)r[u] * ldg);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[u][j] = (__bf16)0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] += (float)v[u][j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = 8 * q + j - 3;
        if (c >= 0 && c < C) gfeat[b * sb + n * sn + c * sc] = acc[j];
    }
}

}  // namespace

extern "C" int ov3d_group_inverse(const int32_t* idx, int B, int N, int M, int S, int32_t* cnt,
                                  int32_t* offsets, int32_t* cursor, int32_t* rows, void* stream) {
    if (!idx || !cnt || !offsets || !cursor || !rows || B <= 0 || N <= 0 || M < 0 || S <= 0)
        return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    const long long total = (long long)B * M * S, n = (long long)B * N;
    if (hipMemsetAsync(cnt, 0, n * sizeof(int32_t), s) != hipSuccess) return OV3D_ELAUNCH;
    if (total > 0)
        hipLaunchKernelGGL(inv_count_kernel, dim3(ov3d_cdiv(total, 256)), dim3(256), 0, s, idx, N,
                           (long long)M * S, total, cnt);
    hipLaunchKernelGGL(inv_scan_kernel, dim3(1), dim3(1024), 0, s, cnt, (int)n, offsets, cursor);
    if (total > 0)
        hipLaunchKernelGGL(inv_fill_kernel, dim3(ov3d_cdiv(total, 256)), dim3(256), 0, s, idx, N,
                           (long long)M * S, total, cursor, rows);
    if (total > 0)
        hipLaunchKernelGGL(inv_sort_kernel, dim3(ov3d_cdiv(n, 4)), dim3(256), 0, s, offsets, n, rows);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_group_bwd_csr(const float* grad_out, const int32_t* offsets,
                                  const int32_t* rows, int B, int C, int N, long long feat_sb,
                                  long long feat_sn, long long feat_sc, float* grad_features,
                                  void* stream) {
    if (!grad_out || !offsets || !rows || !grad_features || B < 0 || C < 0 || N <= 0)
        return OV3D_EINVAL;
    const long long total = (long long)B * N * C;
    if (total == 0) return OV3D_OK;
    hipLaunchKernelGGL(group_bwd_csr_kernel<float>, dim3(ov3d_cdiv(total, 256)), dim3(256), 0,
                       ov3d_stream(stream), grad_out, (long long)(3 + C), offsets, rows, B, C, N,
                       feat_sb, feat_sn, feat_sc, grad_features);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_group_bwd_csr_bf16(const void* grad_out, long long ldg, const int32_t* offsets,
                                       const int32_t* rows, int B, int C, int N, long long feat_sb,
                                       long long feat_sn, long long feat_sc, float* grad_features,
                                       void* stream) {
    if (!grad_out || !offsets || !rows || !grad_features || B < 0 || C < 0 || N <= 0 ||
        ldg < 3 + C)
        return OV3D_EINVAL;
    const long long total = (long long)B * N * C;
    if (total == 0) return OV3D_OK;
    if (ldg % 8 == 0 && reinterpret_cast<uintptr_t>(grad_out) % 16 == 0) {
        const int nq = (3 + C + 7) / 8;   // <= ldg / 8
        const long long tv = (long long)B * N * nq;
        hipLaunchKernelGGL(group_bwd_csr_vec_kernel, dim3(ov3d_cdiv(tv, 256)), dim3(256), 0,
                           ov3d_stream(stream), static_cast<const __bf16*>(grad_out), ldg, offsets,
                           rows, B, C, N, nq, feat_sb, feat_sn, feat_sc, grad_features);
        OV3D_LAUNCH_CHECK();
        return OV3D_OK;
    }
    hipLaunchKernelGGL(group_bwd_csr_kernel<__bf16>, dim3(ov3d_cdiv(total, 256)), dim3(256), 0,
                       ov3d_stream(stream), static_cast<const __bf16*>(grad_out), ldg, offsets, rows,
                       B, C, N, feat_sb, feat_sn, feat_sc, grad_features);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_group_rows_bf16(const float* xyz, const float* new_xyz, const float* features,
                                    long long feat_sb, long long feat_sn, long long feat_sc,
                                    const int32_t* idx, int B, int C, int N, int M, int S,
                                    float radius, int normalize, int ldo, void* out, void* stream) {
    if (B < 0 || C < 0 || N <= 0 || M < 0 || S <= 0 || !xyz || !new_xyz || !idx || !out ||
        ldo < 3 + C || (ldo & 7) || ((uintptr_t)out & 15))
        return OV3D_EINVAL;
    if (C > 0 && !features) return OV3D_EINVAL;
    const long long total = (long long)B * M * S * (ldo / 8);
    if (total == 0) return OV3D_OK;
    const bool vec = C > 0 && feat_sc == 1 && C % 4 == 0 && feat_sb % 4 == 0 && feat_sn % 4 == 0 &&
                     ((uintptr_t)features & 15) == 0;
    if (vec)
        hipLaunchKernelGGL(group_rows_bf16_kernel<true>, dim3(ov3d_cdiv(total, 256)), dim3(256), 0,
                           ov3d_stream(stream), xyz, new_xyz, features, feat_sb, feat_sn, feat_sc,
                           idx, B, C, N, M, S, radius, normalize, ldo, static_cast<__bf16*>(out));
    else
        hipLaunchKernelGGL(group_rows_bf16_kernel<false>, dim3(ov3d_cdiv(total, 256)), dim3(256), 0,
                           ov3d_stream(stream), xyz, new_xyz, C > 0 ? features : nullptr, feat_sb,
                           feat_sn, feat_sc, idx, B, C, N, M, S, radius, normalize, ldo,
                           static_cast<__bf16*>(out));
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_ball_query(const float* xyz, const float* new_xyz, int B, int N, int M,
                               float radius, int S, int32_t* idx_out, void* stream) {
    if (B < 0 || N < 0 || M < 0 || S <= 0 || !xyz || !new_xyz || !idx_out) return OV3D_EINVAL;
    if ((long long)B * M == 0) return OV3D_OK;
    const float r2 = radius * radius;
    hipStream_t s = ov3d_stream(stream);
    const bool aligned = (reinterpret_cast<uintptr_t>(xyz) % 16 == 0) && (N % 4 == 0);
    const int cpw = M % bq_cpw() == 0 ? bq_cpw() : 1;
    if (cpw == 2) launch_bq_multi<2>(aligned, s, xyz, new_xyz, B, N, M, r2, S, idx_out);
    else if (cpw == 4) launch_bq_multi<4>(aligned, s, xyz, new_xyz, B, N, M, r2, S, idx_out);
    else if (cpw == 8) launch_bq_multi<8>(aligned, s, xyz, new_xyz, B, N, M, r2, S, idx_out);
    else launch_bq_multi<1>(aligned, s, xyz, new_xyz, B, N, M, r2, S, idx_out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" long long ov3d_ball_query_ws_bytes(int B, int N) {
    return B > 0 && N > 0 ? bq_ws_bytes(B, N) : 0;
}

extern "C" int ov3d_ball_query_cells(const float* xyz, const float* new_xyz, int B, int N, int M,
                                     float radius, int S, int32_t* idx_out, void* ws,
                                     long long ws_bytes, void* stream) {
    if (B < 0 || N < 0 || M < 0 || S <= 0 || !xyz || !new_xyz || !idx_out) return OV3D_EINVAL;
    if ((long long)B * M == 0) return OV3D_OK;
    // the grid's 16-bit cell counters and the one-value-per-lane sort: N < 65536, S <= 64;
    // beyond that, and below kBQCellsMinN points (the scan of a small scene is cheaper than
    // the build's ~13 us of single-workgroup phases), the index-order scan (same output)
    if (N >= 65536 || N < kBQCellsMinN || S > 64)
        return ov3d_ball_query(xyz, new_xyz, B, N, M, radius, S, idx_out, stream);
    if (!ws || ws_bytes < bq_ws_bytes(B, N) || (reinterpret_cast<uintptr_t>(ws) & 15))
        return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    const BQLayout L = bq_layout(ws, B, N);
    if (N <= 20480)
        hipLaunchKernelGGL(bq_cells_build_kernel<20>, dim3(B), dim3(1024), 0, s, xyz, N, radius, L);
    else if (N <= 32768)
        hipLaunchKernelGGL(bq_cells_build_kernel<32>, dim3(B), dim3(1024), 0, s, xyz, N, radius, L);
    else
        hipLaunchKernelGGL(bq_cells_build_kernel<0>, dim3(B), dim3(1024), 0, s, xyz, N, radius, L);
    OV3D_LAUNCH_CHECK();
    hipLaunchKernelGGL(bq_cells_query_kernel, dim3(ov3d_cdiv((long long)B * M, kBQQWaves)),
                       dim3(64 * kBQQWaves), 0, s, xyz, new_xyz, B, N, M, radius * radius, S, L,
                       idx_out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_group_fwd(const float* xyz, const float* new_xyz, const float* features,
                              long long feat_sb, long long feat_sn, long long feat_sc,
                              const int32_t* idx, int B, int C, int N, int M, int S, float radius,
                              int normalize, float* out, void* stream) {
    if (B < 0 || C < 0 || N <= 0 || M < 0 || S <= 0 || !xyz || !new_xyz || !idx || !out)
        return OV3D_EINVAL;
    if (C > 0 && !features) return OV3D_EINVAL;
    const long long total = (long long)B * M * S * (3 + C);
    if (total == 0) return OV3D_OK;
    if (total < (1ll << 31))
        hipLaunchKernelGGL(group_fwd_kernel<uint32_t>, dim3(ov3d_cdiv(total, 256)), dim3(256), 0,
                           ov3d_stream(stream), xyz, new_xyz, C > 0 ? features : nullptr, feat_sb,
                           feat_sn, feat_sc, idx, B, C, N, M, S, radius, normalize, out);
    else
        hipLaunchKernelGGL(group_fwd_kernel<long long>, dim3(ov3d_cdiv(total, 256)), dim3(256), 0,
                           ov3d_stream(stream), xyz, new_xyz, C > 0 ? features : nullptr, feat_sb,
                           feat_sn, feat_sc, idx, B, C, N, M, S, radius, normalize, out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_group_bwd(const float* grad_out, const int32_t* idx, int B, int C, int N, int M,
                              int S, long long feat_sb, long long feat_sn, long long feat_sc,
                              float* grad_features, void* stream) {
    if (B < 0 || C < 0 || N <= 0 || M < 0 || S <= 0 || !grad_out || !idx || !grad_features)
        return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    // grad_features spans B*C*N elements whatever the stride order
    if ((long long)B * C * N > 0 &&
        hipMemsetAsync(grad_features, 0, sizeof(float) * (size_t)B * C * N, s) != hipSuccess)
        return OV3D_ELAUNCH;
    const long long total = (long long)B * M * S * C;
    if (total == 0) return OV3D_OK;
    hipLaunchKernelGGL(group_bwd_kernel, dim3(ov3d_cdiv(total, 256)), dim3(256), 0, s, grad_out,
                       idx, B, C, M, S, feat_sb, feat_sn, feat_sc, grad_features);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_gather_fwd(const float* features, const int32_t* idx, int B, int C, int N,
                               int M, float* out, void* stream) {
    if (B < 0 || C < 0 || N <= 0 || M < 0 || !features || !idx || !out) return OV3D_EINVAL;
    const long long total = (long long)B * C * M;
    if (total == 0) return OV3D_OK;
    hipLaunchKernelGGL(gather_fwd_kernel, dim3(ov3d_cdiv(total, 256)), dim3(256), 0,
                       ov3d_stream(stream), features, idx, B, C, N, M, out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_gather_bwd(const float* grad_out, const int32_t* idx, int B, int C, int N,
                               int M, float* grad_features, void* stream) {
    if (B < 0 || C < 0 || N <= 0 || M < 0 || !grad_out || !idx || !grad_features)
        return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    if ((long long)B * C * N > 0 &&
        hipMemsetAsync(grad_features, 0, sizeof(float) * (size_t)B * C * N, s) != hipSuccess)
        return OV3D_ELAUNCH;
    const long long total = (long long)B * C * M;
    if (total == 0) return OV3D_OK;
    hipLaunchKernelGGL(gather_bwd_kernel, dim3(ov3d_cdiv(total, 256)), dim3(256), 0, s, grad_out,
                       idx, B, C, N, M, grad_features);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
