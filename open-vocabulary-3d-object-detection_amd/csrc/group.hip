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

// out (B,M,S,3+C) channels-last rows: thread per output element (row, channel);
// features addressed through (sb, sn, sc) element strides, so both the reference
// (B,C,N) layout and the encoder's seq-first (N,B,C) layout are read in place.
__global__ __launch_bounds__(256) void group_fwd_kernel(
    const float* __restrict__ xyz, const float* __restrict__ new_xyz,
    const float* __restrict__ feats, long long sb, long long sn, long long sc,
    const int32_t* __restrict__ idx, int B, int C, int N, int M, int S, float radius,
    int normalize, float* __restrict__ out) {
    const int CW = 3 + C;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long rows = (long long)B * M * S;
    if (t >= rows * CW) return;
    const long long row = t / CW;
    const int c = (int)(t - row * CW);
    const int b = (int)(row / ((long long)M * S));
    const int m = (int)((row / S) % M);
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
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        float x = 0.f;
        if (c < 3) {
            x = xyz[((size_t)b * N + k) * 3 + c] - new_xyz[((size_t)b * M + m) * 3 + c];
            if (normalize) x = x / radius;
        } else if (c < 3 + C) {
            x = f[(c - 3) * sc];
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
    hipLaunchKernelGGL(group_rows_bf16_kernel, dim3(ov3d_cdiv(total, 256)), dim3(256), 0,
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

extern "C" int ov3d_group_fwd(const float* xyz, const float* new_xyz, const float* features,
                              long long feat_sb, long long feat_sn, long long feat_sc,
                              const int32_t* idx, int B, int C, int N, int M, int S, float radius,
                              int normalize, float* out, void* stream) {
    if (B < 0 || C < 0 || N <= 0 || M < 0 || S <= 0 || !xyz || !new_xyz || !idx || !out)
        return OV3D_EINVAL;
    if (C > 0 && !features) return OV3D_EINVAL;
    const long long total = (long long)B * M * S * (3 + C);
    if (total == 0) return OV3D_OK;
    hipLaunchKernelGGL(group_fwd_kernel, dim3(ov3d_cdiv(total, 256)), dim3(256), 0,
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
