// Furthest-point sampling for gfx950.
//
// Replaces third_party.pointnet2 furthest_point_sampling (un-vendored; called at
// models/model_3detr.py:174 and in PointnetSAModuleVotes, model_3detr.py:355-361).
//
// Design (one 1024-thread workgroup = 16 waves per scene, the scene's points
// held in registers for the whole run):
//   * point k lives in thread (k mod 1024), slot (k / 1024): PPT slots per thread,
//     coordinates + running min-distance in VGPRs (4 regs per slot);
//   * per iteration: VALU distance update + per-thread argmax, wave64 u64 max
//     reduction with shuffles, one LDS slot per wave (double-buffered by
//     iteration parity -> ONE barrier per iteration), every thread reduces the
//     16 wave slots and reads the winner's coordinates from LDS;
//   * the winner's coordinates are carried through the reduction, so there is
//     no dependent global load on the serial chain; new_xyz (gather_operation)
//     is written in the same loop.
// Bit-exact contract with oracle/ov3d_oracle.c: d = fmaf(dz,dz,fmaf(dy,dy,dx*dx)),
// skip |p|^2 <= 1e-3 (float vs double literal), min() update, and the upstream
// tie rule: argmax key = (float bits of d, ~rank(k)) where rank(k) orders ties
// exactly as the upstream 512-thread halving-tree reduction does
// (bit-reversed thread id, then k).  Within one of our threads the slots are
// visited in increasing rank order (1024 is a multiple of the upstream block
// size), so strict '>' there and the u64 key across threads reproduce it.
#include "common.h"

namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxPPT = 20;  // 4 VGPRs per slot: 118 VGPRs at PPT=20, spills beyond

__device__ __forceinline__ uint32_t fps_rank(uint32_t k, int L) {
    const uint32_t t = k & ((1u << L) - 1u);
    const uint32_t br = L ? (__builtin_bitreverse32(t) >> (32 - L)) : 0u;
    return (br << 23) | (k >> L);
}

__device__ __forceinline__ int fps_unrank(uint32_t r, int L) {
    const uint32_t br = r >> 23;
    const uint32_t i = r & ((1u << 23) - 1u);
    const uint32_t t = L ? (__builtin_bitreverse32(br) >> (32 - L)) : 0u;
    return (int)((i << L) | t);
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = o > v ? o : v;
    }
    return v;
}

struct Pick {
    float x, y, z;
    int k;
};

// Block-wide argmax over per-thread (key, coords); all threads receive the winner.
__device__ __forceinline__ Pick block_pick(unsigned long long key, float bx, float by, float bz,
                                           int buf, unsigned long long (*s_key)[kWaves],
                                           float4 (*s_xyz)[kWaves], float x0, float y0, float z0,
                                           int L) {
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const unsigned long long wmax = wave_max_u64(key);
    if (key == wmax && wmax != 0ull) s_xyz[buf][wave] = make_float4(bx, by, bz, 0.f);
    if (lane == 0) s_key[buf][wave] = wmax;
    __syncthreads();
    // every wave reduces the 16 wave maxima on its first 16 lanes (no 2nd barrier)
    const unsigned long long v = (lane < kWaves) ? s_key[buf][lane] : 0ull;
    unsigned long long best = v;
#pragma unroll
    for (int off = kWaves / 2; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(best, off);
        best = o > best ? o : best;
    }
    best = __shfl(best, 0);
    const unsigned long long hit = __ballot(lane < kWaves && v == best);
    const int bw = __ffsll((long long)hit) - 1;
    Pick p;
    if (best == 0ull) {  // no candidate anywhere: upstream keeps thread 0's besti = 0
        p.x = x0; p.y = y0; p.z = z0; p.k = 0;
    } else {
        const float4 c = s_xyz[buf][bw];
        p.x = c.x; p.y = c.y; p.z = c.z;
        p.k = fps_unrank(~(uint32_t)(best & 0xffffffffull), L);
    }
    return p;
}

template <int PPT>
__global__ __launch_bounds__(kThreads) void fps_reg_kernel(const float* __restrict__ xyz, int N,
                                                           int M, int L,
                                                           int32_t* __restrict__ idx,
                                                           float* __restrict__ new_xyz) {
    __shared__ unsigned long long s_key[2][kWaves];
    __shared__ float4 s_xyz[2][kWaves];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const float* __restrict__ p = xyz + (size_t)b * N * 3;
    idx += (size_t)b * M;
    if (new_xyz) new_xyz += (size_t)b * M * 3;

    float px[PPT], py[PPT], pz[PPT], td[PPT];
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const int k = tid + i * kThreads;
        if (k < N) {
            const float x = p[3 * k], y = p[3 * k + 1], z = p[3 * k + 2];
            const float mag = fmaf(z, z, fmaf(y, y, x * x));
            px[i] = x; py[i] = y; pz[i] = z;
            td[i] = ((double)mag <= 1e-3) ? -1.f : 1e10f;  // -1: never a candidate
        } else {
            px[i] = 0.f; py[i] = 0.f; pz[i] = 0.f; td[i] = -1.f;
        }
    }
    const float x0 = p[0], y0 = p[1], z0 = p[2];
    float x1 = x0, y1 = y0, z1 = z0;
    if (tid == 0) {
        idx[0] = 0;
        if (new_xyz) { new_xyz[0] = x0; new_xyz[1] = y0; new_xyz[2] = z0; }
    }
    for (int j = 1; j < M; ++j) {
        float best = -1.f, bx = 0.f, by = 0.f, bz = 0.f;
        int bi = 0;
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            const float dx = px[i] - x1, dy = py[i] - y1, dz = pz[i] - z1;
            const float d = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
            const float d2 = fminf(d, td[i]);
            td[i] = d2;
            const bool gt = d2 > best;
            best = gt ? d2 : best;
            bi = gt ? i : bi;
            bx = gt ? px[i] : bx;
            by = gt ? py[i] : by;
            bz = gt ? pz[i] : bz;
        }
        unsigned long long key = 0ull;
        if (best >= 0.f)
            key = ((unsigned long long)__float_as_uint(best) << 32) |
                  (unsigned long long)(~fps_rank((uint32_t)(tid + bi * kThreads), L));
        const Pick pk = block_pick(key, bx, by, bz, j & 1, s_key, s_xyz, x0, y0, z0, L);
        x1 = pk.x; y1 = pk.y; z1 = pk.z;
        if (tid == 0) {
            idx[j] = pk.k;
            if (new_xyz) { new_xyz[3 * j] = pk.x; new_xyz[3 * j + 1] = pk.y; new_xyz[3 * j + 2] = pk.z; }
        }
    }
}

// Large-N path (N > kThreads * kMaxPPT): running distances in a global workspace.
__global__ __launch_bounds__(kThreads) void fps_global_kernel(const float* __restrict__ xyz, int N,
                                                              int M, int L, float* __restrict__ temp,
                                                              int32_t* __restrict__ idx,
                                                              float* __restrict__ new_xyz) {
    __shared__ unsigned long long s_key[2][kWaves];
    __shared__ float4 s_xyz[2][kWaves];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const float* __restrict__ p = xyz + (size_t)b * N * 3;
    temp += (size_t)b * N;
    idx += (size_t)b * M;
    if (new_xyz) new_xyz += (size_t)b * M * 3;
    for (int k = tid; k < N; k += kThreads) {
        const float x = p[3 * k], y = p[3 * k + 1], z = p[3 * k + 2];
        const float mag = fmaf(z, z, fmaf(y, y, x * x));
        temp[k] = ((double)mag <= 1e-3) ? -1.f : 1e10f;
    }
    const float x0 = p[0], y0 = p[1], z0 = p[2];
    float x1 = x0, y1 = y0, z1 = z0;
    if (tid == 0) {
        idx[0] = 0;
        if (new_xyz) { new_xyz[0] = x0; new_xyz[1] = y0; new_xyz[2] = z0; }
    }
    __syncthreads();
    for (int j = 1; j < M; ++j) {
        float best = -1.f, bx = 0.f, by = 0.f, bz = 0.f;
        int bk = 0;
        for (int k = tid; k < N; k += kThreads) {
            const float x = p[3 * k], y = p[3 * k + 1], z = p[3 * k + 2];
            const float t = temp[k];
            const float dx = x - x1, dy = y - y1, dz = z - z1;
            const float d = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
            const float d2 = fminf(d, t);
            temp[k] = d2;
            const bool gt = d2 > best;
            best = gt ? d2 : best;
            bk = gt ? k : bk;
            bx = gt ? x : bx; by = gt ? y : by; bz = gt ? z : bz;
        }
        unsigned long long key = 0ull;
        if (best >= 0.f)
            key = ((unsigned long long)__float_as_uint(best) << 32) |
                  (unsigned long long)(~fps_rank((uint32_t)bk, L));
        const Pick pk = block_pick(key, bx, by, bz, j & 1, s_key, s_xyz, x0, y0, z0, L);
        x1 = pk.x; y1 = pk.y; z1 = pk.z;
        if (tid == 0) {
            idx[j] = pk.k;
            if (new_xyz) { new_xyz[3 * j] = pk.x; new_xyz[3 * j + 1] = pk.y; new_xyz[3 * j + 2] = pk.z; }
        }
    }
}

template <int PPT>
void launch_reg(const float* xyz, int B, int N, int M, int L, int32_t* idx, float* nx,
                hipStream_t s) {
    hipLaunchKernelGGL(fps_reg_kernel<PPT>, dim3(B), dim3(kThreads), 0, s, xyz, N, M, L, idx, nx);
}

}  // namespace

extern "C" int ov3d_fps(const float* xyz, int B, int N, int M, int32_t* idx_out,
                        float* new_xyz_out, float* workspace, void* stream) {
    if (B < 0 || N <= 0 || M < 0 || !xyz || (!idx_out && B * M > 0)) return OV3D_EINVAL;
    if (B == 0 || M == 0) return OV3D_OK;
    // upstream block size: largest power of two <= N, capped at 512
    int bs = 1, L = 0;
    while (bs * 2 <= N && bs < 512) { bs *= 2; ++L; }
    hipStream_t s = ov3d_stream(stream);
    const int ppt = (N + kThreads - 1) / kThreads;
    if (ppt <= kMaxPPT) {
        if (ppt <= 1) launch_reg<1>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 2) launch_reg<2>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 3) launch_reg<3>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 4) launch_reg<4>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 6) launch_reg<6>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 8) launch_reg<8>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 10) launch_reg<10>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 12) launch_reg<12>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 16) launch_reg<16>(xyz, B, N, M, L, idx_out, new_xyz_out, s);

        else launch_reg<20>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
    } else {
        if (!workspace) return OV3D_EINVAL;
        hipLaunchKernelGGL(fps_global_kernel, dim3(B), dim3(kThreads), 0, s, xyz, N, M, L, workspace,
                           idx_out, new_xyz_out);
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" const char* ov3d_version(void) { return "ov3d-hip 0.1 gfx950"; }
