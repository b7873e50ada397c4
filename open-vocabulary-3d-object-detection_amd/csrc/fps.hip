// Furthest-point sampling for gfx950.
//
// Replaces third_party.pointnet2 furthest_point_sampling (un-vendored; called at
// models/model_3detr.py:174 and in PointnetSAModuleVotes, model_3detr.py:355-361).
//
// Design (one 1024-thread workgroup = 16 waves per scene, the scene's points
// held in registers for the whole run):
//   * PPT slots per thread, coordinates + running min-distance in VGPRs
//     (4 regs per slot), points grouped into one spatial cluster per wave;
//   * per iteration: waves whose cluster cannot get closer skip (exact), the
//     others do the VALU distance update + per-thread argmax + DPP reduction;
//     one LDS slot per wave (double-buffered by iteration parity -> ONE barrier
//     per iteration), every wave reduces the 16 wave slots and reads the
//     winner's coordinates from LDS;
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
#include <stdlib.h>

#include "common.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

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

// ---------------------------------------------------------------------------
// Spatially culled FPS (N <= kThreads * kMaxPPT).
//
// Setup (once per launch, one workgroup per scene): scene bbox -> 16^3 Morton
// cell code per point -> LDS counting sort -> wave w owns sorted positions
// [w*64*PPT, (w+1)*64*PPT), i.e. a compact spatial cluster; each thread sorts
// its PPT slots by tie-break rank so that strict '>' inside the thread keeps the
// upstream tie rule; per-wave bounding box.
// Iteration: a wave updates its points only if the new sample can be closer
// than the wave's current max running distance: lb = |gap(new, wave bbox)|^2 is
// evaluated with the same monotone float ops as the point distances, so
// lb >= wave_tmax implies min(d, temp) == temp for every point of the wave
// (exact skip, results unchanged).  Skipping waves re-publish their cached
// best.  ~1/4 of the waves update per iteration on SUN scenes (measured in the
// DESIGN.md simulation), the rest cost ~15 VALU ops.
// Reductions: DPP row reductions + readlane, 32-bit keys (distance bits, then
// min rank only when distances tie).
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ int dpp_mov(int v, int identity) {
    // lanes outside the row mask read `identity`: lets the compiler fold the move into
    // the consuming v_max/v_min (one v_max_i32_dpp per step instead of mov + max)
    return __builtin_amdgcn_update_dpp(identity, v, CTRL, ROWS, 0xf, false);
}

// every lane of each 16-lane row gets the row's max / min
__device__ __forceinline__ int row_max_i32(int v) {
    v = max(v, dpp_mov<0xb1>(v, INT_MIN));   // quad_perm(1,0,3,2)
    v = max(v, dpp_mov<0x4e>(v, INT_MIN));   // quad_perm(2,3,0,1)
    v = max(v, dpp_mov<0x141>(v, INT_MIN));  // row_half_mirror
    v = max(v, dpp_mov<0x140>(v, INT_MIN));  // row_mirror
    return v;
}

__device__ __forceinline__ uint32_t row_min_u32(uint32_t v) {
    v = min(v, (uint32_t)dpp_mov<0xb1>((int)v, -1));
    v = min(v, (uint32_t)dpp_mov<0x4e>((int)v, -1));
    v = min(v, (uint32_t)dpp_mov<0x141>((int)v, -1));
    v = min(v, (uint32_t)dpp_mov<0x140>((int)v, -1));
    return v;
}

// wave64 reductions: rows, then row_bcast15 / row_bcast31 fold rows into lane 63
__device__ __forceinline__ int wave_max_i32(int v) {
    v = row_max_i32(v);
    v = max(v, dpp_mov<0x142, 0xa>(v, INT_MIN));  // row_bcast:15 into rows 1, 3
    v = max(v, dpp_mov<0x143, 0xc>(v, INT_MIN));  // row_bcast:31 into rows 2, 3
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = row_min_u32(v);
    v = min(v, (uint32_t)dpp_mov<0x142, 0xa>((int)v, -1));
    v = min(v, (uint32_t)dpp_mov<0x143, 0xc>((int)v, -1));
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ float wave_fmin(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fminf(v, __shfl_xor(v, off));
    return v;
}
__device__ __forceinline__ float wave_fmax(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}

__device__ __forceinline__ uint32_t spread3(uint32_t x) {  // 4 bits -> every 3rd bit
    x &= 0xf;
    x = (x | (x << 4)) & 0x0c3;
    x = (x | (x << 2)) & 0x249;
    return x;
}

constexpr int kCells = 4096;
constexpr int kMaxOutLDS = 8192;  // deferred outputs: M <= 8192 on the culled path

template <int PPT>
__global__ __launch_bounds__(kThreads) void fps_cull_kernel(const float* __restrict__ xyz, int N,
                                                            int M, int L,
                                                            int32_t* __restrict__ idx,
                                                            float* __restrict__ new_xyz
#ifdef OV3D_FPS_PROBE
                                                            , unsigned long long* __restrict__ dbg
#endif
                                                            ) {
    constexpr int PW = PPT * 64;
    __shared__ uint32_t s_hist[kCells];
    __shared__ uint16_t s_perm[kThreads * PPT];
    __shared__ uint16_t s_out[kMaxOutLDS];     // winner position per iteration (outputs deferred)
    __shared__ float s_red[6][kWaves];
    __shared__ uint32_t s_scan[kWaves];
    __shared__ float4 s_pub[2][kWaves];         // per-wave best: x, y, z, distance bits
    __shared__ int s_pos[2][kWaves];            // per-wave best: sorted position

    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const float* __restrict__ p = xyz + (size_t)b * N * 3;
    idx += (size_t)b * M;
    if (new_xyz) new_xyz += (size_t)b * M * 3;

    // ---- (a) scene bbox
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = tid; k < N; k += kThreads)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float v = p[3 * k + a];
            lo[a] = fminf(lo[a], v);
            hi[a] = fmaxf(hi[a], v);
        }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        lo[a] = wave_fmin(lo[a]);
        hi[a] = wave_fmax(hi[a]);
    }
    if (lane == 0)
#pragma unroll
        for (int a = 0; a < 3; ++a) { s_red[a][w] = lo[a]; s_red[3 + a][w] = hi[a]; }
    for (int i = tid; i < kCells; i += kThreads) s_hist[i] = 0;
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float l = s_red[a][0], h = s_red[3 + a][0];
        for (int q = 1; q < kWaves; ++q) { l = fminf(l, s_red[a][q]); h = fmaxf(h, s_red[3 + a][q]); }
        lo[a] = l;
        hi[a] = 16.f / fmaxf(h - l, 1e-6f);  // cell scale
    }

    // ---- (b) cell codes + LDS counting sort (order inside a cell is irrelevant:
    //          ties are decided by rank, never by layout)
    uint32_t cp[PPT];
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const int k = tid + i * kThreads;
        cp[i] = 0xffffffffu;
        if (k < N) {
            uint32_t q[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const int c = (int)((p[3 * k + a] - lo[a]) * hi[a]);
                q[a] = (uint32_t)min(max(c, 0), 15);
            }
            const uint32_t code = spread3(q[0]) | (spread3(q[1]) << 1) | (spread3(q[2]) << 2);
            const uint32_t old = atomicAdd(&s_hist[code], 1u);
            cp[i] = (code << 16) | old;
        }
    }
    __syncthreads();
    {   // exclusive scan of the 4096 cell counts: 4 per thread
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) { v[q] = s_hist[4 * tid + q]; sum += v[q]; }
        uint32_t inc = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t o = __shfl_up(inc, off);
            if (lane >= off) inc += o;
        }
        if (lane == 63) s_scan[w] = inc;
        __syncthreads();
        uint32_t base = 0;
        for (int q = 0; q < w; ++q) base += s_scan[q];
        uint32_t run = base + inc - sum;
#pragma unroll
        for (int q = 0; q < 4; ++q) { s_hist[4 * tid + q] = run; run += v[q]; }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PPT; ++i)
        if (cp[i] != 0xffffffffu)
            s_perm[s_hist[cp[i] >> 16] + (cp[i] & 0xffffu)] = (uint16_t)(tid + i * kThreads);
    __syncthreads();

    // ---- (c) this thread's slots: wave w, positions w*PW + i*64 + lane, sorted by rank
    uint32_t rk[PPT];
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const int pos = w * PW + i * 64 + lane;
        rk[i] = pos < N ? fps_rank(s_perm[pos], L) : 0xffffffffu;
    }
#pragma unroll
    for (int pass = 0; pass < PPT; ++pass)
#pragma unroll
        for (int i = pass & 1; i + 1 < PPT; i += 2) {
            const uint32_t a = rk[i], c = rk[i + 1];
            rk[i] = min(a, c);
            rk[i + 1] = max(a, c);
        }
    // coordinates as packed pairs (slot 2j, 2j+1): the distance update runs on v_pk_add /
    // v_pk_mul / v_pk_fma, two points per instruction; an odd PPT pads one dead slot
    constexpr int NP = (PPT + 1) / 2;
    f32x2 px[NP], py[NP], pz[NP];
    float td[2 * NP];
    float wlo[3] = {INFINITY, INFINITY, INFINITY}, whi[3] = {-INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int i = 0; i < 2 * NP; ++i) {
        const int pos = w * PW + i * 64 + lane;
        if (i < PPT && rk[i] != 0xffffffffu) {
            const int k = fps_unrank(rk[i], L);
            s_perm[pos] = (uint16_t)k;
            const float x = p[3 * k], y = p[3 * k + 1], z = p[3 * k + 2];
            const float mag = fmaf(z, z, fmaf(y, y, x * x));
            px[i >> 1][i & 1] = x; py[i >> 1][i & 1] = y; pz[i >> 1][i & 1] = z;
            const bool skip = (double)mag <= 1e-3;
            td[i] = skip ? -1.f : 1e10f;
            if (!skip) {
                wlo[0] = fminf(wlo[0], x); wlo[1] = fminf(wlo[1], y); wlo[2] = fminf(wlo[2], z);
                whi[0] = fmaxf(whi[0], x); whi[1] = fmaxf(whi[1], y); whi[2] = fmaxf(whi[2], z);
            }
        } else {
            px[i >> 1][i & 1] = 0.f; py[i >> 1][i & 1] = 0.f; pz[i >> 1][i & 1] = 0.f;
            td[i] = -1.f;
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        wlo[a] = wave_fmin(wlo[a]);
        whi[a] = wave_fmax(whi[a]);
    }
    const float x0 = p[0], y0 = p[1], z0 = p[2];
    float x1 = x0, y1 = y0, z1 = z0;
    // wave cache: best distance (float bits), its sorted position and coordinates
    float wtmax = INFINITY;
    int wdist = __float_as_int(-1.f);
    int wpos = 0;
    float wx = 0.f, wy = 0.f, wz = 0.f;

#ifdef OV3D_FPS_PROBE
    // diagnostic build only (tools/fps_probe.py): per-wave phase cycle totals
    unsigned long long pr_wm = 0, pr_slot = 0, pr_xyz = 0, pr_loop = 0, pr_upd = 0, pr_nupd = 0, pr_cupd = 0, pr_cnupd = 0, pr_bar = 0, pr_post = 0;
    const unsigned long long pr_rt0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long pr_c0 = __builtin_amdgcn_s_memtime();
#endif
    for (int j = 1; j < M; ++j) {
#ifdef OV3D_FPS_PROBE
        const unsigned long long pt0 = __builtin_amdgcn_s_memtime();
        bool pr_did = false;
#endif
        const int buf = j & 1;
        const float gx = fmaxf(fmaxf(wlo[0] - x1, x1 - whi[0]), 0.f);
        const float gy = fmaxf(fmaxf(wlo[1] - y1, y1 - whi[1]), 0.f);
        const float gz = fmaxf(fmaxf(wlo[2] - z1, z1 - whi[2]), 0.f);
        const float lb = fmaf(gz, gz, fmaf(gy, gy, gx * gx));
        if (lb < wtmax) {  // wave-uniform
#ifdef OV3D_FPS_PROBE
            pr_did = true;
#endif
            // per point: the packed distance (3 pk ops per pair), min into the running
            // distance, and max3 into the lane's best -- the slot of the best is found after
            // the wave reduction, on the winning lane only
            const f32x2 cx = {x1, x1}, cy = {y1, y1}, cz = {z1, z1};
            float best = -1.f;
#pragma unroll
            for (int j = 0; j < NP; ++j) {
                const f32x2 dx = px[j] - cx, dy = py[j] - cy, dz = pz[j] - cz;
                const f32x2 d = __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
                td[2 * j] = fminf(d.x, td[2 * j]);   // no NaN canonicalisation: built non-IEEE (Makefile)
                td[2 * j + 1] = fminf(d.y, td[2 * j + 1]);
                best = fmaxf(best, fmaxf(td[2 * j], td[2 * j + 1]));
            }
#ifdef OV3D_FPS_PROBE
            pr_loop += __builtin_amdgcn_s_memtime() - pt0;
#endif
            const int bb = __float_as_int(best);
            // the slot of the lane's best: the first pair whose max is the best, then the first
            // slot of that pair holding it (slots are in rank order: the upstream tie rule inside
            // a thread); a 10-step select chain, independent of the wave reduction below
            int bi = 0;
#pragma unroll
            for (int j = NP - 1; j >= 0; --j) {
                const int in_pair = __float_as_int(td[2 * j]) == bb ? 2 * j : 2 * j + 1;
                bi = __float_as_int(fmaxf(td[2 * j], td[2 * j + 1])) == bb ? in_pair : bi;
            }
            const int wm = wave_max_i32(bb);
#ifdef OV3D_FPS_PROBE
            unsigned long long pq = __builtin_amdgcn_s_memtime();
            pr_wm += pq - pt0;
#endif
            wdist = wm;
            wtmax = __int_as_float(wm);
            if (wm >= 0) {
                const unsigned long long cand = __ballot(bb == wm);
                int wl;
                if (__popcll(cand) == 1) {
                    wl = __ffsll((long long)cand) - 1;
                } else {  // distance tie inside the wave: smallest rank wins
                    uint32_t my = 0xffffffffu;
                    if (bb == wm) my = fps_rank(s_perm[w * PW + bi * 64 + lane], L);
                    const uint32_t mr = wave_min_u32(my);
                    wl = __ffsll((long long)__ballot(my == mr)) - 1;
                }
                const int slot = __builtin_amdgcn_readlane(bi, wl);
#ifdef OV3D_FPS_PROBE
                { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); pr_slot += t_ - pq; pq = t_; }
#endif
                // the winner's coordinates: slot is wave-uniform, so hipcc reads them from a
                // private copy of the slot arrays at a scalar offset (three loads, no branches;
                // round 5's uniform switch over the slots was 0.11 us per iteration slower, the
                // slots as vector values indexed by the GPR-index mode 0.08 us slower)
                wx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(px[slot >> 1][slot & 1]), wl));
                wy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(py[slot >> 1][slot & 1]), wl));
                wz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pz[slot >> 1][slot & 1]), wl));
                wpos = w * PW + slot * 64 + wl;
#ifdef OV3D_FPS_PROBE
                pr_xyz += __builtin_amdgcn_s_memtime() - pq;
#endif
            }
        }
#ifdef OV3D_FPS_PROBE
        const unsigned long long pt1 = __builtin_amdgcn_s_memtime();
        if (pr_did) { pr_upd++; pr_cupd += pt1 - pt0; } else { pr_nupd++; pr_cnupd += pt1 - pt0; }
#endif
        if (lane == 0) {
            s_pub[buf][w] = make_float4(wx, wy, wz, __int_as_float(wdist));
            s_pos[buf][w] = wpos;
        }
        // only LDS is shared inside the loop: wait for LDS, not for global memory
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#ifdef OV3D_FPS_PROBE
        const unsigned long long pt2 = __builtin_amdgcn_s_memtime();
        pr_bar += pt2 - pt1;
#endif
        // every row of the wave reads the 16 wave slots (lane & 15): the row reduction
        // leaves the maximum in every lane, no lane masking
        const float4 v = s_pub[buf][lane & (kWaves - 1)];
        int vp = s_pos[buf][lane & (kWaves - 1)];
        // both LDS reads in flight together (hipcc would sink the position read below the
        // branch: a second LDS round trip on the iteration's serial chain)
        asm volatile("" : "+v"(vp));
        const int dv = __float_as_int(v.w);
        const int dm = __builtin_amdgcn_readfirstlane(row_max_i32(dv));
        int pj;
        if (dm < 0) {  // no candidate anywhere: upstream keeps thread 0's besti = 0
            pj = 0xffff;
            x1 = x0; y1 = y0; z1 = z0;
        } else {
            const unsigned long long cand = __ballot(dv == dm) & 0xffffull;
            int ws;
            if (__popcll(cand) == 1) {
                ws = __ffsll((long long)cand) - 1;
            } else {  // distance tie across waves: smallest rank wins
                const uint32_t r = dv == dm ? fps_rank(s_perm[vp], L) : 0xffffffffu;
                const uint32_t rm = __builtin_amdgcn_readfirstlane(row_min_u32(r));
                ws = __ffsll((long long)(__ballot(r == rm) & 0xffffull)) - 1;
            }
            x1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), ws));
            y1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), ws));
            z1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.z), ws));
            pj = __builtin_amdgcn_readlane(vp, ws);
        }
        if (tid == 0) s_out[j] = (uint16_t)pj;
#ifdef OV3D_FPS_PROBE
        pr_post += __builtin_amdgcn_s_memtime() - pt2;
#endif
    }
#ifdef OV3D_FPS_PROBE
    {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime();
        const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            unsigned long long* o = dbg + ((size_t)b * kWaves + w) * 12;
            o[0] = pr_upd; o[1] = pr_cupd; o[2] = pr_nupd; o[3] = pr_cnupd;
            o[4] = pr_bar; o[5] = pr_post; o[6] = c1 - pr_c0; o[7] = rt1 - pr_rt0; o[8] = pr_loop;
            o[9] = pr_wm; o[10] = pr_slot; o[11] = pr_xyz;
        }
    }
#endif
    __syncthreads();
    // ---- deferred outputs: indices + gathered coordinates, coalesced
    for (int j = tid; j < M; j += kThreads) {
        int k = 0;
        if (j > 0 && s_out[j] != 0xffff) k = s_perm[s_out[j]];
        idx[j] = k;
        if (new_xyz) {
            new_xyz[3 * j] = p[3 * k];
            new_xyz[3 * j + 1] = p[3 * k + 1];
            new_xyz[3 * j + 2] = p[3 * k + 2];
        }
    }
}


// ---------------------------------------------------------------------------
// Culled FPS for kThreads*kMaxPPT < N <= kThreads*(kPR+kPS) (ScanNet: 40000 points).
// A CU cannot hold 40000 points (16 B each: 640 KB > 512 KB of VGPRs + 160 KB of LDS), so
// each wave owns TWO spatial clusters of the Morton order: cluster A (kPR slots per lane,
// coordinates + running distance in VGPRs, exactly as fps_cull_kernel) and cluster B
// (kPS slots per lane as float4 (x, y, z, running distance) in a global workspace that stays
// in L2: 384 KB per scene).  Each cluster has its own bounding box, max running distance and
// cached best, and is skipped by the same exact test; only B's updates touch memory (one
// 16-byte load + one 4-byte store per slot, read back only by the lane that wrote it).
// The wave publishes the better of its two candidates (distance, then smaller rank).
constexpr int kPR = 16, kPS = 24;

__device__ __forceinline__ float sgpr_f(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// kCS: slots per cluster-B chunk (kNCB = kPS / kCS chunks, <= 16)
template <int kCS>
__global__ __launch_bounds__(kThreads) void fps_stream_kernel(const float* __restrict__ xyz, int N,
                                                              int M, int L,
                                                              float4* __restrict__ ws,
                                                              int32_t* __restrict__ idx,
                                                              float* __restrict__ new_xyz) {
    constexpr int PA = kPR * 64, PB = kPS * 64;   // positions per wave: cluster A, cluster B
    constexpr int NA = kWaves * PA;               // cluster B positions start here
    constexpr int NS = kPR + kPS;                 // slots per thread in the setup
    constexpr int kNCB = kPS / kCS;
    static_assert(kPS % kCS == 0 && kNCB <= 16, "cluster B chunking");
    __shared__ uint32_t s_hist[kCells];
    __shared__ uint16_t s_perm[kThreads * NS];
    __shared__ uint16_t s_out[kMaxOutLDS];
    __shared__ float s_red[6][kWaves];
    __shared__ uint32_t s_scan[kWaves];
    __shared__ float4 s_pub[2][kWaves];
    __shared__ int s_pos[2][kWaves];

    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar addressing)
    const float* __restrict__ p = xyz + (size_t)b * N * 3;
    idx += (size_t)b * M;
    if (new_xyz) new_xyz += (size_t)b * M * 3;
    // slot i of this lane at wsw[64 i + lane]: scalar base + 32-bit lane offset per access
    float4* __restrict__ wsw = ws + ((size_t)b * kWaves + w) * kPS * 64;

    // ---- (a) scene bbox, (b) Morton cell codes + LDS counting sort (as fps_cull_kernel)
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = tid; k < N; k += kThreads)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float v = p[3 * k + a];
            lo[a] = fminf(lo[a], v);
            hi[a] = fmaxf(hi[a], v);
        }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        lo[a] = wave_fmin(lo[a]);
        hi[a] = wave_fmax(hi[a]);
    }
    if (lane == 0)
#pragma unroll
        for (int a = 0; a < 3; ++a) { s_red[a][w] = lo[a]; s_red[3 + a][w] = hi[a]; }
    for (int i = tid; i < kCells; i += kThreads) s_hist[i] = 0;
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float l = s_red[a][0], h = s_red[3 + a][0];
        for (int q = 1; q < kWaves; ++q) { l = fminf(l, s_red[a][q]); h = fmaxf(h, s_red[3 + a][q]); }
        lo[a] = l;
        hi[a] = 16.f / fmaxf(h - l, 1e-6f);
    }
    uint32_t cp[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const int k = tid + i * kThreads;
        cp[i] = 0xffffffffu;
        if (k < N) {
            uint32_t q[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const int c = (int)((p[3 * k + a] - lo[a]) * hi[a]);
                q[a] = (uint32_t)min(max(c, 0), 15);
            }
            const uint32_t code = spread3(q[0]) | (spread3(q[1]) << 1) | (spread3(q[2]) << 2);
            const uint32_t old = atomicAdd(&s_hist[code], 1u);
            cp[i] = (code << 16) | old;
        }
    }
    __syncthreads();
    {
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) { v[q] = s_hist[4 * tid + q]; sum += v[q]; }
        uint32_t inc = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t o = __shfl_up(inc, off);
            if (lane >= off) inc += o;
        }
        if (lane == 63) s_scan[w] = inc;
        __syncthreads();
        uint32_t base = 0;
        for (int q = 0; q < w; ++q) base += s_scan[q];
        uint32_t run = base + inc - sum;
#pragma unroll
        for (int q = 0; q < 4; ++q) { s_hist[4 * tid + q] = run; run += v[q]; }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NS; ++i)
        if (cp[i] != 0xffffffffu)
            s_perm[s_hist[cp[i] >> 16] + (cp[i] & 0xffffu)] = (uint16_t)(tid + i * kThreads);
    __syncthreads();

    // ---- (c) cluster B slots (first: their ranks are dead before cluster A fills its
    //      registers): positions NA + w*PB + i*64 + lane, sorted by rank, to the workspace.
    //      Cluster B is culled per chunk of 4 slots (256 consecutive Morton positions):
    //      chunk c's bounding box and cached best live in lane c (lane-distributed).
    float qLo[3] = {INFINITY, INFINITY, INFINITY}, qHi[3] = {-INFINITY, -INFINITY, -INFINITY};
    {
        float cLo[kNCB][3], cHi[kNCB][3];
#pragma unroll
        for (int c = 0; c < kNCB; ++c)
#pragma unroll
            for (int a = 0; a < 3; ++a) { cLo[c][a] = INFINITY; cHi[c][a] = -INFINITY; }
        uint32_t rk[kPS];
#pragma unroll
        for (int i = 0; i < kPS; ++i) {
            const int pos = NA + w * PB + i * 64 + lane;
            rk[i] = pos < N ? fps_rank(s_perm[pos], L) : 0xffffffffu;
        }
#pragma unroll
        for (int pass = 0; pass < kPS; ++pass)
#pragma unroll
            for (int i = pass & 1; i + 1 < kPS; i += 2) {
                const uint32_t a = rk[i], c = rk[i + 1];
                rk[i] = min(a, c);
                rk[i + 1] = max(a, c);
            }
#pragma unroll
        for (int i = 0; i < kPS; ++i) {
            const int pos = NA + w * PB + i * 64 + lane;
            float4 e = make_float4(0.f, 0.f, 0.f, -1.f);
            if (rk[i] != 0xffffffffu) {
                const int k = fps_unrank(rk[i], L);
                s_perm[pos] = (uint16_t)k;
                const float x = p[3 * k], y = p[3 * k + 1], z = p[3 * k + 2];
                const bool skip = (double)fmaf(z, z, fmaf(y, y, x * x)) <= 1e-3;
                e = make_float4(x, y, z, skip ? -1.f : 1e10f);
                if (!skip) {
                    float* lo = cLo[i / kCS];
                    float* hi = cHi[i / kCS];
                    lo[0] = fminf(lo[0], x); lo[1] = fminf(lo[1], y); lo[2] = fminf(lo[2], z);
                    hi[0] = fmaxf(hi[0], x); hi[1] = fmaxf(hi[1], y); hi[2] = fmaxf(hi[2], z);
                }
            }
            wsw[64 * i + lane] = e;
        }
#pragma unroll
        for (int c = 0; c < kNCB; ++c)
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const float lo = wave_fmin(cLo[c][a]), hi = wave_fmax(cHi[c][a]);
                if (lane == c) { qLo[a] = lo; qHi[a] = hi; }
            }
    }
    // ---- cluster A slots: positions w*PA + i*64 + lane, sorted by rank, in registers
    float px[kPR], py[kPR], pz[kPR], td[kPR];
    float aLo[3] = {INFINITY, INFINITY, INFINITY}, aHi[3] = {-INFINITY, -INFINITY, -INFINITY};
    {
        uint32_t rk[kPR];
#pragma unroll
        for (int i = 0; i < kPR; ++i) {
            const int pos = w * PA + i * 64 + lane;
            rk[i] = pos < N ? fps_rank(s_perm[pos], L) : 0xffffffffu;
        }
#pragma unroll
        for (int pass = 0; pass < kPR; ++pass)
#pragma unroll
            for (int i = pass & 1; i + 1 < kPR; i += 2) {
                const uint32_t a = rk[i], c = rk[i + 1];
                rk[i] = min(a, c);
                rk[i + 1] = max(a, c);
            }
#pragma unroll
        for (int i = 0; i < kPR; ++i) {
            const int pos = w * PA + i * 64 + lane;
            px[i] = 0.f; py[i] = 0.f; pz[i] = 0.f; td[i] = -1.f;
            if (rk[i] != 0xffffffffu) {
                const int k = fps_unrank(rk[i], L);
                s_perm[pos] = (uint16_t)k;
                const float x = p[3 * k], y = p[3 * k + 1], z = p[3 * k + 2];
                const bool skip = (double)fmaf(z, z, fmaf(y, y, x * x)) <= 1e-3;
                px[i] = x; py[i] = y; pz[i] = z;
                td[i] = skip ? -1.f : 1e10f;
                if (!skip) {
                    aLo[0] = fminf(aLo[0], x); aLo[1] = fminf(aLo[1], y); aLo[2] = fminf(aLo[2], z);
                    aHi[0] = fmaxf(aHi[0], x); aHi[1] = fmaxf(aHi[1], y); aHi[2] = fmaxf(aHi[2], z);
                }
            }
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {   // wave-uniform: scalar registers
        aLo[a] = sgpr_f(wave_fmin(aLo[a]));
        aHi[a] = sgpr_f(wave_fmax(aHi[a]));
    }
    __syncthreads();   // s_perm complete before any tie lookup
    // this wave's cluster-B slots through a buffer descriptor: scalar base + lane offset +
    // a constant slot offset per access (64-bit per-slot addresses would take 48 VGPRs)
    const uint64_t wsa = reinterpret_cast<uint64_t>(wsw);
    float4* const wsu = reinterpret_cast<float4*>(
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(wsa >> 32)) << 32) |
        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wsa));
    const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc(wsu, 0, kPS * 64 * 16, 0x00020000);
    const float x0 = p[0], y0 = p[1], z0 = p[2];
    float x1 = x0, y1 = y0, z1 = z0;
    // per-cluster cache: max running distance, best distance bits, position, coordinates
    float aT = INFINITY;
    int aD = __float_as_int(-1.f), aP = 0;
    float aX = 0.f, aY = 0.f, aZ = 0.f;
    // cluster B chunk caches, chunk c in lane c (lanes >= kNCB: never updated)
    float qT = lane < kNCB ? INFINITY : -INFINITY;
    int qD = __float_as_int(-1.f), qP = 0;
    float qX = 0.f, qY = 0.f, qZ = 0.f;

    // wave argmax of (dist bits bb, slot bi, coords) over the lanes -> cache (T, D, P, X, Y, Z)
    auto wave_pick = [&](float best, int bi, float sx, float sy, float sz, int pbase,
                         float& T, int& Dd, int& P, float& X, float& Y, float& Z)
        __attribute__((always_inline)) {
        const int bb = __float_as_int(best);
        const int wm = wave_max_i32(bb);
        Dd = wm;
        T = __int_as_float(wm);
        if (wm >= 0) {
            const unsigned long long cand = __ballot(bb == wm);
            int wl;
            if (__popcll(cand) == 1) {
                wl = __ffsll((long long)cand) - 1;
            } else {   // distance tie inside the cluster: smallest rank wins
                uint32_t my = 0xffffffffu;
                if (bb == wm) my = fps_rank(s_perm[pbase + bi * 64 + lane], L);
                const uint32_t mr = wave_min_u32(my);
                wl = __ffsll((long long)__ballot(my == mr)) - 1;
            }
            X = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sx), wl));
            Y = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sy), wl));
            Z = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sz), wl));
            P = pbase + __builtin_amdgcn_readlane(bi, wl) * 64 + wl;
        }
    };

    for (int j = 1; j < M; ++j) {
        const int buf = j & 1;
        {   // cluster A (registers)
            const float gx = fmaxf(fmaxf(aLo[0] - x1, x1 - aHi[0]), 0.f);
            const float gy = fmaxf(fmaxf(aLo[1] - y1, y1 - aHi[1]), 0.f);
            const float gz = fmaxf(fmaxf(aLo[2] - z1, z1 - aHi[2]), 0.f);
            if (fmaf(gz, gz, fmaf(gy, gy, gx * gx)) < aT) {
                float best = -1.f, sx = 0.f, sy = 0.f, sz = 0.f;
                int bi = 0;
#pragma unroll
                for (int i = 0; i < kPR; ++i) {
                    const float dx = px[i] - x1, dy = py[i] - y1, dz = pz[i] - z1;
                    const float d2 = fminf(fmaf(dz, dz, fmaf(dy, dy, dx * dx)), td[i]);
                    td[i] = d2;
                    const bool gt = d2 > best;
                    best = gt ? d2 : best;
                    bi = gt ? i : bi;
                    sx = gt ? px[i] : sx; sy = gt ? py[i] : sy; sz = gt ? pz[i] : sz;
                }
                wave_pick(best, bi, sx, sy, sz, w * PA, aT, aD, aP, aX, aY, aZ);
            }
        }
        {   // cluster B (workspace, L2-resident): only the chunks that can change are loaded
            const float gx = fmaxf(fmaxf(qLo[0] - x1, x1 - qHi[0]), 0.f);
            const float gy = fmaxf(fmaxf(qLo[1] - y1, y1 - qHi[1]), 0.f);
            const float gz = fmaxf(fmaxf(qLo[2] - z1, z1 - qHi[2]), 0.f);
            unsigned long long need = __ballot(fmaf(gz, gz, fmaf(gy, gy, gx * gx)) < qT);
            while (need) {
                const int c = __builtin_amdgcn_readfirstlane(__ffsll((long long)need) - 1);
                need &= need - 1;
                float best = -1.f, sx = 0.f, sy = 0.f, sz = 0.f;
                int bi = 0;
                float4 e[kCS];
#pragma unroll
                for (int u = 0; u < kCS; ++u)
                    e[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                               wsr, lane * 16, 1024 * (kCS * c + u), 0));
#pragma unroll
                for (int u = 0; u < kCS; ++u) {
                    const float dx = e[u].x - x1, dy = e[u].y - y1, dz = e[u].z - z1;
                    const float d2 = fminf(fmaf(dz, dz, fmaf(dy, dy, dx * dx)), e[u].w);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(d2), wsr, lane * 16 + 12,
                                                          1024 * (kCS * c + u), 0);
                    const bool gt = d2 > best;
                    best = gt ? d2 : best;
                    bi = gt ? kCS * c + u : bi;
                    sx = gt ? e[u].x : sx; sy = gt ? e[u].y : sy; sz = gt ? e[u].z : sz;
                }
                float T, X = 0.f, Y = 0.f, Z = 0.f;
                int Dd, P = 0;
                wave_pick(best, bi, sx, sy, sz, NA + w * PB, T, Dd, P, X, Y, Z);
                if (lane == c) { qT = T; qD = Dd; qP = P; qX = X; qY = Y; qZ = Z; }
            }
        }
        // cluster B's candidate: the best chunk cache (ties: smallest rank)
        int bD, bP;
        float bX, bY, bZ;
        {
            const int dq = lane < kNCB ? qD : INT_MIN;
            bD = __builtin_amdgcn_readlane(row_max_i32(dq), 0);
            int lc = 0;
            if (bD >= 0) {
                const unsigned long long cand = __ballot(lane < kNCB && qD == bD);
                if (__popcll(cand) == 1) {
                    lc = __ffsll((long long)cand) - 1;
                } else {
                    const uint32_t r = (lane < kNCB && qD == bD) ? fps_rank(s_perm[qP], L) : 0xffffffffu;
                    const uint32_t rm = __builtin_amdgcn_readlane(row_min_u32(r), 0);
                    lc = __ffsll((long long)(__ballot(r == rm) & cand)) - 1;
                }
            }
            bP = __builtin_amdgcn_readlane(qP, lc);
            bX = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qX), lc));
            bY = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qY), lc));
            bZ = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qZ), lc));
        }
        // the wave's candidate: larger distance, equal distances -> smaller rank
        bool useB = bD > aD;
        if (bD == aD && aD >= 0)
            useB = fps_rank(s_perm[bP], L) < fps_rank(s_perm[aP], L);
        if (lane == 0) {
            s_pub[buf][w] = useB ? make_float4(bX, bY, bZ, __int_as_float(bD))
                                 : make_float4(aX, aY, aZ, __int_as_float(aD));
            s_pos[buf][w] = useB ? bP : aP;
        }
        __syncthreads();
        const float4 v = s_pub[buf][lane & (kWaves - 1)];
        const int vp = s_pos[buf][lane & (kWaves - 1)];
        const int dv = __float_as_int(v.w);
        const int dm = __builtin_amdgcn_readfirstlane(row_max_i32(dv));
        int pj;
        if (dm < 0) {
            pj = 0xffff;
            x1 = x0; y1 = y0; z1 = z0;
        } else {
            const unsigned long long cand = __ballot(dv == dm) & 0xffffull;
            int wsel;
            if (__popcll(cand) == 1) {
                wsel = __ffsll((long long)cand) - 1;
            } else {
                const uint32_t r = dv == dm ? fps_rank(s_perm[vp], L) : 0xffffffffu;
                const uint32_t rm = __builtin_amdgcn_readfirstlane(row_min_u32(r));
                wsel = __ffsll((long long)(__ballot(r == rm) & 0xffffull)) - 1;
            }
            x1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), wsel));
            y1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), wsel));
            z1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.z), wsel));
            pj = __builtin_amdgcn_readlane(vp, wsel);
        }
        if (tid == 0) s_out[j] = (uint16_t)pj;
    }
    __syncthreads();
    for (int j = tid; j < M; j += kThreads) {
        int k = 0;
        if (j > 0 && s_out[j] != 0xffff) k = s_perm[s_out[j]];
        idx[j] = k;
        if (new_xyz) {
            new_xyz[3 * j] = p[3 * k];
            new_xyz[3 * j + 1] = p[3 * k + 1];
            new_xyz[3 * j + 2] = p[3 * k + 2];
        }
    }
}

// ---------------------------------------------------------------------------
// Two workgroups (two CUs) per scene for kThreads*kMaxPPT < N <= 2*kThreads*kMaxPPT (ScanNet:
// 40000 points).  Both workgroups sort the whole scene by Morton cell (as fps_cull_kernel) and
// each keeps one half of the sorted order -- a compact spatial half -- in VGPRs (<= 20 slots
// per lane, the 20000-point register kernel's layout).  Per iteration each workgroup runs the
// culled update and its block argmax, then the halves swap their candidates through L2:
// five 64-bit words per (scene, half, iteration parity), each carrying the iteration number
// as a tag (no fences: a word is valid when its tag matches), written by one lane, polled by
// one lane per wave.  The winner is (larger distance, then smaller upstream rank), the same
// rule inside and across the halves, so the indices equal the one-workgroup kernels'.
// Scene b runs on workgroups b and b + B: with B a multiple of 8, the same XCD (one L2) under
// the dispatcher's round robin -- for speed only: the halves first swap their XCC_ID through
// memory (sc1 granules, correct at any placement).  Same XCD: candidates are stored plain (the
// line stays in that XCD's L2) and polled with sc1 loads (L2-served, bypassing L1): one L2 round
// trip per iteration.  Different XCDs: sc1 stores too (the line goes to memory), the guide's
// tagged-granule hand-off.  A slot is four 8-byte {value, tag} granules (distance, x, y, z; tag =
// iteration << 16 | point index) moved by two 16-byte accesses; each granule is read untorn and
// checked against its tag, so no fences are needed.
// The exchange slots are zeroed by the host before each launch (tag 0 is never used).
// polls before giving up on the partner.  A partner that never answers (it was not co-resident:
// the host only picks this kernel when 2B workgroups fit the device, fps_pair_fits) would
// otherwise hang the launch; after the limit the half carries on alone, records `lost` in its
// hand-shake line, and fps_pair_lost_kernel (launched right after) poisons the scene's sampled
// coordinates with NaN and reports it through ov3d_fps_pair_status: a wrong sample never
// passes silently.  OV3D_FPS_PAIR_SPIN overrides the limit (tests force the path with a small
// limit and OV3D_FPS_PAIR_SILENT=1, which makes half 1 return at once).
constexpr int kPairSpin = 1 << 26;

__device__ __forceinline__ unsigned long long xword(uint32_t v, uint32_t tag) {
    return ((unsigned long long)tag << 32) | v;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-byte sc1 load (bypasses this CU's L1; served by the XCD's L2 when the line is there)
__device__ __forceinline__ u32x4 load_sc1_x4(const void* p) {
    u32x4 r;
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    return r;
}
// two 16-byte sc1 loads, both in flight before the wait
struct u32x4x2 { u32x4 a, b; };
__device__ __forceinline__ u32x4x2 load_sc1_x4x2(const void* p) {
    u32x4x2 r;
    asm volatile("global_load_dwordx4 %0, %2, off sc1\n\tglobal_load_dwordx4 %1, %2, off offset:16 sc1\n\t"
                 "s_waitcnt vmcnt(0)" : "=&v"(r.a), "=&v"(r.b) : "v"(p) : "memory");
    return r;
}
// 16-byte store: plain (the line stays in this XCD's L2) or sc1 (written through to memory).
// s_nop 1: a VALU write of the data VGPRs right after a VMEM store of more than 8 bytes needs
// a wait state, and the compiler's hazard pass does not look inside inline asm
__device__ __forceinline__ void store_x4(void* p, u32x4 v, bool through) {
    if (through)
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else
        asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
}

template <int PPT>
__global__ __launch_bounds__(kThreads) void fps_pair_kernel(const float* __restrict__ xyz, int B,
                                                            int N, int M, int L,
                                                            unsigned long long* __restrict__ xch,
                                                            int32_t* __restrict__ idx,
                                                            float* __restrict__ new_xyz,
                                                            int force_mem, int spin_limit,
                                                            int silent_half1) {
    constexpr int PW = PPT * 64;
    constexpr int NSORT = 2 * PPT;   // setup slots per thread (the whole scene)
    __shared__ uint32_t s_hist[kCells];
    __shared__ __attribute__((aligned(16))) uint16_t s_perm[kThreads * NSORT];
    __shared__ uint16_t s_out[kMaxOutLDS];     // winning point index per iteration
    __shared__ float s_red[6][kWaves];
    __shared__ uint32_t s_scan[kWaves];
    __shared__ float4 s_pub[2][kWaves];
    __shared__ int s_pos[2][kWaves];

    const int b = blockIdx.x % B;
    const int half = blockIdx.x / B;
    if (silent_half1 && half) return;   // test hook: a partner that never answers
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const float* __restrict__ p = xyz + (size_t)b * N * 3;
    const int NH = (N + 1) / 2;
    const int base = half * NH;                 // this half's sorted positions [base, end)
    const int end = half ? N : NH;
    // exchange words: [b][half][parity][8] (4 granules: distance, x, y, z, each tagged with
    // (iteration << 16) | point index);
    // XCC_ID hand-shake words after them: [b][half][16] (one 128-byte line each)
    unsigned long long* const mine = xch + ((size_t)b * 2 + half) * 16;
    const unsigned long long* const other = xch + ((size_t)b * 2 + (half ^ 1)) * 16;
    unsigned long long* const hs_mine = xch + (size_t)B * 32 + ((size_t)b * 2 + half) * 16;
    const unsigned long long* const hs_other = xch + (size_t)B * 32 + ((size_t)b * 2 + (half ^ 1)) * 16;
    __shared__ int s_through;
    if (tid == 0) {
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        xcc &= 0xfu;
        const u32x4 hv = {xcc, 1u, 0u, 1u};
        store_x4(hs_mine, hv, true);
        int through = 1;   // partner silent (spin limit): the memory path
        for (int spin = 0; spin < spin_limit; ++spin) {
            const u32x4 o = load_sc1_x4(hs_other);
            if (o[1] == 1u) { through = o[0] != xcc || force_mem; break; }
        }
        s_through = through;
        // the decision, for diagnostics (tools/fps_pair_stress.py reads it after the launch)
        store_x4(hs_mine + 2, (u32x4){(uint32_t)through, 2u, 0u, 2u}, true);
    }

    // ---- the scene's Morton order.  Both halves must own complementary point sets, and the
    //      counting sort's order inside a cell follows the LDS atomics' order, which differs
    //      between two workgroups (a point of the boundary cell could land in both halves or in
    //      neither): half 0 sorts and publishes the order (sc1 16-byte stores, drained, then a
    //      flag), half 1 polls the flag and reads it (sc1 loads).  Half 1 sorts by itself only
    //      if half 0 never answers (spin limit).
    const int NP = (N + 7) & ~7;
    uint16_t* const perm_g = reinterpret_cast<uint16_t*>(xch + (size_t)B * 64) + (size_t)b * NP;
    unsigned long long* const pflag = xch + (size_t)B * 32 + (size_t)b * 2 * 16 + 6;   // half 0's line
    __shared__ int s_have;
    if (tid == 0) {
        int have = 0;
        if (half)
            for (int spin = 0; spin < spin_limit; ++spin)
                if (load_sc1_x4(pflag)[0] == 1u) { have = 1; break; }
        s_have = have;
    }
    __syncthreads();
    if (s_have) {
        for (int c = tid; c < NP / 8; c += kThreads)
            *reinterpret_cast<u32x4*>(&s_perm[8 * c]) = load_sc1_x4(perm_g + 8 * c);
    } else {
        // ---- (a) scene bbox, (b) Morton counting sort of all N points (as fps_cull_kernel)
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int k = tid; k < N; k += kThreads)
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const float v = p[3 * k + a];
                lo[a] = fminf(lo[a], v);
                hi[a] = fmaxf(hi[a], v);
            }
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = wave_fmin(lo[a]);
            hi[a] = wave_fmax(hi[a]);
        }
        if (lane == 0)
#pragma unroll
            for (int a = 0; a < 3; ++a) { s_red[a][w] = lo[a]; s_red[3 + a][w] = hi[a]; }
        for (int i = tid; i < kCells; i += kThreads) s_hist[i] = 0;
        __syncthreads();
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float l = s_red[a][0], h = s_red[3 + a][0];
            for (int q = 1; q < kWaves; ++q) { l = fminf(l, s_red[a][q]); h = fmaxf(h, s_red[3 + a][q]); }
            lo[a] = l;
            hi[a] = 16.f / fmaxf(h - l, 1e-6f);
        }
        {
            uint32_t cp[NSORT];
#pragma unroll
            for (int i = 0; i < NSORT; ++i) {
                const int k = tid + i * kThreads;
                cp[i] = 0xffffffffu;
                if (k < N) {
                    uint32_t q[3];
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        const int c = (int)((p[3 * k + a] - lo[a]) * hi[a]);
                        q[a] = (uint32_t)min(max(c, 0), 15);
                    }
                    const uint32_t code = spread3(q[0]) | (spread3(q[1]) << 1) | (spread3(q[2]) << 2);
                    const uint32_t old = atomicAdd(&s_hist[code], 1u);
                    cp[i] = (code << 16) | old;
                }
            }
            __syncthreads();
            {
                uint32_t v[4], sum = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) { v[q] = s_hist[4 * tid + q]; sum += v[q]; }
                uint32_t inc = sum;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t o = __shfl_up(inc, off);
                    if (lane >= off) inc += o;
                }
                if (lane == 63) s_scan[w] = inc;
                __syncthreads();
                uint32_t basew = 0;
                for (int q = 0; q < w; ++q) basew += s_scan[q];
                uint32_t run = basew + inc - sum;
#pragma unroll
                for (int q = 0; q < 4; ++q) { s_hist[4 * tid + q] = run; run += v[q]; }
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NSORT; ++i)
                if (cp[i] != 0xffffffffu)
                    s_perm[s_hist[cp[i] >> 16] + (cp[i] & 0xffffu)] = (uint16_t)(tid + i * kThreads);
        }
    }
    __syncthreads();
    if (half == 0) {
        for (int c = tid; c < NP / 8; c += kThreads)
            store_x4(perm_g + 8 * c, *reinterpret_cast<const u32x4*>(&s_perm[8 * c]), true);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) store_x4(pflag, (u32x4){1u, 1u, 1u, 1u}, true);
    }

    // ---- (c) this thread's slots: positions base + w*PW + i*64 + lane (< end), by rank
    uint32_t rk[PPT];
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const int pos = base + w * PW + i * 64 + lane;
        rk[i] = pos < end ? fps_rank(s_perm[pos], L) : 0xffffffffu;
    }
#pragma unroll
    for (int pass = 0; pass < PPT; ++pass)
#pragma unroll
        for (int i = pass & 1; i + 1 < PPT; i += 2) {
            const uint32_t a = rk[i], c = rk[i + 1];
            rk[i] = min(a, c);
            rk[i + 1] = max(a, c);
        }
    __syncthreads();   // every thread has read s_perm of its positions before the rewrite
    float px[PPT], py[PPT], pz[PPT], td[PPT];
    float wlo[3] = {INFINITY, INFINITY, INFINITY}, whi[3] = {-INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const int pos = base + w * PW + i * 64 + lane;
        if (rk[i] != 0xffffffffu) {
            const int k = fps_unrank(rk[i], L);
            s_perm[pos] = (uint16_t)k;
            const float x = p[3 * k], y = p[3 * k + 1], z = p[3 * k + 2];
            const float mag = fmaf(z, z, fmaf(y, y, x * x));
            px[i] = x; py[i] = y; pz[i] = z;
            const bool skip = (double)mag <= 1e-3;
            td[i] = skip ? -1.f : 1e10f;
            if (!skip) {
                wlo[0] = fminf(wlo[0], x); wlo[1] = fminf(wlo[1], y); wlo[2] = fminf(wlo[2], z);
                whi[0] = fmaxf(whi[0], x); whi[1] = fmaxf(whi[1], y); whi[2] = fmaxf(whi[2], z);
            }
        } else {
            px[i] = 0.f; py[i] = 0.f; pz[i] = 0.f; td[i] = -1.f;
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        wlo[a] = wave_fmin(wlo[a]);
        whi[a] = wave_fmax(whi[a]);
    }
    __syncthreads();   // s_perm (this half's positions) complete before any tie lookup
    const float x0 = p[0], y0 = p[1], z0 = p[2];
    float x1 = x0, y1 = y0, z1 = z0;
    float wtmax = INFINITY;
    int wdist = __float_as_int(-1.f);
    int wpos = 0;
    float wx = 0.f, wy = 0.f, wz = 0.f;
    bool lost = false;   // the partner never answered (spin limit): stop exchanging
    const bool through = s_through != 0;   // written by tid 0 before the barriers above

    for (int j = 1; j < M; ++j) {
        const int buf = j & 1;
        const float gx = fmaxf(fmaxf(wlo[0] - x1, x1 - whi[0]), 0.f);
        const float gy = fmaxf(fmaxf(wlo[1] - y1, y1 - whi[1]), 0.f);
        const float gz = fmaxf(fmaxf(wlo[2] - z1, z1 - whi[2]), 0.f);
        const float lb = fmaf(gz, gz, fmaf(gy, gy, gx * gx));
        if (lb < wtmax) {  // wave-uniform
            float best = -1.f;
            int bi = 0;
            float sx = 0.f, sy = 0.f, sz = 0.f;
#pragma unroll
            for (int i = 0; i < PPT; ++i) {
                const float dx = px[i] - x1, dy = py[i] - y1, dz = pz[i] - z1;
                const float d = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                const float d2 = fminf(d, td[i]);
                td[i] = d2;
                const bool gt = d2 > best;
                best = gt ? d2 : best;
                bi = gt ? i : bi;
                sx = gt ? px[i] : sx; sy = gt ? py[i] : sy; sz = gt ? pz[i] : sz;
            }
            const int bb = __float_as_int(best);
            const int wm = wave_max_i32(bb);
            wdist = wm;
            wtmax = __int_as_float(wm);
            if (wm >= 0) {
                const unsigned long long cand = __ballot(bb == wm);
                int wl;
                if (__popcll(cand) == 1) {
                    wl = __ffsll((long long)cand) - 1;
                } else {
                    uint32_t my = 0xffffffffu;
                    if (bb == wm) my = fps_rank(s_perm[base + w * PW + bi * 64 + lane], L);
                    const uint32_t mr = wave_min_u32(my);
                    wl = __ffsll((long long)__ballot(my == mr)) - 1;
                }
                wx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sx), wl));
                wy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sy), wl));
                wz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sz), wl));
                wpos = base + w * PW + __builtin_amdgcn_readlane(bi, wl) * 64 + wl;
            }
        }
        if (lane == 0) {
            s_pub[buf][w] = make_float4(wx, wy, wz, __int_as_float(wdist));
            s_pos[buf][w] = wpos;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // this half's winner (every wave reduces the 16 wave slots)
        const float4 v = s_pub[buf][lane & (kWaves - 1)];
        const int vp = s_pos[buf][lane & (kWaves - 1)];
        const int dv = __float_as_int(v.w);
        const int dm = __builtin_amdgcn_readfirstlane(row_max_i32(dv));
        int hk = 0xffff;   // this half's winning point index (none: 0xffff)
        float hx = x0, hy = y0, hz = z0;
        uint32_t hr = 0xffffffffu;
        if (dm >= 0) {
            const unsigned long long cand = __ballot(dv == dm) & 0xffffull;
            int ws;
            if (__popcll(cand) == 1) {
                ws = __ffsll((long long)cand) - 1;
            } else {
                const uint32_t r = dv == dm ? fps_rank(s_perm[vp], L) : 0xffffffffu;
                const uint32_t rm = __builtin_amdgcn_readfirstlane(row_min_u32(r));
                ws = __ffsll((long long)(__ballot(r == rm) & 0xffffull)) - 1;
            }
            hx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.x), ws));
            hy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.y), ws));
            hz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v.z), ws));
            hk = s_perm[__builtin_amdgcn_readlane(vp, ws)];
            hr = fps_rank((uint32_t)hk, L);
        }
        // ---- swap candidates with the other half through L2: 5 tagged 64-bit words
        //      (distance bits, point index, x, y, z) per (scene, half, iteration parity)
        const uint32_t tag = (uint32_t)j;
        // granule tags: (iteration << 16) | point index
        const uint32_t tk = (tag << 16) | (uint32_t)hk;
        if (tid == 0) {
            unsigned long long* const slot = mine + 8 * buf;
            store_x4(slot, (u32x4){(uint32_t)dm, tk, __float_as_uint(hx), tk}, through);
            store_x4(slot + 2, (u32x4){__float_as_uint(hy), tk, __float_as_uint(hz), tk}, through);
        }
        uint32_t ov[5] = {0u, 0u, 0u, 0u, 0u};
        uint32_t ot = 0u;
        if (lane == 0 && !lost) {
            const unsigned long long* const os = other + 8 * buf;
            for (int spin = 0; spin < spin_limit; ++spin) {
                const u32x4x2 g = load_sc1_x4x2(os);
                const uint32_t t0 = g.a[1];
                ov[0] = g.a[0]; ov[1] = t0 & 0xffffu; ov[2] = g.a[2]; ov[3] = g.b[0]; ov[4] = g.b[2];
                if ((t0 >> 16) == tag && g.a[3] == t0 && g.b[1] == t0 && g.b[3] == t0) {
                    ot = tag;
                    break;
                }
            }
        }
        // lane 0's words to the whole wave (scalar registers)
        lost = lost || (uint32_t)__builtin_amdgcn_readfirstlane((int)ot) != tag;
        const int odm = __builtin_amdgcn_readfirstlane((int)ov[0]);
        const int ok = __builtin_amdgcn_readfirstlane((int)ov[1]);
        const float ox = __int_as_float(__builtin_amdgcn_readfirstlane((int)ov[2]));
        const float oy = __int_as_float(__builtin_amdgcn_readfirstlane((int)ov[3]));
        const float oz = __int_as_float(__builtin_amdgcn_readfirstlane((int)ov[4]));
        // the scene's winner: larger distance, equal distances -> smaller upstream rank
        bool useO = !lost && odm > dm;
        if (!lost && odm == dm && dm >= 0) useO = fps_rank((uint32_t)ok, L) < hr;
        int pk;
        if (useO) {
            pk = ok;
            x1 = ox; y1 = oy; z1 = oz;
        } else if (dm >= 0) {
            pk = hk;
            x1 = hx; y1 = hy; z1 = hz;
        } else {   // no candidate anywhere: upstream keeps thread 0's besti = 0
            pk = 0xffff;
            x1 = x0; y1 = y0; z1 = z0;
        }
        if (tid == 0) s_out[j] = (uint16_t)pk;
    }
    __syncthreads();
    // the outcome, read by fps_pair_lost_kernel (poison + status) and the stress tool
    if (tid == 0) store_x4(hs_mine + 4, (u32x4){(uint32_t)lost, 3u, 0u, 3u}, true);
    if (half) return;
    idx += (size_t)b * M;
    if (new_xyz) new_xyz += (size_t)b * M * 3;
    for (int j = tid; j < M; j += kThreads) {
        int k = 0;
        if (j > 0 && s_out[j] != 0xffff) k = s_out[j];
        idx[j] = k;
        if (new_xyz) {
            new_xyz[3 * j] = p[3 * k];
            new_xyz[3 * j + 1] = p[3 * k + 1];
            new_xyz[3 * j + 2] = p[3 * k + 2];
        }
    }
}

// one thread per scene, after fps_pair_kernel: a scene whose halves did not complete every
// exchange (either half's `lost`, or a half that never reported: a zero tag) gets NaN sampled
// coordinates (the forward's loss turns NaN, also inside a captured graph) and status 1
__global__ void fps_pair_lost_kernel(const unsigned long long* __restrict__ xch, int B, int M,
                                     float* __restrict__ new_xyz, int32_t* __restrict__ status) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    int bad = 0;
    for (int half = 0; half < 2; ++half) {
        const u32x4 o = load_sc1_x4(xch + (size_t)B * 32 + ((size_t)b * 2 + half) * 16 + 4);
        bad |= o[1] != 3u || o[0] != 0u;
    }
    if (status) status[b] = bad;
    if (bad && new_xyz)
        for (int j = 0; j < 3 * M; ++j) new_xyz[(size_t)b * M * 3 + j] = __int_as_float(0x7fc00000);
}

// 2B workgroups of the pair kernel must be resident at once (each half spins on its partner):
// one 1024-thread workgroup per CU (its LDS), so 2B <= CUs x occupancy
template <int PPT>
bool fps_pair_fits(int B) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return false;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fps_pair_kernel<PPT>, kThreads, 0) !=
        hipSuccess)
        return false;
    return 2LL * B <= (long long)cus * per;
}

int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}

template <int PPT>
int launch_pair(const float* xyz, int B, int N, int M, int L, unsigned long long* xch, int32_t* idx,
                float* nx, int force_mem, hipStream_t s) {
    const int spin = env_int("OV3D_FPS_PAIR_SPIN", kPairSpin);
    const int silent = env_int("OV3D_FPS_PAIR_SILENT", 0);
    hipLaunchKernelGGL(fps_pair_kernel<PPT>, dim3(2 * B), dim3(kThreads), 0, s, xyz, B, N, M, L,
                       xch, idx, nx, force_mem, spin > 0 ? spin : 1, silent);
    hipLaunchKernelGGL(fps_pair_lost_kernel, dim3(ov3d_cdiv(B, 64)), dim3(64), 0, s, xch, B, M, nx,
                       nullptr);
    return OV3D_OK;
}

#ifdef OV3D_FPS_PROBE
unsigned long long* g_probe_dbg = nullptr;
#define OV3D_FPS_PROBE_ARG , g_probe_dbg
#else
#define OV3D_FPS_PROBE_ARG
#endif

// the two-workgroup kernel for 20480 < N <= 40960 (OV3D_FPS_PAIR=0: the one-workgroup
// two-cluster kernel instead)
bool fps_pair_enabled() {
    const char* e = getenv("OV3D_FPS_PAIR");
    return !(e && e[0] == '0');
}

template <int PPT>
void launch_cull(const float* xyz, int B, int N, int M, int L, int32_t* idx, float* nx,
                 hipStream_t s) {
    hipLaunchKernelGGL(fps_cull_kernel<PPT>, dim3(B), dim3(kThreads), 0, s, xyz, N, M, L, idx, nx
                       OV3D_FPS_PROBE_ARG);
}

int pair_ppt(int N) { return ((N + 1) / 2 + kThreads - 1) / kThreads; }

// the pair kernel's range (20480 < N <= 40960) at a B whose 2B workgroups are co-resident
bool fps_pair_path(int B, int N) {
    if (N <= kThreads * kMaxPPT || N > 2 * kThreads * kMaxPPT) return false;
    const int p = pair_ppt(N);
    return p <= 12 ? fps_pair_fits<12>(B) : p <= 16 ? fps_pair_fits<16>(B) : fps_pair_fits<20>(B);
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
    if (ppt <= kMaxPPT && M <= kMaxOutLDS) {
        if (ppt <= 1) launch_cull<1>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 2) launch_cull<2>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 4) launch_cull<4>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 8) launch_cull<8>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 12) launch_cull<12>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else if (ppt <= 16) launch_cull<16>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
        else launch_cull<20>(xyz, B, N, M, L, idx_out, new_xyz_out, s);
    } else if (N <= 2 * kThreads * kMaxPPT && M <= kMaxOutLDS && fps_pair_enabled() &&
               fps_pair_path(B, N)) {
        // two workgroups per scene, candidates swapped through L2 (fps_pair_kernel)
        if (!workspace) return OV3D_EINVAL;
        const size_t xbytes = (size_t)B * 2 * 2 * 16 * sizeof(unsigned long long);   // slots + XCC_IDs
        if (hipMemsetAsync(workspace, 0, xbytes, s) != hipSuccess) return OV3D_ELAUNCH;
        unsigned long long* xch = reinterpret_cast<unsigned long long*>(workspace);
        // OV3D_FPS_XCH=mem: candidates through memory even for halves on one XCD (diagnostic)
        static const int force_mem = [] {
            const char* e = getenv("OV3D_FPS_XCH");
            return e && e[0] == 'm' ? 1 : 0;
        }();
        const int ppt2 = pair_ppt(N);
        if (ppt2 <= 12)
            launch_pair<12>(xyz, B, N, M, L, xch, idx_out, new_xyz_out, force_mem, s);
        else if (ppt2 <= 16)
            launch_pair<16>(xyz, B, N, M, L, xch, idx_out, new_xyz_out, force_mem, s);
        else
            launch_pair<20>(xyz, B, N, M, L, xch, idx_out, new_xyz_out, force_mem, s);
    } else if (N <= kThreads * (kPR + kPS) && M <= kMaxOutLDS) {
        if (!workspace) return OV3D_EINVAL;
        // chunk size of the workspace cluster's culling (OV3D_FPS_CHUNK: measurement knob)
        static const int cs = [] {
            const char* e = getenv("OV3D_FPS_CHUNK");
            return e ? atoi(e) : 4;
        }();
        float4* ws4 = reinterpret_cast<float4*>(workspace);
        if (cs == 2)
            hipLaunchKernelGGL(fps_stream_kernel<2>, dim3(B), dim3(kThreads), 0, s, xyz, N, M, L, ws4,
                               idx_out, new_xyz_out);
        else if (cs == 3)
            hipLaunchKernelGGL(fps_stream_kernel<3>, dim3(B), dim3(kThreads), 0, s, xyz, N, M, L, ws4,
                               idx_out, new_xyz_out);
        else
            hipLaunchKernelGGL(fps_stream_kernel<4>, dim3(B), dim3(kThreads), 0, s, xyz, N, M, L, ws4,
                               idx_out, new_xyz_out);
    } else {
        if (!workspace) return OV3D_EINVAL;
        hipLaunchKernelGGL(fps_global_kernel, dim3(B), dim3(kThreads), 0, s, xyz, N, M, L, workspace,
                           idx_out, new_xyz_out);
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

#ifdef OV3D_FPS_PROBE
// diagnostic entry (probe build only): dbg = B*16*12 u64 phase counters
extern "C" void ov3d_fps_probe_set(unsigned long long* dbg) { g_probe_dbg = dbg; }
#endif

/* per-scene outcome of the last ov3d_fps launch on this workspace: status[b] = 1 when the
 * two-workgroup kernel's halves lost each other (the scene's new_xyz_out was set to NaN), 0
 * otherwise (and 0 for every scene when (B, N) did not take the two-workgroup path) */
extern "C" int ov3d_fps_pair_status(const float* workspace, int B, int N, int M, int32_t* status,
                                    void* stream) {
    if (B < 0 || N <= 0 || M < 0 || !status) return OV3D_EINVAL;
    if (B == 0) return OV3D_OK;
    hipStream_t s = ov3d_stream(stream);
    if (M == 0 || M > kMaxOutLDS || !fps_pair_enabled() || !fps_pair_path(B, N)) {
        if (hipMemsetAsync(status, 0, (size_t)B * sizeof(int32_t), s) != hipSuccess)
            return OV3D_ELAUNCH;
        return OV3D_OK;
    }
    if (!workspace) return OV3D_EINVAL;
    hipLaunchKernelGGL(fps_pair_lost_kernel, dim3(ov3d_cdiv(B, 64)), dim3(64), 0, s,
                       reinterpret_cast<const unsigned long long*>(workspace), B, M, nullptr, status);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

/* workspace floats ov3d_fps needs for (B, N) (16-byte aligned) */
extern "C" long long ov3d_fps_workspace(int B, int N) {
    if (B <= 0 || N <= kThreads * kMaxPPT) return 0;
    // (both kernels of 20480 < N <= 40960 may run: the pair kernel's exchange slots fit
    // inside the two-cluster kernel's workspace)
    if (N <= kThreads * (kPR + kPS)) return (long long)B * kWaves * kPS * 64 * 4;
    return (long long)B * N;
}

extern "C" const char* ov3d_version(void) { return "ov3d-hip 0.1 gfx950"; }
