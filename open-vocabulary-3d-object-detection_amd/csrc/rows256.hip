// Streaming product Y (M, 256) = X (M, K) . W (256, K)^T, K = 256 or 264, for very long row sets: the
// masked encoder's interim set abstraction in ScanNet training (models/model_3detr.py:377-399
// build_preencoder / interim downsampling, PointnetSAModuleVotes' SharedMLP 1x1 convolutions
// over npoint * nsample = 2^18 grouped rows, mlp widths 256 -> 256 -> 256) forward, and the
// input gradients of the same layers (dy W, W transposed on the host).
//
// gemm256 (csrc/gemm256.hip) runs these at ~105 us (forward) / ~72 us (input gradient) for
// 34 GFLOP and 256 MB of traffic, ~3x the HBM floor: its 256 x 256 tiles reload W for every
// tile and a tile's load, compute and store phases do not overlap at K = 256 (four K-steps).
// Here:
//   * one persistent workgroup a CU, 512 threads = 8 waves; wave w owns output columns
//     32 w .. 32 w + 31 and holds its W rows (all K) in registers for the whole launch
//     (16 fragments = 64 VGPRs), so W is read once per CU;
//   * X streams through LDS in 128-row tiles (64 KB), double buffered by LDS-DMA
//     (buffer_load ... lds, 16 bytes a lane): tile t + 1 lands while tile t is multiplied;
//     the 16-byte chunks of a 512-byte row are XOR-swizzled by row & 15 through the per-lane
//     source offset, so every 16-lane group of a fragment read (ds_read_b128) covers the 64
//     banks once (tools/lds_banks_dy9.py rows256_census);
//   * the product is gemm256's arithmetic: v_mfma_f32_16x16x32_bf16 with the W fragment as
//     the first operand, one fp32 chain per output from k = 0 upward in 32-deep steps, one
//     rounding to bf16 -> the outputs equal gemm256's bit for bit (no bias / residual / ReLU);
//   * the bf16 tile goes back through the LDS buffer it was read from and leaves as whole
//     16-byte chunks, 1 KB (two rows) a wave instruction;
//   * tiles are claimed from a counter, so a late workgroup (a side-stream kernel holding CUs,
//     e.g. the next step's furthest-point sampling) does not add a tail round of its own.
#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 512;                 // threads
constexpr int TM = 128;                 // rows a tile
constexpr int KD = 256;                 // K = N
constexpr int TILE_BYTES = TM * KD * 2; // 64 KB
constexpr int RB = TM / 16;             // 16-row blocks a tile
constexpr int TAIL_BYTES = TM * 16;     // KT: the K = 256 .. 263 chunk of a tile's rows
constexpr int WX_BYTES = 16 * KD * 2;   // NX: W rows 256 .. 271 (zeros past 263), swizzled

__device__ __forceinline__ f32x4 mfma16(i32x4 a, i32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// ds_read_b128 as asm: the compiler would treat an LDS read as aliasing the in-flight
// LDS-DMA and wait for every load (vmcnt(0)) before it.  Results are consumed only after
// lgkm_wait8 names them.
__device__ __forceinline__ i32x4 lds128(uint32_t addr) {
    i32x4 r;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr) : "memory");
    return r;
}
// ds_write_b64 as asm, for the same reason (a plain LDS store waited for every DMA in flight)
__device__ __forceinline__ void lds_write64(uint32_t addr, bf16x4 v) {
    asm volatile("ds_write_b64 %0, %1" : : "v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ void lgkm_wait8(i32x4 (&a)[RB]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                   "+v"(a[6]), "+v"(a[7])
                 :
                 : "memory");
}

// atomicAdd(ctr, 1) as asm: the compiler would wait for its result (vmcnt(0), i.e. the previous
// tile's stores too) at the join of the lane-0 branch.  Untracked by the compiler's wait counts
// (at most an extra wait); the caller waits before using the result.
__device__ __forceinline__ unsigned int claim_async(unsigned int* ctr) {
    unsigned int r;
    asm volatile("global_atomic_add %0, %1, %2, off sc0"
                 : "=v"(r)
                 : "v"(ctr), "v"(1u)
                 : "memory");
    return r;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const uint32_t n = bytes > 0x7fffffffLL ? 0x7fffffffu : (uint32_t)(bytes > 0 ? bytes : 0);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)n, 0x00020000);
}

struct Rows256Args {
    const bf16* X; long long ldx;
    const bf16* W; long long ldw;
    bf16* Y; long long ldy;
    long long M;
    int tiles;
    unsigned int* ctr;   // [next tile, workgroups done]: zero, and left zero by every launch
    // BNIN: X holds the previous layer's pre-BatchNorm rows; the product's input is
    // Z = bf16(relu(X * scale + shift)) (the ov3d_rows_bn_apply arithmetic), written to Z
    const float* scale; const float* shift;
    bf16* Z; long long ldz;
};

// ds_write_b128 as asm (a plain LDS store would wait for every DMA in flight)
__device__ __forceinline__ void lds_write128(uint32_t addr, i32x4 v) {
    asm volatile("ds_write_b128 %0, %1" : : "v"(addr), "v"(v) : "memory");
}

// KT: K = 264 (the interim SA's first layer: 256 features + xyz, zero-padded): gemm256's tail
// K-step (k 256 .. 319, zeros past 264) as two more 32-deep MFMA steps, the rows' chunk 32 in a
// tail image filled by two more DMA pieces (waves 6 and 7)
// BNIN: 0 none, 1 BN + ReLU on the staged rows and Z stored, 2 the same without Z (its weight
// gradient applies the BN on load: ov3d_wgrad_bn).
// NX: N = 264 (the first layer's input gradient, 259 + 5 zero columns): every wave also
// computes output columns 256 .. 271 (W rows past 263 zero) of its own 16-row block, W's rows
// 256 .. 271 read from an LDS image; the 8 real columns leave through a 2 KB tail image
template <int BNIN, bool KT, bool NX>
__global__ void __launch_bounds__(NT, 1) rows256_kernel(Rows256Args a) {
    __shared__ __attribute__((aligned(16))) char L[2 * TILE_BYTES + (KT ? 2 * TAIL_BYTES : 0) +
                                                   (NX ? WX_BYTES + TAIL_BYTES : 0)];
    __shared__ int s_claim[2];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lg = lane >> 4;

    // tiles are claimed from a counter (two ahead of use): a workgroup that starts late, e.g.
    // behind a kernel on another stream holding CUs, finds the work taken and leaves
    if (tid == 0) {
        s_claim[0] = (int)atomicAdd(a.ctr, 1u);
        s_claim[1] = (int)atomicAdd(a.ctr, 1u);
    }

    // W rows n = 32 w + 16 cb + li, k = 32 ks + 8 lg .. + 8: the first MFMA operand
    i32x4 wf[2][8];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int ks = 0; ks < 8; ++ks)
            wf[cb][ks] = *reinterpret_cast<const i32x4*>(a.W + (size_t)(32 * w + 16 * cb + li) * a.ldw +
                                                         32 * ks + 8 * lg);
    const i32x4 zero4 = {0, 0, 0, 0};
    if constexpr (NX) {   // W rows 256 .. 271 -> the WX image (chunk c of row j at c ^ j)
        const int j = tid >> 5, c = tid & 31;
        const i32x4 v = 256 + j < 264
            ? *reinterpret_cast<const i32x4*>(a.W + (size_t)(256 + j) * a.ldw + 8 * c) : zero4;
        *reinterpret_cast<i32x4*>(L + 2 * TILE_BYTES + j * KD * 2 + 16 * (c ^ j)) = v;
    }
    i32x4 wt[2] = {zero4, zero4};   // KT: k = 256 + 8 lg .. (lg = 0 only; zeros past 264)
    if constexpr (KT) {
        if (lg == 0)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
                wt[cb] = *reinterpret_cast<const i32x4*>(a.W + (size_t)(32 * w + 16 * cb + li) * a.ldw + 256);
    }

    // LDS-DMA of a tile: wave w fills rows 16 w + 2 i + (lane >> 5) (i = 0..7), physical chunk
    // lane & 31 <- logical chunk (lane & 31) ^ (row & 15)
    const int prow = 16 * w + (lane >> 5);                    // row for i = 0 (+ 2 i)
    uint32_t voff[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int r = prow + 2 * i;
        voff[i] = (uint32_t)(r * a.ldx * 2) + 16u * ((lane & 31) ^ (r & 15));
    }
    auto issue = [&](int t, int buf) {
        const long long m0 = (long long)t * TM;
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(a.X + m0 * a.ldx, (a.M - m0) * a.ldx * 2);
        char* base = L + buf * TILE_BYTES + (16 * w) * (KD * 2);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void*)(base + i * 2 * KD * 2), 16, voff[i], 0, 0, 0);
        if constexpr (KT) {
            if (w >= 6) {   // rows 64 (w - 6) + lane, chunk 32, lane-linear into the tail image
                const int r = 64 * (w - 6) + lane;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(L + 2 * TILE_BYTES + buf * TAIL_BYTES +
                                                                   64 * (w - 6) * 16),
                    16, (uint32_t)(r * a.ldx * 2) + 512u, 0, 0, 0);
            }
        }
    };

    // fragment reads: row 16 rb + li, logical chunk 4 ks + lg at physical (4 ks + lg) ^ li
    const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)L;
    const uint32_t rowoff = (uint32_t)(li * KD * 2);

    // BNIN: this thread's 8 channels 8 (tid & 31) .. + 7 are the same in every tile
    float bsc[BNIN ? 8 : 1], bsh[BNIN ? 8 : 1];
    if constexpr (BNIN) {
        const int c8 = 8 * (tid & 31);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            bsc[j] = a.scale[c8 + j];
            bsh[j] = a.shift[c8 + j];
        }
    }
    // VMEM operations a lane issues per tile after its DMA: the output stores (8), with BNIN
    // also the Z stores (8)
    constexpr int SPT = BNIN == 1 ? 16 : 8;

    __syncthreads();   // the first claims (nothing in flight yet but the W loads)
    int t = s_claim[0], tn = s_claim[1];
    if (t < a.tiles) issue(t, 0);
    bool prev_stores = false;
    for (int it = 0; t < a.tiles; ++it) {
        const int buf = it & 1;
        const bool has_next = tn < a.tiles;
        // the claim after tn, issued before the next tile's DMA (its result is waited for
        // without draining that DMA) and published at the end of this iteration
        unsigned int claim = 0;
        if (tid == 0 && has_next) claim = claim_async(a.ctr);
        if (has_next) issue(tn, buf ^ 1);
        // this tile's DMA landed: later VMEM ops (the previous tile's 8 stores, the claim, the
        // next tile's 8 DMA pieces) may stay in flight
        if (has_next && prev_stores) asm volatile("s_waitcnt vmcnt(%0)" : : "n"(SPT + 8) : "memory");
        else if (prev_stores) asm volatile("s_waitcnt vmcnt(%0)" : : "n"(SPT) : "memory");
        else if (has_next) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if constexpr (BNIN) {
            // the tile in place: z = bf16(relu(x * scale + shift)), also stored to Z (the
            // weight gradient's input); thread = 8 rows of one 8-channel chunk
            const uint32_t tbuf = lds0 + buf * TILE_BYTES;
            const long long zm0 = (long long)t * TM;
            const int c = tid & 31;
            i32x4 rv[RB];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int r = (tid >> 5) + 16 * i;
                rv[i] = lds128(tbuf + r * KD * 2 + 16 * (c ^ (r & 15)));
            }
            lgkm_wait8(rv);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int r = (tid >> 5) + 16 * i;
                const bf16x8 v = __builtin_bit_cast(bf16x8, rv[i]);
                bf16x8 o;
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = (bf16)fmaxf(fmaf((float)v[j], bsc[j], bsh[j]), 0.f);
                const i32x4 ov = __builtin_bit_cast(i32x4, o);
                lds_write128(tbuf + r * KD * 2 + 16 * (c ^ (r & 15)), ov);
                if constexpr (BNIN == 1)
                    if (zm0 + r < a.M) *reinterpret_cast<i32x4*>(a.Z + (zm0 + r) * a.ldz + 8 * c) = ov;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }

        f32x4 acc[RB][2];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
        const uint32_t tb = lds0 + buf * TILE_BYTES + rowoff;
        f32x4 accx = {0.f, 0.f, 0.f, 0.f};   // NX: columns 256 .. 271 of rows 16 w + li
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            i32x4 xf[RB];
            const uint32_t co = 16u * ((4 * ks + lg) ^ li);
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) xf[rb] = lds128(tb + rb * 16 * KD * 2 + co);
            lgkm_wait8(xf);
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                for (int cb = 0; cb < 2; ++cb) acc[rb][cb] = mfma16(wf[cb][ks], xf[rb], acc[rb][cb]);
            if constexpr (NX) {
                i32x4 xe[2];
                xe[0] = lds128(tb + w * 16 * KD * 2 + co);                       // rows 16 w + li
                xe[1] = lds128(lds0 + 2 * TILE_BYTES + li * KD * 2 + co);        // W row 256 + li
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xe[0]), "+v"(xe[1]) : : "memory");
                accx = mfma16(xe[1], xe[0], accx);
            }
        }
        if constexpr (KT) {
            // k 256 .. 287: chunk 32 from the tail image (lg = 0), zeros (lg > 0); then k 288 ..
            // 319, all zeros: gemm256's K-tail step, both halves
            i32x4 xf[RB];
            const uint32_t tt = lds0 + 2 * TILE_BYTES + buf * TAIL_BYTES + li * 16;
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) xf[rb] = lds128(tt + rb * 16 * 16);
            lgkm_wait8(xf);
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
                const i32x4 x = lg == 0 ? xf[rb] : zero4;
#pragma unroll
                for (int cb = 0; cb < 2; ++cb) acc[rb][cb] = mfma16(wt[cb], x, acc[rb][cb]);
            }
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                for (int cb = 0; cb < 2; ++cb) acc[rb][cb] = mfma16(zero4, zero4, acc[rb][cb]);
        }
        // the tile's bf16 image into the buffer just read (row-major, chunk c of row r at
        // c ^ (r & 15)), then every thread stores 8 whole 16-byte chunks (2 rows a wave): the
        // 8-byte stores straight from the accumulators ran at 68 vs 54 us (tools/rows256_probe.py)
        const long long m0 = (long long)t * TM;
        __builtin_amdgcn_s_barrier();
        const uint32_t ib = lds0 + buf * TILE_BYTES;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const int r = 16 * rb + li;
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
                bf16x4 o;
#pragma unroll
                for (int v = 0; v < 4; ++v) o[v] = (bf16)acc[rb][cb][v];
                const int c = 4 * w + 2 * cb + (lg >> 1);
                lds_write64(ib + r * KD * 2 + 16 * (c ^ li) + 8 * (lg & 1), o);
            }
        }
        const uint32_t ot = lds0 + 2 * TILE_BYTES + WX_BYTES;   // NX: columns 256 .. 263
        if constexpr (NX) {
            if (lg < 2) {
                bf16x4 o;
#pragma unroll
                for (int v = 0; v < 4; ++v) o[v] = (bf16)accx[v];
                lds_write64(ot + (16 * w + li) * 16 + 8 * lg, o);
            }
        }
        // LDS writes done, then the raw barrier (__syncthreads' fence would also wait for the
        // next tile's DMA)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        i32x4 sv[RB];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int q = tid + NT * i, r = q >> 5, c = q & 31;
            sv[i] = lds128(ib + r * KD * 2 + 16 * (c ^ (r & 15)));
        }
        lgkm_wait8(sv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int q = tid + NT * i, r = q >> 5, c = q & 31;
            if (m0 + r < a.M) *reinterpret_cast<i32x4*>(a.Y + (m0 + r) * a.ldy + 8 * c) = sv[i];
        }
        if constexpr (NX) {   // waves 6, 7 (wave 0's claim wait stays exact): row tid - 384
            if (tid >= 384) {
                const int r = tid - 384;
                i32x4 v[RB];
                v[0] = lds128(ot + r * 16);
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]) : : "memory");
                if (m0 + r < a.M) *reinterpret_cast<i32x4*>(a.Y + (m0 + r) * a.ldy + 256) = v[0];
            }
        }
        prev_stores = true;
        if (tid == 0 && has_next) {
            // the claim returned: younger are the next tile's 8 DMA pieces and this tile's stores
            asm volatile("s_waitcnt vmcnt(%1)" : "+v"(claim) : "n"(SPT + 8) : "memory");
            s_claim[buf] = (int)claim;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // this buffer is free for the DMA two tiles on
        t = tn;
        tn = has_next ? s_claim[buf] : a.tiles;
    }
    // the last workgroup out leaves the counters zero for the next launch (every claim of every
    // workgroup has returned by now)
    if (tid == 0) {
        if (atomicAdd(a.ctr + 1, 1u) == gridDim.x - 1) {
            atomicExch(a.ctr, 0u);
            atomicExch(a.ctr + 1, 0u);
        }
    }
}

int g_cus = 0;

}  // namespace

extern "C" int ov3d_rows256_supported(long long M, int N, int K) {
    return M > 0 && (N == KD || (N == KD + 8 && K == KD)) && (K == KD || K == KD + 8) &&
           (M + TM - 1) / TM < (1LL << 31) && M * KD * 2 < (1LL << 40);
}

namespace {
struct BnIn {
    const float* scale; const float* shift; void* Z; long long ldz;
};
int rows256_launch(const void* X, long long ldx, int K, int N, const void* W, long long ldw, void* Y,
                   long long ldy, long long M, unsigned int* counters, const BnIn* bn, void* stream) {
    if (!ov3d_rows256_supported(M, N, K) || (bn && (K != KD || N != KD)) || !X || !W || !Y ||
        !counters || ldx < K || ldw < K ||
        ldy < N || ldx % 8 || ldw % 8 || ldy % 8 || ((uintptr_t)X | (uintptr_t)W | (uintptr_t)Y) % 16 ||
        (uintptr_t)counters % 8)
        return OV3D_EINVAL;
    // the buffer resource of a tile covers at most 2 GB from its first row
    if ((long long)TM * ldx * 2 >= (1LL << 31)) return OV3D_EINVAL;
    if (!g_cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            g_cus <= 0)
            g_cus = 256;
    }
    Rows256Args a{(const bf16*)X, ldx, (const bf16*)W, ldw, (bf16*)Y, ldy, M, (int)((M + TM - 1) / TM),
                  counters, nullptr, nullptr, nullptr, 0};
    const int grid = a.tiles < g_cus ? a.tiles : g_cus;
    if (bn) {
        if (!bn->scale || !bn->shift || (bn->Z && (bn->ldz < KD || bn->ldz % 8)) ||
            ((uintptr_t)bn->scale | (uintptr_t)bn->shift | (uintptr_t)bn->Z) % 16)
            return OV3D_EINVAL;
        a.scale = bn->scale; a.shift = bn->shift; a.Z = (bf16*)bn->Z; a.ldz = bn->ldz;
        if (bn->Z) rows256_kernel<1, false, false><<<grid, NT, 0, ov3d_stream(stream)>>>(a);
        else rows256_kernel<2, false, false><<<grid, NT, 0, ov3d_stream(stream)>>>(a);
    } else if (N != KD) {
        rows256_kernel<0, false, true><<<grid, NT, 0, ov3d_stream(stream)>>>(a);
    } else if (K == KD) {
        rows256_kernel<0, false, false><<<grid, NT, 0, ov3d_stream(stream)>>>(a);
    } else {
        rows256_kernel<0, true, false><<<grid, NT, 0, ov3d_stream(stream)>>>(a);
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
}  // namespace

extern "C" int ov3d_rows256(const void* X, long long ldx, int K, int N, const void* W, long long ldw,
                            void* Y, long long ldy, long long M, unsigned int* counters,
                            void* stream) {
    return rows256_launch(X, ldx, K, N, W, ldw, Y, ldy, M, counters, nullptr, stream);
}

extern "C" int ov3d_rows256_bn(const void* X, long long ldx, const float* scale, const float* shift,
                               const void* W, long long ldw, void* Y, long long ldy, void* Z,
                               long long ldz, long long M, unsigned int* counters, void* stream) {
    const BnIn bn{scale, shift, Z, ldz};
    return rows256_launch(X, ldx, KD, KD, W, ldw, Y, ldy, M, counters, &bn, stream);
}
