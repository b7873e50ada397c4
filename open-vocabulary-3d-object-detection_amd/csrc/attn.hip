// Flash attention for the 3DETR transformer, head_dim 64,
// bf16 operands, fp32 accumulation, attention-probability dropout, on MFMA 32x32x16.
//
// Replaces nn.MultiheadAttention's core in models/transformer.py:223,271 (encoder
// self-attention, L = 2048) and :307-308,365-372 (decoder self / cross attention,
// 128 queries over 128 / 2048 keys).  Q, K, V are read straight from the
// projection rows: element (l, b, h, d) lives at ptr[(l*B + b)*stride + h*64 + d]
// (the seq-first (L, B, E) layout of the reference, so no head permute copies), and
// O is written in the same row layout for the output projection.
//
// Layout on the matrix cores ("swapped" QK^T): per wave 32 queries; the score tile
// is S^T = K Q^T (32 keys x 32 queries), so each lane owns ONE query and 16 of its
// keys: the softmax statistics are per lane (plus one lane^32 exchange), and
// O^T = V^T P^T keeps the query on the lane as well, so the online-softmax rescale
// is a per-lane scalar.  P^T feeds the PV MFMA straight from the accumulator
// registers (its k order is the MFMA's row order); V^T's operand is read with
// ds_read_b64_tr_b16 from the row-major V tile in LDS.
//
// Dropout: keep(q, k) from a counter-based hash of (seed, site, b*H+h, q, k>>1) (one 32-bit
// hash per key pair, a signed 16-bit half per key).  The forward computes it once and stores
// the DROP bits twice, 16 + 16 MB per encoder layer: query-major words (one per lane and
// 64-key tile, the layout of attn_bwd_dq_kernel's lanes) and, after a 32 x 32 bit transpose
// across the lanes, key-major words (32 queries of one key, the layout of
// attn_bwd_dkdv_kernel's lanes); the backward reads bits instead of re-hashing (the hash was
// half of each kernel's VALU issue).
// Masked encoder (MaskedTransformerEncoder, transformer.py:152-190: mask = cdist(xyz) >= r^2,
// the same for every head): ov3d_attn_mask_pack packs the (B, Lq, Lk) mask into 1-bit words
// in the two drop-word layouts (per batch row instead of per head, 2 + 2 MB per 2048-point
// layer); masked keys get a -inf score before the softmax in every kernel (MASK template).
// Split-K (grid.z) serves the 128-query decoder attention: partial (O, m, l) per
// key split, merged by attn_combine_kernel.
#include <math.h>
#include <type_traits>
#include <stdlib.h>

#include "common.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

constexpr int D = 64;     // head dim
constexpr int KB = 64;    // keys per LDS tile
constexpr int QW = 32;    // queries per wave
constexpr int LDK = 72;   // padded LDS row of the output staging images, bf16 elements (144 B)

// K / V / Q / dO tile images (round 6): unpadded 128-byte rows, 16-byte piece c of row r at
// c ^ isw(r).  One image serves the row reads (ds_read_b128, lanes = rows 32t + r, pieces 2s + h)
// and the transposed reads (ds_read_b64_tr_b16 over 4 rows x 16 columns, v_operand): isw takes
// bits 1-3 of the row so that the 8 same-parity rows of a b128 lane group land on 8 different
// pieces and rows r, r + 2 of a transposed read on opposite 16-bank halves.  Every access is
// conflict-free under the MI355X lane groups (the padded 144-byte rows left the transposed reads
// 2-way: 32 extra LDS cycles per tile and wave; tools/lds_banks_dy9.py attn_census).
__device__ __forceinline__ int isw(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int img(int r, int c) { return r * D + 8 * ((c >> 3) ^ isw(r)) + (c & 7); }

struct AttnArgs {
    const bf16* q;
    const bf16* k;
    const bf16* v;
    long long sq, sk, sv;  // row strides (elements)
    int B, H, Lq, Lk;
    float scale2;          // softmax scale * log2(e)
    uint32_t thresh;       // dropout: drop when the 16-bit hash half < thresh (0 = off)
    float keep_scale;      // 1 / (1 - p)
    const int64_t* seed;   // device counter (advanced once per step by the host code)
    uint32_t site;         // call-site id
    bf16* o;
    long long so;
    float* lse;            // (B*H, Lq), log2 domain: m*scale2 + log2(l)
    float* part_o;         // split-K partials (nsplit, B*H, Lq, 64) unnormalised
    float* part_ml;        // (nsplit, B*H, Lq, 2): m*scale2 (-inf: no attended key), l
    int nsplit, keys_per_split;
    uint32_t* wq;          // drop bits, query-major: [nkt][B*H][Lq][2] (see drop_word)
    uint32_t* wk;          // drop bits, key-major:   [Lq/32][B*H][nkt*64]
    int nkt;               // 64-key tiles = ceil(Lk / 64)
    const uint32_t* mq;    // mask bits (1 = not attended), query-major: [nkt][B][Lq][2]
    const uint32_t* mk;    // mask bits, key-major: [Lq/32][B][nkt*64]
    unsigned long long* stamp;   // in-kernel launch stamps (measurement) or null: ov3d_stamps_arm
};

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// per (seed, site, b*H+h) scalar mix; per query base; per (query, key) hash
__device__ __forceinline__ uint32_t drop_head_mix(const int64_t* seed, uint32_t site, uint32_t bh) {
    const uint64_t s = (uint64_t)*seed;
    return mix32((uint32_t)s ^ mix32((uint32_t)(s >> 32) + site * 0x9E3779B9u) ^ (bh * 0x85EBCA6Bu));
}
__device__ __forceinline__ uint32_t drop_query_base(uint32_t hm, uint32_t q) {
    return mix32(hm ^ (q * 0xC2B2AE35u));
}
// Per-element finaliser of the dropout hash: two 24-bit multiply rounds; every fold is a
// 16-bit word or a top byte (x ^ x >> 16 and p ^ x >> 24 are ONE v_xor_b32_sdwa each), so 6
// vector ops per key pair (round 3's finaliser also folded by 15 bits: 9).  v_mul_u32_u24
// issues at the full VALU rate (the 32-bit v_mul_lo_u32 of mix32 is quarter rate).  Screened
// over 16384 queries x 2048 keys x 4 heads at p = 0.1 / 0.3 (tools/drop_hash_screen.py, "b2":
// drop rate, byte chi2, pair / neighbour / rectangle correlations within noise, as the round-3
// finaliser; without the first top-byte fold ("b1") the byte chi2 reads 483 on 255 dof).
__device__ __forceinline__ uint32_t drop_mix(uint32_t x) {
    x ^= x >> 16;
    x = __umul24(x, 0x7feb35u) ^ (x >> 24);
    x ^= x >> 16;
    x = __umul24(x, 0x846ca7u);
    return x ^ (x >> 16);
}

// one 32-bit hash per (query, key pair k>>1): its low half decides the even key, the
// high half the odd key; keep iff int16(half) >= thresh - 32768 (thresh = round(p * 2^16)),
// i.e. (half ^ 0x8000) >= thresh unsigned
constexpr uint32_t kPairMul = 0x27D4EB2Fu;

// two fp32 -> two bf16 in one dword (one v_cvt_pk_bf16_f32), the even key in the low half
__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

// 0xFFFF in each 16-bit half of the pair hash whose key is DROPPED: a saturating packed
// subtract of the signed threshold leaves the sign of (half - tsig), an arithmetic shift
// spreads it (v_pk_sub_i16 clamp + v_pk_ashrrev_i16)
__device__ __forceinline__ uint32_t drop_halves(uint32_t hsh, s16x2 tsig) {
    const s16x2 d = __builtin_elementwise_sub_sat(__builtin_bit_cast(s16x2, hsh), tsig);
    return __builtin_bit_cast(uint32_t, (s16x2)(d >> (s16x2){15, 15}));
}

// Drop words.  A lane (query q, half h) of a 64-key tile owns the 32 keys
// kb + 32t + 2(m&1) + 8(m>>1) + 4h + e  (t, e in {0,1}, m in 0..7); bit 8t + m of its word is
// the even key (e = 0), bit 16 + 8t + m the odd key.  drop_key(b, h) = that key's offset.
__device__ __forceinline__ int drop_key(int b, int h) {
    const int e = b >> 4, j = b & 15, t = j >> 3, m = j & 7;
    return 32 * t + 2 * (m & 1) + 8 * (m >> 1) + 4 * h + e;
}

// value of lane ^ J within 32 lanes: DPP quad_perm for 1 and 2, ds_swizzle in bit-mask mode
// (offset = xor_mask << 10 | or_mask << 5 | and_mask) above
template <int J>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
    if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
    else if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);
    else return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (J << 10) | 0x1F);
}

// one butterfly stage of a 32 x 32 bit-matrix transpose across lanes r = lane & 31 (rows)
// and bits (columns): swap row-index bit J with column-index bit J
template <int J, uint32_t MLOW>
__device__ __forceinline__ uint32_t transpose_stage(uint32_t a, int r) {
    const uint32_t p = lane_xor<J>(a);
    const bool low = (r & J) == 0;
    // low rows take the partner's bits c - J into columns with bit J set (rotl J), high
    // rows its bits c + J into columns with bit J clear (rotr J)
    const uint32_t rot = __builtin_amdgcn_alignbit(p, p, low ? 32 - J : J);
    const uint32_t keep = low ? MLOW : ~MLOW;
    return (a & keep) | (rot & ~keep);
}

__device__ __forceinline__ uint32_t transpose32(uint32_t a, int r) {
    a = transpose_stage<16, 0x0000FFFFu>(a, r);
    a = transpose_stage<8, 0x00FF00FFu>(a, r);
    a = transpose_stage<4, 0x0F0F0F0Fu>(a, r);
    a = transpose_stage<2, 0x33333333u>(a, r);
    return transpose_stage<1, 0x55555555u>(a, r);
}


__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// the value of lane ^ 32 combined with this lane's: one v_permlane32_swap (swaps the two
// 32-lane halves of its operands) instead of a ds_bpermute round trip
__device__ __forceinline__ float max_halves(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, x),
                                                    __builtin_bit_cast(uint32_t, x), false, false);
    return fmaxf(__builtin_bit_cast(float, (uint32_t)r[0]), __builtin_bit_cast(float, (uint32_t)r[1]));
}

// Operand rows scaled by scale * log2(e) and rounded to bf16 once: the score MFMAs then give
// log2-domain scores and the softmax needs no multiply per element.  The forward and the dQ
// pass prescale the query rows identically (the same P); the dK / dV pass prescales its key rows.
__device__ __forceinline__ bf16x8 prescale8(bf16x8 v, float c) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (bf16)((float)v[j] * c);
    return r;
}

// Row constants by one more MFMA k-step instead of per-element initial values (a 32x32 tile's
// 16 accumulators per lane would take 16 v_mov per tile): k-slots 0 and 1 live in the h = 0
// lanes' elements 0 and 1, every other slot is zero.  One side holds x0, x1, the other 1, 1:
// the product adds x0 + x1 to every element of the row / column.
__device__ __forceinline__ bf16x8 kslots(float x0, float x1, bool on) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (bf16)0.f;
    if (on) {
        r[0] = (bf16)x0;
        r[1] = (bf16)x1;
    }
    return r;
}
// x as bf16 hi + lo (x to ~2^-16 relative); +-inf -> (inf, 0)
__device__ __forceinline__ float bf16_hi(float x) { return (float)(bf16)x; }
__device__ __forceinline__ float bf16_lo(float x) {
    return __builtin_isinf(x) ? 0.f : x - bf16_hi(x);
}

// online-softmax rescale only when a query's running max grows by more than this
// (log2 units): P stays <= 2^8 between rescales (cdna_hip_programming.md T13)
constexpr float RESCALE_THR = 8.f;

// split-K merges with at most this many key splits load every partial up front
constexpr int kMaxCombine = 16;

#ifdef OV3D_ATTN_PROBE
// diagnostic build only (tools/attn_probe_phases.py): per-wave s_memtime totals of the tile
// phases of attn_fwd_kernel
__device__ unsigned long long* g_attn_probe;
#define PROBE_ENTRY const unsigned long long pr_entry = __builtin_amdgcn_s_memtime();
#define PROBE_DECL unsigned long long pr_t = __builtin_amdgcn_s_memtime(), pr_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
    pr_acc[7] = pr_t - pr_entry;
#define PROBE(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); pr_acc[i] += t_ - pr_t; pr_t = t_; } while (0)
#define PROBE_END do { if ((threadIdx.x & 63) == 0 && g_attn_probe) { \
    unsigned long long* o_ = g_attn_probe + (((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 32 + (threadIdx.x >> 6) * 8; \
    for (int i_ = 0; i_ < 8; ++i_) o_[i_] = pr_acc[i_]; } } while (0)
#else
#define PROBE_ENTRY
#define PROBE_DECL
#define PROBE(i) do { } while (0)
#define PROBE_END do { } while (0)
#endif

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x4 tr16(const bf16* p) {
    s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(p));
    return __builtin_bit_cast(bf16x4, r);
}

// A operand of O^T += V^T P^T for d-tile dt and key k-step (t, s): lane (r = d, h)
// element j = V[32t + 16s + 8(j>>2) + 4h + (j&3)][32dt + r]  (see header)
__device__ __forceinline__ bf16x8 v_operand(const bf16* Vs, int lane, int dt, int t, int s) {
    const int g = lane >> 4, i = lane & 15;
    const int d0 = 32 * dt + 16 * (g & 1) + 4 * (i & 3);
    const int k0 = 32 * t + 16 * s + 4 * (g >> 1) + (i >> 2);
    const bf16x4 lo = tr16(Vs + img(k0, d0));
    const bf16x4 hi = tr16(Vs + img(k0 + 8, d0));
    bf16x8 a;
    a[0] = lo[0]; a[1] = lo[1]; a[2] = lo[2]; a[3] = lo[3];
    a[4] = hi[0]; a[5] = hi[1]; a[6] = hi[2]; a[7] = hi[3];
    return a;
}

// 0xFFFFFFFF where bit b of w is set, else 0 (one v_bfe_i32; written as asm so that the
// masking below stays bfe + bfi instead of the compiler's bit test + compare + select)
__device__ __forceinline__ uint32_t bit_mask(uint32_t w, int b) {   // b: a constant after unrolling
    uint32_t m;
    asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(w), "s"(b));
    return m;
}

// -inf where bit b of w is set (masked key), else x: v_bfe_i32 + v_bfi_b32 (asm: hipcc turns
// the select into xor + bitop3).  Only for values that are NOT an MFMA's result: the
// compiler's MFMA -> VALU hazard padding does not see inside inline asm, so the masks are
// applied to the score accumulators' initial values (-inf + products = -inf).
__device__ __forceinline__ float neg_inf_if(float x, uint32_t w, int b) {
    const uint32_t m = bit_mask(w, b);
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "s"(0xFF800000u), "v"(__builtin_bit_cast(uint32_t, x)));
    return __builtin_bit_cast(float, r);
}

// score bit of element i of score tile t in a query-major (drop / mask) word
__device__ __forceinline__ constexpr int score_bit(int t, int i) { return ((i & 1) << 4) + 8 * t + (i >> 1); }

// XCD-aware workgroup order: workgroup L of a launch runs on XCD L % 8 (the dispatcher's
// round robin; an assumption for speed only, any order is correct).  With the (block, b*H+h)
// grid taken in launch order every XCD would get 2 of the 16 workgroups of each (b, h), so
// each XCD's L2 fetched every head's K / V (Q / dO): 8x the HBM reads (rocprofv3 FETCH_SIZE,
// profiles/r03_pmc_summary_v1.json).  Remapped, XCD x runs all workgroups of heads
// [x * H/8, (x+1) * H/8): each K / V reaches one L2.  Single-split grids with gridDim.y % 8 == 0.
__device__ __forceinline__ void xcd_block(int& bx, int& by) {
    const int nx = gridDim.x, ny = gridDim.y;
    if (gridDim.z != 1 || (ny & 7)) {
        bx = blockIdx.x;
        by = blockIdx.y;
        return;
    }
    const int L = blockIdx.x + nx * blockIdx.y;
    const int j = L >> 3;
    by = (L & 7) * (ny >> 3) + j / nx;
    bx = j - (j / nx) * nx;
}

// Drop bits ahead of the forward (long attentions: the encoder's L = 2048): the query-major
// and key-major words the forward would store, from the same hash, in a VALU-only pass; the
// forward then reads one word per lane and tile (BITS) instead of hashing 16 key pairs on the
// softmax's critical path (the hash was ~40 % of the forward's vector issue).  Same grid and
// lane layout as attn_fwd_kernel (a wave = 32 queries, lane = (query r, half h)), every
// 64-key tile of the key range.
__global__ void __launch_bounds__(256) attn_dropgen_kernel(AttnArgs a) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    int bx, bh;
    xcd_block(bx, bh);
    const int q0 = bx * (4 * QW) + wave * QW;
    if (q0 >= a.Lq) return;
    const uint32_t qh = drop_query_base(drop_head_mix(a.seed, a.site, bh), q0 + r) +
                        (uint32_t)(2 * h) * kPairMul;
    uint32_t* const wq_lane = a.wq + ((size_t)bh * a.Lq + q0 + r) * 2 + h;
    const size_t wq_tile = (size_t)gridDim.y * a.Lq * 2;
    uint32_t* const wk_lane = a.wk + ((size_t)(q0 >> 5) * gridDim.y + bh) * ((size_t)a.nkt * 64) +
                              drop_key(r, h);
    const short ts = (short)((int)a.thresh - 32768);
    const s16x2 tsig = {ts, ts};
    // blockIdx.z: a range of the key tiles (4x the waves of one per 32 queries; measured 33.5 ->
    // 30.9 us: the pass sits at its vector-issue bound either way)
    const int per = (a.nkt + gridDim.z - 1) / gridDim.z;
    const int kt1 = min(a.nkt, (int)(blockIdx.z + 1) * per);
    for (int kt = blockIdx.z * per; kt < kt1; ++kt) {
        const uint32_t hb = qh + (uint32_t)(32 * kt) * kPairMul;
        uint32_t dw = 0;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                const uint32_t c = 16 * t + ((i & 3) >> 1) + 4 * (i >> 2);
                const uint32_t dm = drop_halves(drop_mix(hb + c * kPairMul), tsig);
                const int jb = 8 * t + (i >> 1);
                dw |= dm & ((1u << jb) | (1u << (16 + jb)));
            }
        wq_lane[(size_t)kt * wq_tile] = dw;
        wk_lane[64 * kt] = transpose32(dw, r);
    }
}

// BITS: dropout from the words of attn_dropgen_kernel (read, not hashed, not stored)
template <bool DROP, bool MASK, bool BITS>
__device__ __forceinline__ void attn_fwd_body(const AttnArgs& a) {
    PROBE_ENTRY
    // K and V tiles in one array: its 36 KB also stage the output rows after the loop
    __shared__ __attribute__((aligned(16))) bf16 KVs[2][2][KB * LDK];
    bf16 (*const Ks)[KB * LDK] = KVs[0];
    bf16 (*const Vs)[KB * LDK] = KVs[1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    int bx, bh;
    xcd_block(bx, bh);
    const int b = bh / a.H, hh = bh - b * a.H;
    const int q0 = bx * (4 * QW) + wave * QW;
    const bool active = q0 < a.Lq;
    const int kbeg = blockIdx.z * a.keys_per_split;
    const int kend = min(a.Lk, kbeg + a.keys_per_split);

    bf16x8 qf[4];
    {
        const int qi = active ? q0 + r : 0;
        const bf16* qrow = a.q + ((size_t)qi * a.B + b) * a.sq + hh * D;
#pragma unroll
        for (int s = 0; s < 4; ++s)
            qf[s] = prescale8(*reinterpret_cast<const bf16x8*>(qrow + 16 * s + 8 * h), a.scale2);
    }
    // dropout hash input of key pair (kb >> 1) + 2h + c: qh + (kb >> 1) * kPairMul (wave-
    // uniform, once per tile) + c * kPairMul (a constant per unrolled pair)
    uint32_t qh = 0;
    if (DROP && !BITS) qh = drop_query_base(drop_head_mix(a.seed, a.site, bh), active ? q0 + r : 0) +
                            (uint32_t)(2 * h) * kPairMul;
    // drop-word destinations (BITS: sources): query-major word (kt, bh, q, h), key-major word
    // (q0/32, bh, key)
    uint32_t* const wq_lane = DROP ? a.wq + ((size_t)bh * a.Lq + (active ? q0 + r : 0)) * 2 + h : nullptr;
    const size_t wq_tile = (size_t)gridDim.y * a.Lq * 2;
    uint32_t* const wk_lane = (DROP && !BITS) ? a.wk + ((size_t)(q0 >> 5) * gridDim.y + bh) * ((size_t)a.nkt * 64) +
                                         drop_key(r, h) : nullptr;
    uint32_t dw_prev = 0;   // drop word of the tile before this one
    // BITS: this tile's drop word, loaded one tile ahead (its latency off the softmax)
    uint32_t dw_cur = 0, dw_next = 0;
    uint32_t mw_cur = 0, mw_next = 0;   // MASK: the same for the mask word
    // mask words of this lane (query q0 + r, half h), one per 64-key tile
    const uint32_t* const mrow = MASK ? a.mq + ((size_t)b * a.Lq + (active ? q0 + r : 0)) * 2 + h : nullptr;
    const size_t mtile = (size_t)a.B * a.Lq * 2;
    auto store_drop = [&](int kbp) {
        wq_lane[(size_t)(kbp >> 6) * wq_tile] = dw_prev;
        wk_lane[kbp] = transpose32(dw_prev, r);   // lane r: key drop_key(r, h), bit n = query q0 + n
    };

    // cooperative tile load: 64 keys x 8 chunks of 8 bf16 = 512 chunks, 2 per thread; the
    // per-thread offsets of key tid>>3 are formed once, a tile adds kb * B * s (scalar unit)
    bf16x8 kr[2], vr[2];
    const size_t rowk = (size_t)a.B * a.sk, rowv = (size_t)a.B * a.sv;
    const size_t k0off = (size_t)b * a.sk + hh * D + 8 * (tid & 7) + (size_t)(tid >> 3) * rowk;
    const size_t v0off = (size_t)b * a.sv + hh * D + 8 * (tid & 7) + (size_t)(tid >> 3) * rowv;
    auto load = [&](int kb) {
        if (kb + KB <= a.Lk) {   // whole tile (wave-uniform): scalar offsets, no clamps
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                kr[c] = *reinterpret_cast<const bf16x8*>(a.k + k0off + (size_t)(kb + 32 * c) * rowk);
                vr[c] = *reinterpret_cast<const bf16x8*>(a.v + v0off + (size_t)(kb + 32 * c) * rowv);
            }
            return;
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int key = kb + (tid >> 3) + 32 * c;
            size_t ko = k0off + (size_t)(kb + 32 * c) * rowk, vo = v0off + (size_t)(kb + 32 * c) * rowv;
            if (key >= a.Lk) {   // past the last key (partial tile): repeat the last row
                ko -= (size_t)(key - (a.Lk - 1)) * rowk;
                vo -= (size_t)(key - (a.Lk - 1)) * rowv;
            }
            kr[c] = *reinterpret_cast<const bf16x8*>(a.k + ko);
            vr[c] = *reinterpret_cast<const bf16x8*>(a.v + vo);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int idx = tid + 256 * c, key = idx >> 3, ch = idx & 7;
            *reinterpret_cast<bf16x8*>(&Ks[buf][img(key, 8 * ch)]) = kr[c];
            *reinterpret_cast<bf16x8*>(&Vs[buf][img(key, 8 * ch)]) = vr[c];
        }
    };

    f32x16 o[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) o[0][i] = o[1][i] = 0.f;
    // running max of the lane's query (log2 domain), bf16-exact: the score chains start with
    // one MFMA k-step that subtracts it (A = 1 in k-slot 0, B = -mb), so S' = S - mb comes out
    // of the matrix cores; the first tile with an attended key sets it to that tile's max
    float mb = 0.f;
    bool unset = true;
    const bf16x8 k1 = kslots(1.f, 0.f, h == 0);
    bf16x8 kmb = kslots(0.f, 0.f, false);
    // row sums on the matrix cores: an all-ones A operand times the (undropped) P^T packs
    // gives every accumulator row the column sums = each lane's query row sum over the 64 keys
    // of the tile (both lane halves), 4 MFMAs per tile instead of 32 VALU adds (the loop is
    // VALU-issue bound); element 0 carries the running sum (the rescale touches only it)
    f32x16 lacc;
#pragma unroll
    for (int i = 0; i < 16; ++i) lacc[i] = 0.f;
    bf16x8 ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.f;

    if (kbeg < kend) {
        load(kbeg);
        store(0);
        if (DROP && BITS && active) dw_cur = wq_lane[(size_t)(kbeg >> 6) * wq_tile];
        if (MASK && active) mw_cur = mrow[(size_t)(kbeg >> 6) * mtile];
    }
    __syncthreads();
    PROBE_DECL
    int buf = 0;
    for (int kb = kbeg; kb < kend; kb += KB, buf ^= 1) {
        const bool more = kb + KB < kend;
        PROBE(0);
        // every wave computes (a wave past Lq on the clamped query row 0, storing nothing): a
        // branch around the tile would make the accumulators' loop-carried registers a phi of
        // two paths, and hipcc then copied o / lacc back every tile (dQ: 32 v_mov per tile)
        {
            const bf16* K = Ks[buf];
            const bf16* V = Vs[buf];
            if (MASK && more) mw_next = mrow[(size_t)((kb >> 6) + 1) * mtile];
            const uint32_t mw = mw_cur;
            if (DROP && BITS && more) dw_next = wq_lane[(size_t)((kb >> 6) + 1) * wq_tile];
            const uint32_t kwin = ~dw_cur;
            // all LDS operand reads of the tile are issued ahead of their MFMAs, so their
            // latency overlaps the matrix / softmax work instead of stalling each MFMA
            bf16x8 ka[2][4];
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    ka[t][s] = *reinterpret_cast<const bf16x8*>(K + img(32 * t + r, 16 * s + 8 * h));
            // masked keys (MASK): -inf initial scores, so the MFMA results carry the mask
            f32x16 st[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    st[t][i] = MASK ? __builtin_bit_cast(float, bit_mask(mw, score_bit(t, i)) & 0xFF800000u) : 0.f;
                st[t] = mfma(k1, kmb, st[t]);   // - mb
            }
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int t = 0; t < 2; ++t) st[t] = mfma(ka[t][s], qf[s], st[t]);
            bf16x8 va[2][2][2];
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int s = 0; s < 2; ++s) va[dt][t][s] = v_operand(V, lane, dt, t, s);
            // next tile's global loads go out after this tile's LDS operand reads: issued
            // earlier, their address registers collide with the operand registers and the
            // compiler waits for the loads inside the score MFMAs
            if (more) load(kb + KB);
            // the previous tile's drop word goes out while the score MFMAs run: the lane
            // transpose's swizzle round trips would otherwise sit on this tile's critical path
            if (DROP && !BITS && kb > kbeg && active) store_drop(kb - KB);
            PROBE(1);
            // keys past Lk (last partial tile) do not take part
            const int nvalid = kend - kb;
            if (nvalid < KB) {
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        if (32 * t + (i & 3) + 8 * (i >> 2) + 4 * h >= nvalid) st[t][i] = -INFINITY;
            }
            float mx = -INFINITY;   // max of S - mb over the lane's keys
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) mx = fmaxf(mx, st[t][i]);
            mx = max_halves(mx);
            PROBE(2);
            // deferred rescale (T13): keep the stale max unless some query's max grew a lot
            const bool seen = mx > -INFINITY;   // some key of the tile attended
            if (__any(mx > RESCALE_THR || (unset && seen))) {
                // new stabiliser: the running max rounded to bf16 (nearest: never below mb when
                // mx > 0); a query's first attended tile sets it up or down
                const float mn = (mx > 0.f || (unset && seen)) ? bf16_hi(mb + mx) : mb;
                const float d = mn - mb;
                // o and the sums of a query with no attended key yet are zero (alpha = 1 keeps
                // them so even when exp2(-d) would overflow)
                const float alpha = unset ? 1.f : fast_exp2(-d);
                lacc[0] *= alpha;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    o[0][i] *= alpha;
                    o[1][i] *= alpha;
                }
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int i = 0; i < 16; ++i) st[t][i] -= d;
                mb = mn;
                kmb = kslots(-mb, 0.f, h == 0);
                unset = unset && !seen;
            }
            // p = exp2(S - mb), one bf16 pack per key pair; dropout zeroes p after the row sum.
            // Scalar f32 ops on purpose: packed v_pk_* issue slower than two scalar ops beside
            // the MFMAs (MI355X_MICROARCH.md cycle table; the file is built with -fno-slp-vectorize)
            const uint32_t hb = qh + (uint32_t)(kb >> 1) * kPairMul;
            const short ts = (short)((int)a.thresh - 32768);
            const s16x2 tsig = {ts, ts};
            uint32_t dw = 0;   // this lane's drop word of the tile
            u32x4 pw[2][2], praw[2][2];
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    float p0 = fast_exp2(st[t][i]);
                    float p1 = fast_exp2(st[t][i + 1]);
#ifdef OV3D_ATTN_VALU_ROWSUM
#endif
                    uint32_t pk = pack_bf16(p0, p1);
                    praw[t][i >> 3][(i & 7) >> 1] = pk;
                    if (DROP && BITS) {
                        // keep bits 8t + (i>>1) (even key) and 16 + 8t + (i>>1) (odd key) move
                        // to bits 15 and 31; one packed arithmetic shift spreads each over its
                        // bf16 half: shift, v_pk_ashrrev_i16, and
                        const int jb = 8 * t + (i >> 1);
                        const s16x2 kh = __builtin_bit_cast(s16x2, kwin << (15 - jb));
                        pk &= __builtin_bit_cast(uint32_t, (s16x2)(kh >> (s16x2){15, 15}));
                    } else if (DROP) {
                        // key 32t + (i&3) + 8(i>>2) + 4h (even): pair 16t + (i&3)/2 + 4(i>>2) + 2h
                        const uint32_t c = 16 * t + ((i & 3) >> 1) + 4 * (i >> 2);
                        const uint32_t dm = drop_halves(drop_mix(hb + c * kPairMul), tsig);
                        // 1/(1-p) is applied once to the output (keep_scale below)
                        pk &= ~dm;
                        const int jb = 8 * t + (i >> 1);
                        dw |= dm & ((1u << jb) | (1u << (16 + jb)));
                    }
                    pw[t][i >> 3][(i & 7) >> 1] = pk;
                }
            if (DROP && !BITS) dw_prev = dw;
            if (DROP && BITS) dw_cur = dw_next;
            if (MASK) mw_cur = mw_next;
            PROBE(3);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const bf16x8 pf = __builtin_bit_cast(bf16x8, pw[t][s]);
#pragma unroll
                    for (int dt = 0; dt < 2; ++dt) o[dt] = mfma(va[dt][t][s], pf, o[dt]);
#ifndef OV3D_ATTN_VALU_ROWSUM
                    lacc = mfma(ones, __builtin_bit_cast(bf16x8, praw[t][s]), lacc);
#endif
                }
        }
        PROBE(4);
        if (more) store(buf ^ 1);
        PROBE(5);
        __syncthreads();
        PROBE(6);
    }
    PROBE_END;
    if (active && DROP && !BITS && kend > kbeg) store_drop((kend - 1) & ~(KB - 1));
#ifdef OV3D_ATTN_VALU_ROWSUM
    const float ltot = l + __shfl_xor(l, 32);
#else
    const float ltot = lacc[0];
#endif
    const int q = q0 + r;
    // The workgroup's 128 output rows go through LDS (free after the loop's last barrier): a
    // lane holds 4-dim pieces of its query's row, stored directly those are 8 / 16-byte writes
    // at a row stride (32 rows per instruction); staged, whole rows leave 16 bytes a lane.
    const int ql = wave * QW + r;
    if (a.nsplit == 1) {
        const float inv = ltot > 0.f ? a.keep_scale / ltot : 0.f;
        bf16* const so = &KVs[0][0][0];   // [128 queries][LDK]
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                bf16x4 w;
#pragma unroll
                for (int j = 0; j < 4; ++j) w[j] = (bf16)(o[dt][4 * g + j] * inv);
                *reinterpret_cast<bf16x4*>(so + ql * LDK + 32 * dt + 8 * g + 4 * h) = w;
            }
        if (active && h == 0) a.lse[(size_t)bh * a.Lq + q] = mb + log2f(ltot);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = tid + 256 * i, row = c >> 3, d8 = (c & 7) * 8;
            const int qq = bx * (4 * QW) + row;
            if (qq < a.Lq)
                *reinterpret_cast<bf16x8*>(a.o + ((size_t)qq * a.B + b) * a.so + hh * D + d8) =
                    *reinterpret_cast<const bf16x8*>(so + row * LDK + d8);
        }
    } else {
        constexpr int LDF = D + 4;   // fp32 staging row (272 B)
        float* const sf = reinterpret_cast<float*>(&KVs[0][0][0]);   // [128 queries][LDF]
        static_assert(sizeof(KVs) >= 128 * LDF * sizeof(float), "fp32 staging rows overrun KVs");
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                *reinterpret_cast<float4*>(sf + ql * LDF + 32 * dt + 8 * g + 4 * h) =
                    make_float4(o[dt][4 * g] * a.keep_scale, o[dt][4 * g + 1] * a.keep_scale,
                                o[dt][4 * g + 2] * a.keep_scale, o[dt][4 * g + 3] * a.keep_scale);
        const size_t rbase = ((size_t)blockIdx.z * gridDim.y + bh) * a.Lq;
        if (active && h == 0) {
            a.part_ml[2 * (rbase + q)] = ltot > 0.f ? mb : -INFINITY;
            a.part_ml[2 * (rbase + q) + 1] = ltot;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int c = tid + 256 * i, row = c >> 4, d4 = (c & 15) * 4;
            const int qq = bx * (4 * QW) + row;
            if (qq < a.Lq)
                *reinterpret_cast<float4*>(a.part_o + (rbase + qq) * D + d4) =
                    *reinterpret_cast<const float4*>(sf + row * LDF + d4);
        }
    }
}

template <bool DROP, bool MASK, bool BITS>
__global__ void __launch_bounds__(256, 2) attn_fwd_kernel(AttnArgs a) {
    ov3d_stamp(a.stamp, 0);
    attn_fwd_body<DROP, MASK, BITS>(a);
    ov3d_stamp(a.stamp, 1);
}

// merge split-K partials: one 64-lane wave per (b*H+h, query); lane = d
// NS: the split count rounded up to a power of two (<= kMaxCombine), the loads clamped to the
// last split (with NS = 16 for every split count, 8 splits loaded each partial twice)
template <int NS>
__global__ void __launch_bounds__(256) attn_combine_kernel(AttnArgs a) {
    const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, d = threadIdx.x & 63;
    const int BH = a.B * a.H;
    if (w >= BH * a.Lq) return;
    const int bh = w / a.Lq, q = w - bh * a.Lq;
    const int b = bh / a.H, hh = bh - b * a.H;
    float M = -INFINITY;
    float L = 0.f, acc = 0.f;
    if (a.nsplit <= NS) {
        // every split's (m, l, o) is loaded up front: the generic loops below are 2·nsplit
        // dependent global round trips
        float ms[NS], ls[NS], os[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {   // unpredicated loads (split clamped)
            const int sc = s < a.nsplit ? s : a.nsplit - 1;
            const size_t row = ((size_t)sc * BH + bh) * a.Lq + q;
            ms[s] = a.part_ml[2 * row];
            ls[s] = a.part_ml[2 * row + 1];
            os[s] = a.part_o[row * D + d];
        }
#pragma unroll
        for (int s = 0; s < NS; ++s)
            if (s >= a.nsplit) ms[s] = -INFINITY;
#pragma unroll
        for (int s = 0; s < NS; ++s) M = fmaxf(M, ms[s]);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (ms[s] == -INFINITY) continue;
            const float wgt = exp2f(ms[s] - M);
            L = fmaf(ls[s], wgt, L);
            acc = fmaf(os[s], wgt, acc);
        }
        a.o[((size_t)q * a.B + b) * a.so + hh * D + d] = (bf16)(L > 0.f ? acc / L : 0.f);
        if (d == 0) a.lse[(size_t)bh * a.Lq + q] = M + log2f(L);
        return;
    }
    for (int s = 0; s < a.nsplit; ++s) M = fmaxf(M, a.part_ml[2 * (((size_t)s * BH + bh) * a.Lq + q)]);
    for (int s = 0; s < a.nsplit; ++s) {
        const size_t row = ((size_t)s * BH + bh) * a.Lq + q;
        const float ms = a.part_ml[2 * row];
        if (ms == -INFINITY) continue;
        const float wgt = exp2f(ms - M);
        L = fmaf(a.part_ml[2 * row + 1], wgt, L);
        acc = fmaf(a.part_o[row * D + d], wgt, acc);
    }
    a.o[((size_t)q * a.B + b) * a.so + hh * D + d] = (bf16)(L > 0.f ? acc / L : 0.f);
    if (d == 0) a.lse[(size_t)bh * a.Lq + q] = M + log2f(L);
}


// ---------------------------------------------------------------- backward
// Gradients of O = dropout(softmax(scale Q K^T)) V with the saved lse (log2 domain):
//   P = exp2(scale2 S - lse2), P~ = P Z/(1-p), dP~ = dO V^T, dS = P (dP~ Z/(1-p) - D),
//   D = rowsum(dO o O), dQ = scale dS K, dK = scale dS^T Q, dV = P~^T dO.
// attn_bwd_dq_kernel (swapped layout as the forward, a lane owns a query) computes D,
// stores it, and dQ; attn_bwd_dkdv_kernel (a lane owns a key) computes dK and dV.

struct AttnBwdArgs {
    AttnArgs f;
    const bf16* o;        // forward output rows (stride f.so)
    const bf16* dout;     // grad rows (stride sdo)
    long long sdo;
    float* dvec;          // (B*H, Lq) D
    bf16* dq;
    bf16* dk;
    bf16* dv;
    long long sdq, sdk, sdv;
    float scale;
    unsigned long long* stamp2;   // the dK / dV launch's stamps (f.stamp: the dQ launch's)
};

// RAGGED: Lk % 64 != 0 (the last key tile is partial); the key check exists only then
template <bool DROP, bool MASK, bool RAGGED>
__device__ __forceinline__ void attn_bwd_dq_body(const AttnBwdArgs& A) {
    const AttnArgs& a = A.f;
    // K and V tiles in one array: its 36 KB also stage the dQ rows after the loop
    __shared__ __attribute__((aligned(16))) bf16 KVs[2][2][KB * LDK];
    bf16 (*const Ks)[KB * LDK] = KVs[0];
    bf16 (*const Vs)[KB * LDK] = KVs[1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    int bx, bh;
    xcd_block(bx, bh);
    const int b = bh / a.H, hh = bh - b * a.H;
    const int q0 = bx * (4 * QW) + wave * QW;
    const bool active = q0 < a.Lq;
    const int qi = active ? q0 + r : 0;

    bf16x8 qf[4], df[4];
    float dsum = 0.f;
    {
        const bf16* qrow = a.q + ((size_t)qi * a.B + b) * a.sq + hh * D;
        const bf16* drow = A.dout + ((size_t)qi * a.B + b) * A.sdo + hh * D;
        const bf16* orow = A.o + ((size_t)qi * a.B + b) * a.so + hh * D;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            qf[s] = prescale8(*reinterpret_cast<const bf16x8*>(qrow + 16 * s + 8 * h), a.scale2);
            df[s] = *reinterpret_cast<const bf16x8*>(drow + 16 * s + 8 * h);
            const bf16x8 ov = *reinterpret_cast<const bf16x8*>(orow + 16 * s + 8 * h);
#pragma unroll
            for (int j = 0; j < 8; ++j) dsum = fmaf((float)df[s][j], (float)ov[j], dsum);
        }
    }
    dsum += __shfl_xor(dsum, 32);
    float lse2 = active ? a.lse[(size_t)bh * a.Lq + qi] : 0.f;
    if (MASK && lse2 == -INFINITY) lse2 = INFINITY;   // no attended key: P = 0
    // row constants of the lane's query added by one more MFMA k-step each (kslots): with the
    // prescaled queries S' = S scale2 + s_init gives p' = exp2(S') = P / (1 - p) directly,
    // dP' = dP + d_init gives dS = p' (Z ? dP' : d_init) = P (Z dP / (1 - p) - D): no initial
    // values, multiply or subtraction per element, and the dropout select is one v_bfi_b32
    const float s_init = -lse2 + (DROP ? __log2f(a.keep_scale) : 0.f);
    const float d_init = -dsum / a.keep_scale;
    const bf16x8 k11 = kslots(1.f, 1.f, h == 0);
    const bf16x8 ks = kslots(bf16_hi(s_init), bf16_lo(s_init), h == 0);
    const bf16x8 kd = kslots(bf16_hi(d_init), bf16_lo(d_init), h == 0);
    if (active && h == 0 && blockIdx.z == 0) A.dvec[(size_t)bh * a.Lq + qi] = dsum;
    // the forward's query-major drop words of this lane, one per 64-key tile (prefetched a
    // tile ahead with the K / V rows)
    const uint32_t* wrow = DROP ? a.wq + ((size_t)bh * a.Lq + qi) * 2 + h : nullptr;
    const size_t wstride = (size_t)gridDim.y * a.Lq * 2;
    uint32_t wcur = 0, wnext = 0;
    const uint32_t* mrow = MASK ? a.mq + ((size_t)b * a.Lq + qi) * 2 + h : nullptr;
    const size_t mtile = (size_t)a.B * a.Lq * 2;
    uint32_t mcur = 0, mnext = 0;

    bf16x8 kr[2], vr[2];
    // row (key) r of the tile starts at r * B * s: the per-thread offsets of key tid>>3 are
    // formed once and a tile adds kb * B * s (wave-uniform, scalar unit), so the loads carry
    // no per-tile 64-bit vector multiplies
    const size_t rowk = (size_t)a.B * a.sk, rowv = (size_t)a.B * a.sv;
    const size_t k0off = (size_t)b * a.sk + hh * D + 8 * (tid & 7) + (size_t)(tid >> 3) * rowk;
    const size_t v0off = (size_t)b * a.sv + hh * D + 8 * (tid & 7) + (size_t)(tid >> 3) * rowv;
    auto load = [&](int kb) {
        if (kb + KB <= a.Lk) {   // whole tile (wave-uniform): scalar offsets, no clamps
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                kr[c] = *reinterpret_cast<const bf16x8*>(a.k + k0off + (size_t)(kb + 32 * c) * rowk);
                vr[c] = *reinterpret_cast<const bf16x8*>(a.v + v0off + (size_t)(kb + 32 * c) * rowv);
            }
            return;
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int key = kb + (tid >> 3) + 32 * c;
            size_t ko = k0off + (size_t)(kb + 32 * c) * rowk, vo = v0off + (size_t)(kb + 32 * c) * rowv;
            if (key >= a.Lk) {   // past the last key (partial tile): repeat the last row
                ko -= (size_t)(key - (a.Lk - 1)) * rowk;
                vo -= (size_t)(key - (a.Lk - 1)) * rowv;
            }
            kr[c] = *reinterpret_cast<const bf16x8*>(a.k + ko);
            vr[c] = *reinterpret_cast<const bf16x8*>(a.v + vo);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int idx = tid + 256 * c, key = idx >> 3, ch = idx & 7;
            *reinterpret_cast<bf16x8*>(&Ks[buf][img(key, 8 * ch)]) = kr[c];
            *reinterpret_cast<bf16x8*>(&Vs[buf][img(key, 8 * ch)]) = vr[c];
        }
    };
    f32x16 dqt[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) dqt[0][i] = dqt[1][i] = 0.f;
    const int kbeg = blockIdx.z * a.keys_per_split;
    const int kend = min(a.Lk, kbeg + a.keys_per_split);
    if (kbeg < kend) {
        load(kbeg);
        store(0);
        if (DROP && active) wcur = wrow[(size_t)(kbeg >> 6) * wstride];
        if (MASK && active) mcur = mrow[(size_t)(kbeg >> 6) * mtile];
    }
    __syncthreads();
    int buf = 0;
    for (int kb = kbeg; kb < kend; kb += KB, buf ^= 1) {
        const bool more = kb + KB < kend;
        if (more) load(kb + KB);
        if (DROP && active && more) wnext = wrow[(size_t)((kb >> 6) + 1) * wstride];
        if (MASK && active && more) mnext = mrow[(size_t)((kb >> 6) + 1) * mtile];
        // the tile body as a generic lambda, instantiated twice when RAGGED: the partial-tile key
        // check exists only in the copy the last tile takes (inline, hipcc if-converts it into
        // every tile)
        auto tile = [&](auto partial) {
            constexpr bool PARTIAL = decltype(partial)::value;
            const bf16* K = Ks[buf];
            const bf16* V = Vs[buf];
            const int nvalid = kend - kb;
            const uint32_t kcur = ~wcur;   // keep bits
            u32x4 dsw[2][2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                f32x16 st, dpt;
#pragma unroll
                for (int i = 0; i < 16; ++i) {   // masked keys: -inf initial scores
                    st[i] = MASK ? neg_inf_if(0.f, mcur, score_bit(t, i)) : 0.f;
                    dpt[i] = 0.f;
                }
                st = mfma(k11, ks, st);
                dpt = mfma(k11, kd, dpt);
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const bf16x8 ka = *reinterpret_cast<const bf16x8*>(K + img(32 * t + r, 16 * s + 8 * h));
                    const bf16x8 va = *reinterpret_cast<const bf16x8*>(V + img(32 * t + r, 16 * s + 8 * h));
                    st = mfma(ka, qf[s], st);
                    dpt = mfma(va, df[s], dpt);
                }
                // keys past Lk (last partial tile, wave-uniform branch): score -inf -> P = 0
                if (PARTIAL) {
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        if (32 * t + (i & 3) + 8 * (i >> 2) + 4 * h >= nvalid) st[i] = -INFINITY;
                }
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    const float p0 = fast_exp2(st[i]);
                    const float p1 = fast_exp2(st[i + 1]);
                    float dp0 = dpt[i], dp1 = dpt[i + 1];
                    if (DROP) {   // keep bits 8t + (i>>1) (even key), 16 + 8t + (i>>1) (odd key)
                        const uint32_t k0 = bit_mask(kcur, 8 * t + (i >> 1));
                        const uint32_t k1 = bit_mask(kcur, 16 + 8 * t + (i >> 1));
                        const uint32_t di = __builtin_bit_cast(uint32_t, d_init);
                        dp0 = __builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, dp0) & k0) | (di & ~k0));
                        dp1 = __builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, dp1) & k1) | (di & ~k1));
                    }
                    dsw[t][i >> 3][(i & 7) >> 1] = pack_bf16(p0 * dp0, p1 * dp1);
                }
            }
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int s = 0; s < 2; ++s)
                        dqt[dt] = mfma(v_operand(K, lane, dt, t, s), __builtin_bit_cast(bf16x8, dsw[t][s]), dqt[dt]);
        };
        {   // every wave (see attn_fwd_body: no branch around the accumulators)
            if constexpr (RAGGED) {
                if (kend - kb < KB) tile(std::true_type{});
                else tile(std::false_type{});
            } else {
                tile(std::false_type{});
            }
        }
        if (more) store(buf ^ 1);
        wcur = wnext;
        mcur = mnext;
        __syncthreads();
    }
    // dQ rows through LDS, whole rows 16 bytes a lane (see attn_fwd_kernel)
    const int ql = wave * QW + r;
    if (a.nsplit > 1) {   // fp32 partial per key split, summed by attn_dq_combine_kernel
        constexpr int LDF = D + 4;
        float* const sf = reinterpret_cast<float*>(&KVs[0][0][0]);   // [128 queries][LDF]
        static_assert(sizeof(KVs) >= 128 * LDF * sizeof(float), "fp32 staging rows overrun KVs");
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                *reinterpret_cast<float4*>(sf + ql * LDF + 32 * dt + 8 * g + 4 * h) =
                    make_float4(dqt[dt][4 * g], dqt[dt][4 * g + 1], dqt[dt][4 * g + 2], dqt[dt][4 * g + 3]);
        __syncthreads();
        const size_t rbase = ((size_t)blockIdx.z * gridDim.y + bh) * a.Lq;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int c = tid + 256 * i, row = c >> 4, d4 = (c & 15) * 4;
            const int qq = bx * (4 * QW) + row;
            if (qq < a.Lq)
                *reinterpret_cast<float4*>(a.part_o + (rbase + qq) * D + d4) =
                    *reinterpret_cast<const float4*>(sf + row * LDF + d4);
        }
        return;
    }
    bf16* const sq = &KVs[0][0][0];   // [128 queries][LDK]
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            bf16x4 w;
#pragma unroll
            for (int j = 0; j < 4; ++j) w[j] = (bf16)(dqt[dt][4 * g + j] * A.scale);
            *reinterpret_cast<bf16x4*>(sq + ql * LDK + 32 * dt + 8 * g + 4 * h) = w;
        }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = tid + 256 * i, row = c >> 3, d8 = (c & 7) * 8;
        const int qq = bx * (4 * QW) + row;
        if (qq < a.Lq)
            *reinterpret_cast<bf16x8*>(A.dq + ((size_t)qq * a.B + b) * A.sdq + hh * D + d8) =
                *reinterpret_cast<const bf16x8*>(sq + row * LDK + d8);
    }
}

template <bool DROP, bool MASK, bool RAGGED>
__global__ void __launch_bounds__(256, 2) attn_bwd_dq_kernel(AttnBwdArgs A) {
    ov3d_stamp(A.f.stamp, 0);
    attn_bwd_dq_body<DROP, MASK, RAGGED>(A);
    ov3d_stamp(A.f.stamp, 1);
}

// dq = scale * sum over key splits; one thread per (b*H+h, query, 4 dims)
__global__ void __launch_bounds__(256) attn_dq_combine_kernel(AttnBwdArgs A) {
    const AttnArgs& a = A.f;
    const int BH = a.B * a.H;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)BH * a.Lq * (D / 4)) return;
    const int d4 = (int)(t % (D / 4));
    const long long w = t / (D / 4);
    const int bh = (int)(w / a.Lq), q = (int)(w - (long long)bh * a.Lq);
    const int b = bh / a.H, hh = bh - b * a.H;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int sp = 0; sp < a.nsplit; ++sp) {
        const float4 v = *reinterpret_cast<const float4*>(
            a.part_o + (((size_t)sp * BH + bh) * a.Lq + q) * D + 4 * d4);
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
    }
    bf16x4 o;
    o[0] = (bf16)(acc.x * A.scale);
    o[1] = (bf16)(acc.y * A.scale);
    o[2] = (bf16)(acc.z * A.scale);
    o[3] = (bf16)(acc.w * A.scale);
    *reinterpret_cast<bf16x4*>(A.dq + ((size_t)q * a.B + b) * A.sdq + hh * D + 4 * d4) = o;
}

// a lane owns a key: S = Q K^T tiles (32 queries x 32 keys) with the query on the registers
// OWN_D: D = rowsum(dO . O) of each query tile computed here from the forward output (the
// split small backward, whose dQ pass runs beside it in another workgroup) instead of read
// from the dQ pass's dvec
template <bool DROP, bool MASK, bool OWN_D = false>
__device__ __forceinline__ void attn_bwd_dkdv_body(const AttnBwdArgs& A) {
    const AttnArgs& a = A.f;
    constexpr int QB = 64;   // queries per LDS tile
    __shared__ __attribute__((aligned(16))) bf16 Qs[2][QB * LDK];
    __shared__ __attribute__((aligned(16))) bf16 Ds[2][QB * LDK];
    __shared__ __attribute__((aligned(16))) float Ls[2][QB];
    __shared__ __attribute__((aligned(16))) float Dv[2][QB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    int bx, bh;
    xcd_block(bx, bh);
    const int b = bh / a.H, hh = bh - b * a.H;
    const int k0 = bx * (4 * 32) + wave * 32;
    const bool active = k0 < a.Lk;
    const int ki = active ? min(k0 + r, a.Lk - 1) : 0;
    // the forward's key-major drop words of this lane's key: bit n of word (qblk, key) is
    // query 32 qblk + n (two 32-query blocks per tile, prefetched a tile ahead)
    const uint32_t* wcol = DROP ? a.wk + (size_t)bh * ((size_t)a.nkt * 64) + ki : nullptr;
    const size_t wstride = (size_t)gridDim.y * a.nkt * 64;
    uint32_t wn[2] = {0u, 0u};
    // mask words of this lane's key (batch row b), same key-major layout
    const uint32_t* mcol = MASK ? a.mk + (size_t)b * ((size_t)a.nkt * 64) + ki : nullptr;
    const size_t mstride = (size_t)a.B * a.nkt * 64;
    uint32_t mn[2] = {0u, 0u};

    bf16x8 kf[4], vf[4];
    {
        const bf16* krow = a.k + ((size_t)ki * a.B + b) * a.sk + hh * D;
        const bf16* vrow = a.v + ((size_t)ki * a.B + b) * a.sv + hh * D;
#pragma unroll
        for (int s = 0; s < 4; ++s) {   // key rows prescaled: log2-domain scores (see prescale8)
            kf[s] = prescale8(*reinterpret_cast<const bf16x8*>(krow + 16 * s + 8 * h), a.scale2);
            vf[s] = *reinterpret_cast<const bf16x8*>(vrow + 16 * s + 8 * h);
        }
    }

    bf16x8 qr[2], dr[2], orr[2];
    float lr = 0.f, dvr = 0.f;
    // per-thread offsets of query row tid>>3, advanced per tile by qb * B * s (scalar unit)
    const size_t rowq = (size_t)a.B * a.sq, rowd = (size_t)a.B * A.sdo;
    const size_t q0off = (size_t)b * a.sq + hh * D + 8 * (tid & 7) + (size_t)(tid >> 3) * rowq;
    const size_t d0off = (size_t)b * A.sdo + hh * D + 8 * (tid & 7) + (size_t)(tid >> 3) * rowd;
    auto load = [&](int qb) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int qq = qb + (tid >> 3) + 32 * c;
            const int qc = qq < a.Lq ? qq : a.Lq - 1;   // past the last query: repeat the last row
            if (qb + QB <= a.Lq) {   // whole tile (wave-uniform): scalar offsets, no clamps
                qr[c] = *reinterpret_cast<const bf16x8*>(a.q + q0off + (size_t)(qb + 32 * c) * rowq);
                dr[c] = *reinterpret_cast<const bf16x8*>(A.dout + d0off + (size_t)(qb + 32 * c) * rowd);
            } else {
                size_t qo = q0off + (size_t)(qb + 32 * c) * rowq, dof = d0off + (size_t)(qb + 32 * c) * rowd;
                if (qq >= a.Lq) {
                    qo -= (size_t)(qq - (a.Lq - 1)) * rowq;
                    dof -= (size_t)(qq - (a.Lq - 1)) * rowd;
                }
                qr[c] = *reinterpret_cast<const bf16x8*>(a.q + qo);
                dr[c] = *reinterpret_cast<const bf16x8*>(A.dout + dof);
            }
            if (OWN_D)
                orr[c] = *reinterpret_cast<const bf16x8*>(A.o + ((size_t)qc * a.B + b) * a.so + hh * D + 8 * (tid & 7));
        }
        if (tid < QB) {
            const int qq = qb + tid;
            const int qc = qq < a.Lq ? qq : a.Lq - 1;
            // queries past Lq: lse = +inf -> P = 0
            lr = qq < a.Lq ? a.lse[(size_t)bh * a.Lq + qc] : INFINITY;
            if (MASK && lr == -INFINITY) lr = INFINITY;   // query with no attended key
            if (!OWN_D) dvr = A.dvec[(size_t)bh * a.Lq + qc];
            // the row constants as the S / dP accumulators' initial values (see the loop); the
            // key rows are prescaled, so S is in the log2 domain and so is -lse2
            lr = -lr;
            if (!OWN_D) dvr = -dvr / a.keep_scale;
        }
        if (DROP && active) {
#pragma unroll
            for (int u = 0; u < 2; ++u)
                wn[u] = qb + 32 * u < a.Lq ? wcol[(size_t)((qb >> 5) + u) * wstride] : 0u;
        }
        if (MASK && active) {
#pragma unroll
            for (int u = 0; u < 2; ++u)
                mn[u] = qb + 32 * u < a.Lq ? mcol[(size_t)((qb >> 5) + u) * mstride] : 0u;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int idx = tid + 256 * c, qq = idx >> 3, ch = idx & 7;
            *reinterpret_cast<bf16x8*>(&Qs[buf][img(qq, 8 * ch)]) = qr[c];
            *reinterpret_cast<bf16x8*>(&Ds[buf][img(qq, 8 * ch)]) = dr[c];
        }
        if (tid < QB) {
            Ls[buf][tid] = lr;
            if (!OWN_D) Dv[buf][tid] = dvr;
        }
        if (OWN_D) {   // 8 lanes per query row, 8 of its 64 dims each
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                float t = 0.f;
#pragma unroll
                for (int j = 0; j < 8; ++j) t = fmaf((float)dr[c][j], (float)orr[c][j], t);
                t += __shfl_xor(t, 1);
                t += __shfl_xor(t, 2);
                t += __shfl_xor(t, 4);
                if ((tid & 7) == 0) Dv[buf][(tid >> 3) + 32 * c] = -t / a.keep_scale;
            }
        }
    };
    f32x16 dkt[2], dvt[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) dkt[0][i] = dkt[1][i] = dvt[0][i] = dvt[1][i] = 0.f;
    // a lane past the last key holds a copy of the last key's row: finite values, never stored
    load(0);
    store(0);
    uint32_t wc[2] = {wn[0], wn[1]};
    uint32_t mc[2] = {mn[0], mn[1]};
    __syncthreads();
    int buf = 0;
    for (int qb = 0; qb < a.Lq; qb += QB, buf ^= 1) {
        const bool more = qb + QB < a.Lq;
        if (more) load(qb + QB);
        {   // every wave (see attn_fwd_body: no branch around the accumulators)
            const bf16* Q = Qs[buf];
            const bf16* DO = Ds[buf];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                // row constants (per element = query row 8g + 4h + j) as the initial
                // accumulators: S' = S scale2 - lse2 gives P = exp2(S') (prescaled keys), dP' =
                // dP - D (1-p) gives dS = P (Z dP / (1-p) - D) = P (Z ? dP' : -D (1-p)) / (1-p),
                // the 1/(1-p) applied to dK once at the end as it is to dV.  (Here the initial
                // values stay: the k-slot MFMA step of the dQ pass lengthened this pass's chains
                // and measured slower, 109 -> 113 us.)
                float lv[16], dv[16];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int qrow = 32 * u + 8 * g + 4 * h;      // rows 4g..4g+3 of the tile
                    const float4 l4 = *reinterpret_cast<const float4*>(&Ls[buf][qrow]);
                    const float4 d4 = *reinterpret_cast<const float4*>(&Dv[buf][qrow]);
                    lv[4 * g] = l4.x; lv[4 * g + 1] = l4.y; lv[4 * g + 2] = l4.z; lv[4 * g + 3] = l4.w;
                    dv[4 * g] = d4.x; dv[4 * g + 1] = d4.y; dv[4 * g + 2] = d4.z; dv[4 * g + 3] = d4.w;
                }
                // masked (query, key): -inf initial score
                const uint32_t msh = MASK ? mc[u] >> (4 * h) : 0u;
                f32x16 st, dpt;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    st[i] = MASK ? neg_inf_if(lv[i], msh, 8 * (i >> 2) + (i & 3)) : lv[i];
                    dpt[i] = dv[i];
                }
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const bf16x8 qa = *reinterpret_cast<const bf16x8*>(Q + img(32 * u + r, 16 * s + 8 * h));
                    const bf16x8 da = *reinterpret_cast<const bf16x8*>(DO + img(32 * u + r, 16 * s + 8 * h));
                    st = mfma(qa, kf[s], st);
                    dpt = mfma(da, vf[s], dpt);
                }
                // keep bit of row 8g + 4h + j of this 32-query block: bit 8g + j of ~w >> 4h
                const uint32_t ksh = DROP ? ~wc[u] >> (4 * h) : 0u;
                u32x4 pw[2], dsw[2];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    float pd[4], ds[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int i = 4 * g + j;
                        const float p = fast_exp2(st[i]);
                        float pk = p, dp = dpt[i];
                        if (DROP) {   // 1/(1-p) applied to dV once at the end
                            const uint32_t km = bit_mask(ksh, 8 * g + j);
                            pk = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, p) & km);
                            dp = __builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, dp) & km) |
                                                               (__builtin_bit_cast(uint32_t, dv[i]) & ~km));
                        }
                        pd[j] = pk;
                        ds[j] = p * dp;
                    }
                    pw[g >> 1][2 * (g & 1)] = pack_bf16(pd[0], pd[1]);
                    pw[g >> 1][2 * (g & 1) + 1] = pack_bf16(pd[2], pd[3]);
                    dsw[g >> 1][2 * (g & 1)] = pack_bf16(ds[0], ds[1]);
                    dsw[g >> 1][2 * (g & 1) + 1] = pack_bf16(ds[2], ds[3]);
                }
#pragma unroll
                for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int tt = u;   // query sub-tile = k-step block of 32 rows
                        dvt[dt] = mfma(v_operand(DO, lane, dt, tt, s), __builtin_bit_cast(bf16x8, pw[s]), dvt[dt]);
                        dkt[dt] = mfma(v_operand(Q, lane, dt, tt, s), __builtin_bit_cast(bf16x8, dsw[s]), dkt[dt]);
                    }
            }
        }
        if (more) store(buf ^ 1);
        wc[0] = wn[0];
        wc[1] = wn[1];
        mc[0] = mn[0];
        mc[1] = mn[1];
        __syncthreads();
    }
    // dK / dV rows through LDS (the Q / dO tiles are free now): a lane holds 4-dim pieces of its
    // key's rows, stored directly those are 8-byte writes at a row stride (32 rows per
    // instruction); staged, the workgroup writes whole 128-byte rows, 16 bytes a lane
    bf16* const sk = &Qs[0][0];   // [128 keys][LDK]
    bf16* const sv = &Ds[0][0];
    const int kl = wave * 32 + r;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            bf16x4 wk, wv;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                wk[j] = (bf16)(dkt[dt][4 * g + j] * (A.scale * a.keep_scale));
                wv[j] = (bf16)(dvt[dt][4 * g + j] * a.keep_scale);
            }
            *reinterpret_cast<bf16x4*>(sk + kl * LDK + 32 * dt + 8 * g + 4 * h) = wk;
            *reinterpret_cast<bf16x4*>(sv + kl * LDK + 32 * dt + 8 * g + 4 * h) = wv;
        }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = tid + 256 * i, row = c >> 3, d8 = (c & 7) * 8;   // 128 rows x 8 pieces
        const int key = bx * 128 + row;
        if (key < a.Lk) {
            *reinterpret_cast<bf16x8*>(A.dk + ((size_t)key * a.B + b) * A.sdk + hh * D + d8) =
                *reinterpret_cast<const bf16x8*>(sk + row * LDK + d8);
            *reinterpret_cast<bf16x8*>(A.dv + ((size_t)key * a.B + b) * A.sdv + hh * D + d8) =
                *reinterpret_cast<const bf16x8*>(sv + row * LDK + d8);
        }
    }
}

template <bool DROP, bool MASK>
__global__ void __launch_bounds__(256, 2) attn_bwd_dkdv_kernel(AttnBwdArgs A) {
    ov3d_stamp(A.stamp2, 0);
    attn_bwd_dkdv_body<DROP, MASK>(A);
    ov3d_stamp(A.stamp2, 1);
}

// The whole backward of a short attention (Lq, Lk <= 128, one key split: the decoder's
// 128 x 128 self attention) in ONE launch: a workgroup per (b, h) runs the dQ pass over its
// queries (which also writes D), then, after the barrier that publishes D to the
// workgroup, the dK / dV pass over its keys.  Same arithmetic as the two kernels.
template <bool DROP, bool RAGGED>
__global__ void __launch_bounds__(256, 2) attn_bwd_small_kernel(AttnBwdArgs A) {
    attn_bwd_dq_body<DROP, false, RAGGED>(A);
    __syncthreads();
    attn_bwd_dkdv_body<DROP, false>(A);
}

// The same backward as two workgroups per (b, h) that run side by side: blockIdx.z = 0 the dQ
// pass, 1 the dK / dV pass with its own D (the two passes share no data)
template <bool DROP, bool RAGGED>
__global__ void __launch_bounds__(256, 2) attn_bwd_small2_kernel(AttnBwdArgs A) {
    if (blockIdx.z == 0) attn_bwd_dq_body<DROP, false, RAGGED>(A);
    else attn_bwd_dkdv_body<DROP, false, true>(A);
}

// dK / dV of several attention calls with the same shape in one launch (blockIdx.z = call):
// the decoder's 8 cross attentions, deferred to the end of the decoder backward because
// their K / V gradients only feed the shared memory-K/V projection (transformer._MemoryKV)
constexpr int kDkdvBatchMax = 8;
struct AttnBwdBatch {
    AttnBwdArgs a[kDkdvBatchMax];
};
static_assert(sizeof(AttnBwdBatch) <= 4000, "kernel argument space");

template <bool DROP>
__global__ void __launch_bounds__(256, 2) attn_bwd_dkdv_batch_kernel(AttnBwdBatch g) {
    attn_bwd_dkdv_body<DROP, false>(g.a[blockIdx.z]);
}

// mask (B, Lq, Lk) -> 1-bit words: words [0, W) query-major [nkt][B][Lq][2] (bit n of lane
// (q, h) = key 64 kt + drop_key(n, h)), words [W, 2W) key-major [Lq/32][B][nkt*64] (bit n =
// query 32 qb + n).  KIND 0: uint8 mask, nonzero = not attended; KIND 1: fp32 distances, not
// attended iff d >= thr (MaskedTransformerEncoder.compute_mask).
// Query-major: a thread per (b, q, 64-key tile) reads the tile's 64 contiguous values and
// writes both halves' words; key-major: a thread per (32-query block, b, key) reads one
// column (consecutive threads = consecutive keys: coalesced).
// KIND 0: bool mask; 1: distances, masked iff d >= thr; 2: the squared-distance matrix of
// torch.cdist's matmul form before its clamp_min(0).sqrt() (ATen _euclidean_dist), masked iff
// sqrt(max(g, 0)) >= thr — the same correctly rounded sqrt as torch's, so the same bits as
// packing cdist's output, without the clamp and sqrt passes over the (B, L, L) matrix.
template <int KIND>
__device__ __forceinline__ bool masked_value(float v, float thr) {
    if (KIND == 2) v = sqrtf(fmaxf(v, 0.f));
    return v >= thr;
}

// KIND 3: the distances from the points themselves, src = (B, L, 4) fp32 rows (x, y, z,
// |p|^2) with Lq == Lk == L: the squared distance as cdist's matmul form computes it, one fma
// per term of [-2 p_q, |p_q|^2, 1] . [p_k, 1, |p_k|^2] in that order (the fp32 GEMM's
// accumulation: bit for bit the library result, tools/cdist_probe.py), then KIND 2's clamp and
// sqrt folded into the bound: sqrt(max(g, 0)) >= thr  <=>  g >= g0, g0 the least float whose
// (correctly rounded) sqrt reaches thr, found on the host.  No (B, L, L) distance matrix, no GEMM.
__device__ __forceinline__ float point_sqdist(const float4 pq, const float4 pk) {
    float acc = 0.f;
    acc = fmaf(-2.f * pq.x, pk.x, acc);
    acc = fmaf(-2.f * pq.y, pk.y, acc);
    acc = fmaf(-2.f * pq.z, pk.z, acc);
    acc = fmaf(pq.w, 1.f, acc);
    acc = fmaf(1.f, pk.w, acc);
    return acc;
}

template <int KIND>
__device__ __forceinline__ bool mask_at(const void* src, size_t e, float thr, int Lk = 0) {
    if (KIND == 0) return ((const uint8_t*)src)[e] != 0;
    if (KIND == 3) {
        const size_t bq = e / (size_t)Lk, k = e - bq * (size_t)Lk, b = bq / (size_t)Lk;
        const float4* pts = (const float4*)src;
        return point_sqdist(pts[bq], pts[b * Lk + k]) >= thr;   // thr: the squared-form bound
    }
    return masked_value<KIND>(((const float*)src)[e], thr);
}

template <int KIND>
__global__ void __launch_bounds__(256) attn_mask_pack_kernel(const void* __restrict__ src, float thr,
                                                             int B, int Lq, int Lk, int nkt,
                                                             uint32_t* __restrict__ words) {
    const long long W = (long long)nkt * B * Lq * 2;
    const long long nq = (long long)B * Lq * nkt;   // query-major threads
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < nq) {
        const int kt = (int)(t % nkt);
        const long long bq = t / nkt;
        const int q = (int)(bq % Lq), b = (int)(bq / Lq);
        const size_t row = ((size_t)b * Lq + q) * Lk + 64 * kt;
        uint32_t w0 = 0, w1 = 0;
        const bool full = 64 * kt + 64 <= Lk;
        if (KIND == 3 && full) {   // the query point once, the 64 key points of the tile
            const float4* pts = (const float4*)src;
            const float4 pq = pts[(size_t)b * Lq + q];
            const float4* pk = pts + (size_t)b * Lk + 64 * kt;
#pragma unroll 8
            for (int kk = 0; kk < 64; ++kk) {
                const int rem = kk & 31;
                const int bit = (kk & 1) * 16 + (kk >> 5) * 8 + (rem >> 3) * 2 + ((rem >> 1) & 1);
                const uint32_t m = point_sqdist(pq, pk[kk]) >= thr ? 1u << bit : 0u;
                if ((rem >> 2) & 1) w1 |= m; else w0 |= m;
            }
        } else if (KIND != 0 && KIND != 3 && full && (row & 3) == 0) {
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                const float4 v = *reinterpret_cast<const float4*>((const float*)src + row + 4 * c);
                const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int kk = 4 * c + u;   // key offset in the tile -> (half, bit)
                    const int rem = kk & 31;
                    const int bit = (kk & 1) * 16 + (kk >> 5) * 8 + (rem >> 3) * 2 + ((rem >> 1) & 1);
                    const uint32_t m = masked_value<KIND>(vv[u], thr) ? 1u << bit : 0u;
                    if ((rem >> 2) & 1) w1 |= m; else w0 |= m;
                }
            }
        } else {
            for (int kk = 0; kk < 64 && 64 * kt + kk < Lk; ++kk) {
                const int rem = kk & 31;
                const int bit = (kk & 1) * 16 + (kk >> 5) * 8 + (rem >> 3) * 2 + ((rem >> 1) & 1);
                const uint32_t m = mask_at<KIND>(src, row + kk, thr, Lk) ? 1u << bit : 0u;
                if ((rem >> 2) & 1) w1 |= m; else w0 |= m;
            }
        }
        uint32_t* o = words + (((size_t)kt * B + b) * Lq + q) * 2;
        *reinterpret_cast<uint2*>(o) = make_uint2(w0, w1);
        return;
    }
    const long long u = t - nq;
    if (u >= W) return;
    const int k = (int)(u % ((long long)nkt * 64));
    const long long qb = u / ((long long)nkt * 64);
    const int b = (int)(qb % B), q0 = 32 * (int)(qb / B);
    uint32_t w = 0;
    if (k < Lk) {
        if (KIND == 3) {   // the key point once, the block's 32 query points
            const float4* pts = (const float4*)src;
            const float4 pk = pts[(size_t)b * Lk + k];
#pragma unroll 8
            for (int n = 0; n < 32; ++n)
                if (q0 + n < Lq && point_sqdist(pts[(size_t)b * Lq + q0 + n], pk) >= thr)
                    w |= 1u << n;
        } else {
#pragma unroll 8
            for (int n = 0; n < 32; ++n)
                if (q0 + n < Lq && mask_at<KIND>(src, ((size_t)b * Lq + q0 + n) * Lk + k, thr)) w |= 1u << n;
        }
    }
    words[W + u] = w;
}

// Kind 3 with the points staged in LDS: every query-major word of a (scene, 64-key tile)
// block reads the tile's 64 key points from LDS (broadcast) instead of 1 KB from L2 per
// thread, every key-major word of a (scene, 32-query block) reads the block's 32 query points.
// Blocks [0, nA): query-major, (kt, b, 256-query chunk); blocks [nA, ...): key-major, 256
// consecutive words of one (32-query block, scene) row ((nkt * 64) % 256 == 0).
__global__ void __launch_bounds__(256) attn_mask_points_kernel(const float4* __restrict__ pts,
                                                               float g0, int B, int L, int nkt,
                                                               int nA, uint32_t* __restrict__ words) {
    __shared__ float4 sp[64];
    const int tid = threadIdx.x;
    const int qchunks = (L + 255) / 256;
    if ((int)blockIdx.x < nA) {
        const int blk = blockIdx.x;
        const int qc = blk % qchunks, rest = blk / qchunks;
        const int b = rest % B, kt = rest / B;
        if (tid < 64) {
            const int k = min(64 * kt + tid, L - 1);
            sp[tid] = pts[(size_t)b * L + k];
        }
        __syncthreads();
        const int q = qc * 256 + tid;
        if (q >= L) return;
        const float4 pq = pts[(size_t)b * L + q];
        const int nk = min(64, L - 64 * kt);
        uint32_t w0 = 0, w1 = 0;
#pragma unroll 8
        for (int kk = 0; kk < 64; ++kk) {
            const int rem = kk & 31;
            const int bit = (kk & 1) * 16 + (kk >> 5) * 8 + (rem >> 3) * 2 + ((rem >> 1) & 1);
            const uint32_t m = (kk < nk && point_sqdist(pq, sp[kk]) >= g0) ? 1u << bit : 0u;
            if ((rem >> 2) & 1) w1 |= m; else w0 |= m;
        }
        *reinterpret_cast<uint2*>(words + (((size_t)kt * B + b) * L + q) * 2) = make_uint2(w0, w1);
        return;
    }
    const long long W = (long long)nkt * B * L * 2;
    const long long u = (long long)(blockIdx.x - nA) * 256 + tid;
    const long long row = (long long)nkt * 64;
    const long long qb = ((long long)(blockIdx.x - nA) * 256) / row;   // uniform over the block
    const int b = (int)(qb % B), q0 = 32 * (int)(qb / B);
    if (tid < 32) sp[tid] = pts[(size_t)b * L + min(q0 + tid, L - 1)];
    __syncthreads();
    const int k = (int)(u % row);
    uint32_t w = 0;
    if (k < L) {
        const float4 pk = pts[(size_t)b * L + k];
#pragma unroll 8
        for (int n = 0; n < 32; ++n)
            if (q0 + n < L && point_sqdist(sp[n], pk) >= g0) w |= 1u << n;
    }
    words[W + u] = w;
}

}  // namespace

/* uint32 words of the drop bits ov3d_attn_fwd writes and ov3d_attn_bwd reads (p > 0):
 * query-major [nkt][B*H][Lq][2] followed by key-major [Lq/32][B*H][nkt*64], nkt = ceil(Lk/64) */
extern "C" long long ov3d_attn_dropbits_words(int B, int H, int Lq, int Lk) {
    if (B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || (Lq % QW)) return 0;
    return 4LL * ((Lk + KB - 1) / KB) * B * H * Lq;
}

static void set_dropbits(AttnArgs& a, uint32_t* bits) {
    a.nkt = (a.Lk + KB - 1) / KB;
    a.wq = bits;
    a.wk = bits ? bits + 2 * (size_t)a.nkt * a.B * a.H * a.Lq : nullptr;
}

// one-launch backward of short attentions (attn_bwd_small_kernel); OV3D_ATTN_SMALL_BWD=0 or
// ov3d_attn_small_bwd(0) restores the two launches (A/B measurement, tests)
// the short backward as two side-by-side workgroups per (b, h) (attn_bwd_small2_kernel);
// OV3D_ATTN_SMALL_SPLIT=0: both passes in one workgroup (read per call: tests flip it)
static bool small_bwd_split() {
    const char* e = getenv("OV3D_ATTN_SMALL_SPLIT");
    return !(e && e[0] == '0');
}

static int g_small_bwd = -1;
static bool fuse_small_bwd() {
    if (g_small_bwd < 0) {
        const char* e = getenv("OV3D_ATTN_SMALL_BWD");
        g_small_bwd = (e && e[0] == '0') ? 0 : 1;
    }
    return g_small_bwd != 0;
}

extern "C" int ov3d_attn_small_bwd(int on) {
    const int prev = fuse_small_bwd() ? 1 : 0;
    if (on >= 0) g_small_bwd = on ? 1 : 0;
    return prev;
}

// drop bits from attn_dropgen_kernel for attentions with at least this many (query, key)
// pairs per head (OV3D_ATTN_DROPGEN_MIN overrides; 0 = always, -1 = never)
// Off by default: measured on the encoder (B 8, H 4, L 2048, p 0.1) the pre-pass costs 33.5 us
// and saves the forward 21.6 us (82.4 -> 60.8 us, profiles/r03_dropgen_trace.json): hashing
// beside the MFMAs is cheaper than hashing alone.  OV3D_ATTN_DROPGEN_MIN = the query x key
// count from which the pre-pass runs (0 = always).
constexpr int kDropgenSplit = 4;   // key-tile ranges of attn_dropgen_kernel (grid.z)
static bool dropgen_ahead(int Lq, int Lk) {
    const char* e = getenv("OV3D_ATTN_DROPGEN_MIN");   // read per call: tests flip it
    const long long min_pairs = e ? atoll(e) : -1;
    return min_pairs >= 0 && (long long)Lq * Lk >= min_pairs;
}

static void set_maskbits(AttnArgs& a, const uint32_t* bits) {
    a.mq = bits;
    a.mk = bits ? bits + 2 * (size_t)a.nkt * a.B * a.Lq : nullptr;
}

/* uint32 words of a packed attention mask (ov3d_attn_mask_pack): query-major
 * [nkt][B][Lq][2] followed by key-major [Lq/32][B][nkt*64], nkt = ceil(Lk/64) */
extern "C" long long ov3d_attn_maskbits_words(int B, int Lq, int Lk) {
    if (B <= 0 || Lq <= 0 || Lk <= 0 || (Lq % QW)) return 0;
    return 4LL * ((Lk + KB - 1) / KB) * B * Lq;
}

extern "C" int ov3d_attn_mask_pack(const void* src, int kind, float thr, int B, int Lq, int Lk,
                                   uint32_t* words, void* stream) {
    if (!src || !words || kind < 0 || kind > 3 || B <= 0 || Lq <= 0 || Lk <= 0 || (Lq % QW))
        return OV3D_EINVAL;
    if (kind == 3 && (Lq != Lk || ((uintptr_t)src & 15))) return OV3D_EINVAL;   // self pairs, float4 rows
    const int nkt = (Lk + KB - 1) / KB;
    // threads: B*Lq*nkt query-major (two words each) + W key-major
    const long long n = (long long)B * Lq * nkt + ov3d_attn_maskbits_words(B, Lq, Lk) / 2;
    hipStream_t st = ov3d_stream(stream);
    if (kind == 0)
        attn_mask_pack_kernel<0><<<ov3d_cdiv(n, 256), 256, 0, st>>>(src, thr, B, Lq, Lk, nkt, words);
    else if (kind == 1)
        attn_mask_pack_kernel<1><<<ov3d_cdiv(n, 256), 256, 0, st>>>(src, thr, B, Lq, Lk, nkt, words);
    else if (kind == 2)
        attn_mask_pack_kernel<2><<<ov3d_cdiv(n, 256), 256, 0, st>>>(src, thr, B, Lq, Lk, nkt, words);
    else {
        // the squared-form bound of kind 3: the least g0 with sqrtf(g0) >= thr (sqrtf is
        // monotonic and correctly rounded on host and device), -inf when every key is masked
        float g0 = -INFINITY;
        if (thr > 0.f) {
            g0 = thr * thr;
            while (sqrtf(g0) < thr) g0 = nextafterf(g0, INFINITY);
            while (g0 > 0.f && sqrtf(nextafterf(g0, -INFINITY)) >= thr) g0 = nextafterf(g0, -INFINITY);
        }
        if ((nkt * 64) % 256 == 0) {
            const int nA = nkt * B * ((Lq + 255) / 256);
            const long long nBk = ov3d_attn_maskbits_words(B, Lq, Lk) / 2 / 256;   // key-major words / 256
            attn_mask_points_kernel<<<(unsigned)(nA + nBk), 256, 0, st>>>((const float4*)src, g0, B, Lq,
                                                                        nkt, nA, words);
        } else {
            attn_mask_pack_kernel<3><<<ov3d_cdiv(n, 256), 256, 0, st>>>(src, g0, B, Lq, Lk, nkt, words);
        }
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

// ---- in-kernel launch stamps (bench.py's in-step timing of the roofline kernel).  While armed,
// every forward / dQ / dK-dV launch of Lq * Lk >= min_work takes 2 words per wave of the buffer
// (kernel writes: entry and exit wall clock of each wave, see ov3d_stamp); the host reads the
// launch table back (ov3d_stamps_get) and takes max(exit) - min(entry) per launch.
namespace {
unsigned long long* g_stamp_buf = nullptr;
long long g_stamp_cap = 0, g_stamp_used = 0, g_stamp_min_work = 0;
constexpr int kStampRecs = 256;
int g_stamp_n = 0;
int g_stamp_kind[kStampRecs];
long long g_stamp_off[kStampRecs], g_stamp_waves[kStampRecs], g_stamp_work[kStampRecs];

}  // namespace

unsigned long long* ov3d_stamp_take(int kind, long long work, long long waves) {
    if (!g_stamp_buf || work < g_stamp_min_work || g_stamp_n >= kStampRecs ||
        g_stamp_used + 2 * waves > g_stamp_cap)
        return nullptr;
    g_stamp_kind[g_stamp_n] = kind;
    g_stamp_off[g_stamp_n] = g_stamp_used;
    g_stamp_waves[g_stamp_n] = waves;
    g_stamp_work[g_stamp_n] = work;
    ++g_stamp_n;
    unsigned long long* p = g_stamp_buf + g_stamp_used;
    g_stamp_used += 2 * waves;
    return p;
}

/* kinds: 0 forward, 1 dQ, 2 dK/dV, 3 gemm256 (work = flops).  buf = null disarms (the table stays readable). */
extern "C" int ov3d_stamps_arm(unsigned long long* buf, long long words, long long min_work) {
    g_stamp_buf = buf;
    g_stamp_cap = buf ? words : 0;
    g_stamp_min_work = min_work;
    if (buf) g_stamp_used = g_stamp_n = 0;
    return OV3D_OK;
}
extern "C" int ov3d_stamps_count(void) { return g_stamp_n; }
extern "C" int ov3d_stamps_get(int i, int* kind, long long* word_off, long long* waves,
                               long long* work) {
    if (i < 0 || i >= g_stamp_n || !kind || !word_off || !waves || !work) return OV3D_EINVAL;
    *kind = g_stamp_kind[i];
    *word_off = g_stamp_off[i];
    *waves = g_stamp_waves[i];
    *work = g_stamp_work[i];
    return OV3D_OK;
}
extern "C" long long ov3d_wall_clock_khz(void) {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
        return 0;
    return khz;
}

// pregen: the drop bits of this forward are already in dropbits (ov3d_attn_dropgen, usually
// on another stream ahead of time); the forward reads them instead of hashing
static int attn_fwd_impl(const void* q, const void* k, const void* v, long long sq, long long sk,
                         long long sv, int B, int H, int Lq, int Lk, float scale, float dropout_p,
                         const int64_t* seed, int site, void* o, long long so, float* lse,
                         uint32_t* dropbits, float* workspace, int nsplit, const uint32_t* maskbits,
                         bool pregen, void* stream) {
    if (!q || !k || !v || !o || !lse || B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || (Lq % QW) ||
        nsplit <= 0 || dropout_p < 0.f || dropout_p >= 1.f ||
        (dropout_p > 0.f && (!seed || !dropbits)) || (nsplit > 1 && !workspace))
        return OV3D_EINVAL;
    AttnArgs a;
    a.q = (const bf16*)q;
    a.k = (const bf16*)k;
    a.v = (const bf16*)v;
    a.sq = sq;
    a.sk = sk;
    a.sv = sv;
    a.B = B;
    a.H = H;
    a.Lq = Lq;
    a.Lk = Lk;
    a.scale2 = scale * 1.4426950408889634f;
    a.thresh = dropout_p > 0.f ? (uint32_t)fminf(rintf(dropout_p * 65536.0f), 65535.0f) : 0u;
    a.keep_scale = 1.f / (1.f - dropout_p);
    a.seed = seed;
    a.site = (uint32_t)site;
    a.o = (bf16*)o;
    a.so = so;
    a.lse = lse;
    // keys per split: a multiple of the tile
    int kps = (Lk + nsplit - 1) / nsplit;
    kps = (kps + KB - 1) / KB * KB;
    nsplit = (Lk + kps - 1) / kps;
    a.keys_per_split = kps;
    a.nsplit = nsplit;
    a.part_o = workspace;
    a.part_ml = workspace ? workspace + (size_t)nsplit * B * H * Lq * D : nullptr;
    set_dropbits(a, dropbits);
    set_maskbits(a, maskbits);
    hipStream_t st = ov3d_stream(stream);
    dim3 grid((Lq + 4 * QW - 1) / (4 * QW), B * H, nsplit);
    a.stamp = ov3d_stamp_take(0, (long long)Lq * Lk, (long long)grid.x * grid.y * grid.z * 4);
    // long attentions take their drop bits from a separate VALU pass (attn_dropgen_kernel);
    // short ones (the decoder) hash in the forward, where one more launch would cost more
    const bool bits = a.thresh && (pregen || dropgen_ahead(Lq, Lk));
    if (bits && !pregen) {
        attn_dropgen_kernel<<<dim3(grid.x, grid.y, min(a.nkt, kDropgenSplit)), 256, 0, st>>>(a);
        OV3D_LAUNCH_CHECK();
    }
    if (maskbits) {
        if (bits)
            attn_fwd_kernel<true, true, true><<<grid, 256, 0, st>>>(a);
        else if (a.thresh)
            attn_fwd_kernel<true, true, false><<<grid, 256, 0, st>>>(a);
        else
            attn_fwd_kernel<false, true, false><<<grid, 256, 0, st>>>(a);
    } else if (bits) {
        attn_fwd_kernel<true, false, true><<<grid, 256, 0, st>>>(a);
    } else if (a.thresh) {
        attn_fwd_kernel<true, false, false><<<grid, 256, 0, st>>>(a);
    } else {
        attn_fwd_kernel<false, false, false><<<grid, 256, 0, st>>>(a);
    }
    OV3D_LAUNCH_CHECK();
    if (nsplit > 1) {
        const long long waves = (long long)B * H * Lq;
        const int nb = ov3d_cdiv(waves * 64, 256);
        if (nsplit <= 2) attn_combine_kernel<2><<<nb, 256, 0, st>>>(a);
        else if (nsplit <= 4) attn_combine_kernel<4><<<nb, 256, 0, st>>>(a);
        else if (nsplit <= 8) attn_combine_kernel<8><<<nb, 256, 0, st>>>(a);
        else attn_combine_kernel<kMaxCombine><<<nb, 256, 0, st>>>(a);
        OV3D_LAUNCH_CHECK();
    }
    return OV3D_OK;
}

extern "C" int ov3d_attn_fwd_masked(const void* q, const void* k, const void* v, long long sq,
                                    long long sk, long long sv, int B, int H, int Lq, int Lk,
                                    float scale, float dropout_p, const int64_t* seed, int site,
                                    void* o, long long so, float* lse, uint32_t* dropbits,
                                    float* workspace, int nsplit, const uint32_t* maskbits,
                                    void* stream) {
    return attn_fwd_impl(q, k, v, sq, sk, sv, B, H, Lq, Lk, scale, dropout_p, seed, site, o, so, lse,
                         dropbits, workspace, nsplit, maskbits, false, stream);
}

extern "C" int ov3d_attn_fwd_pregen(const void* q, const void* k, const void* v, long long sq,
                                    long long sk, long long sv, int B, int H, int Lq, int Lk,
                                    float scale, float dropout_p, const int64_t* seed, int site,
                                    void* o, long long so, float* lse, uint32_t* dropbits,
                                    float* workspace, int nsplit, const uint32_t* maskbits,
                                    void* stream) {
    if (!(dropout_p > 0.f)) return OV3D_EINVAL;
    return attn_fwd_impl(q, k, v, sq, sk, sv, B, H, Lq, Lk, scale, dropout_p, seed, site, o, so, lse,
                         dropbits, workspace, nsplit, maskbits, true, stream);
}

extern "C" int ov3d_attn_dropgen(int B, int H, int Lq, int Lk, float dropout_p, const int64_t* seed,
                                 int site, uint32_t* dropbits, void* stream) {
    if (!seed || !dropbits || B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || (Lq % QW) ||
        !(dropout_p > 0.f) || dropout_p >= 1.f)
        return OV3D_EINVAL;
    AttnArgs a{};
    a.B = B;
    a.H = H;
    a.Lq = Lq;
    a.Lk = Lk;
    a.thresh = (uint32_t)fminf(rintf(dropout_p * 65536.0f), 65535.0f);
    a.seed = seed;
    a.site = (uint32_t)site;
    set_dropbits(a, dropbits);
    const dim3 grid((Lq + 4 * QW - 1) / (4 * QW), B * H, min(a.nkt, kDropgenSplit));
    attn_dropgen_kernel<<<grid, 256, 0, ov3d_stream(stream)>>>(a);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_attn_fwd(const void* q, const void* k, const void* v, long long sq,
                             long long sk, long long sv, int B, int H, int Lq, int Lk, float scale,
                             float dropout_p, const int64_t* seed, int site, void* o, long long so,
                             float* lse, uint32_t* dropbits, float* workspace, int nsplit,
                             void* stream) {
    return ov3d_attn_fwd_masked(q, k, v, sq, sk, sv, B, H, Lq, Lk, scale, dropout_p, seed, site, o,
                                so, lse, dropbits, workspace, nsplit, nullptr, stream);
}

#ifdef OV3D_ATTN_PROBE
extern "C" int ov3d_attn_probe_set(unsigned long long* p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_attn_probe), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
#endif

/* workspace floats needed by ov3d_attn_fwd for a given split count */
extern "C" long long ov3d_attn_fwd_workspace(int B, int H, int Lq, int Lk, int nsplit) {
    if (nsplit <= 1) return 0;
    int kps = (Lk + nsplit - 1) / nsplit;
    kps = (kps + KB - 1) / KB * KB;
    nsplit = (Lk + kps - 1) / kps;
    if (nsplit <= 1) return 0;
    return (long long)nsplit * B * H * Lq * (D + 2);
}

extern "C" int ov3d_attn_bwd_masked(const void* q, const void* k, const void* v, long long sq,
                                    long long sk, long long sv, const void* o, long long so,
                                    const void* dout, long long sdo, const float* lse, int B, int H,
                                    int Lq, int Lk, float scale, float dropout_p,
                                    const uint32_t* dropbits, float* dvec, void* dq, long long sdq,
                                    void* dk, long long sdk, void* dv, long long sdv,
                                    float* workspace, int nsplit, const uint32_t* maskbits,
                                    void* stream) {
    if (!q || !k || !v || !o || !dout || !lse || !dvec || !dq || (!dk != !dv) || B <= 0 || H <= 0 ||
        Lq <= 0 || Lk <= 0 || (Lq % QW) || dropout_p < 0.f || dropout_p >= 1.f ||
        (dropout_p > 0.f && !dropbits))
        return OV3D_EINVAL;
    AttnBwdArgs A;
    AttnArgs& a = A.f;
    a.q = (const bf16*)q;
    a.k = (const bf16*)k;
    a.v = (const bf16*)v;
    a.sq = sq;
    a.sk = sk;
    a.sv = sv;
    a.B = B;
    a.H = H;
    a.Lq = Lq;
    a.Lk = Lk;
    a.scale2 = scale * 1.4426950408889634f;
    a.thresh = dropout_p > 0.f ? (uint32_t)fminf(rintf(dropout_p * 65536.0f), 65535.0f) : 0u;
    a.keep_scale = 1.f / (1.f - dropout_p);
    a.seed = nullptr;
    a.site = 0;
    a.so = so;
    a.lse = (float*)lse;
    a.o = nullptr;
    A.o = (const bf16*)o;
    A.dout = (const bf16*)dout;
    A.sdo = sdo;
    A.dvec = dvec;
    A.dq = (bf16*)dq;
    A.dk = (bf16*)dk;
    A.dv = (bf16*)dv;
    A.sdq = sdq;
    A.sdk = sdk;
    A.sdv = sdv;
    A.scale = scale;
    int kps = (Lk + (nsplit > 0 ? nsplit : 1) - 1) / (nsplit > 0 ? nsplit : 1);
    kps = (kps + KB - 1) / KB * KB;
    nsplit = (Lk + kps - 1) / kps;
    if (nsplit > 1 && !workspace) return OV3D_EINVAL;
    a.keys_per_split = kps;
    a.nsplit = nsplit;
    a.part_o = workspace;
    set_dropbits(a, (uint32_t*)dropbits);
    set_maskbits(a, maskbits);
    a.stamp = nullptr;
    A.stamp2 = nullptr;
    hipStream_t st = ov3d_stream(stream);
    if (dk && !maskbits && nsplit == 1 && Lq <= 4 * QW && Lk <= 128 && fuse_small_bwd()) {
        if (small_bwd_split()) {
            const dim3 g2(1, B * H, 2);
            if (Lk % KB)
                (a.thresh ? attn_bwd_small2_kernel<true, true> : attn_bwd_small2_kernel<false, true>)<<<g2, 256, 0, st>>>(A);
            else
                (a.thresh ? attn_bwd_small2_kernel<true, false> : attn_bwd_small2_kernel<false, false>)<<<g2, 256, 0, st>>>(A);
            OV3D_LAUNCH_CHECK();
            return OV3D_OK;
        }
        const dim3 g1(1, B * H);
        if (Lk % KB)
            (a.thresh ? attn_bwd_small_kernel<true, true> : attn_bwd_small_kernel<false, true>)<<<g1, 256, 0, st>>>(A);
        else
            (a.thresh ? attn_bwd_small_kernel<true, false> : attn_bwd_small_kernel<false, false>)<<<g1, 256, 0, st>>>(A);
        OV3D_LAUNCH_CHECK();
        return OV3D_OK;
    }
    const dim3 gq((Lq + 4 * QW - 1) / (4 * QW), B * H, nsplit);
    const bool ragged = Lk % KB != 0;
    a.stamp = ov3d_stamp_take(1, (long long)Lq * Lk, (long long)gq.x * gq.y * gq.z * 4);
    if (maskbits) {
        if (a.thresh)
            (ragged ? attn_bwd_dq_kernel<true, true, true> : attn_bwd_dq_kernel<true, true, false>)<<<gq, 256, 0, st>>>(A);
        else
            (ragged ? attn_bwd_dq_kernel<false, true, true> : attn_bwd_dq_kernel<false, true, false>)<<<gq, 256, 0, st>>>(A);
    } else if (a.thresh) {
        (ragged ? attn_bwd_dq_kernel<true, false, true> : attn_bwd_dq_kernel<true, false, false>)<<<gq, 256, 0, st>>>(A);
    } else {
        (ragged ? attn_bwd_dq_kernel<false, false, true> : attn_bwd_dq_kernel<false, false, false>)<<<gq, 256, 0, st>>>(A);
    }
    OV3D_LAUNCH_CHECK();
    if (nsplit > 1) {
        attn_dq_combine_kernel<<<ov3d_cdiv((long long)B * H * Lq * (D / 4), 256), 256, 0, st>>>(A);
        OV3D_LAUNCH_CHECK();
    }
    if (!dk) return OV3D_OK;   // dQ (and D) only: dK / dV follow in ov3d_attn_bwd_dkdv_batch
    const dim3 gk((Lk + 127) / 128, B * H);
    A.stamp2 = ov3d_stamp_take(2, (long long)Lq * Lk, (long long)gk.x * gk.y * 4);
    if (maskbits) {
        if (a.thresh)
            attn_bwd_dkdv_kernel<true, true><<<gk, 256, 0, st>>>(A);
        else
            attn_bwd_dkdv_kernel<false, true><<<gk, 256, 0, st>>>(A);
    } else if (a.thresh) {
        attn_bwd_dkdv_kernel<true, false><<<gk, 256, 0, st>>>(A);
    } else {
        attn_bwd_dkdv_kernel<false, false><<<gk, 256, 0, st>>>(A);
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_attn_bwd(const void* q, const void* k, const void* v, long long sq,
                             long long sk, long long sv, const void* o, long long so,
                             const void* dout, long long sdo, const float* lse, int B, int H,
                             int Lq, int Lk, float scale, float dropout_p, const uint32_t* dropbits,
                             float* dvec, void* dq, long long sdq, void* dk, long long sdk,
                             void* dv, long long sdv, float* workspace, int nsplit, void* stream) {
    return ov3d_attn_bwd_masked(q, k, v, sq, sk, sv, o, so, dout, sdo, lse, B, H, Lq, Lk, scale,
                                dropout_p, dropbits, dvec, dq, sdq, dk, sdk, dv, sdv, workspace,
                                nsplit, nullptr, stream);
}

extern "C" int ov3d_attn_bwd_dkdv_batch(const ov3d_attn_dkdv_job* jobs, int njobs, int B, int H,
                                        int Lq, int Lk, float scale, float dropout_p, void* stream) {
    if (!jobs || njobs <= 0 || B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || (Lq % QW) ||
        dropout_p < 0.f || dropout_p >= 1.f)
        return OV3D_EINVAL;
    hipStream_t st = ov3d_stream(stream);
    for (int first = 0; first < njobs; first += kDkdvBatchMax) {
        const int n = njobs - first < kDkdvBatchMax ? njobs - first : kDkdvBatchMax;
        AttnBwdBatch g;
        for (int j = 0; j < n; ++j) {
            const ov3d_attn_dkdv_job& J = jobs[first + j];
            if (!J.q || !J.k || !J.v || !J.dout || !J.lse || !J.dvec || !J.dk || !J.dv ||
                (dropout_p > 0.f && !J.dropbits))
                return OV3D_EINVAL;
            AttnBwdArgs& A = g.a[j];
            AttnArgs& a = A.f;
            a.q = (const bf16*)J.q;
            a.k = (const bf16*)J.k;
            a.v = (const bf16*)J.v;
            a.sq = J.sq;
            a.sk = J.sk;
            a.sv = J.sv;
            a.B = B;
            a.H = H;
            a.Lq = Lq;
            a.Lk = Lk;
            a.scale2 = scale * 1.4426950408889634f;
            a.thresh = dropout_p > 0.f ? (uint32_t)fminf(rintf(dropout_p * 65536.0f), 65535.0f) : 0u;
            a.keep_scale = 1.f / (1.f - dropout_p);
            a.seed = nullptr;
            a.site = 0;
            a.o = nullptr;
            a.so = 0;
            a.lse = (float*)J.lse;
            a.part_o = nullptr;
            a.part_ml = nullptr;
            a.nsplit = 1;
            a.keys_per_split = Lk;
            set_dropbits(a, (uint32_t*)J.dropbits);
            set_maskbits(a, nullptr);
            A.o = nullptr;
            A.dout = (const bf16*)J.dout;
            A.sdo = J.sdo;
            A.dvec = (float*)J.dvec;
            A.dq = nullptr;
            A.dk = (bf16*)J.dk;
            A.dv = (bf16*)J.dv;
            A.sdq = 0;
            A.sdk = J.sdk;
            A.sdv = J.sdv;
            A.scale = scale;
            a.stamp = nullptr;
            A.stamp2 = nullptr;
        }
        const dim3 gk((Lk + 127) / 128, B * H, n);
        if (dropout_p > 0.f)
            attn_bwd_dkdv_batch_kernel<true><<<gk, 256, 0, st>>>(g);
        else
            attn_bwd_dkdv_batch_kernel<false><<<gk, 256, 0, st>>>(g);
        OV3D_LAUNCH_CHECK();
    }
    return OV3D_OK;
}
