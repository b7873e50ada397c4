// Output projection + residual + dropout + LayerNorm of a pre-norm transformer sub-layer in ONE
// launch (forward).  Reference: models/transformer.py — every attention sub-layer ends with
// `out_proj(attn)` (nn.MultiheadAttention, 223 / 307-308) and the FFN with `linear2(...)`
// (275-277 / 375-377), then `x = x + dropout(branch)` and the next sub-layer's `norm(x)`
// (forward_pre 262-280 / 355-379; the decoder's final norm of every layer output, 124-133).
// The unfused path is rows_gemm (y = bf16(x W^T + b)) followed by resnorm_fwd (resnorm.hip);
// here a workgroup owns 16 whole 256-wide rows, computes their y on the matrix cores and runs
// the resnorm epilogue on them: y never reaches HBM and one launch (~5 us on the decoder's
// 1024-row blocks: latency-bound) goes away per sub-layer.
//
//   y   = bf16(x W^T + b)                   x (R, K) bf16 rows, W (256, K) bf16, b bf16
//   s   = src + dropout(y)                   dropout(y) = bf16(y / (1-p)) where kept (rowdrop.h)
//   xa  = bf16(LN_a(s)), xap = bf16(LN_a(s) + pos), xb = LN_b(s)     (as resnorm_fwd)
//
// Layout on the matrix cores: 4 waves, wave w owns output columns 64w .. 64w+63 as four
// 16x16 tiles; the product is computed transposed (W rows as the A operand, x rows as B), so
// lane l holds row r0 + (l & 15) and FOUR consecutive columns of each tile: 16-byte row loads
// / stores of s, src and the norm operands.  Every load (x, W, bias, src, pos, norm weights)
// is issued before the first MFMA: the launch is one memory round trip plus the row
// reductions (two shuffles and an LDS exchange across the 4 waves, two-pass variance as
// resnorm_fwd).
#include "common.h"
#include "rowdrop.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int C = 256;      // the model width (enc_dim = dec_dim = 256)
constexpr int RB = 16;      // rows per workgroup
constexpr int KMAX = 256;

struct LinResArgs {
    long long R;
    int K;
    const bf16* x; long long ldx;
    const bf16* w; long long ldw;
    const bf16* bias;
    const void* src; int src_bf16;
    const void* pos; int pos_bf16;
    uint32_t thresh; float keep_scale; const int64_t* seed; uint32_t site;
    const float *ga, *ba, *gb, *bb;
    float eps;
    float* s; float* mean; float* rstd;
    bf16* xa; bf16* xap; void* xb; int xb_bf16;
    long long xb_inner, xb_s0, xb_s1;
};

__device__ __forceinline__ f32x4 ld4(const void* p, int is_bf16, long long off) {
    if (is_bf16) {
        const bf16x4 v = *reinterpret_cast<const bf16x4*>((const bf16*)p + off);
        return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
    }
    return *reinterpret_cast<const f32x4*>((const float*)p + off);
}
__device__ __forceinline__ void st4h(bf16* p, long long off, f32x4 v) {
    *reinterpret_cast<bf16x4*>(p + off) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}

template <int NK>   // K / 32
__global__ void __launch_bounds__(256) linres_fwd_kernel(LinResArgs a) {
    __shared__ float red[2][4][RB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const long long r0 = (long long)blockIdx.x * RB;
    const long long r = r0 + fr;
    const bool live = r < a.R;
    const long long rc = live ? r : a.R - 1;   // clamped row: computed, never stored

    // ---- every load first
    bf16x8 xf[NK], wf[4][NK];
#pragma unroll
    for (int s = 0; s < NK; ++s)
        xf[s] = *reinterpret_cast<const bf16x8*>(a.x + rc * a.ldx + 32 * s + 8 * fq);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int s = 0; s < NK; ++s)
            wf[j][s] = *reinterpret_cast<const bf16x8*>(a.w + (long long)(64 * wave + 16 * j + fr) * a.ldw + 32 * s + 8 * fq);
    f32x4 bias[4], sv[4], ga[4], ba[4], gb[4], bb[4], pv[4];
    const bool na = a.xa || a.xap;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = 64 * wave + 16 * j + 4 * fq;
        const long long off = rc * C + c;
        bias[j] = a.bias ? ld4(a.bias, 1, c) : f32x4{0.f, 0.f, 0.f, 0.f};
        sv[j] = a.src ? ld4(a.src, a.src_bf16, off) : f32x4{0.f, 0.f, 0.f, 0.f};
        if (na) {
            ga[j] = *reinterpret_cast<const f32x4*>(a.ga + c);
            ba[j] = *reinterpret_cast<const f32x4*>(a.ba + c);
        }
        if (a.xap) pv[j] = ld4(a.pos, a.pos_bf16, off);
        if (a.xb) {
            gb[j] = *reinterpret_cast<const f32x4*>(a.gb + c);
            bb[j] = *reinterpret_cast<const f32x4*>(a.bb + c);
        }
    }

    // ---- y^T tiles: acc[j] lane l = y[r][64 wave + 16 j + 4 fq + e]
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NK; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][s], xf[s], acc[j], 0, 0, 0);

    // ---- s = src + dropout(bf16(y + b))
    const uint32_t rb = a.thresh ? rowdrop::row_base(rowdrop::seed_mix(a.seed, a.site), rc) : 0u;
    float part = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = 64 * wave + 16 * j + 4 * fq;
        bool keep[4] = {true, true, true, true};
        if (a.thresh) {
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
                const uint32_t h = rowdrop::mix24(rb + (uint32_t)((c + e) >> 1) * 0x27D4EB2Fu);
                keep[e] = (h & 0xffffu) >= a.thresh;
                keep[e + 1] = (h >> 16) >= a.thresh;
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float y = (float)(bf16)(acc[j][e] + bias[j][e]);
            const float d = a.thresh ? (float)(bf16)(y * a.keep_scale) : y;
            sv[j][e] += keep[e] ? d : 0.f;
            part += sv[j][e];
        }
        if (live) *reinterpret_cast<f32x4*>(a.s + r * C + c) = sv[j];
    }
    if (!a.xa && !a.xap && !a.xb) return;
    // ---- row statistics: the row's 256 values are 16 per lane over lanes fr, fr+16, +32, +48
    // of the 4 waves
    part += __shfl_xor(part, 16);
    part += __shfl_xor(part, 32);
    if (fq == 0) red[0][wave][fr] = part;
    __syncthreads();
    const float mu = (red[0][0][fr] + red[0][1][fr] + red[0][2][fr] + red[0][3][fr]) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) q += (sv[j][e] - mu) * (sv[j][e] - mu);
    q += __shfl_xor(q, 16);
    q += __shfl_xor(q, 32);
    if (fq == 0) red[1][wave][fr] = q;
    __syncthreads();
    const float rs = rsqrtf((red[1][0][fr] + red[1][1][fr] + red[1][2][fr] + red[1][3][fr]) / (float)C + a.eps);
    if (!live) return;
    if (wave == 0 && fq == 0) {
        a.mean[r] = mu;
        a.rstd[r] = rs;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = 64 * wave + 16 * j + 4 * fq;
        const long long off = r * C + c;
        f32x4 xh;
#pragma unroll
        for (int e = 0; e < 4; ++e) xh[e] = (sv[j][e] - mu) * rs;
        if (na) {
            f32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = xh[e] * ga[j][e] + ba[j][e];
            if (a.xa) st4h(a.xa, off, o);
            if (a.xap) {
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] += pv[j][e];
                st4h(a.xap, off, o);
            }
        }
        if (a.xb) {
            f32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = xh[e] * gb[j][e] + bb[j][e];
            const long long ob = a.xb_inner ? (r / a.xb_inner) * a.xb_s0 + (r % a.xb_inner) * a.xb_s1 + c : off;
            if (a.xb_bf16) st4h((bf16*)a.xb, ob, o);
            else *reinterpret_cast<f32x4*>((float*)a.xb + ob) = o;
        }
    }
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int ov3d_linres_supported(int Cout, int K) {
    return Cout == C && K > 0 && K % 32 == 0 && K <= KMAX;
}

extern "C" int ov3d_linres_fwd(long long R, int K, const void* x, long long ldx, const void* w,
                               long long ldw, const void* bias, const void* src, int src_bf16,
                               float dropout_p, const int64_t* seed, int site, const float* ga,
                               const float* ba, const void* pos, int pos_bf16, const float* gb,
                               const float* bb, float eps, float* s, float* mean, float* rstd,
                               void* xa, void* xap, void* xb, int xb_bf16, long long xb_inner,
                               long long xb_s0, long long xb_s1, void* stream) {
    if (!ov3d_linres_supported(C, K) || R <= 0 || !x || !w || !s || ldx < K || ldw < K ||
        ldx % 8 || ldw % 8 || !al16(x) || !al16(w) || !al16(s) || dropout_p < 0.f ||
        dropout_p >= 1.f || (dropout_p > 0.f && !seed))
        return OV3D_EINVAL;
    if (bias && ((uintptr_t)bias & 7)) return OV3D_EINVAL;
    if (src && !al16(src)) return OV3D_EINVAL;
    if ((xa || xap) && (!ga || !ba)) return OV3D_EINVAL;
    if (xap && !pos) return OV3D_EINVAL;
    if (xb && (!gb || !bb)) return OV3D_EINVAL;
    if ((xa || xap || xb) && (!mean || !rstd)) return OV3D_EINVAL;
    if (xb_inner < 0 || (xb_inner > 0 && (xb_s0 < C || xb_s1 < C))) return OV3D_EINVAL;
    LinResArgs a{R, K, (const bf16*)x, ldx, (const bf16*)w, ldw, (const bf16*)bias, src, src_bf16,
                 pos, pos_bf16, rowdrop::thresh(dropout_p), 1.f / (1.f - dropout_p), seed,
                 (uint32_t)site, ga, ba, gb, bb, eps, s, mean, rstd, (bf16*)xa, (bf16*)xap, xb,
                 xb_bf16, xb_inner, xb_s0, xb_s1};
    const unsigned grid = (unsigned)((R + RB - 1) / RB);
    hipStream_t st = ov3d_stream(stream);
    switch (K / 32) {
        case 1: linres_fwd_kernel<1><<<grid, 256, 0, st>>>(a); break;
        case 2: linres_fwd_kernel<2><<<grid, 256, 0, st>>>(a); break;
        case 3: linres_fwd_kernel<3><<<grid, 256, 0, st>>>(a); break;
        case 4: linres_fwd_kernel<4><<<grid, 256, 0, st>>>(a); break;
        case 5: linres_fwd_kernel<5><<<grid, 256, 0, st>>>(a); break;
        case 6: linres_fwd_kernel<6><<<grid, 256, 0, st>>>(a); break;
        case 7: linres_fwd_kernel<7><<<grid, 256, 0, st>>>(a); break;
        default: linres_fwd_kernel<8><<<grid, 256, 0, st>>>(a); break;
    }
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
