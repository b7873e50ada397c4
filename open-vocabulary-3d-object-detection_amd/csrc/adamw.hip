// Gradient-norm clipping + AdamW over every parameter tensor of the model in three launches.
//
// Reference: main.py builds torch.optim.AdamW(lr, weight_decay) and engine.py:104-112 runs
// torch.nn.utils.clip_grad_norm_(model.parameters(), clip_gradient) then optimizer.step()
// per iteration.  Here the ~200 parameter tensors are one launch space: a device table
// lists (param, grad, exp_avg, exp_avg_sq, bf16 shadow, numel, lr, weight decay) per
// tensor and every workgroup owns a 4096-element chunk of one tensor.
//
//   1. adamw_norm_kernel     : per-chunk sum of grad^2 (fp64 partials, fixed order)
//   2. adamw_finalize_kernel : total norm, clip coefficient min(1, max_norm/(norm+1e-6))
//                              (clip_grad_norm_), step += 1, bias corrections
//   3. adamw_update_kernel   : g *= clip (written back, as clip_grad_norm_ does), then the
//                              AdamW update of torch.optim.AdamW (decoupled decay):
//        p -= lr*wd*p;  m = lerp(m, g, 1-b1);  v = b2*v + (1-b2)*g*g
//        p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
//      and refreshes the parameter's bf16 copy used by the autocast GEMMs (gemm.py).
// Coalesced fp32 element streams; HBM-bound (28 B per parameter, + 2 B with a shadow).
#include "common.h"

namespace {

typedef __bf16 bf16;
constexpr int kThreads = 256;
constexpr int kPer = 16;                 // elements per thread
constexpr int kChunk = kThreads * kPer;  // elements per workgroup

__global__ void __launch_bounds__(kThreads) adamw_norm_kernel(const ov3d_adamw_tensor* __restrict__ T,
                                                              const int* __restrict__ blk_t,
                                                              const int* __restrict__ blk_c,
                                                              double* __restrict__ partials,
                                                              float grad_scale) {
    const ov3d_adamw_tensor t = T[blk_t[blockIdx.x]];
    const long long base = (long long)blk_c[blockIdx.x] * kChunk;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const long long e = base + j * kThreads + threadIdx.x;
        if (e < t.numel) {
            const float g = t.grad[e] * grad_scale;
            s = fmaf(g, g, s);
        }
    }
    double d = (double)s;
    for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
    __shared__ double red[kThreads / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// coefs: [0] clip multiplier, [1] 1 - b1^t, [2] sqrt(1 - b2^t), [3] total grad norm
// (fp64 like the Python-float bias corrections of torch.optim.AdamW)
__global__ void __launch_bounds__(kThreads) adamw_finalize_kernel(const double* __restrict__ partials,
                                                                  int nblocks, float max_norm,
                                                                  float* step, double beta1,
                                                                  double beta2, double* coefs) {
    double s = 0.0;
    for (int i = threadIdx.x; i < nblocks; i += kThreads) s += partials[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __shared__ double red[kThreads / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x != 0) return;
    const float norm = (float)sqrt((red[0] + red[1]) + (red[2] + red[3]));
    float clip = 1.f;
    if (max_norm > 0.f) clip = fminf(max_norm / (norm + 1e-6f), 1.f);
    const float t = *step + 1.f;
    *step = t;
    coefs[0] = clip;
    coefs[1] = 1.0 - pow(beta1, (double)t);
    coefs[2] = sqrt(1.0 - pow(beta2, (double)t));
    coefs[3] = norm;
}

__global__ void __launch_bounds__(kThreads) adamw_update_kernel(const ov3d_adamw_tensor* __restrict__ T,
                                                                const int* __restrict__ blk_t,
                                                                const int* __restrict__ blk_c,
                                                                const double* __restrict__ coefs,
                                                                float beta2, float omb1, float omb2,
                                                                float eps, int write_grad,
                                                                float grad_scale,
                                                                const double* __restrict__ hyper) {
    const ov3d_adamw_tensor t = T[blk_t[blockIdx.x]];
    const long long base = (long long)blk_c[blockIdx.x] * kChunk;
    const float clip = (float)coefs[0];
    // lr / weight decay of the tensor's group: Python floats (f64) in torch's AdamW
    const double lr = hyper[2 * t.group], wd = hyper[2 * t.group + 1];
    const float step_size = (float)(lr / coefs[1]);
    const float inv_bc2s = 1.f / (float)coefs[2];   // tensor / python float: * fp32 reciprocal
    const float decay = (float)(1.0 - lr * wd);
#pragma unroll 4
    for (int j = 0; j < kPer; ++j) {
        const long long e = base + j * kThreads + threadIdx.x;
        if (e >= t.numel) break;
        float g = t.grad[e] * grad_scale;   // 1/world: the all-reduced sum -> mean (DDP)
        if (clip != 1.f) g *= clip;
        if (write_grad && (clip != 1.f || grad_scale != 1.f)) t.grad[e] = g;
        // torch.optim.AdamW's single-tensor / foreach arithmetic, operation for operation:
        // p.mul_(1 - lr*wd); m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
        // p.addcdiv_(m, v.sqrt() / sqrt(bc2) + eps, -lr/bc1)
        float p = t.param[e] * decay;
        const float m0 = t.exp_avg[e];
        // (single-kernel torch ops contract to FMA: lerp, addcmul, addcdiv)
        const float m = omb1 < 0.5f ? fmaf(omb1, g - m0, m0) : fmaf(-(g - m0), 1.f - omb1, g);
        const float v = fmaf(omb2, g * g, beta2 * t.exp_avg_sq[e]);
        const float denom = sqrtf(v) * inv_bc2s + eps;
        p = fmaf(-step_size, m / denom, p);
        t.param[e] = p;
        t.exp_avg[e] = m;
        t.exp_avg_sq[e] = v;
        if (t.shadow) reinterpret_cast<bf16*>(t.shadow)[e] = (bf16)p;
    }
}

constexpr int kGradsPerLaunch = 256;
struct GradPtrs {
    float* g[kGradsPerLaunch];
};
// table[first + i].grad = p.g[i]: the gradient pointers travel as kernel arguments, so a
// captured step graph carries its own (graph-pool) gradient addresses
__global__ void adamw_set_grads_kernel(ov3d_adamw_tensor* table, int first, int count, GradPtrs p) {
    const int i = threadIdx.x;
    if (i < count) table[first + i].grad = p.g[i];
}

}  // namespace

extern "C" int ov3d_adamw_chunk(void) { return kChunk; }

extern "C" int ov3d_adamw_set_grads(ov3d_adamw_tensor* table, int ntensors, float* const* grads,
                                    void* stream) {
    if (!table || ntensors <= 0 || !grads) return OV3D_EINVAL;
    for (int first = 0; first < ntensors; first += kGradsPerLaunch) {
        const int count = ntensors - first < kGradsPerLaunch ? ntensors - first : kGradsPerLaunch;
        GradPtrs p;
        for (int i = 0; i < kGradsPerLaunch; ++i) p.g[i] = i < count ? grads[first + i] : nullptr;
        adamw_set_grads_kernel<<<1, kGradsPerLaunch, 0, ov3d_stream(stream)>>>(table, first, count, p);
        OV3D_LAUNCH_CHECK();
    }
    return OV3D_OK;
}

extern "C" int ov3d_adamw_step(const ov3d_adamw_tensor* table, const int* blk_t, const int* blk_c,
                               int nblocks, double* partials, float max_norm, float* step,
                               double beta1, double beta2, float eps, double* coefs, int write_grad,
                               float grad_scale, const double* hyper, void* stream) {
    if (!table || !blk_t || !blk_c || nblocks <= 0 || !partials || !step || !coefs || !hyper ||
        beta1 < 0.0 || beta1 >= 1.0 || beta2 < 0.0 || beta2 >= 1.0 || eps < 0.f)
        return OV3D_EINVAL;
    hipStream_t s = ov3d_stream(stream);
    adamw_norm_kernel<<<nblocks, kThreads, 0, s>>>(table, blk_t, blk_c, partials, grad_scale);
    OV3D_LAUNCH_CHECK();
    adamw_finalize_kernel<<<1, kThreads, 0, s>>>(partials, nblocks, max_norm, step, beta1, beta2,
                                                 coefs);
    OV3D_LAUNCH_CHECK();
    // 1 - beta in fp64 first (Python floats in torch), then fp32
    adamw_update_kernel<<<nblocks, kThreads, 0, s>>>(table, blk_t, blk_c, coefs, (float)beta2,
                                                     (float)(1.0 - beta1), (float)(1.0 - beta2), eps,
                                                     write_grad, grad_scale, hyper);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

// ---- several device buffers copied by ONE launch (graphs.StepGraph's static batch) ----
namespace {
constexpr int kCopyMax = 120;   // kernel-argument space (< 4 KB)
struct CopyList {   // static_assert below
    const void* src[kCopyMax];
    void* dst[kCopyMax];
    long long bytes[kCopyMax];
    long long blk[kCopyMax + 1];   // workgroup offsets, 16 B x 256 threads x 4 per workgroup
    int n;
};
static_assert(sizeof(CopyList) <= 4000, "kernel argument space");
__global__ void __launch_bounds__(256) multi_copy_kernel(CopyList c) {
    const long long b = blockIdx.x;
    int i = 0;
    while (i + 1 < c.n && b >= c.blk[i + 1]) ++i;
    const long long base = (b - c.blk[i]) * 256 * 4 * 16;
    const char* s = (const char*)c.src[i];
    char* d = (char*)c.dst[i];
    const long long nb = c.bytes[i];
    const bool vec = ((uintptr_t)s % 16 == 0) && ((uintptr_t)d % 16 == 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const long long o = base + ((long long)u * 256 + threadIdx.x) * 16;
        if (o + 16 <= nb && vec) {
            *reinterpret_cast<uint4*>(d + o) = *reinterpret_cast<const uint4*>(s + o);
        } else {
            for (long long k = o; k < o + 16 && k < nb; ++k) d[k] = s[k];
        }
    }
}
}  // namespace

// the attention / dropout seed of a training forward: live += 1, snapshot = live (one thread)
namespace {
__global__ void seed_next_kernel(long long* live, long long* snap) {
    const long long v = *live + 1;
    *live = v;
    *snap = v;
}
}  // namespace

extern "C" int ov3d_seed_next(long long* live, long long* snap, void* stream) {
    if (!live || !snap) return OV3D_EINVAL;
    seed_next_kernel<<<1, 1, 0, ov3d_stream(stream)>>>(live, snap);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

// the decoder's shared memory rows: sum = bf16(a + b) (fp32 add, one rounding, as torch.add
// into a bf16 output; a fp32 or bf16, b fp32) and ac = bf16(a) for a fp32 (NULL: skipped), 8
// elements a thread (the add was a mixed-type torch launch, the cast another)
namespace {
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
template <bool ABF16>
__global__ void __launch_bounds__(256) add_cast_kernel(const void* __restrict__ a,
                                                       const float* __restrict__ b, long long n8,
                                                       bf16* __restrict__ sum, bf16* __restrict__ ac) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n8) return;
    float av[8];
    if (ABF16) {
        const bf16x8_t a8 = reinterpret_cast<const bf16x8_t*>(a)[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) av[j] = (float)a8[j];
    } else {
        const float4 a0 = reinterpret_cast<const float4*>(a)[2 * i];
        const float4 a1 = reinterpret_cast<const float4*>(a)[2 * i + 1];
        av[0] = a0.x; av[1] = a0.y; av[2] = a0.z; av[3] = a0.w;
        av[4] = a1.x; av[5] = a1.y; av[6] = a1.z; av[7] = a1.w;
    }
    const float4 b0 = reinterpret_cast<const float4*>(b)[2 * i];
    const float4 b1 = reinterpret_cast<const float4*>(b)[2 * i + 1];
    const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    bf16x8_t s8, c8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        s8[j] = (bf16)(av[j] + bv[j]);
        c8[j] = (bf16)av[j];
    }
    reinterpret_cast<bf16x8_t*>(sum)[i] = s8;
    if (!ABF16 && ac) reinterpret_cast<bf16x8_t*>(ac)[i] = c8;
}
}  // namespace

extern "C" int ov3d_add_cast_bf16(const void* a, int a_bf16, const float* b, long long n,
                                  void* sum, void* ac, void* stream) {
    if (n < 0 || (n > 0 && (!a || !b || !sum)) || n % 8 ||
        (((uintptr_t)a | (uintptr_t)b | (uintptr_t)sum | (uintptr_t)ac) % 16))
        return OV3D_EINVAL;
    if (n == 0) return OV3D_OK;
    const unsigned nb = (unsigned)ov3d_cdiv(n / 8, 256);
    if (a_bf16) add_cast_kernel<true><<<nb, 256, 0, ov3d_stream(stream)>>>(a, b, n / 8, (bf16*)sum, nullptr);
    else add_cast_kernel<false><<<nb, 256, 0, ov3d_stream(stream)>>>(a, b, n / 8, (bf16*)sum, (bf16*)ac);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}

extern "C" int ov3d_multi_copy(int n, const void* const* srcs, void* const* dsts,
                               const long long* bytes, void* stream) {
    if (n < 0 || (n > 0 && (!srcs || !dsts || !bytes))) return OV3D_EINVAL;
    for (int first = 0; first < n; first += kCopyMax) {
        CopyList c;
        c.n = n - first < kCopyMax ? n - first : kCopyMax;
        long long blk = 0;
        for (int j = 0; j < c.n; ++j) {
            c.src[j] = srcs[first + j];
            c.dst[j] = dsts[first + j];
            c.bytes[j] = bytes[first + j];
            if (c.bytes[j] < 0 || (c.bytes[j] > 0 && (!c.src[j] || !c.dst[j]))) return OV3D_EINVAL;
            c.blk[j] = blk;
            blk += (c.bytes[j] + 256 * 4 * 16 - 1) / (256 * 4 * 16);
        }
        c.blk[c.n] = blk;
        if (blk == 0) continue;
        multi_copy_kernel<<<(unsigned)blk, 256, 0, ov3d_stream(stream)>>>(c);
        OV3D_LAUNCH_CHECK();
    }
    return OV3D_OK;
}

/* A HIP stream of the caller's own (non-blocking, never handed out by PyTorch's stream pool):
 * graphs.StepGraph / dist.GradBuckets keep the streams that join a graph capture apart from the
 * streams that carry eager collectives (dist.dedicated_stream). */
extern "C" int ov3d_stream_create(void** out) {
    if (!out) return OV3D_EINVAL;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return OV3D_ELAUNCH;
    *out = (void*)s;
    return OV3D_OK;
}
