// Which fp32 arithmetic reproduces torch.cdist's matmul-form squared distances bit for bit
// (ATen _euclidean_dist: [-2x, |x|^2, 1] . [y, 1, |y|^2], a K = 5 fp32 GEMM on hipBLASLt)?
// Measurement only (tools/cdist_probe.py): mode 0 = fma chain over k = 0..4, 1 = two
// v_mfma_f32_16x16x4_f32 (k 0-3, then k 4 with zero padding), 2 = separate mul / add chain.
#include <hip/hip_runtime.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void cdist_probe_kernel(const float* x, const float* xn, int L, int mode, float* out) {
    const int b = blockIdx.z;
    const float* xb = x + (size_t)b * L * 3;
    const float* nb = xn + (size_t)b * L;
    float* ob = out + (size_t)b * L * L;
    const int i0 = blockIdx.y * 16, j0 = blockIdx.x * 16;
    const int lane = threadIdx.x;   // 64 lanes
    if (mode == 1) {
        const int r = lane & 15, kk = lane >> 4;
        const int i = i0 + r, j = j0 + r;
        auto a_at = [&](int k) -> float {
            if (k < 3) return -2.f * xb[i * 3 + k];
            if (k == 3) return nb[i];
            if (k == 4) return 1.f;
            return 0.f;
        };
        auto b_at = [&](int k) -> float {
            if (k < 3) return xb[j * 3 + k];
            if (k == 3) return 1.f;
            if (k == 4) return nb[j];
            return 0.f;
        };
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a_at(kk), b_at(kk), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a_at(4 + kk), b_at(4 + kk), acc, 0, 0, 0);
        // D[i][j]: lane holds column j = lane & 15, rows 4 * (lane >> 4) + v
#pragma unroll
        for (int v = 0; v < 4; ++v) ob[(size_t)(i0 + 4 * kk + v) * L + j0 + r] = acc[v];
        return;
    }
    for (int t = lane; t < 256; t += 64) {
        const int i = i0 + t / 16, j = j0 + t % 16;
        const float a[5] = {-2.f * xb[i * 3], -2.f * xb[i * 3 + 1], -2.f * xb[i * 3 + 2], nb[i], 1.f};
        const float c[5] = {xb[j * 3], xb[j * 3 + 1], xb[j * 3 + 2], 1.f, nb[j]};
        float acc = 0.f;
        if (mode == 0) {
            for (int k = 0; k < 5; ++k) acc = fmaf(a[k], c[k], acc);
        } else {
            for (int k = 0; k < 5; ++k) {
                const float p = a[k] * c[k];
                acc = acc + p;
            }
        }
        ob[(size_t)i * L + j] = acc;
    }
}

extern "C" int cdist_probe(const float* x, const float* xn, int B, int L, int mode, float* out) {
    if (L % 16) return -1;
    cdist_probe_kernel<<<dim3(L / 16, L / 16, B), 64>>>(x, xn, L, mode, out);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
