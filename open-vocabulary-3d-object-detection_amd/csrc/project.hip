// 3D box -> 2D image box projection of the RegionCLIP alignment branch.
// Reference: utils/image_util.py:117-134 project_box_3d_cuda (rotz(-heading), corners with the
// FULL predicted size as half-extent: quirk Q4), :286-298 SUNRGBD_Calibration_cuda
// (Rtilt^T p, flip_axis_to_camera (x, -z, y), K, perspective divide), the [min v, min u,
// max v, max u] order (:131-133) and criterion.py:386-391's clamp to [0, (w, h, w, h)].
// float32 throughout, as the reference (Rtilt / K cast with .float(), image_util.py:276-277).
// One thread per box; rows ordered (.., scene, query): scene = (row / Q) % B, so the L decoder
// layers' boxes stacked as (L*B, Q) go through one launch.
#include "common.h"

namespace {

// torch's min / max reductions propagate NaN: once NaN, stay NaN
__device__ __forceinline__ float nmin(float a, float b) { return (b < a || b != b) && a == a ? b : a; }
__device__ __forceinline__ float nmax(float a, float b) { return (b > a || b != b) && a == a ? b : a; }

__global__ __launch_bounds__(256) void project_box2d_kernel(
    const float* __restrict__ center, const float* __restrict__ size,
    const float* __restrict__ heading, long long n, int Q, int B, const float* __restrict__ Rt,
    const float* __restrict__ Kc, const int64_t* __restrict__ img_h,
    const int64_t* __restrict__ img_w, float* __restrict__ out) {
    const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int b = (int)((r / Q) % B);
    const float cx = center[3 * r], cy = center[3 * r + 1], cz = center[3 * r + 2];
    const float l = size[3 * r], w = size[3 * r + 1], h = size[3 * r + 2];
    const float a = -heading[r];
    const float c = cosf(a), s = sinf(a);
    const float* R = Rt + 9 * b;
    const float* K = Kc + 9 * b;
    float umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        // x_corners [-l,l,l,-l,-l,l,l,-l], y [w,w,-w,-w,w,w,-w,-w], z [h,h,h,h,-h,-h,-h,-h]
        const float x = ((k + 1) & 2) ? l : -l;
        const float y = (k & 2) ? -w : w;
        const float z = (k & 4) ? -h : h;
        const float X = c * x - s * y + cx;
        const float Y = s * x + c * y + cy;
        const float Z = z + cz;
        const float dx = R[0] * X + R[3] * Y + R[6] * Z;   // Rtilt^T p
        const float dy = R[1] * X + R[4] * Y + R[7] * Z;
        const float dz = R[2] * X + R[5] * Y + R[8] * Z;
        const float px = dx, py = -dz, pz = dy;             // flip_axis_to_camera
        const float uu = K[0] * px + K[1] * py + K[2] * pz;
        const float vv = K[3] * px + K[4] * py + K[5] * pz;
        const float ww = K[6] * px + K[7] * py + K[8] * pz;
        const float u = uu / ww, v = vv / ww;
        umin = nmin(umin, u);
        umax = nmax(umax, u);
        vmin = nmin(vmin, v);
        vmax = nmax(vmax, v);
    }
    const float wf = (float)img_w[b], hf = (float)img_h[b];
    const float box[4] = {vmin, umin, vmax, umax};
    const float lim[4] = {wf, hf, wf, hf};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float v = box[i] < 0.f ? 0.f : box[i];       // clamp_min(0), NaN kept
        v = v > lim[i] ? lim[i] : v;                 // minimum(., [w, h, w, h]), NaN kept
        out[4 * r + i] = v;
    }
}

}  // namespace

extern "C" int ov3d_project_box2d(const float* center, const float* size, const float* heading,
                                  long long n, int Q, int B, const float* Rtilt, const float* K,
                                  const int64_t* img_h, const int64_t* img_w, float* out,
                                  void* stream) {
    if (n < 0 || Q <= 0 || B <= 0 || (n > 0 && (!center || !size || !heading || !Rtilt || !K ||
                                                 !img_h || !img_w || !out)))
        return OV3D_EINVAL;
    if (n == 0) return OV3D_OK;
    hipLaunchKernelGGL(project_box2d_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       ov3d_stream(stream), center, size, heading, n, Q, B, Rtilt, K, img_h, img_w,
                       out);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
