// Library GEMM with the bottleneck close in its epilogue, for the RegionCLIP ModifiedResNet's
// conv3: y = act(x W^T + bias + residual) as ONE hipBLASLt matmul —
// out-of-place C (the identity rows) and D (the block output), bias + ReLU epilogue — where
// torch's addmm would first copy the identity into its output and the bias add and ReLU
// would be two more passes over the rows.  Host code only: the matrix work is hipBLASLt's
// (a plain library GEMM, MI355X_MICROARCH.md), this file only plans and issues it.
//
// Row-major (M, N) rows are hipBLASLt's column-major (N, M): D^T = W · X^T with A = W
// (column-major K x N, op T), B = X (column-major K x M), C / D column-major N x M; the bias
// runs along D's rows, i.e. the output channels.  Plans (descriptors + the heuristic's
// algorithm) are cached per (device, shape, strides, act); the bias pointer is set per call
// under the cache lock.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

namespace {

struct LtPlan {
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
    hipblasLtMatmulAlgo_t algo{};
    size_t ws = 0;
};

using LtKey = std::tuple<int, long long, long long, long long, long long, long long, long long,
                         long long, int, long long>;

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<LtKey, LtPlan> g_plans;

bool make_plan(hipblasLtHandle_t h, long long M, long long N, long long K, long long ldx, long long ldw,
               long long ldr, long long ldo, int relu, long long ws_bytes, LtPlan* p) {
    const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    const hipblasLtEpilogue_t epi = relu ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS;
    const int32_t bias_type = HIP_R_16BF;
    if (hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS)
        return false;
    if (hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)) ||
        hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)) ||
        hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)) ||
        hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bias_type,
                                        sizeof(bias_type)))
        return false;
    if (hipblasLtMatrixLayoutCreate(&p->a, HIP_R_16BF, K, N, ldw) ||
        hipblasLtMatrixLayoutCreate(&p->b, HIP_R_16BF, K, M, ldx) ||
        hipblasLtMatrixLayoutCreate(&p->c, HIP_R_16BF, N, M, ldr) ||
        hipblasLtMatrixLayoutCreate(&p->d, HIP_R_16BF, N, M, ldo))
        return false;
    hipblasLtMatmulPreference_t pref = nullptr;
    if (hipblasLtMatmulPreferenceCreate(&pref)) return false;
    const uint64_t wmax = (uint64_t)ws_bytes;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wmax,
                                          sizeof(wmax));
    hipblasLtMatmulHeuristicResult_t res[1];
    int n = 0;
    const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, p->desc, p->a, p->b, p->c, p->d,
                                                               pref, 1, res, &n);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (st != HIPBLAS_STATUS_SUCCESS || n < 1) return false;
    p->algo = res[0].algo;
    p->ws = res[0].workspaceSize;
    return true;
}

}  // namespace

extern "C" int ov3d_lt_gemm_bias_residual(long long M, int N, int K, const void* x, long long ldx,
                                          const void* w, long long ldw, const void* bias,
                                          const void* residual, long long ldr, int relu, void* out,
                                          long long ldo, void* workspace, long long ws_bytes,
                                          void* stream) {
    if (!x || !w || !bias || !residual || !out || M < 0 || N <= 0 || K <= 0 || ldx < K || ldw < K ||
        ldr < N || ldo < N || ws_bytes < 0 || (ws_bytes > 0 && !workspace) ||
        ((uintptr_t)workspace & 15))
        return OV3D_EINVAL;
    if (M == 0) return OV3D_OK;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return OV3D_ELAUNCH;
    std::lock_guard<std::mutex> lock(g_mu);
    hipblasLtHandle_t& h = g_handles[dev];
    if (!h && hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) {
        h = nullptr;
        return OV3D_ELAUNCH;
    }
    const LtKey key{dev, M, (long long)N, (long long)K, ldx, ldw, ldr, ldo, relu, ws_bytes};
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
        LtPlan p;
        if (!make_plan(h, M, N, K, ldx, ldw, ldr, ldo, relu, ws_bytes, &p)) return OV3D_ELAUNCH;
        it = g_plans.emplace(key, p).first;
    }
    LtPlan& p = it->second;
    if ((long long)p.ws > ws_bytes) return OV3D_EINVAL;
    if (hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias,
                                        sizeof(bias)))
        return OV3D_ELAUNCH;
    const float alpha = 1.f, beta = 1.f;
    const hipblasStatus_t st = hipblasLtMatmul(h, p.desc, &alpha, w, p.a, x, p.b, &beta, residual, p.c,
                                               out, p.d, &p.algo, workspace, p.ws, ov3d_stream(stream));
    return st == HIPBLAS_STATUS_SUCCESS ? OV3D_OK : OV3D_ELAUNCH;
}
