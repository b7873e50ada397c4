// Hungarian matching (linear sum assignment) for the set criterion, on the device.
//
// The reference matcher copies the (B, Q, G) cost to the host and calls
// scipy.optimize.linear_sum_assignment per scene (criterion.py:65-86): a device
// sync in the middle of every training step plus L*B = 64 serial solves.  Here
// each problem is one wave64 workgroup running scipy 1.15's algorithm
// (Crouse's shortest augmenting path, rectangular_lsap.cpp) with identical
// float64 arithmetic and tie rule, so assignments equal scipy's bit for bit:
//   * tall problems are transposed so rows <= columns (Q queries vs n GT boxes:
//     rows = GT, columns = queries);
//   * per row, a Dijkstra search over the remaining columns; path costs
//     r = ((minVal + c) - u[i]) - v[j] in double;
//   * the remaining-column list starts in descending column order and shrinks
//     by swap-with-last; the picked column is the LAST unassigned minimum in
//     list order if there is one, else the FIRST minimum.  That order is kept
//     explicitly (rem / pos arrays in LDS) and the pick is a wave-wide
//     lexicographic min of (path cost, key(pos, assigned)).
// Columns are spread over the 64 lanes (j = lane + 64 t); the per-step serial
// bookkeeping (list removal, augmentation walk) is done by lane 0.
#include <climits>

#include "common.h"

namespace {

constexpr int kMaxDim = 1024;

__device__ __forceinline__ void lex_min(double& m, int& k, double om, int ok) {
    if (om < m || (om == m && ok < k)) {
        m = om;
        k = ok;
    }
}

// one DPP step of the wave reduction: combine with the (value, key) of the lane that dpp_ctrl
// names; a lane whose source is outside its row (or whose row is masked off) keeps its own
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void lex_dpp(double& m, int& k) {
    const long long mb = __double_as_longlong(m);
    const int lo = (int)mb, hi = (int)(mb >> 32);
    const int olo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROW_MASK, 0xf, false);
    const int ohi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROW_MASK, 0xf, false);
    const int ok = __builtin_amdgcn_update_dpp(k, k, CTRL, ROW_MASK, 0xf, false);
    lex_min(m, k, __longlong_as_double(((long long)ohi << 32) | (unsigned)olo), ok);
}

// (value, key) lexicographic minimum over the 64 lanes, returned to every lane: row_shr 1/2/4/8
// leave each row's minimum in its lane 15, row_bcast 15/31 carry it into lane 63, one readlane
// broadcasts it (a total order with unique keys: the same result as any reduction order, i.e.
// as the xor-shuffle tree this replaces, without its LDS-routed permutes)
__device__ __forceinline__ void wave_lex_min(double& m, int& k) {
    lex_dpp<0x111, 0xf>(m, k);   // row_shr:1
    lex_dpp<0x112, 0xf>(m, k);   // row_shr:2
    lex_dpp<0x114, 0xf>(m, k);   // row_shr:4
    lex_dpp<0x118, 0xf>(m, k);   // row_shr:8
    lex_dpp<0x142, 0xa>(m, k);   // row_bcast:15 into rows 1, 3
    lex_dpp<0x143, 0xc>(m, k);   // row_bcast:31 into rows 2, 3
    const long long mb = __double_as_longlong(m);
    const int lo = __builtin_amdgcn_readlane((int)mb, 63);
    const int hi = __builtin_amdgcn_readlane((int)(mb >> 32), 63);
    k = __builtin_amdgcn_readlane(k, 63);
    m = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// STAGED: the problem's Q x n costs are copied to LDS in the solver's (row, column) order while
// the NaN screen reads them, so every augmenting step reads its row from LDS (consecutive lanes,
// consecutive columns) instead of a strided row of the global matrix at L2 latency.
template <bool STAGED>
__global__ __launch_bounds__(64) void hungarian_kernel(const float* __restrict__ cost,
                                                       const int32_t* __restrict__ nactual, int Q,
                                                       int G, int64_t* __restrict__ gt_inds,
                                                       float* __restrict__ matched,
                                                       int32_t* __restrict__ status) {
    extern __shared__ double smem[];
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    const double INF = __builtin_huge_val();
    int n = nactual[p];
    n = n < 0 ? 0 : (n > G ? G : n);
    const float* C = cost + (size_t)p * Q * G;
    int64_t* out_i = gt_inds + (size_t)p * Q;
    float* out_m = matched + (size_t)p * Q;

    const bool tr = n < Q;                 // rows = GT boxes, columns = queries
    const int nr = tr ? n : Q, nc = tr ? Q : n;
    const int NC = Q > G ? Q : G, NR = Q < G ? Q : G;   // LDS capacity (host-sized)
    double* v = smem;
    double* spc = v + NC;
    double* u = spc + NC;
    int* path = reinterpret_cast<int*>(u + NR);
    int* row4col = path + NC;
    int* rem = row4col + NC;
    int* pos = rem + NC;
    int* col4row = pos + NC;
    unsigned char* SC = reinterpret_cast<unsigned char*>(col4row + NR);
    unsigned char* SR = SC + NC;
    float* Cs = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(SR + NR) + 3) &
                                         ~(uintptr_t)3);   // STAGED: nr x nc costs

    // scipy rejects NaN and -inf entries (ValueError) before solving
    int bad = 0;
    for (int e = lane; e < Q * n; e += 64) {
        const int q = e / n, g = e - q * n;
        const float c = C[(size_t)q * G + g];
        bad |= (c != c) || (c == -__builtin_huge_valf());
        if (STAGED) Cs[tr ? g * nc + q : q * nc + g] = c;
    }
    const bool invalid = __ballot(bad) != 0ull;
    if (n == 0 || invalid) {
        for (int q = lane; q < Q; q += 64) {
            out_i[q] = 0;
            out_m[q] = 0.f;
        }
        if (status && lane == 0) status[p] = invalid ? -1 : 0;
        return;
    }

    for (int j = lane; j < nc; j += 64) {
        v[j] = 0.0;
        row4col[j] = -1;
        path[j] = -1;
    }
    for (int r = lane; r < nr; r += 64) {
        u[r] = 0.0;
        col4row[r] = -1;
    }
    __syncthreads();

    int rc = 0;
    for (int cur = 0; cur < nr; ++cur) {
        for (int j = lane; j < nc; j += 64) {
            spc[j] = INF;
            SC[j] = 0;
            pos[j] = nc - 1 - j;
            rem[nc - 1 - j] = j;
        }
        for (int r = lane; r < nr; r += 64) SR[r] = 0;
        __syncthreads();
        double minv = 0.0;
        int nrem = nc, i = cur, sink = -1;
        while (sink < 0) {
            if (lane == 0) SR[i] = 1;
            const double ui = u[i];
            double bm = INF;
            int bk = INT_MAX;
            for (int j = lane; j < nc; j += 64) {
                if (SC[j]) continue;
                const double c = STAGED ? (double)Cs[i * nc + j]
                                 : tr ? (double)C[(size_t)j * G + i] : (double)C[(size_t)i * G + j];
                const double r = minv + c - ui - v[j];
                double s = spc[j];
                if (r < s) {
                    path[j] = i;
                    spc[j] = r;
                    s = r;
                }
                // list-order key: unassigned columns first, the later (larger pos) the better;
                // then assigned columns, the earlier the better
                const int k = row4col[j] < 0 ? (nc - 1 - pos[j]) : (nc + pos[j]);
                lex_min(bm, bk, s, k);
            }
            wave_lex_min(bm, bk);
            minv = bm;
            if (!(bm < INF)) {
                rc = -2;
                break;
            }
            const int ps = bk < nc ? (nc - 1 - bk) : (bk - nc);
            const int j = rem[ps];
            const int rj = row4col[j];
            __syncthreads();
            if (lane == 0) {
                SC[j] = 1;
                const int last = rem[nrem - 1];
                rem[ps] = last;
                pos[last] = ps;
            }
            --nrem;
            if (rj < 0)
                sink = j;
            else
                i = rj;
            __syncthreads();
        }
        if (rc) break;
        // dual update (u[cur] += minVal; other visited rows and visited columns)
        for (int r = lane; r < nr; r += 64) {
            if (r == cur)
                u[r] += minv;
            else if (SR[r])
                u[r] += minv - spc[col4row[r]];
        }
        for (int j = lane; j < nc; j += 64)
            if (SC[j]) v[j] -= minv - spc[j];
        __syncthreads();
        if (lane == 0) {
            for (int j = sink;;) {
                const int r = path[j];
                row4col[j] = r;
                const int nj = col4row[r];
                col4row[r] = j;
                j = nj;
                if (r == cur) break;
            }
        }
        __syncthreads();
    }

    for (int q = lane; q < Q; q += 64) {
        int g = -1;
        if (rc == 0) g = tr ? row4col[q] : col4row[q];
        out_i[q] = g < 0 ? 0 : g;
        out_m[q] = g < 0 ? 0.f : 1.f;
    }
    if (status && lane == 0) status[p] = rc;
}

}  // namespace

extern "C" int ov3d_hungarian(const float* cost, const int32_t* nactual, int P, int Q, int G,
                              int64_t* gt_inds, float* matched, int32_t* status, void* stream) {
    if (P < 0 || Q < 0 || G < 0 || Q > kMaxDim || G > kMaxDim) return OV3D_EINVAL;
    if (P == 0 || Q == 0) return OV3D_OK;
    if (!cost || !nactual || !gt_inds || !matched) return OV3D_EINVAL;
    const int NC = Q > G ? Q : G, NR = Q < G ? Q : G;
    const size_t lds = (size_t)(2 * NC + NR) * sizeof(double) + (size_t)(4 * NC + NR) * sizeof(int) +
                       (size_t)(NC + NR) + 3;
    const size_t staged = lds + (size_t)Q * G * sizeof(float);
    if (staged <= (64u << 10))
        hipLaunchKernelGGL(hungarian_kernel<true>, dim3(P), dim3(64), staged, ov3d_stream(stream),
                           cost, nactual, Q, G, gt_inds, matched, status);
    else
        hipLaunchKernelGGL(hungarian_kernel<false>, dim3(P), dim3(64), lds, ov3d_stream(stream),
                           cost, nactual, Q, G, gt_inds, matched, status);
    OV3D_LAUNCH_CHECK();
    return OV3D_OK;
}
