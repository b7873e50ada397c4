/*
 * ov3d_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference hot-path kernels, used as the parity
 * checker for the HIP library (libov3d_hip.so) and as the "port" CPU
 * baseline in bench.py.  Nothing in the product package links or calls this
 * file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load it.
 *
 * Floating-point contract: compiled with -O2 -ffp-contract=off; every
 * fused multiply-add that the HIP kernels use is written here as an explicit
 * fmaf(), so the two implementations round identically (bit-exact indices,
 * bit-exact GIoU/NMS arithmetic).
 *
 * Sources restated (file:line under the reference tree):
 *   FPS / ball query / grouping : un-vendored third_party/pointnet2 (imported at
 *       models/model_3detr.py:8-9); semantics from SURVEY.md Appendix A.1-A.3.
 *       PARITY UNPINNED by the reference (no sources, no fixtures): the tie
 *       rule below emulates the upstream 512-thread tree reduction exactly.
 *   GIoU  : utils/box_util.py:624-714 (Cython dispatch) + utils/box_intersection.pyx:
 *       13-70 (polygon_clip_unnest, double precision Python floats), 166-198
 *       (box_intersection, K2 = rect2.shape[2] bug), and utils/box_util.py:517-618
 *       (TorchScript path, float32, all K2).
 *   NMS   : utils/nms.py:79-162 (nms_3d_faster / nms_3d_faster_samecls).
 *   gather: un-vendored pointnet2 gather_operation (model_3detr.py:174-186, 355-361).
 *   2D projection: utils/image_util.py:117-134, 286-298 + criterion.py:386-391.
 *   SA MLP + max-pool: upstream SharedMLP / PointnetSAModuleVotes (model_3detr.py:353-362),
 *       float64 (a tolerance checker of the bf16 path, not bit-exact).
 * The §8(b) boundary's entry points have twins here with the suffix _cpu and no stream argument:
 * fps, ball_query, group (+ bwd), gather (+ bwd), sa_mlp (+ bwd), giou3d, nms3d, project_box2d,
 * roi_align (and lsap for the matcher).  Not twinned: the GIoU backward (checked against the
 * reference's own autograd through tests/golden/giou.npz instead).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ FPS */

/* Largest power of two <= n, capped at 512 — upstream opt_n_threads(). */
static int fps_block_size(int n) {
    int bs = 1;
    while (bs * 2 <= n && bs < 512) bs *= 2;
    return bs;
}

static uint32_t bitrev(uint32_t v, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; ++i) r |= ((v >> i) & 1u) << (bits - 1 - i);
    return r;
}

/* Tie-break rank of point k: the upstream kernel gives point k to thread
 * t = k mod bs (strict '>' inside a thread keeps the lowest k), then reduces
 * over threads with a halving tree that keeps the lower slot on ties.  The
 * winner among equal maxima is the thread with the smallest bit-reversed id,
 * then the smallest k.  rank(k) orders exactly that way; smaller wins. */
uint32_t ov3d_fps_rank_cpu(int k, int n) {
    int bs = fps_block_size(n);
    int bits = 0;
    while ((1 << bits) < bs) ++bits;
    uint32_t t = (uint32_t)(k & (bs - 1));
    uint32_t i = (uint32_t)(k >> bits);
    return (bitrev(t, bits) << 23) | i;
}

int ov3d_fps_cpu(const float* xyz, int B, int N, int M, int32_t* idx_out) {
    if (B < 0 || N <= 0 || M < 0) return -1;
    float* temp = (float*)malloc(sizeof(float) * (size_t)N);
    uint32_t* rank = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)N);
    unsigned char* skip = (unsigned char*)malloc((size_t)N);
    if (!temp || !rank || !skip) { free(temp); free(rank); free(skip); return -2; }
    for (int k = 0; k < N; ++k) rank[k] = ov3d_fps_rank_cpu(k, N);
    for (int b = 0; b < B; ++b) {
        const float* p = xyz + (size_t)b * N * 3;
        int32_t* idx = idx_out + (size_t)b * M;
        for (int k = 0; k < N; ++k) {
            temp[k] = 1e10f;
            float x = p[3 * k], y = p[3 * k + 1], z = p[3 * k + 2];
            float mag = fmaf(z, z, fmaf(y, y, x * x));
            skip[k] = ((double)mag <= 1e-3);   /* float vs double literal */
        }
        if (M == 0) continue;
        int old = 0;
        idx[0] = 0;
        for (int j = 1; j < M; ++j) {
            float x1 = p[3 * old], y1 = p[3 * old + 1], z1 = p[3 * old + 2];
            uint64_t best = 0; /* key 0 == "no candidate" -> index 0 */
            int besti = 0;
            for (int k = 0; k < N; ++k) {
                if (skip[k]) continue;
                float dx = p[3 * k] - x1, dy = p[3 * k + 1] - y1, dz = p[3 * k + 2] - z1;
                float d = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                float d2 = fminf(d, temp[k]);
                temp[k] = d2;
                uint32_t bits;
                memcpy(&bits, &d2, 4);
                uint64_t key = ((uint64_t)bits << 32) | (uint64_t)(~rank[k]);
                if (key > best) { best = key; besti = k; }
            }
            old = besti;
            idx[j] = old;
        }
    }
    free(temp); free(rank); free(skip);
    return 0;
}

/* ------------------------------------------------------------ ball query */

int ov3d_ball_query_cpu(const float* xyz, const float* new_xyz, int B, int N, int M,
                        float radius, int S, int32_t* idx_out) {
    if (B < 0 || N < 0 || M < 0 || S <= 0) return -1;
    const float r2 = radius * radius;
    for (int b = 0; b < B; ++b) {
        const float* p = xyz + (size_t)b * N * 3;
        for (int j = 0; j < M; ++j) {
            const float* c = new_xyz + ((size_t)b * M + j) * 3;
            int32_t* idx = idx_out + ((size_t)b * M + j) * S;
            for (int l = 0; l < S; ++l) idx[l] = 0;
            int cnt = 0;
            for (int k = 0; k < N && cnt < S; ++k) {
                float dx = c[0] - p[3 * k], dy = c[1] - p[3 * k + 1], dz = c[2] - p[3 * k + 2];
                float d2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                if (d2 < r2) {
                    if (cnt == 0)
                        for (int l = 0; l < S; ++l) idx[l] = k;
                    idx[cnt++] = k;
                }
            }
        }
    }
    return 0;
}

/* features (B,C,N), idx (B,M,S) -> out (B,C,M,S) */
int ov3d_group_cpu(const float* feats, const int32_t* idx, int B, int C, int N, int M, int S,
                   float* out) {
    for (int b = 0; b < B; ++b)
        for (int c = 0; c < C; ++c)
            for (int j = 0; j < M; ++j)
                for (int s = 0; s < S; ++s) {
                    int k = idx[((size_t)b * M + j) * S + s];
                    out[(((size_t)b * C + c) * M + j) * S + s] =
                        (k >= 0 && k < N) ? feats[((size_t)b * C + c) * N + k] : 0.f;
                }
    return 0;
}

/* its backward (grouping_operation's, the interim SA's input gradient): grad_out (B,C,M,S) ->
 * grad_features (B,C,N), zero-filled, added in (j, s) order.  Twin of ov3d_group_bwd (equal
 * up to float summation order where a point has several (centroid, slot) hits). */
int ov3d_group_bwd_cpu(const float* grad_out, const int32_t* idx, int B, int C, int N, int M,
                       int S, float* grad_feats) {
    if (B < 0 || C < 0 || N < 0 || M < 0 || S < 0) return -1;
    memset(grad_feats, 0, sizeof(float) * (size_t)B * C * N);
    for (int b = 0; b < B; ++b)
        for (int c = 0; c < C; ++c)
            for (int j = 0; j < M; ++j)
                for (int s = 0; s < S; ++s) {
                    int k = idx[((size_t)b * M + j) * S + s];
                    if (k >= 0 && k < N)
                        grad_feats[((size_t)b * C + c) * N + k] +=
                            grad_out[(((size_t)b * C + c) * M + j) * S + s];
                }
    return 0;
}

/* ------------------------------------------------------------------ GIoU */

typedef struct { double x, y; } pt_d;
typedef struct { float x, y; } pt_f;

/* Sutherland–Hodgman in double, as the Cython polygon_clip_unnest evaluates it
 * (untyped Python floats: box_intersection.pyx:13-23, 27-70). */
static int clip_double(const pt_d* subj, int ns, const pt_d* clip, int nc, pt_d* out) {
    pt_d in[16], cur[16];
    int nout = ns;
    for (int i = 0; i < ns; ++i) cur[i] = subj[i];
    pt_d cp1 = clip[nc - 1];
    for (int ci = 0; ci < nc; ++ci) {
        pt_d cp2 = clip[ci];
        int nin = nout;
        for (int i = 0; i < nin; ++i) in[i] = cur[i];
        nout = 0;
        if (nin == 0) break;
        pt_d s = in[nin - 1];
        for (int ii = 0; ii < nin; ++ii) {
            pt_d e = in[ii];
            int e_in = (cp2.x - cp1.x) * (e.y - cp1.y) > (cp2.y - cp1.y) * (e.x - cp1.x);
            int s_in = (cp2.x - cp1.x) * (s.y - cp1.y) > (cp2.y - cp1.y) * (s.x - cp1.x);
            if (e_in || s_in) {
                if (e_in != s_in) {
                    double dc0 = cp1.x - cp2.x, dc1 = cp1.y - cp2.y;
                    double dp0 = s.x - e.x, dp1 = s.y - e.y;
                    double n1 = cp1.x * cp2.y - cp1.y * cp2.x;
                    double n2 = s.x * e.y - s.y * e.x;
                    double n3 = 1.0 / (dc0 * dp1 - dc1 * dp0);
                    pt_d q = {(n1 * dp0 - n2 * dc0) * n3, (n1 * dp1 - n2 * dc1) * n3};
                    if (nout < 16) cur[nout++] = q;
                }
                if (e_in && nout < 16) cur[nout++] = e;
            }
            s = e;
        }
        cp1 = cp2;
        if (nout == 0) break;
    }
    for (int i = 0; i < nout; ++i) out[i] = cur[i];
    return nout;
}

/* Same algorithm on float32 scalars: the TorchScript path (box_util.py:387-440)
 * evaluates every step as a float32 0-d tensor op. */
static int clip_float(const pt_f* subj, int ns, const pt_f* clip, int nc, pt_f* out) {
    pt_f in[16], cur[16];
    int nout = ns;
    for (int i = 0; i < ns; ++i) cur[i] = subj[i];
    pt_f cp1 = clip[nc - 1];
    for (int ci = 0; ci < nc; ++ci) {
        pt_f cp2 = clip[ci];
        int nin = nout;
        for (int i = 0; i < nin; ++i) in[i] = cur[i];
        nout = 0;
        if (nin == 0) break;
        pt_f s = in[nin - 1];
        for (int ii = 0; ii < nin; ++ii) {
            pt_f e = in[ii];
            int e_in = (cp2.x - cp1.x) * (e.y - cp1.y) > (cp2.y - cp1.y) * (e.x - cp1.x);
            int s_in = (cp2.x - cp1.x) * (s.y - cp1.y) > (cp2.y - cp1.y) * (s.x - cp1.x);
            if (e_in || s_in) {
                if (e_in != s_in) {
                    float dc0 = cp1.x - cp2.x, dc1 = cp1.y - cp2.y;
                    float dp0 = s.x - e.x, dp1 = s.y - e.y;
                    float n1 = cp1.x * cp2.y - cp1.y * cp2.x;
                    float n2 = s.x * e.y - s.y * e.x;
                    float n3 = 1.0f / (dc0 * dp1 - dc1 * dp0);
                    pt_f q = {(n1 * dp0 - n2 * dc0) * n3, (n1 * dp1 - n2 * dc1) * n3};
                    if (nout < 16) cur[nout++] = q;
                }
                if (e_in && nout < 16) cur[nout++] = e;
            }
            s = e;
        }
        cp1 = cp2;
        if (nout == 0) break;
    }
    for (int i = 0; i < nout; ++i) out[i] = cur[i];
    return nout;
}

/* 0.5*|dot(xs, roll(ys,1)) - dot(ys, roll(xs,1))| with float accumulation */
static float shoelace_f(const float* xs, const float* ys, int n) {
    float s1 = 0.f, s2 = 0.f;
    for (int i = 0; i < n; ++i) {
        int im = (i + n - 1) % n;
        s1 = s1 + xs[i] * ys[im];
        s2 = s2 + ys[i] * xs[im];
    }
    return 0.5f * fabsf(s1 - s2);
}

/* rect[i] = (corner[3-i].x, corner[3-i].z): box_util.py:656-661 */
static void rect_of(const float* c, float* rx, float* rz) {
    for (int i = 0; i < 4; ++i) { rx[i] = c[(3 - i) * 3 + 0]; rz[i] = c[(3 - i) * 3 + 2]; }
}

static float box_vol(const float* c) { /* box3d_vol_tensor, box_util.py:443-463 */
    const float EPS = 1e-6f;
    float d[3];
    float a, b, cc;
    for (int i = 0; i < 3; ++i) d[i] = c[0 * 3 + i] - c[1 * 3 + i];
    a = sqrtf(fmaxf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2], EPS));
    for (int i = 0; i < 3; ++i) d[i] = c[1 * 3 + i] - c[2 * 3 + i];
    b = sqrtf(fmaxf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2], EPS));
    for (int i = 0; i < 3; ++i) d[i] = c[0 * 3 + i] - c[4 * 3 + i];
    cc = sqrtf(fmaxf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2], EPS));
    return a * b * cc;
}

/* mode 0: Cython path (double clip, K2 < min(4,nums) bug when cython_k2_bug);
 * mode 1: TorchScript path (float clip, all k2 < nums). */
int ov3d_giou3d_cpu(const float* corners1, const float* corners2, const int32_t* nums,
                    int B, int K1, int K2, int mode, int rotated, int cython_k2_bug,
                    float* out) {
    const float EPS = 1e-8f;
    for (int b = 0; b < B; ++b) {
        int nk = nums ? nums[b] : K2;
        for (int k1 = 0; k1 < K1; ++k1) {
            const float* c1 = corners1 + (((size_t)b * K1 + k1) * 8) * 3;
            float r1x[4], r1z[4];
            rect_of(c1, r1x, r1z);
            float v1 = fmaxf(box_vol(c1), EPS);
            float mn1[3], mx1[3];
            for (int a = 0; a < 3; ++a) { mn1[a] = INFINITY; mx1[a] = -INFINITY; }
            for (int v = 0; v < 8; ++v)
                for (int a = 0; a < 3; ++a) {
                    float val = c1[v * 3 + a];
                    if (a == 1) val = -val;
                    if (val < mn1[a]) mn1[a] = val;
                    if (val > mx1[a]) mx1[a] = val;
                }
            for (int k2 = 0; k2 < K2; ++k2) {
                const float* c2 = corners2 + (((size_t)b * K2 + k2) * 8) * 3;
                float* o = out + ((size_t)b * K1 + k1) * K2 + k2;
                /* height on -Y */
                float ymax = fminf(c1[0 * 3 + 1], c2[0 * 3 + 1]);
                float ymin = fmaxf(c1[4 * 3 + 1], c2[4 * 3 + 1]);
                float height = fmaxf(ymax - ymin, 0.f);
                float r2x[4], r2z[4];
                rect_of(c2, r2x, r2z);
                float ltx = fmaxf(r1x[1], r2x[1]), ltz = fmaxf(r1z[1], r2z[1]);
                float rbx = fminf(r1x[3], r2x[3]), rbz = fminf(r1z[3], r2z[3]);
                float whx = fmaxf(rbx - ltx, 0.f), whz = fmaxf(rbz - ltz, 0.f);
                float non_rot = whx * whz;
                if (k2 >= nk) non_rot = 0.f;
                /* enclosing box (Y flipped), box_util.py:466-514 */
                float mn2[3], mx2[3];
                for (int a = 0; a < 3; ++a) { mn2[a] = INFINITY; mx2[a] = -INFINITY; }
                for (int v = 0; v < 8; ++v)
                    for (int a = 0; a < 3; ++a) {
                        float val = c2[v * 3 + a];
                        if (a == 1) val = -val;
                        if (val < mn2[a]) mn2[a] = val;
                        if (val > mx2[a]) mx2[a] = val;
                    }
                float al_xmin = fminf(mn1[0], mn2[0]);
                float al_ymin = fmaxf(mx1[1], mx2[1]);
                float al_zmin = fminf(mn1[2], mn2[2]);
                float al_xmax = fmaxf(mx1[0], mx2[0]);
                float al_ymax = fminf(mn1[1], mn2[1]);
                float al_zmax = fmaxf(mx1[2], mx2[2]);
                float enc = fabsf(al_xmax - al_xmin) * fabsf(al_ymax - al_ymin) * fabsf(al_zmax - al_zmin);
                float v2 = fmaxf(box_vol(c2), EPS);
                float sum_vols = v1 + v2;
                float good = (enc > 2e-8f && sum_vols > 4e-8f) ? 1.f : 0.f;

                float inter_area;
                if (rotated) {
                    inter_area = 0.f;
                    int limit = nk;
                    if (mode == 0 && cython_k2_bug && limit > 4) limit = 4; /* K2 = rect2.shape[2] */
                    if (k2 < limit && non_rot != 0.f) {
                        if (mode == 0) {
                            pt_d s[4], c[4], res[16];
                            for (int i = 0; i < 4; ++i) {
                                s[i].x = r1x[i]; s[i].y = r1z[i];
                                c[i].x = r2x[i]; c[i].y = r2z[i];
                            }
                            int n = clip_double(s, 4, c, 4, res);
                            if (n > 0) {
                                float xs[16], ys[16];
                                for (int i = 0; i < n; ++i) { xs[i] = (float)res[i].x; ys[i] = (float)res[i].y; }
                                inter_area = shoelace_f(xs, ys, n);
                            }
                        } else {
                            pt_f s[4], c[4], res[16];
                            for (int i = 0; i < 4; ++i) {
                                s[i].x = r1x[i]; s[i].y = r1z[i];
                                c[i].x = r2x[i]; c[i].y = r2z[i];
                            }
                            int n = clip_float(s, 4, c, 4, res);
                            if (n > 0) {
                                float xs[16], ys[16];
                                for (int i = 0; i < n; ++i) { xs[i] = res[i].x; ys[i] = res[i].y; }
                                inter_area = shoelace_f(xs, ys, n);
                            }
                        }
                    }
                } else {
                    inter_area = non_rot;
                }
                float inter_vol = inter_area * height;
                float uni = fmaxf(sum_vols - inter_vol, EPS);
                float iou = inter_vol / uni;
                float second = -(1.f - uni / enc);
                float g = (iou + second) * good;
                if (k2 >= nk) g = g * 0.f;
                *o = g;
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------- NMS */

static double np_max(double a, double b) { return (isnan(a) || isnan(b)) ? NAN : (a > b ? a : b); }
static double np_min(double a, double b) { return (isnan(a) || isnan(b)) ? NAN : (a < b ? a : b); }

static const double* g_scores;
static int g_stride;
static int cmp_desc(const void* pa, const void* pb) {
    int a = *(const int*)pa, b = *(const int*)pb;
    double sa = g_scores[(size_t)a * g_stride + 6], sb = g_scores[(size_t)b * g_stride + 6];
    if (sa > sb) return -1;
    if (sa < sb) return 1;
    return (a > b) ? -1 : (a < b ? 1 : 0); /* ties: larger index first (stable argsort) */
}

/* boxes (K, stride) float64 [x1,y1,z1,x2,y2,z2,score(,cls)]; returns #picks,
 * pick_out[0..n) in pick order, keep_out[K] (0/1) if non-null. */
int ov3d_nms3d_cpu(const double* boxes, int K, int stride, double thr, int old_type, int samecls,
                   int32_t* pick_out, uint8_t* keep_out) {
    if (K < 0 || stride < 7 || (samecls && stride < 8)) return -1;
    int* order = (int*)malloc(sizeof(int) * (size_t)(K > 0 ? K : 1));
    unsigned char* sup = (unsigned char*)calloc((size_t)(K > 0 ? K : 1), 1);
    double* area = (double*)malloc(sizeof(double) * (size_t)(K > 0 ? K : 1));
    for (int i = 0; i < K; ++i) {
        const double* p = boxes + (size_t)i * stride;
        order[i] = i;
        area[i] = (p[3] - p[0]) * (p[4] - p[1]) * (p[5] - p[2]);
    }
    g_scores = boxes; g_stride = stride;
    qsort(order, (size_t)K, sizeof(int), cmp_desc);
    int n = 0;
    if (keep_out) memset(keep_out, 0, (size_t)K);
    for (int pi = 0; pi < K; ++pi) {
        int i = order[pi];
        if (sup[i]) continue;
        pick_out[n++] = i;
        if (keep_out) keep_out[i] = 1;
        const double* a = boxes + (size_t)i * stride;
        for (int qi = pi + 1; qi < K; ++qi) {
            int j = order[qi];
            if (sup[j]) continue;
            const double* c = boxes + (size_t)j * stride;
            double xx1 = np_max(a[0], c[0]), yy1 = np_max(a[1], c[1]), zz1 = np_max(a[2], c[2]);
            double xx2 = np_min(a[3], c[3]), yy2 = np_min(a[4], c[4]), zz2 = np_min(a[5], c[5]);
            double l = np_max(0.0, xx2 - xx1), w = np_max(0.0, yy2 - yy1), h = np_max(0.0, zz2 - zz1);
            double o;
            if (old_type) {
                o = (l * w * h) / area[j];
            } else {
                double inter = l * w * h;
                o = inter / (area[i] + area[j] - inter);
            }
            if (samecls) o = o * (double)(a[7] == c[7]);
            if (o > thr) sup[j] = 1;
        }
    }
    free(order); free(sup); free(area);
    return n;
}

/* ----------------------------------------------------- Hungarian (LSAP) */
/* Restates scipy.optimize.linear_sum_assignment (scipy 1.15.3, the version in
 * this image; the reference calls it at criterion.py:79 on final_cost[b, :, :n],
 * a float32 (Q, n) slice converted to float64).  scipy's algorithm is Crouse's
 * shortest-augmenting-path LSAP (rectangular_lsap.cpp): a tall matrix is
 * transposed so rows <= cols; one Dijkstra search per row over the remaining
 * columns, kept in a list initialised in DESCENDING column order and shrunk by
 * swap-with-last removal; the next column is the first minimum of the path
 * costs in list order, replaced by a later equal-cost column whenever that one
 * is unassigned (so: the LAST unassigned minimum if any, else the FIRST
 * minimum).  Path costs r = ((minVal + c) - u[i]) - v[j] in double.
 * Tie behaviour therefore matches scipy exactly.
 *
 * cost: element (q, g) at cost[q*ld + g], q < nq, g < ng.
 * Output: gt_of_q[q] = matched g or -1 for all q < nq.  Returns 0, or -1 for
 * NaN / -inf entries (scipy raises ValueError), -2 if infeasible.          */
int ov3d_lsap_cpu(const float* cost, int nq, int ng, int ld, int32_t* gt_of_q) {
    for (int q = 0; q < nq; q++) gt_of_q[q] = -1;
    if (nq == 0 || ng == 0) return 0;
    for (int q = 0; q < nq; q++)
        for (int g = 0; g < ng; g++) {
            double c = cost[(size_t)q * ld + g];
            if (c != c || c == -INFINITY) return -1;
        }
    const int tr = ng < nq;             /* rows = gts, cols = queries */
    const int nr = tr ? ng : nq, nc = tr ? nq : ng;
#define COST(i, j) ((double)(tr ? cost[(size_t)(j) * ld + (i)] : cost[(size_t)(i) * ld + (j)]))
    double* u = calloc(nr, sizeof(double));
    double* v = calloc(nc, sizeof(double));
    double* spc = malloc(nc * sizeof(double));
    int* path = malloc(nc * sizeof(int));
    int* col4row = malloc(nr * sizeof(int));
    int* row4col = malloc(nc * sizeof(int));
    char* SR = malloc(nr);
    char* SC = malloc(nc);
    int* rem = malloc(nc * sizeof(int));
    int rc = 0;
    for (int i = 0; i < nr; i++) col4row[i] = -1;
    for (int j = 0; j < nc; j++) { row4col[j] = -1; path[j] = -1; }
    for (int cur = 0; cur < nr && rc == 0; cur++) {
        double minv = 0;
        int nrem = nc;
        for (int t = 0; t < nc; t++) rem[t] = nc - 1 - t;
        memset(SR, 0, nr);
        memset(SC, 0, nc);
        for (int j = 0; j < nc; j++) spc[j] = INFINITY;
        int i = cur, sink = -1;
        while (sink < 0) {
            int best = -1;
            double lo = INFINITY;
            SR[i] = 1;
            for (int t = 0; t < nrem; t++) {
                int j = rem[t];
                double r = minv + COST(i, j) - u[i] - v[j];
                if (r < spc[j]) { path[j] = i; spc[j] = r; }
                if (spc[j] < lo || (spc[j] == lo && row4col[j] < 0)) { lo = spc[j]; best = t; }
            }
            minv = lo;
            if (minv == INFINITY) { rc = -2; break; }
            int j = rem[best];
            if (row4col[j] < 0) sink = j; else i = row4col[j];
            SC[j] = 1;
            rem[best] = rem[--nrem];
        }
        if (rc) break;
        u[cur] += minv;
        for (int r = 0; r < nr; r++)
            if (SR[r] && r != cur) u[r] += minv - spc[col4row[r]];
        for (int j = 0; j < nc; j++)
            if (SC[j]) v[j] -= minv - spc[j];
        for (int j = sink;;) {
            int r = path[j];
            row4col[j] = r;
            int nj = col4row[r];
            col4row[r] = j;
            j = nj;
            if (r == cur) break;
        }
    }
#undef COST
    if (rc == 0) {
        for (int r = 0; r < nr; r++) {
            if (tr) gt_of_q[col4row[r]] = r;
            else gt_of_q[r] = col4row[r];
        }
    }
    free(u); free(v); free(spc); free(path); free(col4row); free(row4col); free(SR); free(SC); free(rem);
    return rc;
}

/* ------------------------------------------------------------- ROIAlign */
/* ROIAlignV2 of the RegionCLIP ROI heads [upstream: detectron2 ROIPooler ->
 * torchvision roi_align_forward_kernel_impl, aligned=True], reached from
 * clip.inference at criterion.py:397.  PARITY UNPINNED by the reference
 * (RegionCLIP / detectron2 / torchvision are not vendored); this restates the
 * published kernel operation by operation in float:
 *   start = box * scale - 0.5; size = end - start; bin = size / P;
 *   grid = sampling_ratio > 0 ? sampling_ratio : ceil(size / P);
 *   y = start_h + ph*bin_h + (iy + .5) * bin_h / grid_h  (x likewise)
 *   bilinear: zero outside [-1, H] x [-1, W], clamp to 0, edge rows/cols
 *   collapse; val = w1*v1 + w2*v2 + w3*v3 + w4*v4; out = sum / max(gh*gw, 1).
 * Layout: feat (N,H,W,C) channels-last, boxes (R,4), roi r reads image
 * (r / per_image) % nimages, out (R,P,P,C). */
static float roi_bilinear(const float* f, int H, int W, int C, float y, float x) {
    if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) return 0.f;
    if (y <= 0) y = 0;
    if (x <= 0) x = 0;
    int yl = (int)y, xl = (int)x, yh, xh;
    if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
    if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
    float ly = y - (float)yl, lx = x - (float)xl, hy = 1.f - ly, hx = 1.f - lx;
    float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
    float v1 = f[((size_t)yl * W + xl) * C], v2 = f[((size_t)yl * W + xh) * C];
    float v3 = f[((size_t)yh * W + xl) * C], v4 = f[((size_t)yh * W + xh) * C];
    return w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4;
}

int ov3d_roi_align_cpu(const float* feat, int N, int H, int W, int C, const float* boxes, int R,
                       int per_image, int nimages, float scale, int P, int sampling_ratio,
                       int aligned, float* out) {
    if (per_image <= 0 || nimages <= 0 || nimages > N) return -1;
    const float off = aligned ? 0.5f : 0.f;
    for (int r = 0; r < R; r++) {
        const float* bx = boxes + 4 * (size_t)r;
        const float* f = feat + (size_t)((r / per_image) % nimages) * H * W * C;
        float sw = bx[0] * scale - off, sh = bx[1] * scale - off;
        float ew = bx[2] * scale - off, eh = bx[3] * scale - off;
        float rw = ew - sw, rh = eh - sh;
        if (!aligned) { rw = rw > 1.f ? rw : 1.f; rh = rh > 1.f ? rh : 1.f; }
        float bh = rh / (float)P, bw = rw / (float)P;
        int gh = sampling_ratio > 0 ? sampling_ratio : (int)ceilf(rh / (float)P);
        int gw = sampling_ratio > 0 ? sampling_ratio : (int)ceilf(rw / (float)P);
        float count = (float)(gh * gw > 1 ? gh * gw : 1);
        for (int ph = 0; ph < P; ph++)
            for (int pw = 0; pw < P; pw++)
                for (int c = 0; c < C; c++) {
                    float acc = 0.f;
                    for (int iy = 0; iy < gh; iy++) {
                        float y = sh + (float)ph * bh + (float)(iy + .5f) * bh / (float)gh;
                        for (int ix = 0; ix < gw; ix++) {
                            float x = sw + (float)pw * bw + (float)(ix + .5f) * bw / (float)gw;
                            acc += roi_bilinear(f + c, H, W, C, y, x);
                        }
                    }
                    out[(((size_t)r * P + ph) * P + pw) * C + c] = acc / count;
                }
    }
    return 0;
}

/* ------------------------------------------------------- gather (pointnet2 gather_operation) */

/* gather_operation [upstream pointnet2, called at models/model_3detr.py:355-361 through the SA
 * module and :174-186 for the query points]: features (B,C,N), idx (B,M) -> out (B,C,M); an
 * index outside [0, N) reads 0 (the HIP kernel's guard).  Twin of ov3d_gather_fwd. */
int ov3d_gather_fwd_cpu(const float* feats, const int32_t* idx, int B, int C, int N, int M,
                        float* out) {
    if (B < 0 || C < 0 || N < 0 || M < 0) return -1;
    for (int b = 0; b < B; ++b)
        for (int c = 0; c < C; ++c)
            for (int j = 0; j < M; ++j) {
                int k = idx[(size_t)b * M + j];
                out[((size_t)b * C + c) * M + j] =
                    (k >= 0 && k < N) ? feats[((size_t)b * C + c) * N + k] : 0.f;
            }
    return 0;
}

/* its backward: grad_out (B,C,M) -> grad_features (B,C,N), zero-filled, then added in index
 * order j = 0..M-1 (the upstream kernel's atomicAdd has no fixed order: equal to the HIP
 * result whenever the indices of a scene are distinct, as FPS indices are).  Twin of
 * ov3d_gather_bwd. */
int ov3d_gather_bwd_cpu(const float* grad_out, const int32_t* idx, int B, int C, int N, int M,
                        float* grad_feats) {
    if (B < 0 || C < 0 || N < 0 || M < 0) return -1;
    memset(grad_feats, 0, sizeof(float) * (size_t)B * C * N);
    for (int b = 0; b < B; ++b)
        for (int c = 0; c < C; ++c)
            for (int j = 0; j < M; ++j) {
                int k = idx[(size_t)b * M + j];
                if (k >= 0 && k < N)
                    grad_feats[((size_t)b * C + c) * N + k] += grad_out[((size_t)b * C + c) * M + j];
            }
    return 0;
}

/* ------------------------------------------------------------- 2D projection (a14) */

/* NaN-propagating min / max (torch's min / max reductions: once NaN, stay NaN) */
static float nmin_f(float a, float b) { return ((b < a || b != b) && a == a) ? b : a; }
static float nmax_f(float a, float b) { return ((b > a || b != b) && a == a) ? b : a; }

/* 3D box -> clamped 2D image box of the RegionCLIP alignment branch: utils/image_util.py:117-134
 * (project_box_3d_cuda: rotz(-heading), corners with the FULL size as half-extent, quirk Q4),
 * :286-298 (SUNRGBD_Calibration_cuda: Rtilt^T p, flip_axis_to_camera (x, -z, y), K, divide),
 * :131-133 ([min v, min u, max v, max u]) and criterion.py:386-391 (clamp to [0, (w,h,w,h)]).
 * float32 arithmetic in the reference's order.  Rows ordered (.., scene, query): scene of row r
 * = (r / Q) % B.  Twin of ov3d_project_box2d (the HIP kernel evaluates the same expressions;
 * cosf / sinf are libm's here, ocml's there: equal to ~1 ulp). */
int ov3d_project_box2d_cpu(const float* center, const float* size, const float* heading,
                           long long n, int Q, int B, const float* Rt, const float* Kc,
                           const int64_t* img_h, const int64_t* img_w, float* out) {
    if (n < 0 || Q <= 0 || B <= 0) return -1;
    for (long long r = 0; r < n; ++r) {
        const int b = (int)((r / Q) % B);
        const float cx = center[3 * r], cy = center[3 * r + 1], cz = center[3 * r + 2];
        const float l = size[3 * r], w = size[3 * r + 1], h = size[3 * r + 2];
        const float a = -heading[r];
        const float c = cosf(a), s = sinf(a);
        const float* R = Rt + 9 * b;
        const float* K = Kc + 9 * b;
        float umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY;
        for (int k = 0; k < 8; ++k) {
            /* x [-l,l,l,-l,-l,l,l,-l], y [w,w,-w,-w,w,w,-w,-w], z [h,h,h,h,-h,-h,-h,-h] */
            const float x = ((k + 1) & 2) ? l : -l;
            const float y = (k & 2) ? -w : w;
            const float z = (k & 4) ? -h : h;
            const float X = c * x - s * y + cx;
            const float Y = s * x + c * y + cy;
            const float Z = z + cz;
            const float dx = R[0] * X + R[3] * Y + R[6] * Z;
            const float dy = R[1] * X + R[4] * Y + R[7] * Z;
            const float dz = R[2] * X + R[5] * Y + R[8] * Z;
            const float px = dx, py = -dz, pz = dy;
            const float uu = K[0] * px + K[1] * py + K[2] * pz;
            const float vv = K[3] * px + K[4] * py + K[5] * pz;
            const float ww = K[6] * px + K[7] * py + K[8] * pz;
            const float u = uu / ww, v = vv / ww;
            umin = nmin_f(umin, u);
            umax = nmax_f(umax, u);
            vmin = nmin_f(vmin, v);
            vmax = nmax_f(vmax, v);
        }
        const float wf = (float)img_w[b], hf = (float)img_h[b];
        const float box[4] = {vmin, umin, vmax, umax};
        const float lim[4] = {wf, hf, wf, hf};
        for (int i = 0; i < 4; ++i) {
            float v = box[i] < 0.f ? 0.f : box[i];
            v = v > lim[i] ? lim[i] : v;
            out[4 * r + i] = v;
        }
    }
    return 0;
}

/* ------------------------------------------------- SA MLP + max-pool (a4), float64 checker */

#define SA_MAX_LAYERS 4

typedef struct {
    long long R;
    int S, nl, ch[SA_MAX_LAYERS + 1];
    double* xhat[SA_MAX_LAYERS];   /* (R, ch[l+1]) normalised pre-activations */
    double* z[SA_MAX_LAYERS];      /* (R, ch[l+1]) layer outputs relu(gamma xhat + beta) */
    double* invstd[SA_MAX_LAYERS];
} sa_state;

static void sa_free(sa_state* st) {
    for (int l = 0; l < SA_MAX_LAYERS; ++l) {
        free(st->xhat[l]);
        free(st->z[l]);
        free(st->invstd[l]);
    }
}

/* the forward of every layer, kept for the backward */
static int sa_forward(const float* x0, long long R, int S, int nl, const int* ch,
                      const float* const* W, const float* const* gamma, const float* const* beta,
                      double eps, sa_state* st, double* mean_out, double* var_out) {
    memset(st, 0, sizeof(*st));
    if (R <= 0 || S <= 0 || R % S || nl < 1 || nl > SA_MAX_LAYERS || !x0 || !W) return -1;
    st->R = R;
    st->S = S;
    st->nl = nl;
    for (int l = 0; l <= nl; ++l) {
        if (ch[l] <= 0) return -1;
        st->ch[l] = ch[l];
    }
    size_t moff = 0;
    for (int l = 0; l < nl; ++l) {
        const int K = ch[l], C = ch[l + 1];
        st->xhat[l] = (double*)malloc(sizeof(double) * (size_t)R * C);
        st->z[l] = (double*)malloc(sizeof(double) * (size_t)R * C);
        st->invstd[l] = (double*)malloc(sizeof(double) * (size_t)C);
        double* mean = (double*)calloc((size_t)C, sizeof(double));
        double* var = (double*)calloc((size_t)C, sizeof(double));
        if (!st->xhat[l] || !st->z[l] || !st->invstd[l] || !mean || !var) {
            free(mean);
            free(var);
            sa_free(st);
            return -1;
        }
        double* y = st->xhat[l];
        for (long long r = 0; r < R; ++r)
            for (int c = 0; c < C; ++c) {
                double acc = 0.0;
                for (int k = 0; k < K; ++k) {
                    const double xv = l == 0 ? (double)x0[r * K + k] : st->z[l - 1][r * K + k];
                    acc += xv * (double)W[l][(size_t)c * K + k];
                }
                y[r * C + c] = acc;
                mean[c] += acc;
            }
        for (int c = 0; c < C; ++c) mean[c] /= (double)R;
        for (long long r = 0; r < R; ++r)
            for (int c = 0; c < C; ++c) {
                const double d = y[r * C + c] - mean[c];
                var[c] += d * d;
            }
        for (int c = 0; c < C; ++c) {
            var[c] /= (double)R;   /* biased: BatchNorm's normalisation in train mode */
            st->invstd[l][c] = 1.0 / sqrt(var[c] + eps);
            if (mean_out) mean_out[moff + c] = mean[c];
            if (var_out) var_out[moff + c] = var[c];
        }
        for (long long r = 0; r < R; ++r)
            for (int c = 0; c < C; ++c) {
                const double xh = (y[r * C + c] - mean[c]) * st->invstd[l][c];
                y[r * C + c] = xh;
                const double g = gamma && gamma[l] ? (double)gamma[l][c] : 1.0;
                const double bb = beta && beta[l] ? (double)beta[l][c] : 0.0;
                const double t = g * xh + bb;
                st->z[l][r * C + c] = t > 0.0 ? t : 0.0;
            }
        moff += (size_t)C;
        free(mean);
        free(var);
    }
    return 0;
}

/* SharedMLP(ch) + max over S of PointnetSAModuleVotes in train mode [upstream pointnet2
 * pointnet2_modules.py; configured at models/model_3detr.py:353-362]: per layer a 1x1 Conv2d
 * without bias (y = x W^T), BatchNorm2d with the batch statistics (biased variance in the
 * normalisation), ReLU; then F.max_pool2d over the S neighbours of each centroid.
 *   x0 (R, ch[0]) rows, centroid-major (row = p*S + s), R % S == 0; W[l] (ch[l+1], ch[l]);
 *   gamma[l] / beta[l] (ch[l+1]) or NULL (1 / 0); nl <= 4 layers.
 *   out (R/S, ch[nl]) f32; mean / var (sum of ch[1..nl]) f64 per layer, concatenated, or NULL;
 *   argmax (R/S, ch[nl]) int32 the first s attaining the maximum, or NULL.
 * float64 throughout: the checker of the fp32 / bf16 device path (ov3d_sa_layer_* kernels via
 * sa_fused.py), compared within tolerance, not a bit-exact twin. */
int ov3d_sa_mlp_fwd_cpu(const float* x0, long long R, int S, int nl, const int* ch,
                        const float* const* W, const float* const* gamma,
                        const float* const* beta, double eps, float* out, double* mean,
                        double* var, int32_t* argmax) {
    sa_state st;
    if (sa_forward(x0, R, S, nl, ch, W, gamma, beta, eps, &st, mean, var)) return -1;
    const int C = ch[nl];
    const double* z = st.z[nl - 1];
    for (long long p = 0; p < R / S; ++p)
        for (int c = 0; c < C; ++c) {
            int best = 0;
            double v = z[(p * S) * C + c];
            for (int s = 1; s < S; ++s) {
                const double u = z[(p * S + s) * C + c];
                if (u > v) {
                    v = u;
                    best = s;
                }
            }
            out[p * C + c] = (float)v;
            if (argmax) argmax[p * C + c] = best;
        }
    sa_free(&st);
    return 0;
}

/* Gradients of sum(out * dout) (dout (R/S, ch[nl]) f32) for the forward above: the max-pool
 * routes each centroid's gradient to its first maximum, ReLU passes where gamma xhat + beta > 0,
 * BatchNorm's train-mode backward (batch statistics), the conv's dW = dy^T x.
 *   dW[l] (ch[l+1], ch[l]) f32; dgamma[l] / dbeta[l] (ch[l+1]) f32, or NULL arrays / entries. */
int ov3d_sa_mlp_bwd_cpu(const float* x0, long long R, int S, int nl, const int* ch,
                        const float* const* W, const float* const* gamma,
                        const float* const* beta, double eps, const float* dout,
                        float* const* dW, float* const* dgamma, float* const* dbeta) {
    sa_state st;
    if (sa_forward(x0, R, S, nl, ch, W, gamma, beta, eps, &st, NULL, NULL)) return -1;
    int Cmax = 0;
    for (int l = 0; l <= nl; ++l) Cmax = ch[l] > Cmax ? ch[l] : Cmax;
    double* dz = (double*)calloc((size_t)R * Cmax, sizeof(double));
    double* dy = (double*)malloc(sizeof(double) * (size_t)R * Cmax);
    double* s1 = (double*)malloc(sizeof(double) * (size_t)Cmax);
    double* s2 = (double*)malloc(sizeof(double) * (size_t)Cmax);
    if (!dz || !dy || !s1 || !s2) {
        free(dz);
        free(dy);
        free(s1);
        free(s2);
        sa_free(&st);
        return -1;
    }
    {   /* max-pool backward into dz of the last layer */
        const int C = ch[nl];
        const double* z = st.z[nl - 1];
        for (long long p = 0; p < R / S; ++p)
            for (int c = 0; c < C; ++c) {
                int best = 0;
                double v = z[(p * S) * C + c];
                for (int s = 1; s < S; ++s) {
                    const double u = z[(p * S + s) * C + c];
                    if (u > v) {
                        v = u;
                        best = s;
                    }
                }
                dz[(p * S + best) * C + c] = (double)dout[p * C + c];
            }
    }
    for (int l = nl - 1; l >= 0; --l) {
        const int K = ch[l], C = ch[l + 1];
        const double* xh = st.xhat[l];
        for (int c = 0; c < C; ++c) s1[c] = s2[c] = 0.0;
        /* dt = dz * relu'(t); dxhat = gamma dt; s1 = sum dxhat, s2 = sum dxhat xhat */
        for (long long r = 0; r < R; ++r)
            for (int c = 0; c < C; ++c) {
                const double g = gamma && gamma[l] ? (double)gamma[l][c] : 1.0;
                const double dt = st.z[l][r * C + c] > 0.0 ? dz[r * C + c] : 0.0;
                dy[r * C + c] = dt;   /* dt kept for dgamma / dbeta */
                s1[c] += g * dt;
                s2[c] += g * dt * xh[r * C + c];
            }
        if (dgamma && dgamma[l])
            for (int c = 0; c < C; ++c) {
                double a = 0.0;
                for (long long r = 0; r < R; ++r) a += dy[r * C + c] * xh[r * C + c];
                dgamma[l][c] = (float)a;
            }
        if (dbeta && dbeta[l])
            for (int c = 0; c < C; ++c) {
                double a = 0.0;
                for (long long r = 0; r < R; ++r) a += dy[r * C + c];
                dbeta[l][c] = (float)a;
            }
        for (long long r = 0; r < R; ++r)
            for (int c = 0; c < C; ++c) {
                const double g = gamma && gamma[l] ? (double)gamma[l][c] : 1.0;
                const double dxh = g * dy[r * C + c];
                dy[r * C + c] = st.invstd[l][c] / (double)R *
                                ((double)R * dxh - s1[c] - xh[r * C + c] * s2[c]);
            }
        if (dW && dW[l])
            for (int c = 0; c < C; ++c)
                for (int k = 0; k < K; ++k) {
                    double a = 0.0;
                    for (long long r = 0; r < R; ++r) {
                        const double xv = l == 0 ? (double)x0[r * K + k] : st.z[l - 1][r * K + k];
                        a += dy[r * C + c] * xv;
                    }
                    dW[l][(size_t)c * K + k] = (float)a;
                }
        if (l > 0)   /* dz of the layer below = dy W */
            for (long long r = 0; r < R; ++r)
                for (int k = 0; k < K; ++k) {
                    double a = 0.0;
                    for (int c = 0; c < C; ++c) a += dy[r * C + c] * (double)W[l][(size_t)c * K + k];
                    dz[r * K + k] = a;
                }
    }
    free(dz);
    free(dy);
    free(s1);
    free(s2);
    sa_free(&st);
    return 0;
}
