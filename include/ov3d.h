/*
 * ov3d.h — C ABI of libov3d_hip.so, the MI355X (gfx950) kernels of the
 * open-vocabulary 3D detection hot path.
 *
 * Conventions:
 *   - plain pointers to DEVICE memory, sizes as int; the caller (PyTorch)
 *     allocates every output and workspace, the library owns no memory;
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream);
 *     every entry point is stream-ordered and asynchronous (no host sync),
 *     so it can be captured into a hipGraph;
 *   - return 0 on success, OV3D_EINVAL on a bad argument, OV3D_ELAUNCH on a
 *     HIP launch error.  The library never prints and never exit()s (the
 *     upstream pointnet2 wrappers print and call exit(-1) on CUDA errors).
 *
 * Each entry point names the reference interface it replaces.
 */
#ifndef OV3D_H_
#define OV3D_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OV3D_OK 0
#define OV3D_EINVAL (-1)
#define OV3D_ELAUNCH (-2)

/* Library version / build tag (host-only, no device work). */
const char* ov3d_version(void);

/* Iterative furthest-point sampling.
 * Replaces third_party.pointnet2.pointnet2_utils.furthest_point_sample
 * (called at models/model_3detr.py:174 and inside PointnetSAModuleVotes,
 * models/model_3detr.py:355-361, 385-391).
 *   xyz      (B,N,3) f32      idx_out (B,M) int32, idx_out[:,0] = 0
 *   new_xyz_out (B,M,3) f32 or NULL: fused gather_operation of the samples
 *   workspace: ov3d_fps_workspace(B, N) floats, 16-byte aligned (N > 20480: up to 40960
 *   points a two-cluster kernel keeps half of each wave's points in this L2-resident
 *   scratch; beyond, the running distances), may be NULL when that is 0.
 * Tie rule = the upstream 512-thread tree reduction. */
int ov3d_fps(const float* xyz, int B, int N, int M, int32_t* idx_out, float* new_xyz_out,
             float* workspace, void* stream);
long long ov3d_fps_workspace(int B, int N);
/* Outcome of the last ov3d_fps on `workspace` (same B, N, M): status (B,) int32 on the device,
 * 1 where the two-workgroup kernel (20480 < N <= 40960, taken only when its 2B workgroups fit
 * the device at once) lost its partner workgroup -- that scene's new_xyz_out is NaN --, else 0.
 * Replaces nothing upstream: its FPS has no such path (it prints and exit()s on launch errors). */
int ov3d_fps_pair_status(const float* workspace, int B, int N, int M, int32_t* status,
                         void* stream);

/* Max over the S neighbour rows of each centroid (F.max_pool2d(kernel [1, nsample]) in
 * PointnetSAModuleVotes, models/model_3detr.py:353-362, 385-391) on channels-last bf16 rows:
 *   y (P*S, C) -> out (P, C), arg (P, C) uint8 = the first row (0..S-1) holding the max;
 *   backward: g (P, C) -> dy (P*S, C) bf16, g on the arg rows, zero elsewhere.  C % 8 == 0,
 *   S <= 256. */
int ov3d_nbr_max_fwd(const void* y, long long P, int S, int C, void* out, uint8_t* arg,
                     void* stream);
int ov3d_nbr_max_bwd(const void* g, const uint8_t* arg, long long P, int S, int C, void* dy,
                     void* stream);
/* ov3d_nbr_max_fwd of z = bf16(relu(y * scale + shift)) (the ov3d_rows_bn_apply arithmetic, no
 * dropout) without storing z: y (P*S, C) bf16 rows of the last SA layer before its BatchNorm */
int ov3d_nbr_max_bnrelu_fwd(const void* y, long long P, int S, int C, const float* scale,
                            const float* shift, void* out, uint8_t* arg, void* stream);

/* Ball query: first S point indices (ascending) with |p - c|^2 < radius^2,
 * padded with the first hit, zeros if none.
 * Replaces pointnet2_utils.ball_query (QueryAndGroup, model_3detr.py:355-361).
 *   xyz (B,N,3), new_xyz (B,M,3) f32  ->  idx_out (B,M,S) int32 */
int ov3d_ball_query(const float* xyz, const float* new_xyz, int B, int N, int M, float radius,
                    int S, int32_t* idx_out, void* stream);

/* The same output from a uniform-grid index of each scene (two launches: a per-scene counting
 * sort into ws, then one wave per centroid over the 27 cells around it) instead of a scan of
 * the whole scene.  ws: >= ov3d_ball_query_ws_bytes(B, N) bytes of device memory, 16-B aligned,
 * owned by the stream until the call's work is done.  N < 8192 (the scan is cheaper there),
 * N >= 65536 or S > 64: the scan above. */
long long ov3d_ball_query_ws_bytes(int B, int N);
int ov3d_ball_query_cells(const float* xyz, const float* new_xyz, int B, int N, int M,
                          float radius, int S, int32_t* idx_out, void* ws, long long ws_bytes,
                          void* stream);

/* QueryAndGroup output with use_xyz=True (pointnet2_utils.QueryAndGroup.forward),
 * written as channels-last rows (the GEMM layout of the SA MLP):
 *   out[b,m,s, 0:3]   = (xyz[b,idx] - new_xyz[b,m]) (/ radius if normalize)
 *   out[b,m,s, 3:3+C] = features[b, :, idx]          (features may be NULL, C = 0)
 * features element (b, n, c) lives at features[b*feat_sb + n*feat_sn + c*feat_sc]
 * ((B,C,N) contiguous: sb = C*N, sn = 1, sc = N; seq-first (N,B,C): sb = C, sn = B*C, sc = 1).
 *   xyz (B,N,3) f32, new_xyz (B,M,3), idx (B,M,S) int32 -> out (B,M,S,3+C) f32 */
int ov3d_group_fwd(const float* xyz, const float* new_xyz, const float* features,
                   long long feat_sb, long long feat_sn, long long feat_sc, const int32_t* idx,
                   int B, int C, int N, int M, int S, float radius, int normalize, float* out,
                   void* stream);

/* Backward of the feature part of ov3d_group_fwd (grouping_operation backward):
 *   grad_out (B,M,S,3+C) -> grad_features (B*C*N elements, same strides as the forward);
 *   the callee zero-fills grad_features on the stream, then scatter-adds. */
int ov3d_group_bwd(const float* grad_out, const int32_t* idx, int B, int C, int N, int M, int S,
                   long long feat_sb, long long feat_sn, long long feat_sc, float* grad_features,
                   void* stream);

/* Inverse of a ball-query index, for a gather-form grouping backward (no float atomics):
 *   idx (B,M,S) -> offsets (B*N+1) and rows (B*M*S): the rows r = (b*M + m)*S + s with
 *   idx[r] = n are rows[offsets[b*N+n] .. offsets[b*N+n+1]), ascending (deterministic sums).
 *   cnt, cursor: B*N int32 scratch.  (B*N up to ~10^6: the scan is one workgroup.) */
int ov3d_group_inverse(const int32_t* idx, int B, int N, int M, int S, int32_t* cnt,
                       int32_t* offsets, int32_t* cursor, int32_t* rows, void* stream);
/* ov3d_group_bwd through the inverse: every grad_features element written (no zero fill). */
int ov3d_group_bwd_csr(const float* grad_out, const int32_t* offsets, const int32_t* rows, int B,
                       int C, int N, long long feat_sb, long long feat_sn, long long feat_sc,
                       float* grad_features, void* stream);

/* ov3d_group_fwd's rows in bf16 with row stride ldo (a multiple of 8, >= 3 + C; columns
 * 3 + C .. ldo-1 written as zeros; out 16-byte aligned): the input of an SA MLP's first GEMM
 * under bf16 autocast, with an aligned K (the masked encoder's interim SA: 259 -> 264). */
int ov3d_group_rows_bf16(const float* xyz, const float* new_xyz, const float* features,
                         long long feat_sb, long long feat_sn, long long feat_sc,
                         const int32_t* idx, int B, int C, int N, int M, int S, float radius,
                         int normalize, int ldo, void* out, void* stream);
/* ov3d_group_bwd_csr for bf16 grad rows with row stride ldg (feature columns 3 .. 3+C). */
int ov3d_group_bwd_csr_bf16(const void* grad_out, long long ldg, const int32_t* offsets,
                            const int32_t* rows, int B, int C, int N, long long feat_sb,
                            long long feat_sn, long long feat_sc, float* grad_features,
                            void* stream);

/* gather_operation (pointnet2_utils): features (B,C,N), idx (B,M) -> out (B,C,M) */
int ov3d_gather_fwd(const float* features, const int32_t* idx, int B, int C, int N, int M,
                    float* out, void* stream);
/* gather_operation backward: grad_out (B,C,M) -> grad_features (B,C,N) (zero-filled here) */
int ov3d_gather_bwd(const float* grad_out, const int32_t* idx, int B, int C, int N, int M,
                    float* grad_features, void* stream);

/* 3D generalized IoU, (B,K1) predicted vs (B,K2) GT boxes given as corners
 * (B,K,8,3) f32 with up = -Y.  Replaces utils/box_util.py:717-737:
 *   mode OV3D_GIOU_CYTHON (0): generalized_box3d_iou_cython (box_util.py:624-714)
 *        + utils/box_intersection.pyx (double-precision clipping); with
 *        k2_bug != 0 the rotated intersection is evaluated only for
 *        k2 < min(4, nums[b]) (box_intersection.pyx:180, K2 = rect2.shape[2]).
 *   mode OV3D_GIOU_TENSOR (1): generalized_box3d_iou_tensor (box_util.py:517-618),
 *        float32 clipping, all k2 < nums[b].
 *   rotated == 0: axis-aligned (x,z) rectangle intersection (box_util.py:695-696).
 * rotated_dev: optional DEVICE int32 flag that overrides `rotated` when non-NULL
 *   (the reference decides rotated = any(gt_box_angles > 0) on the host,
 *   criterion.py:317-330; reading it on the device keeps the step sync-free).
 * nums (B,) int32 = number of valid GT boxes per scene, or NULL (= K2).
 * out (B,K1,K2) f32. */
#define OV3D_GIOU_CYTHON 0
#define OV3D_GIOU_TENSOR 1
int ov3d_giou3d(const float* corners1, const float* corners2, const int32_t* nums, int B, int K1,
                int K2, int mode, int rotated, const int32_t* rotated_dev, int k2_bug, float* out,
                void* stream);

/* Backward of the differentiable GIoU (OV3D_GIOU_TENSOR semantics, box_util.py:517-618 under
 * autograd) w.r.t. corners1: grad_out (B,K1,K2) -> grad_corners1 (B,K1,8,3) (overwritten).
 * rotated / rotated_dev as ov3d_giou3d: the rotated intersection is differentiated through
 * every Sutherland-Hodgman intersection vertex (box_util.py:387-440, 579-600). */
int ov3d_giou3d_bwd(const float* corners1, const float* corners2, const int32_t* nums, int B,
                    int K1, int K2, int rotated, const int32_t* rotated_dev, const float* grad_out,
                    float* grad_corners1, void* stream);

/* ov3d_giou3d_bwd with rotated = 0 (axis-aligned GIoU). */
int ov3d_giou3d_bwd_aligned(const float* corners1, const float* corners2, const int32_t* nums,
                            int B, int K1, int K2, const float* grad_out, float* grad_corners1,
                            void* stream);

/* Hungarian matching for a stack of P problems, one workgroup each.
 * Replaces the host loop of criterion.py:77-86 (scipy.optimize.linear_sum_assignment
 * on final_cost[b, :, :nactual_gt[b]]) with scipy 1.15's algorithm restated
 * exactly (Crouse shortest augmenting path, float64 path costs, the same
 * tie rule), so assignments are identical to scipy's for the same costs.
 *   cost (P,Q,G) f32, nactual (P,) int32 (columns 0..nactual-1 are used)
 *   -> gt_inds (P,Q) int64 (0 where unmatched), matched (P,Q) f32 (1/0),
 *      status (P,) int32 or NULL: 0 ok, -1 NaN/-inf cost (scipy raises
 *      ValueError), -2 infeasible.  Q and G <= 1024. */
int ov3d_hungarian(const float* cost, const int32_t* nactual, int P, int Q, int G, int64_t* gt_inds,
                   float* matched, int32_t* status, void* stream);

/* ---- Fused set-abstraction MLP (training, bf16 activations, fp32 accumulate) ----
 * Replaces pointnet2 SharedMLP([3, C1, C2, C3], bn=True) + F.max_pool2d([1, nsample])
 * inside PointnetSAModuleVotes (model_3detr.py:353-362) for training under bf16
 * autocast.  Rows are channels-last (R = B*npoint*nsample, C); bf16 buffers are
 * passed as void*.  BN statistics: each kernel writes fp64 partials (nparts, 2, C)
 * (sum, sum of squares), ov3d_reduce_partials sums them (an all-reduce may follow
 * for SyncBatchNorm), ov3d_bn_finalize folds them into scale/shift.  See
 * DESIGN.md "Fused SA MLP" for the algebra. */
/* layer 1: x0 (R,3) f32, W1 (C1,3) f32 -> y1 (R,C1) bf16, partials (nparts,2,C1) */
int ov3d_sa_l1_fwd(const float* x0, const float* W1, int R, int C1, void* y1, double* partials,
                   int nparts, void* stream);
/* the same for x0 (R, cin) with cin = 3 or 6 (xyz + colour, ScanNet --use_color), W1 (C1, cin) */
int ov3d_sa_l1_fwd_cin(const float* x0, int cin, const float* W1, int R, int C1, void* y1,
                       double* partials, int nparts, void* stream);
/* (y1 may be NULL: statistics only, for consumers that recompute the layer from x0) */
/* 1 if the MFMA layer kernel is built for (K, N) */
int ov3d_sa_layer_supported(int K, int N);
/* layer k: z = relu(scale*yprev + shift) (bf16, optionally stored to zout) ->
 * y = z W^T (W (N,K) bf16) -> yout (R,N) bf16 + partials (nparts,2,N).  R % 64 == 0. */
int ov3d_sa_layer_fwd(const void* yprev, const float* scale, const float* shift, const void* W,
                      int R, int K, int N, void* zout, void* yout, double* partials, int nparts,
                      void* stream);
/* layer 2 with its input recomputed: yprev = bf16(x0 W1^T) per row (ov3d_sa_l1_fwd's value,
 * bit for bit) instead of read, so the first layer's (R, 64) output is never stored:
 * x0 (R, 3) f32, W1 (K, 3) f32; K = 64, N = 128. */
int ov3d_sa_layer_fwd_x0(const float* x0, const float* W1, const float* scale, const float* shift,
                         const void* W, int R, int K, int N, void* yout, double* partials,
                         int nparts, void* stream);
/* last layer + pool: as ov3d_sa_layer_fwd but y is not stored; per centroid (S rows,
 * S in {32,64}) and channel: max/min of y (bf16 values) and their rows. */
/* gamma (N) or NULL: the layer's BN weight.  Given, a channel with gamma >= 0 gets only its
 * max (pmax, imax) and one with gamma < 0 only its min (pmin, imin), the one extreme
 * ov3d_sa_pool_fwd reads (a = gamma * invstd has gamma's sign); NULL: both. */
int ov3d_sa_layer_pool_fwd(const void* yprev, const float* scale, const float* shift,
                           const void* W, int R, int K, int N, int S, void* zout, float* pmax,
                           float* pmin, uint8_t* imax, uint8_t* imin, const float* gamma,
                           double* partials, int nparts, void* stream);
/* backward of the last layer: recompute y, dy = cA*g + cB*y + cC with g = gsel at
 * row isel of each centroid (0 elsewhere) -> dyout (R,N) bf16. */
int ov3d_sa_layer_dy(const void* yprev, const float* scale, const float* shift, const void* W,
                     int R, int K, int N, int S, const float* gsel, const uint8_t* isel,
                     const float* cA, const float* cB, const float* cC, void* dyout, int nparts,
                     void* stream);
/* Backward of the pooled last layer in one pass (csrc/sa_bwd.hip): recomputes
 * z = relu(scale*yprev + shift) and y = z W^T, dy = cA*g + cB*y + cC (g = gsel at the isel
 * row), and writes dz = dy W (R, K) bf16 and the per-workgroup dW = dy^T z partials
 * dwpart (nwg, N, K) fp32 (sum them over nwg); dy and z never reach HBM.  K = 128, N = 256.
 * stats (nwg, 2, K) fp64 or NULL: the previous layer's ReLU + BN backward partials (sum dt,
 * sum dt * (yprev - mean) * invstd with dt = (scale*yprev + shift > 0) * dz), the pass 0
 * of ov3d_bn_relu_bwd on the dz written. */
int ov3d_sa_dy_fused_supported(int K, int N);
/* The middle layer's backward in one pass (csrc/sa_bwd.hip): from dz2 and the layer-2 BN
 * backward coefficients: dy2 = cA*dt + cB*y2 + cC (dt = (a2*y2 + b2 > 0) * dz2), z1 =
 * relu(a1*y1 + b1) recomputed; writes dz1 = dy2 W2 (R, K) bf16, dW2 = dy2^T z1 partials
 * dwpart (nwg, N, K) and layer 1's ReLU + BN backward partials stats (2*nwg, 2, K) (sum dt1,
 * sum dt1 * (y1 - mean1) * invstd1 on the stored dz1).  K = 64, N = 128. */
/* (y1 == NULL: y1 recomputed from x0 (R, 3) and W1 (K, 3) as ov3d_sa_layer_fwd_x0) */
int ov3d_sa_dy2_fused(const void* y1, const float* x0, const float* W1, const float* a1,
                      const float* b1, const void* y2, const float* a2, const float* b2,
                      const void* dz2, const float* cA, const float* cB, const float* cC,
                      const void* W, const float* mean1, const float* invstd1, int R, int K, int N,
                      void* dz1, float* dwpart, double* stats, int nwg, void* stream);
/* (ysel (P, N): the pooled y3 value at the isel row, as ov3d_sa_pool_fwd wrote it; the dy of
 * that row is cA*g + cB*ysel + cC, every other row's cB*y + cC) */
int ov3d_sa_dy_fused(const void* yprev, const float* scale, const float* shift, const void* W,
                     int R, int K, int N, int S, const float* gsel, const uint8_t* isel,
                     const float* ysel, const float* cA, const float* cB, const float* cC,
                     void* dz, float* dwpart, const float* mean, const float* invstd,
                     double* stats, int nwg, void* stream);
/* (nparts, width) fp64 -> (width) sums */
int ov3d_reduce_partials(const double* partials, int nparts, int width, double* totals,
                         void* stream);
/* the same sums rounded once to fp32 (the fused SA's first-layer weight gradient) */
int ov3d_reduce_partials_f32(const double* partials, int nparts, int width, float* totals,
                             void* stream);
/* training BN: totals (2,C) over `count` rows -> mean, invstd, scale = gamma*invstd,
 * shift = beta - mean*scale; running stats updated (momentum, unbiased var) if non-NULL;
 * num_batches_tracked (int64) += 1 if non-NULL (nn.BatchNorm1d's counter) */
int ov3d_bn_finalize(const double* totals, double count, int C, const float* gamma,
                     const float* beta, float eps, float momentum, float* running_mean,
                     float* running_var, float* mean_out, float* invstd_out, float* scale_out,
                     float* shift_out, long long* num_batches_tracked, void* stream);
/* ov3d_reduce_partials(2C) + ov3d_bn_finalize in one launch (single-replica BatchNorm):
 * partials (nparts, 2C) of (sum, sum of squares); bit-identical to the two launches */
int ov3d_bn_stats_finalize(const double* partials, int nparts, int C, double count,
                           const float* gamma, const float* beta, float eps, float momentum,
                           float* running_mean, float* running_var, float* mean_out,
                           float* invstd_out, float* scale_out, float* shift_out,
                           long long* num_batches_tracked, void* stream);
/* ov3d_reduce_partials(2C) + ov3d_bn_bwd_finalize in one launch (single replica) */
int ov3d_bn_bwd_stats_finalize(const double* partials, int nparts, int C, double count,
                               const float* gamma, const float* mean, const float* invstd,
                               float* cA, float* cB, float* cC, float* dgamma, float* dbeta,
                               void* stream);
/* out[c] = sum over the nparts rows of parts (nparts, width) f32, fixed order (the fused SA
 * backward's per-workgroup dW partials; replaces torch's part.sum(0) in sa_fused.py) */
int ov3d_colsum_f32(const float* parts, int nparts, int width, float* out, void* stream);
/* pooled output (P,N) f32 = relu(scale*(scale >= 0 ? pmax : pmin) + shift), plus the
 * selected value / row for the backward.  seq_m = 0: out row p = b*M + m; seq_m = M > 0:
 * out row m*B + b (sequence-first, the encoder's input layout; P % M == 0) */
int ov3d_sa_pool_fwd(const float* pmax, const float* pmin, const uint8_t* imax,
                     const uint8_t* imin, const float* scale, const float* shift, int P, int N,
                     int seq_m, float* out, float* ysel, uint8_t* isel, void* stream);
/* pooled-gradient ReLU mask + BN-backward partials (sum g, sum g*xhat); dout in the
 * forward's output row order (seq_m) */
int ov3d_sa_pool_bwd(const float* dout, const float* ysel, const float* scale, const float* shift,
                     const float* mean, const float* invstd, int P, int N, int seq_m, float* gsel,
                     double* partials, int nparts, void* stream);
/* BN backward coefficients: dx = cA*g + cB*y + cC; dgamma, dbeta (may be NULL) */
int ov3d_bn_bwd_finalize(const double* totals, double count, int C, const float* gamma,
                         const float* mean, const float* invstd, float* cA, float* cB, float* cC,
                         float* dgamma, float* dbeta, void* stream);
/* ReLU + BN backward over (R,C) bf16 rows (dz = grad of the ReLU output, y = BN input):
 * pass 0: partials (nparts,2,C) of dt and dt*xhat;  pass 1: dyout = cA*dt + cB*y + cC;
 * pass 2: dW1 partials (nparts,C,3) = sum_r dy[r,c] * x0[r,k] (first layer, dy not stored) */
/* (pass 2 with y == NULL: the first layer's y recomputed from x0 and W1 (C, 3)) */
int ov3d_bn_relu_bwd(int pass, const void* dz, const void* y, const float* scale,
                     const float* shift, const float* mean, const float* invstd, const float* cA,
                     const float* cB, const float* cC, const float* x0, int R, int C,
                     double* partials, void* dyout, int nparts, const float* W1, void* stream);
/* the same with x0 (R, cin), cin = 3 or 6: pass 2 writes dW1 partials (nparts, C, cin)
 * (y == NULL recompute only for cin = 3) */
int ov3d_bn_relu_bwd_cin(int pass, const void* dz, const void* y, const float* scale,
                         const float* shift, const float* mean, const float* invstd,
                         const float* cA, const float* cB, const float* cC, const float* x0, int cin,
                         int R, int C, double* partials, void* dyout, int nparts, const float* W1,
                         void* stream);

/* Greedy 3D NMS, batched over scenes.  Replaces utils/nms.py:79-162
 * (nms_3d_faster / nms_3d_faster_samecls) as called per scene by
 * utils/ap_calculator.py:153-190.
 *   boxes (B,K,stride) f64 rows [x1,y1,z1,x2,y2,z2,score(,cls)], stride 7|8
 *   valid (B,K) uint8 or NULL: rows with 0 do not take part (nonempty mask)
 *   keep_out (B,K) uint8 (1 = picked).  samecls: suppress only same class.
 * Ties in score: larger index first (== np.argsort(kind="stable")).  K <= 512. */
int ov3d_nms3d(const double* boxes, const uint8_t* valid, int B, int K, int stride, double thr,
               int old_type, int samecls, uint8_t* keep_out, void* stream);

/* NMS box table straight from predicted corners (ap_calculator.py:153-190):
 *   corners (B,K,8,3) f32, obj (B,K) f32, cls (B,K) int64 -> boxes (B,K,8) f64 */
int ov3d_nms_boxes_from_corners(const float* corners, const float* obj, const int64_t* cls, int B,
                                int K, double* boxes_out, void* stream);

/* ---- RegionCLIP ROI-feature path (CLIPFastRCNN.inference, criterion.py:397) ---- */

/* CLIPFastRCNN.preprocess_image + ImageList.from_tensors [upstream RegionCLIP]
 * fed with the per-scene image views of criterion.py:371-375,394:
 *   images (B, img_stride) f32: scene b's (H_b, W_b, 3) image in its first H_b*W_b*3
 *   values; heights/widths (B,) int32 on the device
 *   -> out (B, Hp, Wp, 3) NHWC, ((v / div) - mean[c]) / std[c], 0 outside (H_b, W_b);
 *   out_bf16 selects bf16 (1) or f32 (0) output. */
int ov3d_clip_preprocess(const float* images, long long img_stride, const int32_t* heights,
                         const int32_t* widths, int B, int Hp, int Wp, float div, float m0,
                         float m1, float m2, float s0, float s1, float s2, int out_bf16, void* out,
                         void* stream);

/* 3D box -> 2D image box of the RegionCLIP alignment branch.  Replaces
 * utils/image_util.py:117-134 project_box_3d_cuda with SUNRGBD_Calibration_cuda
 * (image_util.py:275-298) and the clamp of criterion.py:386-391 (quirk Q4: the full size
 * as half-extent; [min v, min u, max v, max u]).
 *   center / size (n, 3), heading (n) f32, rows ordered (.., scene, query): the scene of
 *   row r is (r / Q) % B; Rtilt / K (B, 3, 3) f32 row-major; img_h / img_w (B) int64
 *   -> out (n, 4) f32 clamped to [0, (w, h, w, h)].  float32 arithmetic as the reference. */
int ov3d_project_box2d(const float* center, const float* size, const float* heading, long long n,
                       int Q, int B, const float* Rtilt, const float* K, const int64_t* img_h,
                       const int64_t* img_w, float* out, void* stream);

/* Output layers of the five prediction heads + the query <-> text alignment, one launch.
 * Replaces the last Conv1d of each GenericMLP head (models/model_3detr.py:_build_heads,
 * models/helpers.py:45-112) and sem_cls_head = Linear(640, T, bias=False) over the visual
 * embedding (model_3detr.py:152-154, 237-238).
 *   z (R, ldz) bf16 hidden rows: visual head columns [0, 256), box head i at kcol[i]
 *   wv (Nv, 256) bf16, bv (Nv) f32 -> out_v (R, Nv) f32 (Nv = 640, the CLIP embedding)
 *   text (T, Nv) f32 (T <= ov3d_heads_out_max_text(); null = no alignment) -> logits f32,
 *     row-major (R, T) when lq == 0, else the reference's transposed layout of quirk Q8:
 *     (lb, q, t) at lb*lq*T + t*lq + q
 *   box head i (ns <= 4): ws[i] (n[i] <= 32, 256) bf16, bs[i] (n[i]) f32 ->
 *     out_s[:, ocol[i] : ocol[i] + n[i]] of (R, Ns) f32
 *   work: ov3d_heads_out_workspace(R, T) floats (the column groups' partial logits) */
int ov3d_heads_out_max_text(void);
long long ov3d_heads_out_workspace(int R, int T);
int ov3d_heads_out_fwd(const void* z, long long ldz, int R, const void* wv, const float* bv, int Nv,
                       const float* text, int T, int lq, float* out_v, float* logits, int ns,
                       const void* const* ws, const float* const* bs, const int* n,
                       const int* kcol, const int* ocol, float* out_s, int Ns, float* work,
                       void* stream);
/* Its backward: gvb = bf16(gv + glog . text) (R, Nv) (gv may be NULL: zero); gsb = bf16(gs)
 * (R, Ns); the box heads'
 * input gradient dz[:, kcol[i] + c] = bf16(sum_j gsb[:, ocol[i] + j] ws[i][j, c]), c < 256
 * (dz (R, lddz) bf16; its visual columns are left to the caller's dgrad GEMM on gvb). */
int ov3d_heads_out_bwd(const float* gv, const float* glog, const float* text, int R, int Nv, int T,
                       int lq, const float* gs, int Ns, int ns, const void* const* ws,
                       const int* n, const int* kcol, const int* ocol, void* gvb, void* gsb,
                       void* dz, long long lddz, void* stream);

/* ROIAlign forward on channels-last features.  Replaces the ROIAlignV2 pooler of
 * CLIPRes5ROIHeads (detectron2 ROIPooler -> torchvision roi_align, aligned=True)
 * [upstream RegionCLIP] used by clip.inference at criterion.py:397.
 *   feat (N, H, W, C) f32 (is_bf16 = 0, C % 4 == 0) or bf16 (is_bf16 = 1, C % 8 == 0)
 *   boxes (R, 4) f32 [x1, y1, x2, y2] in image pixels; roi r samples image
 *   (r / per_image) % nimages  (rows ordered (layer, scene, query))
 *   -> out (R, pooled, pooled, C), same dtype; sampling_ratio <= 0 = adaptive
 *   (ceil(roi_size / pooled)).  fp32 arithmetic in torchvision's order.  feat and out
 *   16-byte aligned (one 16-byte channel run per corner load). */
int ov3d_roi_align_fwd(const void* feat, int is_bf16, int N, int H, int W, int C,
                       const float* boxes, int R, int per_image, int nimages, float spatial_scale,
                       int pooled, int sampling_ratio, int aligned, void* out, void* stream);

/* ov3d_roi_align_fwd plus the 2x2 average pool of its output [the AvgPool2d(2) of res5's first
 * Bottleneck identity path, upstream CLIP ModifiedResNet] in the same launch:
 *   pooled_out (R, pooled/2, pooled/2, C) = ov3d_avgpool2_nhwc(out), bit for bit; pooled even. */
int ov3d_roi_align_pool2_fwd(const void* feat, int is_bf16, int N, int H, int W, int C,
                             const float* boxes, int R, int per_image, int nimages,
                             float spatial_scale, int pooled, int sampling_ratio, int aligned,
                             void* out, void* pooled_out, void* stream);

/* NHWC im2col for a 3x3 convolution (pad 1, stride 1|2) of the RegionCLIP
 * ModifiedResNet [upstream CLIP/RegionCLIP; the convolutions of clip.inference,
 * criterion.py:397], so that the convolution is one GEMM against the
 * channels-last weight viewed as (Cout, 9*C):
 *   in (N, H, W, C), elem_bytes 2 (bf16) or 4 (f32)
 *   -> out (N*Ho*Wo, Kpad), column k = (ky*3 + kx)*C + c, zeros outside the image
 *      and for 9*C <= k < Kpad;  Ho = (H-1)/stride + 1, Wo likewise. */
int ov3d_im2col3x3(const void* in, int elem_bytes, int N, int H, int W, int C, int stride,
                   int Kpad, void* out, void* stream);

/* Bottleneck close of the RegionCLIP ModifiedResNet [upstream CLIP Bottleneck.forward:
 * out = relu(bn3(conv3(out)) + identity); clip.inference, criterion.py:397] after the 1x1
 * conv3 GEMM, with BN folded into the bias:
 *   y (rows, cols) <- act(y + bias + residual), in place, fp32 arithmetic, one rounding;
 *   elem_bytes 2 (bf16) or 4 (f32); cols a multiple of 16/elem_bytes, pointers 16-byte aligned. */
int ov3d_bias_residual_act(void* y, int elem_bytes, long long rows, int cols, const void* bias,
                           const void* residual, int relu, void* stream);

/* 2x2 / stride-2 average pool on NHWC [upstream CLIP ModifiedResNet: the nn.AvgPool2d(2) of the
 * stem and of every strided Bottleneck / downsample; torch avg_pool2d(kernel 2) semantics]:
 *   in (N, H, W, C) -> out (N, H/2, W/2, C), fp32 sum in torch's NHWC order, / 4, one rounding;
 *   elem_bytes 2 (bf16) or 4 (f32); C a multiple of 16/elem_bytes, pointers 16-byte aligned. */
int ov3d_avgpool2_nhwc(const void* in, int elem_bytes, int N, int H, int W, int C, void* out,
                       void* stream);

/* Token rows of CLIP's AttentionPool2d [upstream CLIP AttentionPool2d.forward: the mean token
 * concatenated before the spatial tokens, plus the positional embedding; clip.inference,
 * criterion.py:397]:
 *   x (R, ntok, C), pos (ntok + 1, C) -> t (R, ntok + 1, C):
 *   t[r, 0] = T(mean_j x[r, j]) + pos[0] (fp32 mean in token order), t[r, 1 + j] = x[r, j] + pos[1 + j];
 *   elem_bytes 2 (bf16) or 4 (f32); C a multiple of 16/elem_bytes, pointers 16-byte aligned. */
int ov3d_attnpool_tokens(const void* x, int elem_bytes, int R, int ntok, int C, const void* pos,
                         void* t, void* stream);

/* The same pool's first query without the token rows (csrc/attnpool.hip) [upstream CLIP
 * AttentionPool2d.forward, x[0] only; clip.inference, criterion.py:397; regionclip._pool_tokens]:
 * ov3d_attnpool_mean: x (R, ntok, C) bf16, pos (ntok + 1, C) -> t0 (R, C) = bf16(bf16(mean_j x[r, j])
 *   + pos[0]) (fp32 mean in token order: row 0 of ov3d_attnpool_tokens);
 * ov3d_attnpool_fused: with a (r, h, c) at a[h * sa_h + r * sa_r + c] (= Wk_h^T q[r, h], bf16),
 *   token rows t[r, 0] = t0[r], t[r, 1 + j] = bf16(x[r, j] + pos[1 + j]) built on chip:
 *   s = bf16(a t^T) (fp32 sums), p = bf16(softmax_j(s)) (fp32), y (H, R, C) = bf16(p t) (fp32 sums).
 * ov3d_attnpool_fused_supported(ntok, C, H): ntok + 1 <= 96, C % 64 == 0, H <= 48.  bf16 only;
 * every pointer 16-byte aligned, sa_h and sa_r multiples of 8 elements. */
int ov3d_attnpool_mean(const void* x, int R, int ntok, int C, const void* pos, void* t0, void* stream);
int ov3d_attnpool_fused_supported(int ntok, int C, int H);
int ov3d_attnpool_fused(const void* x, const void* t0, const void* pos, const void* a, long long sa_h,
                        long long sa_r, int R, int ntok, int C, int H, void* y, void* stream);

/* Large bf16 GEMM on 256 x 256 tiles (hand-written MFMA, csrc/gemm256.hip) for the RegionCLIP
 * res5 1x1 convolutions over all L*B*Q ROIs [upstream CLIP ModifiedResNet layer4;
 * clip.inference, criterion.py:397] and the 3DETR decoder's memory K / V projections
 * (models/transformer.py:369-372, nn.MultiheadAttention in_proj of the memory):
 *   C (M, N) = act(A (M, K) . B (N, K)^T + bias (N) + R (M, N)), bf16 in / out, fp32 sums,
 *   one rounding; bias (N) bf16 (bias_f32 = 0) or f32 (1) or null; R bf16 or null;
 *   relu: max(., 0) last.  Row-major, K contiguous; K % 8 == 0 (a K tail past the last multiple
 *   of 64 reads zeros), N % 8 == 0; lda, ldb, ldr,
 *   ldc multiples of 8 elements; every pointer 16-byte aligned; 256 * lda * 2 < 2^31. */
int ov3d_gemm256(const void* A, long long lda, const void* B, long long ldb, const void* bias,
                 int bias_f32, const void* R, long long ldr, void* C, long long ldc, int M, int N,
                 int K, int relu, void* stream);

/* Two products of one shape in one launch of the same kernel (the decoder's K and V
 * projections of the memory for all 8 layers, models/transformer.py:369-372):
 *   C = A B^T + bias, C2 = A2 B2^T + bias2 (no residual, no ReLU); as ov3d_gemm256 otherwise,
 *   the two problems share M, N, K and the leading dimensions; bias and bias2 both or neither. */
int ov3d_gemm256_pair(const void* A, const void* A2, long long lda, const void* B, const void* B2,
                      long long ldb, const void* bias, const void* bias2, int bias_f32, void* C,
                      void* C2, long long ldc, int M, int N, int K, void* stream);

/* nbatch products of one shape in one launch (the RegionCLIP attention pool's per-head
 * products: a_h = q_h Wk_h, o_h = y_h Wv_h^T, regionclip._pool_fused; upstream CLIP
 * AttentionPool2d k / v projections, clip.inference, criterion.py:397): problem p is
 *   C + p sC = act(A + p sA  .  (B + p sB)^T + bias + p sbias) (no residual),
 * strides in elements (multiples of 8; sbias of 4 for f32, 8 for bf16 bias); as ov3d_gemm256
 * otherwise. */
int ov3d_gemm256_batched(const void* A, long long lda, long long sA, const void* B, long long ldb,
                         long long sB, const void* bias, long long sbias, int bias_f32, void* C,
                         long long ldc, long long sC, int M, int N, int K, int nbatch, int relu,
                         void* stream);

/* 3x3 convolution (pad 1, stride 1) + bias (+ residual) (+ ReLU) as an implicit GEMM on the
 * same kernel: no column matrix [upstream CLIP ModifiedResNet Bottleneck conv2 of layer3 /
 * layer4; clip.inference, criterion.py:397]:
 *   X (nimg, H, W, Cin) NHWC bf16, Wt (Cout, 9*Cin) (ldb) the channels-last weight
 *   (Cout, ky, kx, Cin) viewed as rows, Y (nimg*H*W, Cout) (ldc) NHWC rows;
 *   column k = (ky*3 + kx)*Cin + c reads X[n, y+ky-1, x+kx-1, c], zero outside the image.
 *   Cin % 64 == 0; otherwise as ov3d_gemm256 with M = nimg*H*W, N = Cout, K = 9*Cin. */
int ov3d_conv3x3_gemm256(const void* X, int nimg, int H, int W, int Cin, const void* Wt,
                         long long ldb, const void* bias, int bias_f32, const void* R, long long ldr,
                         void* Y, long long ldc, int Cout, int relu, void* stream);

/* Streaming Y (M, N) = X (M, K) . W (N, K)^T, K = 256 or 264 (the first layer's zero-padded
 * 259 inputs), N = 256 or 264 (with K = 256: that layer's input gradient), for long row sets
 * (csrc/rows256.hip): the
 * masked encoder's interim SA 1x1 convolutions [models/model_3detr.py:377-399,
 * third_party/pointnet2/pointnet2_modules.py PointnetSAModuleVotes mlp] and their input
 * gradients.  bf16 rows, 16-byte aligned X / W / Y, ld % 8; equals ov3d_gemm256 with no bias,
 * residual or ReLU bit for bit.  counters: 2 device uints, zero, left zero by every launch (one
 * launch at a time per counter pair). */
int ov3d_rows256_supported(long long M, int N, int K);
int ov3d_rows256(const void* X, long long ldx, int K, int N, const void* W, long long ldw, void* Y,
                 long long ldy, long long M, unsigned int* counters, void* stream);
/* ov3d_rows256 of Z = bf16(relu(X * scale + shift)) (the previous layer's BatchNorm + ReLU, the
 * ov3d_rows_bn_apply arithmetic without dropout; scale / shift (256) fp32) with Z also written
 * when Z != NULL (ldz % 8): Y equals ov3d_rows_bn_apply followed by ov3d_rows256 */
int ov3d_rows256_bn(const void* X, long long ldx, const float* scale, const float* shift,
                    const void* W, long long ldw, void* Y, long long ldy, void* Z, long long ldz,
                    long long M, unsigned int* counters, void* stream);

/* LayerNorm boundary + the adjacent row GEMM in one launch (csrc/lngemm.hip), the decoder's
 * short row blocks [models/transformer.py TransformerDecoderLayer.forward_pre 355-379].
 * ov3d_lngemm_fwd: the ov3d_resnorm_fwd row pass (same arguments and outputs; C = 256, y bf16
 * or null, mean / rstd / ga / ba required) followed by out_i = epi(xsel_i W_i^T + bias_i) for
 * nprob <= 2 problems over the same rows (sel 0: xa, 1: xap; W_i (N_i, 256) bf16 rows,
 * N_i % 128 == 0; epilogue 0 none, 1 dropout_p2(relu(.)) with seed2 / site2 as
 * ov3d_rows_gemm_act).  ov3d_lngemm_bwd: the ov3d_resnorm_bwd row pass (dy bf16 required,
 * partials (ov3d_lngemm_bwd_parts(R), 4, 256) as resnorm_bwd's per-8-row blocks; the column
 * sums are left to ov3d_colsum_group) followed by dx = epi(dy W) for W (256, N) rows (the
 * branch linear's weight; epilogue 0 none, 2 the FFN mask h > 0 ? . / (1 - p2) : 0).
 * R % 32 == 0; the outputs equal the two-launch path's (resnorm + rows GEMM). */
typedef struct {
    const void* W;
    long long ldw;
    const void* bias;
    void* out;
    long long ldo;
    int N;
    int sel;
} ov3d_lngemm_problem;
int ov3d_lngemm_supported(int R, int C, int N);
int ov3d_lngemm_fwd(int R, const void* src, int src_bf16, const void* y, float dropout_p,
                    const int64_t* seed, int site, const float* ga, const float* ba,
                    const void* pos, int pos_bf16, const float* gb, const float* bb, float eps,
                    float* s, float* mean, float* rstd, void* xa, void* xap, void* xb, int xb_bf16,
                    long long xb_inner, long long xb_s0, long long xb_s1, int nprob,
                    const ov3d_lngemm_problem* probs, int epilogue, float dropout_p2,
                    const int64_t* seed2, int site2, void* stream);
int ov3d_lngemm_bwd_parts(int R);
/* measurement only: ov3d_lngemm_fwd launches after this write 5 per-wave phase clocks
 * (s_memtime) into buf, 8 words a wave; NULL disarms */
int ov3d_lngemm_stamps_arm(void* buf);
int ov3d_lngemm_bwd(int R, const float* s, const float* mean, const float* rstd, const float* ds,
                    const void* dxa, const void* dxap, const void* dxb, int dxb_bf16,
                    long long dxb_inner, long long dxb_s0, long long dxb_s1, const float* ga,
                    const float* gb, float dropout_p, const int64_t* seed, int site, float* dsrc,
                    void* dy, void* dpos, int dpos_bf16, float* partials, int accumulate,
                    const void* W, long long ldw, int N, int epilogue, float dropout_p2,
                    const void* H, long long ldh, void* dx, long long lddx, void* stream);

/* ---- Flash attention (head_dim 64, bf16, no mask) ----
 * Replaces the nn.MultiheadAttention core of models/transformer.py:223,271 (encoder
 * self-attention) and :307-308,365-372 (decoder self / cross attention): per head
 * O = dropout(softmax(scale Q K^T)) V.  Q/K/V/O rows in the reference's seq-first
 * layout: element (l, b, h, d) at ptr[(l*B + b)*stride + h*64 + d] (strides in
 * elements), so projection outputs are read in place.  Lq % 32 == 0.
 * Dropout: keep(q, k) from a counter-based hash of (*seed, site, b*H + h, q, k>>1)
 * (signed 16-bit half per key, keep iff (half ^ 0x8000) >= round(p * 65536)).  The
 * forward stores the drop bits (dropbits, ov3d_attn_dropbits_words() uint32 words, needed
 * when p > 0) and the backward reads them.  lse (B*H, Lq) f32 = log2-domain logsumexp
 * saved for the backward.  nsplit > 1 splits the keys over workgroups (decoder: 128
 * queries) and needs ov3d_attn_fwd_workspace() floats of workspace. */
int ov3d_attn_fwd(const void* q, const void* k, const void* v, long long sq, long long sk,
                  long long sv, int B, int H, int Lq, int Lk, float scale, float dropout_p,
                  const int64_t* seed, int site, void* o, long long so, float* lse,
                  uint32_t* dropbits, float* workspace, int nsplit, void* stream);
long long ov3d_attn_fwd_workspace(int B, int H, int Lq, int Lk, int nsplit);
/* uint32 words of the drop bits: query-major [nkt][B*H][Lq][2] then key-major
 * [Lq/32][B*H][nkt*64], nkt = ceil(Lk / 64); 0 for invalid shapes. */
long long ov3d_attn_dropbits_words(int B, int H, int Lq, int Lk);
/* Backward: dq/dk/dv rows (same layout, bf16) from o, dout (stride sdo), lse and the
 * forward's drop bits; dvec (B*H, Lq) f32 scratch receives D = rowsum(dout * o).
 * dk = dv = NULL computes dQ and D only (dK / dV later by ov3d_attn_bwd_dkdv_batch).
 * nsplit > 1 splits the dQ key loop over workgroups (fp32 partials in `workspace`, sized
 * as for the forward by ov3d_attn_fwd_workspace). */
int ov3d_attn_bwd(const void* q, const void* k, const void* v, long long sq, long long sk,
                  long long sv, const void* o, long long so, const void* dout, long long sdo,
                  const float* lse, int B, int H, int Lq, int Lk, float scale, float dropout_p,
                  const uint32_t* dropbits, float* dvec, void* dq, long long sdq, void* dk,
                  long long sdk, void* dv, long long sdv, float* workspace, int nsplit,
                  void* stream);

/* dK / dV of several ov3d_attn_bwd calls of one shape in one launch (the decoder's cross
 * attentions, deferred to the end of the decoder backward): each job is what
 * ov3d_attn_bwd would have read for it, with dvec already written by an ov3d_attn_bwd call
 * with dk = dv = NULL (dQ and D only). */
typedef struct {
    const void* q; long long sq; const void* k; long long sk; const void* v; long long sv;
    const void* dout; long long sdo; const float* lse; const float* dvec;
    const uint32_t* dropbits; void* dk; long long sdk; void* dv; long long sdv;
} ov3d_attn_dkdv_job;
int ov3d_attn_bwd_dkdv_batch(const ov3d_attn_dkdv_job* jobs, int njobs, int B, int H, int Lq,
                             int Lk, float scale, float dropout_p, void* stream);

/* Short attentions (Lq, Lk <= 128, one key split, no mask: the decoder self attention) run
 * their whole ov3d_attn_bwd in one launch (dQ, then dK / dV in the same workgroup).
 * on = 0 / 1 selects the two-launch / one-launch form, -1 only queries; returns the
 * previous setting (host-only). */
int ov3d_attn_small_bwd(int on);

/* ---- Masked attention (the masked encoder) ----
 * Replaces the (B*H, L, L) boolean attn_mask of MaskedTransformerEncoder
 * (models/transformer.py:152-190: mask = cdist(xyz, xyz) >= radius, tiled to the heads,
 * True = not attended) given to nn.MultiheadAttention.  ov3d_attn_mask_pack packs a
 * (B, Lq, Lk) row-major source, shared by the heads, into ov3d_attn_maskbits_words() uint32
 * words (query-major [nkt][B][Lq][2] then key-major [Lq/32][B][nkt*64]): kind 0 = uint8
 * mask (nonzero = not attended), kind 1 = fp32 distances (not attended iff d >= thr),
 * kind 2 = fp32 squared distances g of torch.cdist's matmul form, before its
 * clamp_min(0).sqrt() (not attended iff sqrt(max(g, 0)) >= thr: the bits of kind 1 on cdist),
 * kind 3 = the same bits from the points: src (B, L, 4) fp32 rows (x, y, z, |p|^2 as
 * x.pow(2).sum(-1)), Lq == Lk == L, 16-byte aligned; g formed as the fma chain of cdist's
 * K = 5 GEMM (bit-identical to it), no (B, L, L) distance matrix.
 * The _masked entry points take the words (NULL = no mask) and are otherwise
 * ov3d_attn_fwd / ov3d_attn_bwd.  A query with no attended key gets O = 0 and zero
 * gradients (the reference's softmax would give NaN). */
long long ov3d_attn_maskbits_words(int B, int Lq, int Lk);
int ov3d_attn_mask_pack(const void* src, int kind, float thr, int B, int Lq, int Lk,
                        uint32_t* words, void* stream);
int ov3d_attn_fwd_masked(const void* q, const void* k, const void* v, long long sq, long long sk,
                         long long sv, int B, int H, int Lq, int Lk, float scale, float dropout_p,
                         const int64_t* seed, int site, void* o, long long so, float* lse,
                         uint32_t* dropbits, float* workspace, int nsplit,
                         const uint32_t* maskbits, void* stream);
/* the same forward with this call's drop bits already in dropbits (ov3d_attn_dropgen of the
 * same seed / site / shape, e.g. on another stream ahead of time): no hash in the forward
 * (dropout_p > 0 required) */
int ov3d_attn_fwd_pregen(const void* q, const void* k, const void* v, long long sq, long long sk,
                         long long sv, int B, int H, int Lq, int Lk, float scale, float dropout_p,
                         const int64_t* seed, int site, void* o, long long so, float* lse,
                         uint32_t* dropbits, float* workspace, int nsplit, const uint32_t* maskbits,
                         void* stream);
/* the drop bits of an attention forward (both layouts, ov3d_attn_dropbits_words words) */
int ov3d_attn_dropgen(int B, int H, int Lq, int Lk, float dropout_p, const int64_t* seed, int site,
                      uint32_t* dropbits, void* stream);
int ov3d_attn_bwd_masked(const void* q, const void* k, const void* v, long long sq, long long sk,
                         long long sv, const void* o, long long so, const void* dout, long long sdo,
                         const float* lse, int B, int H, int Lq, int Lk, float scale,
                         float dropout_p, const uint32_t* dropbits, float* dvec, void* dq,
                         long long sdq, void* dk, long long sdk, void* dv, long long sdv,
                         float* workspace, int nsplit, const uint32_t* maskbits, void* stream);

/* ---- Linear-layer weight / bias gradient ----
 * For every row-major dense layer y = x W^T + b of the step (transformer projections
 * and FFNs, GenericMLP heads / projections; models/transformer.py, models/helpers.py):
 *   dW (N, K) f32 (leading dim ldw) = dy^T x,  db (N) f32 = column sums of dy (db may be NULL)
 *   dy (R, N) bf16 (row stride ldy), x (R, K) bf16 (row stride ldx).
 * MFMA over row chunks; nsplit > 1 partials are summed in a fixed order by a second
 * launch (deterministic).  workspace: ov3d_wgrad_workspace() floats; counters: unused
 * (reserved, may be NULL). */
int ov3d_wgrad(const void* dy, long long ldy, const void* x, long long ldx, int R, int N, int K,
               float* dW, long long ldw, float* db, float* workspace, int* counters, int nsplit,
               void* stream);
/* ov3d_wgrad with x = bf16(relu(x_stored * scale + shift)) per input channel (the previous
 * layer's BatchNorm + ReLU applied on load, ov3d_rows_bn_apply's arithmetic; K % 8 == 0, 16-byte
 * aligned x rows): the weight gradient of ov3d_rows256_bn's product without its Z rows */
int ov3d_wgrad_bn(const void* dy, long long ldy, const void* x, long long ldx, int R, int N, int K,
                  const float* scale, const float* shift, float* dW, long long ldw, float* db,
                  float* workspace, int* counters, int nsplit, void* stream);
long long ov3d_wgrad_workspace(int R, int N, int K, int nsplit);
/* several independent weight gradients in one launch (+ one split reduction launch) per
 * 28 problems: the deferred dW / db of a backward pass (gemm.py).  256 x 256 tiles,
 * stream-K over (problem, tile, 32-row stage) units with one workgroup per CU; `nsplit`
 * is not used.  workspace: ov3d_wgrad_group_workspace() floats. */
typedef struct {
    const void* dy; long long ldy; const void* x; long long ldx;
    int R, N, K, nsplit;
    float* dW; long long ldw; float* db;
} ov3d_wgrad_problem;
long long ov3d_wgrad_group_workspace(const ov3d_wgrad_problem* probs, int n);
int ov3d_wgrad_group(const ov3d_wgrad_problem* probs, int n, float* workspace, void* stream);
int ov3d_wgrad_tiles(int N, int K);
/* output tiles of one problem in ov3d_wgrad_group (256 x 256 tiles, 512-thread workgroups) */
int ov3d_wgrad_group_tiles(int N, int K);

/* ---- Training BatchNorm1d + ReLU + Dropout over channels-last rows ----
 * The GenericMLP prediction heads (models/helpers.py:45-112, built by
 * models/model_3detr.py _build_heads) evaluated as one MLP over 5*256 channels.
 * Every operand's channel c of row r lives at base + (c/cb)*bstride + r*ld + (c%cb)
 * (row-major: cb = C, bstride = 0; per-head blocks of a batched GEMM: cb = 256,
 * ld = 256, bstride = R*256).  C % 8 == 0.  Dropout: hash of (*seed, site, r, c).
 * stats: partials (nparts, 2, C) f64 of sum x, sum x^2 (then ov3d_reduce_partials,
 *        ov3d_bn_finalize) */
int ov3d_rows_bn_stats(const void* x, int is_bf16, long long ld, long long bstride, int cb,
                       long long R, int C, double* partials, int nparts, void* stream);
/* apply: out (bf16) = dropout(relu(x*scale + shift)) */
int ov3d_rows_bn_apply(const void* x, int is_bf16, long long ld, long long bstride, int cb,
                       long long R, int C, const float* scale, const float* shift,
                       float dropout_p, const int64_t* seed, int site, void* out, long long ldo,
                       long long bstride_o, int cbo, void* stream);
/* backward, dt = dz * keep/(1-p) * [x*scale+shift > 0]:
 * pass 0: partials (nparts, 2, C) of sum dt, sum dt*(x-mean)*invstd (then
 *         ov3d_reduce_partials, ov3d_bn_bwd_finalize -> cA, cB, cC, dgamma, dbeta);
 * pass 1: dx (bf16) = cA*dt + cB*x + cC */
int ov3d_rows_bn_bwd(int pass, const void* dz, long long ldz, long long bstride_z, int cbz,
                     const void* x, int x_bf16, long long ldx, long long bstride_x, int cbx,
                     long long R, int C, const float* scale, const float* shift, const float* mean,
                     const float* invstd, const float* cA, const float* cB, const float* cC,
                     float dropout_p, const int64_t* seed, int site, double* partials, int nparts,
                     void* dx, long long ldd, long long bstride_d, int cbd, void* stream);
/* ov3d_rows_bn_bwd (row-major bf16 x, no dropout) with dz the dense gradient of the neighbour
 * max-pool rebuilt from its pooled gradient g (P, C) bf16 and arg rows (P, C) uint8 (row
 * p * S + s takes g[p] where arg == s): the backward of ov3d_nbr_max_bnrelu_fwd */
int ov3d_rows_bn_bwd_pooled(int pass, const void* g, const uint8_t* arg, int S, const void* x,
                            long long R, int C, const float* scale, const float* shift,
                            const float* mean, const float* invstd, const float* cA,
                            const float* cB, const float* cC, double* partials, int nparts,
                            void* dx, void* stream);


/* ---- Set-criterion losses (criterion.py SetCriterion.forward, all decoder layers) ----
 * Replaces criterion.py:143-337 (loss_sem_cls, loss_angle, loss_center, loss_size,
 * loss_giou), 121-130 (loss_cardinality) and the weighting / layer sum of 402-442.
 * Proposal (l, b, q) is row (l*B + b)*Q + q of every (L*B*Q, n) operand (row stride ld_*).
 * Dict columns: OV3D_LOSS_COL_* ; dict row i = layer final, aux 0, aux 1, ... */
#define OV3D_LOSS_SEM 1
#define OV3D_LOSS_CENTER 2
#define OV3D_LOSS_SIZE 4
#define OV3D_LOSS_GIOU 8
#define OV3D_LOSS_ALIGN 16
#define OV3D_LOSS_NCOLS 8   /* sem, angle_cls, angle_reg, center, size, giou, 2dalignment, cardinality */
#define OV3D_LOSS_MAX_B 256
typedef struct {
    int L, B, Q, G, T, NB;
    int flags;             /* OV3D_LOSS_* terms computed (angle cls / reg always) */
    int final_last;        /* 1: computation layer L-1 is the final layer; 0: layer 0 is */
    int match_ref_order;   /* inds / matched rows in the reference's problem order (final first) */
    const float* logits;        long long ld_logits;        /* (L*B*Q, T) */
    const float* angle_logits;  long long ld_angle_logits;  /* (L*B*Q, NB) */
    const float* angle_res;     long long ld_angle_res;     /* (L*B*Q, NB), normalised */
    const float* center;        long long ld_center;        /* (L*B*Q, 3) normalised */
    const float* size;          long long ld_size;          /* (L*B*Q, 3) normalised */
    const float* gious;         /* (L*B, Q, G) or NULL */
    const int64_t* inds;        /* (L*B, Q) matched GT slot */
    const float* matched;       /* (L*B, Q) 0/1 */
    const int64_t* gt_sem;      /* (B, G) */
    const int64_t* gt_angle_cls;  /* (B, G) */
    const float* gt_angle_res;  /* (B, G) radians */
    const float* gt_center;     /* (B, G, 3) normalised */
    const float* gt_size;       /* (B, G, 3) normalised */
    const int64_t* nactual;     /* (B,) */
    const float* cls_weights;   /* (T,) */
    const float* num_boxes;     /* device scalar */
    const float* align;         /* (L,) per-layer 2D alignment sums or NULL */
    float dict_w[OV3D_LOSS_NCOLS];   /* dict value = per-layer term * dict_w */
    float total_w[OV3D_LOSS_NCOLS];  /* d total / d term (0 = not in the total) */
    int total_order[OV3D_LOSS_NCOLS]; int n_total;   /* summation order of the total */
    float res_scale;            /* 1 / (float)(pi / NB) */
    const int* match_status;    /* (n_status,) ov3d_hungarian status or NULL: any nonzero
                                 * (NaN / infeasible cost, where scipy raises) -> total = NaN,
                                 * so engine.py's non-finite-loss exit fires */
    int n_status;
} ov3d_set_loss_desc;
/* raw: (L, 9) f32 workspace (kept for the backward); ticket: one int, zero before the first
 * call (the kernel resets it); dict_out (L, 8); total: scalar */
/* Hungarian matcher cost (criterion.py:33-92 Matcher.cost with the center cdist(p=1) of
 * 357-360) for P = L*B problems: prob (P, Q, C) row stride ldp, obj (P, Q), center (P, Q, 3),
 * gious (P, Q, G), gt_center (B, G, 3), gt_label (B, G) -> cost (P, Q, G), written in the
 * reference's problem order (final layer first) when final_last (layer l of the inputs is
 * the computation order with the final layer last) */
int ov3d_matcher_cost(int P, int B, int Q, int G, int C, int final_last, const float* prob,
                      long long ldp,
                      const float* obj, const float* center, const float* gious,
                      const float* gt_center, const int64_t* gt_label, float w_cls, float w_obj,
                      float w_center, float w_giou, float* cost, void* stream);
/* target counts (criterion.py:346-352, 425): nactual per scene (int64, and int32 repeated for
 * the L layers), the replica's total, num_boxes = max(total, 1) (single process; NULL to
 * skip) and the rotated flag (any GT angle > 0) */
int ov3d_targets_prep(int B, int G, int L, const float* present, const float* angles,
                      int64_t* nact64, int32_t* nact32_rep, int64_t* total, float* num_boxes,
                      int32_t* rotated, void* stream);
long long ov3d_set_loss_desc_size(void);   /* sizeof(ov3d_set_loss_desc), for FFI layout checks */
int ov3d_set_loss_fwd(const ov3d_set_loss_desc* desc, float* raw, int* ticket, float* dict_out,
                      float* total, void* stream);
/* The same split over the proposals (the per-layer launch is latency-bound): with T, NB <= 32
 * and L <= 32, 16 lanes per proposal row on workgroups of 16 rows, then a one-workgroup launch
 * that adds the chunks and finalises (ticket unused); otherwise a workgroup per (256 proposals,
 * layer) whose last workgroup finalises.  parts: ov3d_set_loss_fwd_parts(L, B, Q) doubles of
 * scratch.  The chunk sums are added in chunk order: deterministic, equal to the per-layer form
 * up to fp64 rounding. */
long long ov3d_set_loss_fwd_parts(int L, int B, int Q);
int ov3d_set_loss_fwd_split(const ov3d_set_loss_desc* desc, float* raw, int* ticket,
                            float* dict_out, float* total, double* parts, void* stream);
/* d_dict (L, 8) or NULL, d_total scalar (device) or NULL; every non-NULL gradient is written
 * in full (contiguous (L*B*Q, n), g_gious (L*B, Q, G), g_align (L,)); 16 lanes per proposal
 * row when T, NB <= 32 and L <= 32, else a thread per row */
int ov3d_set_loss_bwd(const ov3d_set_loss_desc* desc, const float* raw, const float* d_dict,
                      const float* d_total, float* g_logits, float* g_angle_logits,
                      float* g_angle_res, float* g_center, float* g_size, float* g_gious,
                      float* g_align, void* stream);


/* ---- Residual add + dropout + LayerNorm (pre-norm transformer layers) ----
 * Replaces models/transformer.py:262-280 / 355-379 `x = x + dropout(branch)` followed by the
 * next sub-layer's `norm(x)` (+ pos), and the decoder's per-layer final norm (124-133).
 * Contiguous (R, C) rows, C/8 a power of two <= 64.  Dropout: hash of (*seed, site, r, c).
 *   s = src + dropout(y) (fp32); xa = bf16(LN_a(s)); xap = bf16(LN_a(s) + pos); xb = LN_b(s) (fp32)
 * src / y / pos may be NULL (zero / absent); outputs NULL = not wanted. */
int ov3d_resnorm_supported(int C);
int ov3d_resnorm_fwd(long long R, int C, const void* src, int src_bf16, const void* y, int y_bf16,
                     float dropout_p, const int64_t* seed, int site, const float* ga,
                     const float* ba, const void* pos, int pos_bf16, const float* gb,
                     const float* bb, float eps, float* s, float* mean, float* rstd, void* xa,
                     void* xap, void* xb, int xb_bf16, long long xb_inner, long long xb_s0,
                     long long xb_s1, void* stream);
/* xb (fp32, or bf16 when xb_bf16) rows; xb_inner > 0: row r written at
 * (r / xb_inner) * xb_s0 + (r % xb_inner) * xb_s1 (the decoder writes its layer outputs
 * straight into the heads' (layer, scene, query) rows).
 * backward: ds (fp32, grad of s from its other consumers) or NULL, dxa / dxap (bf16),
 * dxb (fp32, or bf16 when dxb_bf16) or NULL -> dsrc (fp32), dy (bf16 | fp32), dpos (= dxap),
 * dga/dba/dgb/dbb.
 * dxb_inner > 0: dxb row r lives at (r / dxb_inner) * dxb_s0 + (r % dxb_inner) * dxb_s1
 * (a strided (L, B, C) view, e.g. one layer of the stacked decoder outputs' gradient);
 * dxb_inner = 0: contiguous rows.
 * accumulate (bit mask): 1 dpos, 2 dga/dba, 4 dgb/dbb are added to (old + new) instead of
 * written — one gradient buffer shared by the calls that use the same pos / norm (the
 * decoder: query_pos in 16 calls, the decoder norm in 8), summed in backward order as
 * autograd's fan-in would.
 * partials: (nparts, 4, C) f32 workspace with nparts = ov3d_resnorm_bwd_parts(R, C). */
int ov3d_resnorm_bwd_parts(long long R, int C);
/* The LayerNorm weight / bias gradients of a backward pass in one launch: the resnorm
 * backward calls leave their (nparts, 4, C) partials (column blocks k = 0 dga, 1 dba,
 * 2 dgb, 3 dbb) and ov3d_colsum_group writes every output = the ordered sum over its
 * segments of each segment's column total (the ov3d_resnorm_bwd colsum, then the
 * accumulate adds: bit-identical). */
typedef struct {
    const float* partials;
    int nparts;
    int k;
} ov3d_colsum_seg;
typedef struct {
    float* dst;      /* (C) */
    int first_seg;   /* segments [first_seg, first_seg + nseg) of segs */
    int nseg;
} ov3d_colsum_out;
int ov3d_colsum_group(const ov3d_colsum_seg* segs, int nseg, const ov3d_colsum_out* outs, int nout,
                      int C, void* stream);
/* FFN activation h = dropout(relu(y)) over contiguous bf16 (R, C) rows (transformer.py
 * FFN), dropout keep = hash of (*seed, site, r, c); backward dy = dh / (1-p) where h > 0 */
int ov3d_relu_dropout_fwd(const void* y, long long R, int C, float dropout_p, const int64_t* seed,
                          int site, void* h, void* stream);
int ov3d_relu_dropout_bwd(const void* h, const void* dh, long long n, float dropout_p, void* dy,
                          void* stream);
int ov3d_resnorm_bwd(long long R, int C, const float* s, const float* mean, const float* rstd,
                     const float* ds, const void* dxa, const void* dxap, const void* dxb,
                     int dxb_bf16, long long dxb_inner, long long dxb_s0, long long dxb_s1,
                     const float* ga, const float* gb, float dropout_p, const int64_t* seed,
                     int site, float* dsrc, void* dy, int dy_bf16, void* dpos, int dpos_bf16,
                     float* partials, int nparts, float* dga, float* dba, float* dgb, float* dbb,
                     int accumulate, void* stream);


/* ---- Gradient clipping + AdamW over all parameter tensors (3 launches) ----
 * Replaces engine.py:104-112 torch.nn.utils.clip_grad_norm_(params, max_norm) +
 * torch.optim.AdamW.step() (main.py optimizer), torch's fused ADAMW arithmetic.
 * table[i]: one parameter tensor (fp32 param / grad / exp_avg / exp_avg_sq, optional bf16
 * shadow); workgroup b updates elements [blk_c[b]*chunk, +chunk) of tensor blk_t[b]
 * (chunk = ov3d_adamw_chunk()).  partials: (nblocks) f64 workspace; step: device scalar
 * (incremented); coefs (4) f64 out: clip multiplier, 1-b1^t, sqrt(1-b2^t), grad norm.
 * max_norm <= 0: no clipping.  write_grad: store the clipped gradient back.  grad_scale:
 * gradients are multiplied by it first (1/world after an all-reduce sum: DDP's mean). */
typedef struct {
    float* param; float* grad; float* exp_avg; float* exp_avg_sq;
    void* shadow;            /* bf16 copy of param or NULL */
    long long numel;
    int group;               /* parameter group: row of the hyper table */
    int reserved;
} ov3d_adamw_tensor;
int ov3d_adamw_chunk(void);
/* the dropout seed of a training forward (attention.py next_step): *live += 1, *snap = *live
 * (int64 device scalars), one launch */
int ov3d_seed_next(long long* live, long long* snap, void* stream);
/* n device-to-device copies (bytes[i] from srcs[i] to dsts[i], host arrays) in one launch
 * per 120 (the step graph's static input batch, the flat gradient buffer) */
int ov3d_multi_copy(int n, const void* const* srcs, void* const* dsts, const long long* bytes,
                    void* stream);
/* sum = bf16(a + b) in fp32 (a: fp32, or bf16 when a_bf16; b fp32) and, for a fp32, ac = bf16(a)
 * (NULL: skipped), n elements (n % 8 == 0, 16-byte aligned): the decoder's memory + pos and
 * memory rows (transformer._MemoryKV) in one pass */
int ov3d_add_cast_bf16(const void* a, int a_bf16, const float* b, long long n, void* sum, void* ac,
                       void* stream);
/* *out = a new non-blocking HIP stream owned by the caller (never destroyed by the library).
 * Replaces nothing in the reference (torch.cuda.Stream() hands out pool streams, which recycle):
 * graphs.StepGraph and dist.GradBuckets use streams of their own so that no stream that carried
 * an eager collective ever joins a graph capture (the watchdog abort). */
int ov3d_stream_create(void** out);
/* table[i].grad = grads[i] (host array of device pointers) by kernel arguments: graph-safe */
int ov3d_adamw_set_grads(ov3d_adamw_tensor* table, int ntensors, float* const* grads, void* stream);
/* hyper: DEVICE (ngroups, 2) f64 table {lr, weight_decay} per parameter group, read by the
 * update launch (a captured step graph follows lr schedules: the caller rewrites the table
 * before each replay, engine.py:79 adjust_learning_rate) */
int ov3d_adamw_step(const ov3d_adamw_tensor* table, const int* blk_t, const int* blk_c, int nblocks,
                    double* partials, float max_norm, float* step, double beta1, double beta2,
                    float eps, double* coefs, int write_grad, float grad_scale,
                    const double* hyper, void* stream);


/* ---- Box parametrisation of the heads (model_3detr.py BoxProcessor + corners) ----
 * raw: (R, ld) rows [center 3 | size 3 | angle logits NB | angle residual NB], R = L*B*Q
 * rows (l, b, q); qxyz (B, Q, 3), dmin / dmax (B, 3); logits (R, T) or NULL (no probs).
 * Outputs (R, ...) contiguous fp32: center_n / center_u / size_n / size_u (3), angle
 * logits / residual_normalized / residual (NB), angle (1), corners (8, 3), sem_prob (T-1),
 * objectness (1).  Backward: any gradient may be NULL; writes draw (R, ldd) columns 0..6+2NB. */
/* Fourier position embedding (position_embedding.py:89-118): xyz (B, N, 3), optional scene
 * range dmin / dmax (B, 3) (both or neither), gauss_B (3, ldb) first d columns ->
 * out (B, N, 2d) = [sin | cos] of (normalised xyz * 2 pi) @ gauss_B; seq_first != 0: out
 * (N, B, 2d), the transformer's sequence-first rows */
int ov3d_fourier_pe(const float* xyz, int B, int N, const float* dmin, const float* dmax,
                    const float* gauss_b, int ldb, int d, int seq_first, float* out, void* stream);
int ov3d_box_param_fwd(long long R, int B, int Q, int NB, int T, const float* raw, long long ld,
                       const float* qxyz, const float* dmin, const float* dmax,
                       const float* logits, float* center_n, float* center_u, float* size_n,
                       float* size_u, float* alog, float* ares_n, float* ares, float* angle,
                       float* corners, float* sem_prob, float* obj_prob, void* stream);
int ov3d_box_param_bwd(long long R, int B, int Q, int NB, const float* raw, long long ld,
                       const float* qxyz, const float* dmin, const float* dmax,
                       const float* g_center_n, const float* g_center_u, const float* g_size_n,
                       const float* g_size_u, const float* g_alog, const float* g_ares_n,
                       const float* g_ares, const float* g_angle, const float* g_corners,
                       float* draw, long long ldd, void* stream);

/* ---- short row-block GEMMs (csrc/rowsgemm.hip): the decoder's nn.Linear layers ----
 * Replaces the library GEMMs under F.linear / the input-gradient matmul of
 * models/transformer.py:355-379 (M = nqueries * batch rows).  bf16 in / out, fp32 sums:
 *   trans_b = 1: C (M x N) = A (M x K) W^T + bias   W (N x K) row-major (nn.Linear weight)
 *   trans_b = 0: C (M x N) = A (M x K) W             W (K x N) row-major (bias must be NULL)
 * N % 32 == 0, K % 64 == 0, K <= 1024; 16-byte aligned A / W, lda / ldw % 8 == 0,
 * ldc % 4 == 0; bias (N) bf16 or NULL. */
int ov3d_rows_gemm_supported(int M, int N, int K);
int ov3d_rows_gemm(int M, int N, int K, const void* A, long long lda, const void* W,
                   long long ldw, int trans_b, const void* bias, void* C, long long ldc,
                   void* stream);
/* the same with the transformer FFN activation fused into the epilogue:
 *   epilogue 1: C = dropout_p(relu(bf16(A W^T + bias)))  (keep = hash of (*seed, site, row,
 *               column) as ov3d_relu_dropout_fwd — identical output)
 *   epilogue 2: C = H > 0 ? bf16(bf16(A W) / (1 - dropout_p)) : 0  (H: the activation
 *               output, (M x N) bf16 rows of ldh; as ov3d_relu_dropout_bwd)
 *   epilogue 0: ov3d_rows_gemm. */
/* up to 4 problems over the same M rows in one launch (the in-projection blocks of one
 * attention); each as ov3d_rows_gemm with the common trans_b */
typedef struct {
    const void* A; long long lda;
    const void* W; long long ldw;
    const void* bias;   /* bf16 (N) or NULL */
    void* C; long long ldc;
    int N, K;
} ov3d_rows_gemm_problem;
int ov3d_rows_gemm_group(int M, int n, const ov3d_rows_gemm_problem* probs, int trans_b,
                         void* stream);
int ov3d_rows_gemm_act(int M, int N, int K, const void* A, long long lda, const void* W,
                       long long ldw, int trans_b, const void* bias, int epilogue,
                       float dropout_p, const int64_t* seed, int site, const void* H,
                       long long ldh, void* C, long long ldc, void* stream);

/* ---- long row-block GEMMs (csrc/tilegemm.hip): the encoder's nn.Linear layers ----
 * Replaces the library GEMMs under F.linear / the input-gradient matmul of
 * models/transformer.py:262-278 (M = batch * 2048 points).  Same contract as
 * ov3d_rows_gemm (trans_b = 1: C = A W^T + bias; trans_b = 0: C = A W, bias NULL), with a
 * 128 (or 64) x 128 output tile per workgroup: N % 128 == 0, K % 64 == 0; 16-byte aligned
 * A / W / C, lda / ldw / ldc % 8 == 0; bias (N <= 2048) bf16, 8-byte aligned, or NULL.
 * Also the decoder's memory K/V projections (models/transformer.py:355-379, all layers in one
 * N = layers x 256 GEMM) and the heads' 8192-row layers. */
int ov3d_tile_gemm_supported(int M, int N, int K);
int ov3d_tile_gemm(int M, int N, int K, const void* A, long long lda, const void* W,
                   long long ldw, int trans_b, const void* bias, void* C, long long ldc,
                   void* stream);
/* with the FFN activation epilogues of ov3d_rows_gemm_act (1: dropout(relu(.)), 2: the
 * masked input gradient; H 8-byte aligned, ldh % 4 == 0): the encoder's FFN */
int ov3d_tile_gemm_act(int M, int N, int K, const void* A, long long lda, const void* W,
                       long long ldw, int trans_b, const void* bias, int epilogue,
                       float dropout_p, const int64_t* seed, int site, const void* H,
                       long long ldh, void* C, long long ldc, void* stream);
/* C = A1 op(W1) + A2 op(W2) in one launch (K1, K2 each a multiple of 64; lda2 == lda1,
 * ldw2 == ldw1; no bias): the
 * memory gradient of the decoder's batched K / V projections, d memory = dK Wk + dV Wv
 * (models/transformer.py:365-372 backward) */
int ov3d_tile_gemm2(int M, int N, int K1, const void* A1, long long lda1, const void* W1,
                    long long ldw1, int K2, const void* A2, long long lda2, const void* W2,
                    long long ldw2, int trans_b, void* C, long long ldc, void* stream);
/* batch independent products C_b = A_b op(W_b) (no bias), operands at element strides
 * sA / sW / sC per batch (multiples of 8, sC >= M * ldc): the heads' per-head second layer
 * and its input gradient (models/helpers.py GenericMLP x 5 heads, torch.bmm in heads.py) */
int ov3d_tile_gemm_batched(int batch, int M, int N, int K, const void* A, long long lda,
                           long long sA, const void* W, long long ldw, long long sW, int trans_b,
                           void* C, long long ldc, long long sC, void* stream);

/* ---- SUN RGB-D training-data pipeline on the device (csrc/sunaug.hip) ----
 * Replaces SunrgbdDetectionDataset.__getitem__ (datasets/sunrgbd.py:256-462, use_color /
 * use_height off) for a batch of scenes resident in HBM: raw points (S, raw_stride, raw_c)
 * of float32 (pc_f64 = 0) or float64, raw boxes (S, k_stride, 8) float64; scene_idx (B)
 * selects the batch.  The random draws are the reference's numpy draws, made on the host
 * (sunaug.py) and passed in:
 *   params   (B, 8) f64: flip flag, rot_angle, cos(rot_angle), sin(rot_angle), scale_ratio
 *   attempts (B, A, 4) f64: RandomCuboid crop_range xyz + centre index (< 0: the attempt
 *            failed check_aspect), random_cuboid.py:45-53
 *   choices  (B, num_points) int64: np.random.choice of random_sampling (pc_util.py:28)
 * Entry points, in stream order:
 *   ov3d_sun_aug_points : flip / rotz / scale of the points (sunrgbd.py:309-344) ->
 *                         out (B, n_max, 3) T and range_part (B, ov3d_sun_range_parts(n_max), 6)
 *   ov3d_sun_aug_boxes  : support-class filter (train, sunrgbd.py:266-268; n_support = 0 for
 *                         val) of each scene's first ngt[b] boxes (ngt NULL: all of them; the
 *                         rest are use_pbox pseudo boxes, appended unfiltered, :269-271) + the
 *                         same transforms of the boxes -> out (B, k_max, 8), out_n
 *   ov3d_sun_cuboid_eval: all A attempts of RandomCuboid (min_points, box filter "center"),
 *                         counts / accept (B, A), crop_mm (B, A, 6) T, and
 *                         sel (B, 2) int32 = [first accepted attempt or -1, points to sample]
 *   ov3d_sun_crop_sample: order-preserving crop (crop_idx (B, n_max)) + random_sampling gather
 *                         -> points (B, num_points, 3) f32, dims_part (B, range_parts(num_points), 6)
 *   ov3d_sun_labels     : box filter of the selected crop + every label tensor of the
 *                         reference's ret_dict (sunrgbd.py:356-460). */
int ov3d_sun_range_parts(int n);
int ov3d_sun_aug_points(const void* raw, int pc_f64, long long raw_stride, int raw_c,
                        const int32_t* scene_idx, const int32_t* npts, int B, int n_max,
                        const double* params, int augment, void* out, void* range_part,
                        void* stream);
int ov3d_sun_aug_boxes(const double* raw, long long k_stride, const int32_t* scene_idx,
                       const int32_t* nbox, const int32_t* ngt, int B, int k_max,
                       const double* params, int augment, const double* support, int n_support,
                       double* out, int32_t* out_n, void* stream);
int ov3d_sun_cuboid_eval(const void* pts, int pc_f64, int n_max, const int32_t* npts,
                         const void* range_part, const double* attempts, int B, int A,
                         int min_points, const double* boxes, const int32_t* nbox, int k_max,
                         int32_t* counts, void* crop_mm, int32_t* accept, int32_t* sel,
                         void* stream);
int ov3d_sun_crop_sample(const void* pts, int pc_f64, int n_max, const int32_t* npts,
                         const void* range_part, const double* attempts, int B, int A,
                         const int32_t* sel, const int64_t* choices, int num_points,
                         int32_t* crop_idx, float* out, void* dims_part, void* stream);
typedef struct {
    int B, max_num_obj, k_max, num_angle_bin, num_attempts, n_dims_part;
    const double* boxes;      /* (B, k_max, 8) augmented boxes */
    const int32_t* nbox;      /* (B) */
    const int32_t* sel;       /* (B, 2) of ov3d_sun_cuboid_eval, or NULL (no RandomCuboid) */
    const void* crop_mm;      /* (B, num_attempts, 6) T */
    const void* dims_part;    /* (B, n_dims_part, 6) T */
    void* dims_min;           /* (B, 3) T: point_cloud_dims_min */
    void* dims_max;           /* (B, 3) T */
    float* corners;           /* (B, G, 8, 3) gt_box_corners */
    float* centers;           /* (B, G, 3) gt_box_centers */
    float* centers_normalized;/* (B, G, 3) */
    int64_t* sem_cls;         /* (B, G) gt_box_sem_cls_label */
    float* present;           /* (B, G) gt_box_present */
    float* sizes;             /* (B, G, 3) gt_box_sizes */
    float* sizes_normalized;  /* (B, G, 3) */
    float* angles;            /* (B, G) gt_box_angles */
    int64_t* angle_cls;       /* (B, G) gt_angle_class_label */
    float* angle_res;         /* (B, G) gt_angle_residual_label */
} ov3d_sun_labels_args;
int ov3d_sun_labels(const ov3d_sun_labels_args* args, int pc_f64, void* stream);

/* ---- detection evaluation on the device (csrc/evaldet.hip) ----
 * Replaces the CPU evaluation of utils/ap_calculator.py + utils/eval_det.py.
 *   ov3d_box_points_count: remove_empty_box (ap_calculator.py:70-84): for every predicted box
 *     (corners (B,K,8,3) f32, upright camera, flipped to depth as flip_axis_to_depth), the
 *     number of scene points inside its convex hull (in_hull, box_util.py:22-31);
 *     point (b, n) xyz at pts[b*pt_sb + n*pt_sn + 0..2] -> counts (B,K) int32
 *   ov3d_box3d_iou_eval: box3d_iou (box_util.py:116-141) of every (prediction, GT) pair of a
 *     scene: pred (S,K,8,3) f32 with pvalid (S,K) u8, gt (S,G,8,3) f32 with gvalid (S,G) u8
 *     -> iou (S,K,G) f64 (0 where either is invalid)
 *   ov3d_ap_match: eval_det_cls's TP/FP walk (eval_det.py:104-131) per (scene, class):
 *     scores (S,K,C) f32 (-inf: not a detection of that class), gt_cls (S,G) int64 ->
 *     tp (S,K,C) u8 (1 TP, 0 FP) for every detection; K <= 256, G <= 64
 *   ov3d_ap_curve: voc_ap (eval_det.py:20-52, 133-146) per class from the detections' TP flags
 *     in global descending-confidence order, tp_sorted (C, M) u8 with nvalid (C) leading
 *     entries valid, npos (C) GT counts; tp_pos (C, tp_cap) int32 workspace
 *     -> ap (C) f64, rec_last (C) f64 (the recall at the last detection) */
int ov3d_box_points_count(const float* pts, long long pt_sb, long long pt_sn, int N,
                          const float* corners, int B, int K, int32_t* counts, void* stream);
int ov3d_box3d_iou_eval(const float* pred, const uint8_t* pvalid, const float* gt,
                        const uint8_t* gvalid, int S, int K, int G, double* iou, void* stream);
int ov3d_ap_match(const double* iou, const float* scores, const int64_t* gt_cls,
                  const uint8_t* gvalid, int S, int K, int G, int C, double thresh, uint8_t* tp,
                  void* stream);
int ov3d_ap_curve(const uint8_t* tp_sorted, long long M, const int32_t* nvalid,
                  const int32_t* npos, int C, int32_t* tp_pos, long long tp_cap, double* ap,
                  double* rec_last, void* stream);

/* In-kernel launch stamps (measurement, bench.py): while armed, each encoder-size attention
 * launch (Lq * Lk >= min_work) of kind 0 forward, 1 dQ, 2 dK/dV takes 2 words per wave of buf
 * (entry / exit wall clock of each wave, ov3d_wall_clock_khz ticks), recorded in a host table
 * (kind, word offset, waves, work = Lq * Lk) captured launches keep replaying into.  buf = NULL disarms.  No reference counterpart. */
int ov3d_stamps_arm(unsigned long long* buf, long long words, long long min_work);
int ov3d_stamps_count(void);
int ov3d_stamps_get(int i, int* kind, long long* word_off, long long* waves, long long* work);
long long ov3d_wall_clock_khz(void);

#ifdef __cplusplus
}
#endif
#endif /* OV3D_H_ */
