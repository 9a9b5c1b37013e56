/*
 * mvn_hip.h — C ABI of libmvn_hip.so, the MI355X (gfx950) implementation of the
 * volumetric / algebraic triangulation hot path of learnable-triangulation-pytorch.
 *
 * The reference has no FFI layer: its boundary is three module-level Python
 * functions that the models call by attribute lookup.  Each entry
 * point below replaces exactly one of them and is what a ctypes / torch custom-op
 * binding on the reference side would call:
 *
 *   mvn_unproject        <- mvn/utils/op.py:99-163   unproject_heatmaps(...)
 *   mvn_softargmax3d     <- mvn/utils/op.py:84-96    integrate_tensor_3d_with_coordinates(...)
 *   mvn_dlt              <- mvn/utils/multiview.py:162-174 triangulate_batch_of_points(...)
 *                           (+ its per-point solver multiview.py:132-159)
 *   mvn_softargmax2d     <- mvn/utils/op.py:11-47    integrate_tensor_2d(...)  (the algebraic
 *                           path's producer of the DLT's 2D points)
 *   mvn_coord_volumes    <- mvn/models/triangulation.py:280-341 (the per-frame coordinate-
 *                           volume loop feeding unproject and soft-argmax)
 *   mvn_unproject_cuboid, mvn_softargmax3d_cuboid
 *                        <- op.py:99-163 / op.py:84-96 fed by triangulation.py:280-341: the
 *                           coordinate volume formed in-kernel from the per-frame cuboid
 *   mvn_nearest_voxel    <- mvn/models/loss.py:63-67 (VolumetricCELoss's distance volume +
 *                           argmin)
 *   mvn_v2v_front        <- mvn/models/v2v.py:7-17, 145-146 (V2VModel.front_layers[0] =
 *                           Basic3DBlock(32, 16, 7), eval mode; BASELINE config 5)
 *
 * Conventions
 *   - Every buffer is caller-owned device memory (hipMalloc / torch), contiguous,
 *     row-major in the reference's own tensor layout.  Nothing is retained after
 *     return; nothing is allocated (soft-argmax takes a caller workspace).
 *   - `stream` is a hipStream_t passed as void* (0 = the null stream).  Every call
 *     is stream-ordered and asynchronous: no host synchronisation, capturable in a
 *     hipGraph.
 *   - Return value: MVN_OK (0) or a negative MVN_ERR_* code.  Argument checks run
 *     before any HIP call, so they are safe without a GPU.
 *   - Functions are reentrant; the library keeps no mutable global state apart from
 *     the test-only knobs of mvn_debug_set_unproject (atomics).
 */
#ifndef MVN_HIP_H
#define MVN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ------------------------------------------------------- */
#define MVN_OK              0
#define MVN_ERR_ARG        -1   /* null pointer / bad enum / bad flag            */
#define MVN_ERR_SHAPE      -2   /* non-positive or overflowing extent            */
#define MVN_ERR_DTYPE      -3   /* unsupported dtype combination                 */
#define MVN_ERR_LAUNCH     -4   /* hipLaunchKernel / hipGetLastError failed      */
#define MVN_ERR_WORKSPACE  -5   /* workspace missing or too small                */

/* ---- dtypes ------------------------------------------------------------ */
#define MVN_DTYPE_F32   0
#define MVN_DTYPE_BF16  1

/* ---- volume layouts ------------------------------------------------------ */
#define MVN_LAYOUT_NCDHW 0     /* (B, C, Vx, Vy, Vz): the reference's unproject output */
#define MVN_LAYOUT_NDHWC 1     /* (B, Vx, Vy, Vz, C): channels-last (V2V front input)  */

/* ---- unprojection arithmetic -------------------------------------------- */
#define MVN_PRECISION_EXACT 0  /* the reference's f32 op order: sum / max / conf* bit-exact,
                                  softmax <= 1e-5 (the default of every other entry point)  */
#define MVN_PRECISION_FAST  1  /* the north_star contract's tolerance:
                                  reciprocal projection, max-free view softmax, and for bf16
                                  maps bf16 bilinear weights on v_dot2 pixel pairs          */

/* ---- view aggregation (op.py:147-161) ---------------------------------- */
#define MVN_AGG_SUM      0     /* 'sum'                                           */
#define MVN_AGG_MAX      1     /* 'max'                                           */
#define MVN_AGG_SOFTMAX  2     /* 'softmax'                                       */
#define MVN_AGG_CONF     3     /* any string starting with 'conf' (op.py:147)     */

/* Library version, (major << 16) | (minor << 8) | patch. */
int mvn_version(void);

/* Static message for an MVN_* return code. */
const char* mvn_strerror(int code);

/*
 * Unprojection of N views of C-channel maps into a C x Vx x Vy x Vz volume.
 * Replaces mvn/utils/op.py:99-163 (unproject_heatmaps).
 *
 *   feat    (B, N, C, H, W)     feat_dtype (f32 | bf16)
 *   proj    (B, N, 3, 4)        f32, heatmap-resolution projection matrices
 *   coords  (B, Vx, Vy, Vz, 3)  f32 world coordinates per voxel
 *   conf    (B, N, C)           f32, read only when agg == MVN_AGG_CONF (else may be NULL)
 *   out     (B, C, Vx, Vy, Vz)  out_dtype (f32 | bf16)
 *   align_corners: 0 = torch>=1.3 grid_sample default (the importable oracle),
 *                  1 = torch 1.0.1 semantics (requirements.txt:20 pins 1.0.1).
 */
int mvn_unproject(const void* feat, int feat_dtype,
                  const float* proj, const float* coords, const float* conf,
                  void* out, int out_dtype,
                  int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
                  int agg, int align_corners, void* stream);

/*
 * 3D soft-argmax over voxel world coordinates.
 * Replaces mvn/utils/op.py:84-96 (integrate_tensor_3d_with_coordinates), with the
 * caller's `volumes * volume_multiplier` (triangulation.py:353) fused as `multiplier`.
 *
 *   vol       element (b, j, i) at vol[b*vol_bstride + j*vol_jstride + i], i < Vx*Vy*Vz
 *             (strides in elements, so a channel slice of an unprojected volume
 *             needs no copy); vol_dtype f32 | bf16
 *   coords    (B, Vx, Vy, Vz, 3) f32
 *   out_xyz   (B, J, 3) f32
 *   out_vol   (B, J, Vx, Vy, Vz) contiguous, out_dtype f32 | bf16; NULL = do not
 *             write the normalised volume
 *   softmax   1 = softmax over the flattened volume (op.py:89),
 *             0 = relu with no mass normalisation (op.py:91, reference quirk)
 *   workspace >= mvn_softargmax3d_workspace_bytes(B, J, Vx, Vy, Vz) bytes of
 *             device memory, 16-byte aligned; contents need no initialisation.
 */
size_t mvn_softargmax3d_workspace_bytes(int B, int J, int Vx, int Vy, int Vz);

int mvn_softargmax3d(const void* vol, int vol_dtype,
                     int64_t vol_bstride, int64_t vol_jstride,
                     const float* coords, float multiplier, int softmax,
                     float* out_xyz, void* out_vol, int out_dtype,
                     void* workspace, size_t workspace_bytes,
                     int B, int J, int Vx, int Vy, int Vz, void* stream);

/*
 * Confidence-weighted linear (DLT) triangulation of a batch of points.
 * Replaces mvn/utils/multiview.py:162-174 (triangulate_batch_of_points) and its
 * per-point solver multiview.py:132-159.  The 2N x 4 design matrix is formed in
 * f32 exactly as the reference forms it (multiview.py:150-152); its null vector is
 * found in f64 (streaming Givens QR + one-sided Jacobi SVD).
 *
 *   proj  (B, N, 3, 4) f32     image-resolution projection matrices
 *   pts   (B, N, J, 2) f32     2D points, pixels
 *   conf  (B, N, J)    f32     per-view confidences; NULL = all ones (multiview.py:147-148)
 *   out   (B, J, 3)    f32
 */
int mvn_dlt(const float* proj, const float* pts, const float* conf, float* out,
            int B, int N, int J, void* stream);

/*
 * mvn_unproject with a selectable output layout: out_layout = MVN_LAYOUT_NCDHW is exactly
 * mvn_unproject; MVN_LAYOUT_NDHWC writes (B, Vx, Vy, Vz, C) (C % 4 == 0, N <= 8), the
 * input layout of mvn_v2v_front.
 */
int mvn_unproject_ex(const void* feat, int feat_dtype,
                     const float* proj, const float* coords, const float* conf,
                     void* out, int out_dtype, int out_layout,
                     int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
                     int agg, int align_corners, void* stream);

/*
 * mvn_unproject / mvn_unproject_ex / mvn_unproject_cuboid with a selectable arithmetic
 * (op.py:99-163).  Exactly one of coords (B, Vx, Vy, Vz, 3) and cuboids (B, 18; then
 * Vx = Vy = Vz, N <= 8) is non-NULL.  precision = MVN_PRECISION_EXACT is bit-identical
 * to those entry points; MVN_PRECISION_FAST computes the same function within the
 * north_star tolerance (f32 maps: <= 1e-4 max-rel of the volume, measured 2-4e-5; bf16 maps: one bf16 ulp
 * + 2^-8 max|ref|, 2^-7 for softmax; validity masks unchanged), measured in DESIGN.md §4.1a.
 */
int mvn_unproject_precision(const void* feat, int feat_dtype,
                            const float* proj, const float* coords, const float* cuboids, int transfer_cmu,
                            const float* conf, void* out, int out_dtype, int out_layout,
                            int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
                            int agg, int align_corners, int precision, void* stream);

/*
 * V2V front block, eval mode: Conv3d(32 -> 16, k = 7, pad = 3) + BatchNorm3d + ReLU
 * (v2v.py:7-17) on bf16 MFMA, f32 accumulation.
 *   vol_cl         (B, V, V, V, 32) bf16 channels-last (mvn_unproject_ex NDHWC output)
 *   weight_packed  mvn_v2v_front_packed_weight_bytes() bytes: bf16 weights as
 *                  [tap = (dx*7 + dy)*7 + dz][lane 0..63][j 0..7] = W[lane & 15][8*(lane >> 4) + j][dx][dy][dz]
 *   scale, shift   (16) f32: BN folded, y = relu(conv * scale + shift)
 *   out            (B, 16, V, V, V) out_dtype (f32 | bf16);  V % 16 == 0, V <= 256
 */
size_t mvn_v2v_front_packed_weight_bytes(void);
int mvn_v2v_front(const void* vol_cl, const void* weight_packed, const float* scale, const float* shift,
                  void* out, int out_dtype, int B, int V, void* stream);

/*
 * Config 5 in one call: unprojection written channels-last bf16 (as mvn_unproject_ex with
 * MVN_LAYOUT_NDHWC, or mvn_unproject_cuboid when `cuboids` is given instead of `coords`)
 * followed by mvn_v2v_front, pipelined over groups of `group_frames` frames (<= 0: the
 * default, one group's intermediate within half of the 256 MiB MALL: 8 frames at V = 64)
 * through `workspace` (>= mvn_unproject_v2v_front_workspace_bytes(group_frames, V) bytes).
 * Replaces triangulation.py:349-352 up to V2VModel.front_layers[0] (v2v.py:145-146).
 *   C == 32, V % 16 == 0, 1 <= N <= 8 views (the channels-last kernels), B >= 1
 *   (MVN_ERR_SHAPE otherwise; mvn_rocm.v2v.unproject_v2v_front routes more views and empty
 *   batches through the two calls); exactly one of coords / cuboids non-NULL.
 *   out (B, 16, V, V, V) out_dtype.  Bit-identical to the two calls on the whole batch.
 * mvn_unproject_v2v_front takes agg != MVN_AGG_CONF; mvn_unproject_v2v_front_ex also takes
 * MVN_AGG_CONF with conf (B, N, C) f32 — the volumetric model's vol_confidences whenever
 * volume_aggregation_method starts with 'conf' (triangulation.py:268-269, 349; op.py:147-148)
 * — and ignores conf otherwise.
 */
size_t mvn_unproject_v2v_front_workspace_bytes(int group_frames, int V);
int mvn_unproject_v2v_front(const void* feat, int feat_dtype, const float* proj, const float* coords,
                            const float* cuboids, int transfer_cmu, int agg, int align_corners,
                            const void* weight_packed, const float* scale, const float* shift, void* out,
                            int out_dtype, void* workspace, size_t workspace_bytes, int group_frames,
                            int B, int N, int C, int H, int W, int V, void* stream);
int mvn_unproject_v2v_front_ex(const void* feat, int feat_dtype, const float* proj, const float* coords,
                               const float* cuboids, int transfer_cmu, int agg, const float* conf,
                               int align_corners, const void* weight_packed, const float* scale,
                               const float* shift, void* out, int out_dtype, void* workspace,
                               size_t workspace_bytes, int group_frames, int B, int N, int C, int H, int W,
                               int V, void* stream);

/*
 * 2D soft-argmax of heatmaps.  Replaces mvn/utils/op.py:11-47 (integrate_tensor_2d) with
 * the caller's `heatmaps * heatmap_multiplier` (triangulation.py:164) fused.
 *   heatmaps  (B, J, H, W)  dtype (f32 | bf16), contiguous
 *   out_xy    (B, J, 2)     f32: (x, y) = sum p * (w, h) / sum p  (op.py:31-42)
 *   out_maps  (B, J, H, W)  out_dtype: softmax-normalised (softmax = 1) or relu'd maps
 *                           (softmax = 0, not normalised, op.py:27); NULL = not wanted
 */
int mvn_softargmax2d(const void* heatmaps, int dtype, float multiplier, int softmax, float* out_xy,
                     void* out_maps, int out_dtype, int B, int J, int H, int W, void* stream);

/*
 * Coordinate volumes (B, V, V, V, 3) f32 of the volumetric model, replacing the per-frame
 * loop of triangulation.py:280-341 (cuboid grid, rotation about the base point,
 * volumetric.py:87-114, optional CMU -> Human3.6M re-axing).  The caller forms per frame,
 * in float64 and rounded to f32 as torch does: position (B,3) = base - side/2,
 * centre (B,3) = base point, step (B,3) = side / (V-1), rot (B,3,3) the rotation matrix.
 */
int mvn_coord_volumes(const float* position, const float* centre, const float* step, const float* rot,
                      float* out, int B, int V, int transfer_cmu, void* stream);

/*
 * Unprojection and 3D soft-argmax with the coordinate volume formed in-kernel instead of
 * read: the caller of op.py:99 / op.py:84 in triangulation.py:280-353
 * builds coord_volumes from a per-frame cuboid and passes it straight to both ops; these
 * entry points take the cuboid itself and never materialise the (B, V, V, V, 3) volume
 * (12 B per voxel not read by either op).  Coordinates are bit-identical to
 * mvn_coord_volumes on the same cuboid, so results are bit-identical to mvn_unproject_ex /
 * mvn_softargmax3d fed that volume.
 *   cuboids  (B, MVN_CUBOID_FLOATS) f32 per frame: position[3], centre[3], step[3], rot[9]
 *            (the arguments of mvn_coord_volumes, interleaved per frame)
 *   transfer_cmu  0 | 1 as in mvn_coord_volumes;  grid V x V x V
 * mvn_unproject_cuboid needs N <= 8 (the tiled kernel); otherwise the arguments of
 * mvn_unproject_ex / mvn_softargmax3d.
 */
#define MVN_CUBOID_FLOATS 18
int mvn_unproject_cuboid(const void* feat, int feat_dtype,
                         const float* proj, const float* cuboids, int transfer_cmu, const float* conf,
                         void* out, int out_dtype, int out_layout,
                         int B, int N, int C, int H, int W, int V,
                         int agg, int align_corners, void* stream);
int mvn_softargmax3d_cuboid(const void* vol, int vol_dtype,
                            int64_t vol_bstride, int64_t vol_jstride,
                            const float* cuboids, int transfer_cmu, float multiplier, int softmax,
                            float* out_xyz, void* out_vol, int out_dtype,
                            void* workspace, size_t workspace_bytes,
                            int B, int J, int V, void* stream);

/*
 * Nearest voxel per (frame, joint): argmin over the V^3 voxels of the f32 distance
 * sqrt(((c - k)^2).sum(-1)) between coords[b] (B, Vx, Vy, Vz, 3) and keypoints (B, J, 3),
 * IEEE square root, first index on ties (torch.argmin).
 *   out_index (B, J) int32, flat row-major voxel index (VolumetricCELoss, loss.py:63-67).
 */
int mvn_nearest_voxel(const float* coords, const float* keypoints, int* out_index, int B, int J,
                      int Vx, int Vy, int Vz, void* stream);

/* ---- backward (autograd) ------------------------------------------------------------
 * Gradients of the three ops, replacing the ATen autograd the reference relies on
 * (grid_sampler_2d / softmax / einsum / svd backward).  Same buffer conventions as above.
 */

/*
 * d/d(feat) (and d/d(conf) for MVN_AGG_CONF) of mvn_unproject.
 *   grad_out   (B, C, Vx, Vy, Vz)  grad_out_dtype (f32 | bf16)
 *   grad_feat  (B, N, C, H, W) f32, ZERO-INITIALISED by the caller (accumulated with atomics)
 *   grad_conf  (B, N, C) f32 zero-initialised, or NULL (only read for MVN_AGG_CONF)
 * No gradient w.r.t. proj / coords (the reference builds both from numpy constants,
 * triangulation.py:272-341).  N <= 8.  Float atomics: last-bit order nondeterminism.
 */
int mvn_unproject_backward(const void* feat, int feat_dtype, const float* proj, const float* coords,
                           const float* conf, const void* grad_out, int grad_out_dtype,
                           float* grad_feat, float* grad_conf,
                           int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
                           int agg, int align_corners, void* stream);

/*
 * Deterministic variant of mvn_unproject_backward (the reference trains under
 * autograd.detect_anomaly, train.py:178) and mvn_rocm's default backward: every finite
 * contribution is scaled by a power of two 2^e and accumulated as a 64-bit integer (integer
 * adds are associative), then converted to f32 — two runs are bit-identical.  e is chosen per
 * (frame, channel) plane on the device from that plane's finite maxima of |grad_out| (and
 * |feat| for softmax, |conf| and |feat| for conf*) so that no sum of the plane can overflow.
 * Each contribution is rounded to a whole unit u = 2^-62 of the plane's bound
 * nvox * max|g| * factor before it is added, so an element fed by n contributions comes out
 * as the f32 rounding of an integer sum within n/2 units of its exact sum: absolute error
 * <= n/2 * u + half an f32 ulp (relative <= n * 2^-25 + 2^-24 once the element is above
 * 2^-38 of the bound, i.e. 2^24 units).  Non-finite contributions follow the reference's autograd element by element: a
 * NaN / inf grad_out, feature or confidence reaches exactly the gradient elements it reaches
 * in ATen's grid_sampler / softmax / mul backward (NaN if a NaN or both infinities meet there,
 * else the infinity); every other element stays finite.
 *   workspace  >= mvn_unproject_backward_workspace_bytes(B, N, C, H, W) bytes, any content
 *   grad_feat / grad_conf are fully written (no zero-initialisation needed).
 */
size_t mvn_unproject_backward_workspace_bytes(int B, int N, int C, int H, int W);
int mvn_unproject_backward_deterministic(const void* feat, int feat_dtype, const float* proj,
                                         const float* coords, const float* conf, const void* grad_out,
                                         int grad_out_dtype, float* grad_feat, float* grad_conf,
                                         void* workspace, size_t workspace_bytes,
                                         int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
                                         int agg, int align_corners, void* stream);

/*
 * d/d(vol) of mvn_softargmax3d (vol as passed to the forward, i.e. before `multiplier`).
 *   grad_xyz  (B, J, 3) f32 or NULL;  grad_vol (B, J, Vx, Vy, Vz) contiguous or NULL
 *   grad_in   (B, J, Vx, Vy, Vz) contiguous, dtype == vol_dtype, fully written
 *   workspace >= mvn_softargmax3d_backward_workspace_bytes(...) when softmax == 1
 */
size_t mvn_softargmax3d_backward_workspace_bytes(int B, int J, int Vx, int Vy, int Vz);

int mvn_softargmax3d_backward(const void* vol, int vol_dtype, int64_t vol_bstride, int64_t vol_jstride,
                              const float* coords, float multiplier, int softmax,
                              const float* grad_xyz, const void* grad_vol, int grad_vol_dtype,
                              void* grad_in, int grad_in_dtype,
                              void* workspace, size_t workspace_bytes,
                              int B, int J, int Vx, int Vy, int Vz, void* stream);

/*
 * d/d(pts) and d/d(conf) of mvn_dlt (eigenvector perturbation of A^T A, f64).
 *   grad_out (B, J, 3) f32;  grad_pts (B, N, J, 2) f32 written;  grad_conf (B, N, J) f32
 *   written, or NULL (must be NULL when conf is NULL).
 */
int mvn_dlt_backward(const float* proj, const float* pts, const float* conf, const float* grad_out,
                     float* grad_pts, float* grad_conf, int B, int N, int J, void* stream);

/*
 * Test hook (tests only; process-wide, thread-safe): force unprojection code paths.
 *   lds_slots  > 0: LDS slot budget per staging pass of the tiled kernel (small budgets
 *              force the multi-pass and global-gather paths); 0 = the kernel's own budget
 *   kernel     0 = default dispatch, 1 = the simple register-geometry kernel,
 *              2 = the generic tiled kernel (skip the four-view kernel)
 * Returns MVN_OK, or MVN_ERR_ARG for a negative budget or an unknown kernel.
 */
int mvn_debug_set_unproject(int lds_slots, int kernel);

/*
 * Debug build only (make -C learnable-triangulation-pytorch_amd debug -> libmvn_hip_debug.so,
 * -DMVN_DEVICE_ASSERTS): device-side index / layout assertions count their failures instead of
 * trapping.  Reads and clears the counters of every kernel file: *enabled = 1 in the debug
 * build (0 in the release build, whose kernels carry no checks), *count = failures since the
 * last call, *first_line = source line of the first (0 when none).  Synchronise the device
 * first.  Returns MVN_OK, MVN_ERR_ARG for a null pointer, MVN_ERR_LAUNCH if a copy fails.
 */
int mvn_debug_device_asserts(int* enabled, unsigned* count, unsigned* first_line);

/*
 * Self-test of the device-side assertions: one 64-lane launch whose lanes >= n fail a check
 * (64 - n failures in the debug build, none in the release build).  0 <= n <= 64.
 */
int mvn_debug_dassert_selftest(int n, void* stream);

/*
 * Diagnostics: workgroups of the four-view unprojection kernel resident per CU (its LDS and
 * register budget; the persistent grid is this x the CU count), for f32 (bf16_maps = 0) or
 * bf16 (1) feature maps.  Needs a device; returns a count >= 1.
 */
int mvn_debug_unproject_occupancy(int bf16_maps);

#ifdef __cplusplus
}
#endif

#endif /* MVN_HIP_H */
