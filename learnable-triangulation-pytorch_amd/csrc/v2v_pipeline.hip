// Config 5 as one call: unprojection (channels-last bf16) -> V2V front block, pipelined over
// frame groups through a caller workspace of one group's intermediate (SURVEY.md §8a a4 /
// §8f rank 3; reference: triangulation.py:349-352, v2v.py:7-17,145-146).
//
// The two launches of a group run back to back on the caller's stream; the group's
// (G, V, V, V, 32) bf16 intermediate (16.8 MB per 64^3 frame) is written by the first and
// read by the second while it is still in the 256 MiB MALL — the default group keeps it
// within half of it — so the full-batch intermediate (1.07 GB at 64 frames) is never
// allocated.  Why the pair is not one kernel (an LDS-resident halo would recompute every
// halo voxel 3.4x with L2 tap gathers; the conv's 140.8 KB ring leaves no LDS for feature
// staging): DESIGN.md §4.7.  Outputs are bit-identical to mvn_unproject_ex(NDHWC) +
// mvn_v2v_front on the whole batch (every launch is per frame in both kernels).
#include "common.hpp"

namespace {
constexpr int kCin = 32;
constexpr long long kDefaultGroupBytes = 128LL << 20;        // half the MALL

int default_group(int V) {
  const long long per = (long long)V * V * V * kCin * 2;
  const long long g = kDefaultGroupBytes / per;
  return g < 1 ? 1 : int(g > 64 ? 64 : g);
}
}  // namespace

extern "C" size_t mvn_unproject_v2v_front_workspace_bytes(int group_frames, int V) {
  if (V <= 0) return 0;
  const int G = group_frames > 0 ? group_frames : default_group(V);
  return size_t(G) * size_t(V) * V * V * kCin * 2;
}

extern "C" int mvn_unproject_v2v_front_ex(const void* feat, int feat_dtype, const float* proj, const float* coords,
                                          const float* cuboids, int transfer_cmu, int agg, const float* conf,
                                          int align_corners, const void* weight_packed, const float* scale,
                                          const float* shift, void* out, int out_dtype, void* workspace,
                                          size_t workspace_bytes, int group_frames, int B, int N, int C, int H, int W,
                                          int V, void* stream) {
  if (!feat || !proj || !weight_packed || !scale || !shift || !out) return MVN_ERR_ARG;
  if ((coords == nullptr) == (cuboids == nullptr)) return MVN_ERR_ARG;       // exactly one coordinate source
  if (agg == MVN_AGG_CONF && !conf) return MVN_ERR_ARG;                      // conf*: per-view confidences
  if (B <= 0 || N <= 0 || H <= 0 || W <= 0 || V <= 0) return MVN_ERR_SHAPE;
  if (C != kCin || V % 16 != 0 || V > 256) return MVN_ERR_SHAPE;
  if (feat_dtype != MVN_DTYPE_F32 && feat_dtype != MVN_DTYPE_BF16) return MVN_ERR_DTYPE;
  if (out_dtype != MVN_DTYPE_F32 && out_dtype != MVN_DTYPE_BF16) return MVN_ERR_DTYPE;
  const int G = group_frames > 0 ? group_frames : default_group(V);
  if (!workspace || workspace_bytes < mvn_unproject_v2v_front_workspace_bytes(G, V)) return MVN_ERR_WORKSPACE;
  const size_t fe = feat_dtype == MVN_DTYPE_F32 ? 4 : 2, oe = out_dtype == MVN_DTYPE_F32 ? 4 : 2;
  const size_t vox = size_t(V) * V * V;
  const size_t feat_frame = size_t(N) * C * H * W * fe, out_frame = 16 * vox * oe;
  for (int g = 0; g < B; g += G) {
    const int n = B - g < G ? B - g : G;
    const char* f = static_cast<const char*>(feat) + size_t(g) * feat_frame;
    const float* P = proj + size_t(g) * N * 12;
    const float* cf = agg == MVN_AGG_CONF ? conf + size_t(g) * N * C : nullptr;    // (B, N, C) rows of the group
    int rc = cuboids ? mvn_unproject_cuboid(f, feat_dtype, P, cuboids + size_t(g) * MVN_CUBOID_FLOATS, transfer_cmu,
                                            cf, workspace, MVN_DTYPE_BF16, MVN_LAYOUT_NDHWC, n, N, C, H, W, V,
                                            agg, align_corners, stream)
                     : mvn_unproject_ex(f, feat_dtype, P, coords + size_t(g) * vox * 3, cf, workspace,
                                        MVN_DTYPE_BF16, MVN_LAYOUT_NDHWC, n, N, C, H, W, V, V, V, agg, align_corners,
                                        stream);
    if (rc != MVN_OK) return rc;
    rc = mvn_v2v_front(workspace, weight_packed, scale, shift, static_cast<char*>(out) + size_t(g) * out_frame,
                       out_dtype, n, V, stream);
    if (rc != MVN_OK) return rc;
  }
  return MVN_OK;
}

extern "C" int mvn_unproject_v2v_front(const void* feat, int feat_dtype, const float* proj, const float* coords,
                                       const float* cuboids, int transfer_cmu, int agg, int align_corners,
                                       const void* weight_packed, const float* scale, const float* shift, void* out,
                                       int out_dtype, void* workspace, size_t workspace_bytes, int group_frames,
                                       int B, int N, int C, int H, int W, int V, void* stream) {
  if (agg == MVN_AGG_CONF) return MVN_ERR_ARG;        // conf*: mvn_unproject_v2v_front_ex with the confidences
  return mvn_unproject_v2v_front_ex(feat, feat_dtype, proj, coords, cuboids, transfer_cmu, agg, nullptr,
                                    align_corners, weight_packed, scale, shift, out, out_dtype, workspace,
                                    workspace_bytes, group_frames, B, N, C, H, W, V, stream);
}
