/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker.  The product path (libmvn_hip.so) never links it.
 *
 * Plain-C CPU restatement of the reference hot path, written from the reference's
 * semantics (file:line cited per function) and the ATen arithmetic it bottoms out in.
 * Parity of this restatement is pinned by the tests/golden npz fixtures, captured from the
 * reference itself (tests/golden/make_golden.py).
 *
 * Build: make -C oracle   (gcc, -ffp-contract=off: every fused multiply-add below is an
 * explicit fmaf, matching the verified ATen orderings of SURVEY.md Appendix A).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define AGG_SUM 0
#define AGG_MAX 1
#define AGG_SOFTMAX 2
#define AGG_CONF 3

/* One bilinear tap set.  A corner outside the image reads the VALUE 0 (padding_mode
 * 'zeros'; torch's grid_sample gives +0 there whatever the sign of the nearest pixel) and
 * also carries weight 0 (as every corner of an invalid voxel), so its product is +0. */
typedef struct { long o[4]; float w[4]; int in[4]; } taps_t;

/* mvn/utils/op.py:117-134: projection (multiview.py:80-101 via the K=4 sgemm of
 * multiview.py:96), depth mask (op.py:121), divide guard (op.py:123), dehomogenise
 * (multiview.py:75), [-1,1] normalisation (op.py:127-130, x / heatmap_shape[0]),
 * grid_sample bilinear/zeros unnormalisation and weights. */
static taps_t view_taps(const float *Pv, float x, float y, float z, int H, int W, int align_corners) {
    taps_t t;
    float uh = fmaf(1.f, Pv[3], fmaf(z, Pv[2], fmaf(y, Pv[1], x * Pv[0])));
    float vh = fmaf(1.f, Pv[7], fmaf(z, Pv[6], fmaf(y, Pv[5], x * Pv[4])));
    float wh = fmaf(1.f, Pv[11], fmaf(z, Pv[10], fmaf(y, Pv[9], x * Pv[8])));
    int invalid = wh <= 0.f;
    if (wh == 0.f) wh = 1.f;
    float u = uh / wh, v = vh / wh;
    float gx = 2.f * (u / (float)H - 0.5f);
    float gy = 2.f * (v / (float)W - 0.5f);
    float ix, iy;
    if (align_corners) {
        ix = (gx + 1.f) * ((float)(W - 1) * 0.5f);
        iy = (gy + 1.f) * ((float)(H - 1) * 0.5f);
    } else {
        /* ATen CPU: (g + 1) * (size / 2) - 0.5 with one rounding (fused) */
        ix = fmaf(gx + 1.f, (float)W * 0.5f, -0.5f);
        iy = fmaf(gy + 1.f, (float)H * 0.5f, -0.5f);
    }
    float fx0 = floorf(ix), fy0 = floorf(iy);
    float tx = ix - fx0, sx = 1.f - tx, ty = iy - fy0, sy = 1.f - ty;
    int x0in = fx0 >= 0.f && fx0 < (float)W, x1in = fx0 >= -1.f && fx0 < (float)(W - 1);
    int y0in = fy0 >= 0.f && fy0 < (float)H, y1in = fy0 >= -1.f && fy0 < (float)(H - 1);
    long x0 = x0in ? (long)fx0 : 0, x1 = x1in ? (long)fx0 + 1 : 0;
    long y0 = y0in ? (long)fy0 : 0, y1 = y1in ? (long)fy0 + 1 : 0;
    t.in[0] = !invalid && y0in && x0in; t.in[1] = !invalid && y0in && x1in;
    t.in[2] = !invalid && y1in && x0in; t.in[3] = !invalid && y1in && x1in;
    t.o[0] = y0 * W + x0; t.w[0] = t.in[0] ? sy * sx : 0.f;
    t.o[1] = y0 * W + x1; t.w[1] = t.in[1] ? sy * tx : 0.f;
    t.o[2] = y1 * W + x0; t.w[2] = t.in[2] ? ty * sx : 0.f;
    t.o[3] = y1 * W + x1; t.w[3] = t.in[3] ? ty * tx : 0.f;
    return t;
}

static float bf16_to_f32(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* ATen CPU grid sampler combination order. */
static float sample_plane(const float *plane, const taps_t *t) {
    float v[4];
    for (int k = 0; k < 4; ++k) v[k] = t->in[k] ? plane[t->o[k]] : 0.f;
    return fmaf(v[3], t->w[3], fmaf(v[2], t->w[2], fmaf(v[1], t->w[1], v[0] * t->w[0])));
}

static float sample_plane_bf16(const uint16_t *plane, const taps_t *t) {
    float v[4];
    for (int k = 0; k < 4; ++k) v[k] = t->in[k] ? bf16_to_f32(plane[t->o[k]]) : 0.f;
    return fmaf(v[3], t->w[3], fmaf(v[2], t->w[2], fmaf(v[1], t->w[1], v[0] * t->w[0])));
}

/* mvn/utils/op.py:99-163 unproject_heatmaps.  feat is f32 (feat_bf16 == 0) or raw bf16
 * bits; the arithmetic is f32 throughout (the f32 reference on bf16-rounded features). */
int oracle_unproject(const void *feat, int feat_bf16, const float *P, const float *coords,
                     const float *conf, float *out, int B, int N, int C, int H, int W,
                     int Vx, int Vy, int Vz, int agg, int align_corners) {
    long nvox = (long)Vx * Vy * Vz, HW = (long)H * W;
    taps_t *t = (taps_t *)malloc(sizeof(taps_t) * (size_t)N);
    float *s = (float *)malloc(sizeof(float) * (size_t)N);
    if (!t || !s) { free(t); free(s); return -1; }
    for (int b = 0; b < B; ++b) {
        for (long i = 0; i < nvox; ++i) {
            const float *cp = coords + ((long)b * nvox + i) * 3;
            for (int v = 0; v < N; ++v)
                t[v] = view_taps(P + ((long)b * N + v) * 12, cp[0], cp[1], cp[2], H, W, align_corners);
            for (int c = 0; c < C; ++c) {
                for (int v = 0; v < N; ++v) {
                    long plane = (((long)b * N + v) * C + c) * HW;
                    s[v] = feat_bf16 ? sample_plane_bf16((const uint16_t *)feat + plane, &t[v])
                                     : sample_plane((const float *)feat + plane, &t[v]);
                }
                float r = 0.f;
                if (agg == AGG_SUM) {                 /* op.py:150 */
                    r = s[0];
                    for (int v = 1; v < N; ++v) r = r + s[v];
                } else if (agg == AGG_MAX) {          /* op.py:152 */
                    r = s[0];
                    for (int v = 1; v < N; ++v)   /* torch.max(dim): NaN wins, ties to the first */
                        r = (s[v] > r || (isnan(s[v]) && !isnan(r))) ? s[v] : r;
                } else if (agg == AGG_CONF) {         /* op.py:148 */
                    const float *cf = conf + (long)b * N * C + c;
                    r = s[0] * cf[0];
                    for (int v = 1; v < N; ++v) r = r + s[v] * cf[(long)v * C];
                } else {                              /* op.py:154-159 */
                    float m = s[0];
                    for (int v = 1; v < N; ++v) m = s[v] > m ? s[v] : m;
                    float den = 0.f;
                    for (int v = 0; v < N; ++v) den += expf(s[v] - m);
                    r = 0.f;
                    for (int v = 0; v < N; ++v) r = r + s[v] * (expf(s[v] - m) / den);
                }
                out[((long)b * C + c) * nvox + i] = r;
            }
        }
    }
    free(t);
    free(s);
    return 0;
}

/* mvn/utils/op.py:84-96 integrate_tensor_3d_with_coordinates, on vol * multiplier
 * (triangulation.py:353), accumulated in double. */
int oracle_softargmax3d(const float *vol, const float *coords, float multiplier, int softmax,
                        float *out_xyz, float *out_vol, int B, int J, int Vx, int Vy, int Vz) {
    long nvox = (long)Vx * Vy * Vz;
    for (int b = 0; b < B; ++b) {
        const float *cb = coords + (long)b * nvox * 3;
        for (int j = 0; j < J; ++j) {
            const float *vj = vol + ((long)b * J + j) * nvox;
            float *oj = out_vol ? out_vol + ((long)b * J + j) * nvox : NULL;
            double m = -INFINITY, den = 0.0, ax = 0.0, ay = 0.0, az = 0.0;
            if (softmax) {
                for (long i = 0; i < nvox; ++i) {
                    double x = (double)(vj[i] * multiplier);
                    if (x > m) m = x;
                }
                for (long i = 0; i < nvox; ++i) den += exp((double)(vj[i] * multiplier) - m);
            }
            for (long i = 0; i < nvox; ++i) {
                double x = (double)(vj[i] * multiplier);
                double p = softmax ? exp(x - m) / den : (x > 0.0 ? x : 0.0);
                if (oj) oj[i] = (float)p;
                ax += p * cb[i * 3 + 0];
                ay += p * cb[i * 3 + 1];
                az += p * cb[i * 3 + 2];
            }
            float *o = out_xyz + ((long)b * J + j) * 3;
            o[0] = (float)ax; o[1] = (float)ay; o[2] = (float)az;
        }
    }
    return 0;
}

/* mvn/utils/multiview.py:150-152: the 2N x 4 design matrix of one (b, j), formed in
 * f32 with the reference's three separately rounded ops.  A is (2N, 4) row-major. */
int oracle_dlt_design(const float *P, const float *pts, const float *conf, float *A,
                      int B, int N, int J, int b, int j) {
    for (int v = 0; v < N; ++v) {
        const float *Pv = P + ((long)b * N + v) * 12;
        long pj = ((long)b * N + v) * J + j;
        float cf = conf ? conf[pj] : 1.f;
        for (int r = 0; r < 2; ++r) {
            float pt = pts[pj * 2 + r];
            for (int k = 0; k < 4; ++k) {
                float e = Pv[8 + k] * pt;
                e = e - Pv[r * 4 + k];
                e = e * cf;
                A[((long)v * 2 + r) * 4 + k] = e;
            }
        }
    }
    (void)B;
    return 0;
}
