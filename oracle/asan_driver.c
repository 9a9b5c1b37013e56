/* ORACLE — test infrastructure only.  Sanitizer driver for mvn_oracle.c (SURVEY.md §5,
 * 'Race detection / sanitizers': -fsanitize=address,undefined on the CPU restatement).
 *
 *   oracle_asan in.bin out.bin
 *
 * in.bin: int32 header {B, N, C, H, W, Vx, Vy, Vz, agg, align_corners, feat_bf16, J} then
 * feat (f32, or bf16 bits when feat_bf16), P (B,N,3,4), coords (B,Vx,Vy,Vz,3), conf (B,N,C),
 * pts (B,N,J,2), pconf (B,N,J).  Every array is copied into a malloc block of exactly its
 * size, so any read or write past an array is an AddressSanitizer error.  out.bin: the
 * unprojection (B,C,V^3), the soft-argmax of its first J channels (xyz (B,J,3) then the
 * normalised volume), and every (b, j)'s DLT design matrix (2N x 4), all f32.
 * tests/test_oracle.py::test_oracle_under_address_sanitizer compares out.bin with the
 * regular build of the same functions, bit for bit. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_unproject(const void *feat, int feat_bf16, const float *P, const float *coords,
                     const float *conf, float *out, int B, int N, int C, int H, int W,
                     int Vx, int Vy, int Vz, int agg, int align_corners);
int oracle_softargmax3d(const float *vol, const float *coords, float multiplier, int softmax,
                        float *out_xyz, float *out_vol, int B, int J, int Vx, int Vy, int Vz);
int oracle_dlt_design(const float *P, const float *pts, const float *conf, float *A,
                      int B, int N, int J, int b, int j);

static void *read_exact(FILE *f, size_t bytes) {
    void *p = malloc(bytes ? bytes : 1);
    if (!p || fread(p, 1, bytes, f) != bytes) { fprintf(stderr, "short input\n"); exit(2); }
    return p;
}

int main(int argc, char **argv) {
    if (argc != 3) { fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t h[12];
    if (fread(h, sizeof h, 1, f) != 1) return 2;
    const int B = h[0], N = h[1], C = h[2], H = h[3], W = h[4], Vx = h[5], Vy = h[6], Vz = h[7];
    const int agg = h[8], ac = h[9], bf16 = h[10], J = h[11];
    const size_t nvox = (size_t)Vx * Vy * Vz;
    void *feat = read_exact(f, (size_t)B * N * C * H * W * (bf16 ? 2 : 4));
    float *P = read_exact(f, (size_t)B * N * 12 * 4);
    float *coords = read_exact(f, (size_t)B * nvox * 3 * 4);
    float *conf = read_exact(f, (size_t)B * N * C * 4);
    float *pts = read_exact(f, (size_t)B * N * J * 2 * 4);
    float *pconf = read_exact(f, (size_t)B * N * J * 4);
    fclose(f);

    float *vol = malloc((size_t)B * C * nvox * 4);
    if (oracle_unproject(feat, bf16, P, coords, conf, vol, B, N, C, H, W, Vx, Vy, Vz, agg, ac)) return 3;
    /* soft-argmax input: the first J channels of each frame, packed (B, J, V^3) */
    float *sin = malloc((size_t)B * J * nvox * 4), *xyz = malloc((size_t)B * J * 3 * 4);
    float *svol = malloc((size_t)B * J * nvox * 4);
    for (int b = 0; b < B; ++b) memcpy(sin + (size_t)b * J * nvox, vol + (size_t)b * C * nvox, (size_t)J * nvox * 4);
    if (oracle_softargmax3d(sin, coords, 1.0f, 1, xyz, svol, B, J, Vx, Vy, Vz)) return 3;
    float *A = malloc((size_t)B * J * 2 * N * 4 * 4);
    for (int b = 0; b < B; ++b)
        for (int j = 0; j < J; ++j)
            if (oracle_dlt_design(P, pts, pconf, A + ((size_t)b * J + j) * 2 * N * 4, B, N, J, b, j)) return 3;

    FILE *o = fopen(argv[2], "wb");
    if (!o) return 2;
    fwrite(vol, 4, (size_t)B * C * nvox, o);
    fwrite(xyz, 4, (size_t)B * J * 3, o);
    fwrite(svol, 4, (size_t)B * J * nvox, o);
    fwrite(A, 4, (size_t)B * J * 2 * N * 4, o);
    fclose(o);
    free(feat); free(P); free(coords); free(conf); free(pts); free(pconf);
    free(vol); free(sin); free(xyz); free(svol); free(A);
    return 0;
}
