/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker.
 * The product path (kinet_amd) never links or calls it.
 *
 * Plain-C restatement of the reference MultiScaleDeformableAttention kernels
 * (src/trackformer/models/ops/src/cuda/ms_deform_im2col_cuda.cuh), one scalar
 * loop nest per CUDA kernel, same arithmetic in the same scalar type:
 *
 *   msda_oracle_fwd_*   <- ms_deformable_im2col_gpu_kernel (cuh:165-237) with
 *                          ms_deform_attn_im2col_bilinear (cuh:24-67), followed by
 *                          the at::sum(columns, 0) reduction over L*P (cu:80).
 *   msda_oracle_bwd_*   <- ms_deformable_col2im_coord_gpu_kernel (cuh:308-378)
 *                          [grad_sampling_loc, grad_attn_weight] and
 *                          ms_deformable_col2im_gpu_kernel (cuh:239-306)
 *                          [grad_value: the 5x5 neighbourhood scan with
 *                          ms_deform_attn_get_gradient_weight, cuh:69-94].
 *
 * Layouts (cu:25-27, cuh:182-185): value (N,S,M,D); spatial_shapes (L,2) = (H,W);
 * level_start (L); sampling_loc (N,Lq,M,L,P,2) with [x,y]; attn_weight
 * (N,Lq,M,L,P); output (N,Lq,M*D).  grad_* buffers are overwritten (the
 * launcher zero-initialises them, cu:119-121).
 *
 * Parity of this restatement is pinned in tests/test_oracle_golden.py against
 * fixtures produced by the reference's own ms_deform_attn_core_pytorch
 * (tests/golden/make_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define DEFINE_MSDA_ORACLE(T, SUF)                                                          \
static T bilinear_##SUF(const T *v, int H, int W, int M, int D, T h, T w, int m, int c)    \
{ /* cuh:24-67 */                                                                           \
    int hl = (int)floor(h), wl = (int)floor(w);                                             \
    int hh_ = hl + 1, wh_ = wl + 1;                                                         \
    T lh = h - hl, lw = w - wl, hh = 1 - lh, hw = 1 - lw;                                   \
    T v1 = 0, v2 = 0, v3 = 0, v4 = 0;                                                       \
    if (hl >= 0 && wl >= 0) v1 = v[((long)hl * W + wl) * M * D + m * D + c];                \
    if (hl >= 0 && wh_ <= W - 1) v2 = v[((long)hl * W + wh_) * M * D + m * D + c];          \
    if (hh_ <= H - 1 && wl >= 0) v3 = v[((long)hh_ * W + wl) * M * D + m * D + c];          \
    if (hh_ <= H - 1 && wh_ <= W - 1) v4 = v[((long)hh_ * W + wh_) * M * D + m * D + c];    \
    return hh * hw * v1 + hh * lw * v2 + lh * hw * v3 + lh * lw * v4;                       \
}                                                                                           \
                                                                                            \
static T grad_weight_##SUF(T h, T w, int gh, int gw, int H, int W)                          \
{ /* cuh:69-94 */                                                                           \
    if (h <= -1 || h >= H || w <= -1 || w >= W) return 0;                                  \
    int hl = (int)floor(h), wl = (int)floor(w);                                             \
    int hh_ = hl + 1, wh_ = wl + 1;                                                         \
    T weight = 0;                                                                           \
    if (gh == hl && gw == wl) weight = (gh + 1 - h) * (gw + 1 - w);                         \
    if (gh == hl && gw == wh_) weight = (gh + 1 - h) * (w + 1 - gw);                        \
    if (gh == hh_ && gw == wl) weight = (h + 1 - gh) * (gw + 1 - w);                        \
    if (gh == hh_ && gw == wh_) weight = (h + 1 - gh) * (w + 1 - gw);                       \
    return weight;                                                                          \
}                                                                                           \
                                                                                            \
static T coord_weight_##SUF(T h, T w, int m, int c, int H, int W, int M, int D,             \
                            const T *v, int bp_dir)                                         \
{ /* cuh:96-163; bp_dir 0 -> d/dw (x), 1 -> d/dh (y) */                                     \
    if (h <= -1 || h >= H || w <= -1 || w >= W) return 0;                                   \
    int hl = (int)floor(h), wl = (int)floor(w);                                             \
    int hh_ = hl + 1, wh_ = wl + 1;                                                         \
    T weight = 0, v1 = 0, v2 = 0, v3 = 0, v4 = 0;                                           \
    int b1 = hl >= 0 && wl >= 0, b2 = hl >= 0 && wh_ <= W - 1;                              \
    int b3 = hh_ <= H - 1 && wl >= 0, b4 = hh_ <= H - 1 && wh_ <= W - 1;                    \
    if (b1) v1 = v[((long)hl * W + wl) * M * D + m * D + c];                                \
    if (b2) v2 = v[((long)hl * W + wh_) * M * D + m * D + c];                               \
    if (b3) v3 = v[((long)hh_ * W + wl) * M * D + m * D + c];                               \
    if (b4) v4 = v[((long)hh_ * W + wh_) * M * D + m * D + c];                              \
    if (bp_dir == 1) {                                                                      \
        if (b1) weight += -1 * (wl + 1 - w) * v1;                                           \
        if (b2) weight += -1 * (w - wl) * v2;                                               \
        if (b3) weight += (wl + 1 - w) * v3;                                                \
        if (b4) weight += (w - wl) * v4;                                                    \
    } else if (bp_dir == 0) {                                                               \
        if (b1) weight += -1 * (hl + 1 - h) * v1;                                           \
        if (b2) weight += (hl + 1 - h) * v2;                                                \
        if (b3) weight += -1 * (h - hl) * v3;                                               \
        if (b4) weight += (h - hl) * v4;                                                    \
    }                                                                                       \
    return weight;                                                                          \
}                                                                                           \
                                                                                            \
int msda_oracle_fwd_##SUF(const T *value, const int64_t *shapes, const int64_t *lstart,     \
                          const T *loc, const T *attw, T *out,                              \
                          int N, int S, int M, int D, int L, int Lq, int P)                 \
{                                                                                           \
    for (int b = 0; b < N; ++b)                                                             \
    for (int q = 0; q < Lq; ++q)                                                            \
    for (int m = 0; m < M; ++m)                                                             \
    for (int c = 0; c < D; ++c) {                                                           \
        T acc = 0;                                                                          \
        for (int l = 0; l < L; ++l) {                                                       \
            const int H = (int)shapes[2 * l], W = (int)shapes[2 * l + 1];                   \
            const T *vb = value + ((long)b * S + lstart[l]) * M * D;                        \
            for (int p = 0; p < P; ++p) {                                                   \
                long si = ((((long)b * Lq + q) * M + m) * L + l) * P + p;                   \
                T lx = loc[2 * si], ly = loc[2 * si + 1], wt = attw[si];                    \
                T h = ly * H - (T)0.5, w = lx * W - (T)0.5; /* cuh:227-228 */               \
                T val = 0;                                                                  \
                if (h > -1 && w > -1 && h < H && w < W)   /* cuh:229 */                    \
                    val = bilinear_##SUF(vb, H, W, M, D, h, w, m, c);                       \
                acc += val * wt;                                                            \
            }                                                                               \
        }                                                                                   \
        out[(((long)b * Lq + q) * M + m) * D + c] = acc;                                    \
    }                                                                                       \
    return 0;                                                                               \
}                                                                                           \
                                                                                            \
int msda_oracle_bwd_##SUF(const T *value, const int64_t *shapes, const int64_t *lstart,     \
                          const T *loc, const T *attw, const T *grad_out,                   \
                          T *grad_value, T *grad_loc, T *grad_attw,                         \
                          int N, int S, int M, int D, int L, int Lq, int P)                 \
{                                                                                           \
    memset(grad_value, 0, sizeof(T) * (size_t)N * S * M * D);                               \
    for (int b = 0; b < N; ++b)                                                             \
    for (int q = 0; q < Lq; ++q)                                                            \
    for (int m = 0; m < M; ++m)                                                             \
    for (int l = 0; l < L; ++l)                                                             \
    for (int p = 0; p < P; ++p) {                                                           \
        const int H = (int)shapes[2 * l], W = (int)shapes[2 * l + 1];                       \
        const T *vb = value + ((long)b * S + lstart[l]) * M * D;                            \
        T *gvb = grad_value + (long)b * S * M * D;                                          \
        const T *g = grad_out + (((long)b * Lq + q) * M + m) * D;                           \
        long si = ((((long)b * Lq + q) * M + m) * L + l) * P + p;                           \
        const T wt = attw[si];                                                              \
        /* col2im_coord (cuh:330-377): one pass per coordinate, as the two threads do */    \
        for (int lc = 0; lc < 2; ++lc) {                                                    \
            T sx = loc[2 * si] * W - (T)0.5, sy = loc[2 * si + 1] * H - (T)0.5;             \
            T val = 0, wval = 0;                                                            \
            for (int c = 0; c < D; ++c) {                                                   \
                const T col = g[c];                                                         \
                if (sx <= -1 || sy <= -1 || sx >= W || sy >= H) { sx = sy = -2; }           \
                else wval += col * bilinear_##SUF(vb, H, W, M, D, sy, sx, m, c);             \
                val += coord_weight_##SUF(sy, sx, m, c, H, W, M, D, vb, lc) * col * wt;     \
            }                                                                               \
            val *= (lc == 0) ? (T)W : (T)H;                                                 \
            grad_loc[2 * si + lc] = val;                                                    \
            if (lc == 0) grad_attw[si] = wval;                                              \
        }                                                                                   \
        /* col2im (cuh:260-304): 5x5 neighbourhood scan with truncating int cast */         \
        const T sx = loc[2 * si] * W - (T)0.5, sy = loc[2 * si + 1] * H - (T)0.5;           \
        const int ch = (int)sy, cw = (int)sx;                                               \
        for (int c = 0; c < D; ++c) {                                                       \
            const T top = g[c] * wt;                                                        \
            for (int dy = -2; dy <= 2; ++dy)                                                \
            for (int dx = -2; dx <= 2; ++dx) {                                              \
                int gh = ch + dy, gw = cw + dx;                                             \
                if (gh >= 0 && gh < H && gw >= 0 && gw < W &&                               \
                    fabs((double)(sy - gh)) < 1 && fabs((double)(sx - gw)) < 1) {           \
                    T wgt = grad_weight_##SUF(sy, sx, gh, gw, H, W);                        \
                    gvb[((long)lstart[l] + (long)gh * W + gw) * M * D + m * D + c] += wgt * top; \
                }                                                                           \
            }                                                                               \
        }                                                                                   \
    }                                                                                       \
    return 0;                                                                               \
}

DEFINE_MSDA_ORACLE(float, f32)
DEFINE_MSDA_ORACLE(double, f64)
