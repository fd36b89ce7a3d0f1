// Training-path elementwise kernels that replace torch glue around the kinet GEMMs
// (include/kinet_grad.h):
//  * residual dropout + LayerNorm, forward and backward (the post-norm sub-layers
//    `norm(x + dropout(y))`, deformable_transformer.py:100,108,186,196,199);
//  * dropout(relu(x)) and its backward (the FFN hidden, deformable_transformer.py:99,185);
//  * the MSDeformAttn sampling-location / attention-weight preparation (softmax over the
//    L*P logits, query mask, location from the reference points) and its backward
//    (ms_deform_attn.py:64-82);
//  * inverse_sigmoid and its backward (util/misc.py:609-613).
// f32 (the reference trains in f32).  Dropout keep masks come from the counter hash of
// common.h (dropout_keep), keyed by a device int64 seed and the element's flat index, so the
// backward regenerates the forward's mask without storing it.
#include <hip/hip_runtime.h>

#include <math.h>

#include "../../include/kinet_grad.h"
#include "common.h"

namespace kinet {
namespace {

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ------------------------------------------------------------------ dropout + add + LN
// y = LN(x + Z * r), Z in {0, 1/(1-p)} from (seed, row*d + c); one wave per row, d <= 64 * MAXV
// (MAXV = ceil(d / 64) instantiated for the model widths: no dead unrolled iterations)
template <int MAXV>
__global__ __launch_bounds__(256) void drop_add_ln_kernel(const float* __restrict__ x, const float* __restrict__ r,
                                                          const float* __restrict__ g, const float* __restrict__ b,
                                                          float* __restrict__ y, int rows, int d, float eps,
                                                          const int64_t* __restrict__ seedp, uint32_t thresh,
                                                          float keep_scale) {
    const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const uint64_t seed = (uint64_t)*seedp;
    const long base = (long)row * d;
    float v[MAXV];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
        const int c = lane + 64 * j;
        float t = 0.f;
        if (c < d) {
            const float rv = dropout_keep(seed, (uint64_t)(base + c), thresh) ? r[base + c] * keep_scale : 0.f;
            t = x[base + c] + rv;
        }
        v[j] = t;
        s += t;
    }
    const float mean = wsum(s) / (float)d;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
        const int c = lane + 64 * j;
        if (c < d) q += (v[j] - mean) * (v[j] - mean);
    }
    const float rstd = rsqrtf(wsum(q) / (float)d + eps);
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
        const int c = lane + 64 * j;
        if (c < d) y[base + c] = (v[j] - mean) * rstd * g[c] + b[c];
    }
}

// backward: z = x + Z*r recomputed; dz = LN backward; dx = dz, dr = Z * dz; per-workgroup
// partial dgamma / dbeta (4 waves x rpw rows), summed in order by partial_sum_kernel
template <int MAXV>
__global__ __launch_bounds__(256) void drop_add_ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                              const float* __restrict__ r, const float* __restrict__ gamma,
                                                              float* __restrict__ dx, float* __restrict__ dr,
                                                              float* __restrict__ pg, float* __restrict__ pb, int rows,
                                                              int d, float eps, int rpw, const int64_t* __restrict__ seedp,
                                                              uint32_t thresh, float keep_scale) {
    extern __shared__ float red[];   // [4][2][d]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t seed = (uint64_t)*seedp;
    float g_acc[MAXV], b_acc[MAXV];
#pragma unroll
    for (int v = 0; v < MAXV; ++v) g_acc[v] = b_acc[v] = 0.f;
    const int r_begin = (blockIdx.x * 4 + wave) * rpw;
    const int r_end = min(rows, r_begin + rpw);
    // the next row's x / r / dy are loaded while this row is reduced (one row of loads in flight
    // behind the arithmetic instead of a load -> reduce -> store chain per row)
    float nx[MAXV], nr[MAXV], nd[MAXV];
    auto load_row = [&](int row) {
        const long base = (long)row * d;
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            const int c = v * 64 + lane;
            const bool ok = c < d && row < r_end;
            nx[v] = ok ? x[base + c] : 0.f;
            nr[v] = ok ? r[base + c] : 0.f;
            nd[v] = ok ? dy[base + c] : 0.f;
        }
    };
    load_row(r_begin);
    for (int row = r_begin; row < r_end; ++row) {
        const long base = (long)row * d;
        float zv[MAXV], dv[MAXV];
        bool kp[MAXV];
        float s = 0.f;
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            const int c = v * 64 + lane;
            kp[v] = false;
            zv[v] = dv[v] = 0.f;
            if (c < d) {
                kp[v] = dropout_keep(seed, (uint64_t)(base + c), thresh);
                zv[v] = nx[v] + (kp[v] ? nr[v] * keep_scale : 0.f);
                dv[v] = nd[v];
            }
            s += zv[v];
        }
        load_row(row + 1);
        const float mean = wsum(s) / (float)d;
        float q = 0.f;
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            const int c = v * 64 + lane;
            const float t = c < d ? zv[v] - mean : 0.f;
            q += t * t;
        }
        const float rstd = rsqrtf(wsum(q) / (float)d + eps);
        float sg = 0.f, sgx = 0.f;
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            const int c = v * 64 + lane;
            if (c < d) {
                const float xh = (zv[v] - mean) * rstd;
                const float gg = dv[v] * gamma[c];
                sg += gg;
                sgx += gg * xh;
                g_acc[v] += dv[v] * xh;
                b_acc[v] += dv[v];
            }
        }
        sg = wsum(sg);
        sgx = wsum(sgx);
        const float inv_d = 1.f / (float)d;
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            const int c = v * 64 + lane;
            if (c < d) {
                const float xh = (zv[v] - mean) * rstd;
                const float dz = rstd * (dv[v] * gamma[c] - sg * inv_d - xh * sgx * inv_d);
                if (dx) dx[base + c] = dz;
                if (dr) dr[base + c] = kp[v] ? dz * keep_scale : 0.f;
            }
        }
    }
    if (!pg) return;
#pragma unroll
    for (int v = 0; v < MAXV; ++v) {
        const int c = v * 64 + lane;
        if (c < d) {
            red[(wave * 2) * d + c] = g_acc[v];
            red[(wave * 2 + 1) * d + c] = b_acc[v];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < d; c += 256) {
        float sgm = 0.f, sbt = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            sgm += red[(w * 2) * d + c];
            sbt += red[(w * 2 + 1) * d + c];
        }
        pg[(long)blockIdx.x * d + c] = sgm;
        pb[(long)blockIdx.x * d + c] = sbt;
    }
}

// fixed-order sum of the per-workgroup partials: out[c] = sum_b part[b][c]; one workgroup per
// column, 256 threads striding over the partials, then a fixed tree (deterministic)
__global__ __launch_bounds__(256) void partial_sum_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                          int nb, int d) {
    __shared__ float red[256];
    const int c = blockIdx.x;
    float s = 0.f;
    for (int k = threadIdx.x; k < nb; k += 256) s += part[(long)k * d + c];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[c] = red[0];
}

// ------------------------------------------------------------------- dropout(relu(x))
// 4 elements per thread; y = Z * act(x); backward dx = Z * dy * act'(x) (act' from y > 0 for
// relu: a kept positive input is the only way y > 0).  NaN inputs stay NaN as in the torch ops
// replaced: relu(NaN) = NaN, and dropout multiplies by the 0/scale mask (NaN * 0 = NaN)
__device__ __forceinline__ float relu_nan(float t) { return (t > 0.f || t != t) ? t : 0.f; }
__global__ __launch_bounds__(256) void drop_act_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n,
                                                       const int64_t* __restrict__ seedp, uint32_t thresh,
                                                       float keep_scale, int relu) {
    const uint64_t seed = seedp ? (uint64_t)*seedp : 0;
    for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
         i += (int64_t)gridDim.x * blockDim.x * 4) {
        if (i + 4 <= n) {
            float4 v = *reinterpret_cast<const float4*>(x + i);
            float t[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (relu) t[j] = relu_nan(t[j]);
                if (seedp) t[j] *= dropout_keep(seed, (uint64_t)(i + j), thresh) ? keep_scale : 0.f;
            }
            *reinterpret_cast<float4*>(y + i) = make_float4(t[0], t[1], t[2], t[3]);
        } else {
            for (int64_t k = i; k < n; ++k) {
                float t = x[k];
                if (relu) t = relu_nan(t);
                if (seedp) t *= dropout_keep(seed, (uint64_t)k, thresh) ? keep_scale : 0.f;
                y[k] = t;
            }
        }
    }
}

__global__ __launch_bounds__(256) void drop_act_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                           float* __restrict__ dx, int64_t n,
                                                           const int64_t* __restrict__ seedp, uint32_t thresh,
                                                           float keep_scale, int relu) {
    const uint64_t seed = seedp ? (uint64_t)*seedp : 0;
    for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
         i += (int64_t)gridDim.x * blockDim.x * 4) {
        const int m = (int)min((int64_t)4, n - i);
        float g[4] = {0.f, 0.f, 0.f, 0.f}, o[4] = {1.f, 1.f, 1.f, 1.f};
        if (m == 4) {
            const float4 a = *reinterpret_cast<const float4*>(dy + i);
            g[0] = a.x; g[1] = a.y; g[2] = a.z; g[3] = a.w;
            if (relu) {
                const float4 b = *reinterpret_cast<const float4*>(y + i);
                o[0] = b.x; o[1] = b.y; o[2] = b.z; o[3] = b.w;
            }
        } else {
            for (int j = 0; j < m; ++j) {
                g[j] = dy[i + j];
                if (relu) o[j] = y[i + j];
            }
        }
        float t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float v = g[j];
            if (relu && o[j] <= 0.f) v = 0.f;   // torch threshold_backward: a NaN output passes the gradient
            if (seedp) v *= dropout_keep(seed, (uint64_t)(i + j), thresh) ? keep_scale : 0.f;
            t[j] = v;
        }
        if (m == 4) {
            *reinterpret_cast<float4*>(dx + i) = make_float4(t[0], t[1], t[2], t[3]);
        } else {
            for (int j = 0; j < m; ++j) dx[i + j] = t[j];
        }
    }
}

// ------------------------------------------------------------- MSDA sampling preparation
// Input: the packed projection output offlog (nq rows of stride ld): columns [0, M*L*P*2) the
// sampling offsets (m, l, p, xy), then M*L*P attention logits (m, l, p) -- one GEMM over the
// concatenated sampling_offsets | attention_weights weights.  One thread per (query row, head):
// softmax over the head's L*P logits (torch's exp(x - max) / sum), zeroed for masked queries;
// locations loc = ref + off / shape (2-d refs; the reference divides x by H and y by W,
// ms_deform_attn.py:78-79) or ref_xy + off / P * ref_wh * 0.5 (4-d refs).  Threads of one query
// row are M consecutive lanes (M divides 64).
__global__ __launch_bounds__(256) void msda_prep_kernel(const float* __restrict__ offlog, int64_t ld,
                                                        const float* __restrict__ ref, const int64_t* __restrict__ shapes,
                                                        const uint8_t* __restrict__ qmask, float* __restrict__ loc,
                                                        float* __restrict__ attw, int64_t nq, int M, int L, int P,
                                                        int refd) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq * M) return;
    const int64_t nqi = t / M;
    const int m = (int)(t - nqi * M);
    const int LP = L * P;
    const float* o = offlog + nqi * ld + (int64_t)m * LP * 2;
    const float* lg = offlog + nqi * ld + (int64_t)M * LP * 2 + (int64_t)m * LP;
    float* aw = attw + t * LP;
    const bool masked = qmask && qmask[nqi];
    float mx = -INFINITY;
    for (int i = 0; i < LP; ++i) mx = fmaxf(mx, lg[i]);
    float s = 0.f;
    for (int i = 0; i < LP; ++i) s += expf(lg[i] - mx);
    for (int i = 0; i < LP; ++i) aw[i] = masked ? 0.f : expf(lg[i] - mx) / s;
    float* lo = loc + t * LP * 2;
    const float* rf = ref + nqi * L * refd;
    for (int l = 0; l < L; ++l) {
        const float rx = rf[l * refd], ry = rf[l * refd + 1];
        if (refd == 2) {
            const float sh = (float)shapes[2 * l], sw = (float)shapes[2 * l + 1];
            for (int p = 0; p < P; ++p) {
                const int k = (l * P + p) * 2;
                lo[k] = rx + o[k] / sh;
                lo[k + 1] = ry + o[k + 1] / sw;
            }
        } else {
            const float rw = rf[l * refd + 2], rh = rf[l * refd + 3];
            for (int p = 0; p < P; ++p) {
                const int k = (l * P + p) * 2;
                lo[k] = rx + o[k] / (float)P * rw * 0.5f;
                lo[k + 1] = ry + o[k + 1] / (float)P * rh * 0.5f;
            }
        }
    }
}

// Vector form for P = 4 (every config): one thread per (query row, head, level) -- its 4 points'
// 8 offsets / 4 logits are 2 + 1 16-byte loads, consecutive threads read consecutive 32 / 16
// bytes (coalesced); the head's softmax max / sum over its L levels by shuffles inside groups of
// L lanes (L a power of two <= 16).
template <int L>
__global__ __launch_bounds__(256) void msda_prep_v4_kernel(const float* __restrict__ offlog, int64_t ld,
                                                           const float* __restrict__ ref,
                                                           const int64_t* __restrict__ shapes,
                                                           const uint8_t* __restrict__ qmask, float* __restrict__ loc,
                                                           float* __restrict__ attw, int64_t nq, int M, int refd) {
    constexpr int P = 4;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool on = t < nq * M * L;
    const int64_t tt = on ? t : 0;
    const int64_t hm = tt / L;              // (row, head)
    const int l = (int)(tt - hm * L);
    const int64_t nqi = hm / M;
    const int m = (int)(hm - nqi * M);
    const float* row = offlog + nqi * ld;
    const float4 o0 = *reinterpret_cast<const float4*>(row + ((int64_t)m * L + l) * P * 2);
    const float4 o1 = *reinterpret_cast<const float4*>(row + ((int64_t)m * L + l) * P * 2 + 4);
    const float4 lg = *reinterpret_cast<const float4*>(row + (int64_t)M * L * P * 2 + ((int64_t)m * L + l) * P);
    float mx = fmaxf(fmaxf(lg.x, lg.y), fmaxf(lg.z, lg.w));
#pragma unroll
    for (int o = 1; o < L; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    const float e0 = expf(lg.x - mx), e1 = expf(lg.y - mx), e2 = expf(lg.z - mx), e3 = expf(lg.w - mx);
    float s = ((e0 + e1) + e2) + e3;
#pragma unroll
    for (int o = 1; o < L; o <<= 1) s += __shfl_xor(s, o);
    if (!on) return;
    const bool masked = qmask && qmask[nqi];
    *reinterpret_cast<float4*>(attw + tt * P) =
        masked ? make_float4(0.f, 0.f, 0.f, 0.f) : make_float4(e0 / s, e1 / s, e2 / s, e3 / s);
    const float* rf = ref + (nqi * L + l) * refd;
    float4 a, b;
    if (refd == 2) {
        const float rx = rf[0], ry = rf[1];
        const float sh = (float)shapes[2 * l], sw = (float)shapes[2 * l + 1];
        a = make_float4(rx + o0.x / sh, ry + o0.y / sw, rx + o0.z / sh, ry + o0.w / sw);
        b = make_float4(rx + o1.x / sh, ry + o1.y / sw, rx + o1.z / sh, ry + o1.w / sw);
    } else {
        const float4 r = *reinterpret_cast<const float4*>(rf);
        const float fp = (float)P;
        a = make_float4(r.x + o0.x / fp * r.z * 0.5f, r.y + o0.y / fp * r.w * 0.5f, r.x + o0.z / fp * r.z * 0.5f,
                        r.y + o0.w / fp * r.w * 0.5f);
        b = make_float4(r.x + o1.x / fp * r.z * 0.5f, r.y + o1.y / fp * r.w * 0.5f, r.x + o1.z / fp * r.z * 0.5f,
                        r.y + o1.w / fp * r.w * 0.5f);
    }
    *reinterpret_cast<float4*>(loc + tt * P * 2) = a;
    *reinterpret_cast<float4*>(loc + tt * P * 2 + 4) = b;
}

// its backward, same thread map; d_ref[n, q, l] sums over the M heads of a row: lanes l, l + L,
// ... of the row's M*L-lane group (M*L <= 64), reduced by shuffles
template <int L>
__global__ __launch_bounds__(256) void msda_prep_v4_bwd_kernel(const float* __restrict__ dloc,
                                                               const float* __restrict__ dattw,
                                                               const float* __restrict__ attw,
                                                               const float* __restrict__ offlog, int64_t ld,
                                                               const float* __restrict__ ref,
                                                               const int64_t* __restrict__ shapes,
                                                               float* __restrict__ doffl, float* __restrict__ dref,
                                                               int64_t nq, int M, int refd) {
    constexpr int P = 4;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool on = t < nq * M * L;
    const int64_t tt = on ? t : 0;
    const int64_t hm = tt / L;
    const int l = (int)(tt - hm * L);
    const int64_t nqi = hm / M;
    const int m = (int)(hm - nqi * M);
    const float4 g = *reinterpret_cast<const float4*>(dattw + tt * P);
    const float4 av = *reinterpret_cast<const float4*>(attw + tt * P);
    float sga = ((g.x * av.x + g.y * av.y) + g.z * av.z) + g.w * av.w;
#pragma unroll
    for (int o = 1; o < L; o <<= 1) sga += __shfl_xor(sga, o);
    const float4 d0 = *reinterpret_cast<const float4*>(dloc + tt * P * 2);
    const float4 d1 = *reinterpret_cast<const float4*>(dloc + tt * P * 2 + 4);
    float* drow = doffl ? doffl + nqi * ld : nullptr;
    const float* rf = ref + (nqi * L + l) * refd;
    float sx = ((d0.x + d0.z) + d1.x) + d1.z, sy = ((d0.y + d0.w) + d1.y) + d1.w, sw = 0.f, sh = 0.f;
    if (on && drow) {
        *reinterpret_cast<float4*>(drow + (int64_t)M * L * P * 2 + ((int64_t)m * L + l) * P) =
            make_float4(av.x * (g.x - sga), av.y * (g.y - sga), av.z * (g.z - sga), av.w * (g.w - sga));
    }
    if (refd == 2) {
        if (on && drow) {
            const float hh = (float)shapes[2 * l], ww = (float)shapes[2 * l + 1];
            float* dof = drow + ((int64_t)m * L + l) * P * 2;
            *reinterpret_cast<float4*>(dof) = make_float4(d0.x / hh, d0.y / ww, d0.z / hh, d0.w / ww);
            *reinterpret_cast<float4*>(dof + 4) = make_float4(d1.x / hh, d1.y / ww, d1.z / hh, d1.w / ww);
        }
    } else {
        const float4 r = *reinterpret_cast<const float4*>(rf);
        const float fp = (float)P;
        const float* orow = offlog + nqi * ld + ((int64_t)m * L + l) * P * 2;
        const float4 o0 = *reinterpret_cast<const float4*>(orow);
        const float4 o1 = *reinterpret_cast<const float4*>(orow + 4);
        const float4 h0 = make_float4(d0.x * 0.5f, d0.y * 0.5f, d0.z * 0.5f, d0.w * 0.5f);
        const float4 h1 = make_float4(d1.x * 0.5f, d1.y * 0.5f, d1.z * 0.5f, d1.w * 0.5f);
        if (on && drow) {
            float* dof = drow + ((int64_t)m * L + l) * P * 2;
            *reinterpret_cast<float4*>(dof) =
                make_float4(h0.x * r.z / fp, h0.y * r.w / fp, h0.z * r.z / fp, h0.w * r.w / fp);
            *reinterpret_cast<float4*>(dof + 4) =
                make_float4(h1.x * r.z / fp, h1.y * r.w / fp, h1.z * r.z / fp, h1.w * r.w / fp);
        }
        sw = ((h0.x * (o0.x / fp) + h0.z * (o0.z / fp)) + h1.x * (o1.x / fp)) + h1.z * (o1.z / fp);
        sh = ((h0.y * (o0.y / fp) + h0.w * (o0.w / fp)) + h1.y * (o1.y / fp)) + h1.w * (o1.w / fp);
    }
    if (!dref) return;
    for (int o = L; o < M * L; o <<= 1) {
        sx += __shfl_xor(sx, o);
        sy += __shfl_xor(sy, o);
        sw += __shfl_xor(sw, o);
        sh += __shfl_xor(sh, o);
    }
    if (on && m == 0) {
        float* dr = dref + (nqi * L + l) * refd;
        dr[0] = sx;
        dr[1] = sy;
        if (refd == 4) {
            dr[2] = sw;
            dr[3] = sh;
        }
    }
}

// backward into the packed gradient of offlog (same layout and row stride): d_logit =
// a * (g - sum(g * a)) (a = the masked softmax: zero rows give zero gradients, as masked_fill
// blocks them); d_off = d_loc / shape (or ((d_loc * 0.5) * wh) / P); d_ref[n, q, l] = sum over
// heads and points of d_loc (and of (d_loc * 0.5) * off / P for the 4-d refs' w, h), reduced over
// the M lanes of a query row by shuffles.
template <int M>
__global__ __launch_bounds__(256) void msda_prep_bwd_kernel(const float* __restrict__ dloc, const float* __restrict__ dattw,
                                                            const float* __restrict__ attw, const float* __restrict__ offlog,
                                                            int64_t ld, const float* __restrict__ ref,
                                                            const int64_t* __restrict__ shapes, float* __restrict__ doffl,
                                                            float* __restrict__ dref, int64_t nq, int L, int P, int refd) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool on = t < nq * M;
    const int64_t nqi = on ? t / M : 0;
    const int m = on ? (int)(t - nqi * M) : 0;
    const int LP = L * P;
    if (on && doffl) {
        const float* a = attw + t * LP;
        const float* g = dattw + t * LP;
        float* dlg = doffl + nqi * ld + (int64_t)M * LP * 2 + (int64_t)m * LP;
        float sga = 0.f;
        for (int i = 0; i < LP; ++i) sga += g[i] * a[i];
        for (int i = 0; i < LP; ++i) dlg[i] = a[i] * (g[i] - sga);
    }
    const float* dl = dloc + (on ? t : 0) * LP * 2;
    const float* o = offlog + nqi * ld + (int64_t)m * LP * 2;
    float* dof = doffl ? doffl + nqi * ld + (int64_t)m * LP * 2 : nullptr;
    const float* rf = ref + nqi * L * refd;
    for (int l = 0; l < L; ++l) {
        float sx = 0.f, sy = 0.f, sw = 0.f, sh = 0.f;
        if (on) {
            if (refd == 2) {
                const float hh = (float)shapes[2 * l], ww = (float)shapes[2 * l + 1];
                for (int p = 0; p < P; ++p) {
                    const int k = (l * P + p) * 2;
                    const float gx = dl[k], gy = dl[k + 1];
                    if (dof) {
                        dof[k] = gx / hh;
                        dof[k + 1] = gy / ww;
                    }
                    sx += gx;
                    sy += gy;
                }
            } else {
                const float rw = rf[l * refd + 2], rh = rf[l * refd + 3];
                for (int p = 0; p < P; ++p) {
                    const int k = (l * P + p) * 2;
                    const float gx = dl[k] * 0.5f, gy = dl[k + 1] * 0.5f;
                    if (dof) {
                        dof[k] = gx * rw / (float)P;
                        dof[k + 1] = gy * rh / (float)P;
                    }
                    sx += dl[k];
                    sy += dl[k + 1];
                    sw += gx * (o[k] / (float)P);
                    sh += gy * (o[k + 1] / (float)P);
                }
            }
        }
        if (dref) {
#pragma unroll
            for (int s = 1; s < M; s <<= 1) {
                sx += __shfl_xor(sx, s);
                sy += __shfl_xor(sy, s);
                sw += __shfl_xor(sw, s);
                sh += __shfl_xor(sh, s);
            }
            if (on && m == 0) {
                float* dr = dref + nqi * L * refd + l * refd;
                dr[0] = sx;
                dr[1] = sy;
                if (refd == 4) {
                    dr[2] = sw;
                    dr[3] = sh;
                }
            }
        }
    }
}

// ------------------------------------------------------------------------ inverse_sigmoid
// x = clamp(x, 0, 1); log(clamp(x, eps) / clamp(1 - x, eps)) and its backward through torch's
// clamp masks (grad passes where min <= v <= max)
__global__ __launch_bounds__(256) void inv_sigmoid_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n,
                                                          float eps) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float xv = x[i];
    const float xc = fminf(fmaxf(xv, 0.f), 1.f);
    const float x1 = fmaxf(xc, eps), x2 = fmaxf(1.f - xc, eps);
    // torch's clamp chain propagates a NaN input (fminf / fmaxf would drop it)
    y[i] = xv != xv ? xv : logf(x1 / x2);
}

__global__ __launch_bounds__(256) void inv_sigmoid_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                              float* __restrict__ dx, int64_t n, float eps) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float xv = x[i];
    const float xc = fminf(fmaxf(xv, 0.f), 1.f);
    const float x1 = fmaxf(xc, eps), x2 = fmaxf(1.f - xc, eps);
    const float g = dy[i];
    // y = log(q), q = x1 / x2: dq = g / q; dx1 = dq / x2; dx2 = -dq * x1 / x2^2
    const float dq = g / (x1 / x2);
    float d = 0.f;
    if (xc >= eps) d += dq / x2;
    if (1.f - xc >= eps) d += dq * x1 / (x2 * x2);   // d(1 - xc)/dxc = -1
    dx[i] = (xv >= 0.f && xv <= 1.f) ? d : 0.f;
}

inline int grid_for(int64_t work, int per_block) {
    const int64_t b = (work + per_block - 1) / per_block;
    return (int)(b < kMaxGridStride ? (b > 0 ? b : 1) : kMaxGridStride);
}

}  // namespace
}  // namespace kinet

using namespace kinet;

extern "C" int kinet_dropout_add_layernorm(const float* x, const float* r, const float* gamma, const float* beta, float* y,
                                           int rows, int d, float eps, float dropout_p, const int64_t* dropout_seed,
                                           kinet_stream_t stream) {
    KINET_CHECK_ARG(rows >= 0 && d > 0 && d <= 1024 && x && r && gamma && beta && y && dropout_seed,
                    "dropout_add_layernorm: bad arguments (d must be in [1, 1024])");
    KINET_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f, "dropout_add_layernorm: p must be in [0, 1)");
    if (rows == 0) return KINET_OK;
    const dim3 grid((rows + 3) / 4), blk(256);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t th = dropout_thresh(dropout_p);
    const float ks = 1.f / (1.f - dropout_p);
#define KINET_DLN(NV) hipLaunchKernelGGL(drop_add_ln_kernel<NV>, grid, blk, 0, s, x, r, gamma, beta, y, rows, d, eps, \
                                         dropout_seed, th, ks)
    switch ((d + 63) / 64) {
        case 1: KINET_DLN(1); break;
        case 2: KINET_DLN(2); break;
        case 3: KINET_DLN(3); break;
        case 4: KINET_DLN(4); break;
        case 5: KINET_DLN(5); break;
        default: KINET_DLN(16); break;
    }
#undef KINET_DLN
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

namespace {
constexpr int kLnRowsPerWave = 8;   // ~22 waves per CU at the encoder rows (4: no faster)
}

extern "C" int64_t kinet_dropout_add_layernorm_backward_workspace(int rows, int d) {
    const int64_t blocks = (rows + 4 * kLnRowsPerWave - 1) / (4 * kLnRowsPerWave);
    return 2 * blocks * (int64_t)d;
}

extern "C" int kinet_dropout_add_layernorm_backward(const float* dy, const float* x, const float* r, const float* gamma,
                                                    float* dx, float* dr, float* dgamma, float* dbeta, int rows, int d,
                                                    float eps, float dropout_p, const int64_t* dropout_seed,
                                                    float* workspace, kinet_stream_t stream) {
    KINET_CHECK_ARG(rows >= 0 && d > 0 && d <= 1024 && dy && x && r && gamma && dropout_seed,
                    "dropout_add_layernorm_backward: bad arguments");
    KINET_CHECK_ARG((dgamma == nullptr) == (dbeta == nullptr) && (!dgamma || workspace),
                    "dropout_add_layernorm_backward: dgamma and dbeta together, with a workspace");
    KINET_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f, "dropout_add_layernorm_backward: p must be in [0, 1)");
    if (rows == 0) {
        if (dgamma) {
            KINET_CHECK_HIP(hipMemsetAsync(dgamma, 0, sizeof(float) * d, (hipStream_t)stream));
            KINET_CHECK_HIP(hipMemsetAsync(dbeta, 0, sizeof(float) * d, (hipStream_t)stream));
        }
        return KINET_OK;
    }
    hipStream_t s = (hipStream_t)stream;
    const int blocks = (rows + 4 * kLnRowsPerWave - 1) / (4 * kLnRowsPerWave);
    float* pg = dgamma ? workspace : nullptr;
    float* pb = dgamma ? workspace + (int64_t)blocks * d : nullptr;
    const uint32_t th = dropout_thresh(dropout_p);
    const float ks = 1.f / (1.f - dropout_p);
#define KINET_DLNB(NV) hipLaunchKernelGGL(drop_add_ln_bwd_kernel<NV>, dim3(blocks), dim3(256), 8 * d * sizeof(float), s, \
                                          dy, x, r, gamma, dx, dr, pg, pb, rows, d, eps, kLnRowsPerWave, dropout_seed, th, ks)
    switch ((d + 63) / 64) {
        case 1: KINET_DLNB(1); break;
        case 2: KINET_DLNB(2); break;
        case 3: KINET_DLNB(3); break;
        case 4: KINET_DLNB(4); break;
        case 5: KINET_DLNB(5); break;
        default: KINET_DLNB(16); break;
    }
#undef KINET_DLNB
    KINET_LAUNCH_CHECK();
    if (dgamma) {
        hipLaunchKernelGGL(partial_sum_kernel, dim3(d), dim3(256), 0, s, pg, dgamma, blocks, d);
        hipLaunchKernelGGL(partial_sum_kernel, dim3(d), dim3(256), 0, s, pb, dbeta, blocks, d);
        KINET_LAUNCH_CHECK();
    }
    return KINET_OK;
}

extern "C" int kinet_dropout_act(const float* x, float* y, int64_t n, int relu, float dropout_p,
                                 const int64_t* dropout_seed, kinet_stream_t stream) {
    KINET_CHECK_ARG(n >= 0 && x && y && (dropout_p == 0.f || dropout_seed) && dropout_p >= 0.f && dropout_p < 1.f,
                    "dropout_act: bad arguments");
    KINET_CHECK_ARG((((uintptr_t)x | (uintptr_t)y) & 15) == 0, "dropout_act: 16-byte aligned buffers required");
    if (n == 0) return KINET_OK;
    const int64_t* sp = dropout_p > 0.f ? dropout_seed : nullptr;
    hipLaunchKernelGGL(drop_act_kernel, dim3(grid_for((n + 3) / 4, 256)), dim3(256), 0, (hipStream_t)stream, x, y, n, sp,
                       dropout_thresh(dropout_p), 1.f / (1.f - dropout_p), relu);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_dropout_act_backward(const float* dy, const float* y, float* dx, int64_t n, int relu,
                                          float dropout_p, const int64_t* dropout_seed, kinet_stream_t stream) {
    KINET_CHECK_ARG(n >= 0 && dy && dx && (!relu || y) && (dropout_p == 0.f || dropout_seed) && dropout_p >= 0.f &&
                        dropout_p < 1.f,
                    "dropout_act_backward: bad arguments");
    KINET_CHECK_ARG((((uintptr_t)dy | (uintptr_t)dx | (uintptr_t)y) & 15) == 0,
                    "dropout_act_backward: 16-byte aligned buffers required");
    if (n == 0) return KINET_OK;
    const int64_t* sp = dropout_p > 0.f ? dropout_seed : nullptr;
    hipLaunchKernelGGL(drop_act_bwd_kernel, dim3(grid_for((n + 3) / 4, 256)), dim3(256), 0, (hipStream_t)stream, dy, y, dx,
                       n, sp, dropout_thresh(dropout_p), 1.f / (1.f - dropout_p), relu);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

namespace {
// the vector kernels' conditions: P = 4, L a power of two <= 16, 16-byte aligned rows / outputs
bool prep_v4_ok(const float* offlog, int64_t ld, const float* refs, const float* a, const float* b, int heads,
                int levels, int points, int ref_dim) {
    const bool lpow = levels == 1 || levels == 2 || levels == 4 || levels == 8 || levels == 16;
    const bool al = ((((uintptr_t)offlog) | ((uintptr_t)a) | ((uintptr_t)b) |
                      (ref_dim == 4 ? (uintptr_t)refs : 0)) & 15) == 0 && ld % 4 == 0;
    return points == 4 && lpow && al && heads * levels <= 1024;
}
}  // namespace

extern "C" int kinet_msda_prep(const float* offlog, int64_t ld, const float* refs, const int64_t* shapes,
                               const uint8_t* query_mask, float* loc, float* attw, int64_t nq, int heads, int levels,
                               int points, int ref_dim, kinet_stream_t stream) {
    KINET_CHECK_ARG(nq >= 0 && heads > 0 && levels > 0 && points > 0 && (ref_dim == 2 || ref_dim == 4) && offlog &&
                        refs && shapes && loc && attw && ld >= (int64_t)heads * levels * points * 3,
                    "msda_prep: bad arguments");
    if (nq == 0) return KINET_OK;
    const int64_t n = nq * heads;
    if (prep_v4_ok(offlog, ld, refs, loc, attw, heads, levels, points, ref_dim)) {
        const dim3 grid((unsigned)((n * levels + 255) / 256)), blk(256);
        hipStream_t s = (hipStream_t)stream;
        switch (levels) {
            case 1: hipLaunchKernelGGL(msda_prep_v4_kernel<1>, grid, blk, 0, s, offlog, ld, refs, shapes, query_mask, loc, attw, nq, heads, ref_dim); break;
            case 2: hipLaunchKernelGGL(msda_prep_v4_kernel<2>, grid, blk, 0, s, offlog, ld, refs, shapes, query_mask, loc, attw, nq, heads, ref_dim); break;
            case 4: hipLaunchKernelGGL(msda_prep_v4_kernel<4>, grid, blk, 0, s, offlog, ld, refs, shapes, query_mask, loc, attw, nq, heads, ref_dim); break;
            case 8: hipLaunchKernelGGL(msda_prep_v4_kernel<8>, grid, blk, 0, s, offlog, ld, refs, shapes, query_mask, loc, attw, nq, heads, ref_dim); break;
            default: hipLaunchKernelGGL(msda_prep_v4_kernel<16>, grid, blk, 0, s, offlog, ld, refs, shapes, query_mask, loc, attw, nq, heads, ref_dim); break;
        }
        KINET_LAUNCH_CHECK();
        return KINET_OK;
    }
    hipLaunchKernelGGL(msda_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, offlog,
                       ld, refs, shapes, query_mask, loc, attw, nq, heads, levels, points, ref_dim);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_msda_prep_backward(const float* grad_loc, const float* grad_attw, const float* attw,
                                        const float* offlog, int64_t ld, const float* refs, const int64_t* shapes,
                                        float* grad_offlog, float* grad_refs, int64_t nq, int heads, int levels,
                                        int points, int ref_dim, kinet_stream_t stream) {
    KINET_CHECK_ARG(nq >= 0 && levels > 0 && points > 0 && (ref_dim == 2 || ref_dim == 4) && grad_loc && grad_attw &&
                        attw && offlog && refs && shapes && ld >= (int64_t)heads * levels * points * 3,
                    "msda_prep_backward: bad arguments");
    KINET_CHECK_ARG(heads == 1 || heads == 2 || heads == 4 || heads == 8 || heads == 16 || heads == 32 || heads == 64,
                    "msda_prep_backward: heads must be a power of two <= 64 (got %d)", heads);
    if (nq == 0) return KINET_OK;
    const int64_t n = nq * heads;
    hipStream_t s = (hipStream_t)stream;
    if (prep_v4_ok(offlog, ld, refs, grad_loc, grad_attw, heads, levels, points, ref_dim) &&
        (((uintptr_t)attw | (uintptr_t)grad_offlog) & 15) == 0 && heads * levels <= 64) {
        const dim3 g4((unsigned)((n * levels + 255) / 256)), b4(256);
        switch (levels) {
            case 1: hipLaunchKernelGGL(msda_prep_v4_bwd_kernel<1>, g4, b4, 0, s, grad_loc, grad_attw, attw, offlog, ld, refs, shapes, grad_offlog, grad_refs, nq, heads, ref_dim); break;
            case 2: hipLaunchKernelGGL(msda_prep_v4_bwd_kernel<2>, g4, b4, 0, s, grad_loc, grad_attw, attw, offlog, ld, refs, shapes, grad_offlog, grad_refs, nq, heads, ref_dim); break;
            case 4: hipLaunchKernelGGL(msda_prep_v4_bwd_kernel<4>, g4, b4, 0, s, grad_loc, grad_attw, attw, offlog, ld, refs, shapes, grad_offlog, grad_refs, nq, heads, ref_dim); break;
            case 8: hipLaunchKernelGGL(msda_prep_v4_bwd_kernel<8>, g4, b4, 0, s, grad_loc, grad_attw, attw, offlog, ld, refs, shapes, grad_offlog, grad_refs, nq, heads, ref_dim); break;
            default: hipLaunchKernelGGL(msda_prep_v4_bwd_kernel<16>, g4, b4, 0, s, grad_loc, grad_attw, attw, offlog, ld, refs, shapes, grad_offlog, grad_refs, nq, heads, ref_dim); break;
        }
        KINET_LAUNCH_CHECK();
        return KINET_OK;
    }
    const dim3 grid((unsigned)((n + 255) / 256)), blk(256);
#define KINET_PREP_BWD(MM)                                                                                  \
    hipLaunchKernelGGL(msda_prep_bwd_kernel<MM>, grid, blk, 0, s, grad_loc, grad_attw, attw, offlog, ld, refs, \
                       shapes, grad_offlog, grad_refs, nq, levels, points, ref_dim)
    switch (heads) {
        case 1: KINET_PREP_BWD(1); break;
        case 2: KINET_PREP_BWD(2); break;
        case 4: KINET_PREP_BWD(4); break;
        case 8: KINET_PREP_BWD(8); break;
        case 16: KINET_PREP_BWD(16); break;
        case 32: KINET_PREP_BWD(32); break;
        default: KINET_PREP_BWD(64); break;
    }
#undef KINET_PREP_BWD
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_inverse_sigmoid(const float* x, float* y, int64_t n, float eps, kinet_stream_t stream) {
    KINET_CHECK_ARG(n >= 0 && x && y, "inverse_sigmoid: bad arguments");
    if (n == 0) return KINET_OK;
    hipLaunchKernelGGL(inv_sigmoid_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, y, n,
                       eps);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_inverse_sigmoid_backward(const float* dy, const float* x, float* dx, int64_t n, float eps,
                                              kinet_stream_t stream) {
    KINET_CHECK_ARG(n >= 0 && dy && x && dx, "inverse_sigmoid_backward: bad arguments");
    if (n == 0) return KINET_OK;
    hipLaunchKernelGGL(inv_sigmoid_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, dy, x,
                       dx, n, eps);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}
