// Normalisation, pooling, packing and small-attention kernels on the detection path
// (include/kinet_ops.h).  All memory-bound: vectorised 8/16-byte accesses, f32 math.
#include <hip/hip_runtime.h>

#include <math.h>

#include <algorithm>

#include "../../include/kinet_ops.h"
#include "common.h"

namespace kinet {
namespace {

template <typename T> __device__ __forceinline__ void st(T* p, float v) { *p = Cvt<T>::from(v); }
__device__ __forceinline__ void st(double* p, float v) { *p = v; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ---------------------------------------------------------------------------------
// LayerNorm: one wave per row, up to 16 elements per lane kept in registers (d <= 1024)
// ---------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void layernorm_kernel(const T* __restrict__ x, const T* __restrict__ r,
                                                        const float* __restrict__ g, const float* __restrict__ b,
                                                        T* __restrict__ y, int rows, int d, float eps) {
    constexpr int MAXE = 16;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (wave >= rows) return;
    const T* xr = x + (long)wave * d;
    const T* rr = r ? r + (long)wave * d : nullptr;
    float v[MAXE];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < MAXE; ++j) {
        const int c = lane + 64 * j;
        float t = 0.f;
        if (c < d) {
            t = to_f32(xr[c]);
            if (rr) t += to_f32(rr[c]);
        }
        v[j] = t;
        s += t;
    }
    const float mean = wave_sum(s) / (float)d;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < MAXE; ++j) {
        const int c = lane + 64 * j;
        if (c < d) {
            const float t = v[j] - mean;
            q += t * t;
        }
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)d + eps);
    T* yr = y + (long)wave * d;
#pragma unroll
    for (int j = 0; j < MAXE; ++j) {
        const int c = lane + 64 * j;
        if (c < d) st(yr + c, (v[j] - mean) * rstd * g[c] + b[c]);
    }
}

// Vector variant (row length a multiple of one 16-byte vector, at most 64 vectors): lane i of
// the row's wave holds elements [8i, 8i+8) (16-bit) or [4i, 4i+4) (f32) -- one 16-byte load /
// store per lane instead of d/64 strided scalar accesses.  Same f32 math; the sums are formed
// in a different order than the scalar kernel (row results agree to rounding).
template <typename T>
__global__ __launch_bounds__(256) void layernorm_vec_kernel(const T* __restrict__ x, const T* __restrict__ r,
                                                            const float* __restrict__ g, const float* __restrict__ b,
                                                            T* __restrict__ y, int rows, int d, float eps) {
    constexpr int V = 16 / sizeof(T);
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (wave >= rows) return;
    const int c0 = lane * V;
    const bool on = c0 < d;
    float v[V];
    float s = 0.f;
    if (on) {
        const VecT<T, V> xv = *reinterpret_cast<const VecT<T, V>*>(x + (long)wave * d + c0);
#pragma unroll
        for (int j = 0; j < V; ++j) v[j] = to_f32(xv.v[j]);
        if (r) {
            const VecT<T, V> rv = *reinterpret_cast<const VecT<T, V>*>(r + (long)wave * d + c0);
#pragma unroll
            for (int j = 0; j < V; ++j) v[j] += to_f32(rv.v[j]);
        }
#pragma unroll
        for (int j = 0; j < V; ++j) s += v[j];
    }
    const float mean = wave_sum(s) / (float)d;
    float q = 0.f;
    if (on) {
#pragma unroll
        for (int j = 0; j < V; ++j) q += (v[j] - mean) * (v[j] - mean);
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)d + eps);
    if (on) {
        VecT<T, V> o;
#pragma unroll
        for (int j = 0; j < V; ++j) o.v[j] = Cvt<T>::from((v[j] - mean) * rstd * g[c0 + j] + b[c0 + j]);
        *reinterpret_cast<VecT<T, V>*>(y + (long)wave * d + c0) = o;
    }
}

// ---------------------------------------------------------------------------------
// GroupNorm on NHWC: per-block partial (sum, sumsq) per image x group, a fixed-order
// finalize, then apply.  No float atomics anywhere: every reduction runs in a fixed order, so
// reruns (and graph replays, and two batches in flight) are bit-identical.
// Workspace (floats): stats [N][2*groups] then partials [N][nblk][2*groups].
// ---------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void gn_stats_kernel(const T* __restrict__ x, float* __restrict__ part, int HW,
                                                       int C, int groups, int pix_per_block) {
    // thread t sums channels t, t+256, ... over this block's pixel range (coalesced rows); the
    // per-channel sums are parked in LDS and each group summed in channel order
    extern __shared__ float red[];   // [2][C]
    const int n = blockIdx.y;
    const int p0 = blockIdx.x * pix_per_block;
    const int p1 = min(HW, p0 + pix_per_block);
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float s = 0.f, q = 0.f;
        for (int p = p0; p < p1; ++p) {
            const float t = to_f32(x[((long)n * HW + p) * C + c]);
            s += t;
            q += t * t;
        }
        red[c] = s;
        red[C + c] = q;
    }
    __syncthreads();
    const int cpg = C / groups;
    float* out = part + ((long)n * gridDim.x + blockIdx.x) * 2 * groups;
    for (int g = threadIdx.x; g < groups; g += blockDim.x) {
        float s = 0.f, q = 0.f;
        for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
            s += red[c];
            q += red[C + c];
        }
        out[2 * g] = s;
        out[2 * g + 1] = q;
    }
}

// stats[n][i] = sum over the nblk block partials of image n in a fixed order: with w = 2*groups
// outputs, 256/w threads share one output (strided over the blocks, loads unrolled so they are
// all in flight), then their sums are combined in thread order
__global__ __launch_bounds__(256) void gn_finalize_kernel(const float* __restrict__ part, float* __restrict__ stats,
                                                          int nblk, int groups) {
    __shared__ float red[256];
    const int n = blockIdx.x;
    const int w = 2 * groups;
    const int tpo = w <= 256 ? 256 / w : 1;   // threads per output
    const int i0 = threadIdx.x % w, k = threadIdx.x / w;
    for (int base = 0; base < w; base += 256) {
        const int i = base + (tpo > 1 ? i0 : (int)threadIdx.x);
        float a = 0.f;
        if (i < w && k < tpo) {
            const float* pp = part + (long)n * nblk * w + i;
#pragma unroll 8
            for (int b = k; b < nblk; b += tpo) a += pp[(long)b * w];
        }
        if (tpo == 1) {
            if (i < w) stats[(long)n * w + i] = a;
            continue;
        }
        red[threadIdx.x] = a;
        __syncthreads();
        if (k == 0 && i < w) {
            float t = 0.f;
            for (int j = 0; j < tpo; ++j) t += red[j * w + i0];
            stats[(long)n * w + i] = t;
        }
        break;   // tpo > 1 means w <= 256: one pass covers every output
    }
}

template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(const T* __restrict__ x, const float* __restrict__ stats,
                                                       const float* __restrict__ g, const float* __restrict__ b,
                                                       T* __restrict__ y, int N, int HW, int C, int groups,
                                                       long y_bs, float eps) {
    const long total = (long)N * HW * C;
    const int cpg = C / groups;
    const float cnt = (float)HW * cpg;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const long np = i / C;
        const int n = (int)(np / HW);
        const long p = np - (long)n * HW;
        const int grp = c / cpg;
        const float mean = stats[(long)n * 2 * groups + 2 * grp] / cnt;
        const float var = fmaxf(stats[(long)n * 2 * groups + 2 * grp + 1] / cnt - mean * mean, 0.f);
        const float v = (to_f32(x[i]) - mean) * rsqrtf(var + eps) * g[c] + b[c];
        st(y + (long)n * y_bs + p * C + c, v);
    }
}

// 16-byte vector forms (C a multiple of V = 16/sizeof(T)): a thread owns V consecutive
// channels, 16-byte loads and stores, 32-bit index math.  C/groups a multiple of V: the V
// channels are one group (one partial per thread); otherwise (STRADDLE, e.g. d = 288 in 32
// groups of 9) a vector may span two groups, so the partials are kept per channel and summed per
// group over (slot, channel) in a fixed order, and the apply looks the group up per element.
template <typename T, bool STRADDLE = false>
__global__ __launch_bounds__(256) void gn_stats_vec_kernel(const T* __restrict__ x, float* __restrict__ part, int HW,
                                                           int C, int groups, int pix_per_block) {
    constexpr int V = 16 / (int)sizeof(T);
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    __shared__ float red[2][STRADDLE ? 256 * V : 256];   // partials, summed per group in a fixed order
    const int n = blockIdx.y;
    const int p0 = blockIdx.x * pix_per_block;
    const int p1 = min(HW, p0 + pix_per_block);
    const int CV = C / V, nslot = 256 / CV;
    const int cv = threadIdx.x % CV, slot = threadIdx.x / CV;
    float* out = part + ((long)n * gridDim.x + blockIdx.x) * 2 * groups;
    if constexpr (STRADDLE) {
        float s[V], q[V];
#pragma unroll
        for (int j = 0; j < V; ++j) s[j] = q[j] = 0.f;
        if (slot < nslot) {
            const T* xb = x + (long)n * HW * C + cv * V;
            for (int p = p0 + slot; p < p1; p += nslot) {
                const u4 v = *reinterpret_cast<const u4*>(xb + (long)p * C);
                const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const float t = to_f32(e[j]);
                    s[j] += t;
                    q[j] += t * t;
                }
            }
#pragma unroll
            for (int j = 0; j < V; ++j) {
                red[0][slot * C + cv * V + j] = s[j];
                red[1][slot * C + cv * V + j] = q[j];
            }
        }
        __syncthreads();
        const int cpg = C / groups;
        for (int g = threadIdx.x; g < groups; g += blockDim.x) {
            float gs = 0.f, gq = 0.f;
            for (int sl = 0; sl < nslot; ++sl)
                for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
                    gs += red[0][sl * C + c];
                    gq += red[1][sl * C + c];
                }
            out[2 * g] = gs;
            out[2 * g + 1] = gq;
        }
        return;
    }
    float s = 0.f, q = 0.f;
    if (slot < nslot) {
        const T* xb = x + (long)n * HW * C + cv * V;
        for (int p = p0 + slot; p < p1; p += nslot) {
            const u4 v = *reinterpret_cast<const u4*>(xb + (long)p * C);
            const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const float t = to_f32(e[j]);
                s += t;
                q += t * t;
            }
        }
    }
    red[0][threadIdx.x] = s;
    red[1][threadIdx.x] = q;
    __syncthreads();
    const int vpg = C / groups / V;   // channel vectors per group
    for (int g = threadIdx.x; g < groups; g += blockDim.x) {
        float gs = 0.f, gq = 0.f;
        for (int sl = 0; sl < nslot; ++sl)
            for (int k = g * vpg; k < (g + 1) * vpg; ++k) {
                gs += red[0][sl * CV + k];
                gq += red[1][sl * CV + k];
            }
        out[2 * g] = gs;
        out[2 * g + 1] = gq;
    }
}

template <typename T, bool STRADDLE = false>
__global__ __launch_bounds__(256) void gn_apply_vec_kernel(const T* __restrict__ x, const float* __restrict__ stats,
                                                           const float* __restrict__ g, const float* __restrict__ b,
                                                           T* __restrict__ y, int HW, int C, int groups, long y_bs,
                                                           float eps) {
    // grid (ceil(HW*C/V / 256), N)
    constexpr int V = 16 / (int)sizeof(T);
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const int n = blockIdx.y;
    const int CV = C / V;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= HW * CV) return;
    const int p = i / CV, c0 = (i - p * CV) * V;
    const int cpg = C / groups, grp = c0 / cpg;
    const float cnt = (float)HW * cpg;
    const float mean = stats[(long)n * 2 * groups + 2 * grp] / cnt;
    const float var = fmaxf(stats[(long)n * 2 * groups + 2 * grp + 1] / cnt - mean * mean, 0.f);
    const float rstd = rsqrtf(var + eps);
    const u4 v = *reinterpret_cast<const u4*>(x + ((long)n * HW + p) * C + c0);
    const T* e = reinterpret_cast<const T*>(&v);
    u4 o;
    T* oe = reinterpret_cast<T*>(&o);
    if constexpr (STRADDLE) {
        // the vector's second group (if it reaches one): channels from its first channel on
        const int split = (grp + 1) * cpg - c0;
        const int grp2 = min(grp + 1, groups - 1);
        const float mean2 = stats[(long)n * 2 * groups + 2 * grp2] / cnt;
        const float var2 = fmaxf(stats[(long)n * 2 * groups + 2 * grp2 + 1] / cnt - mean2 * mean2, 0.f);
        const float rstd2 = rsqrtf(var2 + eps);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const bool hi = j >= split;
            st(oe + j, (to_f32(e[j]) - (hi ? mean2 : mean)) * (hi ? rstd2 : rstd) * g[c0 + j] + b[c0 + j]);
        }
        *reinterpret_cast<u4*>(y + (long)n * y_bs + (long)p * C + c0) = o;
        return;
    }
#pragma unroll
    for (int j = 0; j < V; ++j) st(oe + j, (to_f32(e[j]) - mean) * rstd * g[c0 + j] + b[c0 + j]);
    *reinterpret_cast<u4*>(y + (long)n * y_bs + (long)p * C + c0) = o;
}

// ---------------------------------------------------------------------------------
// max-pool 3x3 stride 2 pad 1 (NHWC)
// ---------------------------------------------------------------------------------
template <typename T>
__global__ void maxpool_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W, int C, int Ho, int Wo) {
    const long total = (long)N * Ho * Wo * C;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        long r = i / C;
        const int ow = (int)(r % Wo);
        r /= Wo;
        const int oh = (int)(r % Ho);
        const int n = (int)(r / Ho);
        float m = -INFINITY;
        for (int dy = 0; dy < 3; ++dy) {
            const int ih = oh * 2 - 1 + dy;
            if (ih < 0 || ih >= H) continue;
            for (int dx = 0; dx < 3; ++dx) {
                const int iw = ow * 2 - 1 + dx;
                if (iw < 0 || iw >= W) continue;
                m = fmaxf(m, to_f32(x[(((long)n * H + ih) * W + iw) * C + c]));
            }
        }
        st(y + i, m);
    }
}

// 16-byte vector form (C % (16/sizeof(T)) == 0): one thread = one output pixel x 16 bytes
template <typename T>
__global__ void maxpool_vec_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W, int C, int Ho,
                                   int Wo) {
    constexpr int V = 16 / sizeof(T);
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    // grid (ceil(Wo*CV / 256), Ho, N): one thread per (ow, 16-byte channel group) of output
    // row (n, oh) -- 32-bit index math only, and the rows of one image run close together so
    // the input row two output rows share is still in L2
    const int CV = C / V;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < Wo * CV) {
        const int cv = i % CV, ow = i / CV;
        const int oh = blockIdx.y, n = blockIdx.z;
        float m[V];
#pragma unroll
        for (int j = 0; j < V; ++j) m[j] = -INFINITY;
        for (int dy = 0; dy < 3; ++dy) {
            const int ih = oh * 2 - 1 + dy;
            if (ih < 0 || ih >= H) continue;
            for (int dx = 0; dx < 3; ++dx) {
                const int iw = ow * 2 - 1 + dx;
                if (iw < 0 || iw >= W) continue;
                const u4 v = *reinterpret_cast<const u4*>(x + (((long)n * H + ih) * W + iw) * C + cv * V);
                const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
                for (int j = 0; j < V; ++j) m[j] = fmaxf(m[j], to_f32(e[j]));
            }
        }
        u4 o;
        T* oe = reinterpret_cast<T*>(&o);
#pragma unroll
        for (int j = 0; j < V; ++j) st(oe + j, m[j]);
        *reinterpret_cast<u4*>(y + (((long)n * Ho + oh) * Wo + ow) * C + cv * V) = o;
    }
}

template <typename T>
__global__ void pack_image_kernel(const float* __restrict__ x, T* __restrict__ y, int N, int H, int W, int Cp) {
    const long total = (long)N * H * W * Cp;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int c = (int)(i % Cp);
        const long pix = i / Cp;
        const int n = (int)(pix / ((long)H * W));
        const long hw = pix - (long)n * H * W;
        float v = 0.f;
        if (c < 3) v = x[((long)n * 3 + c) * H * W + hw];
        st(y + i, v);
    }
}

// Stem input with the horizontal filter taps folded into channels: for a KH x KW stride-s
// convolution of a 3-channel image, y[n][h][ow][kw*3 + c] = x[n][c][h][ow*s - pad + kw] (0
// outside the image and for channels >= 3*KW up to Cg), so the convolution becomes KH x 1
// with stride (s, 1) over Cg channels: K = KH*Cg (7*24 = 168) instead of KH*KW*8 = 392 for
// the 8-channel-padded image -- 2.3x fewer MFMA flops in ResNet's 7x7 stem (backbone.py:
// torchvision conv1).
constexpr int kFoldPx = 672;    // output pixels per workgroup of pack_image_kwfold_kernel (a 1333-wide image row)

template <typename T>
__global__ __launch_bounds__(256) void pack_image_kwfold_kernel(const float* __restrict__ x, T* __restrict__ y, int H,
                                                                int W, int Wo, int KW, int stride, int pad, int Cg) {
    // grid (ceil(Wo / kFoldPx), H, N).  The input span of this pixel run is staged in LDS by
    // coalesced loads; then work item t writes 16-byte chunk (t % nch) of pixel t / nch, so
    // every store instruction covers one contiguous 1 KiB run of the folded row.
    constexpr int EPC = 16 / (int)sizeof(T);
    extern __shared__ float xs[];               // [3][span]
    const int h = blockIdx.y, n = blockIdx.z;
    const int ow0 = blockIdx.x * kFoldPx;
    const int npx = min(kFoldPx, Wo - ow0);
    const int col0 = ow0 * stride - pad;
    const int span = (kFoldPx - 1) * stride + KW;
    const long plane = (long)H * W;
    const float* xr = x + (long)n * 3 * plane + (long)h * W;
    for (int t = threadIdx.x; t < 3 * span; t += 256) {
        const int c = t / span, k = t - c * span, col = col0 + k;
        xs[t] = (unsigned)col < (unsigned)W ? xr[c * plane + col] : 0.f;
    }
    __syncthreads();
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const int nch = Cg / EPC;
    T* yrow = y + (((long)n * H + h) * Wo + ow0) * Cg;
    for (int t = threadIdx.x; t < npx * nch; t += 256) {
        const int px = t / nch, q = t - px * nch;
        T o[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
            const int j = q * EPC + e, kw = j / 3, c = j - kw * 3;
            o[e] = Cvt<T>::from(kw < KW ? xs[c * span + px * stride + kw] : 0.f);
        }
        reinterpret_cast<u4*>(yrow)[t] = *reinterpret_cast<const u4*>(o);
    }
}

template <typename T>
__global__ void add_kernel(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ y, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        st(y + i, to_f32(a[i]) + to_f32(b[i]));
}

// ---------------------------------------------------------------------------------
// MHA core (decoder query self-attention, a few hundred queries): online softmax.
// Block = 256 threads = 16 queries x 4 lanes per query (each lane D/4 dims, dot products
// reduced by two shuffles) x 4 waves, wave w taking keys w, w+4, ... of each 64-key tile
// staged in LDS as f32 rows (broadcast vector reads); the 4 partial softmax states per
// query are merged through LDS at the end.
// ---------------------------------------------------------------------------------
template <typename T, int D>
__global__ __launch_bounds__(256) void mha_kernel(const T* __restrict__ Q, int ldq, const T* __restrict__ Kt, int ldk,
                                                  const T* __restrict__ V, int ldv, T* __restrict__ O, int ldo,
                                                  int Lq, int Lk, int heads, float scale,
                                                  const uint8_t* __restrict__ kmask, const int64_t* __restrict__ dseed,
                                                  uint32_t dthresh, float dscale) {
    constexpr int KT = 64;
    constexpr int QB = 16;                // queries per block
    constexpr int DPL = D / 4;            // dims per lane
    constexpr int LDR = D + 4;            // LDS row stride (floats)
    __shared__ __attribute__((aligned(16))) float ks[KT][LDR];
    __shared__ __attribute__((aligned(16))) float vs[KT][LDR];
    __shared__ float kvalid[KT];
    __shared__ float pm[4][QB], pl[4][QB];
    __shared__ float po[4][QB][D + 1];
    const int b = blockIdx.z, h = blockIdx.y;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sub = lane & 3, ql = lane >> 2;
    const int qi = blockIdx.x * QB + ql;
    const bool qok = qi < Lq;
    float q[DPL], o[DPL];
#pragma unroll
    for (int j = 0; j < DPL; ++j) {
        q[j] = qok ? to_f32(Q[((long)b * Lq + qi) * ldq + h * D + sub * DPL + j]) * scale : 0.f;
        o[j] = 0.f;
    }
    float mx = -INFINITY, l = 0.f;
    // dropout (training): probabilities of dropped keys leave the numerator only; the softmax
    // normaliser l keeps every key (F.dropout after softmax)
    const uint64_t seed = dseed ? (uint64_t)*dseed : 0ull;
    const uint64_t drow = (((uint64_t)b * heads + h) * (uint64_t)Lq + (uint64_t)(qok ? qi : 0)) * (uint64_t)Lk;
    for (int k0 = 0; k0 < Lk; k0 += KT) {
        __syncthreads();
        for (int i = threadIdx.x; i < KT * D; i += 256) {
            const int kk = i / D, j = i - kk * D;
            const int kr = k0 + kk;
            float kv = 0.f, vv = 0.f;
            if (kr < Lk) {
                kv = to_f32(Kt[((long)b * Lk + kr) * ldk + h * D + j]);
                vv = to_f32(V[((long)b * Lk + kr) * ldv + h * D + j]);
            }
            ks[kk][j] = kv;
            vs[kk][j] = vv;
        }
        if (threadIdx.x < KT) {
            const int kr = k0 + threadIdx.x;
            kvalid[threadIdx.x] = (kr < Lk && !(kmask && kmask[(long)b * Lk + kr])) ? 1.f : 0.f;
        }
        __syncthreads();
        const int kn = min(KT, Lk - k0);
        for (int kk = wave; kk < kn; kk += 4) {
            const float* kr = &ks[kk][sub * DPL];
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < DPL; ++j) s += q[j] * kr[j];
            s += __shfl_xor(s, 1);
            s += __shfl_xor(s, 2);
            if (kvalid[kk] == 0.f) continue;      // uniform across the 4 lanes of a query
            const float nm = fmaxf(mx, s);
            const float corr = __expf(mx - nm);
            const float pexp = __expf(s - nm);
            l = l * corr + pexp;
            const float pz = dseed ? (dropout_keep(seed, drow + (uint64_t)(k0 + kk), dthresh) ? pexp * dscale : 0.f)
                                   : pexp;
            const float* vr = &vs[kk][sub * DPL];
#pragma unroll
            for (int j = 0; j < DPL; ++j) o[j] = o[j] * corr + pz * vr[j];
            mx = nm;
        }
    }
    if (sub == 0) {
        pm[wave][ql] = mx;
        pl[wave][ql] = l;
    }
#pragma unroll
    for (int j = 0; j < DPL; ++j) po[wave][ql][sub * DPL + j] = o[j];
    __syncthreads();
    if (wave != 0 || !qok) return;
    float M_ = -INFINITY;
    for (int w = 0; w < 4; ++w) M_ = fmaxf(M_, pm[w][ql]);
    float L_ = 0.f, acc[DPL];
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc[j] = 0.f;
    for (int w = 0; w < 4; ++w) {
        const float f = pm[w][ql] == -INFINITY ? 0.f : __expf(pm[w][ql] - M_);
        L_ += pl[w][ql] * f;
#pragma unroll
        for (int j = 0; j < DPL; ++j) acc[j] += po[w][ql][sub * DPL + j] * f;
    }
    const float inv = L_ > 0.f ? 1.f / L_ : 0.f;
#pragma unroll
    for (int j = 0; j < DPL; ++j) st(O + ((long)b * Lq + qi) * ldo + h * D + sub * DPL + j, acc[j] * inv);
}

__device__ __forceinline__ float inv_sigmoid(float x) {
    // util/misc.py:609-613 (eps 1e-5)
    x = fminf(fmaxf(x, 0.f), 1.f);
    const float x1 = fmaxf(x, 1e-5f), x2 = fmaxf(1.f - x, 1e-5f);
    return logf(x1 / x2);
}

__global__ void box_refine_kernel(const float* __restrict__ tmp, const float* __restrict__ ref, int rd,
                                  const float* __restrict__ vr, float* __restrict__ nref, float* __restrict__ rin,
                                  int N, int Q, int L) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N * Q) return;
    const int b = i / Q;
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float t = tmp[(long)i * 4 + j];
        if (j < rd) t += inv_sigmoid(ref[(long)i * rd + j]);
        o[j] = 1.f / (1.f + __expf(-t));
        nref[(long)i * 4 + j] = o[j];
    }
    if (rin) {
        for (int l = 0; l < L; ++l) {
            const float vx = vr[((long)b * L + l) * 2], vy = vr[((long)b * L + l) * 2 + 1];
            float* p = rin + ((long)i * L + l) * 4;
            p[0] = o[0] * vx;
            p[1] = o[1] * vy;
            p[2] = o[2] * vx;
            p[3] = o[3] * vy;
        }
    }
}

int grid_for(long n, int block = 256) {
    long g = (n + block - 1) / block;
    if (g > 8 * kMaxGridStride) g = 8 * kMaxGridStride;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace
}  // namespace kinet

using namespace kinet;

#define DISPATCH_T(dtype, F)                                                 \
    switch (dtype) {                                                         \
        case KINET_F32: { typedef float T; F; break; }                       \
        case KINET_BF16: { typedef bf16_t T; F; break; }                     \
        case KINET_F16: { typedef f16_t T; F; break; }                       \
        default: set_error("unsupported dtype %d", dtype); return KINET_ERR_ARG; \
    }

extern "C" int kinet_layernorm(const void* x, const void* r, const float* gamma, const float* beta, void* y, int rows,
                               int d, float eps, int dtype, int reserved, kinet_stream_t stream) {
    (void)reserved;
    KINET_CHECK_ARG(rows >= 0 && d > 0 && d <= 1024, "layernorm: d must be in [1, 1024] (got %d)", d);
    if (rows == 0) return KINET_OK;
    const int blocks = (rows + 3) / 4;
    const int es = dtype == KINET_F32 ? 4 : 2;
    const bool vec = dtype != KINET_F64 && (d * es) % 16 == 0 && d * es <= 64 * 16 &&
                     ((((uintptr_t)x) | ((uintptr_t)y) | (r ? (uintptr_t)r : 0)) & 15) == 0;
    if (vec) {
        DISPATCH_T(dtype, hipLaunchKernelGGL((layernorm_vec_kernel<T>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                                             (const T*)x, (const T*)r, gamma, beta, (T*)y, rows, d, eps));
    } else {
        DISPATCH_T(dtype, hipLaunchKernelGGL((layernorm_kernel<T>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                                             (const T*)x, (const T*)r, gamma, beta, (T*)y, rows, d, eps));
    }
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

namespace {
// pixels per stats block: 128 on the vector path, 64 on the scalar path
bool gn_vec_ok(const void* x, const void* y, int HW, int C, int groups, int y_batch_stride, int N, int dtype) {
    const int V = dtype == KINET_F32 ? 4 : 8;
    // (groups of fewer than V channels would need a third group per vector: scalar path)
    return dtype != KINET_F64 && C % V == 0 && C / groups >= V && C / V <= 256 && y_batch_stride % V == 0 &&
           (((uintptr_t)x | (uintptr_t)y) & 15) == 0 && (long)HW * (C / V) < (1L << 31) && N <= 65535;
}
long gn_workspace(int N, int HW, int groups, int ppb) {
    const long nblk = (HW + ppb - 1) / ppb;
    return 2L * N * groups * (1 + nblk);
}
}  // namespace

extern "C" long kinet_groupnorm_workspace(int N, int HW, int C, int groups, int dtype) {
    (void)C;
    (void)dtype;
    if (N <= 0 || HW <= 0 || groups <= 0) return 0;
    return gn_workspace(N, HW, groups, 64);   // the larger of the two paths' needs
}

extern "C" int kinet_groupnorm(const void* x, const float* gamma, const float* beta, void* y, int N, int HW, int C,
                               int groups, int y_batch_stride, float eps, int dtype, float* stats,
                               kinet_stream_t stream) {
    KINET_CHECK_ARG(N >= 0 && HW > 0 && C > 0 && groups > 0 && C % groups == 0, "groupnorm: bad geometry");
    KINET_CHECK_ARG(y_batch_stride >= HW * C, "groupnorm: y_batch_stride < HW*C");
    KINET_CHECK_ARG(stats != nullptr, "groupnorm: workspace of kinet_groupnorm_workspace() floats required");
    if (N == 0) return KINET_OK;
    hipStream_t s = (hipStream_t)stream;
    const bool vec = gn_vec_ok(x, y, HW, C, groups, y_batch_stride, N, dtype);
    const int ppb = vec ? 128 : 64;
    const int nblk = (HW + ppb - 1) / ppb;
    float* part = stats + 2L * N * groups;
    const dim3 g1(nblk, N);
    if (vec) {
        const int V = dtype == KINET_F32 ? 4 : 8;
        const dim3 g2((unsigned)(((long)HW * (C / V) + 255) / 256), N);
        const bool straddle = (C / groups) % V != 0;
#define GNV(TT, SD)                                                                                              \
    do {                                                                                                         \
        hipLaunchKernelGGL((gn_stats_vec_kernel<TT, SD>), g1, dim3(256), 0, s, (const TT*)x, part, HW, C, groups, \
                           ppb);                                                                                 \
        hipLaunchKernelGGL(gn_finalize_kernel, dim3(N), dim3(256), 0, s, (const float*)part, stats, nblk, groups); \
        hipLaunchKernelGGL((gn_apply_vec_kernel<TT, SD>), g2, dim3(256), 0, s, (const TT*)x, stats, gamma, beta, \
                           (TT*)y, HW, C, groups, (long)y_batch_stride, eps);                                    \
    } while (0)
        if (straddle) {
            if (dtype == KINET_BF16) GNV(bf16_t, true);
            else if (dtype == KINET_F16) GNV(f16_t, true);
            else GNV(float, true);
        } else {
            if (dtype == KINET_BF16) GNV(bf16_t, false);
            else if (dtype == KINET_F16) GNV(f16_t, false);
            else GNV(float, false);
        }
#undef GNV
        KINET_LAUNCH_CHECK();
        return KINET_OK;
    }
    KINET_CHECK_ARG(C <= 8192, "groupnorm: C up to 8192 on the scalar path");
    DISPATCH_T(dtype, hipLaunchKernelGGL((gn_stats_kernel<T>), g1, dim3(256), 2 * C * sizeof(float), s,
                                         (const T*)x, part, HW, C, groups, ppb));
    hipLaunchKernelGGL(gn_finalize_kernel, dim3(N), dim3(256), 0, s, (const float*)part, stats, nblk, groups);
    KINET_LAUNCH_CHECK();
    const long total = (long)N * HW * C;
    DISPATCH_T(dtype, hipLaunchKernelGGL((gn_apply_kernel<T>), dim3(grid_for(total)), dim3(256), 0, s, (const T*)x,
                                         stats, gamma, beta, (T*)y, N, HW, C, groups, (long)y_batch_stride, eps));
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_maxpool2d_3x3s2(const void* x, void* y, int N, int H, int W, int C, int dtype,
                                     kinet_stream_t stream) {
    KINET_CHECK_ARG(N >= 0 && H > 0 && W > 0 && C > 0, "maxpool: bad geometry");
    const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
    const long total = (long)N * Ho * Wo * C;
    if (total == 0) return KINET_OK;
    const bool vec = (dtype == KINET_F32 ? C % 4 : C % 8) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0;
    if (vec) {
        const int cv = C / (dtype == KINET_F32 ? 4 : 8);
        KINET_CHECK_ARG(Ho <= 65535 && N <= 65535 && (long)Wo * cv < (1L << 31), "maxpool: too large");
        const dim3 grid((unsigned)((Wo * cv + 255) / 256), Ho, N);
        DISPATCH_T(dtype, hipLaunchKernelGGL((maxpool_vec_kernel<T>), grid, dim3(256), 0,
                                             (hipStream_t)stream, (const T*)x, (T*)y, N, H, W, C, Ho, Wo));
    } else {
        DISPATCH_T(dtype, hipLaunchKernelGGL((maxpool_kernel<T>), dim3(grid_for(total)), dim3(256), 0,
                                             (hipStream_t)stream, (const T*)x, (T*)y, N, H, W, C, Ho, Wo));
    }
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_pack_image_nhwc(const float* x, void* y, int N, int H, int W, int Cpad, int dtype,
                                     kinet_stream_t stream) {
    KINET_CHECK_ARG(N >= 0 && H > 0 && W > 0 && Cpad >= 3, "pack_image: bad geometry");
    const long total = (long)N * H * W * Cpad;
    if (total == 0) return KINET_OK;
    DISPATCH_T(dtype, hipLaunchKernelGGL((pack_image_kernel<T>), dim3(grid_for(total)), dim3(256), 0,
                                         (hipStream_t)stream, x, (T*)y, N, H, W, Cpad));
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_pack_image_kwfold(const float* x, void* y, int N, int H, int W, int KW, int stride, int pad,
                                       int Cg, int dtype, kinet_stream_t stream) {
    KINET_CHECK_ARG(N >= 0 && H > 0 && W > 0 && KW > 0 && stride > 0 && pad >= 0 && W + 2 * pad >= KW,
                    "pack_image_kwfold: bad geometry");
    KINET_CHECK_ARG(Cg % 8 == 0 && Cg >= 3 * KW, "pack_image_kwfold: Cg (%d) must be a multiple of 8 >= 3*KW", Cg);
    KINET_CHECK_ARG(dtype == KINET_BF16 || dtype == KINET_F16 || dtype == KINET_F32,
                    "pack_image_kwfold: output dtype must be bf16, f16 or f32");
    KINET_CHECK_ARG((((uintptr_t)y) & 15u) == 0, "pack_image_kwfold: y must be 16-byte aligned");
    KINET_CHECK_ARG(H <= 65535 && N <= 65535, "pack_image_kwfold: H and N must be <= 65535");
    const int Wo = (W + 2 * pad - KW) / stride + 1;
    if (N == 0) return KINET_OK;
    const dim3 grid((Wo + kFoldPx - 1) / kFoldPx, H, N);
    const size_t lds = 3 * ((kFoldPx - 1) * stride + KW) * sizeof(float);
    KINET_CHECK_ARG(lds <= 64 * 1024, "pack_image_kwfold: stride / KW too large");
    if (dtype == KINET_BF16)
        hipLaunchKernelGGL((pack_image_kwfold_kernel<bf16_t>), grid, dim3(256), lds, (hipStream_t)stream, x, (bf16_t*)y,
                           H, W, Wo, KW, stride, pad, Cg);
    else if (dtype == KINET_F16)
        hipLaunchKernelGGL((pack_image_kwfold_kernel<f16_t>), grid, dim3(256), lds, (hipStream_t)stream, x, (f16_t*)y,
                           H, W, Wo, KW, stride, pad, Cg);
    else
        hipLaunchKernelGGL((pack_image_kwfold_kernel<float>), grid, dim3(256), lds, (hipStream_t)stream, x, (float*)y,
                           H, W, Wo, KW, stride, pad, Cg);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_add(const void* a, const void* b, void* y, int64_t n, int dtype, kinet_stream_t stream) {
    KINET_CHECK_ARG(n >= 0, "add: n < 0");
    if (n == 0) return KINET_OK;
    DISPATCH_T(dtype, hipLaunchKernelGGL((add_kernel<T>), dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                         (const T*)a, (const T*)b, (T*)y, (long)n));
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

namespace kinet {
// attn.hip: the MFMA kernel for head_dim 32, 16-bit, Lk <= 384 (false = not covered)
bool launch_mha_mfma(const void* Q, int ldq, const void* Kt, int ldk, const void* V, int ldv, void* O, int ldo,
                     int batch, int Lq, int Lk, int heads, int head_dim, float scale, int dtype,
                     const uint8_t* key_mask, hipStream_t stream);
thread_local int mha_use_mfma = 1;   // test-only knob (kinet_mha_set_mfma), per calling thread
}  // namespace kinet

extern "C" int kinet_mha_set_mfma(int enable) {
    const int old = kinet::mha_use_mfma;
    kinet::mha_use_mfma = enable;
    return old;
}

static int mha_core_impl(const void* Q, int ldq, const void* Kt, int ldk, const void* V, int ldv, void* O, int ldo,
                         int batch, int Lq, int Lk, int heads, int head_dim, float scale, int dtype,
                         const uint8_t* key_mask, float dropout_p, const int64_t* dropout_seed, kinet_stream_t stream) {
    KINET_CHECK_ARG(batch >= 0 && Lq >= 0 && Lk >= 0 && heads > 0, "mha: bad sizes");
    KINET_CHECK_ARG(head_dim == 32 || head_dim == 36 || head_dim == 16 || head_dim == 64,
                    "mha: head_dim %d not instantiated (16/32/36/64)", head_dim);
    KINET_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || dropout_seed),
                    "mha: dropout p %g must be in [0, 1) with a seed", (double)dropout_p);
    if (batch == 0 || Lq == 0) return KINET_OK;
    hipStream_t s = (hipStream_t)stream;
    const bool drop = dropout_p > 0.f;
    if (!drop && kinet::mha_use_mfma &&
        kinet::launch_mha_mfma(Q, ldq, Kt, ldk, V, ldv, O, ldo, batch, Lq, Lk, heads, head_dim, scale, dtype, key_mask,
                               s)) {
        KINET_LAUNCH_CHECK();
        return KINET_OK;
    }
    const int64_t* dseed = drop ? dropout_seed : nullptr;
    const uint32_t dthresh = kinet::dropout_thresh(dropout_p);
    const float dscale = drop ? 1.f / (1.f - dropout_p) : 1.f;
    dim3 grid((Lq + 15) / 16, heads, batch);
#define MH(DD) DISPATCH_T(dtype, hipLaunchKernelGGL((mha_kernel<T, DD>), grid, dim3(256), 0, s, (const T*)Q, ldq, \
                                                   (const T*)Kt, ldk, (const T*)V, ldv, (T*)O, ldo, Lq, Lk, heads, \
                                                   scale, key_mask, dseed, dthresh, dscale))
    switch (head_dim) {
        case 16: MH(16); break;
        case 32: MH(32); break;
        case 36: MH(36); break;
        case 64: MH(64); break;
    }
#undef MH
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_mha_core(const void* Q, int ldq, const void* Kt, int ldk, const void* V, int ldv, void* O, int ldo,
                              int batch, int Lq, int Lk, int heads, int head_dim, float scale, int dtype,
                              const uint8_t* key_mask, kinet_stream_t stream) {
    return mha_core_impl(Q, ldq, Kt, ldk, V, ldv, O, ldo, batch, Lq, Lk, heads, head_dim, scale, dtype, key_mask, 0.f,
                         nullptr, stream);
}

extern "C" int kinet_mha_core_dropout(const void* Q, int ldq, const void* Kt, int ldk, const void* V, int ldv, void* O,
                                      int ldo, int batch, int Lq, int Lk, int heads, int head_dim, float scale,
                                      int dtype, const uint8_t* key_mask, float dropout_p, const int64_t* dropout_seed,
                                      kinet_stream_t stream) {
    return mha_core_impl(Q, ldq, Kt, ldk, V, ldv, O, ldo, batch, Lq, Lk, heads, head_dim, scale, dtype, key_mask,
                         dropout_p, dropout_seed, stream);
}

namespace kinet {
namespace {
__global__ void dropout_mask_kernel(const int64_t* __restrict__ dseed, uint8_t* __restrict__ keep, long n,
                                    uint32_t thresh) {
    const uint64_t seed = (uint64_t)*dseed;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        keep[i] = dropout_keep(seed, (uint64_t)i, thresh) ? 1 : 0;
}
}  // namespace
}  // namespace kinet

extern "C" int kinet_dropout_mask(const int64_t* dropout_seed, int64_t n, float dropout_p, uint8_t* keep,
                                  kinet_stream_t stream) {
    KINET_CHECK_ARG(n >= 0 && dropout_seed && dropout_p >= 0.f && dropout_p < 1.f, "dropout_mask: bad arguments");
    if (n == 0) return KINET_OK;
    const long blocks = std::min<long>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(kinet::dropout_mask_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, dropout_seed, keep,
                       (long)n, kinet::dropout_thresh(dropout_p));
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_box_refine(const float* tmp, const float* ref, int ref_dim, const float* valid_ratios,
                                float* new_ref, float* ref_input, int N, int Q, int L, kinet_stream_t stream) {
    KINET_CHECK_ARG(ref_dim == 2 || ref_dim == 4, "box_refine: ref_dim must be 2 or 4");
    if (N * Q == 0) return KINET_OK;
    hipLaunchKernelGGL(box_refine_kernel, dim3((N * Q + 255) / 256), dim3(256), 0, (hipStream_t)stream, tmp, ref,
                       ref_dim, valid_ratios, new_ref, ref_input, N, Q, L);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

// ---------------------------------------------------------------------------------
// sine position embedding (position_encoding.py:85-121 2-d, :12-81 3-d), NHWC rows
// ---------------------------------------------------------------------------------
namespace kinet {
namespace {
// a workgroup owns 64 consecutive pixels: 4 threads per pixel split its column / row
// cumulative counts of unmasked pixels (the reference's two cumsums), the (z, y, x) embedding
// arguments go through LDS, then the 256 threads write the 64 x C outputs channel-fastest
// (coalesced NHWC rows)
constexpr int SE_PIX = 64;
template <typename TO>
__global__ __launch_bounds__(256) void sine_embed_kernel(const uint8_t* __restrict__ mask, const float* __restrict__ dim_t,
                                                         const float* __restrict__ level_embed, TO* __restrict__ out,
                                                         int B, int H, int W, int npf, int three_d, int frame,
                                                         int frames, int normalize, float scale, long out_bs) {
    __shared__ float arg[SE_PIX][3];
    const long total = (long)B * H * W;
    const int C = (three_d ? 3 : 2) * npf;
    for (long p0 = (long)blockIdx.x * SE_PIX; p0 < total; p0 += (long)gridDim.x * SE_PIX) {
        {
            const int pl = threadIdx.x >> 2, part = threadIdx.x & 3;
            const long i = p0 + pl;
            float ycum = 0.f, ytot = 0.f, xcum = 0.f, xtot = 0.f;
            int h = 0, w = 0, b = 0;
            if (i < total) {
                w = (int)(i % W);
                const long r = i / W;
                h = (int)(r % H);
                b = (int)(r / H);
                const uint8_t* mb = mask + (long)b * H * W;
                for (int k = part; k < H; k += 4) {
                    const float v = mb[(long)k * W + w] ? 0.f : 1.f;
                    ytot += v;
                    if (k <= h) ycum += v;
                }
                for (int k = part; k < W; k += 4) {
                    const float v = mb[(long)h * W + k] ? 0.f : 1.f;
                    xtot += v;
                    if (k <= w) xcum += v;
                }
            }
#pragma unroll
            for (int o = 1; o < 4; o <<= 1) {   // the 4 threads of a pixel are adjacent lanes
                ycum += __shfl_xor(ycum, o);
                ytot += __shfl_xor(ytot, o);
                xcum += __shfl_xor(xcum, o);
                xtot += __shfl_xor(xtot, o);
            }
            if (part == 0 && i < total) {
                const bool valid = !mask[(long)b * H * W + (long)h * W + w];
                float ye = ycum, xe = xcum, ze = valid ? (float)(frame + 1) : 0.f;
                if (normalize) {
                    const float eps = 1e-6f;
                    if (three_d) {   // position_encoding.py:49-51, no -0.5 offset
                        ze = ze / ((valid ? (float)frames : 0.f) + eps) * scale;
                        ye = ye / (ytot + eps) * scale;
                        xe = xe / (xtot + eps) * scale;
                    } else {         // :106-108
                        ye = (ye - 0.5f) / (ytot + eps) * scale;
                        xe = (xe - 0.5f) / (xtot + eps) * scale;
                    }
                }
                arg[pl][0] = three_d ? ze : ye;
                arg[pl][1] = three_d ? ye : xe;
                arg[pl][2] = xe;
            }
        }
        __syncthreads();
        const int np = (int)min((long)SE_PIX, total - p0);
        // channel order: [z (3-d only) | y | x], each interleaving sin (even) / cos (odd)
        for (int e = threadIdx.x; e < np * C; e += 256) {
            const int pl = e / C, c = e - pl * C;
            const long i = p0 + pl;
            const int part = c / npf, k = c - part * npf;
            const float a = arg[pl][part] / dim_t[k];
            float v = (k & 1) ? cosf(a) : sinf(a);
            if (level_embed) v += level_embed[c];
            const long b = i / ((long)H * W), hw = i - b * H * W;
            out[b * out_bs + hw * C + c] = Cvt<TO>::from(v);
        }
        __syncthreads();
    }
}
}  // namespace
}  // namespace kinet

extern "C" int kinet_sine_position_embed(const uint8_t* mask, const float* dim_t, const float* level_embed, void* out,
                                         int B, int H, int W, int num_pos_feats, int three_d, int frame, int frames,
                                         int normalize, float scale, int64_t out_batch_stride, int out_dtype,
                                         kinet_stream_t stream) {
    using namespace kinet;
    KINET_CHECK_ARG(mask && dim_t && out && num_pos_feats > 0 && B >= 0 && H >= 0 && W >= 0,
                    "sine_position_embed: bad arguments");
    KINET_CHECK_ARG(!three_d || (frames > 0 && frame >= 0 && frame < frames), "sine_position_embed: frame %d of %d",
                    frame, frames);
    const long n = (long)B * H * W;
    if (n == 0) return KINET_OK;
    const int grid = (int)std::min<long>((n + SE_PIX - 1) / SE_PIX, 8192);
    hipStream_t s = (hipStream_t)stream;
#define SE(TO) hipLaunchKernelGGL(sine_embed_kernel<TO>, dim3(grid), dim3(256), 0, s, mask, dim_t, level_embed, (TO*)out, \
                                  B, H, W, num_pos_feats, three_d, frame, frames, normalize, scale, (long)out_batch_stride)
    if (out_dtype == KINET_F32) SE(float);
    else if (out_dtype == KINET_BF16) SE(bf16_t);
    else if (out_dtype == KINET_F16) SE(f16_t);
    else { set_error("sine_position_embed: unsupported dtype %d", out_dtype); return KINET_ERR_ARG; }
#undef SE
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

// ---------------------------------------------------------------------------------
// greedy non-maximum suppression (torchvision.ops.nms semantics, tracker.py:437, :511)
// ---------------------------------------------------------------------------------
namespace kinet {
namespace {
constexpr int NMS_MAX = 4096;

// one workgroup: rank every box by score (descending, ties by index -- a stable order; NaN
// scores rank first), then
// walk the ranks; each kept box suppresses, in parallel, every later box with IoU > thresh
__global__ __launch_bounds__(1024) void nms_kernel(const float* __restrict__ boxes, const float* __restrict__ scores,
                                                   uint8_t* __restrict__ keep, int n, float thresh) {
    __shared__ int order[NMS_MAX];
    __shared__ uint8_t supp[NMS_MAX];
    __shared__ int cur;
    // scores compared as monotone integer keys: a strict total order even with NaNs (which
    // rank first, as torch.sort(descending=True) places them), so every rank is written once
    auto key = [](float f) -> uint32_t {
        const uint32_t u = __float_as_uint(f);
        if ((u & 0x7fffffffu) > 0x7f800000u) return 0xffffffffu;
        return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    };
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t si = key(scores[i]);
        int r = 0;
        for (int j = 0; j < n; ++j) {
            const uint32_t sj = key(scores[j]);
            r += (sj > si || (sj == si && j < i)) ? 1 : 0;
        }
        order[r] = i;
        supp[i] = 0;
        keep[i] = 0;
    }
    __syncthreads();
    for (int r = 0; r < n; ++r) {
        if (threadIdx.x == 0) cur = supp[order[r]] ? -1 : order[r];
        __syncthreads();
        const int i = cur;
        if (i >= 0) {
            if (threadIdx.x == 0) keep[i] = 1;
            const float x1 = boxes[4 * i], y1 = boxes[4 * i + 1], x2 = boxes[4 * i + 2], y2 = boxes[4 * i + 3];
            const float ai = (x2 - x1) * (y2 - y1);
            for (int k = r + 1 + threadIdx.x; k < n; k += blockDim.x) {
                const int j = order[k];
                const float* b = boxes + 4 * j;
                const float w = fmaxf(fminf(x2, b[2]) - fmaxf(x1, b[0]), 0.f);
                const float h = fmaxf(fminf(y2, b[3]) - fmaxf(y1, b[1]), 0.f);
                const float inter = w * h;
                const float iou = inter / (ai + (b[2] - b[0]) * (b[3] - b[1]) - inter);
                if (iou > thresh) supp[j] = 1;
            }
        }
        __syncthreads();
    }
}
}  // namespace
}  // namespace kinet

extern "C" int kinet_nms(const float* boxes, const float* scores, uint8_t* keep, int n, float iou_threshold,
                         kinet_stream_t stream) {
    using namespace kinet;
    KINET_CHECK_ARG(n >= 0 && n <= NMS_MAX, "nms: %d boxes (at most %d)", n, NMS_MAX);
    if (n == 0) return KINET_OK;
    hipLaunchKernelGGL(nms_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, boxes, scores, keep, n, iou_threshold);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}
