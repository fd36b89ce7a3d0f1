// Multi-scale deformable attention sampling for gfx950 (CDNA4).
//
// Replaces the reference's three CUDA kernels (ms_deform_im2col_cuda.cuh:165-378) and
// their launcher (ms_deform_attn_cuda.cu:19-168).  Design (DESIGN.md "MSDA kernels"):
//
//  * one workgroup = QT consecutive queries x all M heads of one batch image;
//  * phase 1 ("setup"): one thread per sample (q, m, l, p) reads its location and
//    attention weight with coalesced loads (or computes them from the raw projection in
//    the fused module path), and stages the 4 bilinear tap row-offsets + tap weights in
//    LDS -- the bilinear arithmetic happens once per sample, not once per channel as in
//    the reference (which recomputes it for each of the D channel threads, cuh:227-231);
//  * phase 2 ("gather"): LPQ lanes per (q, m) pair, each owning VEC contiguous channels,
//    read the staged taps (LDS broadcast) and issue 16-byte vector loads of the value
//    rows; accumulation in f32 registers; the output is written once.  No (L*P)x larger
//    `columns` buffer and no separate at::sum reduction (cu:68, :80).
//  * backward: the same setup; each lane computes the three channel-partial sums
//    (attention-weight grad, d/dx, d/dy) in one pass over the taps (the reference walks
//    the taps twice per coordinate and per channel, cuh:356-372) and scatters
//    grad_value with f32 atomics over its contiguous channels (cuh:301 scans a 5x5
//    neighbourhood per channel to find the same 4 taps).
#include <hip/hip_runtime.h>

#include <math.h>

#include <algorithm>

#include <type_traits>

#include "../../include/kinet_msda.h"
#include "common.h"
#include "msda_util.h"

namespace kinet {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxLevels = 16;


struct LevelInfo {
    int start[kMaxLevels];
    int H[kMaxLevels];
    int W[kMaxLevels];
    int ok[kMaxLevels];
};

// level_start_index from spatial_shapes (cu:52-58), computed per block in LDS; a level
// that would run past S is disabled instead of reading out of bounds.
__device__ __forceinline__ void load_levels(LevelInfo& li, const int64_t* shapes, int L, int S) {
    if (threadIdx.x == 0) {
        long long acc = 0;
        for (int l = 0; l < L; ++l) {
            const long long H = shapes[2 * l], W = shapes[2 * l + 1];
            li.start[l] = (int)acc;
            li.H[l] = (int)H;
            li.W[l] = (int)W;
            li.ok[l] = (H > 0 && W > 0 && acc + H * W <= S) ? 1 : 0;
            acc += H * W;
        }
    }
}

template <typename TL> __device__ __forceinline__ float ldf(const TL* p) { return (float)*p; }

// ---------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------
// Per-sample setup record in LDS: tap element offsets (within one batch image) and the
// four tap weights already multiplied by the attention weight (0 for taps/samples
// outside the image, with a safe offset so phase 2 needs no branch).
struct Tap4 {
    int off[4];
    float w[4];
};

template <typename T, typename TL>
__device__ __forceinline__ void setup_sample(Tap4& t, float x, float y, float a, const LevelInfo& li,
                                             int l, int MD, int m, int D) {
    const int H = li.H[l], W = li.W[l];
    const float h = y * (float)H - 0.5f;   // cuh:227
    const float w = x * (float)W - 0.5f;   // cuh:228
    const int base = m * D;
    int o0 = base, o1 = base, o2 = base, o3 = base;
    float w0 = 0.f, w1 = 0.f, w2 = 0.f, w3 = 0.f;
    if (li.ok[l] && h > -1.f && w > -1.f && h < (float)H && w < (float)W) {   // cuh:229
        const float hf = floorf(h), wf = floorf(w);
        const int hl = (int)hf, wl = (int)wf;
        const float lh = h - hf, lw = w - wf, hh = 1.f - lh, hw = 1.f - lw;
        const int rowbase = li.start[l];
        const bool h0 = hl >= 0, h1 = hl + 1 <= H - 1, c0 = wl >= 0, c1 = wl + 1 <= W - 1;
        if (h0 && c0) { o0 = (rowbase + hl * W + wl) * MD + base; w0 = hh * hw * a; }
        if (h0 && c1) { o1 = (rowbase + hl * W + wl + 1) * MD + base; w1 = hh * lw * a; }
        if (h1 && c0) { o2 = (rowbase + (hl + 1) * W + wl) * MD + base; w2 = lh * hw * a; }
        if (h1 && c1) { o3 = (rowbase + (hl + 1) * W + wl + 1) * MD + base; w3 = lh * lw * a; }
    }
    t.off[0] = o0; t.off[1] = o1; t.off[2] = o2; t.off[3] = o3;
    t.w[0] = w0; t.w[1] = w1; t.w[2] = w2; t.w[3] = w3;
}

// f64 keeps a double-precision setup so the fp64 path matches test_double_precision.py.
struct Tap4d {
    int off[4];
    double w[4];
};

template <typename T, typename TL, int VEC, int FUSED>
__global__ __launch_bounds__(kThreads) void msda_fwd_kernel(
    const T* __restrict__ value, const int64_t* __restrict__ shapes,
    const TL* __restrict__ loc, const TL* __restrict__ attw,
    const float* __restrict__ offlog, int ld_off, const float* __restrict__ ref, int ref_dim,
    const uint8_t* __restrict__ qmask, float* __restrict__ loc_out, float* __restrict__ attw_out,
    T* __restrict__ out, int S, int M, int D, int L, int Lq, int P, int QT, int LPQ, int VLD) {
    using Acc = typename Acc<T>::type;
    using TapT = typename std::conditional<sizeof(Acc) == 8, Tap4d, Tap4>::type;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LevelInfo& li = *reinterpret_cast<LevelInfo*>(smem);
    TapT* taps = reinterpret_cast<TapT*>(smem + sizeof(LevelInfo));

    const int b = blockIdx.y;
    const int q0 = blockIdx.x * QT;
    const int LP = L * P;
    const int MD = VLD;   // value row stride (elements); == M*D unless the value is a column slice
    load_levels(li, shapes, L, S);
    __syncthreads();

    // ---- phase 1: per-sample setup ----
    const int nsamp = QT * M * LP;
    if (!FUSED) {
        for (int s = threadIdx.x; s < nsamp; s += kThreads) {
            const int qi = s / (M * LP);
            const int q = q0 + qi;
            const int rem = s - qi * (M * LP);
            const int m = rem / LP;
            const int l = (rem - m * LP) / P;
            TapT t;
            if (q < Lq) {
                const long gi = ((long)b * Lq + q0) * M * LP + s;   // (q, m, l, p) contiguous
                if (sizeof(Acc) == 8) {
                    // double path: identical arithmetic in f64
                    const double x = (double)loc[2 * gi], y = (double)loc[2 * gi + 1], a = (double)attw[gi];
                    const int H = li.H[l], W = li.W[l];
                    const double h = y * H - 0.5, w = x * W - 0.5;
                    const int base = m * D;
                    for (int k = 0; k < 4; ++k) { t.off[k] = base; t.w[k] = 0; }
                    if (li.ok[l] && h > -1 && w > -1 && h < H && w < W) {
                        const double hf = floor(h), wf = floor(w);
                        const int hl = (int)hf, wl = (int)wf;
                        const double lh = h - hf, lw = w - wf, hh = 1 - lh, hw = 1 - lw;
                        const int rb = li.start[l];
                        const bool h0 = hl >= 0, h1 = hl + 1 <= H - 1, c0 = wl >= 0, c1 = wl + 1 <= W - 1;
                        if (h0 && c0) { t.off[0] = (rb + hl * W + wl) * MD + base; t.w[0] = hh * hw * a; }
                        if (h0 && c1) { t.off[1] = (rb + hl * W + wl + 1) * MD + base; t.w[1] = hh * lw * a; }
                        if (h1 && c0) { t.off[2] = (rb + (hl + 1) * W + wl) * MD + base; t.w[2] = lh * hw * a; }
                        if (h1 && c1) { t.off[3] = (rb + (hl + 1) * W + wl + 1) * MD + base; t.w[3] = lh * lw * a; }
                    }
                } else {
                    Tap4 t4;
                    setup_sample<T, TL>(t4, ldf(loc + 2 * gi), ldf(loc + 2 * gi + 1), ldf(attw + gi), li, l, MD, m, D);
                    for (int k = 0; k < 4; ++k) { t.off[k] = t4.off[k]; t.w[k] = t4.w[k]; }
                }
            } else {
                for (int k = 0; k < 4; ++k) { t.off[k] = 0; t.w[k] = 0; }
            }
            taps[s] = t;
        }
    } else if ((LP & (LP - 1)) == 0 && LP <= 64) {
        // fused module path (ms_deform_attn.py:69-82), L*P a power of two <= 64: the L*P
        // samples of one (query, head) are LP consecutive lanes, so the softmax max / sum are
        // wave shuffles (the loop bound is rounded up to whole waves for the shuffles).
        const int nsamp_r = (nsamp + 63) & ~63;
        for (int s = threadIdx.x; s < nsamp_r; s += kThreads) {
            const bool sv = s < nsamp;
            const int qi = s / (M * LP);
            const int q = q0 + qi;
            const int rem = s - qi * (M * LP);
            const int m = rem / LP;
            const int lp = rem - m * LP;
            const int l = lp / P;
            const bool ok = sv && q < Lq;
            const float* orow = offlog + ((long)b * Lq + (ok ? q : 0)) * ld_off;
            const float logit = ok ? orow[(long)M * LP * 2 + rem] : -INFINITY;
            float mx = logit;
            for (int o = LP >> 1; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
            const float e = ok ? __expf(logit - mx) : 0.f;
            float sum = e;
            for (int o = LP >> 1; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
            if (!sv) continue;
            Tap4 t4;
            if (ok) {
                float a = e / sum;
                if (qmask && qmask[(long)b * Lq + q]) a = 0.f;
                const float2 o2 = *reinterpret_cast<const float2*>(orow + (long)rem * 2);
                const float* rp = ref + (((long)b * Lq + q) * L + l) * ref_dim;
                float x, y;
                if (ref_dim == 2) {
                    // quirk kept for parity: offsets / spatial_shapes[(H, W)] applied to (x, y)
                    x = rp[0] + o2.x / (float)li.H[l];
                    y = rp[1] + o2.y / (float)li.W[l];
                } else {
                    x = rp[0] + o2.x / (float)P * rp[2] * 0.5f;
                    y = rp[1] + o2.y / (float)P * rp[3] * 0.5f;
                }
                if (loc_out) {
                    const long gi = ((long)b * Lq + q) * M * LP + rem;
                    loc_out[2 * gi] = x;
                    loc_out[2 * gi + 1] = y;
                    attw_out[gi] = a;
                }
                setup_sample<T, float>(t4, x, y, a, li, l, MD, m, D);
            } else {
                for (int k = 0; k < 4; ++k) { t4.off[k] = 0; t4.w[k] = 0.f; }
            }
            TapT t;
            for (int k = 0; k < 4; ++k) { t.off[k] = t4.off[k]; t.w[k] = t4.w[k]; }
            taps[s] = t;
        }
    } else {
        // fused path, general L*P: logits go through LDS for the softmax.
        float* lg = reinterpret_cast<float*>(taps + nsamp);   // nsamp floats after the taps
        for (int s = threadIdx.x; s < nsamp; s += kThreads) {
            const int qi = s / (M * LP);
            const int q = q0 + qi;
            const int rem = s - qi * (M * LP);
            float v = -INFINITY;
            if (q < Lq) v = to_f32(offlog[((long)b * Lq + q) * ld_off + (long)M * LP * 2 + rem]);
            lg[s] = v;
        }
        __syncthreads();
        for (int s = threadIdx.x; s < nsamp; s += kThreads) {
            const int qi = s / (M * LP);
            const int q = q0 + qi;
            const int rem = s - qi * (M * LP);
            const int m = rem / LP;
            const int lp = rem - m * LP;
            const int l = lp / P;
            Tap4 t4;
            if (q < Lq) {
                const float* grp = lg + (s - lp);
                float mx = -INFINITY;
                for (int j = 0; j < LP; ++j) mx = fmaxf(mx, grp[j]);
                float sum = 0.f;
                for (int j = 0; j < LP; ++j) sum += __expf(grp[j] - mx);
                float a = __expf(grp[lp] - mx) / sum;
                if (qmask && qmask[(long)b * Lq + q]) a = 0.f;
                const float* orow = offlog + ((long)b * Lq + q) * ld_off + (long)rem * 2;
                const float ox = to_f32(orow[0]), oy = to_f32(orow[1]);
                const float* rp = ref + (((long)b * Lq + q) * L + l) * ref_dim;
                float x, y;
                if (ref_dim == 2) {
                    // quirk kept for parity: offsets / spatial_shapes[(H, W)] applied to (x, y)
                    x = rp[0] + ox / (float)li.H[l];
                    y = rp[1] + oy / (float)li.W[l];
                } else {
                    x = rp[0] + ox / (float)P * rp[2] * 0.5f;
                    y = rp[1] + oy / (float)P * rp[3] * 0.5f;
                }
                if (loc_out) {
                    const long gi = ((long)b * Lq + q) * M * LP + rem;
                    loc_out[2 * gi] = x;
                    loc_out[2 * gi + 1] = y;
                    attw_out[gi] = a;
                }
                setup_sample<T, float>(t4, x, y, a, li, l, MD, m, D);
            } else {
                for (int k = 0; k < 4; ++k) { t4.off[k] = 0; t4.w[k] = 0.f; }
            }
            TapT t;   // lg lives after the taps array: no overlap, no barrier needed
            for (int k = 0; k < 4; ++k) { t.off[k] = t4.off[k]; t.w[k] = t4.w[k]; }
            taps[s] = t;
        }
    }
    __syncthreads();

    // ---- phase 2: gather ----
    const int g = threadIdx.x / LPQ;
    const int lane = threadIdx.x - g * LPQ;
    const int qi = g / M;
    const int q = q0 + qi;
    if (qi >= QT || q >= Lq) return;
    const int m = g - qi * M;
    const int c0 = lane * VEC;
    const T* vb = value + (long)b * S * MD + c0;
    const TapT* tp = taps + (qi * M + m) * LP;
    Acc acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0;
    // Gather in groups of SG samples: all 4*SG tap loads of a group are issued before any
    // is consumed, so 16 independent 16-byte gathers per lane are in flight (left to
    // itself hipcc interleaves 2-4 loads with vmcnt(0) waits: latency-bound).
    constexpr int SG = 4;
    int s = 0;
    for (; s + SG <= LP; s += SG) {
        TapT t[SG];
#pragma unroll
        for (int g2 = 0; g2 < SG; ++g2) t[g2] = tp[s + g2];
        VecT<T, VEC> v[SG][4];
#pragma unroll
        for (int g2 = 0; g2 < SG; ++g2)
#pragma unroll
            for (int k = 0; k < 4; ++k) v[g2][k] = *reinterpret_cast<const VecT<T, VEC>*>(vb + t[g2].off[k]);
#pragma unroll
        for (int g2 = 0; g2 < SG; ++g2)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int j = 0; j < VEC; ++j) acc[j] += (Acc)t[g2].w[k] * to_acc(v[g2][k].v[j], (Acc*)nullptr);
    }
    for (; s < LP; ++s) {
        const TapT t = tp[s];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const VecT<T, VEC> v = *reinterpret_cast<const VecT<T, VEC>*>(vb + t.off[k]);
#pragma unroll
            for (int j = 0; j < VEC; ++j) acc[j] += (Acc)t.w[k] * to_acc(v.v[j], (Acc*)nullptr);
        }
    }
    VecT<T, VEC> o;
#pragma unroll
    for (int j = 0; j < VEC; ++j) o.v[j] = Cvt<T>::from(acc[j]);
    *reinterpret_cast<VecT<T, VEC>*>(out + ((long)b * Lq + q) * M * D + (long)m * D + c0) = o;
}

// ---------------------------------------------------------------------------------
// fused module forward, head-per-wave decomposition
// ---------------------------------------------------------------------------------
// Workgroup = QT consecutive queries x MH heads (one head per wave, QT = 64 / LPQ queries
// per wave).  With the head-major value layout (heads, B, S, D) the 16 queries of a wave
// sample neighbouring pixels of ONE head map, so a wave's tap loads hit a few contiguous
// cache lines (with the row-major (B, S, M, D) layout a 128-B line holds one pixel of two
// heads and a wave's loads scatter over 16 unrelated pieces).  Value element (b, s, m, c)
// is value[b*vsb + s*vss + m*vsm + c]; both layouts are strides of this form.
template <typename T, int VEC>
__global__ __launch_bounds__(kThreads) void msda_fused_kernel(
    const T* __restrict__ value, long vsb, int vss, long vsm, const int64_t* __restrict__ shapes,
    const float* __restrict__ offlog, int ld_off, const float* __restrict__ ref, int ref_dim,
    const uint8_t* __restrict__ qmask, float* __restrict__ loc_out, float* __restrict__ attw_out,
    T* __restrict__ out, int S, int M, int D, int L, int Lq, int P, int QT, int LPQ, int MH) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LevelInfo& li = *reinterpret_cast<LevelInfo*>(smem);
    Tap4* taps = reinterpret_cast<Tap4*>(smem + sizeof(LevelInfo));
    const int b = blockIdx.y;
    const int q0 = blockIdx.x * QT;
    const int mh0 = blockIdx.z * MH;
    const int LP = L * P;
    const int nsamp = MH * QT * LP;
    load_levels(li, shapes, L, S);
    __syncthreads();

    const bool pow2 = (LP & (LP - 1)) == 0 && LP <= 64;
    float* lg = reinterpret_cast<float*>(taps + nsamp);   // logits staging (general L*P only)
    if (!pow2) {
        for (int s = threadIdx.x; s < nsamp; s += kThreads) {
            const int ml = s / (QT * LP), qi = (s / LP) % QT, lp = s % LP;
            const int m = mh0 + ml, q = q0 + qi;
            lg[s] = (q < Lq && m < M) ? offlog[((long)b * Lq + q) * ld_off + (long)M * LP * 2 + m * LP + lp] : -INFINITY;
        }
        __syncthreads();
    }
    const int nsamp_r = (nsamp + 63) & ~63;
    for (int s = threadIdx.x; s < nsamp_r; s += kThreads) {
        const bool sv = s < nsamp;
        const int ml = s / (QT * LP), qi = (s / LP) % QT, lp = s % LP;
        const int m = mh0 + ml, q = q0 + qi;
        const int l = lp / P;
        const bool ok = sv && q < Lq && m < M;
        const float* orow = offlog + ((long)b * Lq + (ok ? q : 0)) * ld_off;
        float a;
        if (pow2) {   // the LP samples of one (query, head) are LP consecutive lanes
            const float logit = ok ? orow[(long)M * LP * 2 + m * LP + lp] : -INFINITY;
            float mx = logit;
            for (int o = LP >> 1; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
            const float e = ok ? __expf(logit - mx) : 0.f;
            float sum = e;
            for (int o = LP >> 1; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
            a = ok ? e / sum : 0.f;
        } else if (ok) {
            const float* grp = lg + (s - lp);
            float mx = -INFINITY, sum = 0.f;
            for (int j = 0; j < LP; ++j) mx = fmaxf(mx, grp[j]);
            for (int j = 0; j < LP; ++j) sum += __expf(grp[j] - mx);
            a = __expf(grp[lp] - mx) / sum;
        } else {
            a = 0.f;
        }
        if (!sv) continue;
        Tap4 t4;
        if (ok) {
            if (qmask && qmask[(long)b * Lq + q]) a = 0.f;                  // ms_deform_attn.py:73-74
            const float2 o2 = *reinterpret_cast<const float2*>(orow + (long)(m * LP + lp) * 2);
            const float* rp = ref + (((long)b * Lq + q) * L + l) * ref_dim;
            float x, y;
            if (ref_dim == 2) {
                // quirk kept for parity: offsets / spatial_shapes[(H, W)] applied to (x, y) (:77-79)
                x = rp[0] + o2.x / (float)li.H[l];
                y = rp[1] + o2.y / (float)li.W[l];
            } else {                                                       // :80-82
                x = rp[0] + o2.x / (float)P * rp[2] * 0.5f;
                y = rp[1] + o2.y / (float)P * rp[3] * 0.5f;
            }
            if (loc_out) {
                const long gi = (((long)b * Lq + q) * M + m) * LP + lp;
                loc_out[2 * gi] = x;
                loc_out[2 * gi + 1] = y;
                attw_out[gi] = a;
            }
            setup_sample<T, float>(t4, x, y, a, li, l, vss, 0, D);          // offsets within one head map
        } else {
            for (int k = 0; k < 4; ++k) { t4.off[k] = 0; t4.w[k] = 0.f; }
        }
        taps[s] = t4;
    }
    __syncthreads();

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int qi = lane / LPQ;
    const int m = mh0 + wave;
    const int q = q0 + qi;
    if (wave >= MH || m >= M || qi >= QT || q >= Lq) return;
    const int c0 = (lane - qi * LPQ) * VEC;
    const T* vb = value + (long)b * vsb + (long)m * vsm + c0;
    const Tap4* tp = taps + (wave * QT + qi) * LP;
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
    constexpr int SG = 4;   // 4 samples x 4 taps = 16 gathers in flight per lane
    int s = 0;
    for (; s + SG <= LP; s += SG) {
        Tap4 t[SG];
#pragma unroll
        for (int g2 = 0; g2 < SG; ++g2) t[g2] = tp[s + g2];
        VecT<T, VEC> v[SG][4];
#pragma unroll
        for (int g2 = 0; g2 < SG; ++g2)
#pragma unroll
            for (int k = 0; k < 4; ++k) v[g2][k] = *reinterpret_cast<const VecT<T, VEC>*>(vb + t[g2].off[k]);
#pragma unroll
        for (int g2 = 0; g2 < SG; ++g2)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int j = 0; j < VEC; ++j) acc[j] += t[g2].w[k] * to_f32(v[g2][k].v[j]);
    }
    for (; s < LP; ++s) {
        const Tap4 t = tp[s];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const VecT<T, VEC> v = *reinterpret_cast<const VecT<T, VEC>*>(vb + t.off[k]);
#pragma unroll
            for (int j = 0; j < VEC; ++j) acc[j] += t.w[k] * to_f32(v.v[j]);
        }
    }
    VecT<T, VEC> o;
#pragma unroll
    for (int j = 0; j < VEC; ++j) o.v[j] = Cvt<T>::from(acc[j]);
    *reinterpret_cast<VecT<T, VEC>*>(out + ((long)b * Lq + q) * M * D + (long)m * D + c0) = o;
}

// ---------------------------------------------------------------------------------
// fused module forward, specialised: 16-bit values, head_dim 32, L and P compile-time
// ---------------------------------------------------------------------------------
// Same decomposition and results contract as msda_fused_kernel (one head per wave, 16
// queries x 4 lanes x 8 channels), rebuilt around what bounds it on gfx950 -- VALU issue,
// not memory (rocprofv3: ~2.3k VALU wave-instructions per wave for ~80 loads):
//  * the sample index split (head, query, level, point) is shifts on compile-time sizes,
//    not runtime integer division;
//  * the per-level normalisers are reciprocals staged in LDS (one multiply instead of an
//    IEEE divide), the softmax divides through one reciprocal;
//  * taps are byte offsets for raw buffer loads off a per-wave head-map descriptor: an
//    out-of-image corner gets an offset past num_records and the hardware returns 0, so
//    there is neither a per-corner branch nor 64-bit address arithmetic;
//  * the 4-corner x 8-channel accumulation runs as v_pk_fma_f32 on bf16 pairs widened by
//    one shift / one mask.
struct FastLevels {
    int start[kMaxLevels], H[kMaxLevels], W[kMaxLevels], ok[kMaxLevels];
    float Hf[kMaxLevels], Wf[kMaxLevels], rH[kMaxLevels], rW[kMaxLevels];
};

// acc += f16(lo or hi half of x) * w in f32 -- one v_fma_mix_f32, no separate widening
__device__ __forceinline__ float fma_mix_lo(float acc, uint32_t x, float w) {
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(x), "v"(w));
    return acc;
}
__device__ __forceinline__ float fma_mix_hi(float acc, uint32_t x, float w) {
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(x), "v"(w));
    return acc;
}

template <typename T>
__device__ __forceinline__ void widen2(uint32_t u, f32x2& x) {
    if constexpr (std::is_same<T, f16_t>::value) {
        x = f32x2{(float)__builtin_bit_cast(f16_t, (uint16_t)(u & 0xffffu)), (float)__builtin_bit_cast(f16_t, (uint16_t)(u >> 16))};
    } else {
        x = f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
    }
}

// MH heads (waves) per workgroup, SG samples gathered per group (SG x 4 loads in flight per lane)
template <typename T, typename TO, typename TL, int L, int P, int MH = kThreads / 64, int SG = 4>
__global__ __launch_bounds__(MH * 64) void msda_fused_fast_kernel(
    const T* __restrict__ value, long vsb, int vss, long vsm, int head_bytes, const int64_t* __restrict__ shapes,
    const TL* __restrict__ offlog, int ld_off, const float* __restrict__ ref, int ref_dim,
    const uint8_t* __restrict__ qmask, float* __restrict__ loc_out, float* __restrict__ attw_out,
    TO* __restrict__ out, int S, int M, int Lq, const int* __restrict__ torder) {
    static_assert(sizeof(T) == 2 && sizeof(TO) == 2, "16-bit values and output");
    constexpr int D = 32, QT = 16, LP = L * P, NT = MH * 64;
    static_assert((LP & (LP - 1)) == 0 && LP <= 64 && L <= kMaxLevels, "L*P: power of two <= 64");
    constexpr int NSB = MH * QT * LP;               // samples per workgroup
    constexpr unsigned OOB = 0x80000000u;
    __shared__ FastLevels lv;
    // per-sample tap records, split so phase 2 reads the offsets before its gathers and the
    // weights only after them: 4 byte offsets (16 B) + 4 weights as f16 (8 B; v_fma_mix takes
    // them as a 16-bit source directly) -- 24 KiB per workgroup instead of 32, so the LDS no
    // longer caps residency below the register limit
    __shared__ int4 toff[NSB];
    __shared__ uint2 twt[NSB];
    // XCD-aware remap (bijective, cdna_hip_programming.md T1): workgroups are dealt to the 8
    // XCDs round-robin by linear id; give each XCD a contiguous run of query tiles of one
    // (frame, head group) so neighbouring queries -- which sample overlapping value
    // neighbourhoods -- share that XCD's L2
    int b, q0, mh0;
    {
        const int gx = gridDim.x, gy = gridDim.y;
        const int nblk = gx * gy * gridDim.z;
        const int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
        const int qd = nblk >> 3, rm = nblk & 7, xcd = lin & 7;
        const int nid = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + (lin >> 3);
        const int bxl = nid % gx, rest = nid / gx;
        // optional processing order of the query tiles (results unchanged): the encoder
        // interleaves the tiles of all levels by image row so one L2 pass serves them all
        const int bx = torder ? torder[bxl] : bxl;
        b = rest % gy;
        q0 = bx * QT;
        mh0 = (rest / gy) * MH;
    }
    if (threadIdx.x == 0) {
        long long acc = 0;
        for (int l = 0; l < L; ++l) {
            const long long H = shapes[2 * l], W = shapes[2 * l + 1];
            lv.start[l] = (int)acc;
            lv.H[l] = (int)H;
            lv.W[l] = (int)W;
            lv.ok[l] = (H > 0 && W > 0 && acc + H * W <= S) ? 1 : 0;
            lv.Hf[l] = (float)H;
            lv.Wf[l] = (float)W;
            lv.rH[l] = H > 0 ? 1.f / (float)H : 0.f;
            lv.rW[l] = W > 0 ? 1.f / (float)W : 0.f;
            acc += H * W;
        }
    }
    __syncthreads();

    const int rowb = vss * (int)sizeof(T);           // bytes between pixels of one head map
#pragma unroll
    for (int i = 0; i < NSB / NT; ++i) {
        const int s = threadIdx.x + NT * i;
        const int ml = s / (QT * LP), qi = (s / LP) % QT, lp = s % LP, l = lp / P;
        const int m = mh0 + ml, q = q0 + qi;
        const bool ok = q < Lq && m < M;
        const TL* orow = offlog + ((long)b * Lq + (ok ? q : 0)) * ld_off;
        // softmax over the LP consecutive lanes of one (query, head) (ms_deform_attn.py:71-72)
        const float logit = ok ? to_f32(orow[M * LP * 2 + (ok ? m : 0) * LP + lp]) : -INFINITY;
        const float mx = group_reduce<LP, true>(logit);
        const float e = ok ? __expf(logit - mx) : 0.f;
        const float sum = group_reduce<LP, false>(e);
        float a = ok ? e * __builtin_amdgcn_rcpf(sum) : 0.f;
        Tap4 t4;
#pragma unroll
        for (int k = 0; k < 4; ++k) { t4.off[k] = (int)OOB; t4.w[k] = 0.f; }
        if (ok) {
            if (qmask && qmask[(long)b * Lq + q]) a = 0.f;                  // ms_deform_attn.py:73-74
            float2 o2;
            if constexpr (std::is_same<TL, float>::value) {
                o2 = *reinterpret_cast<const float2*>(orow + (m * LP + lp) * 2);
            } else {
                const uint32_t u = *reinterpret_cast<const uint32_t*>(orow + (m * LP + lp) * 2);
                o2.x = (float)__builtin_bit_cast(f16_t, (uint16_t)(u & 0xffffu));
                o2.y = (float)__builtin_bit_cast(f16_t, (uint16_t)(u >> 16));
            }
            const float* rp = ref + (((long)b * Lq + q) * L + l) * ref_dim;
            float x, y;
            if (ref_dim == 2) {   // offsets / spatial_shapes[(H, W)] on (x, y): the reference's quirk (:77-79)
                x = rp[0] + o2.x * lv.rH[l];
                y = rp[1] + o2.y * lv.rW[l];
            } else {              // :80-82
                x = rp[0] + o2.x * (0.5f / (float)P) * rp[2];
                y = rp[1] + o2.y * (0.5f / (float)P) * rp[3];
            }
            if (loc_out) {
                const long gi = (((long)b * Lq + q) * M + m) * LP + lp;
                loc_out[2 * gi] = x;
                loc_out[2 * gi + 1] = y;
                attw_out[gi] = a;
            }
            const int H = lv.H[l], W = lv.W[l];
            const float h = y * lv.Hf[l] - 0.5f, w = x * lv.Wf[l] - 0.5f;   // cuh:227-228
            if (lv.ok[l] && h > -1.f && w > -1.f && h < lv.Hf[l] && w < lv.Wf[l]) {   // cuh:229
                const float hf = floorf(h), wf = floorf(w);
                const int hl = (int)hf, wl = (int)wf;
                const float lh = h - hf, lw = w - wf, hh = 1.f - lh, hw = 1.f - lw;
                const bool h0 = hl >= 0, h1 = hl + 1 < H, c0 = wl >= 0, c1 = wl + 1 < W;
                const int o00 = (lv.start[l] + hl * W + wl) * rowb;
                t4.off[0] = (h0 && c0) ? o00 : (int)OOB;
                t4.off[1] = (h0 && c1) ? o00 + rowb : (int)OOB;
                t4.off[2] = (h1 && c0) ? o00 + W * rowb : (int)OOB;
                t4.off[3] = (h1 && c1) ? o00 + W * rowb + rowb : (int)OOB;
                t4.w[0] = hh * hw * a;
                t4.w[1] = hh * lw * a;
                t4.w[2] = lh * hw * a;
                t4.w[3] = lh * lw * a;
            }
        }
        toff[s] = make_int4(t4.off[0], t4.off[1], t4.off[2], t4.off[3]);
        twt[s] = make_uint2(pack_f16x2(t4.w[0], t4.w[1]), pack_f16x2(t4.w[2], t4.w[3]));
    }
    __syncthreads();

    // wave index made provably uniform: the head-map descriptor below must live in SGPRs,
    // or hipcc wraps every buffer load in a readfirstlane waterfall loop
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int m = mh0 + wave;
    if (m >= M) return;
    const int qi = lane >> 2, q = q0 + qi;
    const unsigned cb = (unsigned)(lane & 3) * 16u;   // this lane's 8 channels, bytes
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(value + (long)b * vsb + (long)m * vsm), (short)0, head_bytes, 0x00020000);
    const int4* tpo = toff + (wave * QT + qi) * LP;
    const uint2* tpw = twt + (wave * QT + qi) * LP;
    f32x2 acc[4] = {};
#pragma unroll 1
    for (int s = 0; s < LP; s += SG) {
        u32x4v v[SG][4];
#pragma unroll
        for (int g = 0; g < SG; ++g) {
            const int4 o = tpo[s + g];
            v[g][0] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, (unsigned)o.x + cb, 0, 0));
            v[g][1] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, (unsigned)o.y + cb, 0, 0));
            v[g][2] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, (unsigned)o.z + cb, 0, 0));
            v[g][3] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, (unsigned)o.w + cb, 0, 0));
        }
        uint2 wq[SG];
#pragma unroll
        for (int g = 0; g < SG; ++g) wq[g] = tpw[s + g];
#pragma unroll
        for (int g = 0; g < SG; ++g)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t wp = k < 2 ? wq[g].x : wq[g].y;   // f16 weights of corners (k & ~1, k | 1)
                if constexpr (std::is_same<T, f16_t>::value) {
                    // f16 values x f16 weights, f32 accumulate: one v_fma_mix_f32 per MAC
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        acc[j][0] = (k & 1) ? fma_mix16_lo_hi(acc[j][0], v[g][k][j], wp) : fma_mix16_lo_lo(acc[j][0], v[g][k][j], wp);
                        acc[j][1] = (k & 1) ? fma_mix16_hi_hi(acc[j][1], v[g][k][j], wp) : fma_mix16_hi_lo(acc[j][1], v[g][k][j], wp);
                    }
                } else {
                    // bf16 values: widen by shift / mask, then v_pk_fma_f32 (1.5 VALU per MAC)
                    const float wk = (float)__builtin_bit_cast(f16_t, (uint16_t)((k & 1) ? (wp >> 16) : (wp & 0xffffu)));
                    const f32x2 w2 = {wk, wk};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        f32x2 x;
                        widen2<T>(v[g][k][j], x);
                        acc[j] = __builtin_elementwise_fma(x, w2, acc[j]);
                    }
                }
            }
    }
    if (q >= Lq) return;
    VecT<TO, 8> o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        o.v[2 * j] = Cvt<TO>::from(acc[j][0]);
        o.v[2 * j + 1] = Cvt<TO>::from(acc[j][1]);
    }
    *reinterpret_cast<VecT<TO, 8>*>(out + ((long)b * Lq + q) * M * D + (long)m * D + (lane & 3) * 8) = o;
}

// ---------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------
template <typename A>
struct BwdTap {
    int off[4];   // -1: tap outside the image (value taken as 0, no scatter)
    A lh, lw, a;
    int valid;    // sample inside (-1,H) x (-1,W)
    A H, W;
};

template <typename T, typename TL, typename GA, int VEC, int POW2, int ALN>
__global__ __launch_bounds__(kThreads) void msda_bwd_kernel(
    const T* __restrict__ value, const int64_t* __restrict__ shapes,
    const TL* __restrict__ loc, const TL* __restrict__ attw, const T* __restrict__ gout,
    GA* __restrict__ gvalue, TL* __restrict__ gloc, TL* __restrict__ gattw,
    int S, int M, int D, int L, int Lq, int P, int QT, int LPQ, int NA) {
    // LPQ lanes per (query, head) group, the first NA = D / VEC of them holding channels (NA <
    // LPQ pads a group to a power of two so the per-sample sums reduce by shuffles)
    using Acc = typename Acc<T>::type;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LevelInfo& li = *reinterpret_cast<LevelInfo*>(smem);
    BwdTap<Acc>* taps = reinterpret_cast<BwdTap<Acc>*>(smem + sizeof(LevelInfo));
    const int b = blockIdx.y;
    const int q0 = blockIdx.x * QT;
    const int LP = L * P;
    const int MD = M * D;
    const int nsamp = QT * M * LP;
    Acc* red = reinterpret_cast<Acc*>(taps + nsamp);   // [nsamp][3] when !POW2
    load_levels(li, shapes, L, S);
    __syncthreads();

    for (int s = threadIdx.x; s < nsamp; s += kThreads) {
        const int qi = s / (M * LP);
        const int q = q0 + qi;
        const int rem = s - qi * (M * LP);
        const int m = rem / LP;
        const int l = (rem - m * LP) / P;
        BwdTap<Acc> t;
        for (int k = 0; k < 4; ++k) t.off[k] = -1;
        t.lh = t.lw = t.a = 0;
        t.valid = 0;
        t.H = (Acc)li.H[l];
        t.W = (Acc)li.W[l];
        if (q < Lq) {
            const long gi = ((long)b * Lq + q0) * M * LP + s;
            const Acc x = (Acc)loc[2 * gi], y = (Acc)loc[2 * gi + 1];
            t.a = (Acc)attw[gi];
            const int H = li.H[l], W = li.W[l];
            const Acc h = y * (Acc)H - (Acc)0.5, w = x * (Acc)W - (Acc)0.5;   // cuh:352-353
            if (li.ok[l] && h > -1 && w > -1 && h < (Acc)H && w < (Acc)W) {  // cuh:359
                const Acc hf = floor(h), wf = floor(w);
                const int hl = (int)hf, wl = (int)wf;
                t.lh = h - hf;
                t.lw = w - wf;
                t.valid = 1;
                const int rb = li.start[l];
                const int base = m * D;
                const bool h0 = hl >= 0, h1 = hl + 1 <= H - 1, c0 = wl >= 0, c1 = wl + 1 <= W - 1;
                if (h0 && c0) t.off[0] = (rb + hl * W + wl) * MD + base;
                if (h0 && c1) t.off[1] = (rb + hl * W + wl + 1) * MD + base;
                if (h1 && c0) t.off[2] = (rb + (hl + 1) * W + wl) * MD + base;
                if (h1 && c1) t.off[3] = (rb + (hl + 1) * W + wl + 1) * MD + base;
            }
        }
        taps[s] = t;
        if (!POW2) { red[3 * s] = 0; red[3 * s + 1] = 0; red[3 * s + 2] = 0; }
    }
    __syncthreads();

    const int g = threadIdx.x / LPQ;
    const int lane = threadIdx.x - g * LPQ;
    const int qi = g / M;
    const int q = q0 + qi;
    const bool active = qi < QT && q < Lq;
    if (active) {
        const int m = g - qi * M;
        const bool cl = lane < NA;                     // a channel-holding lane
        const int c0 = (cl ? lane : 0) * VEC;
        const T* vb = value + (long)b * S * MD + c0;
        const VecT<T, VEC> gv = *reinterpret_cast<const VecT<T, VEC>*>(gout + ((long)b * Lq + q) * MD + (long)m * D + c0);
        Acc gc[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) gc[j] = cl ? to_acc(gv.v[j], (Acc*)nullptr) : (Acc)0;
        // grad_value scatter channel maps. Float atomics leave the chip as one 64-byte request
        // per line a wave-instruction touches, so the map decides the request count:
        //  - lane-STRIDED (channel j*NA + lane): each wave-instruction adds NA contiguous dwords
        //    per (query, head) group instead of dwords VEC apart;
        //  - ALN (16-lane groups, head rows at a fixed dword offset sh in their 64-byte line, i.e.
        //    M*D % 16 == 0): instruction j adds the j-th line the head row touches, channel
        //    16*j + lane - sh, so every request carries a whole line of the row (D=36: 3.25
        //    requests per corner instead of 6)
        const int sh = ALN ? ((m * D) & 15) : 0;
        GA* gvs = gvalue + (long)b * S * MD + (ALN ? lane - sh : (cl ? lane : 0));
        Acc gs[VEC];
        bool gok[VEC];
        {
            const T* go = gout + ((long)b * Lq + q) * MD + (long)m * D;
#pragma unroll
            for (int j = 0; j < VEC; ++j) {
                const int ch = ALN ? 16 * j + lane - sh : (cl ? lane : 0) + j * NA;
                gok[j] = ALN ? (ch >= 0 && ch < D) : cl;
                gs[j] = gok[j] ? to_acc(go[ch], (Acc*)nullptr) : (Acc)0;
            }
        }
        const int sbase = (qi * M + m) * LP;
        for (int s = 0; s < LP; ++s) {
            const BwdTap<Acc> t = taps[sbase + s];
            Acc pa = 0, px = 0, py = 0;
            if (t.valid) {
                const Acc lh = t.lh, lw = t.lw, hh = 1 - lh, hw = 1 - lw;
                Acc v[4][VEC];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (cl && t.off[k] >= 0) {
                        const VecT<T, VEC> vv = *reinterpret_cast<const VecT<T, VEC>*>(vb + t.off[k]);
#pragma unroll
                        for (int j = 0; j < VEC; ++j) v[k][j] = to_acc(vv.v[j], (Acc*)nullptr);
                    } else {
#pragma unroll
                        for (int j = 0; j < VEC; ++j) v[k][j] = 0;
                    }
                }
                const Acc wt[4] = {hh * hw, hh * lw, lh * hw, lh * lw};
#pragma unroll
                for (int j = 0; j < VEC; ++j) {
                    const Acc val = wt[0] * v[0][j] + wt[1] * v[1][j] + wt[2] * v[2][j] + wt[3] * v[3][j];
                    const Acc dw = hh * (v[1][j] - v[0][j]) + lh * (v[3][j] - v[2][j]);   // cuh:150-160
                    const Acc dh = hw * (v[2][j] - v[0][j]) + lw * (v[3][j] - v[1][j]);   // cuh:139-149
                    pa += gc[j] * val;
                    px += gc[j] * dw;
                    py += gc[j] * dh;
                }
                // grad_value scatter (cuh:285-304): 4 taps x VEC channels (lane-strided, see gs)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (t.off[k] >= 0) {
                        const Acc wk = wt[k] * t.a;
#pragma unroll
                        for (int j = 0; j < VEC; ++j)
                            if (gok[j]) atomicAdd(gvs + t.off[k] + j * (ALN ? 16 : NA), (GA)(gs[j] * wk));
                    }
                }
            }
            if (POW2) {
                for (int o = LPQ >> 1; o > 0; o >>= 1) {
                    pa += __shfl_xor(pa, o);
                    px += __shfl_xor(px, o);
                    py += __shfl_xor(py, o);
                }
                if (lane == 0) {
                    const long gi = ((long)b * Lq + q) * M * LP + (long)(sbase - qi * M * LP) + s;
                    gattw[gi] = (TL)pa;
                    gloc[2 * gi] = (TL)(px * t.a * t.W);        // cuh:373
                    gloc[2 * gi + 1] = (TL)(py * t.a * t.H);    // cuh:374
                }
            } else {
                atomicAdd(red + 3 * (sbase + s), pa);
                atomicAdd(red + 3 * (sbase + s) + 1, px * t.a * t.W);
                atomicAdd(red + 3 * (sbase + s) + 2, py * t.a * t.H);
            }
        }
    }
    if (!POW2) {
        __syncthreads();
        for (int s = threadIdx.x; s < nsamp; s += kThreads) {
            const int qq = q0 + s / (M * LP);
            if (qq < Lq) {
                const long gi = ((long)b * Lq + q0) * M * LP + s;
                gattw[gi] = (TL)red[3 * s];
                gloc[2 * gi] = (TL)red[3 * s + 1];
                gloc[2 * gi + 1] = (TL)red[3 * s + 2];
            }
        }
    }
}

// ---------------------------------------------------------------------------------
// backward, grad_value summed on chip (encoder calls of the training path)
// ---------------------------------------------------------------------------------
// Global f32 atomics run at the memory side at one chip-wide byte rate (~1.3 TB/s,
// MI355X_MICROARCH.md "Global float atomics"), so the scatter above is bound by its
// 4 corners x D x 4 bytes per sample.  In an encoder call the queries are the pixels
// themselves in raster order and neighbouring queries sample overlapping value rows.  Here
// one workgroup owns ONE (image, head) and a chunk of consecutive queries, walked in passes
// of QP queries; per pass:
//  1. one thread per sample: bilinear setup; each in-image corner looks its pixel up in an
//     LDS hash (pixel -> slot) and pushes its contribution (corner weight x attention
//     weight, query row) onto the slot's LDS linked list; the pass's grad_output rows are
//     staged in LDS;
//  2. 16 lanes per query: value corners -> grad wrt location / attention weight (as above);
//     corners whose hash probe failed are added to global memory directly;
//  3. lane = (slot, channel): walk the slot's list summing weight x grad_output in a
//     register, then ONE global atomic per row element -- a row touched by c corners of the
//     pass costs one add instead of c.  Exclusive ownership: no LDS float atomics (measured
//     at ~86 cycles per wave-instruction, slower than the global atomics they would save).
// Any sampling pattern is correct; only the saving depends on locality.
//
// LDS: LevelInfo | keys[NS] | head[NS] | plist[NS] | npass | cinfo[QP*L*P*4] (weight,
//      grad_output row) | next[QP*L*P*4] | G[QP][D] f32 | taps[QP*L*P]
// Where the time goes at the config-4 encoder call (tools/msda_bwd_probe.py --phases, r04q):
// 1.12 ms in all; without phase 3 (row sums + atomics) 0.56, without its atomics 0.97, without
// phase 2's value loads 0.95, and 0.43 ms with neither loads, hash inserts nor phase 3 -- the
// per-workgroup setup (serial level info, hash clear) and phase 2's 12 shuffle reductions per
// sample.  Packing each entry with its link (one LDS round trip per list step instead of two)
// measured no change (1.12 ms).
constexpr int kProbe = 8;

struct HTap {
    int off[4];    // element offset of each corner's head row in the image, -1 = outside
    float lh, lw, a;
    int flags;     // bit 0: sample inside the image; bit 1+k: corner k added directly
};

// slot of `key` in the open-addressed table, inserting it (and appending the slot to plist)
// when new; -1 after kProbe occupied probes
__device__ __forceinline__ int hash_slot(int* keys, int* plist, int* npass, int key, int log2ns) {
    const unsigned mask = (1u << log2ns) - 1u;
    unsigned h = ((unsigned)key * 2654435761u) >> (32 - log2ns);
    for (int i = 0; i < kProbe; ++i, h = (h + 1u) & mask) {
        const int cur = __hip_atomic_load(keys + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == key) return (int)h;
        if (cur != -1) continue;
        const int old = atomicCAS(keys + h, -1, key);
        if (old == -1) {
            plist[atomicAdd(npass, 1)] = (int)h;
            return (int)h;
        }
        if (old == key) return (int)h;
    }
    return -1;
}

template <typename T, typename TL, int VEC, int NJ, int SP = 2>
__global__ __launch_bounds__(512) void msda_bwd_list_kernel(
    const T* __restrict__ value, const int64_t* __restrict__ shapes, const TL* __restrict__ loc,
    const TL* __restrict__ attw, const T* __restrict__ gout, float* __restrict__ gvalue,
    TL* __restrict__ gloc, TL* __restrict__ gattw, int S, int M, int D, int L, int Lq, int P, int QC,
    int QP, int NA, int log2ns, int blocked, int dbg) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int blk[kMaxLevels + 1];
    const int NS = 1 << log2ns;
    const int nt = blockDim.x, LP = L * P, MD = M * D, BH = QP / 8;
    const int NSMP = QP * LP;
    LevelInfo& li = *reinterpret_cast<LevelInfo*>(smem);
    int* keys = reinterpret_cast<int*>(smem + sizeof(LevelInfo));
    int* head = keys + NS;
    int* plist = head + NS;
    int* npass = plist + NS;   // [0] slots used by the pass
    int2* cinfo = reinterpret_cast<int2*>(npass + 4);
    int* next = reinterpret_cast<int*>(cinfo + 4 * NSMP);
    float* G = reinterpret_cast<float*>(next + 4 * NSMP);
    HTap* taps = reinterpret_cast<HTap*>(G + QP * D);
    const int b = blockIdx.y, m = blockIdx.z;
    load_levels(li, shapes, L, S);
    for (int i = threadIdx.x; i < NS; i += nt) { keys[i] = -1; head[i] = -1; }
    if (threadIdx.x == 0) {
        *npass = 0;
        // blocked (encoder calls, queries = pixels in raster order): chunk = one 8 x BH block
        // of one level's pixels, blocks numbered level by level
        int acc = 0;
        for (int l = 0; l < L; ++l) {
            blk[l] = acc;
            if (li.ok[l]) acc += ((li.H[l] + BH - 1) / BH) * ((li.W[l] + 7) / 8);
        }
        blk[L] = acc;
    }
    __syncthreads();

    const int lane = threadIdx.x & 15;
    const T* vimg = value + (long)b * S * MD;
    float* gimg = gvalue + (long)b * S * MD + m * D;
    const int nchunk = blocked ? blk[L] : (Lq + QC - 1) / QC;
    for (int chunk = blockIdx.x; chunk < nchunk; chunk += gridDim.x) {
    int qbeg = 0, qend = QP, bl = 0, by = 0, bx = 0;
    if (blocked) {
        while (bl + 1 < L && chunk >= blk[bl + 1]) ++bl;
        const int r = chunk - blk[bl], nbx = (li.W[bl] + 7) / 8;
        by = r / nbx;
        bx = r - by * nbx;
    } else {
        qbeg = chunk * QC;
        qend = min(Lq, qbeg + QC);
    }
    // query of pass slot qi, -1 = none
    auto qof = [&](int qp, int qi) -> int {
        if (blocked) {
            const int y = by * BH + (qi >> 3), x = bx * 8 + (qi & 7);
            return (y < li.H[bl] && x < li.W[bl]) ? li.start[bl] + y * li.W[bl] + x : -1;
        }
        const int q = qp + qi;
        return q < qend ? q : -1;
    };
    for (int qp = qbeg; qp < qend; qp += QP) {
        // phase 1: grad_output rows of the pass; one thread per sample
        for (int i = threadIdx.x; i < QP * D; i += nt) {
            const int qi = i / D, q = qof(qp, qi);
            G[i] = q >= 0 ? to_acc(gout[((long)b * Lq + q) * MD + (long)m * D + (i - qi * D)], (float*)nullptr) : 0.f;
        }
        for (int s = threadIdx.x; s < NSMP; s += nt) {
            const int qi = s / LP, lp = s - qi * LP, l = lp / P, q = qof(qp, qi);
            HTap t;
#pragma unroll
            for (int k = 0; k < 4; ++k) t.off[k] = -1;
            t.lh = t.lw = t.a = 0.f;
            t.flags = 0;
            if (q >= 0) {
                const long gi = ((long)b * Lq + q) * M * LP + (long)m * LP + lp;
                const float x = (float)loc[2 * gi], y = (float)loc[2 * gi + 1];
                t.a = (float)attw[gi];
                const int H = li.H[l], W = li.W[l];
                const float h = y * (float)H - 0.5f, w = x * (float)W - 0.5f;   // cuh:352-353
                if (li.ok[l] && h > -1.f && w > -1.f && h < (float)H && w < (float)W) {   // cuh:359
                    const float hf = floorf(h), wf = floorf(w);
                    const int hl = (int)hf, wl = (int)wf;
                    t.lh = h - hf;
                    t.lw = w - wf;
                    t.flags = 1;
                    const float hh = 1.f - t.lh, hw = 1.f - t.lw;
                    const int p00 = li.start[l] + hl * W + wl;
                    const bool h0 = hl >= 0, h1 = hl + 1 <= H - 1, c0 = wl >= 0, c1 = wl + 1 <= W - 1;
                    const int pix[4] = {p00, p00 + 1, p00 + W, p00 + W + 1};
                    const bool in[4] = {h0 && c0, h0 && c1, h1 && c0, h1 && c1};
                    const float wt[4] = {hh * hw, hh * t.lw, t.lh * hw, t.lh * t.lw};
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (in[k]) {
                            t.off[k] = pix[k] * MD;
                            if (dbg & 8) continue;
                            const int slot = hash_slot(keys, plist, npass, pix[k], log2ns);
                            if (slot < 0) {
                                t.flags |= 2 << k;
                            } else {
                                const int cid = 4 * s + k;
                                cinfo[cid] = make_int2(__float_as_int(wt[k] * t.a), qi * D);
                                next[cid] = atomicExch(head + slot, cid);
                            }
                        }
                }
            }
            taps[s] = t;
        }
        __syncthreads();
        // phase 2: 16 lanes per query -- value corners for the location / weight gradients
        // (lanes < NA hold VEC contiguous channels); overflowed corners added directly
        for (int qi = threadIdx.x >> 4; qi < QP; qi += nt >> 4) {
            const int q = qof(qp, qi);
            if (q < 0) continue;
            const bool cl = lane < NA;
            const int c0 = (cl ? lane : 0) * VEC;
            float gc[VEC];
#pragma unroll
            for (int j = 0; j < VEC; ++j) gc[j] = cl ? G[qi * D + c0 + j] : 0.f;
            const HTap* tq = taps + qi * LP;
            // two samples per step: their 8 corner loads are in flight together
            auto load = [&](const HTap& t, float (&v)[4][VEC]) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (cl && (t.flags & 1) && t.off[k] >= 0 && !(dbg & 1)) {
                        const VecT<T, VEC> vv = *reinterpret_cast<const VecT<T, VEC>*>(vimg + t.off[k] + m * D + c0);
#pragma unroll
                        for (int j = 0; j < VEC; ++j) v[k][j] = to_acc(vv.v[j], (float*)nullptr);
                    } else {
#pragma unroll
                        for (int j = 0; j < VEC; ++j) v[k][j] = 0.f;
                    }
                }
            };
            auto consume = [&](const HTap& t, const float (&v)[4][VEC], int s) {
                float pa = 0.f, px = 0.f, py = 0.f;
                const float lh = t.lh, lw = t.lw, hh = 1.f - lh, hw = 1.f - lw;
                const float wt[4] = {hh * hw, hh * lw, lh * hw, lh * lw};
#pragma unroll
                for (int j = 0; j < VEC; ++j) {
                    const float val = wt[0] * v[0][j] + wt[1] * v[1][j] + wt[2] * v[2][j] + wt[3] * v[3][j];
                    const float dw = hh * (v[1][j] - v[0][j]) + lh * (v[3][j] - v[2][j]);   // cuh:150-160
                    const float dh = hw * (v[2][j] - v[0][j]) + lw * (v[3][j] - v[1][j]);   // cuh:139-149
                    pa += gc[j] * val;
                    px += gc[j] * dw;
                    py += gc[j] * dh;
                }
                if (t.flags & 30) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (!(t.flags & (2 << k))) continue;
                        const float wk = wt[k] * t.a;
#pragma unroll
                        for (int j = 0; j < NJ; ++j) {
                            const int ch = lane + 16 * j;
                            if (ch < D) atomicAdd(gimg + t.off[k] + ch, G[qi * D + ch] * wk);
                        }
                    }
                }
#pragma unroll
                for (int o = 8; o > 0; o >>= 1) {
                    pa += __shfl_xor(pa, o, 16);
                    px += __shfl_xor(px, o, 16);
                    py += __shfl_xor(py, o, 16);
                }
                if (lane == 0) {   // samples outside the image: all three sums are 0
                    const long gi = ((long)b * Lq + q) * M * LP + (long)m * LP + s;
                    const int l = s / P;
                    gattw[gi] = (TL)pa;
                    gloc[2 * gi] = (TL)(px * t.a * (float)li.W[l]);        // cuh:373
                    gloc[2 * gi + 1] = (TL)(py * t.a * (float)li.H[l]);    // cuh:374
                }
            };
            int s = 0;
            if constexpr (SP == 4) {   // four samples' 16 corner loads in flight together
                for (; s + 3 < LP; s += 4) {
                    const HTap t0 = tq[s], t1 = tq[s + 1], t2 = tq[s + 2], t3 = tq[s + 3];
                    float v0[4][VEC], v1[4][VEC], v2[4][VEC], v3[4][VEC];
                    load(t0, v0);
                    load(t1, v1);
                    load(t2, v2);
                    load(t3, v3);
                    consume(t0, v0, s);
                    consume(t1, v1, s + 1);
                    consume(t2, v2, s + 2);
                    consume(t3, v3, s + 3);
                }
            }
            for (; s + 1 < LP; s += 2) {
                const HTap t0 = tq[s], t1 = tq[s + 1];
                float v0[4][VEC], v1[4][VEC];
                load(t0, v0);
                load(t1, v1);
                consume(t0, v0, s);
                consume(t1, v1, s + 1);
            }
            if (s < LP) {
                const HTap t0 = tq[s];
                float v0[4][VEC];
                load(t0, v0);
                consume(t0, v0, s);
            }
        }

        // phase 3 (reads only what phase 1 wrote, so no barrier before it): lane = (slot,
        // channel), consecutive lanes on consecutive channels of the pass's rows
        const int n = (dbg & 4) ? 0 : *npass;
        {
            // thread = (slot group, channel), fixed for the pass: one division per thread instead of
            // one per (slot, channel) item (D is a run-time value): 1.05-1.10 -> 1.03 ms at the
            // config-4 encoder call (tools/msda_bwd_probe.py --ab, profiles/r06t_bwd_phase3.txt)
            // (D <= 64 <= nt on this path: launch_bwd takes it for nj <= 4 and 64-thread multiples)
            const int c = threadIdx.x % D, sg = threadIdx.x / D, nsg = nt / D;
            for (int si = sg; sg < nsg && si < n; si += nsg) {
                const int slot = plist[si];
                float acc = 0.f;
                for (int cid = head[slot]; cid >= 0; cid = next[cid]) {
                    const int2 ci = cinfo[cid];
                    acc += __int_as_float(ci.x) * G[ci.y + c];
                }
                if (!(dbg & 2)) atomicAdd(gimg + (long)keys[slot] * MD + c, acc);
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += nt) {
            const int slot = plist[i];
            keys[slot] = -1;
            head[slot] = -1;
        }
        if (threadIdx.x == 0) *npass = 0;
        __syncthreads();
    }
    }
}

template <typename T>
__global__ void f32_to_kernel(const float* __restrict__ src, T* __restrict__ dst, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        dst[i] = Cvt<T>::from(src[i]);
}

// ---------------------------------------------------------------------------------
// launch configuration
// ---------------------------------------------------------------------------------
struct Cfg {
    int vec, lpq, qt;
};

Cfg pick_cfg(int D, int M, size_t esize) {
    Cfg c{1, D, 1};
    const int maxvec = (int)(16 / esize);
    for (int v = maxvec; v >= 1; v >>= 1) {
        if (D % v == 0) { c.vec = v; break; }
    }
    c.lpq = D / c.vec;
    const int groups = kThreads / c.lpq;
    c.qt = groups / M;
    return c;
}

int common_checks(int N, int S, int M, int D, int L, int Lq, int P, int im2col_step) {
    KINET_CHECK_ARG(N >= 0 && S >= 0 && M > 0 && D > 0 && L > 0 && Lq >= 0 && P > 0,
                    "msda: invalid sizes N=%d S=%d M=%d D=%d L=%d Lq=%d P=%d", N, S, M, D, L, Lq, P);
    KINET_CHECK_ARG(L <= kMaxLevels, "msda: num_levels %d > %d", L, kMaxLevels);
    KINET_CHECK_ARG((long long)S * M * D < (1LL << 31), "msda: S*M*D too large for one image");
    if (N > 0) {
        const int step = im2col_step < N ? im2col_step : N;   // cu:46
        KINET_CHECK_ARG(step > 0 && N % step == 0, "batch(%d) must divide im2col_step(%d)", N, step);   // cu:48
    }
    return KINET_OK;
}

template <typename T, typename TL, int FUSED>
int launch_fwd(const void* value, const int64_t* shapes, const void* loc, const void* attw,
               const void* offlog, int ld_off, const float* ref, int ref_dim, const uint8_t* qmask,
               float* loc_out, float* attw_out, void* out, int N, int S, int M, int D, int L, int Lq,
               int P, hipStream_t stream, int vld = 0) {
    const Cfg c = pick_cfg(D, M, sizeof(T));
    KINET_CHECK_ARG(c.qt >= 1, "msda: heads*channels/vec (%d*%d) exceeds one workgroup", M, c.lpq);
    if (vld == 0) vld = M * D;
    KINET_CHECK_ARG(vld >= M * D && vld % c.vec == 0, "msda: value row stride %d invalid", vld);
    KINET_CHECK_ARG((long long)S * vld < (1LL << 31), "msda: S*value_ld too large for one image");
    if (N == 0 || Lq == 0) return KINET_OK;
    using Acc = typename Acc<T>::type;
    const size_t tap = sizeof(Acc) == 8 ? sizeof(Tap4d) : sizeof(Tap4);
    const size_t nsamp = (size_t)c.qt * M * L * P;
    size_t lds = sizeof(LevelInfo) + nsamp * tap + (FUSED ? nsamp * sizeof(float) : 0);
    KINET_CHECK_ARG(lds <= 160 * 1024, "msda: LDS request %zu too large", lds);
    dim3 grid((Lq + c.qt - 1) / c.qt, N);
#define KF(VEC)                                                                                             \
    hipLaunchKernelGGL((msda_fwd_kernel<T, TL, VEC, FUSED>), grid, dim3(kThreads), lds, stream,             \
                       (const T*)value, shapes, (const TL*)loc, (const TL*)attw, (const float*)offlog, ld_off,  \
                       ref, ref_dim, qmask, loc_out, attw_out, (T*)out, S, M, D, L, Lq, P, c.qt, c.lpq, vld)
    switch (c.vec) {
        case 1: KF(1); break;
        case 2: KF(2); break;
        case 4: if (16 / sizeof(T) >= 4) { KF(4); } break;
        case 8: if (16 / sizeof(T) >= 8) { KF(8); } break;
    }
#undef KF
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

// backward kernel choice for the calling thread (kinet_msda_backward_tune; 0 = automatic):
// mode -1 = the direct-atomic kernel, 1 = the list kernel for any call; log2ns = hash rows,
// qc = queries per workgroup, threads = workgroup size, flush_at = queries per pass
struct BwdTune {
    int mode, log2ns, qc, threads, flush_at;
};
thread_local BwdTune bwd_tune = {0, 0, 0, 0, 0};
// timing-only phase knobs of msda_bwd_list_kernel (kinet_msda_backward_debug; results wrong
// when set): 1 = phase 2 without its value loads, 2 = phase 3 without its global atomics,
// 4 = no phase 3, 8 = no hash inserts (and so no phase-3 work)
thread_local int bwd_dbg = 0;
// the kernel the calling thread's last kinet_msda_backward launched (kinet_msda_backward_last_kernel):
// 1 = msda_bwd_list_kernel (rows summed on chip), 0 = msda_bwd_kernel (per-corner atomics), -1 = none
thread_local int bwd_last = -1;

template <typename T, typename TL>
int launch_bwd(const void* value, const int64_t* shapes, const void* loc, const void* attw,
               const void* gout, void* gvalue, void* gloc, void* gattw, void* workspace, int N, int S,
               int M, int D, int L, int Lq, int P, hipStream_t stream) {
    using Acc = typename Acc<T>::type;
    using GA = typename std::conditional<sizeof(Acc) == 8, double, float>::type;
    const Cfg c = pick_cfg(D, M, sizeof(T));
    KINET_CHECK_ARG(c.qt >= 1, "msda: heads*channels/vec (%d*%d) exceeds one workgroup", M, c.lpq);
    const size_t nval = (size_t)N * S * M * D;
    GA* acc_buf;
    const bool direct = std::is_same<T, float>::value || std::is_same<T, double>::value;
    if (direct) {
        acc_buf = (GA*)gvalue;
    } else {
        KINET_CHECK_ARG(workspace != nullptr || nval == 0, "msda backward: bf16/f16 value needs an f32 workspace");
        acc_buf = (GA*)workspace;
    }
    if (nval) KINET_CHECK_HIP(hipMemsetAsync(acc_buf, 0, nval * sizeof(GA), stream));
    const int LP = L * P;
    const int nj = (D + 15) / 16;
    const BwdTune tn = bwd_tune;
    bool hashed = false;
    if constexpr (sizeof(GA) == 4) {
    // encoder calls (queries = the value pixels, Lq == S): rows summed on chip per pass
    // (msda_bwd_list_kernel); mode 1 forces it, mode -1 forbids it
    if (N > 0 && Lq > 0 && tn.mode >= 0 && (Lq == S || tn.mode == 1) && c.lpq <= 16 && nj <= 4) {
        hashed = true;
        // 256 threads, passes of 16 queries (8 x 2 pixel blocks), 1024-row hash: 35 KB of LDS,
        // 4 workgroups per CU -- 1.03 ms at the config-4 encoder call; 512 threads x 32 queries
        // 1.05, 512 x 16 1.40 (tools/msda_bwd_probe.py --sweep, profiles/r03p_msda_bwd_probe.log)
        const int threads = tn.threads ? tn.threads : 256;
        const int QP = tn.flush_at > 0 ? tn.flush_at : threads / 16;   // queries per pass
        const int log2ns = tn.log2ns ? tn.log2ns : 10;
        const size_t nsmp = (size_t)QP * LP;
        const size_t lds = sizeof(LevelInfo) + ((size_t)3 << log2ns) * sizeof(int) + 4 * sizeof(int) +
                           nsmp * 4 * (sizeof(int2) + sizeof(int)) + (size_t)QP * D * sizeof(float) + nsmp * sizeof(HTap);
        KINET_CHECK_ARG(threads % 64 == 0 && threads <= 512 && QP >= 1 && lds <= 160 * 1024,
                        "msda backward: pass of %d queries x %d samples does not fit LDS", QP, LP);
        // query chunk per workgroup: as long as the grid still fills the chip 4 times over
        int qc = tn.qc;
        if (qc <= 0) {
            qc = QP;   // one pass per workgroup: 1.08 ms at the config-4 encoder call (2 passes 1.11, 4 1.18)
            while (qc > QP && (long)N * M * ((Lq + qc - 1) / qc) < 4L * cu_count()) qc >>= 1;
        }
        qc = std::max(QP, qc / QP * QP);
        // encoder calls: queries in 8 x QP/8 pixel blocks (fewer distinct rows per pass than a
        // run of QP pixels); the grid over-covers the block count (edge blocks) and each
        // workgroup loops over chunks, so any level geometry is covered
        const int blocked = (Lq == S && QP % 8 == 0 && tn.mode != 2) ? 1 : 0;
        const int nq = blocked ? (S + QP - 1) / QP : (Lq + qc - 1) / qc;
        dim3 grid(blocked ? nq + nq / 8 + 2 * L : nq, N, M);
#define KH(VEC, NJ)                                                                                             \
    if (tn.mode == 3)                                                                                           \
        hipLaunchKernelGGL((msda_bwd_list_kernel<T, TL, VEC, NJ, 4>), grid, dim3(threads), lds, stream,         \
                           (const T*)value, shapes, (const TL*)loc, (const TL*)attw, (const T*)gout,            \
                           (float*)acc_buf, (TL*)gloc, (TL*)gattw, S, M, D, L, Lq, P, qc, QP, c.lpq, log2ns,    \
                           blocked, bwd_dbg);                                                                   \
    else                                                                                                        \
    hipLaunchKernelGGL((msda_bwd_list_kernel<T, TL, VEC, NJ>), grid, dim3(threads), lds, stream, (const T*)value, \
                       shapes, (const TL*)loc, (const TL*)attw, (const T*)gout, (float*)acc_buf, (TL*)gloc,     \
                       (TL*)gattw, S, M, D, L, Lq, P, qc, QP, c.lpq, log2ns, blocked, bwd_dbg)
#define KHJ(VEC) switch (nj) { case 1: KH(VEC, 1); break; case 2: KH(VEC, 2); break; case 3: KH(VEC, 3); break; default: KH(VEC, 4); }
        switch (c.vec) {
            case 1: KHJ(1); break;
            case 2: KHJ(2); break;
            case 4: if constexpr (16 / sizeof(T) >= 4) { KHJ(4); } break;
            case 8: if constexpr (16 / sizeof(T) >= 8) { KHJ(8); } break;
        }
#undef KHJ
#undef KH
        KINET_LAUNCH_CHECK();
    }
    }
    bwd_last = hashed ? 1 : (N > 0 && Lq > 0 ? 0 : -1);
    if (hashed) {
    } else if (N > 0 && Lq > 0) {
        // groups padded to a power of two (reductions by shuffles instead of LDS atomics)
        int lpq = c.lpq, qt = c.qt;
        if ((lpq & (lpq - 1)) != 0) {
            int p2 = 1;
            while (p2 < lpq) p2 <<= 1;
            if (p2 <= 64 && (kThreads / p2) / M >= 1) {
                lpq = p2;
                qt = (kThreads / p2) / M;
            }
        }
        const bool pow2 = (lpq & (lpq - 1)) == 0 && lpq <= 64;
        const bool aln = sizeof(GA) == 4 && lpq == 16 && c.vec == 4 && (M * D) % 16 == 0 && D <= 48;
        const size_t nsamp = (size_t)qt * M * L * P;
        const size_t lds = sizeof(LevelInfo) + nsamp * sizeof(BwdTap<Acc>) + (pow2 ? 0 : nsamp * 3 * sizeof(Acc));
        KINET_CHECK_ARG(lds <= 160 * 1024, "msda backward: LDS request %zu too large", lds);
        dim3 grid((Lq + qt - 1) / qt, N);
#define KB(VEC, P2, AL)                                                                                      \
    hipLaunchKernelGGL((msda_bwd_kernel<T, TL, GA, VEC, P2, AL>), grid, dim3(kThreads), lds, stream,            \
                       (const T*)value, shapes, (const TL*)loc, (const TL*)attw, (const T*)gout, acc_buf,   \
                       (TL*)gloc, (TL*)gattw, S, M, D, L, Lq, P, qt, lpq, c.lpq)
#define KBV(VEC) if (pow2) { KB(VEC, 1, 0); } else { KB(VEC, 0, 0); }
        switch (c.vec) {
            case 1: KBV(1); break;
            case 2: KBV(2); break;
            case 4:
                if (16 / sizeof(T) >= 4) {
                    if (aln) { KB(4, 1, 1); } else { KBV(4); }
                }
                break;
            case 8: if (16 / sizeof(T) >= 8) { KBV(8); } break;
        }
#undef KBV
#undef KB
        KINET_LAUNCH_CHECK();
    } else if (N * Lq * M * L * P > 0) {
        KINET_CHECK_HIP(hipMemsetAsync(gloc, 0, (size_t)N * Lq * M * L * P * 2 * sizeof(TL), stream));
        KINET_CHECK_HIP(hipMemsetAsync(gattw, 0, (size_t)N * Lq * M * L * P * sizeof(TL), stream));
    }
    if (!direct && nval) {
        const long n = (long)nval;
        int blocks = (int)((n + 255) / 256);
        if (blocks > kMaxGridStride) blocks = kMaxGridStride;
        hipLaunchKernelGGL((f32_to_kernel<T>), dim3(blocks), dim3(256), 0, stream, (const float*)acc_buf, (T*)gvalue, n);
        KINET_LAUNCH_CHECK();
    }
    return KINET_OK;
}

}  // namespace
}  // namespace kinet

using namespace kinet;

extern "C" int kinet_msda_forward(const void* value, const int64_t* spatial_shapes, const void* sampling_loc,
                                  const void* attn_weight, void* output, int batch, int spatial_size,
                                  int num_heads, int channels, int num_levels, int num_query, int num_point,
                                  int im2col_step, int value_dtype, int loc_dtype, kinet_stream_t stream) {
    int rc = common_checks(batch, spatial_size, num_heads, channels, num_levels, num_query, num_point, im2col_step);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
#define ARGS value, spatial_shapes, sampling_loc, attn_weight, nullptr, 0, nullptr, 0, nullptr, nullptr, nullptr, \
             output, batch, spatial_size, num_heads, channels, num_levels, num_query, num_point, s
    if (value_dtype == KINET_F32 && loc_dtype == KINET_F32) return launch_fwd<float, float, 0>(ARGS);
    if (value_dtype == KINET_F64 && loc_dtype == KINET_F64) return launch_fwd<double, double, 0>(ARGS);
    if (value_dtype == KINET_BF16 && loc_dtype == KINET_F32) return launch_fwd<bf16_t, float, 0>(ARGS);
    if (value_dtype == KINET_F16 && loc_dtype == KINET_F32) return launch_fwd<f16_t, float, 0>(ARGS);
#undef ARGS
    set_error("msda forward: unsupported dtype pair value=%d loc=%d", value_dtype, loc_dtype);
    return KINET_ERR_ARG;
}

namespace kinet {
namespace {
template <typename T, typename TO = T, typename TL = float>
int launch_fused(const void* value, long vsb, int vss, long vsm, const int64_t* shapes, const void* offlog_v,
                 int ld_off, const float* ref, int ref_dim, const uint8_t* qmask, void* out, float* loc_out,
                 float* attw_out, int N, int S, int M, int D, int L, int Lq, int P, const int* torder,
                 hipStream_t stream) {
    const Cfg c = pick_cfg(D, M, sizeof(T));
    KINET_CHECK_ARG(c.lpq <= 64, "msda fused: head_dim/vec (%d) exceeds a wave", c.lpq);
    if (N == 0 || Lq == 0) return KINET_OK;
    if constexpr (sizeof(T) == 2) {
        // specialised kernel: head_dim 32, (L, P) in {(4, 4), (8, 4)}, 16-byte aligned vectors
        const long long head_bytes = ((long long)(S - 1) * vss + D) * (long long)sizeof(T);
        if (D == 32 && P == 4 && (L == 4 || L == 8) && vss % 8 == 0 && vsb % 8 == 0 && vsm % 8 == 0 &&
            ((uintptr_t)value % 16) == 0 && head_bytes < (1LL << 31)) {
            dim3 grid((Lq + 15) / 16, N, (M + 3) / 4);
            if (L == 4) {
                // 2 heads (waves) per workgroup, 2 samples per gather group: 12.5 KiB LDS and
                // 52 VGPRs, 12 workgroups per CU (encoder call 271 -> 258 us vs 4 heads x 4)
                dim3 g2((Lq + 15) / 16, N, (M + 1) / 2);
                hipLaunchKernelGGL((msda_fused_fast_kernel<T, TO, TL, 4, 4, 2, 2>), g2, dim3(128), 0, stream,
                                   (const T*)value, vsb, vss, vsm, (int)head_bytes, shapes, (const TL*)offlog_v,
                                   ld_off, ref, ref_dim, qmask, loc_out, attw_out, (TO*)out, S, M, Lq, torder);
            } else
                hipLaunchKernelGGL((msda_fused_fast_kernel<T, TO, TL, 8, 4>), grid, dim3(kThreads), 0, stream,
                                   (const T*)value, vsb, vss, vsm, (int)head_bytes, shapes, (const TL*)offlog_v, ld_off,
                                   ref, ref_dim, qmask, loc_out,
                                   attw_out, (TO*)out, S, M, Lq, torder);
            KINET_LAUNCH_CHECK();
            return KINET_OK;
        }
    }
    KINET_CHECK_ARG((std::is_same<T, TO>::value && std::is_same<TL, float>::value),
                    "msda fused: output dtype != value dtype or f16 offsets/logits need head_dim 32, "
                    "L*P in {16, 32}, P = 4 and aligned strides");
    const float* offlog = (const float*)offlog_v;
    KINET_CHECK_ARG(vsb % c.vec == 0 && vss % c.vec == 0 && vsm % c.vec == 0 && ((uintptr_t)value % 16) == 0,
                    "msda fused: value strides must keep %d-element vectors aligned", c.vec);
    const int QT = 64 / c.lpq;          // queries per wave (= per workgroup)
    const int MH = kThreads / 64;       // one head per wave
    const int LP = L * P;
    const size_t nsamp = (size_t)MH * QT * LP;
    const bool pow2 = (LP & (LP - 1)) == 0 && LP <= 64;
    const size_t lds = sizeof(LevelInfo) + nsamp * sizeof(Tap4) + (pow2 ? 0 : nsamp * sizeof(float));
    KINET_CHECK_ARG(lds <= 160 * 1024, "msda fused: LDS request %zu too large", lds);
    dim3 grid((Lq + QT - 1) / QT, N, (M + MH - 1) / MH);
    if constexpr (!std::is_same<T, TO>::value || !std::is_same<TL, float>::value) return KINET_ERR_ARG;   // (rejected above)
#define KF(VEC)                                                                                                  \
    hipLaunchKernelGGL((msda_fused_kernel<T, VEC>), grid, dim3(kThreads), lds, stream, (const T*)value, vsb, vss, \
                       vsm, shapes, offlog, ld_off, ref, ref_dim, qmask, loc_out, attw_out, (T*)out, S, M, D, L,   \
                       Lq, P, QT, c.lpq, MH)
    switch (c.vec) {
        case 1: KF(1); break;
        case 2: KF(2); break;
        case 4: if (16 / sizeof(T) >= 4) { KF(4); } break;
        case 8: if (16 / sizeof(T) >= 8) { KF(8); } break;
    }
#undef KF
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}
}  // namespace
}  // namespace kinet

extern "C" int kinet_msda_fused_forward(const void* value, int64_t value_sb, int64_t value_ss, int64_t value_sm,
                                        const int64_t* spatial_shapes, const void* offsets_logits, int ld_off,
                                        const float* ref_points, int ref_dim, const uint8_t* query_attn_mask,
                                        void* output, float* loc_out, float* attw_out, int batch, int spatial_size,
                                        int num_heads, int channels, int num_levels, int num_query, int num_point,
                                        int value_dtype, int output_dtype, int offlog_dtype,
                                        const int32_t* query_tile_order, kinet_stream_t stream) {
    int rc = common_checks(batch, spatial_size, num_heads, channels, num_levels, num_query, num_point, 1);
    if (rc) return rc;
    KINET_CHECK_ARG(ref_dim == 2 || ref_dim == 4, "Last dim of reference_points must be 2 or 4, but get %d instead.", ref_dim);
    KINET_CHECK_ARG(ld_off >= num_heads * num_levels * num_point * 3, "msda fused: ld_off %d too small", ld_off);
    KINET_CHECK_ARG((loc_out == nullptr) == (attw_out == nullptr), "msda fused: loc_out/attw_out must both be set or both NULL");
    if (value_sb == 0 && value_ss == 0 && value_sm == 0) {   // row-major (N, S, M, D)
        value_ss = (int64_t)num_heads * channels;
        value_sm = channels;
        value_sb = value_ss * spatial_size;
    }
    KINET_CHECK_ARG(value_ss >= channels && value_sm >= 0 && value_sb >= 0, "msda fused: invalid value strides");
    KINET_CHECK_ARG((long long)spatial_size * value_ss < (1LL << 31), "msda fused: S*value_ss too large");
    const size_t es = dtype_size(value_dtype);
    const int vec_el = (int)(16 / (es ? es : 1));
    (void)vec_el;
    hipStream_t s = (hipStream_t)stream;
#define ARGS value, (long)value_sb, (int)value_ss, (long)value_sm, spatial_shapes, offsets_logits, ld_off, \
             ref_points, ref_dim, query_attn_mask, output, loc_out, attw_out, batch, spatial_size, num_heads, channels, \
             num_levels, num_query, num_point, (const int*)query_tile_order, s
    KINET_CHECK_ARG(output_dtype == value_dtype || (value_dtype == KINET_F16 && output_dtype == KINET_BF16),
                    "msda fused forward: output dtype %d unsupported for value dtype %d", output_dtype, value_dtype);
    KINET_CHECK_ARG(offlog_dtype == KINET_F32 || offlog_dtype == KINET_F16,
                    "msda fused forward: offsets/logits must be f32 or f16 (got %d)", offlog_dtype);
    if (offlog_dtype == KINET_F16) {
        if (value_dtype == KINET_F16 && output_dtype == KINET_BF16) return launch_fused<f16_t, bf16_t, f16_t>(ARGS);
        if (value_dtype == KINET_F16 && output_dtype == KINET_F16) return launch_fused<f16_t, f16_t, f16_t>(ARGS);
        if (value_dtype == KINET_BF16 && output_dtype == KINET_BF16) return launch_fused<bf16_t, bf16_t, f16_t>(ARGS);
        set_error("msda fused forward: f16 offsets/logits need 16-bit values");
        return KINET_ERR_ARG;
    }
    if (value_dtype == KINET_F16 && output_dtype == KINET_BF16) return launch_fused<f16_t, bf16_t>(ARGS);
    if (value_dtype == KINET_F32) return launch_fused<float>(ARGS);
    if (value_dtype == KINET_BF16) return launch_fused<bf16_t>(ARGS);
    if (value_dtype == KINET_F16) return launch_fused<f16_t>(ARGS);
#undef ARGS
    set_error("msda fused forward: unsupported value dtype %d", value_dtype);
    return KINET_ERR_ARG;
}

extern "C" int kinet_msda_backward(const void* value, const int64_t* spatial_shapes, const void* sampling_loc,
                                   const void* attn_weight, const void* grad_output, void* grad_value,
                                   void* grad_loc, void* grad_attw, void* workspace, int batch, int spatial_size,
                                   int num_heads, int channels, int num_levels, int num_query, int num_point,
                                   int im2col_step, int value_dtype, int loc_dtype, kinet_stream_t stream) {
    int rc = common_checks(batch, spatial_size, num_heads, channels, num_levels, num_query, num_point, im2col_step);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
#define ARGS value, spatial_shapes, sampling_loc, attn_weight, grad_output, grad_value, grad_loc, grad_attw, workspace, \
             batch, spatial_size, num_heads, channels, num_levels, num_query, num_point, s
    if (value_dtype == KINET_F32 && loc_dtype == KINET_F32) return launch_bwd<float, float>(ARGS);
    if (value_dtype == KINET_F64 && loc_dtype == KINET_F64) return launch_bwd<double, double>(ARGS);
    if (value_dtype == KINET_BF16 && loc_dtype == KINET_F32) return launch_bwd<bf16_t, float>(ARGS);
    if (value_dtype == KINET_F16 && loc_dtype == KINET_F32) return launch_bwd<f16_t, float>(ARGS);
#undef ARGS
    set_error("msda backward: unsupported dtype pair value=%d loc=%d", value_dtype, loc_dtype);
    return KINET_ERR_ARG;
}

extern "C" int kinet_msda_backward_last_kernel(void) { return bwd_last; }

extern "C" int kinet_msda_backward_debug(int flags) {
    const int old = bwd_dbg;
    bwd_dbg = flags;
    return old;
}

extern "C" void kinet_msda_backward_tune(int mode, int log2_rows, int queries_per_block, int threads, int flush_at) {
    bwd_tune = BwdTune{mode, log2_rows, queries_per_block, threads, flush_at};
}

extern "C" int64_t kinet_msda_backward_workspace_bytes(int batch, int spatial_size, int num_heads, int channels,
                                                       int value_dtype) {
    if (value_dtype == KINET_F32 || value_dtype == KINET_F64) return 0;
    return (int64_t)batch * spatial_size * num_heads * channels * 4;
}
