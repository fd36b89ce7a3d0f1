// Backward-pass kernels of the training path (gfx950 / CDNA4): what the reference's
// losses.backward() (engine.py:145-149) runs through cuBLAS / cuDNN / ATen for the dense
// layers of the detector, rebuilt as kinet_amd kernels (include/kinet_grad.h):
//
//  * kinet_gemm_tn     C (f32) [+]= A^T B for row-major A (K x M), B (K x N): the weight
//                      gradients (dW = dY^T X of a Linear, dW = dZ^T im2col(X) of a conv) --
//                      a reduction over the long row dimension, so split-K with a fixed-order
//                      finalize (no float atomics); f32 operands on v_mfma_f32_16x16x4_f32 (the
//                      exact-f32 MFMA: bit-for-bit an fma chain), 16-bit operands widened to f32;
//  * kinet_transpose   (rows x cols) -> (cols x rows), LDS-tiled;
//  * kinet_im2col_nhwc / kinet_col2im_nhwc: the patch matrix of an NHWC convolution and its
//                      adjoint as a deterministic gather (every input pixel sums its <= KH*KW
//                      taps in a fixed order);
//  * kinet_colsum      bias gradients (column sums), fixed-order two-pass;
//  * kinet_layernorm_backward / kinet_groupnorm_backward (nn.LayerNorm / nn.GroupNorm);
//  * kinet_mha_backward: scaled-dot-product attention backward (nn.MultiheadAttention core,
//                      deformable_transformer.py:371), probabilities recomputed from Q, K.
#include <hip/hip_runtime.h>

#include <math.h>

#include <algorithm>

#include "../../include/kinet_grad.h"
#include "common.h"
#include "gemm_common.h"   // split_x3 / Mma<f32x3_t> (KINET_F32_X3)

namespace kinet {
namespace {

template <typename T> __device__ __forceinline__ float ld(const T* p) { return to_f32(*p); }
template <typename T> __device__ __forceinline__ void st(T* p, float v) { *p = Cvt<T>::from(v); }

// ------------------------------------------------------------------------------ transpose
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ src, T* __restrict__ dst, int rows,
                                                        int cols, long lds, long ldd) {
    __shared__ T tile[32][33];
    const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
    for (int i = 0; i < 32; i += 8) {
        const int r = r0 + ty + i, c = c0 + tx;
        if (r < rows && c < cols) tile[ty + i][tx] = src[(long)r * lds + c];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 32; i += 8) {
        const int c = c0 + ty + i, r = r0 + tx;
        if (r < rows && c < cols) dst[(long)c * ldd + r] = tile[tx][ty + i];
    }
}

// ----------------------------------------------------------------------- im2col / col2im
struct ConvGeom {
    int B, H, W, C, Ho, Wo, KH, KW, sh, sw, ph, pw;
};

// cols[p][(kh*KW + kw)*C + c] = x[n, ho*sh - ph + kh, wo*sw - pw + kw, c] (0 outside), 4 channels per thread
template <typename T>
__global__ __launch_bounds__(256) void im2col_kernel(const T* __restrict__ x, T* __restrict__ cols, ConvGeom g) {
    const int C4 = g.C >> 2, taps = g.KH * g.KW;
    const long total = (long)g.B * g.Ho * g.Wo * taps * C4;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c4 = (int)(i % C4);
        const long r = i / C4;
        const int tap = (int)(r % taps);
        const long p = r / taps;
        const int wo = (int)(p % g.Wo);
        const long r2 = p / g.Wo;
        const int ho = (int)(r2 % g.Ho), n = (int)(r2 / g.Ho);
        const int kh = tap / g.KW, kw = tap - kh * g.KW;
        const int h = ho * g.sh - g.ph + kh, w = wo * g.sw - g.pw + kw;
        T v[4];
        if (h >= 0 && h < g.H && w >= 0 && w < g.W) {
            const T* s = x + (((long)n * g.H + h) * g.W + w) * g.C + c4 * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = s[k];
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = Cvt<T>::from(0.f);
        }
        T* d = cols + (p * taps + tap) * g.C + c4 * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = v[k];
    }
}

// dx[n, h, w, c] = sum over taps (kh, kw) whose output pixel exists of cols[p(ho, wo)][tap, c]
template <typename T>
__global__ __launch_bounds__(256) void col2im_kernel(const T* __restrict__ cols, T* __restrict__ dx, ConvGeom g) {
    const int C4 = g.C >> 2, taps = g.KH * g.KW;
    const long total = (long)g.B * g.H * g.W * C4;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c4 = (int)(i % C4);
        const long pix = i / C4;
        const int w = (int)(pix % g.W);
        const long r = pix / g.W;
        const int h = (int)(r % g.H), n = (int)(r / g.H);
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int kh = 0; kh < g.KH; ++kh) {
            const int hn = h + g.ph - kh;
            if (hn < 0 || hn % g.sh) continue;
            const int ho = hn / g.sh;
            if (ho >= g.Ho) continue;
            for (int kw = 0; kw < g.KW; ++kw) {
                const int wn = w + g.pw - kw;
                if (wn < 0 || wn % g.sw) continue;
                const int wo = wn / g.sw;
                if (wo >= g.Wo) continue;
                const T* s = cols + ((((long)n * g.Ho + ho) * g.Wo + wo) * taps + kh * g.KW + kw) * g.C + c4 * 4;
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[k] += ld(s + k);
            }
        }
        T* d = dx + pix * g.C + c4 * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) st(d + k, acc[k]);
    }
}

// ------------------------------------------------------------------------------ TN GEMM
// C[m][n] = sum_k A[k*lda + m] * B[k*ldb + n]; 64 x 64 tile, 16-deep K step, 4 waves as 2 x 2
// of 32 x 32 (2 x 2 v_mfma_f32_16x16x4_f32 tiles each); operands staged through registers into
// a double-buffered [k][m] LDS image (row stride 80 floats: the two 16-lane halves of a
// ds_read_b32 group land 16 banks apart).  Split-K: blockIdx.z owns rows [z*kc, (z+1)*kc) and
// writes its partial tile to ws + z*M*N (ldc = N), summed by tn_finalize in slice order.
constexpr int TN_BM = 64, TN_BN = 64, TN_BK = 16, TN_LD = 80;
typedef float tn_f32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ void tn_load4(const T* p, int valid, float* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = i < valid ? to_f32(p[i]) : 0.f;
}
template <>
__device__ __forceinline__ void tn_load4<float>(const float* p, int valid, float* v) {
    if (valid == 4 && ((uintptr_t)p & 15) == 0) {
        const float4 f = *reinterpret_cast<const float4*>(p);
        v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = i < valid ? p[i] : 0.f;
    }
}

template <typename T, bool X3>
__global__ __launch_bounds__(256) void gemm_tn_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                      float* __restrict__ C, int M, int N, int K, long lda,
                                                      long ldb, long ldc, int kc, long slice) {
    __shared__ float As[2][TN_BK][TN_LD];
    __shared__ float Bs[2][TN_BK][TN_LD];
    const int m0 = blockIdx.x * TN_BM, n0 = blockIdx.y * TN_BN;
    const int k_begin = blockIdx.z * kc, k_end = min(K, k_begin + kc);
    float* Cz = C + (long)blockIdx.z * slice;
    const int t = threadIdx.x;
    const int lr = t >> 4, lc = (t & 15) * 4;     // loader: row lr of the K step, 4 columns at lc
    const int wave = t >> 6, lane = t & 63;
    const int wm = (wave & 1) * 32, wn = (wave >> 1) * 32;
    tn_f32x4 acc[2][2] = {};
    float ra[4], rb[4];
    auto load = [&](int k0) {
        const int k = k0 + lr;
        const bool kok = k < k_end;
        tn_load4(A + (long)(kok ? k : k_begin) * lda + m0 + lc, kok ? min(4, M - m0 - lc) : 0, ra);
        tn_load4(B + (long)(kok ? k : k_begin) * ldb + n0 + lc, kok ? min(4, N - n0 - lc) : 0, rb);
    };
    auto stash = [&](int buf) {
        *reinterpret_cast<float4*>(&As[buf][lr][lc]) = make_float4(ra[0], ra[1], ra[2], ra[3]);
        *reinterpret_cast<float4*>(&Bs[buf][lr][lc]) = make_float4(rb[0], rb[1], rb[2], rb[3]);
    };
    if (k_begin < k_end) {
        load(k_begin);
        stash(0);
        __syncthreads();
        int buf = 0;
        for (int k0 = k_begin; k0 < k_end; k0 += TN_BK) {
            const bool more = k0 + TN_BK < k_end;
            if (more) load(k0 + TN_BK);
            if constexpr (X3) {
                // KINET_F32_X3: lane group g holds k = 4g..4g+3 of the 16-deep step (the operand
                // map of v_mfma_f32_16x16x16_bf16), split once into bf16 hi + lo, 3 MFMAs a tile
                const int kr = 4 * (lane >> 4);
                X3Frag a[2], b[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int c = wm + i * 16 + (lane & 15);
                    a[i] = split_x3(tn_f32x4{As[buf][kr][c], As[buf][kr + 1][c], As[buf][kr + 2][c], As[buf][kr + 3][c]});
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int c = wn + j * 16 + (lane & 15);
                    b[j] = split_x3(tn_f32x4{Bs[buf][kr][c], Bs[buf][kr + 1][c], Bs[buf][kr + 2][c], Bs[buf][kr + 3][c]});
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) Mma<f32x3_t>::run(acc[i][j], a[i], b[j]);
            } else {
#pragma unroll
                for (int kk = 0; kk < TN_BK; kk += 4) {
                    const int kr = kk + (lane >> 4);
                    float a[2], b[2];
#pragma unroll
                    for (int i = 0; i < 2; ++i) a[i] = As[buf][kr][wm + i * 16 + (lane & 15)];
#pragma unroll
                    for (int j = 0; j < 2; ++j) b[j] = Bs[buf][kr][wn + j * 16 + (lane & 15)];
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
                }
            }
            if (more) {
                stash(buf ^ 1);
                __syncthreads();
                buf ^= 1;
            }
        }
    }
    // C/D map: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm + i * 16 + (lane >> 4) * 4 + r, n = n0 + wn + j * 16 + (lane & 15);
                if (m < M && n < N) Cz[(long)m * ldc + n] = acc[i][j][r];
            }
}

// KINET_F32_X3 TN GEMM: the same 64 x 64 tile and split-K contract as gemm_tn_kernel, K-steps of
// 32, f32 operands split into bf16 hi / lo ONCE on the way into LDS.  Loader: thread t of each
// 128-thread half (A, then B) reads a 4 (k) x 4 (m) block -- 4 coalesced float4 rows -- transposes
// it in registers and writes per m one 16-byte chunk {hi of k0..k0+3, lo of k0..k0+3} at LDS
// (m, k-quad), XOR-swizzled like the main GEMM's tiles; lane (r, g) of a 16x16x16 fragment reads
// exactly that chunk (ds_read_b128).  3 MFMAs per 16x16x16 block (Mma<f32x3_t>).
constexpr int TX_BK = 32;
__global__ __launch_bounds__(256) void gemm_tn_x3_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                         float* __restrict__ C, int M, int N, int K, long lda,
                                                         long ldb, long ldc, int kc, long slice, int vec4,
                                                         int tiles_m, int tiles, int ks) {
    constexpr int TILE = TN_BM * TX_BK * 4;    // bytes of one operand's LDS image (64 rows x 128 B)
    __shared__ __attribute__((aligned(16))) char lds[2][2][TILE];
    // XCD-aware K-slice placement: block b runs on XCD b % 8.  With ks a multiple of 8 every
    // K-slice's tiles go to ONE XCD, so the slice's rows of A and B are fetched into that XCD's
    // L2 once and shared by all its tiles (which walk K together), instead of every XCD
    // re-reading every slice (measured: the 64 x 64 tiles were Infinity-Cache-bandwidth bound)
    const int b = blockIdx.x;
    int z, tile;
    if ((ks & 7) == 0) {   // (an odd ks from the launcher disables the placement)
        const int j = b >> 3;
        z = (b & 7) + 8 * (j / tiles);
        tile = j - (j / tiles) * tiles;
    } else {
        z = b / tiles;
        tile = b - z * tiles;
    }
    const int m0 = (tile % tiles_m) * TN_BM, n0 = (tile / tiles_m) * TN_BN;
    const int k_begin = z * kc, k_end = min(K, k_begin + kc);
    float* Cz = C + (long)z * slice;
    const int t = threadIdx.x;
    const int op = t >> 7;                            // 0: A, 1: B
    const int mq = t & 15, kq = (t >> 4) & 7;         // m-quad (4 columns), k-quad (4 rows)
    const float* src = op ? B : A;
    const long ld = op ? ldb : lda;
    const int c0 = (op ? n0 : m0) + mq * 4;
    const int lim = op ? N : M;
    const int cvalid = max(0, min(4, lim - c0));
    const int wave = t >> 6, lane = t & 63;
    const int wm = (wave & 1) * 32, wn = (wave >> 1) * 32;
    tn_f32x4 acc[2][2] = {};
    // branch-free staging loads (a conditional load costs a vmcnt(0) drain per branch): buffer
    // loads whose K-tail rows get an offset past num_records (the range check returns zeros);
    // columns past M / N read whatever follows -- they only reach output rows / columns that
    // are never stored
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)min((long)K * ld * 4, (long)INT_MAX), 0x00020000);
    const unsigned cbad = c0 < lim ? 0u : 0x80000000u;
    (void)vec4;
    auto load = [&](int k0, u32x4 (&v)[4]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = k0 + kq * 4 + r;
            const unsigned off = (unsigned)(((long)k * ld + c0) * 4) | (k < k_end ? cbad : 0x80000000u);
            v[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
        }
    };
    auto stash = [&](int buf, const u32x4 (&v)[4]) {
        char* L = lds[buf][op];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = mq * 4 + i;
            *reinterpret_cast<u32x4*>(L + swz(m, kq)) = Mma<f32x3_t>::stage(u32x4{v[0][i], v[1][i], v[2][i], v[3][i]});
        }
    };
    auto compute = [&](int buf) {
        // v_mfma_f32_16x16x32_bf16: lane group g takes the k-quads 2g, 2g+1
        const char* La = lds[buf][0];
        const char* Lb = lds[buf][1];
        const int q0 = 2 * (lane >> 4);
        u32x4 a0[2], a1[2], b0[2], b1[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int r = wm + i * 16 + (lane & 15);
            a0[i] = *reinterpret_cast<const u32x4*>(La + swz(r, q0));
            a1[i] = *reinterpret_cast<const u32x4*>(La + swz(r, q0 + 1));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r = wn + j * 16 + (lane & 15);
            b0[j] = *reinterpret_cast<const u32x4*>(Lb + swz(r, q0));
            b1[j] = *reinterpret_cast<const u32x4*>(Lb + swz(r, q0 + 1));
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) Mma<f32x3_t>::run32(acc[i][j], a0[i], a1[i], b0[j], b1[j]);
    };
    // two register staging sets, loads issued two K-steps ahead (as gemm.hip's main loop):
    // step kt loads kt+2 into the set that held kt, computes kt, stashes kt+1, one barrier;
    // steps past the end load zeros (range check) and multiply them
    const int nk = (k_end - k_begin + TX_BK - 1) / TX_BK;
    if (nk > 0) {
        u32x4 v0[4], v1[4];
        load(k_begin, v0);
        load(k_begin + TX_BK, v1);
        stash(0, v0);
        __syncthreads();
        for (int kt = 0; kt < nk; kt += 2) {
            load(k_begin + (kt + 2) * TX_BK, v0);
            compute(0);
            stash(1, v1);
            __syncthreads();
            if (kt + 1 >= nk) break;
            load(k_begin + (kt + 3) * TX_BK, v1);
            compute(1);
            stash(0, v0);
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm + i * 16 + (lane >> 4) * 4 + r, n = n0 + wn + j * 16 + (lane & 15);
                if (m < M && n < N) Cz[(long)m * ldc + n] = acc[i][j][r];
            }
}

// C[m][n] (+)= sum_z ws[z][m][n], z in order
__global__ __launch_bounds__(256) void tn_finalize_kernel(const float* __restrict__ ws, float* __restrict__ C, int M,
                                                          int N, long ldc, int nz, int accumulate) {
    const long total = (long)M * N;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        float s = 0.f;
        for (int z = 0; z < nz; ++z) s += ws[z * total + i];
        const int m = (int)(i / N), n = (int)(i % N);
        float* c = C + (long)m * ldc + n;
        *c = accumulate ? *c + s : s;
    }
}

// ------------------------------------------------------------------------------ colsum
// pass 1: ws[chunk][c] = sum of rows [chunk*rc, ...) of column c; pass 2: out[c] (+)= sum_chunk
template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const T* __restrict__ A, float* __restrict__ ws, int rows,
                                                             int cols, long lda, int rc) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= cols) return;
    const int r0 = blockIdx.y * rc, r1 = min(rows, r0 + rc);
    float s = 0.f;
    for (int r = r0; r < r1; ++r) s += ld(A + (long)r * lda + c);
    ws[(long)blockIdx.y * cols + c] = s;
}

// f32, 4-column vectors: lane = 4 columns (one float4 per row), the 4 waves take rows
// r0 + w, r0 + w + 4, ... with two independent accumulators each, combined in a fixed order
// through LDS (deterministic); one row-chunk per blockIdx.y like colsum_partial_kernel
__global__ __launch_bounds__(256) void colsum_partial_vec_kernel(const float* __restrict__ A, float* __restrict__ ws,
                                                                 int rows, int cols, long lda, int rc) {
    __shared__ float4 part[4][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c4 = blockIdx.x * 64 + lane;
    const bool cv = c4 * 4 < cols;
    const int r0 = blockIdx.y * rc, r1 = min(rows, r0 + rc);
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
    if (cv) {
        const float* p = A + c4 * 4;
        int r = r0 + wave;
        for (; r + 4 < r1; r += 8) {
            const float4 x = *reinterpret_cast<const float4*>(p + (long)r * lda);
            const float4 y = *reinterpret_cast<const float4*>(p + (long)(r + 4) * lda);
            s0.x += x.x; s0.y += x.y; s0.z += x.z; s0.w += x.w;
            s1.x += y.x; s1.y += y.y; s1.z += y.z; s1.w += y.w;
        }
        if (r < r1) {
            const float4 x = *reinterpret_cast<const float4*>(p + (long)r * lda);
            s0.x += x.x; s0.y += x.y; s0.z += x.z; s0.w += x.w;
        }
    }
    part[wave][lane] = make_float4(s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w);
    __syncthreads();
    if (wave == 0 && cv) {
        float4 t = part[0][lane];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
            const float4 u = part[w][lane];
            t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
        }
        *reinterpret_cast<float4*>(ws + (long)blockIdx.y * cols + c4 * 4) = t;
    }
}

// one workgroup per column: thread t sums chunks t, t+256, ... in order, then a fixed-order
// LDS tree (deterministic; a serial per-column loop over ~10^3 partials was 50 us a call)
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ ws, float* __restrict__ out,
                                                           int cols, int nchunk, int accumulate) {
    __shared__ float red[256];
    const int c = blockIdx.x;
    float s = 0.f;
    for (int k = threadIdx.x; k < nchunk; k += 256) s += ws[(long)k * cols + c];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[c] = accumulate ? out[c] + red[0] : red[0];
}

// ------------------------------------------------------------------------- LayerNorm bwd
// one wave per row; mean / rstd recomputed from x (deformable_transformer.py post-norms);
// per-workgroup partial dgamma/dbeta (4 waves x RPW rows) summed by colsum_final in order
template <typename T>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const float* __restrict__ gamma, T* __restrict__ dx,
                                                            float* __restrict__ pg, float* __restrict__ pb, int rows,
                                                            int d, float eps, int rpw) {
    constexpr int MAXV = 16;   // d <= 1024
    extern __shared__ float red[];   // [4][2][d]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nv = (d + 63) / 64;
    float g_acc[MAXV], b_acc[MAXV];
#pragma unroll
    for (int v = 0; v < MAXV; ++v) g_acc[v] = b_acc[v] = 0.f;
    const int r_begin = (blockIdx.x * 4 + wave) * rpw;
    for (int r = r_begin; r < min(rows, r_begin + rpw); ++r) {
        const T* xr = x + (long)r * d;
        const T* dr = dy + (long)r * d;
        float xv[MAXV], dv[MAXV];
        float s = 0.f;
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            const int c = v * 64 + lane;
            xv[v] = (v < nv && c < d) ? ld(xr + c) : 0.f;
            dv[v] = (v < nv && c < d) ? ld(dr + c) : 0.f;
            s += xv[v];
        }
        for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
        const float mean = s / (float)d;
        float q = 0.f;
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            const int c = v * 64 + lane;
            const float t = (v < nv && c < d) ? xv[v] - mean : 0.f;
            q += t * t;
        }
        for (int o = 32; o; o >>= 1) q += __shfl_xor(q, o);
        const float rstd = rsqrtf(q / (float)d + eps);
        float sg = 0.f, sgx = 0.f;
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            const int c = v * 64 + lane;
            if (v < nv && c < d) {
                const float xh = (xv[v] - mean) * rstd;
                const float g = dv[v] * gamma[c];
                sg += g;
                sgx += g * xh;
                g_acc[v] += dv[v] * xh;
                b_acc[v] += dv[v];
            }
        }
        for (int o = 32; o; o >>= 1) {
            sg += __shfl_xor(sg, o);
            sgx += __shfl_xor(sgx, o);
        }
        const float inv_d = 1.f / (float)d;
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            const int c = v * 64 + lane;
            if (v < nv && c < d) {
                const float xh = (xv[v] - mean) * rstd;
                st(dx + (long)r * d + c, rstd * (dv[v] * gamma[c] - sg * inv_d - xh * sgx * inv_d));
            }
        }
    }
    // per-workgroup partials, waves combined in order
#pragma unroll
    for (int v = 0; v < MAXV; ++v) {
        const int c = v * 64 + lane;
        if (v < nv && c < d) {
            red[(wave * 2) * d + c] = g_acc[v];
            red[(wave * 2 + 1) * d + c] = b_acc[v];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < d; c += 256) {
        float gs = 0.f, bs = 0.f;
        for (int w = 0; w < 4; ++w) {
            gs += red[(w * 2) * d + c];
            bs += red[(w * 2 + 1) * d + c];
        }
        pg[(long)blockIdx.x * d + c] = gs;
        pb[(long)blockIdx.x * d + c] = bs;
    }
}

// ------------------------------------------------------------------------- GroupNorm bwd
// x, dy: (N, HW, C) NHWC.  pass 1 per (image, HW block): per-channel sums of dy, dy*x, x, x^2
template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_partial_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                             float* __restrict__ part, int HW, int C, int rb) {
    const int n = blockIdx.y, blk = blockIdx.x, nblk = gridDim.x;
    const int p0 = blk * rb, p1 = min(HW, p0 + rb);
    for (int c = threadIdx.x; c < C; c += 256) {
        float sdy = 0.f, sdyx = 0.f, sx = 0.f, sxx = 0.f;
        for (int p = p0; p < p1; ++p) {
            const long o = ((long)n * HW + p) * C + c;
            const float xv = ld(x + o), dv = ld(dy + o);
            sdy += dv;
            sdyx += dv * xv;
            sx += xv;
            sxx += xv * xv;
        }
        float* q = part + (((long)n * nblk + blk) * 4) * C + c;
        q[0] = sdy;
        q[C] = sdyx;
        q[2 * C] = sx;
        q[3 * C] = sxx;
    }
}

// pass 1 for C % 4 == 0: a workgroup covers its rows with whole 4-channel vectors per thread
// (256 / (C/4) rows at a time, e.g. 3 rows of 72 float4 at C = 288), so every lane streams
// contiguous 16-byte pieces and the grid has enough workgroups to fill the chip; the row groups'
// sums are added in LDS in a fixed order (deterministic)
template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_partial_vec_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                 float* __restrict__ part, int HW, int C, int rb) {
    __shared__ float red[4 * 1024];   // [row group][4 sums][C], rows_per_it * C <= 1024
    const int n = blockIdx.y, blk = blockIdx.x, nblk = gridDim.x;
    const int p0 = blk * rb, p1 = min(HW, p0 + rb);
    const int C4 = C >> 2, rpi = 256 / C4;
    const int tr = threadIdx.x / C4, tc = threadIdx.x - tr * C4;
    float a[4][4] = {};
    if (tr < rpi) {
        for (int p = p0 + tr; p < p1; p += rpi) {
            const long o = ((long)n * HW + p) * C + tc * 4;
            float xv[4], dv[4];
            if constexpr (std::is_same<T, float>::value) {
                const float4 x4 = *reinterpret_cast<const float4*>(x + o), d4 = *reinterpret_cast<const float4*>(dy + o);
                xv[0] = x4.x; xv[1] = x4.y; xv[2] = x4.z; xv[3] = x4.w;
                dv[0] = d4.x; dv[1] = d4.y; dv[2] = d4.z; dv[3] = d4.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) { xv[j] = ld(x + o + j); dv[j] = ld(dy + o + j); }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                a[0][j] += dv[j];
                a[1][j] += dv[j] * xv[j];
                a[2][j] += xv[j];
                a[3][j] += xv[j] * xv[j];
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) red[(tr * 4 + k) * C + tc * 4 + j] = a[k][j];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * C; i += 256) {
        float v = 0.f;
        for (int r = 0; r < rpi; ++r) v += red[r * 4 * C + i];   // i = k*C + c
        part[((long)n * nblk + blk) * 4 * C + i] = v;
    }
}

// pass 2 (one workgroup per image): per-channel sums over the blocks, then per group the
// statistics and the two backward scalars; writes stats[n][g] = (mean, rstd, a/cnt, bsum/cnt)
// and per-image channel sums for dgamma / dbeta
__global__ __launch_bounds__(1024) void gn_bwd_stats_kernel(const float* __restrict__ part, const float* __restrict__ gamma,
                                                            float* __restrict__ stats, float* __restrict__ chan,
                                                            int HW, int C, int G, int nblk, float eps) {
    extern __shared__ float sm[];   // [4][C]
    const int n = blockIdx.x;
    // one (sum, channel) per thread, the blocks summed in order (4 independent loads in flight)
    for (int i = threadIdx.x; i < 4 * C; i += blockDim.x) {
        const float* q = part + (long)n * nblk * 4 * C + i;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        int b = 0;
        for (; b + 3 < nblk; b += 4) {
            s0 += q[(long)b * 4 * C];
            s1 += q[(long)(b + 1) * 4 * C];
            s2 += q[(long)(b + 2) * 4 * C];
            s3 += q[(long)(b + 3) * 4 * C];
        }
        for (; b < nblk; ++b) s0 += q[(long)b * 4 * C];
        sm[i] = (s0 + s1) + (s2 + s3);
    }
    __syncthreads();
    const int cg = C / G;
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
        float sx = 0.f, sxx = 0.f, a = 0.f, bs = 0.f;
        for (int c = g * cg; c < (g + 1) * cg; ++c) {
            sx += sm[2 * C + c];
            sxx += sm[3 * C + c];
            a += gamma[c] * sm[c];
            bs += gamma[c] * sm[C + c];
        }
        const float cnt = (float)HW * (float)cg;
        const float mean = sx / cnt;
        const float var = fmaxf(sxx / cnt - mean * mean, 0.f);
        const float rstd = rsqrtf(var + eps);
        // sum(dy*gamma*xhat) = rstd * (sum(dy*gamma*x) - mean * sum(dy*gamma))
        const float bx = rstd * (bs - mean * a);
        float* st4 = stats + ((long)n * G + g) * 4;
        st4[0] = mean;
        st4[1] = rstd;
        st4[2] = a / cnt;
        st4[3] = bx / cnt;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const float* st4 = stats + ((long)n * G + c / cg) * 4;
        // dgamma_n[c] = sum dy*xhat = rstd*(sum dy*x - mean*sum dy); dbeta_n[c] = sum dy
        chan[((long)n * 2) * C + c] = st4[1] * (sm[C + c] - st4[0] * sm[c]);
        chan[((long)n * 2 + 1) * C + c] = sm[c];
    }
}

template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                           const float* __restrict__ gamma, const float* __restrict__ stats,
                                                           T* __restrict__ dx, int HW, int C, int G, long total) {
    const int cg = C / G;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c = (int)(i % C);
        const long n = i / ((long)HW * C);
        const float* st4 = stats + (n * G + c / cg) * 4;
        const float xh = (ld(x + i) - st4[0]) * st4[1];
        st(dx + i, st4[1] * (ld(dy + i) * gamma[c] - st4[2] - xh * st4[3]));
    }
}

// the same for C % 4 == 0 and fewer than 2^31 elements: 4 channels per thread, 32-bit index math
template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_apply_vec_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                               const float* __restrict__ gamma, const float* __restrict__ stats,
                                                               T* __restrict__ dx, int HW, int C, int G, int total4) {
    const int cg = C / G, img = HW * C;
    for (int i4 = blockIdx.x * 256 + threadIdx.x; i4 < total4; i4 += gridDim.x * 256) {
        const int i = i4 * 4;
        const int n = i / img;
        const int c0 = (i - n * img) % C;   // C % 4 == 0: the 4 channels lie in one row
        float xv[4], dv[4], o[4];
        if constexpr (std::is_same<T, float>::value) {
            const float4 x4 = *reinterpret_cast<const float4*>(x + i), d4 = *reinterpret_cast<const float4*>(dy + i);
            xv[0] = x4.x; xv[1] = x4.y; xv[2] = x4.z; xv[3] = x4.w;
            dv[0] = d4.x; dv[1] = d4.y; dv[2] = d4.z; dv[3] = d4.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) { xv[j] = ld(x + i + j); dv[j] = ld(dy + i + j); }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 st4 = *reinterpret_cast<const float4*>(stats + ((long)n * G + (c0 + j) / cg) * 4);
            const float xh = (xv[j] - st4.x) * st4.y;
            o[j] = st4.y * (dv[j] * gamma[c0 + j] - st4.z - xh * st4.w);
        }
        if constexpr (std::is_same<T, float>::value) {
            *reinterpret_cast<float4*>(dx + i) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) st(dx + i + j, o[j]);
        }
    }
}

// dgamma/dbeta = sum over images of chan[n]
__global__ __launch_bounds__(256) void gn_bwd_param_kernel(const float* __restrict__ chan, float* __restrict__ dgamma,
                                                           float* __restrict__ dbeta, int N, int C) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    float g = 0.f, b = 0.f;
    for (int n = 0; n < N; ++n) {
        g += chan[((long)n * 2) * C + c];
        b += chan[((long)n * 2 + 1) * C + c];
    }
    if (dgamma) dgamma[c] = g;
    if (dbeta) dbeta[c] = b;
}

// ------------------------------------------------------------------------- attention bwd
// With dropout (scaled keep mask Z): O_i = sum_j P_ij Z_ij V_j, so dV_j = sum_i P_ij Z_ij dO_i,
// dP_ij = Z_ij dO_i.V_j, di = dO_i.O_i = sum_j P_ij dP_ij, dS_ij = P_ij (dP_ij - di); the
// workspace keeps P_ij Z_ij (for dV) and dS_ij (for dK).
struct AttnArgs {
    const float *Q, *K, *V, *dO;
    float *dQ, *dK, *dV, *P, *dS;
    const uint8_t* key_mask;
    int ldq, ldk, ldv, ldo;   // row strides (elements); dQ/dK/dV use ldq/ldk/ldv
    int B, Lq, Lk, H, D;
    float scale;
    const int64_t* dseed;     // attention-probability dropout (nullptr: none), common.h dropout_keep
    uint32_t dthresh;
    float dscale;
};

constexpr int ATT_MAXD = 64;

// Tiled attention backward.  (Wave-per-row kernels, which read every key row per query through
// per-lane strided loads, took ~0.9 ms per decoder self-attention at config 4.)  A lane owns
// one query (q2) or one key (kv2), the eight waves of a workgroup split the other dimension,
// and that dimension's rows are staged in LDS in chunks of 64 and read as broadcasts.
constexpr int AT_T = 64;
// waves per workgroup splitting the other dimension: 8, or 4 for head dims past 36 (LDS)
template <int MD> constexpr int at_nw() { return MD <= 36 ? 8 : 4; }
template <int MD>
__device__ __forceinline__ float dot_lds(const float (&x)[MD], const float* row) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < MD; d += 4) {
        const float4 k = *reinterpret_cast<const float4*>(row + d);
        s += x[d] * k.x + x[d + 1] * k.y + x[d + 2] * k.z + x[d + 3] * k.w;
    }
    return s;
}
// the same 64-row chunk held in registers (this thread's elements), so the next chunk's
// global loads are in flight while the current one is computed
template <int MD, int AT_NT>
struct RowChunk {
    static constexpr int N = (AT_T * MD + AT_NT - 1) / AT_NT;
    float v[N];
    __device__ __forceinline__ void load(const float* src, long ld, int r0, int rows, int c0, int D) {
#pragma unroll
        for (int u = 0; u < N; ++u) {
            const int e = threadIdx.x + AT_NT * u, r = e / MD, d = e - (e / MD) * MD, rr = r0 + r;
            v[u] = (e < AT_T * MD && rr < rows && d < D) ? src[(long)rr * ld + c0 + d] : 0.f;
        }
    }
    __device__ __forceinline__ void store(float (*dst)[MD]) const {
#pragma unroll
        for (int u = 0; u < N; ++u) {
            const int e = threadIdx.x + AT_NT * u;
            if (e < AT_T * MD) dst[e / MD][e - (e / MD) * MD] = v[u];
        }
    }
};

// pass 1: lane = query i; softmax statistics, then di_i = sum_j P_ij dP_ij, then dS_ij and
// dQ_i = scale * sum_j dS_ij K_j; P and dS rows stored to the workspace for pass 2
template <int MD, int AT_NW = at_nw<MD>(), int AT_NT = 64 * AT_NW>
__global__ __launch_bounds__(AT_NT) void attn_bwd_q2_kernel(AttnArgs a) {
    __shared__ __attribute__((aligned(16))) float Ks[AT_T][MD];
    __shared__ __attribute__((aligned(16))) float Vs[AT_T][MD];
    __shared__ float st[AT_NW][AT_T][2];
    __shared__ float red[AT_NW][AT_T][MD + 1];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
    const int i = blockIdx.x * AT_T + lane;
    const bool iv = i < a.Lq;
    float qv[MD], ov[MD];
    {
        const float* q = a.Q + ((long)b * a.Lq + (iv ? i : 0)) * a.ldq + h * a.D;
        const float* o = a.dO + ((long)b * a.Lq + (iv ? i : 0)) * a.ldo + h * a.D;
#pragma unroll
        for (int d = 0; d < MD; ++d) {
            qv[d] = (iv && d < a.D) ? q[d] : 0.f;
            ov[d] = (iv && d < a.D) ? o[d] : 0.f;
        }
    }
    const float* Kb = a.K + (long)b * a.Lk * a.ldk;
    const float* Vb = a.V + (long)b * a.Lk * a.ldv;
    const uint8_t* km = a.key_mask ? a.key_mask + (long)b * a.Lk : nullptr;
    float* Prow = a.P + ((long)bh * a.Lq + (iv ? i : 0)) * a.Lk;
    float* Srow = a.dS + ((long)bh * a.Lq + (iv ? i : 0)) * a.Lk;
    const int r0 = wave * (AT_T / AT_NW);
    auto score = [&](int r, int j) {
        const float sc = dot_lds<MD>(qv, Ks[r]) * a.scale;
        return (km && km[j]) ? -INFINITY : sc;
    };
    // phase A: running max / sum over this wave's keys of every chunk
    float m = -INFINITY, l = 0.f;
    RowChunk<MD, AT_NT> ck, cv;
    // chunk loop with the next chunk's loads issued before the current chunk is computed
    auto chunks = [&](bool withV, auto&& body) {
        ck.load(Kb, a.ldk, 0, a.Lk, h * a.D, a.D);
        if (withV) cv.load(Vb, a.ldv, 0, a.Lk, h * a.D, a.D);
        for (int j0 = 0; j0 < a.Lk; j0 += AT_T) {
            __syncthreads();
            ck.store(Ks);
            if (withV) cv.store(Vs);
            __syncthreads();
            if (j0 + AT_T < a.Lk) {
                ck.load(Kb, a.ldk, j0 + AT_T, a.Lk, h * a.D, a.D);
                if (withV) cv.load(Vb, a.ldv, j0 + AT_T, a.Lk, h * a.D, a.D);
            }
            body(j0);
        }
    };
    chunks(false, [&](int j0) {
        for (int r = r0; r < r0 + AT_T / AT_NW && j0 + r < a.Lk; ++r) {
            const float sc = score(r, j0 + r);
            if (sc == -INFINITY) continue;
            if (sc > m) {
                l = l * __expf(m - sc) + 1.f;
                m = sc;
            } else {
                l += __expf(sc - m);
            }
        }
    });
    st[wave][lane][0] = m;
    st[wave][lane][1] = l;
    __syncthreads();
    float mx = -INFINITY;
#pragma unroll
    for (int w = 0; w < AT_NW; ++w) mx = fmaxf(mx, st[w][lane][0]);
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < AT_NW; ++w)
        if (st[w][lane][0] != -INFINITY) sum += st[w][lane][1] * __expf(st[w][lane][0] - mx);
    const float rs = sum > 0.f ? 1.f / sum : 0.f;
    auto prob = [&](float sc) { return (mx == -INFINITY || sc == -INFINITY) ? 0.f : __expf(sc - mx) * rs; };
    // dropout keep scale of (i, j): 1 without dropout, else 0 or 1 / (1 - p)
    const uint64_t dseed = a.dseed ? (uint64_t)*a.dseed : 0ull;
    const uint64_t drow = ((uint64_t)bh * a.Lq + (uint64_t)(iv ? i : 0)) * (uint64_t)a.Lk;
    auto zf = [&](int j) {
        return a.dseed ? (dropout_keep(dseed, drow + (uint64_t)j, a.dthresh) ? a.dscale : 0.f) : 1.f;
    };
    // phase B: di = sum_j P_ij Z_ij (dO_i . V_j); P Z stored
    float di = 0.f;
    chunks(true, [&](int j0) {
        for (int r = r0; r < r0 + AT_T / AT_NW && j0 + r < a.Lk; ++r) {
            const float pz = prob(score(r, j0 + r)) * zf(j0 + r);
            di += pz * dot_lds<MD>(ov, Vs[r]);
            if (iv) Prow[j0 + r] = pz;
        }
    });
    __syncthreads();
    st[wave][lane][0] = di;
    __syncthreads();
    di = 0.f;
#pragma unroll
    for (int w = 0; w < AT_NW; ++w) di += st[w][lane][0];
    // phase C: dS_ij = P_ij (dP_ij - di), dQ_i partial over this wave's keys
    float dq[MD];
#pragma unroll
    for (int d = 0; d < MD; ++d) dq[d] = 0.f;
    chunks(true, [&](int j0) {
        for (int r = r0; r < r0 + AT_T / AT_NW && j0 + r < a.Lk; ++r) {
            const float p = prob(score(r, j0 + r));
            const float ds = p * (zf(j0 + r) * dot_lds<MD>(ov, Vs[r]) - di);
            if (iv) Srow[j0 + r] = ds;
#pragma unroll
            for (int d = 0; d < MD; d += 4) {
                const float4 k = *reinterpret_cast<const float4*>(&Ks[r][d]);
                dq[d] += ds * k.x;
                dq[d + 1] += ds * k.y;
                dq[d + 2] += ds * k.z;
                dq[d + 3] += ds * k.w;
            }
        }
    });
    __syncthreads();
#pragma unroll
    for (int d = 0; d < MD; ++d) red[wave][lane][d] = dq[d];
    __syncthreads();
    for (int e = threadIdx.x; e < AT_T * MD; e += AT_NT) {
        const int li = e / MD, d = e - (e / MD) * MD, ii = blockIdx.x * AT_T + li;
        if (ii < a.Lq && d < a.D) {
            float v = 0.f;
#pragma unroll
            for (int w = 0; w < AT_NW; ++w) v += red[w][li][d];
            a.dQ[((long)b * a.Lq + ii) * a.ldq + h * a.D + d] = v * a.scale;
        }
    }
}

// pass 2: lane = key j; dK_j = scale * sum_i dS_ij Q_i, dV_j = sum_i P_ij dO_i (P / dS rows read
// coalesced across the 64 keys of the tile)
template <int MD, int AT_NW = at_nw<MD>(), int AT_NT = 64 * AT_NW>
__global__ __launch_bounds__(AT_NT) void attn_bwd_kv2_kernel(AttnArgs a) {
    __shared__ __attribute__((aligned(16))) float Qs[AT_T][MD];
    __shared__ __attribute__((aligned(16))) float Os[AT_T][MD];
    __shared__ float red[AT_NW][AT_T][MD + 1];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
    const int j = blockIdx.x * AT_T + lane;
    const bool jv = j < a.Lk;
    const float* Pc = a.P + (long)bh * a.Lq * a.Lk + (jv ? j : 0);
    const float* Sc = a.dS + (long)bh * a.Lq * a.Lk + (jv ? j : 0);
    const float* Qb = a.Q + (long)b * a.Lq * a.ldq;
    const float* Ob = a.dO + (long)b * a.Lq * a.ldo;
    float dk[MD], dv[MD];
#pragma unroll
    for (int d = 0; d < MD; ++d) dk[d] = dv[d] = 0.f;
    const int r0 = wave * (AT_T / AT_NW);
    RowChunk<MD, AT_NT> cq, co;
    cq.load(Qb, a.ldq, 0, a.Lq, h * a.D, a.D);
    co.load(Ob, a.ldo, 0, a.Lq, h * a.D, a.D);
    for (int i0 = 0; i0 < a.Lq; i0 += AT_T) {
        __syncthreads();
        cq.store(Qs);
        co.store(Os);
        __syncthreads();
        if (i0 + AT_T < a.Lq) {
            cq.load(Qb, a.ldq, i0 + AT_T, a.Lq, h * a.D, a.D);
            co.load(Ob, a.ldo, i0 + AT_T, a.Lq, h * a.D, a.D);
        }
        for (int r = r0; r < r0 + AT_T / AT_NW && i0 + r < a.Lq; ++r) {
            const long ro = (long)(i0 + r) * a.Lk;
            const float p = jv ? Pc[ro] : 0.f, ds = jv ? Sc[ro] : 0.f;
#pragma unroll
            for (int d = 0; d < MD; d += 4) {
                const float4 q = *reinterpret_cast<const float4*>(&Qs[r][d]);
                const float4 o = *reinterpret_cast<const float4*>(&Os[r][d]);
                dk[d] += ds * q.x; dk[d + 1] += ds * q.y; dk[d + 2] += ds * q.z; dk[d + 3] += ds * q.w;
                dv[d] += p * o.x; dv[d + 1] += p * o.y; dv[d + 2] += p * o.z; dv[d + 3] += p * o.w;
            }
        }
    }
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        __syncthreads();
#pragma unroll
        for (int d = 0; d < MD; ++d) red[wave][lane][d] = pass ? dv[d] : dk[d];
        __syncthreads();
        for (int e = threadIdx.x; e < AT_T * MD; e += AT_NT) {
            const int lj = e / MD, d = e - (e / MD) * MD, jj = blockIdx.x * AT_T + lj;
            if (jj < a.Lk && d < a.D) {
                float v = 0.f;
#pragma unroll
                for (int w = 0; w < AT_NW; ++w) v += red[w][lj][d];
                if (pass) a.dV[((long)b * a.Lk + jj) * a.ldv + h * a.D + d] = v;
                else a.dK[((long)b * a.Lk + jj) * a.ldk + h * a.D + d] = v * a.scale;
            }
        }
    }
}

int grid_for(long n) { return (int)std::min<long>((n + 255) / 256, 8192); }

}  // namespace
}  // namespace kinet

using namespace kinet;

extern "C" int kinet_transpose(const void* src, void* dst, int rows, int cols, int64_t ld_src, int64_t ld_dst,
                               int dtype, kinet_stream_t stream) {
    KINET_CHECK_ARG(rows >= 0 && cols >= 0 && ld_src >= cols && ld_dst >= rows, "transpose: bad sizes");
    if (rows == 0 || cols == 0) return KINET_OK;
    dim3 grid((cols + 31) / 32, (rows + 31) / 32);
    hipStream_t s = (hipStream_t)stream;
    if (dtype == KINET_F32)
        hipLaunchKernelGGL(transpose_kernel<float>, grid, dim3(256), 0, s, (const float*)src, (float*)dst, rows, cols,
                           (long)ld_src, (long)ld_dst);
    else if (dtype == KINET_BF16 || dtype == KINET_F16)
        hipLaunchKernelGGL(transpose_kernel<uint16_t>, grid, dim3(256), 0, s, (const uint16_t*)src, (uint16_t*)dst, rows,
                           cols, (long)ld_src, (long)ld_dst);
    else {
        set_error("transpose: unsupported dtype %d", dtype);
        return KINET_ERR_ARG;
    }
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

static int conv_geom(ConvGeom& g, int B, int H, int W, int C, int Ho, int Wo, int KH, int KW, int sh, int sw, int ph,
                     int pw) {
    KINET_CHECK_ARG(C % 4 == 0, "im2col/col2im: channels must be a multiple of 4 (got %d)", C);
    KINET_CHECK_ARG(sh > 0 && sw > 0 && KH > 0 && KW > 0, "im2col/col2im: bad kernel / stride");
    KINET_CHECK_ARG(Ho == (H + 2 * ph - KH) / sh + 1 && Wo == (W + 2 * pw - KW) / sw + 1,
                    "im2col/col2im: output size (%d, %d) does not match the geometry", Ho, Wo);
    g = ConvGeom{B, H, W, C, Ho, Wo, KH, KW, sh, sw, ph, pw};
    return KINET_OK;
}

extern "C" int kinet_im2col_nhwc(const void* x, void* cols, int B, int H, int W, int C, int Ho, int Wo, int KH,
                                 int KW, int sh, int sw, int ph, int pw, int dtype, kinet_stream_t stream) {
    ConvGeom g;
    int rc = conv_geom(g, B, H, W, C, Ho, Wo, KH, KW, sh, sw, ph, pw);
    if (rc) return rc;
    const long n = (long)B * Ho * Wo * KH * KW * (C / 4);
    if (n == 0) return KINET_OK;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == KINET_F32) hipLaunchKernelGGL(im2col_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, (const float*)x, (float*)cols, g);
    else if (dtype == KINET_BF16) hipLaunchKernelGGL(im2col_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)cols, g);
    else if (dtype == KINET_F16) hipLaunchKernelGGL(im2col_kernel<f16_t>, dim3(grid_for(n)), dim3(256), 0, s, (const f16_t*)x, (f16_t*)cols, g);
    else { set_error("im2col: unsupported dtype %d", dtype); return KINET_ERR_ARG; }
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_col2im_nhwc(const void* cols, void* dx, int B, int H, int W, int C, int Ho, int Wo, int KH,
                                 int KW, int sh, int sw, int ph, int pw, int dtype, kinet_stream_t stream) {
    ConvGeom g;
    int rc = conv_geom(g, B, H, W, C, Ho, Wo, KH, KW, sh, sw, ph, pw);
    if (rc) return rc;
    const long n = (long)B * H * W * (C / 4);
    if (n == 0) return KINET_OK;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == KINET_F32) hipLaunchKernelGGL(col2im_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, (const float*)cols, (float*)dx, g);
    else if (dtype == KINET_BF16) hipLaunchKernelGGL(col2im_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, (const bf16_t*)cols, (bf16_t*)dx, g);
    else if (dtype == KINET_F16) hipLaunchKernelGGL(col2im_kernel<f16_t>, dim3(grid_for(n)), dim3(256), 0, s, (const f16_t*)cols, (f16_t*)dx, g);
    else { set_error("col2im: unsupported dtype %d", dtype); return KINET_ERR_ARG; }
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int64_t kinet_gemm_tn_workspace(int M, int N, int K) {
    const long long tiles = (long long)((M + TN_BM - 1) / TN_BM) * ((N + TN_BN - 1) / TN_BN);
    if (tiles <= 0 || K <= 0) return 0;
    int ks = (int)std::min<long long>(64, std::max<long long>(1, 1024 / tiles));
    ks = std::min(ks, std::max(1, K / 64));
    if (ks >= 8) ks = std::min(64, (ks + 7) & ~7);   // whole K-slices per XCD (gemm_tn_x3_kernel)
    return ks > 1 ? (int64_t)ks * M * N : 0;
}

extern "C" int kinet_gemm_tn(const void* A, const void* B, float* C, int M, int N, int K, int64_t lda, int64_t ldb,
                             int64_t ldc, int dtype, int accumulate, float* workspace, kinet_stream_t stream) {
    KINET_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && lda >= M && ldb >= N && ldc >= N, "gemm_tn: bad sizes");
    if (M == 0 || N == 0) return KINET_OK;
    hipStream_t s = (hipStream_t)stream;
    const long long ws_elems = kinet_gemm_tn_workspace(M, N, K);
    int ks = ws_elems ? (int)(ws_elems / ((long long)M * N)) : 1;
    KINET_CHECK_ARG(ks == 1 || workspace, "gemm_tn: needs kinet_gemm_tn_workspace(M, N, K) floats of workspace");
    if (K == 0) {
        if (!accumulate) KINET_CHECK_HIP(hipMemset2DAsync(C, ldc * 4, 0, (size_t)N * 4, M, s));
        return KINET_OK;
    }
    const int kc = ((K + ks - 1) / ks + TN_BK - 1) / TN_BK * TN_BK;
    ks = (K + kc - 1) / kc;
    const bool direct = ks == 1 && !accumulate;
    float* out = direct ? C : workspace;
    const long slice = (long)M * N;
    const long ldo = direct ? (long)ldc : (long)N;
    if (!direct && !workspace) {
        set_error("gemm_tn: accumulate needs a workspace of M*N floats");
        return KINET_ERR_ARG;
    }
    dim3 grid((M + TN_BM - 1) / TN_BM, (N + TN_BN - 1) / TN_BN, ks);
    if (dtype == KINET_F32)
        hipLaunchKernelGGL((gemm_tn_kernel<float, false>), grid, dim3(256), 0, s, (const float*)A, (const float*)B, out, M, N, K,
                           (long)lda, (long)ldb, ldo, kc, slice);
    else if (dtype == KINET_F32_X3 && !(kinet_gemm_flags & 128) &&
             ((long long)K + 2 * TX_BK) * std::max(lda, ldb) * 4 < (1LL << 31)) {   // 31-bit buffer offsets
        const int vec4 = (lda % 4 == 0) && (ldb % 4 == 0) && ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0);
        const int tm = (M + TN_BM - 1) / TN_BM, tiles = tm * ((N + TN_BN - 1) / TN_BN);
        hipLaunchKernelGGL(gemm_tn_x3_kernel, dim3((unsigned)(tiles * ks)), dim3(256), 0, s, (const float*)A,
                           (const float*)B, out, M, N, K, (long)lda, (long)ldb, ldo, kc, slice, vec4, tm, tiles,
                           (kinet_gemm_flags & 256) ? ks | 1 : ks);   // flag 256: no XCD placement
    } else if (dtype == KINET_F32_X3)   // flag 128: split at fragment-read time (the 16-deep kernel)
        hipLaunchKernelGGL((gemm_tn_kernel<float, true>), grid, dim3(256), 0, s, (const float*)A, (const float*)B, out, M, N, K,
                           (long)lda, (long)ldb, ldo, kc, slice);
    else if (dtype == KINET_BF16)
        hipLaunchKernelGGL((gemm_tn_kernel<bf16_t, false>), grid, dim3(256), 0, s, (const bf16_t*)A, (const bf16_t*)B, out, M, N,
                           K, (long)lda, (long)ldb, ldo, kc, slice);
    else if (dtype == KINET_F16)
        hipLaunchKernelGGL((gemm_tn_kernel<f16_t, false>), grid, dim3(256), 0, s, (const f16_t*)A, (const f16_t*)B, out, M, N,
                           K, (long)lda, (long)ldb, ldo, kc, slice);
    else {
        set_error("gemm_tn: unsupported dtype %d", dtype);
        return KINET_ERR_ARG;
    }
    KINET_LAUNCH_CHECK();
    if (!direct) {
        hipLaunchKernelGGL(tn_finalize_kernel, dim3(grid_for(slice)), dim3(256), 0, s, workspace, C, M, N, (long)ldc, ks,
                           accumulate);
        KINET_LAUNCH_CHECK();
    }
    return KINET_OK;
}

extern "C" int64_t kinet_colsum_workspace(int rows, int cols) {
    const int chunks = std::max(1, std::min(256, rows / 64));
    return (int64_t)chunks * cols;
}

extern "C" int kinet_colsum(const void* A, float* out, int rows, int cols, int64_t lda, int dtype, int accumulate,
                            float* workspace, kinet_stream_t stream) {
    KINET_CHECK_ARG(rows >= 0 && cols >= 0 && lda >= cols && workspace, "colsum: bad arguments");
    if (cols == 0) return KINET_OK;
    hipStream_t s = (hipStream_t)stream;
    const int chunks = (int)(kinet_colsum_workspace(rows, cols) / cols);
    const int rc = (rows + chunks - 1) / chunks;
    dim3 g1((cols + 255) / 256, chunks);
    if (dtype == KINET_F32 && cols % 4 == 0 && lda % 4 == 0 && ((uintptr_t)A & 15) == 0)
        hipLaunchKernelGGL(colsum_partial_vec_kernel, dim3((cols / 4 + 63) / 64, chunks), dim3(256), 0, s,
                           (const float*)A, workspace, rows, cols, (long)lda, rc);
    else if (dtype == KINET_F32) hipLaunchKernelGGL(colsum_partial_kernel<float>, g1, dim3(256), 0, s, (const float*)A, workspace, rows, cols, (long)lda, rc);
    else if (dtype == KINET_BF16) hipLaunchKernelGGL(colsum_partial_kernel<bf16_t>, g1, dim3(256), 0, s, (const bf16_t*)A, workspace, rows, cols, (long)lda, rc);
    else if (dtype == KINET_F16) hipLaunchKernelGGL(colsum_partial_kernel<f16_t>, g1, dim3(256), 0, s, (const f16_t*)A, workspace, rows, cols, (long)lda, rc);
    else { set_error("colsum: unsupported dtype %d", dtype); return KINET_ERR_ARG; }
    KINET_LAUNCH_CHECK();
    hipLaunchKernelGGL(colsum_final_kernel, dim3(cols), dim3(256), 0, s, workspace, out, cols, chunks, accumulate);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int64_t kinet_layernorm_backward_workspace(int rows, int d) {
    const int rpw = 16;
    const long long blocks = (rows + 4LL * rpw - 1) / (4LL * rpw);
    return 2 * std::max<long long>(1, blocks) * d;
}

extern "C" int kinet_layernorm_backward(const void* dy, const void* x, const float* gamma, void* dx, float* dgamma,
                                        float* dbeta, int rows, int d, float eps, int dtype, float* workspace,
                                        kinet_stream_t stream) {
    KINET_CHECK_ARG(d > 0 && d <= 1024 && rows >= 0 && workspace && gamma, "layernorm_backward: bad arguments");
    if (rows == 0) return KINET_OK;
    hipStream_t s = (hipStream_t)stream;
    const int rpw = 16;
    const int blocks = (rows + 4 * rpw - 1) / (4 * rpw);
    float* pg = workspace;
    float* pb = workspace + (long)blocks * d;
    const size_t lds = 8 * (size_t)d * sizeof(float);
    if (dtype == KINET_F32) hipLaunchKernelGGL(layernorm_bwd_kernel<float>, dim3(blocks), dim3(256), lds, s, (const float*)dy, (const float*)x, gamma, (float*)dx, pg, pb, rows, d, eps, rpw);
    else if (dtype == KINET_BF16) hipLaunchKernelGGL(layernorm_bwd_kernel<bf16_t>, dim3(blocks), dim3(256), lds, s, (const bf16_t*)dy, (const bf16_t*)x, gamma, (bf16_t*)dx, pg, pb, rows, d, eps, rpw);
    else if (dtype == KINET_F16) hipLaunchKernelGGL(layernorm_bwd_kernel<f16_t>, dim3(blocks), dim3(256), lds, s, (const f16_t*)dy, (const f16_t*)x, gamma, (f16_t*)dx, pg, pb, rows, d, eps, rpw);
    else { set_error("layernorm_backward: unsupported dtype %d", dtype); return KINET_ERR_ARG; }
    KINET_LAUNCH_CHECK();
    dim3 gf(d);
    if (dgamma) { hipLaunchKernelGGL(colsum_final_kernel, gf, dim3(256), 0, s, pg, dgamma, d, blocks, 0); KINET_LAUNCH_CHECK(); }
    if (dbeta) { hipLaunchKernelGGL(colsum_final_kernel, gf, dim3(256), 0, s, pb, dbeta, d, blocks, 0); KINET_LAUNCH_CHECK(); }
    return KINET_OK;
}

// 128-row blocks (up to 512 per image): at the config-4 input projections (2 x 16700 x 288) 260
// workgroups instead of 128 one-channel-per-thread loops over 261 rows
static int gn_blocks(int HW) { return std::max(1, std::min(512, HW / 128)); }

extern "C" int64_t kinet_groupnorm_backward_workspace(int N, int HW, int C, int groups) {
    const long long nb = gn_blocks(HW);
    return (long long)N * nb * 4 * C + (long long)N * groups * 4 + (long long)N * 2 * C;
}

extern "C" int kinet_groupnorm_backward(const void* dy, const void* x, const float* gamma, void* dx, float* dgamma,
                                        float* dbeta, int N, int HW, int C, int groups, float eps, int dtype,
                                        float* workspace, kinet_stream_t stream) {
    KINET_CHECK_ARG(N >= 0 && HW > 0 && C > 0 && groups > 0 && C % groups == 0 && workspace && gamma,
                    "groupnorm_backward: bad arguments");
    if (N == 0) return KINET_OK;
    hipStream_t s = (hipStream_t)stream;
    const int nb = gn_blocks(HW);
    const int rb = (HW + nb - 1) / nb;
    float* part = workspace;
    float* stats = part + (long)N * nb * 4 * C;
    float* chan = stats + (long)N * groups * 4;
    const long total = (long)N * HW * C;
    const bool vec = C % 4 == 0 && C <= 1024 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)dy % 16) == 0;
#define GN_BWD(T)                                                                                                  \
    if (vec)                                                                                                       \
        hipLaunchKernelGGL(gn_bwd_partial_vec_kernel<T>, dim3(nb, N), dim3(256), 0, s, (const T*)dy, (const T*)x, part, \
                           HW, C, rb);                                                                             \
    else                                                                                                           \
        hipLaunchKernelGGL(gn_bwd_partial_kernel<T>, dim3(nb, N), dim3(256), 0, s, (const T*)dy, (const T*)x, part, HW, \
                           C, rb);                                                                                 \
    KINET_LAUNCH_CHECK();                                                                                          \
    hipLaunchKernelGGL(gn_bwd_stats_kernel, dim3(N), dim3(1024), 4 * (size_t)C * sizeof(float), s, part, gamma, stats, \
                       chan, HW, C, groups, nb, eps);                                                              \
    KINET_LAUNCH_CHECK();                                                                                          \
    if (vec && total < (1L << 31) && ((uintptr_t)dx % 16) == 0)                                                 \
        hipLaunchKernelGGL(gn_bwd_apply_vec_kernel<T>, dim3(grid_for(total / 4)), dim3(256), 0, s, (const T*)dy,    \
                           (const T*)x, gamma, stats, (T*)dx, HW, C, groups, (int)(total / 4));                    \
    else                                                                                                           \
        hipLaunchKernelGGL(gn_bwd_apply_kernel<T>, dim3(grid_for(total)), dim3(256), 0, s, (const T*)dy, (const T*)x, \
                           gamma, stats, (T*)dx, HW, C, groups, total);                                            \
    KINET_LAUNCH_CHECK();
    if (dtype == KINET_F32) { GN_BWD(float) }
    else if (dtype == KINET_BF16) { GN_BWD(bf16_t) }
    else if (dtype == KINET_F16) { GN_BWD(f16_t) }
    else { set_error("groupnorm_backward: unsupported dtype %d", dtype); return KINET_ERR_ARG; }
#undef GN_BWD
    if (dgamma || dbeta) {
        hipLaunchKernelGGL(gn_bwd_param_kernel, dim3((C + 255) / 256), dim3(256), 0, s, chan, dgamma, dbeta, N, C);
        KINET_LAUNCH_CHECK();
    }
    return KINET_OK;
}

extern "C" int64_t kinet_mha_backward_workspace(int batch, int Lq, int Lk, int heads) {
    return 2LL * batch * heads * Lq * Lk;
}

extern "C" int kinet_mha_backward(const float* Q, int ldq, const float* K, int ldk, const float* V, int ldv,
                                  const float* dO, int ldo, float* dQ, float* dK, float* dV, int batch, int Lq, int Lk,
                                  int heads, int head_dim, float scale, const uint8_t* key_mask, float* workspace,
                                  float dropout_p, const int64_t* dropout_seed, kinet_stream_t stream) {
    KINET_CHECK_ARG(head_dim > 0 && head_dim <= ATT_MAXD && workspace, "mha_backward: head_dim %d (<= %d) / workspace",
                    head_dim, ATT_MAXD);
    KINET_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || dropout_seed),
                    "mha_backward: dropout p %g must be in [0, 1) with a seed", (double)dropout_p);
    if (batch == 0 || Lq == 0 || Lk == 0) return KINET_OK;
    const bool drop = dropout_p > 0.f;
    AttnArgs a{Q, K, V, dO, dQ, dK, dV, workspace, workspace + (long)batch * heads * Lq * Lk, key_mask,
               ldq, ldk, ldv, ldo, batch, Lq, Lk, heads, head_dim, scale, drop ? dropout_seed : nullptr,
               dropout_thresh(dropout_p), drop ? 1.f / (1.f - dropout_p) : 1.f};
    hipStream_t s = (hipStream_t)stream;
    const dim3 gq((Lq + AT_T - 1) / AT_T, batch * heads), gk((Lk + AT_T - 1) / AT_T, batch * heads);
#define AT2(MD_)                                                                  \
    do {                                                                          \
        hipLaunchKernelGGL(attn_bwd_q2_kernel<MD_>, gq, dim3(64 * at_nw<MD_>()), 0, s, a);      \
        KINET_LAUNCH_CHECK();                                                     \
        hipLaunchKernelGGL(attn_bwd_kv2_kernel<MD_>, gk, dim3(64 * at_nw<MD_>()), 0, s, a);     \
    } while (0)
    if (head_dim <= 32) AT2(32);
    else if (head_dim <= 36) AT2(36);
    else AT2(64);
#undef AT2
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}
