// MFMA GEMM + implicit-GEMM NHWC convolution for gfx950 (CDNA4), fused epilogues.
//
// Tiling (DESIGN.md "GEMM / conv kernel"):
//  * workgroup = 256 threads = 4 waves in a 2 (M) x 2 (N) grid, output tile BM x BN
//    (128/64 each), one K-step = 128 bytes of K per row (64 bf16/f16 or 32 f32);
//  * operands staged global -> registers -> LDS, double-buffered LDS with ONE barrier
//    per K-step (next tile's global loads are in flight under the current MFMAs);
//  * LDS rows are 128 B with the 16-byte chunk index XOR-swizzled by (row & 7), which
//    makes the ds_read_b128 fragment reads (16 rows x one chunk per lane group)
//    bank-conflict free;
//  * the weight tile is the MFMA A operand and the activation tile the B operand, so
//    the 16x16 accumulator has the output row m on the lane and 4 consecutive output
//    channels n in registers -> 8/16-byte stores along the contiguous NHWC channel dim;
//  * blockIdx is remapped XCD-aware (bijective form, cdna_hip_programming.md T1) so the
//    tiles that share an activation panel run on one XCD and hit its L2;
//  * bf16/f16: v_mfma_f32_16x16x32_{bf16,f16}; f32 (parity mode): the exact-f32
//    v_mfma_f32_16x16x4_f32, 4 per 16-byte fragment.
//  * implicit conv: M = batch*Hout*Wout rows, K = KH*KW*Cin with Cin fastest (weights
//    permuted OIHW -> OHWI on the host); each 16-byte chunk lies inside one filter tap
//    (Cin % 8 == 0) so the im2col gather is a 16-byte load or a zero fill.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/kinet_gemm.h"
#include "common.h"

namespace kinet {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
    const void* A;
    const void* B;
    void* C;
    const void* R;
    const float* scale;
    const float* bias;
    const uint8_t* row_mask;
    int M, N, K, lda, ldb, ldc, ldr, relu;
    int Hin, Win, Cin, Hout, Wout, KW, stride, pad;
};

template <typename T> struct Mma;
template <> struct Mma<bf16_t> {
    static constexpr int EPC = 8;
    __device__ __forceinline__ static void run(f32x4& c, const u32x4& a, const u32x4& b) {
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
};
template <> struct Mma<f16_t> {
    static constexpr int EPC = 8;
    __device__ __forceinline__ static void run(f32x4& c, const u32x4& a, const u32x4& b) {
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    }
};
template <> struct Mma<float> {
    static constexpr int EPC = 4;
    // lanes hold 4 consecutive k of a 16-wide k block; MFMA j sums k = 4*(lane>>4) + j over
    // the 4 lane groups, so the 4 MFMAs together cover the block exactly once.
    __device__ __forceinline__ static void run(f32x4& c, const u32x4& a, const u32x4& b) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[j]), __uint_as_float(b[j]), c, 0, 0, 0);
    }
};

template <typename TO> struct Store4;
template <> struct Store4<float> {
    __device__ static void vec(float* p, const float* v) { *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]}; }
    __device__ static void one(float* p, float v) { *p = v; }
    __device__ static void load(const float* p, float* v) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(p);
        v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
    }
};
template <> struct Store4<bf16_t> {
    __device__ static void vec(bf16_t* p, const float* v) {
        uint2 u;
        u.x = (uint32_t)f32_to_bf16(v[0]).x | ((uint32_t)f32_to_bf16(v[1]).x << 16);
        u.y = (uint32_t)f32_to_bf16(v[2]).x | ((uint32_t)f32_to_bf16(v[3]).x << 16);
        *reinterpret_cast<uint2*>(p) = u;
    }
    __device__ static void one(bf16_t* p, float v) { *p = f32_to_bf16(v); }
    __device__ static void load(const bf16_t* p, float* v) {
        const uint2 u = *reinterpret_cast<const uint2*>(p);
        v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
        v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
    }
};
template <> struct Store4<f16_t> {
    __device__ static void vec(f16_t* p, const float* v) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<h4*>(p) = h4{(f16_t)v[0], (f16_t)v[1], (f16_t)v[2], (f16_t)v[3]};
    }
    __device__ static void one(f16_t* p, float v) { *p = (f16_t)v; }
    __device__ static void load(const f16_t* p, float* v) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        const h4 x = *reinterpret_cast<const h4*>(p);
        v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
    }
};

constexpr int ROWB = 128;   // bytes of K per LDS row per K-step

__device__ __forceinline__ int swz(int r, int c) { return r * ROWB + ((c ^ (r & 7)) << 4); }

template <typename T, typename TO, int BM, int BN, bool CONV>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const GemmArgs p, const int nNt) {
    constexpr int EPC = Mma<T>::EPC;
    constexpr int BK = ROWB / (int)sizeof(T);
    constexpr int XR = BM / 32;
    constexpr int WR = BN / 32;
    constexpr int TM = BM / 32;
    constexpr int TN = BN / 32;
    constexpr int STAGE = (BM + BN) * ROWB;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

    // XCD-aware bijective remap: consecutive logical tiles land on one XCD
    int bid = blockIdx.x;
    {
        const int nblk = gridDim.x, q = nblk >> 3, r = nblk & 7, xcd = bid & 7;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    }
    const int mt = bid / nNt, nt = bid - (bid / nNt) * nNt;
    const int m0 = mt * BM, n0 = nt * BN;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int sc = tid & 7, sr = tid >> 3;
    const int M = p.M, N = p.N, K = p.K;

    const T* __restrict__ A = (const T*)p.A;
    const T* __restrict__ B = (const T*)p.B;

    long xbase[XR];
    int xih[XR], xiw[XR];
    bool xok[XR];
#pragma unroll
    for (int i = 0; i < XR; ++i) {
        const int m = m0 + sr + 32 * i;
        xok[i] = m < M;
        if (CONV) {
            const int hw = p.Hout * p.Wout;
            const int img = m / hw;
            const int rem = m - img * hw;
            const int oh = rem / p.Wout, ow = rem - (rem / p.Wout) * p.Wout;
            xih[i] = oh * p.stride - p.pad;
            xiw[i] = ow * p.stride - p.pad;
            xbase[i] = (long)img * p.Hin * p.Win * p.Cin;
        } else {
            xih[i] = xiw[i] = 0;
            xbase[i] = (long)m * p.lda;
        }
    }

    u32x4 xs[XR], ws[WR];
    const u32x4 zero = {0u, 0u, 0u, 0u};

    auto load_tile = [&](int k0) {
        const int k = k0 + sc * EPC;
        const bool kok = k < K;
        int kh = 0, kw = 0, cc = k;
        if (CONV) {
            const int tap = k / p.Cin;
            cc = k - tap * p.Cin;
            kh = tap / p.KW;
            kw = tap - kh * p.KW;
        }
#pragma unroll
        for (int i = 0; i < XR; ++i) {
            bool ok = xok[i] && kok;
            const T* src;
            if (CONV) {
                const int ih = xih[i] + kh, iw = xiw[i] + kw;
                ok = ok && ih >= 0 && ih < p.Hin && iw >= 0 && iw < p.Win;
                src = A + xbase[i] + ((long)ih * p.Win + iw) * p.Cin + cc;
            } else {
                src = A + xbase[i] + k;
            }
            xs[i] = ok ? *reinterpret_cast<const u32x4*>(src) : zero;
        }
#pragma unroll
        for (int i = 0; i < WR; ++i) {
            const int n = n0 + sr + 32 * i;
            ws[i] = (n < N && kok) ? *reinterpret_cast<const u32x4*>(B + (long)n * p.ldb + k) : zero;
        }
    };
    auto store_tile = [&](int buf) {
        char* xl = lds + buf * STAGE;
        char* wl = xl + BM * ROWB;
#pragma unroll
        for (int i = 0; i < XR; ++i) *reinterpret_cast<u32x4*>(xl + swz(sr + 32 * i, sc)) = xs[i];
#pragma unroll
        for (int i = 0; i < WR; ++i) *reinterpret_cast<u32x4*>(wl + swz(sr + 32 * i, sc)) = ws[i];
    };

    f32x4 acc[TN][TM];
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = (K + BK - 1) / BK;
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_tile((kt + 1) * BK);
        const char* xl = lds + buf * STAGE;
        const char* wl = xl + BM * ROWB;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = kk * 4 + (lane >> 4);
            u32x4 bfr[TM], afr[TN];
#pragma unroll
            for (int t = 0; t < TM; ++t)
                bfr[t] = *reinterpret_cast<const u32x4*>(xl + swz(wm * (BM / 2) + t * 16 + (lane & 15), ch));
#pragma unroll
            for (int t = 0; t < TN; ++t)
                afr[t] = *reinterpret_cast<const u32x4*>(wl + swz(wn * (BN / 2) + t * 16 + (lane & 15), ch));
#pragma unroll
            for (int a = 0; a < TN; ++a)
#pragma unroll
                for (int b = 0; b < TM; ++b) Mma<T>::run(acc[a][b], afr[a], bfr[b]);
        }
        if (kt + 1 < nk) store_tile(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue: scale/bias (folded BN or Linear bias), residual, ReLU, row mask ----
    TO* __restrict__ C = (TO*)p.C;
    const TO* __restrict__ R = (const TO*)p.R;
    const bool vec_ok = ((p.ldc & 3) == 0) && (R == nullptr || (p.ldr & 3) == 0);
#pragma unroll
    for (int b = 0; b < TM; ++b) {
        const int m = m0 + wm * (BM / 2) + b * 16 + (lane & 15);
        if (m >= M) continue;
        const bool masked = p.row_mask != nullptr && p.row_mask[m] != 0;
#pragma unroll
        for (int a = 0; a < TN; ++a) {
            const int nb = n0 + wn * (BN / 2) + a * 16 + (lane >> 4) * 4;
            if (nb >= N) continue;
            float v[4] = {acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]};
            const bool full = vec_ok && nb + 3 < N;
            float res[4] = {0.f, 0.f, 0.f, 0.f};
            if (R) {
                if (full) Store4<TO>::load(R + (long)m * p.ldr + nb, res);
                else
                    for (int r = 0; r < 4; ++r)
                        if (nb + r < N) res[r] = to_f32(R[(long)m * p.ldr + nb + r]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = nb + r < N ? nb + r : N - 1;
                float x = v[r];
                if (p.scale) x *= p.scale[n];
                if (p.bias) x += p.bias[n];
                x += res[r];
                if (p.relu) x = fmaxf(x, 0.f);
                if (masked) x = 0.f;
                v[r] = x;
            }
            TO* dst = C + (long)m * p.ldc + nb;
            if (full) Store4<TO>::vec(dst, v);
            else
                for (int r = 0; r < 4; ++r)
                    if (nb + r < N) Store4<TO>::one(dst + r, v[r]);
        }
    }
}

template <typename T, typename TO, bool CONV>
int launch(const GemmArgs& a, hipStream_t stream) {
    if (a.M == 0 || a.N == 0) return KINET_OK;
    const int bn = a.N <= 64 ? 64 : 128;
    const long tiles128 = (long)((a.M + 127) / 128) * ((a.N + bn - 1) / bn);
    const int bm = tiles128 < 512 ? 64 : 128;
    const int nMt = (a.M + bm - 1) / bm, nNt = (a.N + bn - 1) / bn;
    const long nblk = (long)nMt * nNt;
    KINET_CHECK_ARG(nblk < (1L << 31), "gemm: too many tiles");
    dim3 grid((unsigned)nblk), block(256);
#define L_(BM_, BN_) hipLaunchKernelGGL((gemm_kernel<T, TO, BM_, BN_, CONV>), grid, block, 0, stream, a, nNt)
    if (bm == 128 && bn == 128) L_(128, 128);
    else if (bm == 128 && bn == 64) L_(128, 64);
    else if (bm == 64 && bn == 128) L_(64, 128);
    else L_(64, 64);
#undef L_
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

template <bool CONV>
int dispatch(const GemmArgs& a, int in_dtype, int out_dtype, hipStream_t s) {
    if (in_dtype == KINET_BF16 && out_dtype == KINET_BF16) return launch<bf16_t, bf16_t, CONV>(a, s);
    if (in_dtype == KINET_BF16 && out_dtype == KINET_F32) return launch<bf16_t, float, CONV>(a, s);
    if (in_dtype == KINET_F16 && out_dtype == KINET_F16) return launch<f16_t, f16_t, CONV>(a, s);
    if (in_dtype == KINET_F16 && out_dtype == KINET_F32) return launch<f16_t, float, CONV>(a, s);
    if (in_dtype == KINET_F32 && out_dtype == KINET_F32) return launch<float, float, CONV>(a, s);
    set_error("gemm: unsupported dtypes in=%d out=%d", in_dtype, out_dtype);
    return KINET_ERR_ARG;
}

bool aligned16(const void* p) { return (((uintptr_t)p) & 15u) == 0; }

}  // namespace
}  // namespace kinet

using namespace kinet;

extern "C" int kinet_gemm(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                          int in_dtype, const float* scale, const float* bias, const void* R, int ldr, int relu,
                          int out_dtype, const uint8_t* row_mask, int reserved, kinet_stream_t stream) {
    (void)reserved;
    KINET_CHECK_ARG(M >= 0 && N >= 0 && K > 0, "gemm: invalid sizes M=%d N=%d K=%d", M, N, K);
    KINET_CHECK_ARG(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0, "gemm: K, lda, ldb must be multiples of 8 (K=%d lda=%d ldb=%d)", K, lda, ldb);
    KINET_CHECK_ARG(lda >= K && ldb >= K && ldc >= N, "gemm: leading dims too small");
    KINET_CHECK_ARG(aligned16(A) && aligned16(B), "gemm: A and B must be 16-byte aligned");
    KINET_CHECK_ARG(R == nullptr || ldr >= N, "gemm: ldr < N");
    GemmArgs a{};
    a.A = A; a.B = B; a.C = C; a.R = R; a.scale = scale; a.bias = bias; a.row_mask = row_mask;
    a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.ldr = ldr; a.relu = relu;
    return dispatch<false>(a, in_dtype, out_dtype, (hipStream_t)stream);
}

extern "C" int kinet_conv2d(const void* X, const void* Wt, void* Y, int batch, int Hin, int Win, int Cin, int Hout,
                            int Wout, int Cout, int KH, int KW, int stride, int pad, int in_dtype, const float* scale,
                            const float* bias, const void* R, int ldr, int relu, int ldy, kinet_stream_t stream) {
    KINET_CHECK_ARG(batch >= 0 && Hin > 0 && Win > 0 && Cin > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0,
                    "conv2d: invalid geometry");
    KINET_CHECK_ARG(Cin % 8 == 0, "conv2d: Cin (%d) must be a multiple of 8 (pad channels)", Cin);
    KINET_CHECK_ARG(Hout == (Hin + 2 * pad - KH) / stride + 1 && Wout == (Win + 2 * pad - KW) / stride + 1,
                    "conv2d: output size mismatch");
    KINET_CHECK_ARG(ldy >= Cout && (R == nullptr || ldr >= Cout), "conv2d: ldy/ldr < Cout");
    KINET_CHECK_ARG(aligned16(X) && aligned16(Wt), "conv2d: X and W must be 16-byte aligned");
    const long M = (long)batch * Hout * Wout;
    KINET_CHECK_ARG(M < (1L << 31) && (long)batch * Hin * Win * Cin < (1L << 40), "conv2d: too large");
    GemmArgs a{};
    a.A = X; a.B = Wt; a.C = Y; a.R = R; a.scale = scale; a.bias = bias; a.row_mask = nullptr;
    a.M = (int)M; a.N = Cout; a.K = KH * KW * Cin; a.lda = 0; a.ldb = KH * KW * Cin; a.ldc = ldy; a.ldr = ldr;
    a.relu = relu;
    a.Hin = Hin; a.Win = Win; a.Cin = Cin; a.Hout = Hout; a.Wout = Wout; a.KW = KW; a.stride = stride; a.pad = pad;
    return dispatch<true>(a, in_dtype, in_dtype, (hipStream_t)stream);
}
