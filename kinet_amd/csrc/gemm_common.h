// Shared pieces of the GEMM kernels (gemm.hip, gemm_rw.hip): operand vector types, the
// argument block, the MFMA wrappers, 4-wide output I/O, the 128-byte-row LDS swizzle and
// the 16-byte LDS-DMA helper.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.h"

namespace kinet {

struct GemmArgs {
    const void* A;
    const void* A2;        // optional: A + A2 elementwise (same layout as A)
    const void* B;
    void* C;
    const void* R;
    const float* scale;
    const float* bias;
    const float* ln_g;     // LayerNorm over the row (requires N <= BN)
    const float* ln_b;
    const uint8_t* row_mask;
    float ln_eps;
    int a_bytes, b_bytes;   // buffer-descriptor extents (bytes, < 2^31)
    int r_bytes;            // residual extent (gemm_rw.hip stages R by LDS-DMA)
    int c_bytes;            // output extent (gemm_rw.hip writes C by buffer stores)
    // head-major store (hm_rows > 0): row r = b*hm_rows + s, column n = g*hm_d + d goes to
    // C[((g*hm_batch + b)*hm_rows + s)*hm_d + d]  -- the MSDA value layout (heads, B, S, D)
    int hm_rows, hm_d, hm_batch;
    int M, N, K, lda, ldb, ldc, ldr, relu;
    // split-K (gemm_kernel only): blockIdx.y = K slice of kchunk elements, whose f32 partial
    // tile goes to C + blockIdx.y * c_slice (no epilogue; splitk_finalize applies it)
    int kchunk;
    long c_slice;
    // first output row of this launch's tile grid (gemm_kernel / gemm_dma_kernel): a problem
    // split into a full-rounds launch and a remainder launch runs the same M and strides
    int m_begin;
    int Hin, Win, Cin, Hout, Wout, KW, stride, pad;
    int stride_w, pad_w;   // horizontal stride / padding (== stride / pad for square convs)
};

// gemm_rw.hip: resident-weight streaming GEMM; false = problem not eligible
bool launch_rw(const GemmArgs& a, int in_dtype, int out_dtype, hipStream_t stream);
// gemm_rw.hip: the tap-folded stem convolution (conv-row gather); false = not eligible
bool launch_rw_conv(const GemmArgs& a, int in_dtype, hipStream_t stream);
// stem.hip: the tap-folded ResNet stem convolution (7x1, strides (2, 1), 24 -> 64 channels)
// with its input rows shared through LDS; false = not that geometry
bool launch_stem_conv(const GemmArgs& a, int dtype, hipStream_t stream);
extern int rw_min_m;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));


template <typename T> struct Mma;
template <> struct Mma<bf16_t> {
    static constexpr int EPC = 8;
    __device__ __forceinline__ static void run(f32x4& c, const u32x4& a, const u32x4& b) {
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
    __device__ __forceinline__ static u32x4 add(const u32x4& x, const u32x4& y) {
        u32x4 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float lo = __uint_as_float(x[i] << 16) + __uint_as_float(y[i] << 16);
            const float hi = __uint_as_float(x[i] & 0xffff0000u) + __uint_as_float(y[i] & 0xffff0000u);
            r[i] = (uint32_t)f32_to_bf16(lo).x | ((uint32_t)f32_to_bf16(hi).x << 16);
        }
        return r;
    }
};
template <> struct Mma<f16_t> {
    static constexpr int EPC = 8;
    __device__ __forceinline__ static void run(f32x4& c, const u32x4& a, const u32x4& b) {
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    }
    __device__ __forceinline__ static u32x4 add(const u32x4& x, const u32x4& y) {
        return __builtin_bit_cast(u32x4, __builtin_bit_cast(f16x8, x) + __builtin_bit_cast(f16x8, y));
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
    __device__ __forceinline__ static u32x4 add(const u32x4& x, const u32x4& y) {
        return __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, x) + __builtin_bit_cast(f32x4, y));
    }
};

template <typename TO> struct IO4;
template <> struct IO4<float> {
    __device__ static void store(float* p, const float* v) { *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]}; }
    __device__ static void load(const float* p, float* v) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(p);
        v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
    }
    __device__ static void store1(float* p, float v) { *p = v; }
    __device__ static float load1(const float* p) { return *p; }
};
template <> struct IO4<bf16_t> {
    __device__ static void store(bf16_t* p, const float* v) {
        uint2 u;
        u.x = (uint32_t)f32_to_bf16(v[0]).x | ((uint32_t)f32_to_bf16(v[1]).x << 16);
        u.y = (uint32_t)f32_to_bf16(v[2]).x | ((uint32_t)f32_to_bf16(v[3]).x << 16);
        *reinterpret_cast<uint2*>(p) = u;
    }
    __device__ static void load(const bf16_t* p, float* v) {
        const uint2 u = *reinterpret_cast<const uint2*>(p);
        v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
        v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
    }
    __device__ static void store1(bf16_t* p, float v) { *p = f32_to_bf16(v); }
    __device__ static float load1(const bf16_t* p) { return to_f32(*p); }
};
template <> struct IO4<f16_t> {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    __device__ static void store(f16_t* p, const float* v) {
        *reinterpret_cast<h4*>(p) = h4{(f16_t)v[0], (f16_t)v[1], (f16_t)v[2], (f16_t)v[3]};
    }
    __device__ static void load(const f16_t* p, float* v) {
        const h4 x = *reinterpret_cast<const h4*>(p);
        v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
    }
    __device__ static void store1(f16_t* p, float v) { *p = (f16_t)v; }
    __device__ static float load1(const f16_t* p) { return (float)*p; }
};

constexpr int ROWB = 128;   // bytes of K per LDS row per K-step

__device__ __forceinline__ int swz(int r, int c) { return r * ROWB + ((c ^ (r & 7)) << 4); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// one 16-byte-per-lane LDS-DMA: LDS[dst + 16*lane] = buffer[off] (zeros if off is out of
// range).  Kept out of the kernel templates: hipcc (ROCm 7.2) drops the host launch stub
// of a kernel template whose body calls the builtin directly.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* dst, unsigned off) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)dst, 16, off, 0, 0, 0);
}

}  // namespace
}  // namespace kinet
