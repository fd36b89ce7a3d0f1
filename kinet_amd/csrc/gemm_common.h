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
    // A2 with a2_rows rows (0: M rows): row m adds A2 row m % a2_rows -- a per-frame operand shared
    // by every frame of the batch (the position embedding of unpadded equal-size frames)
    int a2_rows;
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
    // split head-major store (hm_split > 0): columns n >= hm_split go to a second plane after the
    // first, C + hm_split*hm_batch*hm_rows, as ((g*hm_batch + b)*hm_rows + s)*hm_d2 + d with
    // n - hm_split = g*hm_d2 + d -- the head_dim-36 MSDA value as a 32-channel plane + a 4-channel plane
    int hm_split, hm_d2;
    // 1 = the resident-weight kernel's 32-column head-major stores go through its LDS transpose
    // (gemm_rw.hip; set by launch_rw from kinet_gemm_flags, never by callers)
    int hm_tr;
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
    // MSDA sampling-record epilogue (gemm_rw.hip, kinet_msda_sample_records): reference
    // points (M rows x 4 levels x prep_refd f32), fixed-point fraction bits, level shapes
    const float* prep_ref;
    int prep_refd, prep_fb;
    int prep_H[4], prep_W[4];
};

// gemm_rw.hip: resident-weight streaming GEMM; false = problem not eligible
bool launch_rw(const GemmArgs& a, int in_dtype, int out_dtype, hipStream_t stream);
// gemm_rw.hip: the tap-folded stem convolution (conv-row gather); false = not eligible
bool launch_rw_conv(const GemmArgs& a, int in_dtype, hipStream_t stream);
// stem.hip: the tap-folded ResNet stem convolution (7x1, strides (2, 1), 24 -> 64 channels)
// with its input rows shared through LDS; false = not that geometry
bool launch_stem_conv(const GemmArgs& a, int dtype, hipStream_t stream);
// conv3x3.hip: the direct 3x3 stride-1 64 -> 64 channel convolution (ResNet layer-1 conv2),
// weights resident in VGPRs, input halo tiles in LDS; false = not that geometry
bool launch_conv3x3_c64(const GemmArgs& a, int dtype, hipStream_t stream);
extern thread_local int rw_min_m;
extern thread_local int kinet_gemm_flags;   // gemm.hip (diagnostic selection flags; 128 = the read-time-split KINET_F32_X3 TN kernel)

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));


// Fragment interface: the register-staged main loops pass every 16-byte chunk of K-contiguous
// elements through stage() on its way into LDS, read one u32x4 per lane and operand tile back,
// turn it into Mma<T>::Frag (frag) and feed the fragments to run().
template <typename T> struct Mma;
template <> struct Mma<bf16_t> {
    static constexpr int EPC = 8;
    typedef u32x4 Frag;
    __device__ __forceinline__ static Frag frag(const u32x4& x) { return x; }
    __device__ __forceinline__ static u32x4 stage(const u32x4& x) { return x; }
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
    typedef u32x4 Frag;
    __device__ __forceinline__ static Frag frag(const u32x4& x) { return x; }
    __device__ __forceinline__ static u32x4 stage(const u32x4& x) { return x; }
    __device__ __forceinline__ static void run(f32x4& c, const u32x4& a, const u32x4& b) {
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    }
    __device__ __forceinline__ static u32x4 add(const u32x4& x, const u32x4& y) {
        return __builtin_bit_cast(u32x4, __builtin_bit_cast(f16x8, x) + __builtin_bit_cast(f16x8, y));
    }
};
template <> struct Mma<float> {
    static constexpr int EPC = 4;
    typedef u32x4 Frag;
    __device__ __forceinline__ static Frag frag(const u32x4& x) { return x; }
    __device__ __forceinline__ static u32x4 stage(const u32x4& x) { return x; }
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

// f32 operands multiplied as three bf16 MFMA passes (KINET_F32_X3; torch's "high" float32
// matmul precision): x = hi + lo with hi = bf16(x) (round to nearest even) and lo =
// bf16(x - hi), a*b ~= hi_a*hi_b + hi_a*lo_b + lo_a*hi_b in f32 accumulation.  The dropped
// lo_a*lo_b term and the rounding of lo leave ~2^-17 relative error per product (exact f32
// MFMA: 2^-24; TF32: 2^-11) at 3 x 8 MFMA cycles per 16x16x16 block instead of 4 x 32 for
// v_mfma_f32_16x16x4_f32.  Same K layout as Mma<float> (4 consecutive k per lane = the
// A/B operand map of v_mfma_f32_16x16x16_bf16).
struct f32x3_t { float v; };
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
struct X3Frag { s16x4 hi, lo; };
__device__ __forceinline__ X3Frag split_x3(const f32x4& x) {
    const bf16x4v h = __builtin_convertvector(x, bf16x4v);
    const f32x4 r = x - __builtin_convertvector(h, f32x4);
    return X3Frag{__builtin_bit_cast(s16x4, h), __builtin_bit_cast(s16x4, __builtin_convertvector(r, bf16x4v))};
}
template <> struct Mma<f32x3_t> {
    static constexpr int EPC = 4;
    typedef X3Frag Frag;
    // split once per element on the way into LDS (not once per wave that reads it): the chunk
    // of 4 f32 becomes {hi of the 4 (8 bytes), lo of the 4 (8 bytes)} in the same 16 bytes
    __device__ __forceinline__ static u32x4 stage(const u32x4& x) {
        const X3Frag f = split_x3(__builtin_bit_cast(f32x4, x));
        const uint2 h = __builtin_bit_cast(uint2, f.hi), l = __builtin_bit_cast(uint2, f.lo);
        return u32x4{h.x, h.y, l.x, l.y};
    }
    __device__ __forceinline__ static Frag frag(const u32x4& x) {
        return X3Frag{__builtin_bit_cast(s16x4, uint2{x[0], x[1]}), __builtin_bit_cast(s16x4, uint2{x[2], x[3]})};
    }
    __device__ __forceinline__ static void run(f32x4& c, const Frag& a, const Frag& b) {
        c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a.lo, b.hi, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a.hi, b.lo, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a.hi, b.hi, c, 0, 0, 0);
    }
    __device__ __forceinline__ static u32x4 add(const u32x4& x, const u32x4& y) { return Mma<float>::add(x, y); }
    // the 16x16x32 form: a lane's 8 consecutive k = two staged chunks {hi4, lo4}
    __device__ __forceinline__ static void run32(f32x4& c, const u32x4& a0, const u32x4& a1, const u32x4& b0,
                                                 const u32x4& b1) {
        const bf16x8 ah = __builtin_bit_cast(bf16x8, u32x4{a0[0], a0[1], a1[0], a1[1]});
        const bf16x8 al = __builtin_bit_cast(bf16x8, u32x4{a0[2], a0[3], a1[2], a1[3]});
        const bf16x8 bh = __builtin_bit_cast(bf16x8, u32x4{b0[0], b0[1], b1[0], b1[1]});
        const bf16x8 bl = __builtin_bit_cast(bf16x8, u32x4{b0[2], b0[3], b1[2], b1[3]});
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
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
