// Shared helpers for the kinet_amd HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>
#include <stdint.h>
#include <stdio.h>

#include "../../include/kinet_common.h"

namespace kinet {

// ---- error reporting (C-ABI returns an int status, the text is kept per thread) ----
void set_error(const char* fmt, ...);

#define KINET_CHECK_ARG(cond, ...)                    \
    do {                                              \
        if (!(cond)) {                                \
            ::kinet::set_error(__VA_ARGS__);          \
            return KINET_ERR_ARG;                     \
        }                                             \
    } while (0)

#define KINET_CHECK_HIP(expr)                                                        \
    do {                                                                             \
        hipError_t e_ = (expr);                                                      \
        if (e_ != hipSuccess) {                                                      \
            ::kinet::set_error("%s failed: %s", #expr, hipGetErrorString(e_));       \
            return KINET_ERR_HIP;                                                    \
        }                                                                            \
    } while (0)

#define KINET_LAUNCH_CHECK()                                                         \
    do {                                                                             \
        hipError_t e_ = hipGetLastError();                                           \
        if (e_ != hipSuccess) {                                                      \
            ::kinet::set_error("kernel launch failed: %s", hipGetErrorString(e_));   \
            return KINET_ERR_HIP;                                                    \
        }                                                                            \
    } while (0)

// ---- storage types ----
struct bf16_t { uint16_t x; };
typedef _Float16 f16_t;

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(double v) { return (float)v; }
__device__ __forceinline__ float to_f32(f16_t v) { return (float)v; }
__device__ __forceinline__ float to_f32(bf16_t v) { return __uint_as_float(((uint32_t)v.x) << 16); }

// round-to-nearest-even, NaN stays NaN: a plain __bf16 cast lowers to v_cvt_pk_bf16_f32
// (MI355X_MICROARCH "Correctness boundaries"), branch-free.
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
    bf16_t r;
    r.x = __builtin_bit_cast(uint16_t, (__bf16)f);
    return r;
}

// VEC elements of T as one aligned vector (16-byte loads / stores)
template <typename T, int VEC>
struct alignas(sizeof(T) * VEC) VecT {
    T v[VEC];
};

template <typename T> struct Cvt;
template <> struct Cvt<float> {
    __device__ static float from(float v) { return v; }
};
template <> struct Cvt<double> {
    __device__ static double from(double v) { return v; }
};
template <> struct Cvt<f16_t> {
    __device__ static f16_t from(float v) { return (f16_t)v; }
};
template <> struct Cvt<bf16_t> {
    __device__ static bf16_t from(float v) { return f32_to_bf16(v); }
};

// accumulator type: f64 stays f64 (reference fp64 path, test_double_precision.py), else f32
template <typename T> struct Acc { typedef float type; };
template <> struct Acc<double> { typedef double type; };

__device__ __forceinline__ double to_acc(double v, double*) { return v; }
template <typename T> __device__ __forceinline__ float to_acc(T v, float*) { return to_f32(v); }

// N explicit wait states pinned between two scheduling barriers.  ROCm 7.2's hazard recognizer
// searches an MFMA result window backwards with ONE visited set shared by all predecessor
// paths, so a window that reaches its reader through a control-flow merge or a loop back edge
// is padded for whichever path it walks first, not the shortest one (a 3-block reproducer and
// the scan of this library: tools/mfma_hazard_check.py).  Placed after the
// last MFMA a loop iteration issues, it covers the back edge.
template <int N>
__device__ __forceinline__ void mfma_window_pad() {
    static_assert(N >= 1 && N <= 16, "s_nop takes 1..16 wait states");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop %0" ::"i"(N - 1));
    __builtin_amdgcn_sched_barrier(0);
}

// launch-fill policy (kinet_set_solo_launch, defined in gemm.hip): 1 = one batch in flight, so
// launches size their tiles to fill the chip on their own; 0 = throughput mode (default)
extern int kinet_solo_launch;

// compute units of the current device (read once; 256 on MI355X) -- launchers size their
// grids in rounds of one workgroup per CU
inline int cu_count() {
    static int n = 0;
    if (n == 0) {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 256;
        n = c;
    }
    return n;
}

inline size_t dtype_size(int dt) {
    switch (dt) {
        case KINET_F32: return 4;
        case KINET_F32_X3: return 4;
        case KINET_F64: return 8;
        case KINET_BF16: return 2;
        case KINET_F16: return 2;
        default: return 0;
    }
}

// max / sum over each aligned group of G lanes (G = 2..64), result in every lane: DPP
// butterflies inside a 16-lane row (quad_perm xor1, xor2, half-mirror, mirror -- each pairs
// lanes of the two halves of the previous group), cross-row steps by swizzle / bpermute.
template <bool MAX>
__device__ __forceinline__ float combine(float a, float b) { return MAX ? fmaxf(a, b) : a + b; }

template <int G, bool MAX>
__device__ __forceinline__ float group_reduce(float x) {
    static_assert(G >= 1 && G <= 64 && (G & (G - 1)) == 0, "group size");
    auto dpp = [](float v, auto ctrl) {
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), decltype(ctrl)::value, 0xf, 0xf, false));
    };
    if constexpr (G >= 2) x = combine<MAX>(x, dpp(x, std::integral_constant<int, 0xB1>{}));    // quad_perm [1,0,3,2]
    if constexpr (G >= 4) x = combine<MAX>(x, dpp(x, std::integral_constant<int, 0x4E>{}));    // quad_perm [2,3,0,1]
    if constexpr (G >= 8) x = combine<MAX>(x, dpp(x, std::integral_constant<int, 0x141>{}));   // row_half_mirror
    if constexpr (G >= 16) x = combine<MAX>(x, dpp(x, std::integral_constant<int, 0x140>{}));  // row_mirror
    if constexpr (G >= 32) x = combine<MAX>(x, __shfl_xor(x, 16));
    if constexpr (G >= 64) x = combine<MAX>(x, __shfl_xor(x, 32));
    return x;
}

// number of workgroups that fill the chip for a grid-stride kernel (256 CUs x 8)
constexpr int kMaxGridStride = 2048;

// Attention-probability dropout (nn.MultiheadAttention(dropout=p), deformable_transformer.py:345;
// torch applies F.dropout to the softmax output): the keep decision of element
// idx = ((b*H + h)*Lq + i)*Lk + j is a counter-based hash of (seed, idx) -- the splitmix64
// finaliser, its top 24 bits the uniform draw u; kept iff u >= thresh, thresh = round(p * 2^24),
// kept values scaled by 1 / (1 - p).  Forward, backward and kinet_dropout_mask regenerate the
// same mask from the same seed (a device int64 drawn from torch's CUDA generator).
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint64_t idx, uint32_t thresh) {
    uint64_t z = seed + idx * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 40) >= thresh;
}
inline uint32_t dropout_thresh(float p) {
    const double t = (double)p * 16777216.0 + 0.5;
    return t >= 16777216.0 ? 16777216u : (t <= 0.0 ? 0u : (uint32_t)t);
}

}  // namespace kinet
