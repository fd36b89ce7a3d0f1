// Shared helpers for the kinet_amd HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
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

inline size_t dtype_size(int dt) {
    switch (dt) {
        case KINET_F32: return 4;
        case KINET_F64: return 8;
        case KINET_BF16: return 2;
        case KINET_F16: return 2;
        default: return 0;
    }
}

// number of workgroups that fill the chip for a grid-stride kernel (256 CUs x 8)
constexpr int kMaxGridStride = 2048;

}  // namespace kinet
