// Helpers shared by the MSDA sampling kernels (msda.hip, msda_enc.hip): 16-bit packed
// values accumulated in f32 by v_fma_mix_f32 (both multiplicands 16-bit sources, no
// separate widening instruction).
#pragma once
#include "common.h"

namespace kinet {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

// acc += f16(half of x) * f16(half of w) in f32 (both multiplicands 16-bit sources)
__device__ __forceinline__ float fma_mix16_lo_lo(float acc, uint32_t x, uint32_t w) {
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,1,0]" : "+v"(acc) : "v"(x), "v"(w));
    return acc;
}
__device__ __forceinline__ float fma_mix16_lo_hi(float acc, uint32_t x, uint32_t w) {
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,0]" : "+v"(acc) : "v"(x), "v"(w));
    return acc;
}
__device__ __forceinline__ float fma_mix16_hi_lo(float acc, uint32_t x, uint32_t w) {
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,0]" : "+v"(acc) : "v"(x), "v"(w));
    return acc;
}
__device__ __forceinline__ float fma_mix16_hi_hi(float acc, uint32_t x, uint32_t w) {
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,1,0]" : "+v"(acc) : "v"(x), "v"(w));
    return acc;
}
__device__ __forceinline__ uint32_t pack_f16x2(float a, float b) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (f16_t)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (f16_t)b) << 16);
}

}  // namespace kinet
