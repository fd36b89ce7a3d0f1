// Decoder query self-attention core on MFMA (gfx950): O = softmax(scale * Q K^T + mask) V per
// (frame, head), head_dim 32, up to 384 keys, bf16 / f16 -- nn.MultiheadAttention inside
// DeformableTransformerDecoderLayer (deformable_transformer.py:367-372), a few hundred object +
// track queries attending to each other.
//
// One workgroup = 64 queries of one (frame, head), 4 waves x 16 queries.  The head's keys
// (row-major, 80-byte rows: conflict-free fragment reads) and values (TRANSPOSED, d-major) are
// staged once in LDS.  Per 32-key block a wave computes S^T = K Q^T (two 16x16x32 MFMAs, the
// head dim is one K-step), so each lane holds 8 scores of ONE query (lane & 15): the online
// softmax needs only in-lane math + two cross-lane steps, the exp(m_old - m_new) rescale is
// per lane, and the 8 probabilities rounded to the 16-bit type ARE the B operand of
// O^T += V^T P^T (K-slot order {4g..4g+3, 16+4g..16+4g+3}, matched by the two 8-byte reads of
// the transposed values).  Fully masked queries give 0, as the FMA kernel in ops.hip.
#include <hip/hip_runtime.h>

#include "../../include/kinet_ops.h"
#include "common.h"
#include "gemm_common.h"

namespace kinet {
namespace {

constexpr int AT_D = 32;
constexpr int AT_MAXK = 384;
constexpr int AT_KROW = 40;   // elements per staged key row (80 bytes)

template <typename T>
__global__ __launch_bounds__(256) void mha_mfma_kernel(const T* __restrict__ Q, int ldq, const T* __restrict__ Kt,
                                                       int ldk, const T* __restrict__ V, int ldv, T* __restrict__ O,
                                                       int ldo, int Lq, int Lk, float scale,
                                                       const uint8_t* __restrict__ kmask) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int Lkp = (Lk + 31) & ~31;
    const int vld = Lkp + 8;                                   // transposed value row (elements)
    T* ks = reinterpret_cast<T*>(smem);                        // [Lkp][AT_KROW]
    T* vt = ks + Lkp * AT_KROW;                                // [AT_D][vld]
    float* kb = reinterpret_cast<float*>(vt + AT_D * vld);     // [Lkp] additive mask
    const int b = blockIdx.z, h = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, c16 = lane & 15;

    // stage keys / transposed values / key bias (keys past Lk: zero rows, -inf bias)
    for (int i = tid; i < Lkp * 4; i += 256) {
        const int k = i >> 2, part = i & 3;
        u32x4 kv = u32x4{0u, 0u, 0u, 0u}, vv = u32x4{0u, 0u, 0u, 0u};
        if (k < Lk) {
            kv = *reinterpret_cast<const u32x4*>(Kt + ((long)b * Lk + k) * ldk + h * AT_D + part * 8);
            vv = *reinterpret_cast<const u32x4*>(V + ((long)b * Lk + k) * ldv + h * AT_D + part * 8);
        }
        *reinterpret_cast<u32x4*>(ks + k * AT_KROW + part * 8) = kv;
        const T* ve = reinterpret_cast<const T*>(&vv);
#pragma unroll
        for (int j = 0; j < 8; ++j) vt[(part * 8 + j) * vld + k] = ve[j];
    }
    for (int k = tid; k < Lkp; k += 256)
        kb[k] = (k < Lk && !(kmask && kmask[(long)b * Lk + k])) ? 0.f : -INFINITY;

    // this wave's 16 queries as the B operand of S^T: lane holds query c16, dims 8g .. 8g+7
    const int q = blockIdx.x * 64 + wave * 16 + c16;
    const bool qok = q < Lq;
    u32x4 qf = u32x4{0u, 0u, 0u, 0u};
    if (qok) qf = *reinterpret_cast<const u32x4*>(Q + ((long)b * Lq + q) * ldq + h * AT_D + 8 * g);
    __syncthreads();

    f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};   // O^T[d = 16t + 4g + i][query c16]
    float m = -INFINITY, l = 0.f;
    for (int k0 = 0; k0 < Lkp; k0 += 32) {
        const u32x4 ka = *reinterpret_cast<const u32x4*>(ks + (k0 + c16) * AT_KROW + 8 * g);
        const u32x4 kc = *reinterpret_cast<const u32x4*>(ks + (k0 + 16 + c16) * AT_KROW + 8 * g);
        f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
        Mma<T>::run(s0, ka, qf);   // S^T[key k0 + 4g + i][query c16]
        Mma<T>::run(s1, kc, qf);   // S^T[key k0 + 16 + 4g + i][query c16]
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(kb + k0 + 4 * g);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(kb + k0 + 16 + 4 * g);
        float sv[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            sv[i] = s0[i] * scale + b0[i];
            sv[4 + i] = s1[i] * scale + b1[i];
        }
        float bm = sv[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) bm = fmaxf(bm, sv[i]);
        bm = fmaxf(bm, __shfl_xor(bm, 16));
        bm = fmaxf(bm, __shfl_xor(bm, 32));
        const float mn = fmaxf(m, bm);
        const float alpha = mn == -INFINITY ? 1.f : __expf(m - mn);
        float p[8], ps = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            p[i] = mn == -INFINITY ? 0.f : __expf(sv[i] - mn);
            ps += p[i];
        }
        ps += __shfl_xor(ps, 16);
        ps += __shfl_xor(ps, 32);
        l = l * alpha + ps;
        m = mn;
        u32x4 pb;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            pb[i] = (uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(p[2 * i])) |
                    ((uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(p[2 * i + 1])) << 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o0[i] *= alpha;
            o1[i] *= alpha;
        }
        // A operand: V^T rows d = 16t + c16, K slots 8g + j -> keys k0 + 4g + j (j < 4) and
        // k0 + 16 + 4g + (j - 4): two 8-byte reads of the transposed values
        u32x4 va, vb;
        {
            const T* r0 = vt + c16 * vld + k0 + 4 * g;
            const T* r1 = vt + (16 + c16) * vld + k0 + 4 * g;
            const uint2 a0 = *reinterpret_cast<const uint2*>(r0), a1 = *reinterpret_cast<const uint2*>(r0 + 16);
            const uint2 c0 = *reinterpret_cast<const uint2*>(r1), c1 = *reinterpret_cast<const uint2*>(r1 + 16);
            va = u32x4{a0.x, a0.y, a1.x, a1.y};
            vb = u32x4{c0.x, c0.y, c1.x, c1.y};
        }
        Mma<T>::run(o0, va, pb);
        Mma<T>::run(o1, vb, pb);
        mfma_window_pad<2>();   // the next iteration's rescale reads o0 / o1 across the back edge
    }
    if (!qok) return;
    const float inv = l > 0.f ? 1.f / l : 0.f;
    T* orow = O + ((long)b * Lq + q) * ldo + h * AT_D + 4 * g;
    uint32_t w[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const f32x4& ot = t ? o1 : o0;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            w[i] = (uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(ot[2 * i] * inv)) |
                   ((uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(ot[2 * i + 1] * inv)) << 16);
        *reinterpret_cast<uint2*>(orow + 16 * t) = uint2{w[0], w[1]};
    }
}

// head_dim 36 (d = 288, configs 3-5: 500 object + track queries attending to each other): the
// same scheme with the head dim padded to two 32-deep K-steps for S^T = K Q^T (dims 36..63 zero
// in the staged keys and in the query fragments) and three 16-row tiles of O^T (V^T rows 36..47
// zero).  Keys in 72-element rows (144 B: 16 rows at one chunk hit 16 distinct bank groups), rows
// of 36 elements are 8-byte aligned only, so global reads / writes move 8-byte pieces.
constexpr int A36_D = 36, A36_DP = 64, A36_KROW = 72, A36_VT = 3, A36_MAXK = 640;

template <typename T>
__global__ __launch_bounds__(256) void mha_mfma36_kernel(const T* __restrict__ Q, int ldq, const T* __restrict__ Kt,
                                                         int ldk, const T* __restrict__ V, int ldv, T* __restrict__ O,
                                                         int ldo, int Lq, int Lk, float scale,
                                                         const uint8_t* __restrict__ kmask) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int Lkp = (Lk + 31) & ~31;
    const int vld = Lkp + 8;
    T* ks = reinterpret_cast<T*>(smem);                             // [Lkp][A36_KROW]
    T* vt = ks + Lkp * A36_KROW;                                    // [48][vld]
    float* kb = reinterpret_cast<float*>(vt + A36_VT * 16 * vld);   // [Lkp]
    const int b = blockIdx.z, h = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, c16 = lane & 15;

    // keys / transposed values: 9 8-byte pieces per row; pad dims 36..63 (keys) and rows 36..47
    // (values) with zeros; keys past Lk: zero rows, -inf bias
    for (int i = tid; i < Lkp * 9; i += 256) {
        const int k = i / 9, part = i - k * 9;
        uint2 kv = uint2{0u, 0u}, vv = uint2{0u, 0u};
        if (k < Lk) {
            kv = *reinterpret_cast<const uint2*>(Kt + ((long)b * Lk + k) * ldk + h * A36_D + part * 4);
            vv = *reinterpret_cast<const uint2*>(V + ((long)b * Lk + k) * ldv + h * A36_D + part * 4);
        }
        *reinterpret_cast<uint2*>(ks + k * A36_KROW + part * 4) = kv;
        const T* ve = reinterpret_cast<const T*>(&vv);
#pragma unroll
        for (int j = 0; j < 4; ++j) vt[(part * 4 + j) * vld + k] = ve[j];
    }
    for (int i = tid; i < Lkp * 7; i += 256) {   // key dims 36..63: 7 pieces of 4
        const int k = i / 7, part = i - k * 7;
        *reinterpret_cast<uint2*>(ks + k * A36_KROW + A36_D + part * 4) = uint2{0u, 0u};
    }
    for (int i = tid; i < (A36_VT * 16 - A36_D) * vld; i += 256) vt[A36_D * vld + i] = Cvt<T>::from(0.f);
    for (int k = tid; k < Lkp; k += 256)
        kb[k] = (k < Lk && !(kmask && kmask[(long)b * Lk + k])) ? 0.f : -INFINITY;

    // this wave's 16 queries as the B operand: lane holds query c16, dims 32s + 8g .. +7
    const int q = blockIdx.x * 64 + wave * 16 + c16;
    const bool qok = q < Lq;
    u32x4 qf0 = u32x4{0u, 0u, 0u, 0u}, qf1 = u32x4{0u, 0u, 0u, 0u};
    if (qok) {
        const T* qr = Q + ((long)b * Lq + q) * ldq + h * A36_D;
        const uint2 a = *reinterpret_cast<const uint2*>(qr + 8 * g), c = *reinterpret_cast<const uint2*>(qr + 8 * g + 4);
        qf0 = u32x4{a.x, a.y, c.x, c.y};
        if (g == 0) {
            const uint2 t = *reinterpret_cast<const uint2*>(qr + 32);
            qf1 = u32x4{t.x, t.y, 0u, 0u};
        }
    }
    __syncthreads();

    f32x4 o[A36_VT];   // O^T[d = 16t + 4g + i][query c16]
#pragma unroll
    for (int t = 0; t < A36_VT; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;
    for (int k0 = 0; k0 < Lkp; k0 += 32) {
        f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
        {
            const T* r0 = ks + (k0 + c16) * A36_KROW + 8 * g;
            const T* r1 = ks + (k0 + 16 + c16) * A36_KROW + 8 * g;
            Mma<T>::run(s0, *reinterpret_cast<const u32x4*>(r0), qf0);
            Mma<T>::run(s1, *reinterpret_cast<const u32x4*>(r1), qf0);
            Mma<T>::run(s0, *reinterpret_cast<const u32x4*>(r0 + 32), qf1);
            Mma<T>::run(s1, *reinterpret_cast<const u32x4*>(r1 + 32), qf1);
        }
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(kb + k0 + 4 * g);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(kb + k0 + 16 + 4 * g);
        float sv[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            sv[i] = s0[i] * scale + b0[i];
            sv[4 + i] = s1[i] * scale + b1[i];
        }
        float bm = sv[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) bm = fmaxf(bm, sv[i]);
        bm = fmaxf(bm, __shfl_xor(bm, 16));
        bm = fmaxf(bm, __shfl_xor(bm, 32));
        const float mn = fmaxf(m, bm);
        const float alpha = mn == -INFINITY ? 1.f : __expf(m - mn);
        float p[8], ps = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            p[i] = mn == -INFINITY ? 0.f : __expf(sv[i] - mn);
            ps += p[i];
        }
        ps += __shfl_xor(ps, 16);
        ps += __shfl_xor(ps, 32);
        l = l * alpha + ps;
        m = mn;
        u32x4 pb;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            pb[i] = (uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(p[2 * i])) |
                    ((uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(p[2 * i + 1])) << 16);
#pragma unroll
        for (int t = 0; t < A36_VT; ++t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) o[t][i] *= alpha;
            const T* r = vt + (16 * t + c16) * vld + k0 + 4 * g;
            const uint2 a0 = *reinterpret_cast<const uint2*>(r), a1 = *reinterpret_cast<const uint2*>(r + 16);
            Mma<T>::run(o[t], u32x4{a0.x, a0.y, a1.x, a1.y}, pb);
        }
    }
    if (!qok) return;
    const float inv = l > 0.f ? 1.f / l : 0.f;
    T* orow = O + ((long)b * Lq + q) * ldo + h * A36_D + 4 * g;
#pragma unroll
    for (int t = 0; t < A36_VT; ++t) {
        if (16 * t + 4 * g >= A36_D) continue;
        uint32_t w[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
            w[i] = (uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(o[t][2 * i] * inv)) |
                   ((uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(o[t][2 * i + 1] * inv)) << 16);
        *reinterpret_cast<uint2*>(orow + 16 * t) = uint2{w[0], w[1]};
    }
}

}  // namespace

// Entry from kinet_mha_core (ops.hip): false = not these kernels' cases (head_dim 32 with
// Lk <= 384 and 16-byte aligned rows, or head_dim 36 with Lk <= 640 and 8-byte aligned rows;
// 16-bit), which the FMA kernel then covers.
bool launch_mha_mfma(const void* Q, int ldq, const void* Kt, int ldk, const void* V, int ldv, void* O, int ldo,
                     int batch, int Lq, int Lk, int heads, int head_dim, float scale, int dtype,
                     const uint8_t* key_mask, hipStream_t stream) {
    if (head_dim == A36_D && (dtype == KINET_BF16 || dtype == KINET_F16) && Lk >= 1 && Lk <= A36_MAXK &&
        (ldq | ldk | ldv | ldo) % 4 == 0 && ((uintptr_t)Q | (uintptr_t)Kt | (uintptr_t)V | (uintptr_t)O) % 8 == 0 &&
        batch <= 65535 && heads <= 65535) {
        const int Lkp = (Lk + 31) & ~31;
        const size_t lds = (size_t)Lkp * A36_KROW * 2 + (size_t)A36_VT * 16 * (Lkp + 8) * 2 + (size_t)Lkp * 4;
        const dim3 grid((Lq + 63) / 64, heads, batch);
        if (dtype == KINET_BF16)
            hipLaunchKernelGGL((mha_mfma36_kernel<bf16_t>), grid, dim3(256), lds, stream, (const bf16_t*)Q, ldq,
                               (const bf16_t*)Kt, ldk, (const bf16_t*)V, ldv, (bf16_t*)O, ldo, Lq, Lk, scale, key_mask);
        else
            hipLaunchKernelGGL((mha_mfma36_kernel<f16_t>), grid, dim3(256), lds, stream, (const f16_t*)Q, ldq,
                               (const f16_t*)Kt, ldk, (const f16_t*)V, ldv, (f16_t*)O, ldo, Lq, Lk, scale, key_mask);
        return true;
    }
    if (head_dim != AT_D || (dtype != KINET_BF16 && dtype != KINET_F16) || Lk < 1 || Lk > AT_MAXK) return false;
    if ((ldq | ldk | ldv | ldo) % 8 != 0 || ((uintptr_t)Q | (uintptr_t)Kt | (uintptr_t)V | (uintptr_t)O) % 16 != 0)
        return false;
    if (batch > 65535 || heads > 65535) return false;
    const int Lkp = (Lk + 31) & ~31;
    const size_t lds = (size_t)Lkp * AT_KROW * 2 + (size_t)AT_D * (Lkp + 8) * 2 + (size_t)Lkp * 4;
    const dim3 grid((Lq + 63) / 64, heads, batch);
    if (dtype == KINET_BF16)
        hipLaunchKernelGGL((mha_mfma_kernel<bf16_t>), grid, dim3(256), lds, stream, (const bf16_t*)Q, ldq,
                           (const bf16_t*)Kt, ldk, (const bf16_t*)V, ldv, (bf16_t*)O, ldo, Lq, Lk, scale, key_mask);
    else
        hipLaunchKernelGGL((mha_mfma_kernel<f16_t>), grid, dim3(256), lds, stream, (const f16_t*)Q, ldq,
                           (const f16_t*)Kt, ldk, (const f16_t*)V, ldv, (f16_t*)O, ldo, Lq, Lk, scale, key_mask);
    return true;
}

}  // namespace kinet
