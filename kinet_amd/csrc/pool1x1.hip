// ResNet stage-1 entry for gfx950: torchvision's maxpool (3x3 / 2, pad 1) and the two 1x1 convs
// that read its output -- layer1[0].conv1 (64 -> 64, + bn1 + ReLU) and layer1[0].downsample
// (64 -> 256, + BN) -- in ONE launch (backbone.py:94-108 builds these from torchvision's
// resnet50 / 101).  The pooled map (137 MB at batch 16) is never written and the two convs do
// not each re-read it:
//  * a persistent workgroup (4 waves) walks tiles of 64 consecutive pooled pixels; per tile,
//    thread items (pixel, 16-byte channel chunk) take the 3x3 window max from the conv map and
//    park the pooled tile in LDS in the MFMA operand layout (chunks XOR-swizzled by pixel);
//  * the 320 output channels (64 conv1 | 256 downsample) are 20 MFMA column tiles; wave w owns
//    tiles w, w+4, .. and keeps their weights (K = 64: 2 K-steps) as A fragments in registers
//    for the whole launch: out^T(channels x pixels) = W x^T;
//  * epilogue: folded BN (+ ReLU on the conv1 half), the 16-bit tile parked in LDS and written
//    as whole pixel rows (128 B of conv1, 512 B of downsample) by 16-byte stores.
#include <hip/hip_runtime.h>

#include "../../include/kinet_gemm.h"
#include "common.h"
#include "gemm_common.h"

namespace kinet {
namespace {

constexpr int PD_PX = 64;              // pooled pixels per tile
constexpr int PD_C = 64;               // conv-map channels (= K)
constexpr int PD_N1 = 64, PD_N2 = 256, PD_N = PD_N1 + PD_N2;
constexpr int PD_NT = PD_N / 16;       // 20 column tiles
constexpr int PD_NTW = PD_NT / 4;      // 5 per wave

struct PoolDualArgs {
    const void* X;        // conv map (N, Ho, Wo, 64)
    const void* W;        // (320, 64): conv1 rows then downsample rows
    const float* scale;   // (320) folded BN
    const float* bias;
    void* T1;             // (N, Hp, Wp, 64)
    void* ID;             // (N, Hp, Wp, 256)
    int N, Ho, Wo, Hp, Wp;
    int x_bytes, t1_bytes, id_bytes;
};

template <typename T>
__global__ __launch_bounds__(256, 2) void pool_dual_kernel(const PoolDualArgs p, const int ntiles) {
    __shared__ __attribute__((aligned(16))) char xs[PD_PX * PD_C * 2];        // 8 KiB pooled tile
    __shared__ __attribute__((aligned(16))) char park[PD_PX * PD_N * 2];      // 40 KiB output tile
    __shared__ float par[2][PD_N];
    constexpr unsigned OOB = 0x80000000u;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, l16 = lane & 15;
    for (int i = tid; i < PD_N; i += 256) {
        par[0][i] = p.scale[i];
        par[1][i] = p.bias[i];
    }
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.X, (short)0, p.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.W, (short)0, PD_N * PD_C * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(p.T1, (short)0, p.t1_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(p.ID, (short)0, p.id_bytes, 0x00020000);
    u32x4 wf[PD_NTW][2];
#pragma unroll
    for (int j = 0; j < PD_NTW; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int n = (j * 4 + wave) * 16 + l16;
            wf[j][ks] = __builtin_amdgcn_raw_buffer_load_b128(rw, (unsigned)(n * PD_C + 32 * ks + 8 * g) * 2u, 0, 0);
        }
    const int M = p.N * p.Hp * p.Wp;
    __syncthreads();
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        // ---- pool: items (pixel, chunk) ----
#pragma unroll
        for (int it = 0; it < PD_PX * 8 / 256; ++it) {
            const int item = it * 256 + tid;
            const int px = item >> 3, c16 = item & 7;
            const int m = t * PD_PX + px;
            const int mm = m < M ? m : M - 1;
            const int pw = mm % p.Wp, rest = mm / p.Wp;
            const int ph = rest % p.Hp, n = rest / p.Hp;
            float mx[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) mx[e] = -INFINITY;
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                const int ih = 2 * ph - 1 + dy;
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    const int iw = 2 * pw - 1 + dx;
                    const bool ok = (unsigned)ih < (unsigned)p.Ho && (unsigned)iw < (unsigned)p.Wo;
                    const unsigned off = ok ? ((unsigned)((n * p.Ho + ih) * p.Wo + iw) * PD_C + c16 * 8) * 2u : OOB;
                    const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
                    if (ok) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            mx[2 * e] = fmaxf(mx[2 * e], to_f32(__builtin_bit_cast(T, (uint16_t)(v[e] & 0xffffu))));
                            mx[2 * e + 1] = fmaxf(mx[2 * e + 1], to_f32(__builtin_bit_cast(T, (uint16_t)(v[e] >> 16))));
                        }
                    }
                }
            }
            u32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                o[e] = (uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(mx[2 * e])) |
                       ((uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(mx[2 * e + 1])) << 16);
            *reinterpret_cast<u32x4*>(xs + px * 128 + ((c16 ^ (px & 7)) << 4)) = o;
        }
        __syncthreads();
        // ---- out^T = W x^T: lane holds channels 16 nt + 4 g + i of pixel 16 q + l16 ----
        f32x4 acc[PD_NTW][4];
#pragma unroll
        for (int j = 0; j < PD_NTW; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[j][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int px = 16 * q + l16;
                const u32x4 b = *reinterpret_cast<const u32x4*>(xs + px * 128 + (((4 * ks + g) ^ (px & 7)) << 4));
#pragma unroll
                for (int j = 0; j < PD_NTW; ++j) Mma<T>::run(acc[j][q], wf[j][ks], b);
            }
        // ---- BN (+ ReLU on conv1), park [pixel][320 channels], chunks XOR-swizzled by pixel ----
#pragma unroll
        for (int j = 0; j < PD_NTW; ++j) {
            const int n0 = (j * 4 + wave) * 16 + 4 * g;
            const f32x4 sc = *reinterpret_cast<const f32x4*>(&par[0][n0]);
            const f32x4 bi = *reinterpret_cast<const f32x4*>(&par[1][n0]);
            const bool relu = n0 < PD_N1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int px = 16 * q + l16;
                float v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    v[i] = acc[j][q][i] * sc[i] + bi[i];
                    if (relu) v[i] = fmaxf(v[i], 0.f);
                }
                uint32_t w[2];
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    w[i] = (uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(v[2 * i])) |
                           ((uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(v[2 * i + 1])) << 16);
                uint32_t* dst = reinterpret_cast<uint32_t*>(park + px * (PD_N * 2) + (((n0 >> 3) ^ (px & 7)) << 4) + (n0 & 4) * 2);
                dst[0] = w[0];
                dst[1] = w[1];
            }
        }
        __syncthreads();
        // ---- whole pixel rows: 8 chunks of conv1, 32 of downsample per pixel ----
#pragma unroll
        for (int it = 0; it < PD_PX * (PD_N / 8) / 256; ++it) {
            const int item = it * 256 + tid;
            const int px = item / (PD_N / 8), c = item - px * (PD_N / 8);
            const int m = t * PD_PX + px;
            const u32x4 v = *reinterpret_cast<const u32x4*>(park + px * (PD_N * 2) + ((c ^ (px & 7)) << 4));
            if (c < PD_N1 / 8)
                __builtin_amdgcn_raw_buffer_store_b128(v, r1, m < M ? ((unsigned)m * PD_N1 + c * 8) * 2u : OOB, 0, 0);
            else
                __builtin_amdgcn_raw_buffer_store_b128(v, r2, m < M ? ((unsigned)m * PD_N2 + (c - PD_N1 / 8) * 8) * 2u : OOB, 0, 0);
        }
        __syncthreads();
    }
}

}  // namespace
}  // namespace kinet

using namespace kinet;

// torchvision maxpool (3x3 / 2, pad 1) + layer1[0].conv1 / bn1 / relu + layer1[0].downsample in
// one launch -- include/kinet_gemm.h
extern "C" int kinet_pool_conv1x1_pair(const void* X, const void* W, const float* scale, const float* bias, void* T1,
                                       void* ID, int N, int Ho, int Wo, int dtype, kinet_stream_t stream) {
    KINET_CHECK_ARG(N >= 0 && Ho > 0 && Wo > 0, "pool_conv1x1_pair: bad geometry");
    KINET_CHECK_ARG(dtype == KINET_BF16 || dtype == KINET_F16, "pool_conv1x1_pair: dtype must be bf16 or f16");
    KINET_CHECK_ARG(X && W && scale && bias && T1 && ID, "pool_conv1x1_pair: NULL argument");
    KINET_CHECK_ARG((((uintptr_t)X) & 15u) == 0 && (((uintptr_t)W) & 15u) == 0 && (((uintptr_t)T1) & 15u) == 0 &&
                        (((uintptr_t)ID) & 15u) == 0 && (((uintptr_t)scale) & 15u) == 0 && (((uintptr_t)bias) & 15u) == 0,
                    "pool_conv1x1_pair: tensors must be 16-byte aligned");
    if (N == 0) return KINET_OK;
    PoolDualArgs a{};
    a.X = X; a.W = W; a.scale = scale; a.bias = bias; a.T1 = T1; a.ID = ID;
    a.N = N; a.Ho = Ho; a.Wo = Wo; a.Hp = (Ho - 1) / 2 + 1; a.Wp = (Wo - 1) / 2 + 1;
    const long long xb = (long long)N * Ho * Wo * PD_C * 2, M = (long long)N * a.Hp * a.Wp;
    KINET_CHECK_ARG(xb < (1LL << 31) && M * PD_N2 * 2 < (1LL << 31), "pool_conv1x1_pair: tensors larger than 2 GiB (split the call)");
    a.x_bytes = (int)xb;
    a.t1_bytes = (int)(M * PD_N1 * 2);
    a.id_bytes = (int)(M * PD_N2 * 2);
    const long long nt = (M + PD_PX - 1) / PD_PX;
    const int grid = nt < 2 * cu_count() ? (int)nt : 2 * cu_count();
    hipStream_t s = (hipStream_t)stream;
    if (dtype == KINET_BF16)
        hipLaunchKernelGGL((pool_dual_kernel<bf16_t>), dim3(grid), dim3(256), 0, s, a, (int)nt);
    else
        hipLaunchKernelGGL((pool_dual_kernel<f16_t>), dim3(grid), dim3(256), 0, s, a, (int)nt);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}
