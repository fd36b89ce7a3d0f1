// Direct 3x3 stride-1 convolution, 64 -> 64 channels, NHWC, 16-bit, for gfx950: the ResNet
// layer-1 bottleneck conv2 (torchvision Bottleneck.conv2 of backbone.py:94-108, FrozenBN +
// ReLU folded into the epilogue).  Entered from gemm.hip's conv dispatcher (launch_conv3x3_c64).
//
// Why a dedicated kernel: as an implicit GEMM this shape has K = 576 = 9 K-steps per tile and
// N = 64, so every 128x64 tile pays a full pipeline fill, its own weight-tile loads and an
// LDS epilogue for 9 steps of MFMA work, and its nine shifted reads of each input row come
// through L2 separately (420-440 TF/s at batch 16, tools/conv_ab.py).  Here
//  * the weights never move: wave w keeps output channels [32 (w & 1), +32) x all 576 K as
//    MFMA A-fragments in 144 VGPRs for the whole (persistent) launch;
//  * a workgroup (8 waves, one per CU) walks output tiles of 8 rows x 32 columns of one
//    image; the tile's input HALO (10 x 34 pixels x 128 B, zeros outside the image = the
//    conv padding) is staged ONCE by LDS-DMA into a double buffer, issued a whole tile
//    ahead, and all 9 taps read it from LDS (16-byte chunks XOR-swizzled by pixel & 7, the
//    swizzle applied on the DMA source side);
//  * wave tile = 64 output pixels (2 rows x 32) x 32 channels: each 1-KiB activation
//    fragment feeds 2 v_mfma_f32_16x16x32 (half the LDS port at full MFMA rate);
//  * epilogue: folded BN scale / bias + ReLU in registers, the 16-bit tile parked in LDS,
//    then streamed as whole 128-byte pixel rows (4 KiB contiguous per tile row).
#include <hip/hip_runtime.h>

#include "common.h"
#include "gemm_common.h"

namespace kinet {
namespace {

constexpr int C3_TH = 8, C3_TW = 32;                         // output tile
constexpr int C3_HH = C3_TH + 2, C3_HW = C3_TW + 2;          // halo 10 x 34
constexpr int C3_HPIX = C3_HH * C3_HW;                       // 340 pixels
constexpr int C3_WAVES = 8;
constexpr int C3_DMA = 6;                                    // DMA wave-instructions per wave per tile
constexpr int C3_HSLOTS = C3_WAVES * C3_DMA * 8;             // 384 pixel slots per halo buffer
static_assert(C3_HSLOTS >= C3_HPIX, "halo fits the DMA slots");
constexpr int C3_HBYTES = C3_HSLOTS * 128;                   // 48 KiB per halo buffer
constexpr int C3_OBYTES = C3_TH * C3_TW * 128;               // 32 KiB output staging
constexpr int C3_KS = 18;                                    // 32-deep K steps (9 taps x 2 halves)

template <int N>
__device__ __forceinline__ void c3_wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void c3_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <typename T>
__global__ __launch_bounds__(C3_WAVES * 64, 1) void conv3x3_c64_kernel(const GemmArgs p, const int ntiles,
                                                                      const int ntw, const int tiles_per_img) {
    __shared__ __attribute__((aligned(16))) char lds[2 * C3_HBYTES + C3_OBYTES + 512];
    char* const obuf = lds + 2 * C3_HBYTES;
    float* const par = reinterpret_cast<float*>(obuf + C3_OBYTES);   // BN scale [64], bias [64]
    constexpr unsigned OOB = 0x80000000u;
    const int P = gridDim.x, bx = blockIdx.x;
    const int cnt = bx < ntiles ? (ntiles - 1 - bx) / P + 1 : 0;
    if (cnt == 0) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int og = wave & 1, pg = wave >> 1;
    const int H = p.Hin, W = p.Win;   // stride 1, pad 1: Hout = H, Wout = W
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.b_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(p.C, (short)0, p.c_bytes, 0x00020000);

    if (tid < 64) {
        par[tid] = p.scale ? p.scale[tid] : 1.f;
        par[64 + tid] = p.bias ? p.bias[tid] : 0.f;
    }
    // DMA instruction j of this wave covers halo pixels [(wave*C3_DMA + j)*8, +8): lane ->
    // pixel + (lane >> 3), its slot (lane & 7) holds logical chunk (lane & 7) ^ (lane >> 3)
    const unsigned dch = (unsigned)(((lane & 7) ^ (lane >> 3)) * 16);
    auto tile_origin = [&](int t, int& b, int& oh0, int& ow0) {
        b = t / tiles_per_img;
        const int r = t - b * tiles_per_img;
        const int th = r / ntw;
        oh0 = th * C3_TH;
        ow0 = (r - th * ntw) * C3_TW;
    };
    auto issue_halo = [&](int t, int buf) {
        int b, oh0, ow0;
        tile_origin(t, b, oh0, ow0);
        char* dst = lds + buf * C3_HBYTES;
#pragma unroll
        for (int j = 0; j < C3_DMA; ++j) {
            const int hp = (wave * C3_DMA + j) * 8 + (lane >> 3);
            const int hr = hp / C3_HW;
            const int ih = oh0 - 1 + hr, iw = ow0 - 1 + (hp - hr * C3_HW);
            const bool ok = hp < C3_HPIX && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
            const unsigned off = ok ? ((unsigned)((b * H + ih) * W + iw) * 128u + dch) : OOB;
            dma16(rx, dst + (wave * C3_DMA + j) * 1024, off);
        }
    };

    // weights: A fragments of output channels 32 og + 16 ot + (lane & 15), K = 32 s + 8 (lane >> 4)
    u32x4 wf[2][C3_KS];
#pragma unroll
    for (int ot = 0; ot < 2; ++ot)
#pragma unroll
        for (int s = 0; s < C3_KS; ++s) {
            const unsigned oc = (unsigned)(32 * og + 16 * ot + (lane & 15));
            wf[ot][s] = __builtin_amdgcn_raw_buffer_load_b128(rw, (oc * 576u + (unsigned)(32 * s + 8 * (lane >> 4))) * 2u, 0, 0);
        }
    // B-fragment halo pixel of sub-tile st (16 consecutive output columns) for tap (0, 0)
    int hp0[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) hp0[st] = (2 * pg + (st >> 1)) * C3_HW + (st & 1) * 16 + (lane & 15);
    const int g4 = lane >> 4;

    issue_halo(bx, 0);
    for (int i = 0; i < cnt; ++i) {
        // tile i's halo landed (younger: the 4 output stores of tile i-1), everyone's; every
        // wave is also past tile i-1 (its halo buffer and the output staging are free)
        if (i == 0) c3_wait_vmcnt<0>();
        else c3_wait_vmcnt<4>();
        c3_lds_barrier();
        if (i + 1 < cnt) issue_halo(bx + (i + 1) * P, (i + 1) & 1);
        const char* hb = lds + (i & 1) * C3_HBYTES;
        f32x4 acc[2][4];
#pragma unroll
        for (int ot = 0; ot < 2; ++ot)
#pragma unroll
            for (int st = 0; st < 4; ++st) acc[ot][st] = f32x4{0.f, 0.f, 0.f, 0.f};
        // activation fragments of K step s (16-byte channel chunk (s & 1)*4 + lane/16 of the
        // tap's shifted pixel), read one step ahead of their MFMAs
        // (the pixel bases pass through an empty asm each tile: otherwise hipcc hoists all 72
        // swizzled addresses out of the tile loop into VGPRs and spills the weights)
        int hq[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            hq[st] = hp0[st];
            asm volatile("" : "+v"(hq[st]));
        }
        auto read_x = [&](int s, u32x4 (&xf)[4]) {
            const int tap = s >> 1, kh = tap / 3, kw = tap - kh * 3;
            const int cc = (s & 1) * 4 + g4;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const int hp = hq[st] + kh * C3_HW + kw;
                xf[st] = *reinterpret_cast<const u32x4*>(hb + hp * 128 + ((cc ^ (hp & 7)) << 4));
            }
        };
        u32x4 xa[4], xb[4];
        read_x(0, xa);
#pragma unroll
        for (int s = 0; s < C3_KS; s += 2) {
            read_x(s + 1, xb);
#pragma unroll
            for (int st = 0; st < 4; ++st)
#pragma unroll
                for (int ot = 0; ot < 2; ++ot) Mma<T>::run(acc[ot][st], wf[ot][s], xa[st]);
            __builtin_amdgcn_sched_barrier(0);
            if (s + 2 < C3_KS) read_x(s + 2, xa);
#pragma unroll
            for (int st = 0; st < 4; ++st)
#pragma unroll
                for (int ot = 0; ot < 2; ++ot) Mma<T>::run(acc[ot][st], wf[ot][s + 1], xb[st]);
            __builtin_amdgcn_sched_barrier(0);
        }
        // ---- epilogue: BN scale / bias + ReLU, park the 16-bit tile, stream whole pixel rows ----
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const int px = (2 * pg + (st >> 1)) * C3_TW + (st & 1) * 16 + (lane & 15);
#pragma unroll
            for (int ot = 0; ot < 2; ++ot) {
                float v[4];
                const int oc0 = 32 * og + 16 * ot + 4 * g4;
                const f32x4 s4 = *reinterpret_cast<const f32x4*>(par + oc0);
                const f32x4 b4 = *reinterpret_cast<const f32x4*>(par + 64 + oc0);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float x = acc[ot][st][r] * s4[r] + b4[r];
                    v[r] = p.relu ? fmaxf(x, 0.f) : x;
                }
                const int c = oc0 >> 3;
                uint2 w2;
                if constexpr (std::is_same<T, bf16_t>::value) {
                    w2.x = (uint32_t)f32_to_bf16(v[0]).x | ((uint32_t)f32_to_bf16(v[1]).x << 16);
                    w2.y = (uint32_t)f32_to_bf16(v[2]).x | ((uint32_t)f32_to_bf16(v[3]).x << 16);
                } else {
                    w2.x = (uint32_t)__builtin_bit_cast(uint16_t, (f16_t)v[0]) |
                           ((uint32_t)__builtin_bit_cast(uint16_t, (f16_t)v[1]) << 16);
                    w2.y = (uint32_t)__builtin_bit_cast(uint16_t, (f16_t)v[2]) |
                           ((uint32_t)__builtin_bit_cast(uint16_t, (f16_t)v[3]) << 16);
                }
                *reinterpret_cast<uint2*>(obuf + px * 128 + ((c ^ (px & 7)) << 4) + (oc0 & 4) * 2) = w2;
            }
        }
        c3_lds_barrier();
        int b, oh0, ow0;
        tile_origin(bx + i * P, b, oh0, ow0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q = tid + k * C3_WAVES * 64;   // 16-byte chunk of the 256 x 128 B tile
            const int px = q >> 3, c = q & 7;
            const int oh = oh0 + px / C3_TW, ow = ow0 + (px & (C3_TW - 1));
            const u32x4 v = *reinterpret_cast<const u32x4*>(obuf + px * 128 + ((c ^ (px & 7)) << 4));
            const bool ok = oh < H && ow < W;
            const unsigned off =
                ok ? ((unsigned)((b * H + oh) * W + ow) * (unsigned)p.ldc + (unsigned)(c * 8)) * 2u : OOB;
            __builtin_amdgcn_raw_buffer_store_b128(v, ry, off, 0, 0);
        }
    }
}

}  // namespace

// Entry from gemm.hip's conv dispatcher: the 3x3 / stride 1 / pad 1, 64 -> 64 channel conv
// without residual (Bottleneck.conv2 of ResNet layer 1); false leaves it to the implicit GEMM.
bool launch_conv3x3_c64(const GemmArgs& a, int dtype, hipStream_t stream) {
    if (dtype != KINET_BF16 && dtype != KINET_F16) return false;
    if (a.Cin != 64 || a.N != 64 || a.K != 576 || a.KW != 3 || a.stride != 1 || a.stride_w != 1 || a.pad != 1 ||
        a.pad_w != 1 || a.Hout != a.Hin || a.Wout != a.Win)
        return false;
    if (a.R != nullptr || a.ln_g != nullptr || a.row_mask != nullptr || a.A2 != nullptr || a.kchunk != 0 ||
        a.hm_rows != 0 || a.m_begin != 0)
        return false;
    if (a.ldc < 64 || a.ldc % 8 != 0 || (((uintptr_t)a.C) & 15) != 0) return false;
    const long long hw = (long long)a.Hout * a.Wout;
    if (a.M % hw != 0) return false;
    const int batch = (int)(a.M / hw);
    const long long cb = ((long long)(a.M - 1) * a.ldc + 64) * 2;
    if (cb >= (1LL << 31) || (long long)a.M * 128 >= (1LL << 31)) return false;
    GemmArgs g = a;
    g.c_bytes = (int)cb;
    const int nth = (a.Hout + C3_TH - 1) / C3_TH, ntw = (a.Wout + C3_TW - 1) / C3_TW;
    const long long nt = (long long)batch * nth * ntw;
    if (nt >= (1LL << 31)) return false;
    const int cus = cu_count();
    const int grid = (int)(nt < cus ? nt : cus);
    if (dtype == KINET_BF16)
        hipLaunchKernelGGL((conv3x3_c64_kernel<bf16_t>), dim3(grid), dim3(C3_WAVES * 64), 0, stream, g, (int)nt, ntw,
                           nth * ntw);
    else
        hipLaunchKernelGGL((conv3x3_c64_kernel<f16_t>), dim3(grid), dim3(C3_WAVES * 64), 0, stream, g, (int)nt, ntw,
                           nth * ntw);
    return true;
}

}  // namespace kinet
