// Tap-folded ResNet stem convolution for gfx950 (torchvision conv1: 7x7, stride 2, pad 3,
// 3 -> 64 channels, + folded FrozenBatchNorm + ReLU; backbone.py).
//
// Input: pack_image_kwfold's layout (ops.hip) -- F[n][ih][ow][kw*3 + c] (24 channels, the 7
// horizontal taps of output column ow folded in), so the convolution is 7 x 1 with vertical
// stride 2 and no horizontal halo: output (oh, ow) = sum over kh of F[2*oh - 3 + kh][ow][:] . W.
// The implicit-GEMM kernels re-gather every folded row once per output row that uses it
// (7 taps / stride 2 = 3.5x the input through the load path, ~0.7 GB per batch-8 call) and
// with K = 168 a tiled K-loop never gets going.  Here a persistent workgroup walks 4-row x
// 64-column output tiles (the next tile's input loads in flight under the current one):
//  * its 13 folded input rows (2*3 + 7) are loaded ONCE into LDS (39 KiB, 16-byte loads,
//    zeros outside the image) and shared by the 4 output rows (1.6x the input instead of 3.5x);
//  * each wave computes one output row (64 pixels x 64 channels = 16 MFMA tiles) over the
//    6 K-steps of 32 (21 valid 8-channel chunks, the rest zero) with the weights as MFMA
//    A-fragments in registers and the pixel fragments read straight from the folded rows;
//  * epilogue: scale / bias / ReLU on the accumulators, the bf16 tile parked in LDS (16-byte
//    chunks XOR-swizzled by pixel) and written back as whole 128-byte pixel rows.
#include <hip/hip_runtime.h>

#include "../../include/kinet_gemm.h"
#include "common.h"
#include "gemm_common.h"

namespace kinet {
namespace {

constexpr int SK_KH = 7, SK_CG = 24, SK_CO = 64;
constexpr int SK_RH = 4;                              // output rows per workgroup (one per wave)
constexpr int SK_PX = 64;                             // output columns per workgroup
constexpr int SK_ROWS = 2 * (SK_RH - 1) + SK_KH;      // 13 folded input rows
constexpr int SK_ROWB = SK_PX * SK_CG * 2;            // 3072 bytes per folded row segment
constexpr int SK_NCH = SK_KH * SK_CG / 8;             // 21 valid 8-channel chunks of K
constexpr int SK_KS = (SK_NCH + 3) / 4;               // 6 K-steps of 32
constexpr int SK_IN_CH = SK_ROWS * SK_PX * 3;         // 2496 16-byte input chunks
constexpr int SK_IN_OPS = (SK_IN_CH + 255) / 256;     // 10 per thread
static_assert(SK_RH * SK_PX * SK_CO * 2 <= SK_ROWS * SK_ROWB, "output tile fits the input LDS");

template <typename T>
__global__ __launch_bounds__(256, 2) void stem_conv_kernel(const GemmArgs p, const int tiles_x, const int tiles_y,
                                                           const int ntiles) {
    __shared__ __attribute__((aligned(16))) char lds[SK_ROWS * SK_ROWB];
    __shared__ float par[2][SK_CO];             // folded BN scale / bias
    __shared__ __attribute__((aligned(16))) u32x4 wl[4 * SK_KS][64];   // weight fragments (24 KiB)
    constexpr unsigned OOB = 0x80000000u;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (tid < SK_CO) {
        par[0][tid] = p.scale ? p.scale[tid] : 1.f;
        par[1][tid] = p.bias ? p.bias[tid] : 0.f;
    }
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.b_bytes, 0x00020000);

    // persistent: tiles blockIdx.x, +gridDim.x, ...; tile -> (image, 4-row block, 64-column block)
    struct Tile { int n, oh0, ow0; };
    auto decode = [&](int t) {
        const int bx = t % tiles_x, rest = t / tiles_x;
        return Tile{rest / tiles_y, (rest % tiles_y) * SK_RH, bx * SK_PX};
    };
    // folded input rows 2*oh0 - 3 .. +12, columns ow0 .. ow0+63 -> registers (zeros outside)
    u32x4 xin[SK_IN_OPS];
    auto load_in = [&](const Tile& tl) {
        const int ih0 = tl.oh0 * 2 - 3;
#pragma unroll
        for (int i = 0; i < SK_IN_OPS; ++i) {
            const int idx = i * 256 + tid;
            const int r = idx / (SK_PX * 3), rem = idx - r * (SK_PX * 3);
            const int px = rem / 3, part = rem - px * 3;
            const int ih = ih0 + r, ow = tl.ow0 + px;
            const bool ok = idx < SK_IN_CH && (unsigned)ih < (unsigned)p.Hin && ow < p.Win;
            const unsigned off = ok ? ((unsigned)(((tl.n * p.Hin + ih) * p.Win + ow) * SK_CG + part * 8)) * 2u : OOB;
            xin[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
        }
    };
    int t = blockIdx.x;
    Tile cur = decode(t);
    load_in(cur);

    // weights (Cout, 168) as MFMA A-fragments, staged once into LDS fragment-major: lane l of
    // fragment (a, s) holds out channel a*16 + (l&15), k = 32*s + 8*(l>>4) .. +7 (zero past K)
    for (int f = wave; f < 4 * SK_KS; f += 4) {
        const int a = f / SK_KS, s = f - a * SK_KS;
        const int k = 32 * s + 8 * (lane >> 4);
        const unsigned off = k < SK_NCH * 8 ? ((unsigned)((a * 16 + (lane & 15)) * p.ldb + k)) * 2u : OOB;
        wl[f][lane] = __builtin_amdgcn_raw_buffer_load_b128(rw, off, 0, 0);
    }
    T* __restrict__ C = (T*)p.C;

    for (; t < ntiles; t += gridDim.x) {
#pragma unroll
        for (int i = 0; i < SK_IN_OPS; ++i) {
            const int idx = i * 256 + tid;
            if (idx < SK_IN_CH) *reinterpret_cast<u32x4*>(lds + idx * 16) = xin[i];   // = r*ROWB + px*48 + part*16
        }
        __syncthreads();
        // the next tile's input loads fly under this tile's MFMAs and epilogue
        const int tn = t + gridDim.x;
        const Tile nxt = decode(tn < ntiles ? tn : t);
        if (tn < ntiles) load_in(nxt);

        // wave w: output row oh0 + w; pixel fragment of K-step s = 8 channels of chunk
        // ci = 4s + (l>>4) (tap kh = ci / 3, part ci % 3) of folded row 2w + kh, pixel l&15
        f32x4 acc[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[a][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < SK_KS; ++s) {
            const int ci = 4 * s + (lane >> 4);
            const int kh = ci / 3, part = ci - 3 * kh;
            const bool valid = ci < SK_NCH;
            const char* rowp = lds + (2 * wave + (valid ? kh : 0)) * SK_ROWB + part * 16;
            u32x4 wf[4], b[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) wf[a] = wl[a * SK_KS + s][lane];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                b[q] = *reinterpret_cast<const u32x4*>(rowp + (q * 16 + (lane & 15)) * (SK_CG * 2));
                if (!valid) b[q] = u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int a = 0; a < 4; ++a) Mma<T>::run(acc[a][q], wf[a], b[q]);
        }
        __syncthreads();   // every wave done with the input rows: the LDS now takes the output tile

        // epilogue: lane holds channels a*16 + 4*(l>>4) + i of pixel q*16 + (l&15) -> scale /
        // bias / ReLU -> 8 bytes into the parked tile [row][pixel][64 ch] whose 16-byte
        // chunks are XOR-swizzled by (pixel & 7)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const int ch0 = a * 16 + 4 * (lane >> 4);
            const f32x4 sc = *reinterpret_cast<const f32x4*>(&par[0][ch0]);
            const f32x4 bi = *reinterpret_cast<const f32x4*>(&par[1][ch0]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int px = q * 16 + (lane & 15);
                float v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    v[i] = acc[a][q][i] * sc[i] + bi[i];
                    if (p.relu) v[i] = fmaxf(v[i], 0.f);
                }
                uint32_t w[2];
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    w[i] = (uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(v[2 * i])) |
                           ((uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(v[2 * i + 1])) << 16);
                const int chunk = (ch0 >> 3) ^ (px & 7);
                uint32_t* dst =
                    reinterpret_cast<uint32_t*>(lds + (wave * SK_PX + px) * (SK_CO * 2) + chunk * 16 + (ch0 & 4) * 2);
                dst[0] = w[0];
                dst[1] = w[1];
            }
        }
        __syncthreads();

        // whole 128-byte pixel rows, 16 bytes per lane
#pragma unroll
        for (int i = 0; i < SK_RH * SK_PX * 8 / 256; ++i) {
            const int idx = i * 256 + tid;
            const int r = idx / (SK_PX * 8), rem = idx - r * (SK_PX * 8);
            const int px = rem >> 3, c16 = rem & 7;
            const int oh = cur.oh0 + r, ow = cur.ow0 + px;
            if (oh < p.Hout && ow < p.Wout) {
                const u32x4 v =
                    *reinterpret_cast<const u32x4*>(lds + (r * SK_PX + px) * (SK_CO * 2) + ((c16 ^ (px & 7)) * 16));
                *reinterpret_cast<u32x4*>(C + ((long)(cur.n * p.Hout + oh) * p.Wout + ow) * p.ldc + c16 * 8) = v;
            }
        }
        __syncthreads();   // the parked tile is read out before the next input lands in the LDS
        cur = nxt;
    }
}

// ---------------------------------------------------------------------------------------------
// The stem straight from the f32 NCHW image (kinet_stem_conv_image): the same tiles, weights,
// MFMA schedule and epilogue as stem_conv_kernel, but each tile's 13 folded rows are BUILT in
// LDS from the image instead of read from pack_image_kwfold's folded tensor -- that kernel (a
// 205 MB read + 410 MB write at batch 16) and the stem's 1.6x re-reads of its output go away.
//  * the tile's 13 image rows x 3 planes x 133 columns (2*ow0 - 3 ..) load one tile ahead as
//    f32 (wave w: row-planes w, w+4, ..; lane: columns lane, +64, +128), zeros outside the image;
//  * at the tile start they are rounded to T (as pack_image_kwfold does) into an LDS row-plane
//    area, then every 16-byte chunk (row, pixel, part) of the folded rows is assembled from it:
//    element j = 8 part + e of pixel px is plane j % 3, column 2 px + j / 3 (zero for j >= 21).
constexpr int SI_RAWC = 136;                      // row-plane stride (elements), >= 2*63 + 7
constexpr int SI_PAIRS = SK_ROWS * 3;             // 39 row-planes per tile
constexpr int SI_PPW = (SI_PAIRS + 3) / 4;        // per wave (10)

struct StemImgArgs {
    const float* img;
    const void* W;
    const float* scale;
    const float* bias;
    void* Y;
    int N, H, W_, Ho, Wo, ldy;
    int img_bytes, w_bytes;
};

template <typename T>
__global__ __launch_bounds__(256, 2) void stem_img_kernel(const StemImgArgs p, const int tiles_x, const int tiles_y,
                                                          const int ntiles) {
    __shared__ __attribute__((aligned(16))) char lds[SK_ROWS * SK_ROWB];
    __shared__ float par[2][SK_CO];
    __shared__ __attribute__((aligned(16))) u32x4 wl[4 * SK_KS][64];
    __shared__ __attribute__((aligned(16))) uint16_t raw[SI_PAIRS * SI_RAWC];
    constexpr unsigned OOB = 0x80000000u;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (tid < SK_CO) {
        par[0][tid] = p.scale ? p.scale[tid] : 1.f;
        par[1][tid] = p.bias ? p.bias[tid] : 0.f;
    }
    const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)p.img, (short)0, p.img_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.W, (short)0, p.w_bytes, 0x00020000);
    struct Tile { int n, oh0, ow0; };
    auto decode = [&](int t) {
        const int bx = t % tiles_x, rest = t / tiles_x;
        return Tile{rest / tiles_y, (rest % tiles_y) * SK_RH, bx * SK_PX};
    };
    float xin[SI_PPW][3];
    auto load_in = [&](const Tile& tl) {
        const int ih0 = tl.oh0 * 2 - 3, iw0 = tl.ow0 * 2 - 3;
#pragma unroll
        for (int i = 0; i < SI_PPW; ++i) {
            const int pr = i * 4 + wave;                 // row-plane (wave-uniform)
            const int r = pr / 3, c = pr - 3 * r;
            const int ih = ih0 + r;
            const bool rok = pr < SI_PAIRS && (unsigned)ih < (unsigned)p.H;
            const unsigned rowb = (unsigned)(((tl.n * 3 + c) * p.H + ih) * p.W_);
#pragma unroll
            for (int k3 = 0; k3 < 3; ++k3) {
                const int k = lane + 64 * k3, iw = iw0 + k;
                const bool ok = rok && k < SI_RAWC && (unsigned)iw < (unsigned)p.W_;
                xin[i][k3] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ri, ok ? (rowb + (unsigned)iw) * 4u : OOB, 0, 0));
            }
        }
    };
    int t = blockIdx.x;
    Tile cur = decode(t);
    load_in(cur);
    for (int f = wave; f < 4 * SK_KS; f += 4) {
        const int a = f / SK_KS, s = f - a * SK_KS;
        const int k = 32 * s + 8 * (lane >> 4);
        const unsigned off = k < SK_NCH * 8 ? ((unsigned)((a * 16 + (lane & 15)) * (SK_KH * SK_CG) + k)) * 2u : OOB;
        wl[f][lane] = __builtin_amdgcn_raw_buffer_load_b128(rw, off, 0, 0);
    }
    T* __restrict__ C = (T*)p.Y;

    for (; t < ntiles; t += gridDim.x) {
        // image values -> T row-planes (the rounding pack_image_kwfold applies)
#pragma unroll
        for (int i = 0; i < SI_PPW; ++i) {
            const int pr = i * 4 + wave;
            if (pr < SI_PAIRS) {
#pragma unroll
                for (int k3 = 0; k3 < 3; ++k3) {
                    const int k = lane + 64 * k3;
                    if (k < SI_RAWC) raw[pr * SI_RAWC + k] = __builtin_bit_cast(uint16_t, Cvt<T>::from(xin[i][k3]));
                }
            }
        }
        __syncthreads();
        // folded rows: thread = (row, pixel); its 3 chunks (row, pixel, part) -> lds +
        // ((r*64 + px)*3 + part)*16, element j = 8 part + e from plane j % 3, column 2 px + j / 3
        // (compile-time offsets: no index arithmetic per element)
        for (int rp = tid; rp < SK_ROWS * SK_PX; rp += 256) {
            const int r = rp >> 6, px = rp & (SK_PX - 1);
            const uint16_t* src = raw + r * 3 * SI_RAWC + 2 * px;
            u32x4* dst = reinterpret_cast<u32x4*>(lds + rp * 48);
#pragma unroll
            for (int part = 0; part < 3; ++part) {
                uint32_t w[4];
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) {
                    uint32_t h2[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int j = part * 8 + 2 * e2 + h, kw = j / 3, c = j - 3 * kw;
                        h2[h] = j < SK_KH * 3 ? (uint32_t)src[c * SI_RAWC + kw] : 0u;
                    }
                    w[e2] = h2[0] | (h2[1] << 16);
                }
                dst[part] = u32x4{w[0], w[1], w[2], w[3]};
            }
        }
        __syncthreads();
        const int tn = t + gridDim.x;
        const Tile nxt = decode(tn < ntiles ? tn : t);
        if (tn < ntiles) load_in(nxt);

        f32x4 acc[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[a][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < SK_KS; ++s) {
            const int ci = 4 * s + (lane >> 4);
            const int kh = ci / 3, part = ci - 3 * kh;
            const bool valid = ci < SK_NCH;
            const char* rowp = lds + (2 * wave + (valid ? kh : 0)) * SK_ROWB + part * 16;
            u32x4 wf[4], b[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) wf[a] = wl[a * SK_KS + s][lane];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                b[q] = *reinterpret_cast<const u32x4*>(rowp + (q * 16 + (lane & 15)) * (SK_CG * 2));
                if (!valid) b[q] = u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int a = 0; a < 4; ++a) Mma<T>::run(acc[a][q], wf[a], b[q]);
        }
        __syncthreads();

#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const int ch0 = a * 16 + 4 * (lane >> 4);
            const f32x4 sc = *reinterpret_cast<const f32x4*>(&par[0][ch0]);
            const f32x4 bi = *reinterpret_cast<const f32x4*>(&par[1][ch0]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int px = q * 16 + (lane & 15);
                float v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = fmaxf(acc[a][q][i] * sc[i] + bi[i], 0.f);
                uint32_t w[2];
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    w[i] = (uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(v[2 * i])) |
                           ((uint32_t)__builtin_bit_cast(uint16_t, Cvt<T>::from(v[2 * i + 1])) << 16);
                const int chunk = (ch0 >> 3) ^ (px & 7);
                uint32_t* dst =
                    reinterpret_cast<uint32_t*>(lds + (wave * SK_PX + px) * (SK_CO * 2) + chunk * 16 + (ch0 & 4) * 2);
                dst[0] = w[0];
                dst[1] = w[1];
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < SK_RH * SK_PX * 8 / 256; ++i) {
            const int idx = i * 256 + tid;
            const int r = idx / (SK_PX * 8), rem = idx - r * (SK_PX * 8);
            const int px = rem >> 3, c16 = rem & 7;
            const int oh = cur.oh0 + r, ow = cur.ow0 + px;
            if (oh < p.Ho && ow < p.Wo) {
                const u32x4 v =
                    *reinterpret_cast<const u32x4*>(lds + (r * SK_PX + px) * (SK_CO * 2) + ((c16 ^ (px & 7)) * 16));
                *reinterpret_cast<u32x4*>(C + ((long)(cur.n * p.Ho + oh) * p.Wo + ow) * p.ldy + c16 * 8) = v;
            }
        }
        __syncthreads();
        cur = nxt;
    }
}

}  // namespace

// Entry from gemm.hip's conv dispatcher (false = not the stem geometry): the 7 x 1 conv with
// strides (2, 1), pads (3, 0) of 24 folded channels into 64 outputs, 16-bit, no residual.
bool launch_stem_conv(const GemmArgs& a, int dtype, hipStream_t stream) {
    if (dtype != KINET_BF16 && dtype != KINET_F16) return false;
    if (a.KW != 1 || a.Cin != SK_CG || a.K != SK_KH * SK_CG || a.N != SK_CO || a.stride != 2 || a.pad != 3 ||
        a.stride_w != 1 || a.pad_w != 0 || a.Win != a.Wout)
        return false;
    if (a.R != nullptr || a.ln_g != nullptr || a.row_mask != nullptr || a.kchunk != 0 || a.ldc % 8 != 0 ||
        (((uintptr_t)a.C) & 15u) != 0 || a.ldb != SK_KH * SK_CG)
        return false;
    const int hw = a.Hout * a.Wout;
    if (hw <= 0 || a.M % hw != 0) return false;
    const int batch = a.M / hw;
    if (batch == 0) return true;
    const int tiles_x = (a.Wout + SK_PX - 1) / SK_PX, tiles_y = (a.Hout + SK_RH - 1) / SK_RH;
    const long long nt = (long long)tiles_x * tiles_y * batch;
    if (nt >= (1LL << 31)) return false;
    const int grid = nt < 512 ? (int)nt : 512;   // persistent: two workgroups per CU
    if (dtype == KINET_BF16)
        hipLaunchKernelGGL((stem_conv_kernel<bf16_t>), dim3(grid), dim3(256), 0, stream, a, tiles_x, tiles_y, (int)nt);
    else
        hipLaunchKernelGGL((stem_conv_kernel<f16_t>), dim3(grid), dim3(256), 0, stream, a, tiles_x, tiles_y, (int)nt);
    return true;
}

}  // namespace kinet

using namespace kinet;

// torchvision conv1 (7x7 / 2, pad 3, 3 -> 64) + folded FrozenBN + ReLU from the f32 NCHW image
// (backbone.py:102's ResNet stem) -- include/kinet_gemm.h
extern "C" int kinet_stem_conv_image(const float* img, const void* w_packed, const float* scale, const float* bias,
                                     void* Y, int N, int H, int W, int dtype, kinet_stream_t stream) {
    KINET_CHECK_ARG(N >= 0 && H > 0 && W > 0, "stem_conv_image: bad geometry");
    KINET_CHECK_ARG(dtype == KINET_BF16 || dtype == KINET_F16, "stem_conv_image: dtype must be bf16 or f16");
    KINET_CHECK_ARG(img && w_packed && Y, "stem_conv_image: NULL argument");
    KINET_CHECK_ARG((((uintptr_t)Y) & 15u) == 0 && (((uintptr_t)w_packed) & 15u) == 0, "stem_conv_image: Y and weights must be 16-byte aligned");
    if (N == 0) return KINET_OK;
    const long long ib = (long long)N * 3 * H * W * 4;
    KINET_CHECK_ARG(ib < (1LL << 31), "stem_conv_image: image batch larger than 2 GiB (split the call)");
    StemImgArgs a{};
    a.img = img; a.W = w_packed; a.scale = scale; a.bias = bias; a.Y = Y;
    a.N = N; a.H = H; a.W_ = W; a.Ho = (H - 1) / 2 + 1; a.Wo = (W - 1) / 2 + 1; a.ldy = SK_CO;
    a.img_bytes = (int)ib;
    a.w_bytes = SK_CO * SK_KH * SK_CG * 2;
    const int tiles_x = (a.Wo + SK_PX - 1) / SK_PX, tiles_y = (a.Ho + SK_RH - 1) / SK_RH;
    const long long nt = (long long)tiles_x * tiles_y * N;
    KINET_CHECK_ARG(nt < (1LL << 31), "stem_conv_image: too many tiles");
    const int grid = nt < 512 ? (int)nt : 512;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == KINET_BF16)
        hipLaunchKernelGGL((stem_img_kernel<bf16_t>), dim3(grid), dim3(256), 0, s, a, tiles_x, tiles_y, (int)nt);
    else
        hipLaunchKernelGGL((stem_img_kernel<f16_t>), dim3(grid), dim3(256), 0, s, a, tiles_x, tiles_y, (int)nt);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}
