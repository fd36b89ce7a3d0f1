// MSDeformAttn sampling for ENCODER calls, value windows staged in LDS (gfx950 / CDNA4).
//
// Same arithmetic contract as msda_fused_fast_kernel (msda.hip) -- softmax over L*P
// logits, 2-d / 4-d reference-point locations (ms_deform_attn.py:70-82), bilinear taps
// with zeros outside the image (ms_deform_im2col_cuda.cuh:24-67, :227-233), f16 values x
// f16 tap weights accumulated in f32 -- for the encoder's query set, where the queries ARE
// the pixels of the value levels (Lq == S, deformable_transformer.py:290-299, :309-321).
//
// Why a separate kernel: the gather kernel reads every bilinear corner (4 x 64 B per
// sample and head) through the texture/L1 path, ~18x the compulsory bytes of an encoder
// call, and that return path (64 B/clk/CU) is what bounds it.  Here a workgroup owns one
// head and a 4 x 16 tile of query pixels of one level (one tile row per wave, 4 lanes per
// query); the samples of a spatially compact tile land in a compact window of every level:
//   1. phase 1: lane (query, j) computes the 4 points of level j (vector loads of its logits,
//      offsets and reference point; softmax across the quad), and the corners' bounding box
//      per level is reduced across the wave and the workgroup;
//   2. the 4 windows (bounding boxes, clipped to ENC_WIN pixels together) are loaded ONCE,
//      all in flight together, by LDS-DMA (no register staging) -- pixels outside the image
//      come back as zeros, which is the reference's zero padding for free;
//   3. the corners are read back with ds_read_b128 (2-4 x the L1 return rate, and conflict
//      free: a 16-lane LDS group reads 4 pixels x 4 chunks of horizontally adjacent queries,
//      i.e. 4 distinct 256-byte bank residues); the sample records move between the quad's
//      lanes by DPP broadcasts, not through LDS;
//   4. a sample whose corners fall outside its window (offsets larger than the window
//      budget allows) takes the global-load path of msda_fused_fast_kernel instead.
// The per-sample arithmetic (f32 location, f16 corner weights, corner-then-sample f32
// accumulation order) is msda_fused_fast_kernel's, so the outputs are bit-identical to it
// (tests/test_msda_gpu.py::test_encoder_kernel_*).
#include <hip/hip_runtime.h>

#include <limits.h>
#include <math.h>

#include <algorithm>

#include "../../include/kinet_msda.h"
#include "common.h"
#include "msda_util.h"

namespace kinet {
namespace {

constexpr int ENC_L = 4, ENC_P = 4, ENC_LP = 16;
constexpr int ENC_TR = 4, ENC_TC = 16;                            // query tile: 4 rows x 16 columns
constexpr int ENC_THREADS = 256;                                  // 4 lanes per query, one tile row per wave
constexpr int ENC_PIX = 64;                                       // bytes per pixel of one head (D=32, 16-bit)
constexpr int ENC_WIN = 760;                                      // window budget of the 4 levels, pixels
constexpr int ENC_WPAD = 16;                                      // levels start at multiples of 16 pixels (1 KiB)
constexpr int ENC_ZPIX = ENC_WIN + ENC_L * ENC_WPAD;              // the zero pixel
constexpr unsigned ENC_OOB = 0x80000000u;

struct EncGeom {
    int start[ENC_L], H[ENC_L], W[ENC_L];
    int tile0[ENC_L + 1];   // first tile of each query level (tile0[L] = total)
    int tiles_x[ENC_L];     // tiles per tile row of each level
    float rH[ENC_L], rW[ENC_L];   // 1/H, 1/W (IEEE, host-computed: the fast kernel's normalisers)
};

struct EncWin {
    int r0, c0, hw, ww;     // rows [r0, r0 + hw), columns [c0, c0 + ww) of the level's pixel grid
    int base;               // first pixel of the level's window in LDS (multiple of ENC_WPAD)
    float rww;              // 1 / ww
};

typedef __attribute__((address_space(3))) void* enc_lds_ptr_t;

// one 16-byte-per-lane LDS-DMA: LDS[dst + 16*lane] = buffer[off] (0 if off is out of range).
// Not a template: hipcc (ROCm 7.2) drops the host stub of a kernel template calling it directly.
__device__ __forceinline__ void enc_dma16(__amdgpu_buffer_rsrc_t r, char* dst, unsigned off) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (enc_lds_ptr_t)dst, 16, off, 0, 0, 0);
}

// broadcast lane (lane & ~3) + S of every quad (DPP quad_perm [S,S,S,S])
template <int S>
__device__ __forceinline__ int quad_bcast(int v) {
    return __builtin_amdgcn_update_dpp(0, v, S | (S << 2) | (S << 4) | (S << 6), 0xf, 0xf, false);
}

template <typename TL, int N>
struct LdVec;
template <int N> struct LdVec<f16_t, N> {
    static __device__ __forceinline__ void load(const f16_t* p, float* v) {
        if constexpr (N == 4) {
            const uint2 u = *reinterpret_cast<const uint2*>(p);
            const uint32_t w[2] = {u.x, u.y};
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = (float)__builtin_bit_cast(f16_t, (uint16_t)(w[i >> 1] >> (16 * (i & 1))));
        } else {
            const uint4 u = *reinterpret_cast<const uint4*>(p);
            const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = (float)__builtin_bit_cast(f16_t, (uint16_t)(w[i >> 1] >> (16 * (i & 1))));
        }
    }
};
template <int N> struct LdVec<float, N> {
    static __device__ __forceinline__ void load(const float* p, float* v) {
#pragma unroll
        for (int i = 0; i < N; i += 4) {
            const float4 f = *reinterpret_cast<const float4*>(p + i);
            v[i] = f.x; v[i + 1] = f.y; v[i + 2] = f.z; v[i + 3] = f.w;
        }
    }
};

// one work item = (tile, frame, head)
struct EncItem {
    int b, m, lq, qy0, qx0;
};

__device__ __forceinline__ EncItem enc_item(const EncGeom& g, int item, int ntiles, int B, const int* torder) {
    EncItem it;
    const int tx = item % ntiles, rest = item / ntiles;
    const int tile = torder ? torder[tx] : tx;
    it.b = rest % B;
    it.m = rest / B;
    int lq = 0;
#pragma unroll
    for (int l = 1; l < ENC_L; ++l) lq += tile >= g.tile0[l] ? 1 : 0;
    const int tl = tile - g.tile0[lq];
    const int tyi = tl / g.tiles_x[lq];
    it.lq = lq;
    it.qy0 = tyi * ENC_TR;
    it.qx0 = (tl - tyi * g.tiles_x[lq]) * ENC_TC;
    return it;
}

// raw phase-1 inputs of one lane: 4 logits, 4 (x, y) offsets, the reference point
struct EncRaw {
    float lg[4], of[8], rp[4];
    bool masked;
};

template <typename TL>
__device__ __forceinline__ void enc_load_raw(EncRaw& r, const TL* offlog, int ld_off, const float* ref, int ref_dim,
                                             const uint8_t* qmask, long row, int M, int m, int j, bool ok) {
    const TL* orow = offlog + row * ld_off;
    LdVec<TL, 4>::load(orow + M * ENC_LP * 2 + m * ENC_LP + j * 4, r.lg);
    LdVec<TL, 8>::load(orow + (m * ENC_LP + j * 4) * 2, r.of);
    const float* rq = ref + (row * ENC_L + j) * ref_dim;
    if (ref_dim == 2) {
        const float2 r2 = *reinterpret_cast<const float2*>(rq);
        r.rp[0] = r2.x; r.rp[1] = r2.y; r.rp[2] = 0.f; r.rp[3] = 0.f;
    } else {
        const float4 r4 = *reinterpret_cast<const float4*>(rq);
        r.rp[0] = r4.x; r.rp[1] = r4.y; r.rp[2] = r4.z; r.rp[3] = r4.w;
    }
    r.masked = ok && qmask && qmask[row];                                   // ms_deform_attn.py:73-74
}

// one lane's 4 samples (points of level j of its query)
struct EncSamples {
    int hl[4], wl[4];
    uint32_t w01[4], w23[4];
    bool live[4];
};

template <typename T, typename TO, typename TL>
__global__ __launch_bounds__(ENC_THREADS) void msda_enc_lds_kernel(
    const T* __restrict__ value, long vsb, long vsm, int head_bytes, EncGeom g, const TL* __restrict__ offlog,
    int ld_off, const float* __restrict__ ref, int ref_dim, const uint8_t* __restrict__ qmask,
    float* __restrict__ loc_out, float* __restrict__ attw_out, TO* __restrict__ out, int B, int M, int Lq,
    int ntiles, const int* __restrict__ torder) {
    static_assert(sizeof(T) == 2 && sizeof(TO) == 2, "16-bit values and output");
    constexpr int D = 32;
    // the windows of the 4 levels back to back, then one permanently zero pixel (the target of
    // samples outside the image)
    __shared__ uint4 win[(ENC_ZPIX + 1) * 4];
    __shared__ int bb[ENC_L][4];
    __shared__ EncWin wn[ENC_L];
    __shared__ int lvH[ENC_L], lvW[ENC_L];

    // ---- persistent: the (tile, frame, head) items are split into 8 contiguous runs, one per
    // XCD (workgroups are dealt to the XCDs round-robin), so neighbouring tiles -- which read
    // overlapping value windows -- run on one XCD and share its L2 (cdna_hip_programming.md T1)
    const int nitems = ntiles * B * M;
    const int xcd = blockIdx.x & 7, nx = (int)(gridDim.x >> 3);   // gridDim.x is a multiple of 8
    const int per = (nitems + 7) >> 3;
    const int i_end = min(nitems, (xcd + 1) * per);
    int item = xcd * per + (int)(blockIdx.x >> 3);

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int j = lane & 3;   // this lane's level in phase 1, its 8 channels in phase 2
    if (threadIdx.x < ENC_L * 4) (&bb[0][0])[threadIdx.x] = (threadIdx.x & 1) ? INT_MIN : INT_MAX;
    if (threadIdx.x < ENC_L) {
        lvH[threadIdx.x] = g.H[threadIdx.x];
        lvW[threadIdx.x] = g.W[threadIdx.x];
    }
    if (threadIdx.x < 4) win[ENC_ZPIX * 4 + threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    if (item >= i_end) return;
    const int Hj = lvH[j], Wj = lvW[j];
    const float Hf = (float)Hj, Wf = (float)Wj;
    const float rHj = j == 0 ? g.rH[0] : j == 1 ? g.rH[1] : j == 2 ? g.rH[2] : g.rH[3];
    const float rWj = j == 0 ? g.rW[0] : j == 1 ? g.rW[1] : j == 2 ? g.rW[2] : g.rW[3];

    auto query_of = [&](const EncItem& it, int& q) {
        const int Hq = g.H[it.lq], Wq = g.W[it.lq];
        const int qy = it.qy0 + wave, qx = it.qx0 + (lane >> 2);
        const bool ok = qy < Hq && qx < Wq;
        q = g.start[it.lq] + (ok ? qy * Wq + qx : 0);
        return ok;
    };

    // phase 1 for one item: softmax over the quad, locations, bilinear corners, bbox atomics
    auto phase1 = [&](const EncItem& it, const EncRaw& r, bool ok, int q, EncSamples& sm) {
        float mx = ok ? fmaxf(fmaxf(r.lg[0], r.lg[1]), fmaxf(r.lg[2], r.lg[3])) : -INFINITY;
        mx = group_reduce<4, true>(mx);
        float e[4], sum = 0.f;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            e[p] = ok ? __expf(r.lg[p] - mx) : 0.f;
            sum += e[p];
        }
        sum = group_reduce<4, false>(sum);
        const float rs = __builtin_amdgcn_rcpf(sum);
        int ymin = INT_MAX, ymax = INT_MIN, xmin = INT_MAX, xmax = INT_MIN;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const float a = (ok && !r.masked) ? e[p] * rs : 0.f;
            float x, y;
            if (ref_dim == 2) {   // offsets / spatial_shapes[(H, W)] on (x, y): the reference's quirk (:77-79)
                x = r.rp[0] + r.of[2 * p] * rHj;
                y = r.rp[1] + r.of[2 * p + 1] * rWj;
            } else {              // :80-82
                x = r.rp[0] + r.of[2 * p] * (0.5f / (float)ENC_P) * r.rp[2];
                y = r.rp[1] + r.of[2 * p + 1] * (0.5f / (float)ENC_P) * r.rp[3];
            }
            if (loc_out && ok) {
                const long gi = (((long)it.b * Lq + q) * M + it.m) * ENC_LP + j * 4 + p;
                loc_out[2 * gi] = x;
                loc_out[2 * gi + 1] = y;
                attw_out[gi] = a;
            }
            const float h = y * Hf - 0.5f, w = x * Wf - 0.5f;                        // cuh:227-228
            sm.hl[p] = sm.wl[p] = 0;
            sm.w01[p] = sm.w23[p] = 0u;
            sm.live[p] = ok && Hj > 0 && Wj > 0 && h > -1.f && w > -1.f && h < Hf && w < Wf;   // cuh:229
            if (sm.live[p]) {
                const float hf = floorf(h), wf = floorf(w);
                const int hl = (int)hf, wl = (int)wf;
                const float lh = h - hf, lw = w - wf, hh = 1.f - lh, hw = 1.f - lw;
                // corners outside the image weigh 0 (cuh:38-61); the window holds zeros there too
                const bool h0 = hl >= 0, h1 = hl + 1 < Hj, c0 = wl >= 0, c1 = wl + 1 < Wj;
                sm.w01[p] = pack_f16x2((h0 && c0) ? hh * hw * a : 0.f, (h0 && c1) ? hh * lw * a : 0.f);
                sm.w23[p] = pack_f16x2((h1 && c0) ? lh * hw * a : 0.f, (h1 && c1) ? lh * lw * a : 0.f);
                sm.hl[p] = hl;
                sm.wl[p] = wl;
                ymin = min(ymin, hl);
                ymax = max(ymax, hl);
                xmin = min(xmin, wl);
                xmax = max(xmax, wl);
            }
        }
        // corner bounding box per level: the 16 lanes of the wave with the same j (xor 4 .. 32),
        // then one LDS atomic per level and wave
#pragma unroll
        for (int sh = 4; sh <= 32; sh <<= 1) {
            ymin = min(ymin, __shfl_xor(ymin, sh));
            ymax = max(ymax, __shfl_xor(ymax, sh));
            xmin = min(xmin, __shfl_xor(xmin, sh));
            xmax = max(xmax, __shfl_xor(xmax, sh));
        }
        if (lane < 4 && ymin <= ymax) {
            atomicMin(&bb[lane][0], ymin);
            atomicMax(&bb[lane][1], ymax);
            atomicMin(&bb[lane][2], xmin);
            atomicMax(&bb[lane][3], xmax);
        }
    };

    // windows from the bounding boxes: when the 4 together exceed ENC_WIN pixels, levels are
    // served coarsest first (they need the least) with an equal share of what is left, each
    // clipped around the tile's nominal footprint (the excess goes down the global path).
    // Fully unrolled: a dynamically indexed private array would become a per-thread LDS copy.
    auto windows = [&](const EncItem& it) {
        const int Hq = g.H[it.lq], Wq = g.W[it.lq];
        int left = ENC_WIN;
        EncWin wv[ENC_L];
#pragma unroll
        for (int k = 0; k < ENC_L; ++k) {
            const int l = ENC_L - 1 - k;
            const bool any = bb[l][0] <= bb[l][1];
            const int y0 = bb[l][0], y1 = bb[l][1] + 1, x0 = bb[l][2], x1 = bb[l][3] + 1;   // corner extent
            int h = any ? y1 - y0 + 1 : 0, w = any ? x1 - x0 + 1 : 0, r0 = y0, c0 = x0;
            const int cap = left / (ENC_L - k);
            if (h * w > cap) {
                const int hcap = max(1, min(h, min(16, cap / 2)));
                const int wcap = max(1, min(w, cap / hcap));
                const float cy = ((float)it.qy0 + 0.5f * ENC_TR) / (float)Hq * (float)g.H[l];
                const float cx = ((float)it.qx0 + 0.5f * ENC_TC) / (float)Wq * (float)g.W[l];
                r0 = min(max((int)floorf(cy) - hcap / 2, y0), y1 + 1 - hcap);
                c0 = min(max((int)floorf(cx) - wcap / 2, x0), x1 + 1 - wcap);
                h = hcap;
                w = wcap;
            }
            left -= h * w;
            wv[l] = EncWin{r0, c0, h, w, 0, w > 0 ? 1.f / (float)w : 0.f};
        }
        int base = 0;
#pragma unroll
        for (int l = 0; l < ENC_L; ++l) {
            wv[l].base = base;
            base += (wv[l].hw * wv[l].ww + ENC_WPAD - 1) / ENC_WPAD * ENC_WPAD;
            wn[l] = wv[l];
        }
    };

    EncItem cur = enc_item(g, item, ntiles, B, torder);
    int qc;
    bool okc = query_of(cur, qc);
    EncSamples sm;
    {
        EncRaw r;
        enc_load_raw(r, offlog, ld_off, ref, ref_dim, qmask, (long)cur.b * Lq + qc, M, cur.m, j, okc);
        phase1(cur, r, okc, qc, sm);
    }
    __syncthreads();
    if (threadIdx.x == 0) windows(cur);
    __syncthreads();

    const unsigned cb = (unsigned)j * 16u;   // this lane's 8 channels, bytes
    const char* wb = reinterpret_cast<const char*>(win);
#pragma unroll 1
    while (true) {
        // ---- fill the current item's windows by LDS-DMA (a wave-instruction writes 64 x 16 B =
        // 16 contiguous pixels of one level; levels start 16-pixel aligned; pixels outside the
        // image come back as zeros from the buffer range check)
        const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(value + (long)cur.b * vsb + (long)cur.m * vsm), (short)0, head_bytes, 0x00020000);
#pragma unroll
        for (int l = 0; l < ENC_L; ++l) {
            const EncWin w = wn[l];
            const int n4 = w.hw * w.ww * 4;
            for (int c0 = wave * 64; c0 < n4; c0 += ENC_THREADS) {
                const int c = c0 + lane;
                const int px = c >> 2;
                const int r = (int)(((float)px + 0.5f) * w.rww);
                const int gy = w.r0 + r, gx = w.c0 + (px - r * w.ww);
                const bool in = c < n4 && gy >= 0 && gy < g.H[l] && gx >= 0 && gx < g.W[l];
                const unsigned off = in ? (unsigned)((g.start[l] + gy * g.W[l] + gx) * ENC_PIX) + (unsigned)(c & 3) * 16u
                                        : ENC_OOB;
                enc_dma16(rv, reinterpret_cast<char*>(win) + (w.base * 4 + c0) * 16, off);
            }
        }
        // per-sample LDS offsets against the windows: >= 0 top-left corner, ZOFF dead,
        // < 0 global path with (hl, wl) packed
        int offs[4];
        {
            const EncWin wj = wn[j];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                offs[p] = ENC_ZPIX * ENC_PIX;
                if (sm.live[p]) {
                    const int rr = sm.hl[p] - wj.r0, cc = sm.wl[p] - wj.c0;
                    if (rr >= 0 && rr + 1 < wj.hw && cc >= 0 && cc + 1 < wj.ww)
                        offs[p] = (wj.base + rr * wj.ww + cc) * ENC_PIX;
                    else
                        offs[p] = -1 - (int)(((uint32_t)(sm.hl[p] + 1) & 0x7fffu) | ((uint32_t)(sm.wl[p] + 1) << 15));
                }
            }
        }
        int drow[ENC_L];
#pragma unroll
        for (int l = 0; l < ENC_L; ++l) drow[l] = wn[l].ww * ENC_PIX;
        // ---- next item's phase-1 inputs, in flight with the DMA
        const int nitem = item + nx;
        const bool more = nitem < i_end;
        EncItem nxt = cur;
        int qn = qc;
        bool okn = false;
        EncRaw rn;
        if (more) {
            nxt = enc_item(g, nitem, ntiles, B, torder);
            okn = query_of(nxt, qn);
            enc_load_raw(rn, offlog, ld_off, ref, ref_dim, qmask, (long)nxt.b * Lq + qn, M, nxt.m, j, okn);
        }
        __builtin_amdgcn_s_waitcnt(0);   // this wave's DMA (and the next item's inputs) landed
        __syncthreads();                 // ... and every other wave's
        if (threadIdx.x < ENC_L * 4) (&bb[0][0])[threadIdx.x] = (threadIdx.x & 1) ? INT_MIN : INT_MAX;

        // ---- sample, level by level: the 4 points of level l come from quad lane l (DPP)
        f32x2 acc[4] = {};
        auto mac = [&](const u32x4v (&v)[4], uint32_t wa, uint32_t wc) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t wp = k < 2 ? wa : wc;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    acc[i][0] = (k & 1) ? fma_mix16_lo_hi(acc[i][0], v[k][i], wp) : fma_mix16_lo_lo(acc[i][0], v[k][i], wp);
                    acc[i][1] = (k & 1) ? fma_mix16_hi_hi(acc[i][1], v[k][i], wp) : fma_mix16_hi_lo(acc[i][1], v[k][i], wp);
                }
            }
        };
        auto level = [&](auto lc) {
            constexpr int L_ = decltype(lc)::value;
            int o[4];
            uint32_t wa[4], wc[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                o[p] = quad_bcast<L_>(offs[p]);
                wa[p] = (uint32_t)quad_bcast<L_>((int)sm.w01[p]);
                wc[p] = (uint32_t)quad_bcast<L_>((int)sm.w23[p]);
            }
            const bool all_in = o[0] >= 0 && o[1] >= 0 && o[2] >= 0 && o[3] >= 0;
            if (__builtin_amdgcn_ballot_w64(!all_in) == 0) {
#pragma unroll
                for (int p0 = 0; p0 < 4; p0 += 2) {
                    u32x4v v[2][4];
#pragma unroll
                    for (int p = 0; p < 2; ++p) {
                        const int op = o[p0 + p];
                        const bool dead = op == ENC_ZPIX * ENC_PIX;
                        const unsigned a0 = (unsigned)op + cb;
                        const unsigned d1 = dead ? 0u : (unsigned)ENC_PIX, d2 = dead ? 0u : (unsigned)drow[L_];
                        v[p][0] = *reinterpret_cast<const u32x4v*>(wb + a0);
                        v[p][1] = *reinterpret_cast<const u32x4v*>(wb + a0 + d1);
                        v[p][2] = *reinterpret_cast<const u32x4v*>(wb + a0 + d2);
                        v[p][3] = *reinterpret_cast<const u32x4v*>(wb + a0 + d2 + d1);
                    }
#pragma unroll
                    for (int p = 0; p < 2; ++p) mac(v[p], wa[p0 + p], wc[p0 + p]);
                }
            } else {
#pragma unroll 1
                for (int p = 0; p < 4; ++p) {
                    u32x4v v[4];
                    const int op = o[p];
                    if (op >= 0) {
                        const bool dead = op == ENC_ZPIX * ENC_PIX;
                        const unsigned a0 = (unsigned)op + cb;
                        const unsigned d1 = dead ? 0u : (unsigned)ENC_PIX, d2 = dead ? 0u : (unsigned)drow[L_];
                        v[0] = *reinterpret_cast<const u32x4v*>(wb + a0);
                        v[1] = *reinterpret_cast<const u32x4v*>(wb + a0 + d1);
                        v[2] = *reinterpret_cast<const u32x4v*>(wb + a0 + d2);
                        v[3] = *reinterpret_cast<const u32x4v*>(wb + a0 + d2 + d1);
                    } else {
                        // outside the window: gather from the head map (corners outside the
                        // image get an offset past num_records -> hardware zero)
                        const uint32_t pk = (uint32_t)(-1 - op);
                        const int hl = (int)(pk & 0x7fffu) - 1, wl = (int)(pk >> 15) - 1;
                        const int H = g.H[L_], W = g.W[L_];
                        const bool h0 = hl >= 0, h1 = hl + 1 < H, c0 = wl >= 0, c1 = wl + 1 < W;
                        const int o00 = (g.start[L_] + hl * W + wl) * ENC_PIX;
                        const unsigned g0 = (h0 && c0) ? (unsigned)o00 + cb : ENC_OOB;
                        const unsigned g1 = (h0 && c1) ? (unsigned)(o00 + ENC_PIX) + cb : ENC_OOB;
                        const unsigned g2 = (h1 && c0) ? (unsigned)(o00 + W * ENC_PIX) + cb : ENC_OOB;
                        const unsigned g3 = (h1 && c1) ? (unsigned)(o00 + W * ENC_PIX + ENC_PIX) + cb : ENC_OOB;
                        v[0] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, g0, 0, 0));
                        v[1] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, g1, 0, 0));
                        v[2] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, g2, 0, 0));
                        v[3] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, g3, 0, 0));
                    }
                    mac(v, wa[p], wc[p]);
                }
            }
        };
        level(std::integral_constant<int, 0>{});
        level(std::integral_constant<int, 1>{});
        level(std::integral_constant<int, 2>{});
        level(std::integral_constant<int, 3>{});

        if (okc) {
            VecT<TO, 8> ov;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ov.v[2 * i] = Cvt<TO>::from(acc[i][0]);
                ov.v[2 * i + 1] = Cvt<TO>::from(acc[i][1]);
            }
            *reinterpret_cast<VecT<TO, 8>*>(out + ((long)cur.b * Lq + qc) * M * D + (long)cur.m * D + j * 8) = ov;
        }
        if (!more) break;   // uniform across the workgroup
        // ---- next item: phase 1 from the inputs that arrived under the sampling
        phase1(nxt, rn, okn, qn, sm);
        __syncthreads();    // every wave done reading the windows; bbox complete
        if (threadIdx.x == 0) windows(nxt);
        __syncthreads();
        cur = nxt;
        qc = qn;
        okc = okn;
        item = nitem;
    }
}

}  // namespace
}  // namespace kinet

extern "C" int kinet_msda_encoder_tiles(const int64_t* host_spatial_shapes, int num_levels) {
    if (num_levels != kinet::ENC_L || !host_spatial_shapes) return -1;
    long long n = 0;
    for (int l = 0; l < num_levels; ++l) {
        const long long H = host_spatial_shapes[2 * l], W = host_spatial_shapes[2 * l + 1];
        n += ((H + kinet::ENC_TR - 1) / kinet::ENC_TR) * ((W + kinet::ENC_TC - 1) / kinet::ENC_TC);
    }
    return (int)n;
}

extern "C" int kinet_msda_encoder_forward(const void* value, int64_t value_sb, int64_t value_sm,
                                          const int64_t* host_spatial_shapes, const void* offsets_logits, int ld_off,
                                          const float* ref_points, int ref_dim, const uint8_t* query_attn_mask,
                                          void* output, float* loc_out, float* attw_out, int batch, int spatial_size,
                                          int num_heads, int channels, int num_levels, int num_point,
                                          int value_dtype, int output_dtype, int offlog_dtype,
                                          const int32_t* tile_order, kinet_stream_t stream) {
    using namespace kinet;
    KINET_CHECK_ARG(host_spatial_shapes != nullptr, "msda encoder: host_spatial_shapes is NULL");
    KINET_CHECK_ARG(num_levels == ENC_L && num_point == ENC_P && channels == 32,
                    "msda encoder: needs 4 levels, 4 points, head_dim 32 (got L=%d P=%d D=%d)", num_levels, num_point,
                    channels);
    KINET_CHECK_ARG(value_dtype == KINET_F16, "msda encoder: values must be f16 (head-major, kinet_gemm_headmajor)");
    KINET_CHECK_ARG(output_dtype == KINET_F16 || output_dtype == KINET_BF16, "msda encoder: output must be 16-bit");
    KINET_CHECK_ARG(offlog_dtype == KINET_F16 || offlog_dtype == KINET_F32, "msda encoder: offsets/logits f16 or f32");
    KINET_CHECK_ARG(ref_dim == 2 || ref_dim == 4, "Last dim of reference_points must be 2 or 4, but get %d instead.", ref_dim);
    KINET_CHECK_ARG(ld_off >= num_heads * num_levels * num_point * 3, "msda encoder: ld_off %d too small", ld_off);
    KINET_CHECK_ARG((loc_out == nullptr) == (attw_out == nullptr), "msda encoder: loc_out/attw_out both or neither");
    KINET_CHECK_ARG(batch >= 0 && num_heads > 0 && spatial_size >= 0, "msda encoder: bad sizes");
    KINET_CHECK_ARG(value_sm % 8 == 0 && value_sb % 8 == 0 && ((uintptr_t)value % 16) == 0,
                    "msda encoder: head maps must be 16-byte aligned");
    EncGeom g{};
    long long acc = 0, tiles = 0;
    for (int l = 0; l < ENC_L; ++l) {
        const long long H = host_spatial_shapes[2 * l], W = host_spatial_shapes[2 * l + 1];
        KINET_CHECK_ARG(H >= 0 && W >= 0 && H < 32768 && W < 32768, "msda encoder: level %d shape (%lld, %lld)", l, H, W);
        g.start[l] = (int)acc;
        g.H[l] = (int)H;
        g.W[l] = (int)W;
        g.tile0[l] = (int)tiles;
        g.tiles_x[l] = (int)((W + ENC_TC - 1) / ENC_TC);
        g.rH[l] = H > 0 ? 1.f / (float)H : 0.f;
        g.rW[l] = W > 0 ? 1.f / (float)W : 0.f;
        tiles += ((H + ENC_TR - 1) / ENC_TR) * g.tiles_x[l];
        acc += H * W;
        if (g.tiles_x[l] == 0) g.tiles_x[l] = 1;
    }
    g.tile0[ENC_L] = (int)tiles;
    KINET_CHECK_ARG(acc == spatial_size, "msda encoder: queries must be the %lld pixels of the levels (S = %d)", acc,
                    spatial_size);
    const long long head_bytes = (long long)spatial_size * ENC_PIX;
    KINET_CHECK_ARG(head_bytes < (1LL << 31), "msda encoder: head map too large");
    if (batch == 0 || tiles == 0) return KINET_OK;
    // persistent: 3 workgroups per CU (the LDS budget) x 256 CUs, a multiple of the 8 XCDs
    const long long items = tiles * (long long)batch * num_heads;
    KINET_CHECK_ARG(items < (1LL << 31), "msda encoder: too many work items");
    const int nwg = (int)std::min<long long>(3 * 256, (items + 7) / 8 * 8);
    dim3 grid((unsigned)((nwg + 7) / 8 * 8));
    hipStream_t s = (hipStream_t)stream;
#define LAUNCH(TO, TL)                                                                                                \
    hipLaunchKernelGGL((msda_enc_lds_kernel<f16_t, TO, TL>), grid, dim3(ENC_THREADS), 0, s, (const f16_t*)value,      \
                       (long)value_sb, (long)value_sm, (int)head_bytes, g, (const TL*)offsets_logits, ld_off, ref_points, \
                       ref_dim, query_attn_mask, loc_out, attw_out, (TO*)output, batch, num_heads, spatial_size,     \
                       (int)tiles, (const int*)tile_order)
    if (output_dtype == KINET_BF16 && offlog_dtype == KINET_F16) LAUNCH(bf16_t, f16_t);
    else if (output_dtype == KINET_BF16) LAUNCH(bf16_t, float);
    else if (offlog_dtype == KINET_F16) LAUNCH(f16_t, f16_t);
    else LAUNCH(f16_t, float);
#undef LAUNCH
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}
