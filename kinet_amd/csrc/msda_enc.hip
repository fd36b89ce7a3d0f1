// Encoder-sized MSDeformAttn sampling (MSDeformAttn.forward, ms_deform_attn.py:69-87, with the
// sampling of ms_deform_im2col_cuda.cuh:165-237) for gfx950: one workgroup per CU owns one
// (frame, head) value map, its coarse levels staged in LDS, and sweeps a share of the map's
// query tiles.  kinet_msda_encoder_forward (include/kinet_msda.h).
//
// Why this shape: at the config-2 encoder call (batch 16, Lq = S = 22,223,
// 8 heads x 32 channels, 4 levels x 4 points) every query gathers 16 samples x 4 corners x
// 64 B = 11.6 GB of corner rows per call.  Through the texture path (64 B per clock per CU)
// that is a ~300 us floor; the two coarse levels of one head (25x42 + 13x21 px, 85 KB) take
// half of those taps and fit in LDS (ds_read_b128, 256 B per clock per CU).  The earlier
// kernel of this design (msda_enc_lds_kernel) was latency-bound: a wave's tile ran phase 1
// (an HBM round trip for the offsets) and then eight dependent gather round trips with two
// samples in flight, so 16 waves per CU kept the texture unit ~60 % busy.  Here:
//  * offsets / logits arrive HEAD-MAJOR (M, B, Lq, 48) f16 [32 offsets (l, p, xy) | 16 logits
//    (l, p)] from the projection GEMM's head-major epilogue: a 16-query tile of one head is
//    1.5 KB contiguous (two vector loads per lane, every fetched line fully used);
//  * the tile's phase-1 loads for tile t+1 are issued while tile t gathers, so phase 1 never
//    waits for HBM;
//  * tap records stay in registers: phase-1 lane (query, level) holds its level's 4 point
//    records, phase-2 lane (query, channel group) fetches them with a quad-broadcast DPP move
//    (same quad = same query in both phases), so no LDS record traffic and no barrier;
//  * all four points of a fine level are gathered at once (16 loads in flight per lane),
//    while the other stream (LDS levels) computes: two gather round trips per tile.
// Per (query, head), each level's 16 taps are summed as f16 pairs by v_pk_fma_f16 (2 MACs per
// instruction; 11-bit significand, above the bf16 compute dtype's 8) and added into f32
// accumulators level by level (fixed order: deterministic).
#include <hip/hip_runtime.h>

#include <math.h>

#include <algorithm>
#include <type_traits>

#include "../../include/kinet_msda.h"
#include "common.h"
#include "msda_util.h"

namespace kinet {
namespace {

constexpr int EW = 16;             // waves per workgroup (one workgroup per CU)
constexpr int EQT = 16;            // queries per wave tile
constexpr int EMAP_ROWS = 2400;    // LDS map rows of 64 B incl. the zero margins (153,600 B)
constexpr int EL = 4, EP = 4;      // levels, points (the configs' values; host-checked)
constexpr int EREC = EL * EP * 3;  // head-major offsets/logits per query and head (48)

struct EncLevels {
    int start[EL], H[EL], W[EL], ok[EL];
    float Hf[EL], Wf[EL], rH[EL], rW[EL];
    int lc;       // first LDS-resident level (EL: none)
    int mstart;   // its token offset in the head map
    int npix;     // staged pixels
    int mtop;     // zero rows before (and after) them: max staged W + 1
};

struct EncArgs {
    const f16_t* value;    // head map (b, m) at value + b*vsb + m*vsm, pixel rows of 32 f16
    long vsb, vsm;
    int head_bytes;        // bytes addressable from a head map's base (buffer range)
    int H[EL], W[EL];      // level shapes (host copy of spatial_shapes)
    int lc;                // first LDS-resident level (host-computed)
    const f16_t* offlog;   // (M, B, Lq, 48) head-major
    const float* ref;      // (B, Lq, L, ref_dim)
    const uint8_t* qmask;  // (B, Lq) or null
    void* out;             // (B, Lq, M*32) row-major
    const int* torder;     // processing order of the 16-query tiles (or null)
    int S, B, M, Lq, nchunk, ref_dim;
};

// quad broadcast: every lane of a quad takes lane `SRC` of its quad
template <int SRC>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, SRC * 0x55, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t pk_fma_lo(uint32_t acc, uint32_t v, uint32_t w) {
    asm("v_pk_fma_f16 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(acc) : "v"(v), "v"(w));
    return acc;
}
__device__ __forceinline__ uint32_t pk_fma_hi(uint32_t acc, uint32_t v, uint32_t w) {
    asm("v_pk_fma_f16 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(v), "v"(w));
    return acc;
}
__device__ __forceinline__ uint32_t pk_mul_lo(uint32_t v, uint32_t w) {
    uint32_t d;
    asm("v_pk_mul_f16 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(d) : "v"(v), "v"(w));
    return d;
}

// one level's 4 points x 4 corners x 8 channels into f16 pairs h (first corner: a multiply)
__device__ __forceinline__ void level_sum16(uint32_t (&h)[4], const u32x4v (&v)[4][4], const uint32_t (&w01)[4],
                                            const uint32_t (&w23)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) h[j] = pk_mul_lo(v[0][0][j], w01[0]);
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (p > 0) h[j] = pk_fma_lo(h[j], v[p][0][j], w01[p]);
            h[j] = pk_fma_hi(h[j], v[p][1][j], w01[p]);
            h[j] = pk_fma_lo(h[j], v[p][2][j], w23[p]);
            h[j] = pk_fma_hi(h[j], v[p][3][j], w23[p]);
        }
}

// the level's f16 pair sums into the f32 accumulators (v_fma_mix with an f16 1.0)
__device__ __forceinline__ void flush16(f32x2 (&acc)[4], const uint32_t (&h)[4]) {
    constexpr uint32_t one = 0x3c003c00u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        acc[j][0] = fma_mix16_lo_lo(acc[j][0], h[j], one);
        acc[j][1] = fma_mix16_hi_lo(acc[j][1], h[j], one);
    }
}

// phase-1 inputs of one tile (this lane: query lane >> 2, level lane & 3)
struct TileIn {
    u32x4v off;     // 4 points x (x, y) f16
    uint2 lg;       // 4 logits f16
    float4 r;       // reference point (x, y[, w, h])
    uint32_t qm;    // query mask byte
};

template <int REFD, bool QM>
__device__ __forceinline__ void load_tile(TileIn& in, const __amdgpu_buffer_rsrc_t& ro,
                                          const __amdgpu_buffer_rsrc_t& rr, const __amdgpu_buffer_rsrc_t& rq,
                                          int b, int Lq, int q, int l) {
    const uint32_t qq = (uint32_t)(q < Lq ? q : Lq - 1);
    const uint32_t ob = qq * (uint32_t)(EREC * 2);
    in.off = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(ro, ob + (uint32_t)l * 16u, 0, 0));
    in.lg = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(ro, ob + 64u + (uint32_t)l * 8u, 0, 0));
    const uint32_t row = (uint32_t)b * (uint32_t)Lq + qq;
    const uint32_t rb = (row * (uint32_t)EL + (uint32_t)l) * (uint32_t)REFD * 4u;
    if constexpr (REFD == 2) {
        const float2 r2 = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rr, rb, 0, 0));
        in.r = make_float4(r2.x, r2.y, 0.f, 0.f);
    } else {
        in.r = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rr, rb, 0, 0));
    }
    in.qm = QM ? __builtin_amdgcn_raw_buffer_load_b8(rq, row, 0, 0) : 0u;
}

// Phase 1: softmax over the query's 16 logits (4 in this lane, 4 lanes of the quad;
// ms_deform_attn.py:70-74), sampling locations (:77-82) and the bilinear setup of cuh:227-233
// for this lane's level: per point, the byte offset of the top-left corner (map-relative;
// a corner outside the level keeps an address -- a neighbouring pixel, a zero margin row of the
// LDS map, or past the buffer range, which reads 0 -- and gets weight 0) + 4 f16 weights.
template <int REFD>
__device__ __forceinline__ void setup_tile(const TileIn& in, const EncLevels& lv, int l, bool ok, uint32_t (&ro)[4],
                                           uint32_t (&rw01)[4], uint32_t (&rw23)[4]) {
    float lg[EP], ox[EP], oy[EP];
#pragma unroll
    for (int p = 0; p < EP; ++p) {
        ox[p] = (float)__builtin_bit_cast(f16_t, (uint16_t)(in.off[p] & 0xffffu));
        oy[p] = (float)__builtin_bit_cast(f16_t, (uint16_t)(in.off[p] >> 16));
        const uint32_t gw = p < 2 ? in.lg.x : in.lg.y;
        lg[p] = (float)__builtin_bit_cast(f16_t, (uint16_t)((p & 1) ? (gw >> 16) : (gw & 0xffffu)));
    }
    float mx = fmaxf(fmaxf(lg[0], lg[1]), fmaxf(lg[2], lg[3]));
    mx = group_reduce<4, true>(mx);
    float e[EP], es = 0.f;
#pragma unroll
    for (int p = 0; p < EP; ++p) {
        e[p] = __expf(lg[p] - mx);
        es += e[p];
    }
    es = group_reduce<4, false>(es);
    const float ra = (in.qm || !ok) ? 0.f : __builtin_amdgcn_rcpf(es);
    const bool in_lds = l >= lv.lc;
    const int H = lv.H[l], W = lv.W[l];
    const int pbase = in_lds ? (lv.mtop + lv.start[l] - lv.mstart) * 64 : lv.start[l] * 64;
    const uint32_t zoff = in_lds ? 0u : 0x80000000u;
    const float Hf = lv.Hf[l], Wf = lv.Wf[l], rH = lv.rH[l], rW = lv.rW[l];
    const bool lok = lv.ok[l] != 0;
#pragma unroll
    for (int p = 0; p < EP; ++p) {
        float x, y;
        if constexpr (REFD == 2) {   // offsets / spatial_shapes[(H, W)] on (x, y): the reference's quirk (:77-79)
            x = in.r.x + ox[p] * rH;
            y = in.r.y + oy[p] * rW;
        } else {                     // :80-82
            x = in.r.x + ox[p] * (0.5f / (float)EP) * in.r.z;
            y = in.r.y + oy[p] * (0.5f / (float)EP) * in.r.w;
        }
        const float a = e[p] * ra;
        const float h = y * Hf - 0.5f, w = x * Wf - 0.5f;                    // cuh:227-228
        const bool valid = lok && h > -1.f && w > -1.f && h < Hf && w < Wf;   // cuh:229
        const float hf = floorf(h), wf = floorf(w);
        const int hl = valid ? (int)hf : 0, wl = valid ? (int)wf : 0;
        const float lh = h - hf, lw = w - wf, hh = 1.f - lh, hw = 1.f - lw;
        const bool h0 = hl >= 0, h1 = hl + 1 < H, c0 = wl >= 0, c1 = wl + 1 < W;
        const float av = valid ? a : 0.f;
        ro[p] = valid ? (uint32_t)(pbase + (__mul24(hl, W) + wl) * 64) : zoff;
        rw01[p] = pack_f16x2((h0 && c0) ? hh * hw * av : 0.f, (h0 && c1) ? hh * lw * av : 0.f);
        rw23[p] = pack_f16x2((h1 && c0) ? lh * hw * av : 0.f, (h1 && c1) ? lh * lw * av : 0.f);
    }
}

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

template <typename TO, int LC, int REFD, bool QM>
__device__ __forceinline__ void enc_tiles(const EncArgs& a, const EncLevels& lv, const u32x4v* vmap, int b, int m,
                                          int chunk, int wave, int lane) {
    constexpr int NGL = LC;            // levels gathered through the texture path
    constexpr int NLL = EL - LC;       // levels read from LDS
    constexpr int NST = NGL > NLL ? NGL : NLL;
    const int Lq = a.Lq, ntile = (Lq + EQT - 1) / EQT;
    const int stride = a.nchunk * EW;
    const int qi = lane >> 2, l1 = lane & 3;
    const uint32_t cb = (uint32_t)l1 * 16u;      // phase 2: this lane's 8 channels, bytes
    const char* hmap = reinterpret_cast<const char*>(a.value + (long)b * a.vsb + (long)m * a.vsm);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)hmap, (short)0, a.head_bytes, 0x00020000);
    const f16_t* omap = a.offlog + ((long)m * a.B + b) * (long)Lq * EREC;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)omap, (short)0, Lq * EREC * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.ref, (short)0, a.B * Lq * EL * REFD * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rq =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.qmask, (short)0, a.qmask ? a.B * Lq : 0, 0x00020000);
    const char* vm = reinterpret_cast<const char*>(vmap) + cb;
    int wb[EL];
#pragma unroll
    for (int l = 0; l < EL; ++l) wb[l] = lv.W[l] * 64;

    int t = chunk * EW + wave;
    if (t >= ntile) return;
    auto tile_q0 = [&](int tt) { return (a.torder ? a.torder[tt] : tt) * EQT; };
    TileIn in;
    int q0 = tile_q0(t);
    load_tile<REFD, QM>(in, ro, rr, rq, b, Lq, q0 + qi, l1);
    uint32_t rec_o[EP], rec_w01[EP], rec_w23[EP];
    setup_tile<REFD>(in, lv, l1, q0 + qi < Lq, rec_o, rec_w01, rec_w23);
#pragma unroll 1
    for (;;) {
        const int tn = t + stride;
        const bool more = tn < ntile;
        const int qn0 = more ? tile_q0(tn) : 0;
        f32x2 acc[4] = {};
        u32x4v g[EP][4];
        // fine level LV: its 4 points' records from quad lane LV, 16 corner loads in flight
        auto issue = [&](auto lvc) {
            constexpr int LV = decltype(lvc)::value;
#pragma unroll
            for (int p = 0; p < EP; ++p) {
                const uint32_t o = quad_bcast<LV>(rec_o[p]) + cb;
                const uint32_t o1 = o + (uint32_t)wb[LV];
                g[p][0] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, o, 0, 0));
                g[p][1] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, o + 64u, 0, 0));
                g[p][2] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, o1, 0, 0));
                g[p][3] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, o1 + 64u, 0, 0));
            }
        };
        // the gathered level: weights fetched from the quad again (registers are the limit)
        auto consume = [&](auto lvc) {
            constexpr int LV = decltype(lvc)::value;
            uint32_t w01[EP], w23[EP], h[4];
#pragma unroll
            for (int p = 0; p < EP; ++p) {
                w01[p] = quad_bcast<LV>(rec_w01[p]);
                w23[p] = quad_bcast<LV>(rec_w23[p]);
            }
            level_sum16(h, g, w01, w23);
            flush16(acc, h);
        };
        // coarse level LV from the LDS map, one point at a time (16 VGPRs beside the gathers)
        auto lds_level = [&](auto lvc) {
            constexpr int LV = decltype(lvc)::value;
            uint32_t h[4];
#pragma unroll
            for (int p = 0; p < EP; ++p) {
                const uint32_t o = quad_bcast<LV>(rec_o[p]);
                const uint32_t w01 = quad_bcast<LV>(rec_w01[p]);
                const uint32_t w23 = quad_bcast<LV>(rec_w23[p]);
                const char* r0 = vm + o;
                const char* r1 = r0 + wb[LV];
                // a corner pair at a time (8 VGPRs beside the gathers in flight)
                const u32x4v v0 = *reinterpret_cast<const u32x4v*>(r0);
                const u32x4v v1 = *reinterpret_cast<const u32x4v*>(r0 + 64);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    h[j] = p == 0 ? pk_mul_lo(v0[j], w01) : pk_fma_lo(h[j], v0[j], w01);
                    h[j] = pk_fma_hi(h[j], v1[j], w01);
                }
                __builtin_amdgcn_sched_barrier(0);
                const u32x4v v2 = *reinterpret_cast<const u32x4v*>(r1);
                const u32x4v v3 = *reinterpret_cast<const u32x4v*>(r1 + 64);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    h[j] = pk_fma_lo(h[j], v2[j], w23);
                    h[j] = pk_fma_hi(h[j], v3[j], w23);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            flush16(acc, h);
        };
        static_for<0, NST>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            if constexpr (s < NGL) issue(std::integral_constant<int, s>{});
            if constexpr (s == 0) {
                // the next tile's phase-1 inputs, behind this tile's first gathers
                if (more) load_tile<REFD, QM>(in, ro, rr, rq, b, Lq, qn0 + qi, l1);
            }
            if constexpr (s < NLL) lds_level(std::integral_constant<int, LC + s>{});
            if constexpr (s < NGL) consume(std::integral_constant<int, s>{});
        });
        const int q = q0 + qi;
        if (q < Lq) {
            VecT<TO, 8> o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o.v[2 * j] = Cvt<TO>::from(acc[j][0]);
                o.v[2 * j + 1] = Cvt<TO>::from(acc[j][1]);
            }
            *reinterpret_cast<VecT<TO, 8>*>(static_cast<TO*>(a.out) + ((long)b * Lq + q) * a.M * 32 + (long)m * 32 +
                                            l1 * 8) = o;
        }
        if (!more) break;
        t = tn;
        q0 = qn0;
        setup_tile<REFD>(in, lv, l1, q0 + qi < Lq, rec_o, rec_w01, rec_w23);
    }
}

template <typename TO, int LC, int REFD, bool QM>
__global__ __launch_bounds__(EW * 64) void msda_enc_kernel(const EncArgs a) {
    constexpr int NT = EW * 64;
    __shared__ EncLevels lv;
    __shared__ u32x4v vmap[EMAP_ROWS * 4];
    // XCD-aware remap (cdna_hip_programming.md T1): the query chunks of one (frame, head)
    // map run on one XCD and share its L2.  Assumes MI355X's 8 XCDs with round-robin dispatch;
    // elsewhere the mapping is still a bijection (only the L2 grouping is lost).
    int b, m, chunk;
    {
        const int nblk = gridDim.x, lin = blockIdx.x;
        const int qd = nblk >> 3, rm = nblk & 7, xcd = lin & 7;
        const int nid = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + (lin >> 3);
        chunk = nid % a.nchunk;
        const int bm = nid / a.nchunk;
        b = bm / a.M;
        m = bm % a.M;
    }
    if (threadIdx.x == 0) {
        int acc = 0, wmax = 0;
        for (int l = 0; l < EL; ++l) {
            const int H = a.H[l], W = a.W[l];
            lv.start[l] = acc;
            lv.H[l] = H;
            lv.W[l] = W;
            lv.ok[l] = 1;
            lv.Hf[l] = (float)H;
            lv.Wf[l] = (float)W;
            lv.rH[l] = 1.f / (float)H;
            lv.rW[l] = 1.f / (float)W;
            if (l >= LC) wmax = W > wmax ? W : wmax;
            acc += H * W;
        }
        // levels LC.. staged with max W + 1 zero rows before and after them (the rows a
        // corner of an edge pixel can address); the host checked that they fit
        lv.lc = LC;
        lv.mstart = LC < EL ? lv.start[LC] : 0;
        lv.npix = LC < EL ? acc - lv.start[LC] : 0;
        lv.mtop = LC < EL ? wmax + 1 : 0;
    }
    __syncthreads();
    {
        const char* hmap = reinterpret_cast<const char*>(a.value + (long)b * a.vsb + (long)m * a.vsm);
        const int npix = lv.npix, mstart = lv.mstart, mtop = lv.mtop;
        const int rows = npix + 2 * mtop;
        for (int i = threadIdx.x; i < rows * 4; i += NT) {
            const int p = (i >> 2) - mtop;
            u32x4v v = {0u, 0u, 0u, 0u};
            if (p >= 0 && p < npix) v = *reinterpret_cast<const u32x4v*>(hmap + (long)(mstart + p) * 64 + (i & 3) * 16);
            vmap[i] = v;
        }
    }
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    enc_tiles<TO, LC, REFD, QM>(a, lv, vmap, b, m, chunk, wave, lane);
}

}  // namespace
}  // namespace kinet

using namespace kinet;

extern "C" int kinet_msda_encoder_forward(const void* value, int64_t value_sb, int64_t value_sm,
                                          const int64_t* spatial_shapes_host, const void* offsets_logits_hm,
                                          const float* ref_points, int ref_dim, const uint8_t* query_attn_mask,
                                          void* output, int batch, int spatial_size, int num_heads, int channels,
                                          int num_levels, int num_query, int num_point, int output_dtype,
                                          const int32_t* query_tile_order, kinet_stream_t stream) {
    KINET_CHECK_ARG(batch >= 0 && spatial_size > 0 && num_heads > 0 && num_query >= 0, "msda encoder: bad sizes");
    KINET_CHECK_ARG(channels == 32 && num_levels == EL && num_point == EP,
                    "msda encoder: head_dim 32, 4 levels, 4 points (got %d, %d, %d)", channels, num_levels, num_point);
    KINET_CHECK_ARG(ref_dim == 2 || ref_dim == 4, "Last dim of reference_points must be 2 or 4, but get %d instead.", ref_dim);
    KINET_CHECK_ARG(output_dtype == KINET_BF16 || output_dtype == KINET_F16, "msda encoder: output must be bf16 or f16");
    KINET_CHECK_ARG(((uintptr_t)value % 16) == 0 && ((uintptr_t)offsets_logits_hm % 16) == 0 && value_sb % 8 == 0 &&
                        value_sm % 8 == 0,
                    "msda encoder: value / offsets must be 16-byte aligned");
    KINET_CHECK_ARG(spatial_shapes_host != nullptr, "msda encoder: spatial_shapes_host is NULL");
    long long npix = 0;
    for (int l = 0; l < EL; ++l) {
        KINET_CHECK_ARG(spatial_shapes_host[2 * l] > 0 && spatial_shapes_host[2 * l + 1] > 0 &&
                            spatial_shapes_host[2 * l] * spatial_shapes_host[2 * l + 1] < (1LL << 30),
                        "msda encoder: bad level shape");
        npix += spatial_shapes_host[2 * l] * spatial_shapes_host[2 * l + 1];
    }
    KINET_CHECK_ARG(npix == spatial_size, "msda encoder: spatial_shapes cover %lld tokens, value has %d", npix,
                    spatial_size);
    // the coarsest suffix of levels that fits the LDS map with its zero margins
    int lc = EL;
    {
        long long np = 0;
        int wmax = 0;
        for (int l = EL - 1; l >= 0; --l) {
            const long long n = np + spatial_shapes_host[2 * l] * spatial_shapes_host[2 * l + 1];
            const int wm = std::max<int>(wmax, (int)spatial_shapes_host[2 * l + 1]);
            if (n + 2LL * (wm + 1) > EMAP_ROWS) break;
            np = n;
            wmax = wm;
            lc = l;
        }
    }
    KINET_CHECK_ARG(lc < EL, "msda encoder: the coarsest level does not fit the LDS map (use kinet_msda_fused_forward)");
    if (batch == 0 || num_query == 0) return KINET_OK;
    const long long head_bytes = (long long)spatial_size * 64;
    KINET_CHECK_ARG(head_bytes < (1LL << 31) && (long long)num_query * EREC * 2 < (1LL << 31) &&
                        (long long)batch * num_query < (1LL << 24) &&
                        (long long)batch * num_query * EL * ref_dim * 4 < (1LL << 31),
                    "msda encoder: problem too large for 32-bit buffer offsets");
    EncArgs a{};
    a.value = (const f16_t*)value;
    a.vsb = (long)value_sb;
    a.vsm = (long)value_sm;
    a.head_bytes = (int)head_bytes;
    for (int l = 0; l < EL; ++l) {
        a.H[l] = (int)spatial_shapes_host[2 * l];
        a.W[l] = (int)spatial_shapes_host[2 * l + 1];
    }
    a.lc = lc;
    a.offlog = (const f16_t*)offsets_logits_hm;
    a.ref = ref_points;
    a.qmask = query_attn_mask;
    a.out = output;
    a.torder = (const int*)query_tile_order;
    a.S = spatial_size;
    a.B = batch;
    a.M = num_heads;
    a.Lq = num_query;
    a.ref_dim = ref_dim;
    // one round of one-per-CU workgroups: the fewest query chunks per head map whose
    // workgroups fill >= 90 % of their last round (config 2, batch 16: 128 maps x 2 = one round)
    const int cus = cu_count();
    const int maps = batch * num_heads;
    const int ntile = (num_query + EQT - 1) / EQT;
    const int base = (cus + maps - 1) / maps;
    int nchunk = base;
    for (int c = base; c <= 4 * base; ++c) {
        const long long wgs = (long long)maps * c, rounds = (wgs + cus - 1) / cus;
        if (wgs * 10 >= rounds * cus * 9) {
            nchunk = c;
            break;
        }
    }
    nchunk = std::max(1, std::min(nchunk, (ntile + EW - 1) / EW));
    KINET_CHECK_ARG((long long)maps * nchunk < (1LL << 31), "msda encoder: grid too large");
    a.nchunk = nchunk;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(maps * nchunk), block(EW * 64);
#define EK(TO_, LC_, RD_, QM_) hipLaunchKernelGGL((msda_enc_kernel<TO_, LC_, RD_, QM_>), grid, block, 0, s, a)
#define EK_QM(TO_, LC_, RD_) if (query_attn_mask) EK(TO_, LC_, RD_, true); else EK(TO_, LC_, RD_, false)
#define EK_RD(TO_, LC_) if (ref_dim == 2) { EK_QM(TO_, LC_, 2); } else { EK_QM(TO_, LC_, 4); }
#define EK_LC(TO_)                        \
    switch (lc) {                         \
        case 0: EK_RD(TO_, 0) break;      \
        case 1: EK_RD(TO_, 1) break;      \
        case 2: EK_RD(TO_, 2) break;      \
        default: EK_RD(TO_, 3) break;     \
    }
    if (output_dtype == KINET_BF16) {
        EK_LC(bf16_t)
    } else {
        EK_LC(f16_t)
    }
#undef EK_LC
#undef EK_RD
#undef EK_QM
#undef EK
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}
