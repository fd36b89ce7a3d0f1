// Encoder-sized MSDeformAttn sampling (MSDeformAttn.forward, ms_deform_attn.py:69-87, with the
// sampling of ms_deform_im2col_cuda.cuh:165-237) for gfx950: one workgroup per CU owns one
// horizontal STRIP of one (frame, head) value map -- the queries of a contiguous range of the
// row-sorted tile order -- with the rows of the coarse levels that strip samples staged in LDS.
// kinet_msda_encoder_forward / kinet_msda_encoder_plan (include/kinet_msda.h).
//
// Why this shape: at the config-2 encoder call (batch 16, Lq = S = 22,223,
// 8 heads x 32 channels, 4 levels x 4 points) every query gathers 16 samples x 4 corners x
// 64 B = 11.6 GB of corner rows per call.  Through the texture path (one 64-B row per 4 lanes
// of a buffer_load_b128) those gathers are what bounds the kernel (TA ~72 % busy in the
// round-2/3 kernels, which kept only the two coarsest levels -- 85 KB of a head map -- in LDS
// and gathered levels 0 and 1 from HBM/L2).  A strip of 1/8 of the image needs only ~17 rows
// of level 1 (+ a halo for the sampling offsets), ~14 of level 2 and the whole of level 3:
// ~150 KB, so levels 1-3 are read from LDS (ds_read_b128) and only level 0 goes through the
// texture path -- half the gather instructions per tile and ONE gather round trip per tile
// instead of two.  A sample whose 2x2 footprint leaves the staged rows (an offset beyond the
// halo) is gathered from the head map instead: any sampling pattern is correct, the staged
// halo only decides the speed.
//  * offsets / logits arrive HEAD-MAJOR (M, B, Lq, 48) f16 [32 offsets (l, p, xy) | 16 logits
//    (l, p)] from the projection GEMM's head-major epilogue: a 16-query tile of one head is
//    1.5 KB contiguous (two vector loads per lane);
//  * the tile's phase-1 loads for tile t+1 are issued while tile t gathers;
//  * tap records stay in registers: phase-1 lane (query, level) holds its level's 4 point
//    records, phase-2 lane (query, channel group) fetches them with a quad-broadcast DPP move
//    (same quad = same query in both phases), so no LDS record traffic and no barrier;
//  * the staged rows are filled by LDS-DMA (buffer_load ... lds; rows outside the image and
//    padding are the buffer range check's zeros) while the first tile's level-0 gathers fly.
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
constexpr int EMAP_PIX = 2544;     // LDS map pixels of 64 B (162,816 B; the level table fits beside)
// head_dim 36 (TAIL): the value as a 32-channel plane + a 4-channel TAIL plane (8 B per pixel,
// kinet_gemm_headmajor_split); the LDS map holds both, 72 B per pixel: 2256 main pixels, then the
// tail map (pixel x at ETB + 8x, the same pixel indexing as the main map).  Both fills round up
// (main: pieces of 16 pixels, tail: 256-byte pieces), so the main budget is a multiple of 16 (its
// last piece must not reach the tail map) and the tail's rounded fill stays inside the array
constexpr int EMAP_T = 2256;
constexpr int ETB = EMAP_T * 64;
static_assert(EMAP_T % 16 == 0 && ETB + (EMAP_T * 2 + 63) / 64 * 256 <= EMAP_PIX * 64, "tail map layout");
constexpr int EWT = 12;   // TAIL: waves per workgroup (3 per SIMD: the tail's registers need > 128 VGPRs)
constexpr int EL = 4, EP = 4;      // levels, points (the configs' values; host-checked)
constexpr int EREC = EL * EP * 3;  // head-major offsets/logits per query and head (48)
constexpr int EHALO = 4;           // rows staged beyond a strip's query rows on each side
constexpr uint32_t TAF = 0x80000000u;
#ifndef KINET_ENC_DYN
#define KINET_ENC_DYN 1
#endif   // record flag: an LDS level's sample gathered from HBM

// one level's constants as phase 1 reads them: 48 contiguous bytes = three ds_read_b128 from one
// address per lane (its level), instead of eleven ds_read_b32 of the per-field arrays
struct alignas(16) LevelRec {
    int start, H, W, ok;
    float Hf, Wf, rH, rW;
    int r0, r1, lb, pad;   // staged rows [r0, r1] and the LDS map base (LDS levels)
};

struct EncLevels {
    int start[EL], H[EL], W[EL], ok[EL];
    float Hf[EL], Wf[EL], rH[EL], rW[EL];
    int ra[EL];   // LDS level: first staged row (-1 = the zero row above the image)
    int rn[EL];   // LDS level: staged rows
    int lb[EL];   // LDS level: map pixel of (row r, col c) = lb + r*W + c
    LevelRec rec[EL];
    int next_tile;   // the strip's next unclaimed tile (waves claim tiles as they finish one)
};

// launch plan (host): levels [0, fl) are gathered from the head map, levels [fl, EL) staged
// per strip: region l = 1 margin pixel + cap[l] rows x W + 1 margin pixel at map pixel base[l]
struct EncPlan {
    int fl, nstrip, zpix, used;
    int cap[EL], base[EL];
};

struct EncArgs {
    const f16_t* value;    // head map (b, m) at value + b*vsb + m*vsm, pixel rows of 32 f16
    long vsb, vsm;
    int head_bytes;        // bytes addressable from a head map's base (buffer range)
    const f16_t* tail;     // TAIL: the 4-channel plane, head map (b, m) at tail + b*tsb + m*tsm
    long tsb, tsm;
    int tail_bytes;
    int od;                // output channels per head (32, or 36 with the tail)
    int H[EL], W[EL];      // level shapes (host copy of spatial_shapes)
    int cap[EL], base[EL]; // the plan's LDS regions
    const f16_t* offlog;   // (M, B, Lq, 48) head-major
    const float* ref;      // (B, Lq, L, ref_dim)
    const uint8_t* qmask;  // (B, Lq) or null
    void* out;             // (B, Lq, M*32) row-major
    const int* torder;     // processing order of the 16-query tiles (or null)
    int S, B, M, Lq, nstrip, used, ref_dim;
    int fb;                // sampling records (REC): fraction bits of the fixed-point locations
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

// the level's f16 pair sums into the f32 accumulators (v_fma_mix with an f16 1.0); the tile's
// first level widens them instead (exact, and no zeroed accumulators to add to)
template <bool FIRST = false>
__device__ __forceinline__ void flush16(f32x2 (&acc)[4], const uint32_t (&h)[4]) {
    constexpr uint32_t one = 0x3c003c00u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if constexpr (FIRST) {
            acc[j][0] = (float)__builtin_bit_cast(f16_t, (uint16_t)(h[j] & 0xffffu));
            acc[j][1] = (float)__builtin_bit_cast(f16_t, (uint16_t)(h[j] >> 16));
        } else {
            acc[j][0] = fma_mix16_lo_lo(acc[j][0], h[j], one);
            acc[j][1] = fma_mix16_hi_lo(acc[j][1], h[j], one);
        }
    }
}

// max / sum over the 4 lanes of a quad, every lane active (phase 1): plain DPP moves, no
// zeroed "old" operand
template <bool MAX>
__device__ __forceinline__ float quad_reduce(float x) {
    const float a = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xf, 0xf, false));
    x = MAX ? fmaxf(x, a) : x + a;
    const float c = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xf, 0xf, false));
    return MAX ? fmaxf(x, c) : x + c;
}

// phase-1 inputs of one tile (this lane: query lane >> 2, level lane & 3)
struct TileIn {
    u32x4v off;     // 4 points x (x, y) f16
    uint2 lg;       // 4 logits f16
    float4 r;       // reference point (x, y[, w, h])
    uint32_t qm;    // query mask byte
};

// (REC: off = the 4 fixed-point locations, lg = the 4 f16 weights of kinet_msda_sample_records,
// same offsets in the 96-byte row; no reference point or mask: folded into the records)
template <int REFD, bool QM, bool REC = false>
__device__ __forceinline__ void load_tile(TileIn& in, const __amdgpu_buffer_rsrc_t& ro,
                                          const __amdgpu_buffer_rsrc_t& rr, const __amdgpu_buffer_rsrc_t& rq,
                                          int b, int Lq, int q, int l) {
    const uint32_t qq = (uint32_t)(q < Lq ? q : Lq - 1);
    const uint32_t ob = qq * (uint32_t)(EREC * 2);
    in.off = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(ro, ob + (uint32_t)l * 16u, 0, 0));
    in.lg = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(ro, ob + 64u + (uint32_t)l * 8u, 0, 0));
    if constexpr (REC) return;
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
// for this lane's level: per point, the byte offset of the top-left corner + 4 f16 weights.
//  * gathered level (l < FL): map-relative offset; a corner outside the level keeps an address
//    (a neighbouring pixel, or past the buffer range, which reads 0) and gets weight 0;
//  * LDS level: offset into the LDS map when both rows of the footprint are staged; else
//    TAF | (map offset of corner (hl+1, wl+1)) -- non-negative for every footprint that touches
//    the level, its other corners (-64, -W*64, -(W+1)*64) wrap past the range when outside;
//    a sample outside the level points at the zero margin (offset 0) with zero weights.
template <int FL, int REFD>
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
    mx = quad_reduce<true>(mx);
    float e[EP], es = 0.f;
#pragma unroll
    for (int p = 0; p < EP; ++p) {
        e[p] = __expf(lg[p] - mx);
        es += e[p];
    }
    es = quad_reduce<false>(es);
    const float ra = (in.qm || !ok) ? 0.f : __builtin_amdgcn_rcpf(es);
    const bool in_lds = l >= FL;
    const LevelRec L = lv.rec[l];
    const int H = L.H, W = L.W;
    const int start = L.start;
    const int r0 = L.r0, r1 = L.r1;   // staged rows [r0, r1]
    const int lbase = L.lb;
    const float Hf = L.Hf, Wf = L.Wf, rH = L.rH, rW = L.rW;
    const bool lok = L.ok != 0;
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
        // branch-free (the level is lane-divergent: lane & 3): both address forms and a select
        const int pix = __mul24(hl, W) + wl;
        const uint32_t gofs = (uint32_t)(start + pix) * 64u;                  // head-map offset of (hl, wl)
        const uint32_t lo = (uint32_t)(lbase + pix) * 64u;                    // LDS map offset
        const uint32_t go = TAF | (gofs + (uint32_t)(W + 1) * 64u);           // far: corner (hl+1, wl+1)
        const bool staged = hl >= r0 && hl < r1;
        const uint32_t lds_o = staged ? lo : go;
        ro[p] = valid ? (in_lds ? lds_o : gofs) : (in_lds ? 0u : TAF);
        rw01[p] = pack_f16x2((h0 && c0) ? hh * hw * av : 0.f, (h0 && c1) ? hh * lw * av : 0.f);
        rw23[p] = pack_f16x2((h1 && c0) ? lh * hw * av : 0.f, (h1 && c1) ? lh * lw * av : 0.f);
    }
}

// Phase 1 from sampling records (kinet_msda_sample_records: softmax, locations, out-of-level
// corners and samples already folded into the weights): per point, unpack the fixed-point
// location, build the 4 corner weights in packed f16 and choose the address -- no bounds tests.
//   X = (1 + lw, 1 + lh) as f16: the fraction bits shifted into the mantissa of 1.0;
//   HL = (1 - lh, lh), WL = (1 - lw, lw); A = HL * a; rw01 = WL * A.lo, rw23 = WL * A.hi.
struct RecK {
    uint32_t sh_h, fmask2, sh2, wbits;   // 16 + fb, the two fraction fields, (10 - fb) per half, 16 - fb
};
__device__ __forceinline__ uint32_t pk_lsl16(uint32_t x, uint32_t sh2) {
    uint32_t d;
    asm("v_pk_lshlrev_b16 %0, %1, %2" : "=v"(d) : "s"(sh2), "v"(x));
    return d;
}
// (1 - X.hi, X.hi - 1) and (1 - X.lo, X.lo - 1) for X = (1 + lw, 1 + lh): (2 - x, x - 1)
__device__ __forceinline__ uint32_t pk_frac_hi(uint32_t x, uint32_t c) {
    uint32_t d;
    asm("v_pk_add_f16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[1,0]" : "=v"(d) : "v"(x), "s"(c));
    return d;
}
__device__ __forceinline__ uint32_t pk_frac_lo(uint32_t x, uint32_t c) {
    uint32_t d;
    asm("v_pk_add_f16 %0, %1, %2 op_sel:[0,0] op_sel_hi:[0,1] neg_lo:[1,0]" : "=v"(d) : "v"(x), "s"(c));
    return d;
}
template <int HALF>
__device__ __forceinline__ uint32_t pk_mul_bcast(uint32_t x, uint32_t y) {   // x * (y.HALF, y.HALF)
    uint32_t d;
    if constexpr (HALF == 0) asm("v_pk_mul_f16 %0, %1, %2 op_sel:[0,0] op_sel_hi:[1,0]" : "=v"(d) : "v"(x), "v"(y));
    else asm("v_pk_mul_f16 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(d) : "v"(x), "v"(y));
    return d;
}

template <int FL>
__device__ __forceinline__ void setup_tile_rec(const TileIn& in, const EncLevels& lv, int l, const RecK& rk,
                                               uint32_t (&ro)[4], uint32_t (&rw01)[4], uint32_t (&rw23)[4]) {
    const bool in_lds = l >= FL;
    const LevelRec L = lv.rec[l];
    const uint32_t W = (uint32_t)L.W;
    const uint32_t st64 = (uint32_t)L.start * 64u, lb64 = (uint32_t)L.lb * 64u, far64 = (W + 1u) * 64u;
    const uint32_t r0 = (uint32_t)L.r0, rn = (uint32_t)(L.r1 - L.r0);
    constexpr uint32_t CF = 0xBC004000u;   // (2.0, -1.0) f16
#pragma unroll
    for (int p = 0; p < EP; ++p) {
        const uint32_t u = in.off[p];
        const uint32_t hl = u >> rk.sh_h;
        const uint32_t wl = __builtin_amdgcn_ubfe(u, 16u - rk.wbits, rk.wbits);
        const uint32_t x = pk_lsl16(u & rk.fmask2, rk.sh2) | 0x3C003C00u;
        const uint32_t hlw = pk_frac_hi(x, CF), wlw = pk_frac_lo(x, CF);
        const uint32_t aw = (p & 1) ? pk_mul_bcast<1>(hlw, p < 2 ? in.lg.x : in.lg.y)
                                    : pk_mul_bcast<0>(hlw, p < 2 ? in.lg.x : in.lg.y);
        rw01[p] = pk_mul_bcast<0>(wlw, aw);
        rw23[p] = pk_mul_bcast<1>(wlw, aw);
        const uint32_t pix = (uint32_t)__mul24((int)hl, (int)W) + wl;
        const uint32_t gofs = pix * 64u + st64;                              // head-map offset of (hl, wl)
        const uint32_t lo = pix * 64u + lb64;                                // LDS map offset
        const uint32_t go = TAF + (gofs + far64);                            // far: corner (hl+1, wl+1)
        const bool staged = hl - r0 < rn;                                    // rows hl, hl+1 staged
        ro[p] = in_lds ? (staged ? lo : go) : gofs;
    }
}

// the lane id recomputed where it is used (volatile: not hoisted out of the tile loop, so the
// lane-constant offsets derived from it cost a VALU op instead of a register across the loop)
__device__ __forceinline__ int lane_id_here() {
    int x;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(x));
    return x;
}

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

__device__ __forceinline__ float wave_min(float x) {
    x = fminf(x, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xf, 0xf, false)));
    x = fminf(x, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xf, 0xf, false)));
    x = fminf(x, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xf, 0xf, false)));
    x = fminf(x, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xf, 0xf, false)));
    x = fminf(x, __shfl_xor(x, 16));
    x = fminf(x, __shfl_xor(x, 32));
    return x;
}

// The strip's query rows, in normalised image height, from its level-0 queries (the bulk of
// them; coarser-level queries sample the same band) -- or from every tile's first query when
// the strip holds no level-0 query.  Every wave computes it (same result in each).
__device__ __forceinline__ void strip_rows(const EncArgs& a, const EncLevels& lv, int t0, int t1, int lane,
                                           float& ylo, float& yhi) {
    float lo0 = INFINITY, hi0 = INFINITY, loa = INFINITY, hia = INFINITY;   // hi kept negated
    const int end0 = min(lv.start[1], a.Lq);
    const int W0 = lv.W[0];
    for (int t = t0 + lane; t < t1; t += 64) {
        const int q0 = (a.torder ? a.torder[t] : t) * EQT;
        if (q0 < end0) {
            const int qb = min(q0 + EQT, end0) - 1;
            lo0 = fminf(lo0, ((float)(q0 / W0) + 0.5f) * lv.rH[0]);
            hi0 = fminf(hi0, -((float)(qb / W0) + 0.5f) * lv.rH[0]);
        }
        int l = 0;
#pragma unroll
        for (int k = 1; k < EL; ++k) l = q0 >= lv.start[k] ? k : l;
        const float y = ((float)((q0 - lv.start[l]) / lv.W[l]) + 0.5f) * lv.rH[l];
        loa = fminf(loa, y);
        hia = fminf(hia, -y);
    }
    lo0 = wave_min(lo0);
    hi0 = wave_min(hi0);
    loa = wave_min(loa);
    hia = wave_min(hia);
    const bool any0 = lo0 < INFINITY;
    ylo = any0 ? lo0 : loa;
    yhi = any0 ? -hi0 : -hia;
    if (!(ylo <= yhi)) {   // no tile (not planned): the whole height
        ylo = 0.f;
        yhi = 1.f;
    }
}

// TAIL (head_dim 36): the 4 tail channels of a query are summed by its quad too -- lane l1 takes
// corner (row l1 >> 1, column l1 & 1) of every footprint: one 8-byte read of that pixel's 4 tail
// channels per sample (vs four 16-byte main reads), two packed-f16 MACs with that corner's
// weight, per-level f16 pair sums widened into 4 f32 accumulators; at the tile's end the quad's 4
// corners are summed by two DPP steps and lane 0 of the quad stores the 4 channels
__device__ __forceinline__ void tail_flush(float (&t)[4], const uint32_t (&th)[2]) {
    constexpr uint32_t one = 0x3c003c00u;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        t[2 * j] = fma_mix16_lo_lo(t[2 * j], th[j], one);
        t[2 * j + 1] = fma_mix16_hi_lo(t[2 * j + 1], th[j], one);
    }
}
// the f16 weight of this lane's corner (row tr, column tc) in the low half
__device__ __forceinline__ uint32_t tail_w(uint32_t w01, uint32_t w23, int tr, int tc) {
    const uint32_t w = tr ? w23 : w01;
    return __builtin_amdgcn_alignbyte(w, w, (uint32_t)tc * 2u);
}
__device__ __forceinline__ void tail_mac(uint32_t (&th)[2], uint2 v, uint32_t wq, bool first) {
    th[0] = first ? pk_mul_lo(v.x, wq) : pk_fma_lo(th[0], v.x, wq);
    th[1] = first ? pk_mul_lo(v.y, wq) : pk_fma_lo(th[1], v.y, wq);
}

template <typename TO, int FL, int REFD, bool QM, bool REC, bool TAIL, int NW>
__device__ __forceinline__ void enc_tiles(const EncArgs& a, EncLevels& lv, u32x4v* vmap, int b, int m, int strip,
                                          int wave, int lane) {
    constexpr int NGL = FL;            // levels gathered through the texture path
    constexpr int NLL = EL - FL;       // levels read from LDS
    constexpr int NST = NGL > 1 ? NGL : 1;
    // the tile's first flush: LDS level FL when slot 0 holds one (below), else gathered level 0
    constexpr bool LDS_FIRST = NLL / NST > 0;
    const int Lq = a.Lq, ntile = (Lq + EQT - 1) / EQT;
    const int t0 = (int)((long)strip * ntile / a.nstrip), t1 = (int)((long)(strip + 1) * ntile / a.nstrip);
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
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(a.out, (short)0, a.B * Lq * a.M * a.od * 2, 0x00020000);
    const char* tmap = TAIL ? reinterpret_cast<const char*>(a.tail + (long)b * a.tsb + (long)m * a.tsm) : hmap;
    const __amdgpu_buffer_rsrc_t rt =
        __builtin_amdgcn_make_buffer_rsrc((void*)tmap, (short)0, TAIL ? a.tail_bytes : 0, 0x00020000);
    const int tr = l1 >> 1, tc = l1 & 1;   // TAIL: this lane's footprint corner

    const char* vm = reinterpret_cast<const char*>(vmap) + cb;
    const char* vmb = reinterpret_cast<const char*>(vmap);
    RecK rk;
    if constexpr (REC) {
        const uint32_t fb = (uint32_t)a.fb;
        rk.sh_h = 16u + fb;
        rk.fmask2 = ((1u << fb) - 1u) * 0x10001u;
        rk.sh2 = (10u - fb) * 0x10001u;
        rk.wbits = 16u - fb;
    }
    int wb[EL];
#pragma unroll
    for (int l = 0; l < EL; ++l) wb[l] = a.W[l] * 64;

    int t = t0 + wave;
    const bool has = t < t1;
    // the tile order read by scalar loads (lgkmcnt: never waits behind the gathers in flight)
    typedef __attribute__((address_space(4))) const int* cint_p;
    const cint_p tord = (cint_p)a.torder;
    auto tile_q0 = [&](int tt) {
        tt = __builtin_amdgcn_readfirstlane(tt);
        return (tord ? tord[tt] : tt) * EQT;
    };
    TileIn in;
    int q0 = has ? tile_q0(t) : 0;
    uint32_t rec_o[EP], rec_w01[EP], rec_w23[EP];
    u32x4v g[EP][4];
    uint2 gt[EP];   // TAIL: the gathered level's tail corner of each point
    // gathered level LV: its 4 points' records from quad lane LV, 16 corner loads in flight
    auto issue = [&](auto lvc) {
        constexpr int LV = decltype(lvc)::value;
#pragma unroll
        for (int p = 0; p < EP; ++p) {
            const uint32_t ob = quad_bcast<LV>(rec_o[p]);
            const uint32_t o = ob + cb;
            if constexpr (TAIL) {
                // head-map offset / 8 = tail-plane offset; this lane's corner is added in the
                // 64-byte domain first, where a footprint starting at row / column -1 wraps back
                // to its in-level corners exactly as the main loads' offsets do (the shift must
                // not see the wrapped value); an invalid sample's TAF offset lands past the tail
                // plane's range (reads 0)
                const uint32_t co = (tr ? (uint32_t)wb[LV] : 0u) + (uint32_t)tc * 64u;
                gt[p] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rt, (ob + co) >> 3, 0, 0));
            }
            const uint32_t o1 = o + (uint32_t)wb[LV];
            g[p][0] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, o, 0, 0));
            g[p][1] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, o + 64u, 0, 0));
            g[p][2] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, o1, 0, 0));
            g[p][3] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rv, o1 + 64u, 0, 0));
        }
    };
    // ---- the strip's staged rows (every wave derives the same values) ----
    float ylo, yhi;
    strip_rows(a, lv, t0, t1, lane, ylo, yhi);
    int ra_[EL], lb_[EL];
#pragma unroll
    for (int l = FL; l < EL; ++l) {
        const int H = a.H[l], W = a.W[l], cap = a.cap[l];
        const int hmin = (int)floorf(ylo * (float)H - 0.5f), hmax = (int)floorf(yhi * (float)H - 0.5f) + 1;
        int r = hmin - max(0, (cap - (hmax - hmin + 1)) / 2);
        r = max(-1, min(r, H + 1 - cap));
        ra_[l] = __builtin_amdgcn_readfirstlane(r);
        lb_[l] = a.base[l] + 1 - ra_[l] * W;
    }
    if (lane < EL) {   // identical values from every wave
        int r = lv.ra[lane], bb = lv.lb[lane];
#pragma unroll
        for (int l = FL; l < EL; ++l)
            if (lane == l) { r = ra_[l]; bb = lb_[l]; }
        if (lane >= FL) {
            lv.ra[lane] = r;
            lv.lb[lane] = bb;
        }
        LevelRec rc;
        rc.start = lv.start[lane];
        rc.H = lv.H[lane];
        rc.W = lv.W[lane];
        rc.ok = lv.ok[lane];
        rc.Hf = lv.Hf[lane];
        rc.Wf = lv.Wf[lane];
        rc.rH = lv.rH[lane];
        rc.rW = lv.rW[lane];
        rc.r0 = r;
        rc.r1 = r + lv.rn[lane] - 1;
        rc.lb = bb;
        rc.pad = 0;
        lv.rec[lane] = rc;
    }

    if (KINET_ENC_DYN && wave == 0 && lane == 0) lv.next_tile = t0 + NW;
    // the first tile's phase-1 inputs ahead of the DMA (so waiting for them does not wait for it)
    if (has) load_tile<REFD, QM, REC>(in, ro, rr, rq, b, Lq, q0 + qi, l1);
    // ---- LDS-DMA fill of the staged regions, in flight with the first tile's setup and gathers (pieces
    // of 16 map pixels = 1 KiB per wave-instruction; map pixels outside every region and rows
    // outside the image: the range check's zeros) ----
    {
        const int npiece = (a.used + 15) >> 4;
        for (int j = wave; j < npiece; j += NW) {
            const int x = j * 16 + (lane >> 2);
            uint32_t off = TAF;
#pragma unroll
            for (int l = FL; l < EL; ++l) {
                const int W = a.W[l];
                const int k = x - a.base[l] - 1;                  // -1 .. cap*W within the region
                const int rel = ra_[l] * W + k;                   // level pixel it mirrors
                const bool in = k >= -1 && k <= a.cap[l] * W && rel >= 0 && rel < a.H[l] * W;
                off = in ? (uint32_t)(lv.start[l] + rel) * 64u + (uint32_t)(lane & 3) * 16u : off;
            }
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (__attribute__((address_space(3))) void*)(vmap + j * 64), 16,
                                                     off, 0, 0, 0);
        }
        if constexpr (TAIL) {
            // the tail map: dword pieces (one dword = half a pixel's 4 channels), 256 B per
            // wave-instruction, the same pixel indexing and zero fill as the main map
            const int ndw = (a.used * 2 + 63) >> 6;
            for (int j = wave; j < ndw; j += NW) {
                const int dw = j * 64 + lane;
                const int x = dw >> 1;
                uint32_t off = TAF;
#pragma unroll
                for (int l = FL; l < EL; ++l) {
                    const int W = a.W[l];
                    const int k = x - a.base[l] - 1;
                    const int rel = ra_[l] * W + k;
                    const bool in = k >= -1 && k <= a.cap[l] * W && rel >= 0 && rel < a.H[l] * W;
                    off = in ? (uint32_t)(lv.start[l] + rel) * 8u + (uint32_t)(dw & 1) * 4u : off;
                }
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rt, (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(vmap) + ETB + j * 256), 4, off,
                    0, 0, 0);
            }
        }
    }

    if (has) {
        if constexpr (REC) setup_tile_rec<FL>(in, lv, l1, rk, rec_o, rec_w01, rec_w23);
        else setup_tile<FL, REFD>(in, lv, l1, q0 + qi < Lq, rec_o, rec_w01, rec_w23);
        if constexpr (NGL > 0) issue(std::integral_constant<int, 0>{});
    }
    // every wave: its DMA pieces (and the first gathers) landed, then everyone's
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (!has) return;
    const int stride = NW;
#pragma unroll 1
    for (;;) {
        int tn = t + stride;
        if constexpr (KINET_ENC_DYN) {
            // dynamic claim: a wave that finishes early takes the next tile, so the strip ends
            // when the tiles run out rather than with the slowest wave's fixed share
            int c = 0;
            if (lane_id_here() == 0) c = atomicAdd(&lv.next_tile, 1);
            tn = __builtin_amdgcn_readfirstlane(c);
        }
        const bool more = tn < t1;
        const int qn0 = more ? tile_q0(tn) : 0;
        // the next tile's phase-1 inputs, behind this tile's gathers
        if (more) {
            const int li = lane_id_here();
            load_tile<REFD, QM, REC>(in, ro, rr, rq, b, Lq, qn0 + (li >> 2), li & 3);
        }
        f32x2 acc[4] = {};
        float tacc[4] = {0.f, 0.f, 0.f, 0.f};   // TAIL: this lane's corner of every sample
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
            flush16<!LDS_FIRST && LV == 0>(acc, h);
            if constexpr (TAIL) {
                uint32_t th[2];
#pragma unroll
                for (int p = 0; p < EP; ++p) tail_mac(th, gt[p], tail_w(w01[p], w23[p], tr, tc), p == 0);
                tail_flush(tacc, th);
            }
        };
        // LDS level LV, one point at a time (8 VGPRs of corner data beside the gathers).  A
        // footprint outside the staged rows (record flag TAF) is gathered from the head map:
        // when any lane of the wave has one at this level, the level runs the FAR variant
        // (per corner pair, the far lanes' corners loaded in place and waited for inside the
        // branch, so the common path keeps its gathers in flight and holds no extra registers)
        // the level's f16 sums into h; the flush into acc follows the FAR / common branch merge,
        // so only h (not the 8 accumulators) crosses it
        auto lds_level = [&](auto lvc, auto farc, uint32_t (&h)[4], uint32_t (&th)[2]) {
            constexpr int LV = decltype(lvc)::value;
            constexpr bool FAR = decltype(farc)::value;
#pragma unroll
            for (int p = 0; p < EP; ++p) {
                const uint32_t o = quad_bcast<LV>(rec_o[p]);
                const uint32_t w01 = quad_bcast<LV>(rec_w01[p]);
                const uint32_t w23 = quad_bcast<LV>(rec_w23[p]);
                const bool far = FAR && (o & TAF) != 0u;
                const uint32_t lo = far ? 0u : o;
                const char* r0 = vm + lo;
                const char* r1 = r0 + wb[LV];
                const bool any_far = FAR && __builtin_amdgcn_ballot_w64(far) != 0;
                auto corner = [&](const char* lp, uint32_t back) -> u32x4v {
                    u32x4v v = *reinterpret_cast<const u32x4v*>(lp);
                    if (FAR && any_far) {
                        if (far) {   // exec-masked: the other lanes keep their LDS data
                            const uint32_t go = (o & ~TAF) + cb - back;
                            asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)"
                                         : "+v"(v)
                                         : "v"(go), "s"(rv)
                                         : "memory");
                        }
                    }
                    return v;
                };
                const uint32_t wrow = (uint32_t)wb[LV];
                const u32x4v v0 = corner(r0, wrow + 64u);
                const u32x4v v1 = corner(r0 + 64, wrow);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    h[j] = p == 0 ? pk_mul_lo(v0[j], w01) : pk_fma_lo(h[j], v0[j], w01);
                    h[j] = pk_fma_hi(h[j], v1[j], w01);
                }
                __builtin_amdgcn_sched_barrier(0);
                const u32x4v v2 = corner(r1, 64u);
                const u32x4v v3 = corner(r1 + 64, 0u);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    h[j] = pk_fma_lo(h[j], v2[j], w23);
                    h[j] = pk_fma_hi(h[j], v3[j], w23);
                }
                if constexpr (TAIL) {
                    // this lane's corner from the tail map (a far sample: from the tail plane)
                    const uint32_t tco = (tr ? wrow >> 3 : 0u) + (uint32_t)tc * 8u;
                    uint2 tv = *reinterpret_cast<const uint2*>(vmb + ETB + (lo >> 3) + tco);
                    if (FAR && any_far) {
                        if (far) {
                            const uint32_t go = ((o & ~TAF) >> 3) - ((wrow >> 3) + 8u) + tco;
                            asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)"
                                         : "+v"(tv)
                                         : "v"(go), "s"(rt)
                                         : "memory");
                        }
                    }
                    tail_mac(th, tv, tail_w(w01, w23, tr, tc), p == 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        auto lds_level_any = [&](auto lvc) {
            constexpr int LV = decltype(lvc)::value;
            const uint32_t f = quad_bcast<LV>(rec_o[0] | rec_o[1] | rec_o[2] | rec_o[3]);
            uint32_t h[4], th[2];
            if (__builtin_amdgcn_ballot_w64((f & TAF) != 0u) != 0)
                lds_level(lvc, std::true_type{}, h, th);
            else
                lds_level(lvc, std::false_type{}, h, th);
            flush16<LDS_FIRST && LV == FL>(acc, h);
            if constexpr (TAIL) tail_flush(tacc, th);
        };
        // LDS levels interleaved between the gathered levels' consumes (slot s: LDS levels
        // FL + [s*NLL/NST, (s+1)*NLL/NST))
        static_for<0, NST>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            static_for<FL + s * NLL / NST, FL + (s + 1) * NLL / NST>([&](auto lc) { lds_level_any(lc); });
            if constexpr (s < NGL) {
                consume(std::integral_constant<int, s>{});
                if constexpr (s + 1 < NGL) issue(std::integral_constant<int, s + 1>{});
            }
        });
        const int lis = lane_id_here();
        const int q = q0 + (lis >> 2);
        if constexpr (TAIL) {
            // the quad's 4 corners: two DPP steps (every lane active)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                tacc[i] += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(tacc[i]), 0xB1, 0xf, 0xf, false));
                tacc[i] += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(tacc[i]), 0x4E, 0xf, 0xf, false));
            }
        }
        if (q < Lq) {
            VecT<TO, 8> o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o.v[2 * j] = Cvt<TO>::from(acc[j][0]);
                o.v[2 * j + 1] = Cvt<TO>::from(acc[j][1]);
            }
            const uint32_t od = (uint32_t)a.od;
            const uint32_t ob = ((uint32_t)(b * Lq + q) * (uint32_t)a.M + (uint32_t)m) * od;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, o), rw, (ob + (uint32_t)(lis & 3) * 8u) * 2u,
                                                   0, 0);
            if constexpr (TAIL) {
                if ((lis & 3) == 0) {
                    VecT<TO, 4> t;
#pragma unroll
                    for (int i = 0; i < 4; ++i) t.v[i] = Cvt<TO>::from(tacc[i]);
                    typedef uint32_t u32x2_ __attribute__((ext_vector_type(2)));
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_, t), rw, (ob + 32u) * 2u, 0, 0);
                }
            }
        }
        if (!more) break;
        t = tn;
        q0 = qn0;
        {
            const int li = lane_id_here();
            if constexpr (REC) setup_tile_rec<FL>(in, lv, li & 3, rk, rec_o, rec_w01, rec_w23);
            else setup_tile<FL, REFD>(in, lv, li & 3, q0 + (li >> 2) < Lq, rec_o, rec_w01, rec_w23);
        }
        if constexpr (NGL > 0) issue(std::integral_constant<int, 0>{});
    }
}

template <typename TO, int FL, int REFD, bool QM, bool REC = false, bool TAIL = false, int NW = EW>
__global__ __launch_bounds__(NW * 64) void msda_enc_kernel(const EncArgs a) {
    __shared__ EncLevels lv;
    __shared__ u32x4v vmap[EMAP_PIX * 4];
    // XCD-aware remap (cdna_hip_programming.md T1): the strips of one (frame, head) map run
    // on one XCD.  Assumes MI355X's 8 XCDs with round-robin dispatch; elsewhere the mapping is
    // still a bijection (only the L2 grouping is lost).
    int b, m, strip;
    {
        const int nblk = gridDim.x, lin = blockIdx.x;
        const int qd = nblk >> 3, rm = nblk & 7, xcd = lin & 7;
        const int nid = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + (lin >> 3);
        strip = nid % a.nstrip;
        const int bm = nid / a.nstrip;
        b = bm / a.M;
        m = bm % a.M;
    }
    if (threadIdx.x == 0) {
        int acc = 0;
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
            lv.ra[l] = 0;
            lv.rn[l] = a.cap[l];
            lv.lb[l] = 0;
            acc += H * W;
        }
    }
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    enc_tiles<TO, FL, REFD, QM, REC, TAIL, NW>(a, lv, vmap, b, m, strip, wave, lane);
}

// LDS regions for strips of 1/n of the image: rows ceil(H/n) + 3 (pixel centres, the +1 corner
// row, a tile spilling into the next row) + 2*EHALO, at most the whole level + the two zero rows
bool plan_layout(const int64_t* shapes, int fl, int n, EncPlan& pl, int budget = EMAP_PIX) {
    int wmax = 0;
    for (int l = fl; l < EL; ++l) wmax = std::max<int>(wmax, (int)shapes[2 * l + 1]);
    long long pos = ((long long)wmax + 2 + 15) / 16 * 16;   // zero margin: a whole 2x2 footprint of any level
    pl.zpix = (int)pos;
    for (int l = 0; l < EL; ++l) pl.cap[l] = pl.base[l] = 0;
    for (int l = fl; l < EL; ++l) {
        const long long H = shapes[2 * l], W = shapes[2 * l + 1];
        const long long cap = std::min<long long>(H + 2, (H + n - 1) / n + 3 + 2 * EHALO);
        pl.cap[l] = (int)cap;
        pl.base[l] = (int)pos;
        pos += (cap * W + 2 + 15) / 16 * 16;
        if (pos > budget) return false;
    }
    pl.used = (int)pos;
    pl.fl = fl;
    pl.nstrip = n;
    return true;
}

// strips per head map requested by kinet_msda_encoder_set_strips for the calling thread (0 = the
// plan's own choice; honoured when that many strips fit the LDS map)
thread_local int enc_strips = 0;

// the fewest gathered levels whose staged levels fit with strips of at least 16 tiles, then the
// fewest strips (>= what fits) whose workgroups fill >= 90 % of their last round of one per CU
bool enc_plan(const int64_t* shapes, int batch, int heads, int num_query, EncPlan& pl, bool tail = false) {
    const int budget = tail ? EMAP_T : EMAP_PIX;
    const int cus = cu_count();
    const int maps = batch * heads;
    const int ntile = (num_query + EQT - 1) / EQT;
    const int nmax = std::max(1, ntile / EQT);
    for (int fl = 0; fl < EL; ++fl) {
        int nmin = 0;
        for (int n = 1; n <= nmax && n <= 64; ++n)
            if (plan_layout(shapes, fl, n, pl, budget)) {
                nmin = n;
                break;
            }
        if (!nmin) continue;
        int n = nmin;
        for (int c = nmin; c <= std::min(nmax, 2 * nmin + cus / std::max(1, maps)); ++c) {
            const long long wgs = (long long)maps * c, rounds = (wgs + cus - 1) / cus;
            if (wgs * 10 >= rounds * cus * 9) {
                n = c;
                break;
            }
        }
        if (enc_strips >= nmin && enc_strips <= std::min(nmax, 64) && plan_layout(shapes, fl, enc_strips, pl, budget))
            return true;
        return plan_layout(shapes, fl, n, pl, budget);
    }
    return false;
}

}  // namespace
}  // namespace kinet

using namespace kinet;

extern "C" int kinet_msda_encoder_set_strips(int strips) {
    KINET_CHECK_ARG(strips >= 0 && strips <= 64, "msda encoder: strips must be in [0, 64] (got %d)", strips);
    const int old = enc_strips;
    enc_strips = strips;
    return old;
}

extern "C" int kinet_msda_encoder_plan(const int64_t* spatial_shapes_host, int batch, int num_heads, int num_query,
                                       int32_t* plan_out) {
    KINET_CHECK_ARG(spatial_shapes_host != nullptr && batch > 0 && num_heads > 0 && num_query > 0,
                    "msda encoder plan: bad arguments");
    for (int l = 0; l < EL; ++l)
        KINET_CHECK_ARG(spatial_shapes_host[2 * l] > 0 && spatial_shapes_host[2 * l + 1] > 0 &&
                            spatial_shapes_host[2 * l] * spatial_shapes_host[2 * l + 1] < (1LL << 30),
                        "msda encoder plan: bad level shape");
    EncPlan pl{};
    KINET_CHECK_ARG(enc_plan(spatial_shapes_host, batch, num_heads, num_query, pl),
                    "msda encoder: no strip plan fits the LDS map (use kinet_msda_fused_forward)");
    if (plan_out) {
        plan_out[0] = pl.fl;
        plan_out[1] = pl.nstrip;
        plan_out[2] = pl.used;
        plan_out[3] = batch * num_heads * pl.nstrip;
    }
    return KINET_OK;
}

namespace {
// kinet_msda_encoder_forward (rec = false: f16 offsets / logits + reference points) and
// kinet_msda_encoder_forward_records (rec = true: sampling records)
int encoder_forward(const void* value, int64_t value_sb, int64_t value_sm, const int64_t* spatial_shapes_host,
                    const void* offlog, const float* ref_points, int ref_dim, const uint8_t* query_attn_mask,
                    int frac_bits, bool rec, void* output, int batch, int spatial_size, int num_heads, int channels,
                    int num_levels, int num_query, int num_point, int output_dtype, const int32_t* query_tile_order,
                    kinet_stream_t stream, const void* tail = nullptr, int64_t tail_sb = 0, int64_t tail_sm = 0) {
    KINET_CHECK_ARG(batch >= 0 && spatial_size > 0 && num_heads > 0 && num_query >= 0, "msda encoder: bad sizes");
    const bool has_tail = tail != nullptr;
    KINET_CHECK_ARG(channels == (has_tail ? 36 : 32) && num_levels == EL && num_point == EP,
                    "msda encoder: head_dim %d, 4 levels, 4 points (got %d, %d, %d)", has_tail ? 36 : 32, channels,
                    num_levels, num_point);
    KINET_CHECK_ARG(!has_tail || (!rec && ((uintptr_t)tail % 8) == 0 && tail_sb % 4 == 0 && tail_sm % 4 == 0 &&
                                  tail_sb >= (int64_t)spatial_size * 4 && tail_sm >= tail_sb),
                    "msda encoder: tail plane must be an 8-byte aligned (M, B, S, 4) plane, offsets/logits input");
    if (!rec)
        KINET_CHECK_ARG(ref_dim == 2 || ref_dim == 4, "Last dim of reference_points must be 2 or 4, but get %d instead.",
                        ref_dim);
    else
        KINET_CHECK_ARG(frac_bits >= 6 && frac_bits <= 10, "msda encoder: frac_bits in [6, 10] (got %d)", frac_bits);
    KINET_CHECK_ARG(output_dtype == KINET_BF16 || output_dtype == KINET_F16, "msda encoder: output must be bf16 or f16");
    KINET_CHECK_ARG(((uintptr_t)value % 16) == 0 && ((uintptr_t)offlog % 16) == 0 && value_sb % 8 == 0 &&
                        value_sm % 8 == 0,
                    "msda encoder: value / offsets must be 16-byte aligned");
    KINET_CHECK_ARG(spatial_shapes_host != nullptr, "msda encoder: spatial_shapes_host is NULL");
    long long npix = 0;
    for (int l = 0; l < EL; ++l) {
        KINET_CHECK_ARG(spatial_shapes_host[2 * l] > 0 && spatial_shapes_host[2 * l + 1] > 0 &&
                            spatial_shapes_host[2 * l] * spatial_shapes_host[2 * l + 1] < (1LL << 30),
                        "msda encoder: bad level shape");
        if (rec)
            KINET_CHECK_ARG(spatial_shapes_host[2 * l] <= (1LL << (16 - frac_bits)) &&
                                spatial_shapes_host[2 * l + 1] <= (1LL << (16 - frac_bits)),
                            "msda encoder: level %d exceeds the records' %d-bit integer part", l, 16 - frac_bits);
        npix += spatial_shapes_host[2 * l] * spatial_shapes_host[2 * l + 1];
    }
    KINET_CHECK_ARG(npix == spatial_size, "msda encoder: spatial_shapes cover %lld tokens, value has %d", npix,
                    spatial_size);
    if (batch == 0 || num_query == 0) return KINET_OK;
    EncPlan pl{};
    KINET_CHECK_ARG(enc_plan(spatial_shapes_host, batch, num_heads, num_query, pl, has_tail),
                    "msda encoder: no strip plan fits the LDS map (use kinet_msda_fused_forward)");
    const long long head_bytes = (long long)spatial_size * 64;
    // the tail plane's range stays below TAF >> 3 (an invalid gathered sample's offset)
    KINET_CHECK_ARG(!has_tail || (long long)spatial_size * 8 < (1LL << 28), "msda encoder: tail plane too large");
    long long wmax = 0;
    for (int l = 0; l < EL; ++l) wmax = std::max<long long>(wmax, spatial_shapes_host[2 * l + 1]);
    const int rd = rec ? 2 : ref_dim;
    // far-sample records carry a map offset up to (S + W + 1) * 64 below the TAF flag bit
    KINET_CHECK_ARG((spatial_size + wmax + 2) * 64 < (1LL << 31) && (long long)num_query * EREC * 2 < (1LL << 31) &&
                        (long long)batch * num_query < (1LL << 24) &&
                        (long long)batch * num_query * EL * rd * 4 < (1LL << 31) &&
                        (long long)batch * num_query * num_heads * channels * 2 < (1LL << 31),
                    "msda encoder: problem too large for 32-bit buffer offsets");
    EncArgs a{};
    a.value = (const f16_t*)value;
    a.vsb = (long)value_sb;
    a.vsm = (long)value_sm;
    a.head_bytes = (int)head_bytes;
    a.tail = (const f16_t*)tail;
    a.tsb = (long)tail_sb;
    a.tsm = (long)tail_sm;
    a.tail_bytes = has_tail ? spatial_size * 8 : 0;
    a.od = channels;
    for (int l = 0; l < EL; ++l) {
        a.H[l] = (int)spatial_shapes_host[2 * l];
        a.W[l] = (int)spatial_shapes_host[2 * l + 1];
        a.cap[l] = pl.cap[l];
        a.base[l] = pl.base[l];
    }
    a.offlog = (const f16_t*)offlog;
    a.ref = rec ? nullptr : ref_points;
    a.qmask = rec ? nullptr : query_attn_mask;
    a.out = output;
    a.torder = (const int*)query_tile_order;
    a.S = spatial_size;
    a.B = batch;
    a.M = num_heads;
    a.Lq = num_query;
    a.ref_dim = rd;
    a.nstrip = pl.nstrip;
    a.used = pl.used;
    a.fb = rec ? frac_bits : 0;
    const long long maps = (long long)batch * num_heads;
    KINET_CHECK_ARG(maps * pl.nstrip < (1LL << 31), "msda encoder: grid too large");
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)(maps * pl.nstrip)), block(EW * 64);
    if (has_tail) {
        const dim3 tblock(EWT * 64);
#define TK(TO_, FL_, RD_, QM_) hipLaunchKernelGGL((msda_enc_kernel<TO_, FL_, RD_, QM_, false, true, EWT>), grid, tblock, 0, s, a)
#define TK_QM(TO_, FL_, RD_) if (query_attn_mask) TK(TO_, FL_, RD_, true); else TK(TO_, FL_, RD_, false)
#define TK_RD(TO_, FL_) if (ref_dim == 2) { TK_QM(TO_, FL_, 2); } else { TK_QM(TO_, FL_, 4); }
#define TK_FL(TO_)                        \
    switch (pl.fl) {                      \
        case 0: TK_RD(TO_, 0) break;      \
        case 1: TK_RD(TO_, 1) break;      \
        case 2: TK_RD(TO_, 2) break;      \
        default: TK_RD(TO_, 3) break;     \
    }
        if (output_dtype == KINET_BF16) {
            TK_FL(bf16_t)
        } else {
            TK_FL(f16_t)
        }
#undef TK_FL
#undef TK_RD
#undef TK_QM
#undef TK
        KINET_LAUNCH_CHECK();
        return KINET_OK;
    }
#define EK(TO_, FL_, RD_, QM_) hipLaunchKernelGGL((msda_enc_kernel<TO_, FL_, RD_, QM_>), grid, block, 0, s, a)
#define EK_QM(TO_, FL_, RD_) if (query_attn_mask) EK(TO_, FL_, RD_, true); else EK(TO_, FL_, RD_, false)
#define EK_RD(TO_, FL_)                                                                                  \
    if (rec) hipLaunchKernelGGL((msda_enc_kernel<TO_, FL_, 2, false, true>), grid, block, 0, s, a);     \
    else if (ref_dim == 2) { EK_QM(TO_, FL_, 2); } else { EK_QM(TO_, FL_, 4); }
#define EK_FL(TO_)                        \
    switch (pl.fl) {                      \
        case 0: EK_RD(TO_, 0) break;      \
        case 1: EK_RD(TO_, 1) break;      \
        case 2: EK_RD(TO_, 2) break;      \
        default: EK_RD(TO_, 3) break;     \
    }
    if (output_dtype == KINET_BF16) {
        EK_FL(bf16_t)
    } else {
        EK_FL(f16_t)
    }
#undef EK_FL
#undef EK_RD
#undef EK_QM
#undef EK
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}
}  // namespace

extern "C" int kinet_msda_encoder_forward(const void* value, int64_t value_sb, int64_t value_sm,
                                          const int64_t* spatial_shapes_host, const void* offsets_logits_hm,
                                          const float* ref_points, int ref_dim, const uint8_t* query_attn_mask,
                                          void* output, int batch, int spatial_size, int num_heads, int channels,
                                          int num_levels, int num_query, int num_point, int output_dtype,
                                          const int32_t* query_tile_order, kinet_stream_t stream) {
    return encoder_forward(value, value_sb, value_sm, spatial_shapes_host, offsets_logits_hm, ref_points, ref_dim,
                           query_attn_mask, 0, false, output, batch, spatial_size, num_heads, channels, num_levels,
                           num_query, num_point, output_dtype, query_tile_order, stream);
}

extern "C" int kinet_msda_encoder_forward_split(const void* value_main, int64_t main_sb, int64_t main_sm,
                                                const void* value_tail, int64_t tail_sb, int64_t tail_sm,
                                                const int64_t* spatial_shapes_host, const void* offsets_logits_hm,
                                                const float* ref_points, int ref_dim, const uint8_t* query_attn_mask,
                                                void* output, int batch, int spatial_size, int num_heads, int channels,
                                                int num_levels, int num_query, int num_point, int output_dtype,
                                                const int32_t* query_tile_order, kinet_stream_t stream) {
    KINET_CHECK_ARG(value_tail != nullptr, "msda encoder split: value_tail is NULL");
    return encoder_forward(value_main, main_sb, main_sm, spatial_shapes_host, offsets_logits_hm, ref_points, ref_dim,
                           query_attn_mask, 0, false, output, batch, spatial_size, num_heads, channels, num_levels,
                           num_query, num_point, output_dtype, query_tile_order, stream, value_tail, tail_sb, tail_sm);
}

extern "C" int kinet_msda_encoder_plan_ex(const int64_t* spatial_shapes_host, int batch, int num_heads, int num_query,
                                          int channels, int32_t* plan_out) {
    KINET_CHECK_ARG(channels == 32 || channels == 36, "msda encoder plan: head_dim 32 or 36 (got %d)", channels);
    KINET_CHECK_ARG(spatial_shapes_host != nullptr && batch > 0 && num_heads > 0 && num_query > 0,
                    "msda encoder plan: bad arguments");
    EncPlan pl{};
    KINET_CHECK_ARG(enc_plan(spatial_shapes_host, batch, num_heads, num_query, pl, channels == 36),
                    "msda encoder: no strip plan fits the LDS map (use kinet_msda_fused_forward)");
    if (plan_out) {
        plan_out[0] = pl.fl;
        plan_out[1] = pl.nstrip;
        plan_out[2] = pl.used;
        plan_out[3] = batch * num_heads * pl.nstrip;
    }
    return KINET_OK;
}

extern "C" int kinet_msda_encoder_forward_records(const void* value, int64_t value_sb, int64_t value_sm,
                                                  const int64_t* spatial_shapes_host, const void* records,
                                                  int frac_bits, void* output, int batch, int spatial_size,
                                                  int num_heads, int channels, int num_levels, int num_query,
                                                  int num_point, int output_dtype, const int32_t* query_tile_order,
                                                  kinet_stream_t stream) {
    KINET_CHECK_ARG(records != nullptr, "msda encoder: records is NULL");
    return encoder_forward(value, value_sb, value_sm, spatial_shapes_host, records, nullptr, 2, nullptr, frac_bits,
                           true, output, batch, spatial_size, num_heads, channels, num_levels, num_query, num_point,
                           output_dtype, query_tile_order, stream);
}
