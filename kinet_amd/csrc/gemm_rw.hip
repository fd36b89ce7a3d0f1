// Resident-weight streaming GEMM for gfx950: C[M, N] = epilogue(A[M, K] @ W[N, K]^T) for
// large M and K <= 256 -- the deformable-encoder projections (value_proj, output_proj +
// residual + LayerNorm, FFN linear1, sampling offsets / attention logits) and the 1x1
// stride-1 convolutions of the ResNet body (NHWC activations are plain row-major GEMM
// operands).  DESIGN.md "Resident-weight GEMM".
//
// Why a second GEMM: with K = 256 the MFMA work per output byte is small and the tiled
// kernel (gemm.hip) spends its time re-loading W tiles and re-reading A once per N-tile
// through the CU load path.  Here
//  * a workgroup (4 waves) owns a column group of GW = 4*NT*16 output columns for the
//    whole launch; wave w keeps W rows [w*NT*16, (w+1)*NT*16) x K as MFMA A-fragments in
//    VGPRs (NT*KC*4 registers), loaded once;
//  * the workgroup walks row tiles of BMR rows (persistent: tile = blockIdx.x + i*gridDim.x);
//    each A tile (and the residual tile and the row-mask bytes) is staged into an NS-deep
//    LDS ring by LDS-DMA (buffer_load_dwordx4 ... lds, XOR swizzle on the source side,
//    hardware zero fill past the edges), issued NS-1 tiles ahead;  a counted
//    `s_waitcnt vmcnt` + raw s_barrier retires one tile per iteration, so the DMA of later
//    tiles stays in flight across the barrier (cdna_hip_programming.md §5 "Pipelining
//    across barriers");  no VGPR-destination global load appears in the loop, so hipcc
//    never drains the ring with a vmcnt(0) of its own;
//  * W rows are assigned to fragment rows so that every lane ends up holding NT*4
//    CONSECUTIVE output columns of one row: the epilogue (scale/bias, residual, ReLU,
//    LayerNorm across the 4 waves through a tiny LDS exchange, row mask, plain or
//    head-major store) runs straight from the accumulators with 16-byte stores;
//  * the packed outputs of tile i are stored after the barrier of iteration i+1, behind
//    the newest DMA, so outstanding stores never hold up the ring's counted wait.
#include <hip/hip_runtime.h>

#include "../../include/kinet_gemm.h"
#include "../../include/kinet_msda.h"
#include "common.h"
#include "gemm_common.h"

namespace kinet {
namespace {

// NW waves per workgroup (4, or 6 for the d = 288 LayerNorm rows: 6 x 48 = 288 columns);
// rows of K = 32*KC 16-bit elements: a power-of-two number of 16-byte chunks, or a multiple of
// 4 (K = 288: 36 chunks).  A tile region whose bytes are not whole DMA rounds (NW*64 lanes x
// 16 B) is padded to whole rounds; the padding chunks read zeros (out of range) and nothing
// reads them back.
template <int KC, int NT, int BMR, int NS, bool HAS_R, bool LN, bool HAS_A2, bool PREP = false, int NW = 4>
struct RwCfg {
    static constexpr int NTHR = NW * 64;
    static constexpr int OPB = NTHR * 16;                   // bytes per DMA round
    static constexpr int ROW = KC * 64;                     // A row bytes (K = 32*KC, 16-bit)
    static constexpr int CPR = ROW / 16;                    // 16-byte chunks per A row
    static constexpr bool POW2 = (CPR & (CPR - 1)) == 0;
    static constexpr int SWM = (CPR < 16 ? CPR : 16) - 1;   // source-side XOR swizzle mask
    static constexpr int GW = NW * NT * 16;                 // columns per workgroup
    static constexpr int A_BYTES = BMR * ROW;
    static constexpr int A_OPS = (A_BYTES + OPB - 1) / OPB;   // DMA instructions per thread per tile
    static constexpr int A_SPAN = A_OPS * OPB;
    static constexpr int A2_BYTES = HAS_A2 ? A_SPAN : 0;    // second A operand (A + A2)
    static constexpr int R_ROW = GW * 2;
    static constexpr int R_CPR = R_ROW / 16;
    static constexpr bool R_POW2 = (R_CPR & (R_CPR - 1)) == 0;
    static constexpr int R_SWM = (R_CPR < 16 ? R_CPR : 16) - 1;
    static constexpr int R_OPS = HAS_R ? (BMR * R_ROW + OPB - 1) / OPB : 0;
    static constexpr int R_BYTES = R_OPS * OPB;
    static constexpr int R_OFF = A_SPAN + A2_BYTES;
    static constexpr int MASK_OFF = R_OFF + R_BYTES;
    static constexpr int REF_OFF = MASK_OFF + 1024;         // PREP: the tile's reference points
    static constexpr int REF_OPS = PREP ? BMR / 16 : 0;     // 1 KiB DMAs: BMR rows x 4 levels x <= 16 B
    static constexpr int STAGE = REF_OFF + REF_OPS * 1024;  // + one DMA of row-mask bytes (+ refs)
    static constexpr int PAR = 4 * GW * 4;                  // scale, bias, gamma, beta (f32)
    static constexpr int LNS = LN ? 2 * BMR * NW * 4 : 0;   // [2][BMR][NW waves] partial sums
    static constexpr int BYTES = PAR + LNS + NS * STAGE;
    static constexpr int D = A_OPS * (HAS_A2 ? 2 : 1) + R_OPS + 1 + REF_OPS;
    // LDS position of 16-byte chunk c of tile row r (an involution: the DMA fills position c
    // with source chunk sw(r, c), a reader of logical chunk q reads position sw(r, q)).  Rows of
    // 36 chunks (K = 288, 576 B = 144 banks: rows r and r + 4 share banks) swap chunks within
    // aligned groups of 4 by (r >> 2) & 3, so 16 rows read at one chunk hit 16 distinct
    // 4-bank groups
    __device__ static constexpr int sw(int r, int c) { return POW2 ? c ^ (r & SWM) : c ^ ((r >> 2) & 3); }
    __device__ static constexpr int rsw(int r, int c) { return R_POW2 ? c ^ (r & R_SWM) : c ^ ((r >> 2) & 3); }
    static_assert(!PREP || (NT == 3 && (NW == 4 || NW == 8) && (BMR == 16 || BMR == 32) && !HAS_R && !LN),
                  "sampling records: one head per wave (12 columns per lane), 16- or 32-row tiles");
    static_assert(POW2 || CPR % 4 == 0, "A rows: power-of-two or multiple-of-4 chunks");
    static_assert(!HAS_R || R_POW2 || R_CPR % 4 == 0, "residual rows: power-of-two or multiple-of-4 chunks");
    static_assert(BMR / 16 <= 64, "mask DMA lanes");
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// raw workgroup barrier for LDS traffic only: unlike __syncthreads() it does not drain the
// vector-memory counter, so LDS-DMA issued earlier stays in flight across it
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// the NW waves' partial sums of one row, in wave order
template <int NW>
__device__ __forceinline__ float wave_sum(const float* w) {
    if constexpr (NW == 4) {
        const f32x4 w4 = *reinterpret_cast<const f32x4*>(w);
        return w4[0] + w4[1] + w4[2] + w4[3];
    } else {
        float s = w[0];
#pragma unroll
        for (int i = 1; i < NW; ++i) s += w[i];
        return s;
    }
}

template <typename TO> struct Pack;
template <> struct Pack<bf16_t> {
    static constexpr int WORDS_PER_4 = 2;
    __device__ static void put(uint32_t* w, const float* v) {
        w[0] = (uint32_t)f32_to_bf16(v[0]).x | ((uint32_t)f32_to_bf16(v[1]).x << 16);
        w[1] = (uint32_t)f32_to_bf16(v[2]).x | ((uint32_t)f32_to_bf16(v[3]).x << 16);
    }
};
template <> struct Pack<f16_t> {
    static constexpr int WORDS_PER_4 = 2;
    __device__ static void put(uint32_t* w, const float* v) {
        const f16_t a = (f16_t)v[0], b = (f16_t)v[1], c = (f16_t)v[2], d = (f16_t)v[3];
        w[0] = (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
        w[1] = (uint32_t)__builtin_bit_cast(uint16_t, c) | ((uint32_t)__builtin_bit_cast(uint16_t, d) << 16);
    }
};
template <> struct Pack<float> {
    static constexpr int WORDS_PER_4 = 4;
    __device__ static void put(uint32_t* w, const float* v) {
        for (int i = 0; i < 4; ++i) w[i] = __float_as_uint(v[i]);
    }
};

__device__ __forceinline__ void unpack8(const u32x4& u, float* v, bool f16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (f16) {
            v[2 * i] = (float)__builtin_bit_cast(f16_t, (uint16_t)(u[i] & 0xffffu));
            v[2 * i + 1] = (float)__builtin_bit_cast(f16_t, (uint16_t)(u[i] >> 16));
        } else {
            v[2 * i] = __uint_as_float(u[i] << 16);
            v[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
        }
    }
}

// Sampling records of one (query, head, level) from the 12 projection outputs this lane holds
// (ms_deform_attn.py:69-82 + the bilinear setup of ms_deform_im2col_cuda.cuh:227-233):
//   v = [x0 y0 x1 y1 x2 y2 x3 y3 | logit0..3] of level l (offsets in level pixels, the head's
//   16 logits spread over the 4 lanes lane, lane^16, lane^32, lane^48 -- one per level);
// softmax over the head's 16 logits, the locations (the reference's offsets / (H, W) on (x, y)
// quirk for 2-d refs, :77-82), then per point, with h = y H - 0.5, w = x W - 0.5:
//   * the corner rows / columns outside the level folded into the weight by ONE factor per axis,
//     clamp(min(h + 1, H - h), 0, 1): 1 inside, lh = h + 1 when the top row is -1 (the footprint
//     becomes row 0 with weight a lh), 1 - lh = H - h when the bottom row is H (row H-1 keeps
//     a (1 - lh)), 0 outside the level (cuh:229) -- so the sampler needs no bounds tests (its
//     second row / column only ever gets weight 0); the same for columns;
//   * location = round(clamp(h, 0, H-1) 2^fb) << 16 | round(clamp(w, 0, W-1) 2^fb): the
//     fixed-point corner + fraction, (hl << (16+fb)) | (round(lh 2^fb) << 16) | (wl << fb) |
//     round(lw 2^fb) with a rounded-up fraction carried into the corner (h 2^fb + 0.5 is exact in
//     f32 for every level that fits the 16-bit field); a folded axis has fraction 0; a sample
//     outside the level (weight 0) points at the query's own pixel of the level, which the
//     sampler's strip always stages (finite values assumed: it multiplies that pixel by 0);
//   * weight = f16.
// out: 4 location words, then the 4 weights as 2 packed f16 words.
// max / sum over the 4 lanes lane ^ {0, 16, 32, 48} (the 4 levels of one row): gfx950's row-swap
// permutes (v_permlane16_swap / v_permlane32_swap) return {own, partner} in some order, so one
// op per step combines them -- no LDS round trip as __shfl_xor's ds_bpermute takes
template <bool MAX>
__device__ __forceinline__ float level_reduce(float x) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = MAX ? fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1])) : __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return MAX ? fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1])) : __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// r: the (query, level) reference point (x, y[, w, h]), qmasked: the query's mask byte, both read
// from the tile's LDS stage by the caller
__device__ __forceinline__ void prep_records(const GemmArgs& p, const float4 r, bool qmasked, int Hl, int Wl,
                                             const float (&v)[12], uint32_t* out) {
    const float Hf = (float)Hl, Wf = (float)Wl;
    const float fs = (float)(1 << p.prep_fb);
    const float mx = level_reduce<true>(fmaxf(fmaxf(v[8], v[9]), fmaxf(v[10], v[11])));
    float e[4], es = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        e[q] = __expf(v[8 + q] - mx);
        es += e[q];
    }
    es = level_reduce<false>(es);
    const float ra = qmasked ? 0.f : __builtin_amdgcn_rcpf(es);
    float rx, ry, sx, sy;   // reference point and the offset scale of each axis
    if (p.prep_refd == 2) {
        rx = r.x;
        ry = r.y;
        sx = __builtin_amdgcn_rcpf(Hf);   // :77-79 (offsets / spatial_shapes, (H, W) on (x, y))
        sy = __builtin_amdgcn_rcpf(Wf);
    } else {
        rx = r.x;
        ry = r.y;
        sx = 0.125f * r.z;   // :80-82 (/ n_points * wh * 0.5, n_points = 4)
        sy = 0.125f * r.w;
    }
    const float H1 = Hf - 1.f, W1 = Wf - 1.f;
    // the query's own pixel of this level: where a sample outside the level points (weight 0)
    const int hr = min(max((int)floorf(ry * Hf), 0), Hl - 1), wr = min(max((int)floorf(rx * Wf), 0), Wl - 1);
    const uint32_t own = ((uint32_t)hr << (16 + p.prep_fb)) | ((uint32_t)wr << p.prep_fb);
    float aw[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float x = fmaf(v[2 * q], sx, rx), y = fmaf(v[2 * q + 1], sy, ry);
        const float h = fmaf(y, Hf, -0.5f), w = fmaf(x, Wf, -0.5f);
        const float fh = __builtin_amdgcn_fmed3f(fminf(h + 1.f, Hf - h), 0.f, 1.f);
        const float fw = __builtin_amdgcn_fmed3f(fminf(w + 1.f, Wf - w), 0.f, 1.f);
        aw[q] = e[q] * ra * fh * fw;
        const uint32_t ph = (uint32_t)(int)fmaf(__builtin_amdgcn_fmed3f(h, 0.f, H1), fs, 0.5f);
        const uint32_t pw = (uint32_t)(int)fmaf(__builtin_amdgcn_fmed3f(w, 0.f, W1), fs, 0.5f);
        out[q] = fminf(fh, fw) > 0.f ? (ph << 16) | pw : own;   // fh, fw > 0: inside (-1, H) x (-1, W)
    }
    out[4] = (uint32_t)__builtin_bit_cast(uint16_t, (f16_t)aw[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, (f16_t)aw[1]) << 16);
    out[5] = (uint32_t)__builtin_bit_cast(uint16_t, (f16_t)aw[2]) | ((uint32_t)__builtin_bit_cast(uint16_t, (f16_t)aw[3]) << 16);
}

// CR (conv-row mode): A row m is output pixel (img, oh, ow) of a KH x 1, horizontally
// stride-1 unpadded NHWC convolution (the tap-folded ResNet stem, ops.hip
// pack_image_kwfold_kernel): K = KH*Cin, logical chunk q of the row = 8 channels of tap
// kh = q / (Cin/8) read from input row oh*stride - pad + kh (zeros outside the image and past K)
template <typename T, typename TO, int KC, int NT, int BMR, int NS, bool HAS_R, bool LN, bool HAS_A2, bool CR,
          bool PREP = false, int OCC = 2, int NW = 4>
__global__ __launch_bounds__(NW * 64, OCC) void gemm_rw_kernel(const GemmArgs p, const int n_mtiles) {
    using C_ = RwCfg<KC, NT, BMR, NS, HAS_R, LN, HAS_A2, PREP, NW>;
    constexpr int NTHR = C_::NTHR;
    constexpr int TMR = BMR / 16;             // 16-row MFMA tiles per row tile
    constexpr int GW = C_::GW;
    constexpr int NC = NT * 4;                // consecutive columns per lane
    constexpr int PW = NC / 4 * Pack<TO>::WORDS_PER_4;   // packed 32-bit words per lane-row
    constexpr unsigned OOB = 0x80000000u;
    __shared__ __attribute__((aligned(16))) char lds[C_::BYTES];
    float* par = reinterpret_cast<float*>(lds);
    float* lns = reinterpret_cast<float*>(lds + C_::PAR);
    char* stages = lds + C_::PAR + C_::LNS;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int P = gridDim.x, bx = blockIdx.x;
    const int ncol0 = blockIdx.y * GW;
    const int M = p.M, N = p.N;
    const int cnt = bx < n_mtiles ? (n_mtiles - 1 - bx) / P + 1 : 0;

    for (int i = tid; i < GW; i += NTHR) {
        const int n = ncol0 + i;
        const bool ok = n < N;
        par[i] = (ok && p.scale) ? p.scale[n] : 1.f;
        par[GW + i] = (ok && p.bias) ? p.bias[n] : 0.f;
        par[2 * GW + i] = (LN && ok) ? p.ln_g[n] : 0.f;
        par[3 * GW + i] = (LN && ok) ? p.ln_b[n] : 0.f;
    }

    // this wave's W slice as MFMA A-fragments: fragment row i of n-tile a is output column
    // ncol0 + wave*NC*4 + (i>>2)*NC + a*4 + (i&3), so lane group g = lane>>4 of the result
    // holds columns [g*NC, g*NC + NC) of the wave's range -- NC consecutive columns
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.b_bytes, 0x00020000);
    u32x4 wf[NT][KC];
    {
        const int i = lane & 15;
#pragma unroll
        for (int a = 0; a < NT; ++a) {
            const int n = ncol0 + wave * NC * 4 + (i >> 2) * NC + a * 4 + (i & 3);
#pragma unroll
            for (int c = 0; c < KC; ++c) {
                const int k = c * 32 + (lane >> 4) * 8;
                const unsigned off = (n < N && k < p.K) ? ((unsigned)n * (unsigned)p.ldb + (unsigned)k) * 2u : OOB;
                wf[a][c] = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 0);
            }
        }
    }

    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.a_bytes, 0x00020000);
    const int a2_bytes = (HAS_A2 && p.a2_rows) ? ((p.a2_rows - 1) * p.lda + p.K) * 2 : p.a_bytes;
    const __amdgpu_buffer_rsrc_t ra2 =
        __builtin_amdgcn_make_buffer_rsrc((void*)(HAS_A2 ? p.A2 : p.A), (short)0, a2_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr =
        __builtin_amdgcn_make_buffer_rsrc((void*)(HAS_R ? p.R : p.A), (short)0, HAS_R ? p.r_bytes : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rm =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p.row_mask ? (const void*)p.row_mask : p.A), (short)0,
                                          p.row_mask ? M : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(PREP ? (const void*)p.prep_ref : p.A), (short)0, PREP ? M * 16 * p.prep_refd : 0, 0x00020000);

    // per-thread DMA offsets, split into a scalar tile base (m0 * ld) and lane constants
    unsigned a_lo[C_::A_OPS];
    int a_row[C_::A_OPS];
    int cr_kh[C_::A_OPS];
#pragma unroll
    for (int j = 0; j < C_::A_OPS; ++j) {
        const int idx = j * NTHR + tid;
        const int row = idx / C_::CPR, s = idx % C_::CPR;
        a_row[j] = row < BMR ? row : (1 << 30);   // round padding: never in range
        a_lo[j] = ((unsigned)row * (unsigned)p.lda + (unsigned)(C_::sw(row, s) * 8)) * 2u;
        cr_kh[j] = 0;
        if (CR) {
            // tap and in-tap channel offset of logical chunk q (lane constants); chunks past K
            // get a tap index that never lands inside the image
            const int q = C_::sw(row, s), cpt = p.Cin >> 3;
            const int kh = q / cpt;
            cr_kh[j] = q * 8 < p.K ? kh : (1 << 28);
            a_lo[j] = (unsigned)((q - kh * cpt) * 8);
        }
    }
    unsigned r_lo[C_::R_OPS > 0 ? C_::R_OPS : 1];
    int r_row[C_::R_OPS > 0 ? C_::R_OPS : 1];
#pragma unroll
    for (int j = 0; j < C_::R_OPS; ++j) {
        const int idx = j * NTHR + tid;
        const int row = idx / C_::R_CPR, s = idx % C_::R_CPR;
        const int n = ncol0 + C_::rsw(row, s) * 8;
        r_row[j] = (n < N && row < BMR) ? row : (1 << 30);   // columns past N, round padding: never in range
        r_lo[j] = ((unsigned)row * (unsigned)p.ldr + (unsigned)n) * 2u;
    }
    auto issue = [&](int i) {
        const int m0 = (bx + i * P) * BMR;
        char* st = stages + (i % NS) * C_::STAGE;
        const unsigned abase = (unsigned)m0 * (unsigned)p.lda * 2u;
        // conv-row mode: the tile's first pixel on the scalar unit, then row r of the tile is
        // that pixel + r with at most one carry into the next output row (host: Wout >= BMR)
        const int hw = p.Hout * p.Wout;
        const int img0 = CR ? m0 / hw : 0;
        const int oh0 = CR ? (m0 - img0 * hw) / p.Wout : 0;
        const int ow0 = CR ? m0 - img0 * hw - oh0 * p.Wout : 0;
        // A2 of a2_rows rows (row m reads row m % a2_rows): the tile's rows sit in period q0 up
        // to tile row a2_bnd, in q0 + 1 after it (host: a2_rows >= BMR, so at most one wrap)
        unsigned a2_sub = 0u, a2_sub1 = 0u;
        int a2_bnd = 1 << 30;
        if (HAS_A2 && p.a2_rows) {
            const int q0 = m0 / p.a2_rows;
            a2_sub = (unsigned)(q0 * p.a2_rows) * (unsigned)p.lda * 2u;
            a2_sub1 = a2_sub + (unsigned)p.a2_rows * (unsigned)p.lda * 2u;
            a2_bnd = (q0 + 1) * p.a2_rows - m0;
        }
#pragma unroll
        for (int j = 0; j < C_::A_OPS; ++j) {
            unsigned off = m0 + a_row[j] < M ? abase + a_lo[j] : OOB;
            if (CR) {
                int ow = ow0 + a_row[j], oh = oh0, img = img0;
                const bool c1 = ow >= p.Wout;
                ow = c1 ? ow - p.Wout : ow;
                oh = c1 ? oh + 1 : oh;
                const bool c2 = oh >= p.Hout;
                oh = c2 ? 0 : oh;
                img = c2 ? img + 1 : img;
                const int ih = oh * p.stride - p.pad + cr_kh[j];
                const bool ok = m0 + a_row[j] < M && (unsigned)ih < (unsigned)p.Hin;
                off = ok ? ((unsigned)((img * p.Hin + ih) * p.Win + ow * p.stride_w) * (unsigned)p.Cin + a_lo[j]) * 2u : OOB;
            }
            dma16(ra, st + (j * NTHR + wave * 64) * 16, off);
            if (HAS_A2)
                dma16(ra2, st + C_::A_SPAN + (j * NTHR + wave * 64) * 16,
                      off == OOB ? OOB : off - (a_row[j] >= a2_bnd ? a2_sub1 : a2_sub));
        }
        const unsigned rbase = (unsigned)m0 * (unsigned)p.ldr * 2u;
#pragma unroll
        for (int j = 0; j < C_::R_OPS; ++j) {
            const unsigned off = m0 + r_row[j] < M ? rbase + r_lo[j] : OOB;
            dma16(rr, st + C_::R_OFF + (j * NTHR + wave * 64) * 16, off);
        }
        // row-mask bytes m0 .. m0+BMR (every wave writes the same 1 KiB; bytes past M read 0)
        dma16(rm, st + C_::MASK_OFF, lane < TMR ? (unsigned)(m0 + lane * 16) : OOB);
        // PREP: the tile's reference points, BMR rows x 4 levels x prep_refd f32 (<= 1 KiB; every
        // wave writes the same bytes, rows past M read 0)
        if constexpr (PREP) {
            const unsigned rbytes = (unsigned)(BMR * 16 * p.prep_refd);
#pragma unroll
            for (int j = 0; j < C_::REF_OPS; ++j) {
                const unsigned o = (unsigned)(j * 1024 + lane * 16);
                dma16(rf, st + C_::REF_OFF + j * 1024, o < rbytes ? (unsigned)m0 * 16u * (unsigned)p.prep_refd + o : OOB);
            }
        }
    };

    __syncthreads();   // parameters visible; no DMA in flight yet
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < cnt) issue(s);

    const int cl0 = wave * NC * 4 + (lane >> 4) * NC;   // this lane's first column in the group
    // PREP: this lane's level (lane >> 4, fixed for the launch) and its shape, selected once and
    // pinned in VGPRs.  Selected inside the loop, the compiler turned the select chain into an
    // indexed load from the kernel-argument segment, and that load's s_waitcnt vmcnt(0) before
    // the epilogue also waited for the DMA of the next row tile: the ring's prefetch was exposed
    // once per tile
    int lvl_H = 0, lvl_W = 0;
    if constexpr (PREP) {
        const int l = lane >> 4;
        lvl_H = l == 0 ? p.prep_H[0] : l == 1 ? p.prep_H[1] : l == 2 ? p.prep_H[2] : p.prep_H[3];
        lvl_W = l == 0 ? p.prep_W[0] : l == 1 ? p.prep_W[1] : l == 2 ? p.prep_W[2] : p.prep_W[3];
        asm volatile("" : "+v"(lvl_H), "+v"(lvl_W));
    }
    uint32_t pend[TMR][PW] = {};
    int pend_m0 = 0;
    // packed outputs of one row tile: ALWAYS S buffer stores per lane (offsets past the
    // descriptor for rows / columns outside C and for the dummy call of iteration 0), so the
    // counted waits below know exactly how many vector-memory ops are younger than a DMA
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(p.C, (short)0, p.c_bytes, 0x00020000);
    constexpr int EPC16 = 16 / (int)sizeof(TO);     // elements per 16-byte store
    // store unit: 16 bytes, or 4 columns when a lane's NC columns are not whole 16-byte runs
    // (NT = 3: 12 columns = 16-bit 8-byte units, never straddling a head of 4k columns; the
    // 9-wave K = 288 groups without LayerNorm store 4-column units too: head-major d = 36)
    constexpr int SU = (NC % EPC16 == 0 && !(KC == 9 && NT == 2 && !LN)) ? EPC16 : 4;
    constexpr int NU = NC / SU;                     // store units per lane-row
    constexpr int WPU = SU * (int)sizeof(TO) / 4;   // packed words per unit
    // stores per lane per row tile (PREP: one 16-byte location store + one 8-byte weight store)
    constexpr int S = TMR * (PREP ? 2 : NU);
    static_assert(NS >= 2 && NS <= 4 && (NS - 2) * (C_::D + S) <= 63, "ring depth / vmcnt range");
    // element offset of (row m, column n): m * rs + colpart(n); head-major (hm_rows > 0):
    // ((g*hm_batch + b)*hm_rows + s)*hm_d + d = g*M*hm_d + m*hm_d + d for m = b*hm_rows + s;
    // split head-major (hm_split > 0): columns n >= hm_split in the second plane at
    // hm_split*M elements, row stride hm_d2 (one 4-column unit per head)
    const int rs = PREP ? 96 / (int)sizeof(TO) : (p.hm_rows ? p.hm_d : p.ldc);
    constexpr int NSL = PREP ? 2 : NU;
    unsigned s_lo[TMR][NSL];
    unsigned s_rs[NSL];
    bool s_nok[NSL];
    if constexpr (PREP) {
        // record (head h, row m) at (h*M + m)*96 bytes: [4 levels x 16 B locations | 4 levels x 8 B weights];
        // this lane writes level lane >> 4 of head blockIdx.y*NW + wave
        const unsigned hb = (unsigned)(blockIdx.y * NW + wave) * (unsigned)M;
        const unsigned l = (unsigned)(lane >> 4);
#pragma unroll
        for (int t = 0; t < TMR; ++t) {
            const unsigned r = (hb + (unsigned)(t * 16 + (lane & 15))) * 96u;
            s_lo[t][0] = r + l * 16u;
            s_lo[t][1] = r + 64u + l * 8u;
        }
        s_nok[0] = s_nok[1] = false;
        s_rs[0] = s_rs[1] = (unsigned)rs;
    }
#pragma unroll
    for (int h = 0; h < (PREP ? 0 : NU); ++h) {
        const int n = ncol0 + cl0 + h * SU;
        s_nok[h] = n >= N;
        unsigned colpart = (unsigned)n, r_s = (unsigned)rs;
        if (p.hm_rows) {
            if (p.hm_split && n >= p.hm_split) {
                const int n2 = n - p.hm_split, g = n2 / p.hm_d2;
                colpart = (unsigned)p.hm_split * (unsigned)M + (unsigned)g * (unsigned)M * (unsigned)p.hm_d2 +
                          (unsigned)(n2 - g * p.hm_d2);
                r_s = (unsigned)p.hm_d2;
            } else {
                const int g = n / p.hm_d;
                colpart = (unsigned)g * (unsigned)M * (unsigned)p.hm_d + (unsigned)(n - g * p.hm_d);
            }
        }
        s_rs[h] = r_s;
#pragma unroll
        for (int t = 0; t < TMR; ++t)
            s_lo[t][h] = ((unsigned)(t * 16 + (lane & 15)) * r_s + colpart) * (unsigned)sizeof(TO);
    }
    // head-major outputs of 32-column heads (the d = 256 value projections): each wave's 16 x 64
    // output block is 2 heads; transposed through LDS (the pending tile's ring slot, free after the
    // tile's barrier until the next DMA is issued into it) so each store instruction writes one
    // head plane's 16 rows x 64 B = 1 KiB contiguous instead of 8-byte pieces 64 B apart
    constexpr bool HM32_OK = !PREP && !LN && sizeof(TO) == 2 && NC == 16 && WPU == 4 && TMR * 2048 * NW <= C_::STAGE;
    const bool hm32 = HM32_OK && p.hm_tr && p.hm_rows && p.hm_d == 32 && !p.hm_split && N % 64 == 0;
    int pend_slot = 0;
    auto store_pending = [&](bool valid) {
        if constexpr (HM32_OK) {
            if (hm32) {
                if (!valid) return;   // nothing pending (and pend_slot may be the slot about to be computed)
                char* scr = stages + pend_slot * C_::STAGE + wave * (TMR * 2048);
                const int g = lane >> 4, r = lane & 15;
#pragma unroll
                for (int t = 0; t < TMR; ++t) {
                    char* b = scr + t * 2048 + (g >> 1) * 1024 + r * 64 + (g & 1) * 32;
                    *reinterpret_cast<u32x4*>(b) = u32x4{pend[t][0], pend[t][1], pend[t][2], pend[t][3]};
                    *reinterpret_cast<u32x4*>(b + 16) = u32x4{pend[t][4], pend[t][5], pend[t][6], pend[t][7]};
                }
                const int hg0 = (ncol0 + wave * 64) >> 5;
                const bool wok = ncol0 + wave * 64 < N;
#pragma unroll
                for (int t = 0; t < TMR; ++t)
#pragma unroll
                    for (int hl = 0; hl < 2; ++hl) {
                        const u32x4 w = *reinterpret_cast<const u32x4*>(scr + t * 2048 + hl * 1024 + lane * 16);
                        const int row = pend_m0 + t * 16 + (lane >> 2);
                        const unsigned off = (wok && row < M) ? (((unsigned)(hg0 + hl) * (unsigned)M + (unsigned)row) * 32u +
                                                                 (unsigned)(lane & 3) * 8u) * 2u
                                                              : OOB;
                        __builtin_amdgcn_raw_buffer_store_b128(w, rc, off, 0, 0);
                    }
                return;
            }
        }
        if constexpr (PREP) {
            const unsigned base = (unsigned)pend_m0 * (unsigned)rs * (unsigned)sizeof(TO);
#pragma unroll
            for (int t = 0; t < TMR; ++t) {
                const bool mok = valid && pend_m0 + t * 16 + (lane & 15) < M;
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{pend[t][0], pend[t][1], pend[t][2], pend[t][3]}, rc,
                                                       mok ? base + s_lo[t][0] : OOB, 0, 0);
                typedef uint32_t u32x2_ __attribute__((ext_vector_type(2)));
                __builtin_amdgcn_raw_buffer_store_b64(u32x2_{pend[t][4], pend[t][5]}, rc, mok ? base + s_lo[t][1] : OOB,
                                                      0, 0);
            }
            return;
        }
#pragma unroll
        for (int t = 0; t < TMR; ++t) {
            const bool mok = valid && pend_m0 + t * 16 + (lane & 15) < M;
#pragma unroll
            for (int h = 0; h < NU; ++h) {
                const unsigned base = (unsigned)pend_m0 * s_rs[h] * (unsigned)sizeof(TO);
                const unsigned off = (mok && !s_nok[h]) ? base + s_lo[t][h] : OOB;
                if constexpr (WPU == 4) {
                    __builtin_amdgcn_raw_buffer_store_b128(
                        u32x4{pend[t][4 * h], pend[t][4 * h + 1], pend[t][4 * h + 2], pend[t][4 * h + 3]}, rc, off, 0, 0);
                } else {
                    typedef uint32_t u32x2_ __attribute__((ext_vector_type(2)));
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2_{pend[t][2 * h], pend[t][2 * h + 1]}, rc, off, 0, 0);
                }
            }
        }
    };

    for (int i = 0; i < cnt; ++i) {
        // retire tile i's DMA.  Younger vector-memory ops: the DMA of the (NS-2) later tiles
        // (D each) and the stores (S each) of the min(i, NS-2) iterations issued after it
        if (i + NS - 2 >= cnt) wait_vmcnt<0>();
        else if (NS <= 2 || i >= NS - 2) wait_vmcnt<(NS - 2) * (C_::D + S)>();
        else if (i == 0) wait_vmcnt<(NS - 2) * C_::D>();
        else wait_vmcnt<(NS - 2) * C_::D + S>();   // i == 1 (NS == 4)
        if (HAS_A2) {
            // q = src + pos rounded to the operand type, exactly as gemm.hip's load-time add:
            // each thread sums the chunks its own DMA delivered (landed: the wait above), once
            // per tile instead of once per wave; the barrier publishes the sums
            char* st = stages + (i % NS) * C_::STAGE;
#pragma unroll
            for (int j = 0; j < C_::A_OPS; ++j) {
                u32x4* pa = reinterpret_cast<u32x4*>(st + (j * NTHR + tid) * 16);
                *pa = Mma<T>::add(*pa, *reinterpret_cast<const u32x4*>(st + C_::A_SPAN + (j * NTHR + tid) * 16));
            }
        }
        lds_barrier();
        // PREP: the tile's mask bytes and reference points read BEFORE the next tile's DMA is
        // issued: an LDS read after it gets an s_waitcnt vmcnt(0) from the compiler (it cannot
        // prove the DMA's stage disjoint), which would wait for that DMA before the epilogue
        float4 pref[PREP ? TMR : 1];
        bool pmask[PREP ? TMR : 1];
        if constexpr (PREP) {
            const char* sc = stages + (i % NS) * C_::STAGE;
#pragma unroll
            for (int t = 0; t < TMR; ++t) {
                const int rl = t * 16 + (lane & 15), l = lane >> 4;
                pmask[t] = sc[C_::MASK_OFF + rl] != 0;
                pref[t] = *reinterpret_cast<const float4*>(sc + C_::REF_OFF + (rl * 4 + l) * (p.prep_refd == 2 ? 8 : 16));
            }
        }
        store_pending(i > 0);
        if (hm32) lds_barrier();   // every wave done with its transpose scratch (the slot refilled below)
        if (i + NS - 1 < cnt) issue(i + NS - 1);

        const char* st = stages + (i % NS) * C_::STAGE;
        const int m0 = (bx + i * P) * BMR;
        f32x4 acc[NT][TMR];
#pragma unroll
        for (int a = 0; a < NT; ++a)
#pragma unroll
            for (int t = 0; t < TMR; ++t) {
                // PREP: the accumulators start at the bias (one LDS read per 4 columns instead of
                // an add per column after the K loop)
                if constexpr (PREP) acc[a][t] = *reinterpret_cast<const f32x4*>(par + GW + cl0 + a * 4);
                else acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
        for (int c = 0; c < KC; ++c)
#pragma unroll
            for (int t = 0; t < TMR; ++t) {
                const int row = t * 16 + (lane & 15);
                const int q = c * 4 + (lane >> 4);
                const int xo = row * C_::ROW + (C_::sw(row, q) << 4);
                const u32x4 xf = *reinterpret_cast<const u32x4*>(st + xo);
#pragma unroll
                for (int a = 0; a < NT; ++a) Mma<T>::run(acc[a][t], wf[a][c], xf);
            }

        // ---- epilogue (registers) ----
        float v[TMR][NC];
        if constexpr (PREP) {
#pragma unroll
            for (int t = 0; t < TMR; ++t) {
#pragma unroll
                for (int j = 0; j < NC; ++j) v[t][j] = acc[j >> 2][t][j & 3];
                prep_records(p, pref[t], pmask[t], lvl_H, lvl_W, v[t], pend[t]);
            }
            pend_m0 = m0;
            continue;
        }
#pragma unroll
        for (int t = 0; t < TMR; ++t) {
            const int rl = t * 16 + (lane & 15);
#pragma unroll
            for (int j = 0; j < NC; ++j)
                v[t][j] = acc[j >> 2][t][j & 3] * par[cl0 + j] + par[GW + cl0 + j];
            if constexpr (HAS_R && NC % 8 == 0) {
#pragma unroll
                for (int h = 0; h < NC / 8; ++h) {
                    const int q = (cl0 >> 3) + h;
                    const u32x4 u = *reinterpret_cast<const u32x4*>(st + C_::R_OFF + rl * C_::R_ROW +
                                                                    (C_::rsw(rl, q) << 4));
                    float r8[8];
                    unpack8(u, r8, std::is_same<TO, f16_t>::value);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[t][h * 8 + e] += r8[e];
                }
            } else if constexpr (HAS_R) {
                // 4-column pieces (NT = 3: a lane's 12 columns start at a multiple of 4)
#pragma unroll
                for (int h = 0; h < NC / 4; ++h) {
                    const int col = cl0 + 4 * h, q = col >> 3;
                    const uint2 u = *reinterpret_cast<const uint2*>(st + C_::R_OFF + rl * C_::R_ROW +
                                                                    (C_::rsw(rl, q) << 4) + ((col >> 2) & 1) * 8);
                    float r8[8];
                    unpack8(u32x4{u.x, u.y, 0u, 0u}, r8, std::is_same<TO, f16_t>::value);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[t][h * 4 + e] += r8[e];
                }
            }
            if (p.relu)
#pragma unroll
                for (int j = 0; j < NC; ++j) v[t][j] = fmaxf(v[t][j], 0.f);
        }
        if (LN) {
            // columns past N are exactly 0 here (zero W rows, zero bias, zero residual)
            float mean[TMR], rstd[TMR];
#pragma unroll
            for (int t = 0; t < TMR; ++t) {
                float s = 0.f;
#pragma unroll
                for (int j = 0; j < NC; ++j) s += v[t][j];
                s += __shfl_xor(s, 16);
                s += __shfl_xor(s, 32);
                if ((lane >> 4) == 0) lns[(t * 16 + (lane & 15)) * NW + wave] = s;
            }
            lds_barrier();
#pragma unroll
            for (int t = 0; t < TMR; ++t) {
                mean[t] = wave_sum<NW>(lns + (t * 16 + (lane & 15)) * NW) / (float)N;
                float q = 0.f;
#pragma unroll
                for (int j = 0; j < NC; ++j) {
                    const float d = (ncol0 + cl0 + j < N) ? v[t][j] - mean[t] : 0.f;
                    q += d * d;
                }
                q += __shfl_xor(q, 16);
                q += __shfl_xor(q, 32);
                if ((lane >> 4) == 0) lns[BMR * NW + (t * 16 + (lane & 15)) * NW + wave] = q;
            }
            lds_barrier();
#pragma unroll
            for (int t = 0; t < TMR; ++t) {
                rstd[t] = rsqrtf(wave_sum<NW>(lns + BMR * NW + (t * 16 + (lane & 15)) * NW) / (float)N + p.ln_eps);
#pragma unroll
                for (int j = 0; j < NC; ++j)
                    v[t][j] = (v[t][j] - mean[t]) * rstd[t] * par[2 * GW + cl0 + j] + par[3 * GW + cl0 + j];
            }
        }
#pragma unroll
        for (int t = 0; t < TMR; ++t) {
            const int rl = t * 16 + (lane & 15);
            if (st[C_::MASK_OFF + rl])
#pragma unroll
                for (int j = 0; j < NC; ++j) v[t][j] = 0.f;
#pragma unroll
            for (int j4 = 0; j4 < NC / 4; ++j4) Pack<TO>::put(&pend[t][j4 * Pack<TO>::WORDS_PER_4], &v[t][j4 * 4]);
        }
        pend_m0 = m0;
        pend_slot = i % NS;
    }
    if (cnt > 0) {
        if (hm32) lds_barrier();   // the last tile's slot: every wave done reading it
        store_pending(true);
    }
}

template <typename T, typename TO, int KC, int BMR, int NS, bool HAS_R, bool LN, bool HAS_A2 = false, int NT = 4,
          bool CR = false, bool PREP = false, int OCC = 2, int NW = 4>
void launch_cfg(const GemmArgs& a, hipStream_t stream) {
    constexpr int GW = NW * NT * 16;
    const int n_mtiles = (a.M + BMR - 1) / BMR;
    const int ng = (a.N + GW - 1) / GW;
    // 2 resident workgroups per CU over all groups: never more than the 512 slots (a second
    // round of workgroups would double the launch), and a multiple of 8 so the column groups
    // of one row tile land on one XCD (linear id bx + y*P) and share its L2 copy of the tile
    // (OCC resident workgroups per CU: 256 * OCC slots)
    const int slots = 256 * OCC;
    int P = slots / ng >= 8 ? slots / ng / 8 * 8 : slots / ng;
    if (P > n_mtiles) P = n_mtiles;
    dim3 grid(P, ng), block(NW * 64);
    hipLaunchKernelGGL((gemm_rw_kernel<T, TO, KC, NT, BMR, NS, HAS_R, LN, HAS_A2, CR, PREP, OCC, NW>), grid, block, 0,
                       stream, a, n_mtiles);
}

// deepest DMA ring (<= 4 row tiles) that keeps the workgroup within 80 KiB of LDS (two per CU)
template <int KC, int BMR, bool HAS_R, bool LN, bool HAS_A2, int NT = 4, bool PREP = false, int NW = 4,
          int BUDGET = 80 * 1024>
constexpr int ring_depth() {
    constexpr int base = RwCfg<KC, NT, BMR, 1, HAS_R, LN, HAS_A2, PREP, NW>::BYTES -
                         RwCfg<KC, NT, BMR, 1, HAS_R, LN, HAS_A2, PREP, NW>::STAGE;
    constexpr int stage = RwCfg<KC, NT, BMR, 1, HAS_R, LN, HAS_A2, PREP, NW>::STAGE;
    return (BUDGET - base) / stage >= 4 ? 4 : (BUDGET - base) / stage;
}

// K = 288 (d = 288: configs 3-5): 16-row tiles, 12 columns per lane (NT = 3, 108 weight VGPRs;
// 180-210 in all: two waves per SIMD).  LayerNorm rows (N <= 288) need the whole row in one
// workgroup: 9 waves x 32 columns (NT = 2, 126-152 VGPRs; the 6-wave x 48-column group under
// flag 4194304), one workgroup per CU with a ring of up to 4 tiles in 160 KiB; the other
// epilogues take 4-wave 192-column groups, two per CU (a row tile is shared by its groups
// through the XCD's L2, as at K = 256).
template <typename T, typename TO, bool HAS_R, bool LN, bool HAS_A2, int NW, int NT = 3, int OCC = NW == 4 ? 2 : 1>
void launch_288(const GemmArgs& a, hipStream_t stream) {
    constexpr int NS = ring_depth<9, 16, HAS_R, LN, HAS_A2, NT, false, NW, 160 * 1024 / OCC>();
    static_assert(NS >= 2, "LDS budget");
    launch_cfg<T, TO, 9, 16, NS, HAS_R, LN, HAS_A2, NT, false, false, OCC, NW>(a, stream);
}

template <typename T, typename TO, int KC, bool HAS_R, bool LN, bool HAS_A2, int NT = 4>
void launch_ring(const GemmArgs& a, hipStream_t stream) {
    // 16-row tiles when a tile carries a second operand (residual / A2) or the LayerNorm
    // epilogue (which needs them at K = 256 to stay in 256 VGPRs) or a K of 512+ (1-2 KiB
    // rows): a 2-4 deep ring then fits; K = 64 rows (128 B) need 32-row tiles for whole 4 KiB
    // DMA rounds
    constexpr int BMR = (KC == 2 || (KC <= 8 && !HAS_R && !LN && !HAS_A2)) ? 32 : 16;
    constexpr int NS = ring_depth<KC, BMR, HAS_R, LN, HAS_A2, NT>();
    static_assert(NS >= 2, "LDS budget");
    if constexpr (BMR == 32 && KC >= 4) {
        // flag 131072 (tests): the same problem on 16-row tiles -- the 32-row tiles' two MFMA row
        // tiles per wave (TMR = 2) must give the 16-row tiles' results bit for bit
        if (kinet_gemm_flags & 131072) {
            constexpr int NS16 = ring_depth<KC, 16, HAS_R, LN, HAS_A2, NT>();
            launch_cfg<T, TO, KC, 16, NS16, HAS_R, LN, HAS_A2, NT>(a, stream);
            return;
        }
    }
    launch_cfg<T, TO, KC, BMR, NS, HAS_R, LN, HAS_A2, NT>(a, stream);
}

template <typename T, typename TO, int KC, int NT = 4>
void launch_k(const GemmArgs& a, hipStream_t stream) {
    const bool r = a.R != nullptr, ln = a.ln_g != nullptr;
    if (a.A2 != nullptr) {
        // the query + position-embedding projections (no residual / LayerNorm there)
        if (r || ln) return;
        launch_ring<T, TO, KC, false, false, true, NT>(a, stream);
    } else if (r && ln) launch_ring<T, TO, KC, true, true, false, NT>(a, stream);
    else if (r) {
        // + residual with N > 256 (the stage-end conv3s, 128 -> 512 and 256 -> 1024): 8-wave
        // 512-column groups, one workgroup per CU, so each row tile's x rows are fetched by half as
        // many groups (one instead of two at N = 512); flag 268435456: the 4-wave 256-column groups
        if constexpr (NT == 4 && KC <= 8) {
            if (a.N > 256 && !(kinet_gemm_flags & 268435456)) {
                constexpr int NS8 = ring_depth<KC, 16, true, false, false, 4, false, 8, 160 * 1024>();
                launch_cfg<T, TO, KC, 16, NS8, true, false, false, 4, false, false, 1, 8>(a, stream);
                return;
            }
        }
        launch_ring<T, TO, KC, true, false, false, NT>(a, stream);
    } else if (ln) launch_ring<T, TO, KC, false, true, false, NT>(a, stream);
    // (plain epilogues keep the 4-wave groups: 8-wave 512-column groups ran config 2's six decoder
    // value projections (N = 1536) slower, 669 vs 648 us, profiles/r06ar_wide_8wave_ab.txt)
    else launch_ring<T, TO, KC, false, false, false, NT>(a, stream);
}

// K = 512 (the ResNet 1x1 convs into the layer-2 bottlenecks, input_proj of level 0): the
// weight slice stays at 128 VGPRs per wave by narrowing the column group to 128 columns
// (NT = 2) -- the host routes only N <= 256 without residual / LayerNorm / A2 here (at most
// 2 column groups, which share each row tile through the XCD's L2)
template <typename T, typename TO>
void launch_t(const GemmArgs& a, hipStream_t stream) {
    if (a.K == 288) {
        const bool r = a.R != nullptr, ln = a.ln_g != nullptr;
        if (a.A2 != nullptr) {
            // x + pos rows (the d = 288 offsets / logits and value projections): one 8-wave group of
            // up to 384 columns per row tile, so each tile's x + pos rows are read once -- as the
            // records GEMM (kinet_msda_sample_records); flag 268435456: the 4-wave 192-column groups
            if (a.N > 192 && a.N <= 384 && !(kinet_gemm_flags & 268435456)) launch_288<T, TO, false, false, true, 8, 3, 1>(a, stream);
            else launch_288<T, TO, false, false, true, 4>(a, stream);
            return;
        }
        // LayerNorm rows: 9 waves x 32 columns (one 288-column group; flag 4194304: the 6-wave x
        // 48-column groups, A/B and tests); without LayerNorm 4-wave 192-column groups (one 9-wave
        // group measured within noise, round 5: profiles/r05s_split_nine_waves.log)
        if (r && ln) {
            if (kinet_gemm_flags & 4194304) launch_288<T, TO, true, true, false, 6>(a, stream);
            else launch_288<T, TO, true, true, false, 9, 2>(a, stream);
        } else if (ln) {
            if (kinet_gemm_flags & 4194304) launch_288<T, TO, false, true, false, 6>(a, stream);
            else launch_288<T, TO, false, true, false, 9, 2>(a, stream);
        } else if (r) {
            launch_288<T, TO, true, false, false, 4>(a, stream);
        } else if (a.N > 384 && !(kinet_gemm_flags & 268435456)) {
            // N > 384 (the d = 288 decoder's six value projections in one launch, N = 1728): 8-wave
            // 384-column groups, one workgroup per CU -- half as many groups fetch each row tile:
            // 1048 -> 948 us in config 3 (profiles/r06ar_wide_8wave_ab.txt); at 192 < N <= 384 (the
            // value projection's split planes) 89 vs 91 us, bench within noise: not taken (r06at)
            launch_288<T, TO, false, false, false, 8, 3, 1>(a, stream);
        } else {
            launch_288<T, TO, false, false, false, 4>(a, stream);
        }
        return;
    }
    if (a.K == 64) launch_k<T, TO, 2>(a, stream);
    else if (a.K == 128) launch_k<T, TO, 4>(a, stream);
    else if (a.K == 256) launch_k<T, TO, 8>(a, stream);
    else if (a.N > 128 && a.N <= 256 && !(kinet_gemm_flags & 268435456)) {
        // K == 512, N == 256 (config 2's level-0 input projection, 512 -> 256): one 8-wave
        // 256-column group per row tile, one workgroup per CU, so each tile's 1 KiB rows are read
        // once (the two 4-wave 128-column groups fetched 2x the operand, profiles/pmc_traffic.json)
        constexpr int NS = ring_depth<16, 16, false, false, false, 2, false, 8, 160 * 1024>();
        launch_cfg<T, TO, 16, 16, NS, false, false, false, 2, false, false, 1, 8>(a, stream);
    } else launch_ring<T, TO, 16, false, false, false, 2>(a, stream);   // K == 512
}

bool al16(const void* p) { return (((uintptr_t)p) & 15u) == 0; }

}  // namespace

thread_local int rw_min_m = 4096;   // smallest M routed to the resident-weight kernel (kinet_gemm_set_flags bit 3: 256)

// Entry from gemm.hip's dispatcher: launch the resident-weight kernel when the problem
// fits it; false leaves the call to the tiled kernel.
bool launch_rw(const GemmArgs& a, int in_dtype, int out_dtype, hipStream_t stream) {
    if (in_dtype != KINET_BF16 && in_dtype != KINET_F16) return false;
    if (a.M < rw_min_m || (a.K != 64 && a.K != 128 && a.K != 256 && a.K != 512 && a.K != 288)) return false;
    if (a.K == 288 && (kinet_gemm_flags & 1048576)) return false;   // flag: K = 288 on the tiled kernels (A/B)
    if (a.K == 512 && (a.N > 256 || a.R != nullptr || a.ln_g != nullptr || a.A2 != nullptr || (kinet_gemm_flags & 256)))
        return false;
    if (a.A2 != nullptr && (a.R != nullptr || a.ln_g != nullptr || !al16(a.A2))) return false;
    if (a.N % 8 != 0 || (a.ln_g != nullptr && a.N > (a.K == 288 ? 288 : 256))) return false;
    const bool o16 = out_dtype == in_dtype || (in_dtype == KINET_BF16 && out_dtype == KINET_F16);
    const bool o32 = out_dtype == KINET_F32;
    if (!o16 && !o32) return false;
    if (o16 ? (a.ldc % 8 != 0) : (a.ldc % 4 != 0)) return false;
    if (!al16(a.C) || (a.R != nullptr && (!o16 || a.ldr % 8 != 0 || !al16(a.R)))) return false;
    // head-major stores: 16-byte units need hm_d % 8 == 0; the K = 288 path stores 4-column
    // units (hm_d % 4 == 0) and takes the split planes (hm_d2 == 4)
    if (a.hm_rows && (a.K == 288 ? (a.hm_d % 4 != 0 || (a.hm_split && (a.hm_d2 != 4 || a.hm_split % a.hm_d != 0)))
                                 : (a.hm_d % 8 != 0 || a.hm_split)))
        return false;
    // output descriptor extent (buffer stores; offsets must stay below 2^31)
    const long long osz = out_dtype == KINET_F32 ? 4 : 2;
    const long long cb = a.hm_rows ? (long long)a.M * a.N * osz
                                   : (a.M > 0 ? ((long long)(a.M - 1) * a.ldc + a.N) * osz : 0);
    if (cb >= (1LL << 31)) return false;
    GemmArgs ac = a;
    ac.c_bytes = (int)cb;
    ac.hm_tr = (kinet_gemm_flags & 1073741824) ? 0 : 1;   // flag: 32-column head-major stores without the LDS transpose (A/B)
    if (in_dtype == KINET_BF16) {
        if (out_dtype == KINET_F16) launch_t<bf16_t, f16_t>(ac, stream);
        else if (o16) launch_t<bf16_t, bf16_t>(ac, stream);
        else launch_t<bf16_t, float>(ac, stream);
    } else {
        if (o16) launch_t<f16_t, f16_t>(ac, stream);
        else launch_t<f16_t, float>(ac, stream);
    }
    return true;
}

// Entry from gemm.hip's conv dispatcher: the KH x 1, horizontally stride-1 unpadded conv of
// the tap-folded stem (K = KH*Cin <= 256) as a resident-weight stream with the conv-row gather
// (a short-K conv in the tiled kernel exposes a full load latency per 3-step tile); false
// leaves the call to the tiled kernel.
bool launch_rw_conv(const GemmArgs& a, int in_dtype, hipStream_t stream) {
    if (in_dtype != KINET_BF16 && in_dtype != KINET_F16) return false;
    // strided 1x1 (the ResNet downsample of stage 2, 256 -> 512 at stride 2): row m = output
    // pixel, its A row = input pixel (img, 2 oh, 2 ow) -- the conv-row DMA with a horizontal
    // stride; weights resident (K = 256), 256-column groups sharing each row tile through L2.
    // The implicit-GEMM kernel ran it at ~310 TF/s (1.8 TB/s of compulsory bytes)
    if (a.K == 256 && a.Cin == 256 && a.KW == 1 && a.pad == 0 && a.pad_w == 0 && a.stride > 1 &&
        a.stride_w == a.stride && a.M >= rw_min_m && a.Wout >= 32 && a.N % 256 == 0 && a.R == nullptr &&
        a.ln_g == nullptr && a.row_mask == nullptr && a.ldc % 8 == 0 && al16(a.C) && !(kinet_gemm_flags & 2048)) {
        const long long cb = ((long long)(a.M - 1) * a.ldc + a.N) * 2;
        if (cb >= (1LL << 31)) return false;
        GemmArgs ac = a;
        ac.c_bytes = (int)cb;
        constexpr int NS = ring_depth<8, 32, false, false, false, 4>();
        constexpr int NS16 = ring_depth<8, 16, false, false, false, 4>();
        if (kinet_gemm_flags & 131072) {   // tests: 16-row tiles (bit-identical to the 32-row ones)
            if (in_dtype == KINET_BF16) launch_cfg<bf16_t, bf16_t, 8, 16, NS16, false, false, false, 4, true>(ac, stream);
            else launch_cfg<f16_t, f16_t, 8, 16, NS16, false, false, false, 4, true>(ac, stream);
            return true;
        }
        if (in_dtype == KINET_BF16) launch_cfg<bf16_t, bf16_t, 8, 32, NS, false, false, false, 4, true>(ac, stream);
        else launch_cfg<f16_t, f16_t, 8, 32, NS, false, false, false, 4, true>(ac, stream);
        return true;
    }
    if (a.M < rw_min_m || a.K > 256 || a.KW != 1 || a.stride_w != 1 || a.pad_w != 0 || a.Win != a.Wout) return false;
    if (a.Cin % 8 != 0 || a.Wout < 32 || a.N > 128 || a.N % 8 != 0 || a.R != nullptr || a.ln_g != nullptr) return false;
    if (a.ldc % 8 != 0 || !al16(a.C) || a.row_mask != nullptr) return false;
    const long long cb = ((long long)(a.M - 1) * a.ldc + a.N) * 2;
    if (cb >= (1LL << 31)) return false;
    GemmArgs ac = a;
    ac.c_bytes = (int)cb;
    constexpr int NS = ring_depth<8, 32, false, false, false>();
    constexpr int NS16 = ring_depth<8, 16, false, false, false>();
    if (kinet_gemm_flags & 131072) {   // tests: 16-row tiles (bit-identical to the 32-row ones)
        if (in_dtype == KINET_BF16) launch_cfg<bf16_t, bf16_t, 8, 16, NS16, false, false, false, 2, true>(ac, stream);
        else launch_cfg<f16_t, f16_t, 8, 16, NS16, false, false, false, 2, true>(ac, stream);
        return true;
    }
    if (in_dtype == KINET_BF16) launch_cfg<bf16_t, bf16_t, 8, 32, NS, false, false, false, 2, true>(ac, stream);
    else launch_cfg<f16_t, f16_t, 8, 32, NS, false, false, false, 2, true>(ac, stream);
    return true;
}

}  // namespace kinet

using namespace kinet;

// The MSDA sampling-offsets | attention-weights projection of an encoder call, with the
// softmax, sampling locations and bilinear setup in its epilogue (prep_records): writes the
// head-major sampling records kinet_msda_encoder_forward_records reads.  include/kinet_msda.h.
extern "C" int kinet_msda_sample_records(const void* A, const void* A2, const void* W, const float* bias, int M,
                                         int num_heads, int K, int lda, int in_dtype, const float* ref_points,
                                         int ref_dim, const uint8_t* query_attn_mask, const int64_t* spatial_shapes_host,
                                         int num_levels, int num_point, int frac_bits, void* records,
                                         int a2_rows, kinet_stream_t stream) {
    KINET_CHECK_ARG(a2_rows == 0 || (A2 != nullptr && a2_rows >= 32 && M % a2_rows == 0),
                    "msda records: a2_rows must be 0 or >= 32 dividing M (got %d)", a2_rows);
    KINET_CHECK_ARG(M >= 0 && num_heads > 0 && num_heads % 4 == 0, "msda records: heads must be a multiple of 4 (got %d)",
                    num_heads);
    KINET_CHECK_ARG(num_levels == 4 && num_point == 4, "msda records: 4 levels x 4 points (got %d, %d)", num_levels,
                    num_point);
    KINET_CHECK_ARG(K == 256 && lda % 8 == 0 && lda >= K, "msda records: K must be 256 (got %d), lda %% 8 == 0", K);
    KINET_CHECK_ARG(in_dtype == KINET_BF16 || in_dtype == KINET_F16, "msda records: bf16 / f16 operands");
    KINET_CHECK_ARG(ref_dim == 2 || ref_dim == 4, "Last dim of reference_points must be 2 or 4, but get %d instead.",
                    ref_dim);
    KINET_CHECK_ARG(frac_bits >= 6 && frac_bits <= 10, "msda records: frac_bits in [6, 10] (got %d)", frac_bits);
    KINET_CHECK_ARG(spatial_shapes_host != nullptr && ref_points != nullptr && records != nullptr && W != nullptr &&
                        bias != nullptr, "msda records: NULL argument");
    KINET_CHECK_ARG((((uintptr_t)A) & 15) == 0 && (((uintptr_t)W) & 15) == 0 && (((uintptr_t)records) & 15) == 0 &&
                        (A2 == nullptr || (((uintptr_t)A2) & 15) == 0) && (((uintptr_t)ref_points) & 15) == 0,
                    "msda records: A, A2, W, refs and records must be 16-byte aligned");
    for (int l = 0; l < 4; ++l) {
        const long long H = spatial_shapes_host[2 * l], Wd = spatial_shapes_host[2 * l + 1];
        KINET_CHECK_ARG(H > 0 && Wd > 0 && H <= (1LL << (16 - frac_bits)) && Wd <= (1LL << (16 - frac_bits)),
                        "msda records: level %d (%lld x %lld) exceeds the %d-bit integer part", l, H, Wd, 16 - frac_bits);
    }
    if (M == 0) return KINET_OK;
    const int N = num_heads * 48;
    const long long ab = ((long long)(M - 1) * lda + K) * 2, bb = (long long)N * K * 2;
    const long long cb = (long long)num_heads * M * 96, rb = (long long)M * 16 * ref_dim;
    KINET_CHECK_ARG(ab < (1LL << 31) && cb < (1LL << 31) && rb < (1LL << 31), "msda records: operands larger than 2 GiB");
    GemmArgs a{};
    a.A = A; a.A2 = A2; a.B = W; a.C = records; a.bias = bias; a.row_mask = query_attn_mask; a.a2_rows = a2_rows;
    a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = K; a.ldc = N;
    a.a_bytes = (int)ab; a.b_bytes = (int)bb; a.c_bytes = (int)cb;
    a.prep_ref = ref_points; a.prep_refd = ref_dim; a.prep_fb = frac_bits;
    for (int l = 0; l < 4; ++l) {
        a.prep_H[l] = (int)spatial_shapes_host[2 * l];
        a.prep_W[l] = (int)spatial_shapes_host[2 * l + 1];
    }
    hipStream_t s = (hipStream_t)stream;
    constexpr int NS1 = ring_depth<8, 16, false, false, false, 3, true>();
    // With the position embedding added on load (A2, the encoder): ONE 8-wave 384-column group per
    // 16-row tile, one workgroup per CU (166 VGPRs, a 4-slot ring): each row tile's x + pos rows
    // are read once.  The two 4-wave 192-column groups before it (three workgroups per CU, a
    // 2-slot ring) were meant to share each row tile through the XCD's L2 (same XCD by linear id),
    // but PMC showed 1.11 GB fetched per batch-28 call against ~0.35 GB of operands: 270 -> 238 us
    // per call, encoder call 0.72-0.74 -> 0.69-0.70 ms, bench 1416 / 1429 -> 1441 / 1446 frames/s
    // interleaved, records bit-identical (profiles/r06am_records_8wave_ab.txt; two 8-wave groups per
    // CU: 245 us, 1435 / 1445).  Flag 268435456 keeps the 4-wave groups (A/B, tests).  Round 4's
    // notes on the 4-wave grid: three per CU beat two with a 4-slot ring under three streams
    // (profiles/r04z_occ_ab.log), four per CU spilled.  The 32-row tile (two MFMA row tiles per
    // wave) is not used here: its epilogue, interleaved by the compiler with the second tile's
    // MFMA chain, differed from the 16-row tile in a few hundred record words from run to run
    // (round 4-5)
    if (A2 && !(kinet_gemm_flags & 268435456)) {
        constexpr int NS8 = ring_depth<8, 16, false, false, true, 3, true, 8, 160 * 1024>();
        if (in_dtype == KINET_BF16) launch_cfg<bf16_t, f16_t, 8, 16, NS8, false, false, true, 3, false, true, 1, 8>(a, s);
        else launch_cfg<f16_t, f16_t, 8, 16, NS8, false, false, true, 3, false, true, 1, 8>(a, s);
        KINET_LAUNCH_CHECK();
        return KINET_OK;
    }
    if (in_dtype == KINET_BF16) {
        if (A2) launch_cfg<bf16_t, f16_t, 8, 16, 2, false, false, true, 3, false, true, 3>(a, s);
        else launch_cfg<bf16_t, f16_t, 8, 16, NS1, false, false, false, 3, false, true>(a, s);
    } else {
        if (A2) launch_cfg<f16_t, f16_t, 8, 16, 2, false, false, true, 3, false, true, 3>(a, s);
        else launch_cfg<f16_t, f16_t, 8, 16, NS1, false, false, false, 3, false, true>(a, s);
    }
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}
