// MFMA GEMM + implicit-GEMM NHWC convolution for gfx950 (CDNA4), fused epilogues.
//
// Tiling (DESIGN.md "GEMM / conv kernel"):
//  * workgroup = 256 threads = 4 waves in a WGM x WGN grid, output tile BM x BN, one
//    K-step = 128 bytes of K per row (64 bf16/f16 or 32 f32);
//  * operands staged global -> registers -> LDS, double-buffered LDS with ONE barrier
//    per K-step (the next tile's global loads are in flight under the current MFMAs);
//  * LDS rows are 128 B with the 16-byte chunk index XOR-swizzled by (row & 7), which
//    makes the ds_read_b128 fragment reads (16 rows x one chunk per lane group)
//    bank-conflict free;
//  * bf16/f16: v_mfma_f32_16x16x32_{bf16,f16}; f32 (parity mode): the exact-f32
//    v_mfma_f32_16x16x4_f32, 4 per 16-byte fragment;
//  * epilogue through LDS: the f32 accumulator tile is parked in the (now idle) staging
//    buffers, then each wave streams whole output rows -- 16-byte residual loads and
//    8/16-byte stores per lane, every row written by consecutive lanes (the direct
//    MFMA-layout store writes 32-byte pieces of 16 rows per instruction);  bias / folded
//    BatchNorm scale, residual add, ReLU, padding-row mask and, when one tile spans the
//    whole row (N <= BN), the post-norm LayerNorm (deformable_transformer.py:287 etc.)
//    are applied there, so the sub-layer output is written exactly once;
//  * optional second A operand added at load time (q = src + pos, deformable_transformer.py:
//    292, :369, :377) -- the bf16 sum is rounded exactly as a separate add would;
//  * blockIdx is remapped XCD-aware (bijective form, cdna_hip_programming.md T1) so the
//    tiles that share an activation panel run on one XCD and hit its L2;
//  * implicit conv: M = batch*Hout*Wout rows, K = KH*KW*Cin with Cin fastest (weights
//    permuted OIHW -> OHWI on the host); each 16-byte chunk lies inside one filter tap
//    (Cin % 8 == 0) so the im2col gather is a 16-byte load or a zero fill.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/kinet_gemm.h"
#include "common.h"
#include "gemm_common.h"

namespace kinet {
namespace {

// diagnostic kernel-selection flags (kinet_gemm_set_flags), by value: 2 = the 8-wave LDS-DMA
// tiles (gemm_dma.h) wherever eligible; 4 = never the resident-weight kernel (gemm_rw.hip);
// 8 = resident-weight kernel from M >= 256; 16 = LDS-DMA staging for the 4-wave tiles;
// 32 = never the dedicated stem convolution (stem.hip); 64 = no full-rounds split of the
// multi-tap convolutions; 128 = KINET_F32_X3 weight-gradient GEMM splitting at fragment-read time;
// 256 = no XCD placement of that GEMM's K-slices; 512 = the wave-per-row attention backward;
// 1024 = never the direct 3x3 64 -> 64 convolution (conv3x3.hip)
}  // namespace
// test / A-B selection knobs (kinet_gemm_set_flags, kinet_gemm_force_tile): per calling thread,
// never read by default paths except as "0 = automatic"
thread_local int kinet_gemm_flags = 0;   // declared in gemm_common.h (read by grad.hip too)
int kinet_solo_launch = 0;                 // declared in common.h (kinet_set_solo_launch)
namespace {
// diagnostic tile override for gemm_kernel (kinet_gemm_force_tile; 0 = heuristic)
thread_local int force_bm = 0, force_bn = 0;


template <int BM, int BN>
struct Smem {
    static constexpr int STAGE = (BM + BN) * ROWB;
    static constexpr int EPI_LD = BN + 4;                 // f32 row stride of the epilogue tile
    static constexpr int EPI = BM * EPI_LD * 4;
    static constexpr int BYTES = (2 * STAGE > EPI) ? 2 * STAGE : EPI;
};

// Residual rows of one epilogue pass, loaded ahead: every wave issues the loads of ALL its
// rows (branch-free buffer loads, zeros past the edges) before the accumulators are parked,
// so their latency overlaps the park + barrier instead of serialising one HBM round trip per
// row.  Used when the residual rows are 4-column aligned (ldr % 4 == 0, N % 4 == 0); other
// shapes fall back to in-loop loads.
template <typename TO, int BN, int NW, int ROWS>
struct ResRows {
    static constexpr int LPR = BN / 4 < 64 ? BN / 4 : 64;
    static constexpr int NCH = (BN + 4 * LPR - 1) / (4 * LPR);
    static constexpr int RPW = 64 / LPR;
    static constexpr int NR = (ROWS + NW * RPW - 1) / (NW * RPW);
    static constexpr int WPC = 4 * (int)sizeof(TO) / 4;   // 32-bit words per 4-column chunk
    uint32_t w[NR][NCH][WPC];
    bool on;

    __device__ __forceinline__ void issue(const GemmArgs& p, int m0, int n0, int r0, int wave, int lane) {
        on = p.R != nullptr && (p.ldr & 3) == 0 && (p.N & 3) == 0;
        if (!on) return;
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)p.R, (short)0, p.r_bytes, 0x00020000);
        const int lr = lane / LPR, lc = lane - (lane / LPR) * LPR;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            const int rl = wave * RPW + lr + i * NW * RPW;
            const int m = m0 + r0 + rl;
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                const int nl0 = (c * LPR + lc) * 4, n = n0 + nl0;
                const bool ok = rl < ROWS && m < p.M && nl0 < BN && n < p.N;
                const unsigned off = ok ? ((unsigned)m * (unsigned)p.ldr + (unsigned)n) * (unsigned)sizeof(TO) : 0x80000000u;
                if constexpr (WPC == 4) {
                    const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0));
                    for (int k = 0; k < 4; ++k) w[i][c][k] = v[k];
                } else {
                    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                    const u32x2 v = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rr, off, 0, 0));
                    w[i][c][0] = v[0];
                    w[i][c][1] = v[1];
                }
            }
        }
    }
    __device__ __forceinline__ void get(int i, int c, float* r) const {
        if constexpr (WPC == 4) {
            for (int k = 0; k < 4; ++k) r[k] = __uint_as_float(w[i][c][k]);
        } else if constexpr (std::is_same<TO, f16_t>::value) {
            for (int k = 0; k < 2; ++k) {
                r[2 * k] = (float)__builtin_bit_cast(f16_t, (uint16_t)(w[i][c][k] & 0xffffu));
                r[2 * k + 1] = (float)__builtin_bit_cast(f16_t, (uint16_t)(w[i][c][k] >> 16));
            }
        } else {
            for (int k = 0; k < 2; ++k) {
                r[2 * k] = __uint_as_float(w[i][c][k] << 16);
                r[2 * k + 1] = __uint_as_float(w[i][c][k] & 0xffff0000u);
            }
        }
    }
};

// Fused epilogue over tile rows [r0, r0 + ROWS): the f32 accumulators of those rows are
// parked in LDS at ep[(row - r0) * EPI_LD + col]; each wave streams whole rows (LPR lanes
// per row, 4 columns per lane): scale/bias, residual, ReLU, LayerNorm (DPP row reductions),
// row mask, plain or head-major store.
template <typename TO, int BN, int EPI_LD, int NW, bool LN, int ROWS>
__device__ __forceinline__ void epilogue_rows(const GemmArgs& p, const float* ep, int m0, int n0, int r0, int wave,
                                              int lane, const ResRows<TO, BN, NW, ROWS>& rp) {
    using RR = ResRows<TO, BN, NW, ROWS>;
    const int M = p.M, N = p.N;
    constexpr int LPR = RR::LPR, NCH = RR::NCH, RPW = RR::RPW;
    static_assert(64 % LPR == 0, "row mapping");
    TO* __restrict__ C = (TO*)p.C + (long)blockIdx.y * p.c_slice;
    const TO* __restrict__ R = (const TO*)p.R;
    const int lr = lane / LPR, lc = lane - (lane / LPR) * LPR;
    const bool ld_ok = ((p.ldc & 3) == 0) && (R == nullptr || (p.ldr & 3) == 0);
    float sc4[NCH][4], bi4[NCH][4], g4[NCH][4], be4[NCH][4];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            int nn = n0 + (c * LPR + lc) * 4 + r;
            nn = nn < N ? nn : N - 1;
            sc4[c][r] = p.scale ? p.scale[nn] : 1.f;
            bi4[c][r] = p.bias ? p.bias[nn] : 0.f;
            g4[c][r] = LN ? p.ln_g[nn] : 1.f;
            be4[c][r] = LN ? p.ln_b[nn] : 0.f;
        }
#pragma unroll
    for (int i = 0; i < RR::NR; ++i) {
        const int rl = wave * RPW + lr + i * NW * RPW;
        if (RR::NR * NW * RPW > ROWS && rl >= ROWS) break;   // (wave-uniform: ROWS % RPW == 0)
        const int rr = r0 + rl;
        const int m = m0 + rr;
        // (LN needs every lane of the row in the reductions, so no early exit on m)
        const bool mok = m < M;
        float v[NCH][4];
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int nl0 = (c * LPR + lc) * 4;
            const int n = n0 + nl0;
            const bool cin = nl0 < BN;
            f32x4 t = {0.f, 0.f, 0.f, 0.f};
            if (cin) t = *reinterpret_cast<const f32x4*>(ep + rl * EPI_LD + nl0);
            float res[4] = {0.f, 0.f, 0.f, 0.f};
            if (rp.on) {
                rp.get(i, c, res);
            } else if (R && mok && cin && n < N) {
                if (ld_ok && n + 3 < N) IO4<TO>::load(R + (long)m * p.ldr + n, res);
                else
                    for (int r = 0; r < 4; ++r)
                        if (n + r < N) res[r] = IO4<TO>::load1(R + (long)m * p.ldr + n + r);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float x = t[r] * sc4[c][r] + bi4[c][r] + res[r];
                if (p.relu) x = fmaxf(x, 0.f);
                x = (cin && n + r < N) ? x : 0.f;
                v[c][r] = x;
                s += x;
            }
        }
        if (LN) {
            s = group_reduce<LPR, false>(s);
            const float mean = s / (float)N;
            float q = 0.f;
#pragma unroll
            for (int c = 0; c < NCH; ++c)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int n = n0 + (c * LPR + lc) * 4 + r;
                    const float d = ((c * LPR + lc) * 4 < BN && n < N) ? v[c][r] - mean : 0.f;
                    q += d * d;
                }
            q = group_reduce<LPR, false>(q);
            const float rstd = rsqrtf(q / (float)N + p.ln_eps);
#pragma unroll
            for (int c = 0; c < NCH; ++c)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[c][r] = (v[c][r] - mean) * rstd * g4[c][r] + be4[c][r];
        }
        if (!mok) continue;
        const bool masked = p.row_mask && p.row_mask[m];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int nl0 = (c * LPR + lc) * 4;
            const int n = n0 + nl0;
            if (nl0 >= BN || n >= N) continue;
            if (masked) v[c][0] = v[c][1] = v[c][2] = v[c][3] = 0.f;
            TO* dst;
            if (p.hm_rows) {
                const int bb = m / p.hm_rows, ss = m - bb * p.hm_rows;
                if (p.hm_split && n >= p.hm_split) {   // the tail plane (4-column groups never straddle)
                    const int n2 = n - p.hm_split, g = n2 / p.hm_d2, dd = n2 - g * p.hm_d2;
                    dst = C + (long)p.hm_split * p.hm_batch * p.hm_rows +
                          (((long)g * p.hm_batch + bb) * p.hm_rows + ss) * p.hm_d2 + dd;
                } else {
                    const int g = n / p.hm_d, dd = n - g * p.hm_d;
                    dst = C + (((long)g * p.hm_batch + bb) * p.hm_rows + ss) * p.hm_d + dd;
                }
            } else {
                dst = C + (long)m * p.ldc + n;
            }
            if (ld_ok && n + 3 < N) IO4<TO>::store(dst, v[c]);
            else
                for (int r = 0; r < 4; ++r)
                    if (n + r < N) IO4<TO>::store1(dst + r, v[c][r]);
        }
    }
}

template <typename T, typename TO, int BM, int BN, int WGM, int WGN, bool CONV, bool LN>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const GemmArgs p, const int nNt) {
    static_assert(WGM * WGN == 4, "4 waves");
    constexpr int EPC = Mma<T>::EPC;
    constexpr int BK = ROWB / (int)sizeof(T);
    constexpr int XR = BM / 32;                 // 16-byte staging chunks per thread (A)
    constexpr int WR = BN / 32;                 // (B)
    constexpr int WTM = BM / WGM, WTN = BN / WGN;   // wave tile
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int STAGE = Smem<BM, BN>::STAGE;
    constexpr int EPI_LD = Smem<BM, BN>::EPI_LD;
    __shared__ __attribute__((aligned(16))) char lds[Smem<BM, BN>::BYTES];

    int bid = blockIdx.x;
    {
        const int nblk = gridDim.x, q = nblk >> 3, r = nblk & 7, xcd = bid & 7;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    }
    const int mt = bid / nNt, nt = bid - (bid / nNt) * nNt;
    const int m0 = p.m_begin + mt * BM, n0 = nt * BN;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave % WGM, wn = wave / WGM;
    const int sc = tid & 7, sr = tid >> 3;
    const int M = p.M, N = p.N;
    // K range of this block: the whole K, or slice blockIdx.y of a split-K launch
    const int kbeg = p.kchunk ? (int)blockIdx.y * p.kchunk : 0;
    const int K = p.kchunk ? min(p.K, kbeg + p.kchunk) : p.K;

    // Buffer descriptors over the whole operands (kernel arguments -> wave-uniform SGPRs).
    // A lane that must contribute zeros (row/col past the edge, K tail, conv padding)
    // gets an offset past num_records: the hardware range check returns 0, so the
    // staging loads are branch-free and all stay in flight (a `cond ? load : 0` compiles
    // to a branch + vmcnt(0) per load, cdna_hip_programming.md §5 item 4(c)).
    constexpr unsigned OOB = 0x80000000u;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.a_bytes, 0x00020000);
    const int a2_bytes = (p.A2 && p.a2_rows) ? ((p.a2_rows - 1) * p.lda + p.K) * (int)sizeof(T) : p.a_bytes;
    const __amdgpu_buffer_rsrc_t ra2 =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p.A2 ? p.A2 : p.A), (short)0, a2_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.b_bytes, 0x00020000);
    const bool has_a2 = p.A2 != nullptr;

    unsigned xbase[XR], x2sub[XR];   // x2sub: elements back from row m to A2 row m % a2_rows
    int xih[XR], xiw[XR];
    bool xok[XR];
#pragma unroll
    for (int i = 0; i < XR; ++i) {
        const int m = m0 + sr + 32 * i;
        xok[i] = m < M;
        x2sub[i] = (!CONV && p.a2_rows) ? (unsigned)(m - m % p.a2_rows) * (unsigned)p.lda : 0u;
        if (CONV) {
            const int hw = p.Hout * p.Wout;
            const int img = m / hw;
            const int rem = m - img * hw;
            const int oh = rem / p.Wout, ow = rem - (rem / p.Wout) * p.Wout;
            xih[i] = oh * p.stride - p.pad;
            xiw[i] = ow * p.stride_w - p.pad_w;
            // element offset of the receptive field's (0, 0) tap (may lie outside the image:
            // only ever used behind the bounds test)
            xbase[i] = (unsigned)img * (unsigned)(p.Hin * p.Win * p.Cin) +
                       (unsigned)((xih[i] * p.Win + xiw[i]) * p.Cin);
        } else {
            xih[i] = xiw[i] = 0;
            xbase[i] = (unsigned)m * (unsigned)p.lda;
        }
    }
    unsigned wbase[WR];
    bool wok[WR];
#pragma unroll
    for (int i = 0; i < WR; ++i) {
        const int n = n0 + sr + 32 * i;
        wok[i] = n < N;
        wbase[i] = (unsigned)n * (unsigned)p.ldb;
    }

    // two register staging sets: the loads of K-step k+2 are issued while k computes and
    // k+1 (issued one step earlier) is written to LDS -- two steps of load latency covered
    u32x4 xs0[XR], ws0[WR], xs1[XR], ws1[WR];

    // when Cin is a multiple of the K-step, one K-step lies inside one filter tap: the tap
    // (kh, kw) is wave-uniform and computed on the scalar unit, not per lane
    const bool tap_uniform = CONV && (p.Cin % BK) == 0;
    const int nk = (K - kbeg + BK - 1) / BK;
    // K-step order of a multi-tap conv: channel-chunk-major, tap-minor -- the KH*KW shifted
    // reads of one input-channel chunk run in consecutive K-steps (the rows they touch are
    // still in L2) instead of KH*KW passes over all channels; the weight columns follow
    const int ntaps = CONV ? p.K / p.Cin : 1;
    const bool korder = tap_uniform && p.kchunk == 0 && ntaps > 1;
    const int nchunk = p.Cin / BK;
    auto kmap = [&](int kt) -> int {
        if (!korder || kt >= nk) return kt * BK;
        const int c = kt / ntaps, t = kt - c * ntaps;
        return (t * nchunk + c) * BK;
    };
    // Offsets past the edges / padding taps get bit 31 set: past num_records, so the range
    // check returns zeros.  Computed arithmetically (no select): hipcc otherwise branches
    // around the offset math of each load (s_and_saveexec) to skip it for masked lanes.
    auto load_tile = [&](int k0, u32x4 (&xs)[XR], u32x4 (&ws)[WR]) {
        const int k = kbeg + k0 + sc * EPC;
        const unsigned kbad = k < K ? 0u : OOB;
        int kh = 0, kw = 0, dk = 0;
        if (CONV) {
            if (tap_uniform) {
                const int ks0 = __builtin_amdgcn_readfirstlane(kbeg + k0);
                const int tap = ks0 / p.Cin;
                kh = tap / p.KW;
                kw = tap - kh * p.KW;
                dk = __builtin_amdgcn_readfirstlane((kh * p.Win + kw) * p.Cin + ks0 - tap * p.Cin) + sc * EPC;
            } else {
                const int tap = k / p.Cin;
                kh = tap / p.KW;
                kw = tap - kh * p.KW;
                dk = (kh * p.Win + kw) * p.Cin + k - tap * p.Cin;
            }
        }
#pragma unroll
        for (int i = 0; i < XR; ++i) {
            unsigned off, bad = kbad | (xok[i] ? 0u : OOB);
            if (CONV) {
                const bool in = (unsigned)(xih[i] + kh) < (unsigned)p.Hin && (unsigned)(xiw[i] + kw) < (unsigned)p.Win;
                bad |= in ? 0u : OOB;
                off = xbase[i] + (unsigned)dk;
            } else {
                off = xbase[i] + (unsigned)k;
            }
            const unsigned boff = (off * (unsigned)sizeof(T)) | bad;
            xs[i] = __builtin_amdgcn_raw_buffer_load_b128(ra, boff, 0, 0);
            if (!CONV && has_a2)
                xs[i] = Mma<T>::add(xs[i], __builtin_amdgcn_raw_buffer_load_b128(
                                               ra2, ((off - x2sub[i]) * (unsigned)sizeof(T)) | bad, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < WR; ++i) {
            const unsigned boff = ((wbase[i] + (unsigned)k) * (unsigned)sizeof(T)) | kbad | (wok[i] ? 0u : OOB);
            ws[i] = __builtin_amdgcn_raw_buffer_load_b128(rb, boff, 0, 0);
        }
    };
    auto store_tile = [&](int buf, const u32x4 (&xs)[XR], const u32x4 (&ws)[WR]) {
        char* xl = lds + buf * STAGE;
        char* wl = xl + BM * ROWB;
#pragma unroll
        for (int i = 0; i < XR; ++i) *reinterpret_cast<u32x4*>(xl + swz(sr + 32 * i, sc)) = Mma<T>::stage(xs[i]);
#pragma unroll
        for (int i = 0; i < WR; ++i) *reinterpret_cast<u32x4*>(wl + swz(sr + 32 * i, sc)) = Mma<T>::stage(ws[i]);
    };

    f32x4 acc[TN][TM];
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int buf) {
        const char* xl = lds + buf * STAGE;
        const char* wl = xl + BM * ROWB;
        if constexpr (std::is_same<T, f32x3_t>::value) {
            // KINET_F32_X3 on v_mfma_f32_16x16x32_bf16: lane group g takes chunks 2g, 2g+1
            const int c0 = 2 * (lane >> 4);
            u32x4 b0[TM], b1[TM], a0[TN], a1[TN];
#pragma unroll
            for (int t = 0; t < TM; ++t) {
                const int r = wm * WTM + t * 16 + (lane & 15);
                b0[t] = *reinterpret_cast<const u32x4*>(xl + swz(r, c0));
                b1[t] = *reinterpret_cast<const u32x4*>(xl + swz(r, c0 + 1));
            }
#pragma unroll
            for (int t = 0; t < TN; ++t) {
                const int r = wn * WTN + t * 16 + (lane & 15);
                a0[t] = *reinterpret_cast<const u32x4*>(wl + swz(r, c0));
                a1[t] = *reinterpret_cast<const u32x4*>(wl + swz(r, c0 + 1));
            }
#pragma unroll
            for (int a = 0; a < TN; ++a)
#pragma unroll
                for (int b = 0; b < TM; ++b) Mma<f32x3_t>::run32(acc[a][b], a0[a], a1[a], b0[b], b1[b]);
            return;
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = kk * 4 + (lane >> 4);
            typename Mma<T>::Frag bfr[TM], afr[TN];
#pragma unroll
            for (int t = 0; t < TM; ++t)
                bfr[t] = Mma<T>::frag(*reinterpret_cast<const u32x4*>(xl + swz(wm * WTM + t * 16 + (lane & 15), ch)));
#pragma unroll
            for (int t = 0; t < TN; ++t)
                afr[t] = Mma<T>::frag(*reinterpret_cast<const u32x4*>(wl + swz(wn * WTN + t * 16 + (lane & 15), ch)));
#pragma unroll
            for (int a = 0; a < TN; ++a)
#pragma unroll
                for (int b = 0; b < TM; ++b) Mma<T>::run(acc[a][b], afr[a], bfr[b]);
        }
    };
    // step kt: issue K-step kt+2 into the set that held kt (already in LDS), compute kt,
    // write kt+1 (loaded one step ago) into the other LDS buffer, one barrier
    // the loads of K-steps past the end are issued too (range check -> zeros, no traffic):
    // a conditional load makes hipcc's vmcnt count assume the short path and drain the
    // younger prefetch before every LDS write
    auto step = [&](int kt, u32x4 (&xi)[XR], u32x4 (&wi)[WR], const u32x4 (&xn)[XR], const u32x4 (&wn)[WR]) {
        load_tile(kmap(kt + 2), xi, wi);
        compute(kt & 1);
        store_tile((kt + 1) & 1, xn, wn);
        __syncthreads();
        // the next step's loads / fragment reads may reuse registers of this step's last MFMAs
        // (their windows cross the loop back edge)
        mfma_window_pad<4>();
    };
    load_tile(kmap(0), xs0, ws0);
    load_tile(kmap(1), xs1, ws1);
    store_tile(0, xs0, ws0);
    __syncthreads();
    // two K-steps per iteration, both unconditional (an odd last step multiplies zeros)
    for (int kt = 0; kt < nk; kt += 2) {
        step(kt, xs0, ws0, xs1, ws1);
        step(kt + 1, xs1, ws1, xs0, ws0);
    }

    // ---- epilogue: residual rows in flight, park the f32 tile in LDS, stream whole rows ----
    ResRows<TO, BN, 4, BM> rp;
    rp.issue(p, m0, n0, 0, wave, lane);
    float* ep = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) {
            const int ml = wm * WTM + b * 16 + (lane & 15);
            const int nl = wn * WTN + a * 16 + (lane >> 4) * 4;
            *reinterpret_cast<f32x4*>(ep + ml * EPI_LD + nl) = acc[a][b];
        }
    __syncthreads();
    epilogue_rows<TO, BN, EPI_LD, 4, LN, BM>(p, ep, m0, n0, 0, wave, lane, rp);
}

#include "gemm_dma.h"   // gemm_dma_kernel: the same tiles staged by LDS-DMA through a 3-slot ring
template <typename T, typename TO, bool CONV>
int launch(const GemmArgs& a, hipStream_t stream) {
    if (a.M == 0 || a.N == 0) return KINET_OK;
    const bool ln = a.ln_g != nullptr;
    int bm, bn;
    if (ln) {
        KINET_CHECK_ARG(a.N <= 320, "gemm: fused LayerNorm needs N <= 320 (got %d)", a.N);
        bm = a.M <= 8192 ? 32 : 64;     // small M (decoder queries): more workgroups
        bn = a.N <= 256 ? 256 : 320;
        // rows of 257..320 (d = 288, configs 3-5) at encoder sizes: 128 x 320 LDS-DMA tiles --
        // the 64 x 320 register-staged tile re-reads the whole 320 x K weight through its
        // staging registers for every 64 rows (~100 TF/s at M = 172k)
        if (sizeof(T) == 2 && a.N > 256 && a.M >= 8192 && a.A2 == nullptr && a.kchunk == 0) bm = 128;
    } else if (a.kchunk && a.M <= 4096) {
        bm = bn = 64;                   // split-K slices of a small-M, long-K problem
    } else if (a.M <= 4096 && a.N <= 1024) {
        bm = 32;                        // decoder-sized GEMMs: more workgroups
        bn = 64;
    } else {
        // 64x128 (128x64 for N <= 64): fastest main-loop tile on every 3x3 / K >= 512 conv and
        // GEMM shape of the detector at batch 8 (tools/sweep_conv.py) -- more tiles per CU-round
        // than 128x128 and no worse per flop
        bn = a.N <= 64 ? 64 : 128;
        bm = a.N <= 64 ? 128 : 64;
        // big square-ish problems: the 128x128 tile's lower operand traffic per flop wins
        const long t128 = (long)((a.M + 127) / 128) * ((a.N + 127) / 128);
        if (a.N >= 512 && t128 >= 2048) bm = bn = 128;
        // 3x3 convs (K >= 9*128) with >= ~2 rounds of 128x128 tiles over the 512 resident
        // slots: 3-6 % faster than 64x128 at batch 16 (tools/sweep_conv.py 16), neutral at 8
        if (CONV && a.K >= 1152 && a.N >= 128 && t128 >= 1000) bm = bn = 128;
        // KINET_F32_X3 with N just past a multiple of 128 (d = 288 of the config-4 training
        // GEMMs): 128 x 64 tiles waste 10 % of the columns instead of 25 % -- x3 (44446, 288,
        // 1024) 157 -> 132 us, (44446, 288, 288) 60 -> 51 us (profiles/r05x_x3_tiles.log);
        // flag 33554432 keeps the default (A/B)
        if (std::is_same<T, f32x3_t>::value && a.N > 64 && a.N % 128 != 0 && a.N % 128 <= 64 &&
            !(kinet_gemm_flags & 33554432)) {
            bm = 128;
            bn = 64;
        }
    }
    // 8-wave LDS-DMA tiles (one workgroup per CU: 256 slots per round): chosen for long-K
    // problems whose rounds of tiles are well filled (a square 4096^3 bf16 GEMM: 1115 TF/s
    // on 256x256 vs 456 on the 4-wave 128x128 tile, tools/gemm_probe.py); on the detector's
    // conv / GEMM shapes their last, partly filled round costs more than the faster main loop
    // gains (DESIGN.md "GEMM / conv kernel"), so those keep the 4-wave tiles.  Flag 2 forces
    // them wherever eligible.
    int bm8 = 0, bn8 = 0;
    // (not for head-major stores: only gemm_kernel's epilogue writes them)
    if (sizeof(T) == 2 && a.A2 == nullptr && a.kchunk == 0 && a.hm_rows == 0 && a.M >= 4096 && a.N >= 128 &&
        (!ln || a.N <= 256)) {
        const int tn = (a.N > 128 || ln) ? 256 : 128;
        const long t = (long)((a.M + 255) / 256) * ((a.N + tn - 1) / tn);
        const double eff = (double)a.M * a.N / ((double)((t + 255) / 256) * 256.0 * 256.0 * tn);
        if ((kinet_gemm_flags & 2) || (!ln && a.K >= 1024 && eff >= 0.9)) {
            bm8 = 256;
            bn8 = tn;
        }
    }
    if (bm8) {
        bm = bm8;
        bn = bn8;
    }
    if (force_bm && !ln) {
        bm = force_bm;
        bn = force_bn;
    }
    // LDS-DMA staging (opt-in, flag 16): measured 0-10 % slower than the register-staged
    // kernel on the detector's conv / GEMM shapes at batch 8 (tools/sweep_conv.py), so the
    // register path stays the default; A2 (load-time add) needs the register path anyway
    // (not for KINET_F32_X3: its operands are split into bf16 hi / lo on the way into LDS)
    const bool dma = a.A2 == nullptr && (kinet_gemm_flags & 16) && !std::is_same<T, f32x3_t>::value;
    const int nslice = a.kchunk ? (a.K + a.kchunk - 1) / a.kchunk : 1;
    // one launch of the tile grid over rows [g.m_begin, g.m_begin + mtiles * BM)
    auto run = [&](const GemmArgs& g, int tbm, int tbn, long mtiles) -> int {
        const int nNt = (g.N + tbn - 1) / tbn;
        const long nblk = mtiles * nNt;
        KINET_CHECK_ARG(nblk < (1L << 31), "gemm: too many tiles");
        dim3 grid((unsigned)nblk, (unsigned)nslice), block(256);
        // 8-wave LDS-DMA tiles (16-bit operands, no load-time A2 add; LayerNorm on 256-wide rows)
        if constexpr (sizeof(T) == 2) {
            if (ln && tbm == 128 && tbn == 320) {
                hipLaunchKernelGGL((gemm_dma_kernel<T, TO, 128, 320, 2, 2, CONV, true, 2>), grid, block, 0, stream, g, nNt);
                KINET_LAUNCH_CHECK();
                return KINET_OK;
            }
            if (g.A2 == nullptr && (tbm == 256 || tbn == 256)) {
                const dim3 blk(512);
                if (ln)
                    hipLaunchKernelGGL((gemm_dma_kernel<T, TO, 256, 256, 2, 4, CONV, true, 2>), grid, blk, 0, stream, g, nNt);
                else if (tbm == 256 && tbn == 256)
                    hipLaunchKernelGGL((gemm_dma_kernel<T, TO, 256, 256, 2, 4, CONV, false, 2>), grid, blk, 0, stream, g, nNt);
                else if (tbm == 256)
                    hipLaunchKernelGGL((gemm_dma_kernel<T, TO, 256, 128, 4, 2, CONV, false>), grid, blk, 0, stream, g, nNt);
                else
                    hipLaunchKernelGGL((gemm_dma_kernel<T, TO, 128, 256, 2, 4, CONV, false>), grid, blk, 0, stream, g, nNt);
                KINET_LAUNCH_CHECK();
                return KINET_OK;
            }
        }
#define L_(BM_, BN_, WM_, WN_, LN_)                                                                             \
    do {                                                                                                        \
        if constexpr (!std::is_same<T, f32x3_t>::value) {                                                     \
            if (dma) { hipLaunchKernelGGL((gemm_dma_kernel<T, TO, BM_, BN_, WM_, WN_, CONV, LN_>), grid, block, 0, \
                                          stream, g, nNt); break; }                                             \
        }                                                                                                       \
        hipLaunchKernelGGL((gemm_kernel<T, TO, BM_, BN_, WM_, WN_, CONV, LN_>), grid, block, 0, stream, g, \
                                nNt);                                                                           \
    } while (0)
        if (ln) {
            if (tbm == 32 && tbn == 256) L_(32, 256, 1, 4, true);
            else if (tbm == 32) L_(32, 320, 1, 4, true);
            else if (tbn == 256) L_(64, 256, 1, 4, true);
            else L_(64, 320, 1, 4, true);
        } else if (tbm == 32) L_(32, 64, 2, 2, false);
        else if (tbm == 128 && tbn == 128) L_(128, 128, 2, 2, false);
        else if (tbm == 128 && tbn == 64) L_(128, 64, 2, 2, false);
        else if (tbm == 64 && tbn == 128) L_(64, 128, 2, 2, false);
        else L_(64, 64, 2, 2, false);
#undef L_
        KINET_LAUNCH_CHECK();
        return KINET_OK;
    };
    // Multi-tap convolutions (3x3, 7x1): whole rounds of one-per-CU 8-wave 256-row tiles (the
    // faster main loop: half the LDS reads per MFMA and half the L2 bytes per flop of the
    // 4-wave tiles), then the rows left over -- less than a round -- on the 4-wave tiles in a
    // second launch, instead of a partly filled last round of 8-wave tiles (flag 64: off)
    if constexpr (sizeof(T) == 2) {
        if (CONV && !ln && a.A2 == nullptr && a.kchunk == 0 && !force_bm && !bm8 && !(kinet_gemm_flags & 64) &&
            a.K > a.Cin && a.N >= 256 && a.M >= 8192) {
            // (256x256 tiles only: at N = 128 the 8-wave 256x128 tile measured no faster per
            // round than the 4-wave 128x128 one, tools/gemm_probe.py)
            const int tn = 256;
            const int nN8 = (a.N + tn - 1) / tn;
            const long mt_all = (a.M + 255) / 256;
            long mfull = (mt_all * nN8 / 256) * 256 / nN8;   // m-tiles that fill whole rounds
            if (mfull > mt_all) mfull = mt_all;
            // less than one round but at least half of one: a single partial round of 8-wave
            // tiles still beats the 4-wave grid (layer-4 3x3 at batch 16: 119 vs 128 us)
            if (mfull == 0 && mt_all * nN8 >= 128) {
                // ... unless one batch is in flight (kinet_set_solo_launch), it fills less than 60 %
                // of the CUs and 128 x 256 tiles (twice as many, same 8-wave main loop, same sums)
                // fill them better: config 5's stage-3 3x3 convs (M = 32,640, N = 256: 128 vs 255
                // tiles) 74.8 -> 48.5 us alone (profiles/r06aa_config5_shapes.txt), but -1 % on 3
                // streams, whose other batches fill the idle CUs (profiles/r06ab_solo_launch_ab.txt)
                const long t128 = (long)((a.M + 127) / 128) * nN8;
                if (kinet_solo_launch && mt_all * nN8 * 10 < 256L * 6 && t128 <= 256)
                    return run(a, 128, 256, (a.M + 127) / 128);
                mfull = mt_all;
            }
            // a remainder of more than a quarter round: the partly filled last round of 8-wave
            // tiles beats the 4-wave tail (layer-3 3x3 at batch 24: 394 m-tiles = 256 + 138,
            // 140 vs 151 us, profiles/r05f2_conv24.log); flag 8388608 keeps the split (A/B)
            if (mfull >= 1 && (mt_all - mfull) * nN8 > 64 && !(kinet_gemm_flags & 8388608)) mfull = mt_all;
            if (mfull >= 1) {
                int rc = run(a, 256, tn, mfull);
                if (rc) return rc;
                const long rem = a.M - mfull * 256;
                if (rem <= 0) return KINET_OK;
                GemmArgs g = a;
                g.m_begin = (int)(mfull * 256);
                return run(g, 64, 128, (rem + 63) / 64);   // less than a round: the smaller tile
            }
        }
    }
    return run(a, bm, bn, (a.M + bm - 1) / bm);
}

template <bool CONV>
int dispatch(const GemmArgs& a, int in_dtype, int out_dtype, hipStream_t s) {
    if (!CONV && a.kchunk == 0 && !(kinet_gemm_flags & 4) && launch_rw(a, in_dtype, out_dtype, s)) {
        KINET_LAUNCH_CHECK();
        return KINET_OK;
    }
    if (CONV && !(kinet_gemm_flags & 1024) && out_dtype == in_dtype && launch_conv3x3_c64(a, in_dtype, s)) {
        KINET_LAUNCH_CHECK();
        return KINET_OK;
    }
    if (CONV && !(kinet_gemm_flags & 32) && out_dtype == in_dtype && launch_stem_conv(a, in_dtype, s)) {
        KINET_LAUNCH_CHECK();
        return KINET_OK;
    }
    if (CONV && a.kchunk == 0 && !(kinet_gemm_flags & 4) && out_dtype == in_dtype && launch_rw_conv(a, in_dtype, s)) {
        KINET_LAUNCH_CHECK();
        return KINET_OK;
    }
    if (in_dtype == KINET_BF16 && out_dtype == KINET_BF16) return launch<bf16_t, bf16_t, CONV>(a, s);
    if (in_dtype == KINET_BF16 && out_dtype == KINET_F32) return launch<bf16_t, float, CONV>(a, s);
    if (!CONV && in_dtype == KINET_BF16 && out_dtype == KINET_F16) return launch<bf16_t, f16_t, false>(a, s);
    if (in_dtype == KINET_F16 && out_dtype == KINET_F16) return launch<f16_t, f16_t, CONV>(a, s);
    if (in_dtype == KINET_F16 && out_dtype == KINET_F32) return launch<f16_t, float, CONV>(a, s);
    if (in_dtype == KINET_F32 && out_dtype == KINET_F32) return launch<float, float, CONV>(a, s);
    if (in_dtype == KINET_F32_X3 && (out_dtype == KINET_F32 || out_dtype == KINET_F32_X3))
        return launch<f32x3_t, float, CONV>(a, s);
    set_error("gemm: unsupported dtypes in=%d out=%d", in_dtype, out_dtype);
    return KINET_ERR_ARG;
}

// split-K finalize: out[m, n] = epilogue(sum over slices of ws[s][m][n]) -- one wave per row,
// column n = j*64 + lane (coalesced); the same epilogue as the GEMM kernels (scale/bias,
// residual, ReLU, LayerNorm over the row, row mask).
template <typename TO, bool LN>
__global__ __launch_bounds__(256) void splitk_finalize_kernel(const GemmArgs p, const float* __restrict__ ws,
                                                              int nslice, long slice) {
    constexpr int MAXJ = 16;   // LN rows up to 1024 columns
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= p.M) return;
    const int N = p.N;
    const int nj = (N + 63) / 64;
    const TO* __restrict__ R = (const TO*)p.R;
    TO* __restrict__ C = (TO*)p.C;
    float v[MAXJ];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
        v[j] = 0.f;
        if (j >= nj) continue;
        const int n = j * 64 + lane;
        if (n >= N) continue;
        float x = 0.f;
        for (int t = 0; t < nslice; ++t) x += ws[t * slice + (long)row * N + n];
        x = x * (p.scale ? p.scale[n] : 1.f) + (p.bias ? p.bias[n] : 0.f);
        if (R) x += IO4<TO>::load1(R + (long)row * p.ldr + n);
        if (p.relu) x = fmaxf(x, 0.f);
        v[j] = x;
        s += x;
    }
    if (LN) {
        s = group_reduce<64, false>(s);
        const float mean = s / (float)N;
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < MAXJ; ++j)
            if (j < nj && j * 64 + lane < N) q += (v[j] - mean) * (v[j] - mean);
        q = group_reduce<64, false>(q);
        const float rstd = rsqrtf(q / (float)N + p.ln_eps);
#pragma unroll
        for (int j = 0; j < MAXJ; ++j) {
            const int n = j * 64 + lane;
            if (j < nj && n < N) v[j] = (v[j] - mean) * rstd * p.ln_g[n] + p.ln_b[n];
        }
    }
    const bool masked = p.row_mask && p.row_mask[row];
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
        const int n = j * 64 + lane;
        if (j < nj && n < N) IO4<TO>::store1(C + (long)row * p.ldc + n, masked ? 0.f : v[j]);
    }
    // columns past 16*64 (non-LN rows wider than 1024)
    for (int n = MAXJ * 64 + lane; n < N; n += 64) {
        float x = 0.f;
        for (int t = 0; t < nslice; ++t) x += ws[t * slice + (long)row * N + n];
        x = x * (p.scale ? p.scale[n] : 1.f) + (p.bias ? p.bias[n] : 0.f);
        if (R) x += IO4<TO>::load1(R + (long)row * p.ldr + n);
        if (p.relu) x = fmaxf(x, 0.f);
        IO4<TO>::store1(C + (long)row * p.ldc + n, masked ? 0.f : x);
    }
}

// Run a GEMM / implicit conv as split-K: partial f32 tiles into ws (nslice x M x N), then the
// finalize pass applies the caller's epilogue into C.  kchunk is rounded to whole K-steps.
template <bool CONV>
int run_splitk(const GemmArgs& user, int in_dtype, int out_dtype, float* ws, int ksplit, hipStream_t s) {
    KINET_CHECK_ARG(ksplit >= 1 && ws != nullptr, "split-K: need ksplit >= 1 and a workspace");
    KINET_CHECK_ARG(user.ln_g == nullptr || user.N <= 1024, "split-K: LayerNorm rows up to 1024 columns");
    const int step = dtype_size(in_dtype) == 4 ? 32 : 64;
    int kchunk = (user.K + ksplit - 1) / ksplit;
    kchunk = (kchunk + step - 1) / step * step;
    const int nslice = (user.K + kchunk - 1) / kchunk;
    GemmArgs a = user;
    a.C = ws;
    a.ldc = user.N;
    a.R = nullptr;
    a.scale = nullptr;
    a.bias = nullptr;
    a.ln_g = a.ln_b = nullptr;
    a.row_mask = nullptr;
    a.relu = 0;
    a.hm_rows = 0;
    a.kchunk = kchunk;
    a.c_slice = (long)user.M * user.N;
    int rc = dispatch<CONV>(a, in_dtype, KINET_F32, s);
    if (rc) return rc;
    dim3 grid((user.M + 3) / 4), block(256);
#define F_(TO_)                                                                                                 \
    if (user.ln_g) hipLaunchKernelGGL((splitk_finalize_kernel<TO_, true>), grid, block, 0, s, user, ws, nslice, a.c_slice); \
    else hipLaunchKernelGGL((splitk_finalize_kernel<TO_, false>), grid, block, 0, s, user, ws, nslice, a.c_slice)
    if (out_dtype == KINET_BF16) { F_(bf16_t); }
    else if (out_dtype == KINET_F16) { F_(f16_t); }
    else { F_(float); }
#undef F_
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

bool aligned16(const void* p) { return (((uintptr_t)p) & 15u) == 0; }

}  // namespace
}  // namespace kinet

using namespace kinet;

extern "C" int kinet_gemm_headmajor(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                                    int in_dtype, int out_dtype, const float* bias, const uint8_t* row_mask,
                                    int rows_per_batch, int head_dim, kinet_stream_t stream);
extern "C" int kinet_gemm_headmajor_ex(const void* A, const void* A2, const void* B, void* C, int M, int N, int K,
                                       int lda, int ldb, int in_dtype, int out_dtype, const float* bias,
                                       const uint8_t* row_mask, int rows_per_batch, int head_dim, int a2_rows,
                                       kinet_stream_t stream);

extern "C" int kinet_gemm_ex(const void* A, const void* A2, const void* B, void* C, int M, int N, int K, int lda,
                             int ldb, int ldc, int in_dtype, const float* scale, const float* bias, const void* R,
                             int ldr, int relu, const float* ln_gamma, const float* ln_beta, float ln_eps,
                             int out_dtype, const uint8_t* row_mask, kinet_stream_t stream) {
    KINET_CHECK_ARG(M >= 0 && N >= 0 && K > 0, "gemm: invalid sizes M=%d N=%d K=%d", M, N, K);
    KINET_CHECK_ARG(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0, "gemm: K, lda, ldb must be multiples of 8 (K=%d lda=%d ldb=%d)", K, lda, ldb);
    KINET_CHECK_ARG(lda >= K && ldb >= K && ldc >= N, "gemm: leading dims too small");
    KINET_CHECK_ARG(aligned16(A) && aligned16(B) && (A2 == nullptr || aligned16(A2)), "gemm: A, A2 and B must be 16-byte aligned");
    KINET_CHECK_ARG(R == nullptr || ldr >= N, "gemm: ldr < N");
    KINET_CHECK_ARG((ln_gamma == nullptr) == (ln_beta == nullptr), "gemm: LayerNorm needs both gamma and beta");
    KINET_CHECK_ARG(ln_gamma == nullptr || relu == 0, "gemm: LayerNorm and ReLU are exclusive");
    GemmArgs a{};
    a.A = A; a.A2 = A2; a.B = B; a.C = C; a.R = R; a.scale = scale; a.bias = bias; a.row_mask = row_mask;
    a.ln_g = ln_gamma; a.ln_b = ln_beta; a.ln_eps = ln_eps;
    a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.ldr = ldr; a.relu = relu;
    const long long es = (long long)dtype_size(in_dtype);
    const long long ab = M > 0 ? ((long long)(M - 1) * lda + K) * es : 0;
    const long long bb = N > 0 ? ((long long)(N - 1) * ldb + K) * es : 0;
    KINET_CHECK_ARG(ab < (1LL << 31) && bb < (1LL << 31), "gemm: operand larger than 2 GiB (split the call)");
    a.a_bytes = (int)ab;
    a.b_bytes = (int)bb;
    if (R != nullptr) {
        const long long rb = ((long long)(M > 0 ? M - 1 : 0) * ldr + N) * (long long)dtype_size(out_dtype);
        KINET_CHECK_ARG(rb < (1LL << 31), "gemm: residual larger than 2 GiB (split the call)");
        a.r_bytes = (int)rb;
    }
    return dispatch<false>(a, in_dtype, out_dtype, (hipStream_t)stream);
}

extern "C" int kinet_gemm_headmajor(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                                    int in_dtype, int out_dtype, const float* bias, const uint8_t* row_mask,
                                    int rows_per_batch, int head_dim, kinet_stream_t stream) {
    return kinet_gemm_headmajor_ex(A, nullptr, B, C, M, N, K, lda, ldb, in_dtype, out_dtype, bias, row_mask,
                                   rows_per_batch, head_dim, 0, stream);
}

extern "C" int kinet_gemm_headmajor_ex(const void* A, const void* A2, const void* B, void* C, int M, int N, int K,
                                       int lda, int ldb, int in_dtype, int out_dtype, const float* bias,
                                       const uint8_t* row_mask, int rows_per_batch, int head_dim, int a2_rows,
                                       kinet_stream_t stream) {
    KINET_CHECK_ARG(a2_rows == 0 || (A2 != nullptr && a2_rows >= 32 && M % a2_rows == 0),
                    "gemm_headmajor: a2_rows must be 0 or >= 32 dividing M (got %d)", a2_rows);
    KINET_CHECK_ARG(out_dtype == in_dtype || (in_dtype == KINET_BF16 && out_dtype == KINET_F16),
                    "gemm_headmajor: out_dtype must equal in_dtype (or f16 from bf16)");
    KINET_CHECK_ARG(M >= 0 && N > 0 && K > 0, "gemm_headmajor: invalid sizes");
    KINET_CHECK_ARG(rows_per_batch > 0 && M % rows_per_batch == 0, "gemm_headmajor: M must be batch*rows_per_batch");
    KINET_CHECK_ARG(head_dim > 0 && head_dim % 4 == 0 && N % head_dim == 0, "gemm_headmajor: N must be a multiple of head_dim (%% 4)");
    KINET_CHECK_ARG(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && lda >= K && ldb >= K, "gemm_headmajor: bad K/lda/ldb");
    KINET_CHECK_ARG(aligned16(A) && aligned16(B) && (A2 == nullptr || aligned16(A2)),
                    "gemm_headmajor: A, A2 and B must be 16-byte aligned");
    GemmArgs a{};
    a.A = A; a.A2 = A2; a.B = B; a.C = C; a.bias = bias; a.row_mask = row_mask; a.a2_rows = a2_rows;
    a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = N;
    a.hm_rows = rows_per_batch; a.hm_d = head_dim; a.hm_batch = M / rows_per_batch;
    const long long es = (long long)dtype_size(in_dtype);
    const long long ab = M > 0 ? ((long long)(M - 1) * lda + K) * es : 0;
    const long long bb = ((long long)(N - 1) * ldb + K) * es;
    KINET_CHECK_ARG(ab < (1LL << 31) && bb < (1LL << 31), "gemm_headmajor: operand larger than 2 GiB");
    a.a_bytes = (int)ab;
    a.b_bytes = (int)bb;
    return dispatch<false>(a, in_dtype, out_dtype, (hipStream_t)stream);
}

extern "C" int kinet_gemm_headmajor_split(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                                          int in_dtype, int out_dtype, const float* bias, const uint8_t* row_mask,
                                          int rows_per_batch, int head_dim, int split_cols, int tail_dim,
                                          kinet_stream_t stream) {
    KINET_CHECK_ARG(out_dtype == in_dtype || (in_dtype == KINET_BF16 && out_dtype == KINET_F16),
                    "gemm_headmajor_split: out_dtype must equal in_dtype (or f16 from bf16)");
    KINET_CHECK_ARG(M >= 0 && N > 0 && K > 0, "gemm_headmajor_split: invalid sizes");
    KINET_CHECK_ARG(rows_per_batch > 0 && M % rows_per_batch == 0, "gemm_headmajor_split: M must be batch*rows_per_batch");
    KINET_CHECK_ARG(head_dim > 0 && head_dim % 4 == 0 && tail_dim > 0 && tail_dim % 4 == 0 && split_cols > 0 &&
                        split_cols % head_dim == 0 && split_cols < N && (N - split_cols) % tail_dim == 0 &&
                        split_cols / head_dim == (N - split_cols) / tail_dim,
                    "gemm_headmajor_split: N = heads*head_dim + heads*tail_dim, dims multiples of 4");
    KINET_CHECK_ARG(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && lda >= K && ldb >= K, "gemm_headmajor_split: bad K/lda/ldb");
    KINET_CHECK_ARG(aligned16(A) && aligned16(B), "gemm_headmajor_split: A and B must be 16-byte aligned");
    GemmArgs a{};
    a.A = A; a.B = B; a.C = C; a.bias = bias; a.row_mask = row_mask;
    a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = N;
    a.hm_rows = rows_per_batch; a.hm_d = head_dim; a.hm_batch = M / rows_per_batch;
    a.hm_split = split_cols; a.hm_d2 = tail_dim;
    const long long es = (long long)dtype_size(in_dtype);
    const long long ab = M > 0 ? ((long long)(M - 1) * lda + K) * es : 0;
    const long long bb = ((long long)(N - 1) * ldb + K) * es;
    KINET_CHECK_ARG(ab < (1LL << 31) && bb < (1LL << 31), "gemm_headmajor_split: operand larger than 2 GiB");
    a.a_bytes = (int)ab;
    a.b_bytes = (int)bb;
    if (M == 0) return KINET_OK;
    return dispatch<false>(a, in_dtype, out_dtype, (hipStream_t)stream);
}

extern "C" int kinet_gemm_splitk(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                                 int in_dtype, const float* scale, const float* bias, const void* R, int ldr, int relu,
                                 const float* ln_gamma, const float* ln_beta, float ln_eps, int out_dtype,
                                 const uint8_t* row_mask, float* workspace, int ksplit, kinet_stream_t stream) {
    KINET_CHECK_ARG(M >= 0 && N >= 0 && K > 0, "gemm_splitk: invalid sizes M=%d N=%d K=%d", M, N, K);
    KINET_CHECK_ARG(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0, "gemm_splitk: K, lda, ldb must be multiples of 8");
    KINET_CHECK_ARG(lda >= K && ldb >= K && ldc >= N, "gemm_splitk: leading dims too small");
    KINET_CHECK_ARG(aligned16(A) && aligned16(B), "gemm_splitk: A and B must be 16-byte aligned");
    KINET_CHECK_ARG(R == nullptr || ldr >= N, "gemm_splitk: ldr < N");
    KINET_CHECK_ARG((ln_gamma == nullptr) == (ln_beta == nullptr), "gemm_splitk: LayerNorm needs both gamma and beta");
    KINET_CHECK_ARG(ln_gamma == nullptr || relu == 0, "gemm_splitk: LayerNorm and ReLU are exclusive");
    if (M == 0 || N == 0) return KINET_OK;
    GemmArgs a{};
    a.A = A; a.B = B; a.C = C; a.R = R; a.scale = scale; a.bias = bias; a.row_mask = row_mask;
    a.ln_g = ln_gamma; a.ln_b = ln_beta; a.ln_eps = ln_eps;
    a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.ldr = ldr; a.relu = relu;
    const long long es = (long long)dtype_size(in_dtype);
    const long long ab = ((long long)(M - 1) * lda + K) * es;
    const long long bb = ((long long)(N - 1) * ldb + K) * es;
    KINET_CHECK_ARG(ab < (1LL << 31) && bb < (1LL << 31), "gemm_splitk: operand larger than 2 GiB");
    a.a_bytes = (int)ab;
    a.b_bytes = (int)bb;
    return run_splitk<false>(a, in_dtype, out_dtype, workspace, ksplit, (hipStream_t)stream);
}

extern "C" int kinet_gemm_force_tile(int bm, int bn) {
    KINET_CHECK_ARG((bm == 0 && bn == 0) || ((bm == 32 && bn == 64) || ((bm == 64 || bm == 128) && (bn == 64 || bn == 128))) ||
                        (bm == 256 && bn == 128) || (bm == 128 && bn == 256) || (bm == 256 && bn == 256),
                    "gemm_force_tile: unsupported tile %dx%d", bm, bn);
    force_bm = bm;
    force_bn = bn;
    return KINET_OK;
}

extern "C" int kinet_set_solo_launch(int on) {
    const int old = kinet_solo_launch;
    kinet_solo_launch = on ? 1 : 0;
    return old;
}

extern "C" int kinet_gemm_set_flags(int flags) {
    const int old = kinet_gemm_flags;
    kinet_gemm_flags = flags;
    kinet::rw_min_m = (flags & 8) ? 256 : 4096;
    return old;
}

extern "C" int kinet_gemm(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                          int in_dtype, const float* scale, const float* bias, const void* R, int ldr, int relu,
                          int out_dtype, const uint8_t* row_mask, int reserved, kinet_stream_t stream) {
    (void)reserved;
    return kinet_gemm_ex(A, nullptr, B, C, M, N, K, lda, ldb, ldc, in_dtype, scale, bias, R, ldr, relu, nullptr,
                         nullptr, 0.f, out_dtype, row_mask, stream);
}

static int conv_args(GemmArgs& a, const void* X, const void* Wt, void* Y, int batch, int Hin, int Win, int Cin,
                     int Hout, int Wout, int Cout, int KH, int KW, int stride, int pad, int stride_w, int pad_w, int in_dtype,
                     const float* scale, const float* bias, const void* R, int ldr, int relu, int ldy) {
    KINET_CHECK_ARG(batch >= 0 && Hin > 0 && Win > 0 && Cin > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0 && stride_w > 0 && pad_w >= 0,
                    "conv2d: invalid geometry");
    KINET_CHECK_ARG(Cin % 8 == 0, "conv2d: Cin (%d) must be a multiple of 8 (pad channels)", Cin);
    KINET_CHECK_ARG(Hout == (Hin + 2 * pad - KH) / stride + 1 && Wout == (Win + 2 * pad_w - KW) / stride_w + 1,
                    "conv2d: output size mismatch");
    KINET_CHECK_ARG(ldy >= Cout && (R == nullptr || ldr >= Cout), "conv2d: ldy/ldr < Cout");
    KINET_CHECK_ARG(aligned16(X) && aligned16(Wt), "conv2d: X and W must be 16-byte aligned");
    const long M = (long)batch * Hout * Wout;
    KINET_CHECK_ARG(M < (1L << 31) && (long)batch * Hin * Win * Cin < (1L << 40), "conv2d: too large");
    a.A = X; a.B = Wt; a.C = Y; a.R = R; a.scale = scale; a.bias = bias; a.row_mask = nullptr;
    a.M = (int)M; a.N = Cout; a.K = KH * KW * Cin; a.lda = 0; a.ldb = KH * KW * Cin; a.ldc = ldy; a.ldr = ldr;
    a.relu = relu;
    a.Hin = Hin; a.Win = Win; a.Cin = Cin; a.Hout = Hout; a.Wout = Wout; a.KW = KW; a.stride = stride; a.pad = pad;
    a.stride_w = stride_w; a.pad_w = pad_w;
    const long long es = (long long)dtype_size(in_dtype);
    const long long ab = (long long)batch * Hin * Win * Cin * es;
    const long long bb = (long long)Cout * KH * KW * Cin * es;
    KINET_CHECK_ARG(ab < (1LL << 31) && bb < (1LL << 31), "conv2d: operand larger than 2 GiB (split the batch)");
    a.a_bytes = (int)ab;
    a.b_bytes = (int)bb;
    if (R != nullptr) {
        const long long rb = ((long long)(M > 0 ? M - 1 : 0) * ldr + Cout) * es;
        KINET_CHECK_ARG(rb < (1LL << 31), "conv2d: residual larger than 2 GiB (split the batch)");
        a.r_bytes = (int)rb;
    }
    if (KH == 1 && KW == 1 && stride == 1 && pad == 0 && stride_w == 1 && pad_w == 0) a.lda = Cin;   // plain GEMM over NHWC rows
    return KINET_OK;
}

extern "C" int kinet_conv2d_ex(const void* X, const void* Wt, void* Y, int batch, int Hin, int Win, int Cin,
                               int Hout, int Wout, int Cout, int KH, int KW, int stride_h, int stride_w, int pad_h,
                               int pad_w, int in_dtype, const float* scale, const float* bias, const void* R, int ldr,
                               int relu, int ldy, kinet_stream_t stream) {
    GemmArgs a{};
    int rc = conv_args(a, X, Wt, Y, batch, Hin, Win, Cin, Hout, Wout, Cout, KH, KW, stride_h, pad_h, stride_w, pad_w,
                       in_dtype, scale, bias, R, ldr, relu, ldy);
    if (rc) return rc;
    // a 1x1 stride-1 convolution over NHWC rows is the plain GEMM Y = X W^T (lda = Cin)
    if (a.lda) return dispatch<false>(a, in_dtype, in_dtype, (hipStream_t)stream);
    return dispatch<true>(a, in_dtype, in_dtype, (hipStream_t)stream);
}

extern "C" int kinet_conv2d(const void* X, const void* Wt, void* Y, int batch, int Hin, int Win, int Cin, int Hout,
                            int Wout, int Cout, int KH, int KW, int stride, int pad, int in_dtype, const float* scale,
                            const float* bias, const void* R, int ldr, int relu, int ldy, kinet_stream_t stream) {
    return kinet_conv2d_ex(X, Wt, Y, batch, Hin, Win, Cin, Hout, Wout, Cout, KH, KW, stride, stride, pad, pad, in_dtype,
                           scale, bias, R, ldr, relu, ldy, stream);
}

extern "C" int kinet_conv2d_splitk(const void* X, const void* Wt, void* Y, int batch, int Hin, int Win, int Cin,
                                   int Hout, int Wout, int Cout, int KH, int KW, int stride, int pad, int in_dtype,
                                   const float* scale, const float* bias, const void* R, int ldr, int relu, int ldy,
                                   float* workspace, int ksplit, kinet_stream_t stream) {
    GemmArgs a{};
    int rc = conv_args(a, X, Wt, Y, batch, Hin, Win, Cin, Hout, Wout, Cout, KH, KW, stride, pad, stride, pad, in_dtype,
                       scale, bias, R, ldr, relu, ldy);
    if (rc) return rc;
    if (a.M == 0) return KINET_OK;
    if (a.lda) return run_splitk<false>(a, in_dtype, in_dtype, workspace, ksplit, (hipStream_t)stream);
    return run_splitk<true>(a, in_dtype, in_dtype, workspace, ksplit, (hipStream_t)stream);
}
