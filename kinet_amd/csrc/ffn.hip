// Fused post-norm FFN sub-layer for gfx950: y = LN(x + W2 relu(W1 x + b1) + b2), one launch.
//
// Reference: DeformableTransformerEncoderLayer.forward_ffn (deformable_transformer.py:284-288)
// and the decoder twin (:361-365) -- two GEMMs whose (M, F) hidden tensor (F = 1024, i.e. 4x
// the activations) is written to and re-read from HBM.  Here it never leaves the CU:
//
//  * each wave owns 16*RT rows of x, held for the whole launch in VGPRs as MFMA B-operand
//    fragments (lane l: row l&15, 8 consecutive k);
//  * the weights stream through a 2-slot LDS ring, one 32-unit hidden chunk per slot
//    (W1 rows + W2 columns, pre-packed fragment-major by kinet_ffn_pack so one LDS-DMA
//    wave-instruction moves one 1-KiB operand fragment and every ds_read_b128 is a linear,
//    conflict-free 1 KiB); all waves of the workgroup share the ring;
//  * phase A: H^T(32 x rows) = W1c x^T on v_mfma_f32_16x16x32 -- the accumulator layout
//    puts 4 consecutive hidden units of one row in each lane;  + b1, ReLU, round to the
//    16-bit type: that IS the B operand of phase B once W2's hidden index is permuted the
//    same way (done in the pack), so H goes register -> MFMA with no LDS round trip;
//  * phase B: out^T(D x rows) += W2c H^T, accumulated over the F/32 chunks in VGPRs;
//  * epilogue in registers: + b2 + residual x (re-read, L2-hot), LayerNorm over the row
//    (each row's D outputs live in 4 lanes: in-lane sums + 2 cross-lane steps), 8-byte
//    stores.
// One barrier per chunk: wait own DMA -> barrier -> issue the next chunk's DMA into the
// slot everyone just finished -> compute.  Arithmetic intensity per workgroup = its row
// count (each weight byte feeds 16*RT*WAVES rows), 256 rows at D = 256.
#include <hip/hip_runtime.h>

#include "../../include/kinet_ffn.h"
#include "common.h"
#include "gemm_common.h"

namespace kinet {
namespace {

struct FfnArgs {
    const void* X;
    const void* W;
    const float* b1;
    const float* b2;
    const float* ln_g;
    const float* ln_b;
    void* Y;
    float eps;
    int ldx, ldy, M, F;
    int x_bytes, w_bytes, y_bytes;
    int dbg;   // diagnostic knobs (kinet_ffn_set_debug): 1 = no weight DMA after the prologue
               // (timing only, results are garbage); 2 = the 4-wave x 32-row tile at D = 256;
               // 8 = the 8-wave x 16-row tile (default: 8 waves x 32 rows, ffn_fused_rt2_kernel);
               // 16 = kinet_bottleneck_pair at D = 64 on the LDS-ring kernel (bneck_pair_kernel);
               // 128 / 256 = kinet_bottleneck_pair at D = 128 / 256 on 1- / 2-row-tile waves
};

thread_local int ffn_debug = 0;   // test-only knob (kinet_ffn_set_debug), per calling thread

template <int D>
struct FfnGeo {
    static_assert(D % 32 == 0, "D must be a multiple of 32");
    static constexpr int KS = D / 32;        // 32-deep K steps of linear1
    static constexpr int NT = D / 16;        // 16-wide output tiles of linear2
    static constexpr int FR = 2 * KS + NT;   // 1-KiB fragments per 32-unit hidden chunk
    static constexpr int CHUNK = FR * 1024;
};

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <typename T>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
    if constexpr (std::is_same<T, bf16_t>::value) {
        return (uint32_t)f32_to_bf16(a).x | ((uint32_t)f32_to_bf16(b).x << 16);
    } else {
        return (uint32_t)__builtin_bit_cast(uint16_t, (f16_t)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (f16_t)b) << 16);
    }
}

template <typename T>
__device__ __forceinline__ void unpack4(u32x2 u, float* v) {
    if constexpr (std::is_same<T, bf16_t>::value) {
        v[0] = __uint_as_float(u[0] << 16); v[1] = __uint_as_float(u[0] & 0xffff0000u);
        v[2] = __uint_as_float(u[1] << 16); v[3] = __uint_as_float(u[1] & 0xffff0000u);
    } else {
        v[0] = (float)__builtin_bit_cast(f16_t, (uint16_t)(u[0] & 0xffffu));
        v[1] = (float)__builtin_bit_cast(f16_t, (uint16_t)(u[0] >> 16));
        v[2] = (float)__builtin_bit_cast(f16_t, (uint16_t)(u[1] & 0xffffu));
        v[3] = (float)__builtin_bit_cast(f16_t, (uint16_t)(u[1] >> 16));
    }
}

// 16-byte pieces of an accumulator chunk row: lane group g holds hidden 4g..4g+3 (a, 2 packed
// words) and 16+4g..16+4g+3 (b).  One v_permlane16_swap per word exchanges between lane groups
// g and g^1 so that even g hold hidden 4g..4g+7 and odd g hold 4g+12..4g+19 (contiguous 8
// each: a row's 64 bytes in four 16-byte lanes); chunk_piece_off is that piece's first hidden
// index.  The swap is its own inverse (residual loads take the same route back).
__device__ __forceinline__ u32x4 chunk_swap(u32x2 a, u32x2 b) {
    const auto s0 = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
    return u32x4{s0[0], s1[0], s0[1], s1[1]};
}
__device__ __forceinline__ int chunk_piece_off(int g) { return (g & 1) ? 4 * g + 12 : 4 * g; }

template <int N>
__device__ __forceinline__ void ffn_wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// raw workgroup barrier for LDS traffic only: LDS-DMA issued earlier stays in flight
__device__ __forceinline__ void ffn_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

constexpr int FFN_MAX_F = 2048;

// output column of MFMA row m of phase-B tile nt: lane group g holds, for the tile pair
// (2kp, 2kp+1), the 8 consecutive columns 32kp + 8g .. +7 -- the same columns its phase-A
// x fragment xr[kp] holds, so the residual comes from registers and stores are 16 bytes
__host__ __device__ constexpr int ffn_sigma(int nt, int m) { return 32 * (nt >> 1) + 8 * (m >> 2) + 4 * (nt & 1) + (m & 3); }

template <typename T, int D, int RT, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void ffn_fused_kernel(const FfnArgs p, const int ntiles) {
    using G = FfnGeo<D>;
    constexpr int KS = G::KS, NT = G::NT, FR = G::FR;
    static_assert(FR % WAVES == 0, "whole DMA rounds per chunk");
    constexpr int FRW = FR / WAVES;          // LDS-DMA instructions per wave per chunk
    constexpr int XN = RT * KS;              // x-fragment loads per wave per tile
    constexpr int NST = RT * NT / 2;         // 16-byte stores per wave per tile
    static_assert(XN == NST, "one extra-count class");
    constexpr int ROWS = WAVES * 16 * RT;
    constexpr int NS = 4;                    // ring slots: 2 chunks in flight, the chunk in phase A,
                                             // the previous chunk in phase B
    constexpr unsigned OOB = 0x80000000u;
    constexpr int PAR = (FFN_MAX_F + 3 * D) * 4;
    __shared__ __attribute__((aligned(16))) char lds[PAR + NS * G::CHUNK];
    float* const pb1 = reinterpret_cast<float*>(lds);
    float* const pb2 = pb1 + FFN_MAX_F;
    float* const pg = pb2 + D;
    float* const pbe = pg + D;
    char* const ring = lds + PAR;

    const int P = gridDim.x, bx = blockIdx.x;
    const int cnt = bx < ntiles ? (ntiles - 1 - bx) / P + 1 : 0;
    if (cnt == 0) return;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, c16 = lane & 15;
    const int nch = p.F / 32, pfi = nch / 2;
    const bool ln = p.ln_g != nullptr;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.X, (short)0, p.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.W, (short)0, p.w_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(p.Y, (short)0, p.y_bytes, 0x00020000);

    for (int i = threadIdx.x; i < p.F; i += WAVES * 64) pb1[i] = p.b1[i];
    for (int i = threadIdx.x; i < D; i += WAVES * 64) {
        pb2[i] = p.b2[i];
        pg[i] = ln ? p.ln_g[i] : 1.f;
        pbe[i] = ln ? p.ln_b[i] : 0.f;
    }

    auto load_x = [&](int tile, u32x4 (&dst)[RT][KS]) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int r = tile * ROWS + wave * 16 * RT + 16 * rt + c16;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const unsigned off = r < p.M ? ((unsigned)r * (unsigned)p.ldx + (unsigned)(32 * ks + 8 * g)) * 2u : OOB;
                dst[rt][ks] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
            }
        }
    };
    // global chunk q of this workgroup (hidden chunk c = q mod nch, passed in: a runtime
    // modulo is a ~20-instruction scalar division) -> ring slot q % NS; wave w moves
    // fragments w, w+WAVES, ..
    auto dma_chunk = [&](int q, int c) {
        char* dst = ring + (q % NS) * G::CHUNK;
        const unsigned src = (unsigned)c * (unsigned)G::CHUNK + (unsigned)lane * 16u;
#pragma unroll
        for (int k = 0; k < FRW; ++k) {
            const int f = k * WAVES + wave;
            dma16(rw, dst + f * 1024, src + (unsigned)f * 1024u);
        }
    };
    // VMEM ops a wave issues in chunk iteration (tile t, chunk c) AFTER that iteration's DMA
    // (x prefetch, epilogue stores): they are younger than the DMA of the next two chunks.
    // Every per-chunk index here is wave-uniform scalar work shared by all waves of the CU
    // (one SALU issue per cycle per CU), so no divisions: the caller steps (t, c) back itself.
    auto extra = [&](int c, int t) {
        if (t < 0) return 0;
        return ((c == pfi && t + 1 < cnt) ? XN : 0) + (c == nch - 1 ? NST : 0);
    };

    u32x4 xr[RT][KS], xn[RT][KS];
    load_x(bx, xr);
    __syncthreads();   // parameters in LDS (drains the x loads too: nothing else in flight yet)
    const int total = cnt * nch;
    dma_chunk(0, 0);
    if (total > 1) dma_chunk(1, nch > 1 ? 1 : 0);

    f32x4 acc[RT][NT];
    constexpr int PB = 4;                      // W2 fragments read ahead of phase B
    auto fragA = [&](const char* slot, int ks, int h) {
        return *reinterpret_cast<const u32x4*>(slot + lane * 16 + (h * KS + ks) * 1024);
    };
    auto fragB = [&](const char* slot, int nt) {
        return *reinterpret_cast<const u32x4*>(slot + lane * 16 + (2 * KS + nt) * 1024);
    };
    // ReLU + round one 32-bit word (2 hidden units) of row tile w/4's phase-B operand: lane
    // holds H[row l&15][4g+i] (h0) and [16+4g+i] (h1) = the 8 K slots of the operand in the
    // order kinet_ffn_pack permuted W2 to
    auto hword = [&](const f32x4 (&q0)[RT], const f32x4 (&q1)[RT], int w) {
        const int rt = w >> 2, i = w & 3;
        const f32x4& src = i < 2 ? q0[rt] : q1[rt];
        const int e = 2 * (i & 1);
        return pack2<T>(fmaxf(src[e], 0.f), fmaxf(src[e + 1], 0.f));
    };
    // phase B of one chunk: out[row l&15][sigma(nt, 4g+i)] += W2c . H^T; fw[0..PB) preloaded
    auto phase_b = [&](const char* slot, u32x4 (&fw)[PB + 1], const u32x4 (&hb)[RT]) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            if (nt + PB < NT) fw[(nt + PB) % (PB + 1)] = fragB(slot, nt + PB);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) Mma<T>::run(acc[rt][nt], fw[nt % (PB + 1)], hb[rt]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    for (int ti = 0; ti < cnt; ++ti) {
    // consume the x fragments HERE (hipcc places the wait for their loads before this
    // statement, once per tile) so no vmcnt wait of the compiler's lands inside the chunk
    // loop, where it would retire the ring's DMA early
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(xr[rt][ks]));
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[rt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // Software pipeline over the hidden chunks: iteration c runs phase A of chunk c with the
    // ReLU/convert of chunk c-1 spread over its steps (VALU beside MFMA), then phase B of
    // chunk c-1; the tile's last chunk gets its phase B after the loop.  Operand fragments are
    // read from the ring two steps ahead and the steps are fenced with sched_barrier: with one
    // wave per SIMD nothing else hides LDS latency, and hipcc otherwise sinks every ds_read
    // next to its MFMA.
    f32x4 hp0[RT], hp1[RT];
    const char* wprev = ring;
    for (int c = 0; c < nch; ++c) {
        const int q = ti * nch + c;
        // retire chunk q: still allowed in flight = everything issued after its DMA
        if (q + 1 < total) {
            int c1 = c - 1, t1 = ti, c2 = c - 2, t2 = ti;
            if (c1 < 0) { c1 += nch; --t1; }
            if (c2 < 0) { c2 += nch; --t2; }
            if (c2 < 0) { c2 += nch; --t2; }   // nch == 1
            const int e = extra(c2, t2) + extra(c1, t1);
            if (p.dbg & 1) ffn_wait_vmcnt<0>();
            else if (e == 0) ffn_wait_vmcnt<FRW>();
            else ffn_wait_vmcnt<FRW + XN>();   // XN == NST; e == 2 XN only waits more
        } else {
            ffn_wait_vmcnt<0>();
        }
        ffn_lds_barrier();     // chunk q visible to all; slot (q+2)%NS free (chunk q-2 done)
        if (q + 2 < total && !(p.dbg & 1)) {
            int cn = c + 2;
            if (cn >= nch) cn -= nch;
            if (cn >= nch) cn -= nch;       // nch == 1
            dma_chunk(q + 2, cn);
        }
        if (c == pfi && ti + 1 < cnt) load_x(bx + (ti + 1) * P, xn);
        const char* wb = ring + (q % NS) * G::CHUNK;
        const bool pipe = c > 0;
        f32x4 h0[RT], h1[RT];
        {
            const f32x4 bb0 = *reinterpret_cast<const f32x4*>(pb1 + c * 32 + 4 * g);
            const f32x4 bb1 = *reinterpret_cast<const f32x4*>(pb1 + c * 32 + 16 + 4 * g);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {   // b1 folded into the accumulator init
                h0[rt] = bb0;
                h1[rt] = bb1;
            }
        }
        u32x4 fa[3][2], fw[PB + 1], hb[RT];
        fa[0][0] = fragA(wb, 0, 0); fa[0][1] = fragA(wb, 0, 1);
        fa[1][0] = fragA(wb, 1, 0); fa[1][1] = fragA(wb, 1, 1);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (ks + 2 < KS) {
                fa[(ks + 2) % 3][0] = fragA(wb, ks + 2, 0);
                fa[(ks + 2) % 3][1] = fragA(wb, ks + 2, 1);
            } else if (pipe) {
#pragma unroll
                for (int j = 0; j < PB / 2; ++j) {
                    const int nt = (ks + 2 - KS) * (PB / 2) + j;
                    fw[nt] = fragB(wprev, nt);
                }
            }
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                Mma<T>::run(h0[rt], fa[ks % 3][0], xr[rt][ks]);
                Mma<T>::run(h1[rt], fa[ks % 3][1], xr[rt][ks]);
            }
            if (pipe && ks < 4 * RT) hb[ks >> 2][ks & 3] = hword(hp0, hp1, ks);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (pipe) {
#pragma unroll
            for (int w = KS; w < 4 * RT; ++w) hb[w >> 2][w & 3] = hword(hp0, hp1, w);
            phase_b(wprev, fw, hb);
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            hp0[rt] = h0[rt];
            hp1[rt] = h1[rt];
        }
        wprev = wb;
    }
    {   // phase B of the tile's last chunk (its slot is still held: the next DMA into it is
        // issued only after the next iteration's barrier)
        u32x4 fw[PB + 1], hb[RT];
#pragma unroll
        for (int j = 0; j < PB; ++j) fw[j] = fragB(wprev, j);
#pragma unroll
        for (int w = 0; w < 4 * RT; ++w) hb[w >> 2][w & 3] = hword(hp0, hp1, w);
        phase_b(wprev, fw, hb);
    }

        // ---- tile epilogue, registers only: + b2 + residual x (= xr), LayerNorm, store ----
        const int tile = bx + ti * P;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int r = tile * ROWS + wave * 16 * RT + 16 * rt + c16;
            float s = 0.f;
#pragma unroll
            for (int kp = 0; kp < KS; ++kp) {
                float x8[8];
                unpack4<T>(u32x2{xr[rt][kp][0], xr[rt][kp][1]}, x8);
                unpack4<T>(u32x2{xr[rt][kp][2], xr[rt][kp][3]}, x8 + 4);
                const f32x4 b2a = *reinterpret_cast<const f32x4*>(pb2 + 32 * kp + 8 * g);
                const f32x4 b2b = *reinterpret_cast<const f32x4*>(pb2 + 32 * kp + 8 * g + 4);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float v0 = acc[rt][2 * kp][i] + b2a[i] + x8[i];
                    const float v1 = acc[rt][2 * kp + 1][i] + b2b[i] + x8[4 + i];
                    acc[rt][2 * kp][i] = v0;
                    acc[rt][2 * kp + 1][i] = v1;
                    s += v0 + v1;
                }
            }
            float mean = 0.f, rstd = 1.f;
            if (ln) {
                s += __shfl_xor(s, 16);
                s += __shfl_xor(s, 32);
                mean = s * (1.f / (float)D);
                float qv = 0.f;
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float d = acc[rt][nt][i] - mean;
                        qv += d * d;
                    }
                qv += __shfl_xor(qv, 16);
                qv += __shfl_xor(qv, 32);
                rstd = rsqrtf(qv * (1.f / (float)D) + p.eps);
            }
#pragma unroll
            for (int kp = 0; kp < KS; ++kp) {
                const int n0 = 32 * kp + 8 * g;
                float o[8];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    o[i] = acc[rt][2 * kp][i];
                    o[4 + i] = acc[rt][2 * kp + 1][i];
                }
                if (ln) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) o[e] = (o[e] - mean) * rstd * pg[n0 + e] + pbe[n0 + e];
                }
                u32x4 w;
#pragma unroll
                for (int e = 0; e < 4; ++e) w[e] = pack2<T>(o[2 * e], o[2 * e + 1]);
                // unconditional (OOB rows dropped by the range check): the store count per
                // tile is fixed, which the counted vmcnt above relies on
                const unsigned off = r < p.M ? ((unsigned)r * (unsigned)p.ldy + (unsigned)n0) * 2u : OOB;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, w), ry, off, 0, 0);
            }
        }
        if (ti + 1 < cnt) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) xr[rt][ks] = xn[rt][ks];
        }
    }
}

// 8 waves x 32 rows (two 16-row tiles per wave; the default at D = 256): every 1-KiB weight
// fragment read from the ring feeds two MFMAs -- half the LDS reads per MFMA of the 16-row tile,
// whose 8 waves saturate the LDS read port.  To stay within 256 VGPRs (two waves
// per SIMD) the tile's x fragments are loaded at the tile start instead of one tile ahead, phase
// B of a chunk follows its own phase A (no cross-chunk software pipeline) and the ring holds 3
// chunks (2 in flight + the one being computed).  Same packed weights, same sums in the same
// order per output element as ffn_fused_kernel (bit-identical results).
template <typename T, int D>
__global__ __launch_bounds__(512) void ffn_fused_rt2_kernel(const FfnArgs p, const int ntiles) {
    constexpr int RT = 2, WAVES = 8;
    using G = FfnGeo<D>;
    constexpr int KS = G::KS, NT = G::NT, FR = G::FR;
    static_assert(FR % WAVES == 0, "whole DMA rounds per chunk");
    constexpr int FRW = FR / WAVES;
    constexpr int ROWS = WAVES * 16 * RT;
    constexpr int NS = 3;
    constexpr unsigned OOB = 0x80000000u;
    constexpr int PAR = (FFN_MAX_F + 3 * D) * 4;
    __shared__ __attribute__((aligned(16))) char lds[PAR + NS * G::CHUNK];
    float* const pb1 = reinterpret_cast<float*>(lds);
    float* const pb2 = pb1 + FFN_MAX_F;
    float* const pg = pb2 + D;
    float* const pbe = pg + D;
    char* const ring = lds + PAR;

    const int P = gridDim.x, bx = blockIdx.x;
    const int cnt = bx < ntiles ? (ntiles - 1 - bx) / P + 1 : 0;
    if (cnt == 0) return;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, c16 = lane & 15;
    const int nch = p.F / 32;
    const bool ln = p.ln_g != nullptr;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.X, (short)0, p.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.W, (short)0, p.w_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(p.Y, (short)0, p.y_bytes, 0x00020000);

    for (int i = threadIdx.x; i < p.F; i += WAVES * 64) pb1[i] = p.b1[i];
    for (int i = threadIdx.x; i < D; i += WAVES * 64) {
        pb2[i] = p.b2[i];
        pg[i] = ln ? p.ln_g[i] : 1.f;
        pbe[i] = ln ? p.ln_b[i] : 0.f;
    }
    auto dma_chunk = [&](int q, int c) {
        char* dst = ring + (q % NS) * G::CHUNK;
        const unsigned src = (unsigned)c * (unsigned)G::CHUNK + (unsigned)lane * 16u;
#pragma unroll
        for (int k = 0; k < FRW; ++k) {
            const int f = k * WAVES + wave;
            dma16(rw, dst + f * 1024, src + (unsigned)f * 1024u);
        }
    };
    const int total = cnt * nch;
    __syncthreads();   // parameters in LDS
    dma_chunk(0, 0);
    if (total > 1) dma_chunk(1, nch > 1 ? 1 : 0);

    u32x4 xr[RT][KS];
    f32x4 acc[RT][NT];
    for (int ti = 0; ti < cnt; ++ti) {
        const int tile = bx + ti * P;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int r = tile * ROWS + wave * 16 * RT + 16 * rt + c16;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const unsigned off = r < p.M ? ((unsigned)r * (unsigned)p.ldx + (unsigned)(32 * ks + 8 * g)) * 2u : OOB;
                xr[rt][ks] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
            }
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[rt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < nch; ++c) {
            const int q = ti * nch + c;
            // chunk q landed: younger are at most chunk q+1's DMA (plus, at a tile boundary, the
            // previous tile's stores and this tile's x loads -- then this waits for those too)
            if (q + 1 < total) ffn_wait_vmcnt<FRW>();
            else ffn_wait_vmcnt<0>();
            ffn_lds_barrier();   // chunk q visible; slot (q+2) % NS (chunk q-1) free
            if (q + 2 < total) {
                int cn = c + 2;
                if (cn >= nch) cn -= nch;
                if (cn >= nch) cn -= nch;
                dma_chunk(q + 2, cn);
            }
            const char* wb = ring + (q % NS) * G::CHUNK;
            f32x4 h0[RT], h1[RT];
            {
                const f32x4 bb0 = *reinterpret_cast<const f32x4*>(pb1 + c * 32 + 4 * g);
                const f32x4 bb1 = *reinterpret_cast<const f32x4*>(pb1 + c * 32 + 16 + 4 * g);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    h0[rt] = bb0;
                    h1[rt] = bb1;
                }
            }
            // Fragments are read ahead of their MFMAs: phase A's two k-steps ahead, phase B's four
            // fragments ahead, the first four issued during phase A's last two k-steps (so the
            // ReLU / rounding between the phases overlaps their latency).  The scheduling barriers
            // keep the compiler from sinking the reads back next to their uses, where each pair of
            // MFMAs waited for its own LDS round trip: 593-599 -> 566-569 us per batch-28 encoder
            // FFN, bit-identical (profiles/r06af_ffn_prefetch_ab.txt; 3 or 6 ahead: the same time)
            auto frag = [&](int f) { return *reinterpret_cast<const u32x4*>(wb + lane * 16 + f * 1024); };
            constexpr int PDA = 2, PDB = 4;
            static_assert(KS >= PDA && NT >= PDB, "prefetch depths");
            u32x4 fa[KS][2], fw[NT];
#pragma unroll
            for (int i = 0; i < PDA; ++i) {
                fa[i][0] = frag(i);
                fa[i][1] = frag(KS + i);
            }
            // phase A: H^T chunk (32 hidden x 32 rows) = W1c x^T + b1
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                if (ks + PDA < KS) {
                    fa[ks + PDA][0] = frag(ks + PDA);
                    fa[ks + PDA][1] = frag(KS + ks + PDA);
                } else {   // phase B's first PDB reads, spread over phase A's last PDA k-steps
                    const int t = ks + PDA - KS;
#pragma unroll
                    for (int j = t * PDB / PDA; j < (t + 1) * PDB / PDA; ++j) fw[j] = frag(2 * KS + j);
                }
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    Mma<T>::run(h0[rt], fa[ks][0], xr[rt][ks]);
                    Mma<T>::run(h1[rt], fa[ks][1], xr[rt][ks]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            // ReLU + round: the B operand of phase B (hidden order as kinet_ffn_pack permuted W2).
            // ReLU as a signed-integer max on the bit pattern (one VALU op; fmaxf on an MFMA
            // result costs a canonicalising max first): the same value for every finite input
            auto relu = [](float v) { return __builtin_bit_cast(float, max(__builtin_bit_cast(int, v), 0)); };
            u32x4 hb[RT];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                hb[rt][0] = pack2<T>(relu(h0[rt][0]), relu(h0[rt][1]));
                hb[rt][1] = pack2<T>(relu(h0[rt][2]), relu(h0[rt][3]));
                hb[rt][2] = pack2<T>(relu(h1[rt][0]), relu(h1[rt][1]));
                hb[rt][3] = pack2<T>(relu(h1[rt][2]), relu(h1[rt][3]));
            }
            __builtin_amdgcn_sched_barrier(0);
            // phase B: out^T += W2c H^T, each W2 fragment feeding both row tiles
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                if (nt + PDB < NT) fw[nt + PDB] = frag(2 * KS + nt + PDB);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) Mma<T>::run(acc[rt][nt], fw[nt], hb[rt]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // ---- tile epilogue (as ffn_fused_kernel): + b2 + residual x, LayerNorm, 16-byte stores ----
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int r = tile * ROWS + wave * 16 * RT + 16 * rt + c16;
            float s = 0.f;
#pragma unroll
            for (int kp = 0; kp < KS; ++kp) {
                float x8[8];
                unpack4<T>(u32x2{xr[rt][kp][0], xr[rt][kp][1]}, x8);
                unpack4<T>(u32x2{xr[rt][kp][2], xr[rt][kp][3]}, x8 + 4);
                const f32x4 b2a = *reinterpret_cast<const f32x4*>(pb2 + 32 * kp + 8 * g);
                const f32x4 b2b = *reinterpret_cast<const f32x4*>(pb2 + 32 * kp + 8 * g + 4);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float v0 = acc[rt][2 * kp][i] + b2a[i] + x8[i];
                    const float v1 = acc[rt][2 * kp + 1][i] + b2b[i] + x8[4 + i];
                    acc[rt][2 * kp][i] = v0;
                    acc[rt][2 * kp + 1][i] = v1;
                    s += v0 + v1;
                }
            }
            float mean = 0.f, rstd = 1.f;
            if (ln) {
                s += __shfl_xor(s, 16);
                s += __shfl_xor(s, 32);
                mean = s * (1.f / (float)D);
                float qv = 0.f;
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float d = acc[rt][nt][i] - mean;
                        qv += d * d;
                    }
                qv += __shfl_xor(qv, 16);
                qv += __shfl_xor(qv, 32);
                rstd = rsqrtf(qv * (1.f / (float)D) + p.eps);
            }
#pragma unroll
            for (int kp = 0; kp < KS; ++kp) {
                const int n0 = 32 * kp + 8 * g;
                float o[8];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    o[i] = acc[rt][2 * kp][i];
                    o[4 + i] = acc[rt][2 * kp + 1][i];
                }
                if (ln) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) o[e] = (o[e] - mean) * rstd * pg[n0 + e] + pbe[n0 + e];
                }
                u32x4 w;
#pragma unroll
                for (int e = 0; e < 4; ++e) w[e] = pack2<T>(o[2 * e], o[2 * e + 1]);
                const unsigned off = r < p.M ? ((unsigned)r * (unsigned)p.ldy + (unsigned)n0) * 2u : OOB;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, w), ry, off, 0, 0);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// ResNet bottleneck pair: block i's conv3 (1x1, D -> F = 4D, + FrozenBN + residual + ReLU) and
// block i+1's conv1 (1x1, F -> D, + FrozenBN + ReLU) in one launch (torchvision Bottleneck as
// instantiated by the reference, backbone.py:94-108).  Same scheme as the FFN: phase A's
// accumulators (the F-wide block output, chunk by chunk) are phase B's operands, so the block
// output is written once (it is the next block's residual) and never re-read by the next conv1.
//  * phase A: H^T(32 x rows) = W3c t2^T + b3 (the BN scales are folded into the packed weight
//    rows, kinet_bottleneck_pack);  + residual, ReLU, round -> stored to Y (two 8-byte pieces
//    per lane and row tile) and used as the B operand of phase B;
//  * the residual slice of each chunk (rows of the tile x 32 channels, 64 B per row) travels
//    with the chunk's weights by LDS-DMA, two chunks ahead, 16-byte pieces XOR-swizzled by
//    row so the 8-byte reads are conflict-free;
//  * phase B: out^T(D x rows) += W1c H^T over the F/32 chunks; epilogue relu(out + b1).
// Weights: kinet_bottleneck_pack(W3 (F, D), W1 (D, F), s3, s1) -- the FFN fragment layout with
// W3 rows scaled by s3 and W1 rows by s1 before rounding.  F == 4D (the bottleneck expansion).
struct PairArgs {
    const void* X;   // t2 (M, D), row stride ldx
    const void* R;   // residual (M, F), dense
    const void* W;   // packed weights (BN scales folded)
    const float* b3;
    const float* b1;
    void* Y;   // block output (M, F), dense
    void* T;   // next conv1 output (M, D), dense
    int ldx, M, F;
    int x_bytes, r_bytes, w_bytes, y_bytes, t_bytes;
};

template <typename T, int D, int RT, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void bneck_pair_kernel(const PairArgs p, const int ntiles) {
    using G = FfnGeo<D>;
    constexpr int KS = G::KS, NT = G::NT, FR = G::FR;
    static_assert(FR % WAVES == 0, "whole DMA rounds per chunk");
    constexpr int FRW = FR / WAVES;             // weight LDS-DMA instructions per wave per chunk
    constexpr int ROWS = WAVES * 16 * RT;
    constexpr int RES = ROWS * 64;              // residual slice per chunk: 32 channels x 2 B per row
    constexpr int RESW = RT;                    // residual LDS-DMA instructions per wave per chunk (1 KiB each)
    constexpr int SLOT = G::CHUNK + RES;
    constexpr int NS = 3;
    constexpr int F4 = 4 * D;
    constexpr int PAR = (F4 + D) * 4;
    constexpr unsigned OOB = 0x80000000u;
    __shared__ __attribute__((aligned(16))) char lds[PAR + NS * SLOT];
    float* const pb3 = reinterpret_cast<float*>(lds);
    float* const pb1 = pb3 + F4;
    char* const ring = lds + PAR;

    const int P = gridDim.x, bx = blockIdx.x;
    const int cnt = bx < ntiles ? (ntiles - 1 - bx) / P + 1 : 0;
    if (cnt == 0) return;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, c16 = lane & 15;
    const int F = p.F, nch = F / 32;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.X, (short)0, p.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)p.R, (short)0, p.r_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.W, (short)0, p.w_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(p.Y, (short)0, p.y_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rt_ = __builtin_amdgcn_make_buffer_rsrc(p.T, (short)0, p.t_bytes, 0x00020000);

    for (int i = threadIdx.x; i < F4; i += WAVES * 64) pb3[i] = p.b3[i];
    for (int i = threadIdx.x; i < D; i += WAVES * 64) pb1[i] = p.b1[i];
    // chunk q = (tile bx + (q / nch) * P, hidden chunk q % nch): its weights + residual slice.
    // Residual piece of lane l in instruction k: row (k*WAVES + wave)*16 + l/4, 16-byte piece
    // (l & 3) ^ ((row >> 2) & 3) of the row's 64 bytes, landing at LDS unit l (row-major).
    auto dma_chunk = [&](int q) {
        const int ti = q / nch, c = q - ti * nch;
        const int tile = bx + ti * P;
        char* dst = ring + (q % NS) * SLOT;
        const unsigned src = (unsigned)c * (unsigned)G::CHUNK + (unsigned)lane * 16u;
#pragma unroll
        for (int k = 0; k < FRW; ++k) {
            const int f = k * WAVES + wave;
            dma16(rw, dst + f * 1024, src + (unsigned)f * 1024u);
        }
#pragma unroll
        for (int k = 0; k < RESW; ++k) {
            const int rl = (k * WAVES + wave) * 16 + (lane >> 2);
            const int r = tile * ROWS + rl;
            const int piece = (lane & 3) ^ ((rl >> 2) & 3);
            const unsigned off =
                r < p.M ? ((unsigned)r * (unsigned)F + (unsigned)(32 * c)) * 2u + (unsigned)piece * 16u : OOB;
            dma16(rr, dst + G::CHUNK + (k * WAVES + wave) * 1024, off);
        }
    };
    const int total = cnt * nch;
    __syncthreads();   // parameters in LDS
    dma_chunk(0);
    if (total > 1) dma_chunk(1);

    u32x4 xr[RT][KS];
    f32x4 acc[RT][NT];
    for (int ti = 0; ti < cnt; ++ti) {
        const int tile = bx + ti * P;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int r = tile * ROWS + wave * 16 * RT + 16 * rt + c16;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const unsigned off = r < p.M ? ((unsigned)r * (unsigned)p.ldx + (unsigned)(32 * ks + 8 * g)) * 2u : OOB;
                xr[rt][ks] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
            }
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[rt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < nch; ++c) {
            const int q = ti * nch + c;
            // chunk q landed.  Younger vector-memory ops (DMA(q) was issued in iteration q-2):
            // chunk q-2's Y stores (RT), chunk q+1's DMA (if any), chunk q-1's Y stores (RT); across
            // a tile start also T stores and x loads (RT*KS >= RT).  At c == 0 only the DMA is
            // counted (waits longer, and right after the prologue nothing else is younger but x)
            if (q + 1 >= total) ffn_wait_vmcnt<0>();
            else if (c == 0) ffn_wait_vmcnt<FRW + RESW>();
            else ffn_wait_vmcnt<FRW + RESW + 2 * RT>();
            ffn_lds_barrier();   // chunk q visible; slot (q+2) % NS (chunk q-1) free
            if (q + 2 < total) dma_chunk(q + 2);
            const char* wb = ring + (q % NS) * SLOT;
            const char* rb = wb + G::CHUNK;
            f32x4 h0[RT], h1[RT];
            {
                const f32x4 ba = *reinterpret_cast<const f32x4*>(pb3 + c * 32 + 4 * g);
                const f32x4 bb = *reinterpret_cast<const f32x4*>(pb3 + c * 32 + 16 + 4 * g);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    h0[rt] = ba;
                    h1[rt] = bb;
                }
            }
            u32x4 fa0 = *reinterpret_cast<const u32x4*>(wb + lane * 16);
            u32x4 fa1 = *reinterpret_cast<const u32x4*>(wb + lane * 16 + KS * 1024);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                u32x4 na0 = fa0, na1 = fa1;
                if (ks + 1 < KS) {
                    na0 = *reinterpret_cast<const u32x4*>(wb + lane * 16 + (ks + 1) * 1024);
                    na1 = *reinterpret_cast<const u32x4*>(wb + lane * 16 + (KS + ks + 1) * 1024);
                }
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    Mma<T>::run(h0[rt], fa0, xr[rt][ks]);
                    Mma<T>::run(h1[rt], fa1, xr[rt][ks]);
                }
                fa0 = na0;
                fa1 = na1;
            }
            // + residual, ReLU, round: the block output (stored) and phase B's operand
            u32x4 hb[RT];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const int rl = wave * 16 * RT + 16 * rt + c16;
                const int sw = (c16 >> 2) & 3;
                const u32x2 ra = *reinterpret_cast<const u32x2*>(rb + rl * 64 + (((g >> 1) ^ sw) << 4) + (g & 1) * 8);
                const u32x2 rb2 = *reinterpret_cast<const u32x2*>(rb + rl * 64 + (((2 + (g >> 1)) ^ sw) << 4) + (g & 1) * 8);
                float r0[4], r1[4];
                unpack4<T>(ra, r0);
                unpack4<T>(rb2, r1);
                float v0[4], v1[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    v0[j] = fmaxf(h0[rt][j] + r0[j], 0.f);
                    v1[j] = fmaxf(h1[rt][j] + r1[j], 0.f);
                }
                hb[rt][0] = pack2<T>(v0[0], v0[1]);
                hb[rt][1] = pack2<T>(v0[2], v0[3]);
                hb[rt][2] = pack2<T>(v1[0], v1[1]);
                hb[rt][3] = pack2<T>(v1[2], v1[3]);
                const int r = tile * ROWS + rl;
                const unsigned yo = ((unsigned)r * (unsigned)F + (unsigned)(32 * c + chunk_piece_off(g))) * 2u;
                __builtin_amdgcn_raw_buffer_store_b128(chunk_swap(u32x2{hb[rt][0], hb[rt][1]}, u32x2{hb[rt][2], hb[rt][3]}),
                                                       ry, r < p.M ? yo : OOB, 0, 0);
            }
            // phase B: out^T += W1c H^T, each W1 fragment feeding the RT row tiles
            u32x4 fw = *reinterpret_cast<const u32x4*>(wb + lane * 16 + (2 * KS) * 1024);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                u32x4 nw = fw;
                if (nt + 1 < NT) nw = *reinterpret_cast<const u32x4*>(wb + lane * 16 + (2 * KS + nt + 1) * 1024);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) Mma<T>::run(acc[rt][nt], fw, hb[rt]);
                fw = nw;
            }
        }
        // ---- tile epilogue: relu(out + b1), 16-byte stores of 8 consecutive channels ----
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int r = tile * ROWS + wave * 16 * RT + 16 * rt + c16;
#pragma unroll
            for (int kp = 0; kp < KS; ++kp) {
                const int n0 = 32 * kp + 8 * g;
                float o[8];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    o[i] = fmaxf(acc[rt][2 * kp][i] + pb1[n0 + i], 0.f);
                    o[4 + i] = fmaxf(acc[rt][2 * kp + 1][i] + pb1[n0 + 4 + i], 0.f);
                }
                u32x4 w;
#pragma unroll
                for (int e = 0; e < 4; ++e) w[e] = pack2<T>(o[2 * e], o[2 * e + 1]);
                const unsigned off = r < p.M ? ((unsigned)r * (unsigned)D + (unsigned)n0) * 2u : OOB;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, w), rt_, off, 0, 0);
            }
        }
    }
}

// D = 64 (ResNet layer 1): the whole packed weight stream is 64 KiB, so it is loaded into LDS
// ONCE per workgroup and every wave then runs on its own -- no ring, no barrier in the loop.
// The pair is HBM-bound here (per row 128 B in + 512 B residual + 512 B out + 128 B out; 16
// MFMAs of work per 16 rows and chunk), so what matters is bytes in flight: each wave owns a
// 16-row tile and holds the tile's whole residual (8 chunks x 2 pieces per lane = 32 VGPRs);
// as chunk c consumes its residual registers, they are refilled with the NEXT tile's chunk c,
// so every residual load has a whole tile of work to land under, and the next tile's t2 rows
// load at the tile start into a second register set.  Residual loads and block-output stores
// move 16 bytes per lane (chunk_swap: a row's 64 chunk bytes in four lanes).
// DB = the next conv1's output width: 64 inside stage 1, 128 for the pair that ends stage 1
// (its last conv3 -> stage 2's first conv1, 256 -> 128 channels at stride 1); then the weights
// take 96 KiB and one 16-wave workgroup runs per CU.
template <typename T, int DB, int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1024 / (WAVES * 64)) void bneck64_kernel(const PairArgs p, const int ntiles) {
    constexpr int D = 64, F = 256, KS = 2, NT = DB / 16, KSB = DB / 32, FR = 2 * KS + NT, NCH = F / 32;
    constexpr unsigned OOB = 0x80000000u;
    __shared__ __attribute__((aligned(16))) char wl[NCH * FR * 1024];
    __shared__ float pb3[F], pb1[DB];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, c16 = lane & 15;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)p.X, (short)0, p.x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)p.R, (short)0, p.r_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.W, (short)0, p.w_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(p.Y, (short)0, p.y_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rt_ = __builtin_amdgcn_make_buffer_rsrc(p.T, (short)0, p.t_bytes, 0x00020000);
    for (int i = threadIdx.x; i < F; i += WAVES * 64) pb3[i] = p.b3[i];
    if (threadIdx.x < DB) pb1[threadIdx.x] = p.b1[threadIdx.x];
    static_assert(NCH * FR % WAVES == 0, "whole DMA rounds");
#pragma unroll
    for (int k = 0; k < NCH * FR / WAVES; ++k) {
        const int f = k * WAVES + wave;
        dma16(rw, wl + f * 1024, (unsigned)f * 1024u + (unsigned)lane * 16u);
    }
    ffn_wait_vmcnt<0>();
    __syncthreads();

    const int nw = gridDim.x * WAVES;
    int tile = blockIdx.x * WAVES + wave;
    if (tile >= ntiles) return;
    auto row_of = [&](int t) { return t * 16 + c16; };
    auto load_x = [&](int t, u32x4 (&dst)[KS]) {
        const int r = row_of(t);
        const bool ok = t < ntiles && r < p.M;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            dst[ks] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rx, ok ? ((unsigned)r * (unsigned)p.ldx + (unsigned)(32 * ks + 8 * g)) * 2u : OOB, 0, 0));
    };
    const int poff = chunk_piece_off(g);
    auto res_off = [&](int t, int c) -> unsigned {
        const int r = row_of(t);
        return (t < ntiles && r < p.M) ? ((unsigned)r * (unsigned)F + (unsigned)(32 * c + poff)) * 2u : OOB;
    };
    u32x4 xr[KS], xn[KS];
    u32x4 res[NCH];   // 16-byte pieces (chunk_swap order)
    load_x(tile, xr);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
        res[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, res_off(tile, c), 0, 0));
    // first tile landed (once per wave): otherwise the compiler's wait for these registers at the
    // loop head, merged with the back edge, drains every residual load of each later tile there
    __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
    for (; tile < ntiles; tile += nw) {
        const int next = tile + nw;
        load_x(next, xn);
        f32x4 acc[NT];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int r = row_of(tile);
        const bool rok = r < p.M;
        // opaque per tile: keeps the 64 weight-fragment reads in the loop (hoisted, they would
        // take 256 VGPRs)
        int woff = lane * 16;
        asm volatile("" : "+v"(woff));
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const char* wb = wl + c * FR * 1024 + woff;
            f32x4 h0 = *reinterpret_cast<const f32x4*>(pb3 + c * 32 + 4 * g);
            f32x4 h1 = *reinterpret_cast<const f32x4*>(pb3 + c * 32 + 16 + 4 * g);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                Mma<T>::run(h0, *reinterpret_cast<const u32x4*>(wb + ks * 1024), xr[ks]);
                Mma<T>::run(h1, *reinterpret_cast<const u32x4*>(wb + (KS + ks) * 1024), xr[ks]);
            }
            const u32x4 rq = chunk_swap(u32x2{res[c][0], res[c][1]}, u32x2{res[c][2], res[c][3]});
            float r0[4], r1[4];
            unpack4<T>(u32x2{rq[0], rq[1]}, r0);
            unpack4<T>(u32x2{rq[2], rq[3]}, r1);
            u32x4 hb;
            hb[0] = pack2<T>(fmaxf(h0[0] + r0[0], 0.f), fmaxf(h0[1] + r0[1], 0.f));
            hb[1] = pack2<T>(fmaxf(h0[2] + r0[2], 0.f), fmaxf(h0[3] + r0[3], 0.f));
            hb[2] = pack2<T>(fmaxf(h1[0] + r1[0], 0.f), fmaxf(h1[1] + r1[1], 0.f));
            hb[3] = pack2<T>(fmaxf(h1[2] + r1[2], 0.f), fmaxf(h1[3] + r1[3], 0.f));
            const unsigned yo = ((unsigned)r * (unsigned)F + (unsigned)(32 * c + poff)) * 2u;
            __builtin_amdgcn_raw_buffer_store_b128(chunk_swap(u32x2{hb[0], hb[1]}, u32x2{hb[2], hb[3]}), ry,
                                                   rok ? yo : OOB, 0, 0);
            // this chunk's residual registers now take the next tile's chunk c
            res[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, res_off(next, c), 0, 0));
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                Mma<T>::run(acc[nt], *reinterpret_cast<const u32x4*>(wb + (2 * KS + nt) * 1024), hb);
        }
#pragma unroll
        for (int kp = 0; kp < KSB; ++kp) {
            const int n0 = 32 * kp + 8 * g;
            u32x4 w;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                w[e] = pack2<T>(fmaxf(acc[2 * kp][2 * e] + pb1[n0 + 2 * e], 0.f),
                                fmaxf(acc[2 * kp][2 * e + 1] + pb1[n0 + 2 * e + 1], 0.f));
                w[2 + e] = pack2<T>(fmaxf(acc[2 * kp + 1][2 * e] + pb1[n0 + 4 + 2 * e], 0.f),
                                    fmaxf(acc[2 * kp + 1][2 * e + 1] + pb1[n0 + 4 + 2 * e + 1], 0.f));
            }
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, w), rt_,
                                                   rok ? ((unsigned)r * (unsigned)DB + (unsigned)n0) * 2u : OOB, 0, 0);
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) xr[ks] = xn[ks];
    }
}

template <typename T, int D, int RT, int WAVES, int WG_PER_CU>
void launch_pair_cfg(const PairArgs& a, hipStream_t s) {
    constexpr int ROWS = WAVES * 16 * RT;
    const int nt = (a.M + ROWS - 1) / ROWS;
    const int cap = 256 * WG_PER_CU;
    hipLaunchKernelGGL((bneck_pair_kernel<T, D, RT, WAVES>), dim3(nt < cap ? nt : cap), dim3(WAVES * 64), 0, s, a, nt);
}

template <typename T>
int launch_pair(const PairArgs& a, int D, int DB, hipStream_t s) {
    if (D == 64 && DB == 128) {
        const int nt = (a.M + 15) / 16, nb = (nt + 15) / 16;
        hipLaunchKernelGGL((bneck64_kernel<T, 128, 16>), dim3(nb < 256 ? nb : 256), dim3(1024), 0, s, a, nt);
        return KINET_OK;
    }
    if (DB != D) return KINET_ERR_ARG;
    switch (D) {
        case 64:
            if (ffn_debug & 16) {   // A/B knob: the LDS-ring pair kernel at D = 64 too
                launch_pair_cfg<T, 64, 2, 8, 2>(a, s);
            } else {
                const int nt = (a.M + 15) / 16, nb = (nt + 7) / 8;
                hipLaunchKernelGGL((bneck64_kernel<T, 64, 8>), dim3(nb < 512 ? nb : 512), dim3(512), 0, s, a, nt);
            }
            break;
        case 128:
        case 256: {
            // one or two 16-row tiles per wave (128- or 256-row workgroup tiles; the same sums per
            // element either way): the 2-tile tile reads each weight fragment once for two MFMAs,
            // but with one batch in flight (kinet_set_solo_launch), when its tiles fill their rounds
            // of one workgroup per CU 1.5x worse than the 1-tile grid, the 1-tile grid wins --
            // config 5's stage-3 pairs (M = 32,640: 128 vs 255 tiles on 256 CUs) 84.7 -> 62.9 us
            // alone (profiles/r06aa_config5_shapes.txt); on 3 streams the other batches fill the
            // idle CUs (neutral, profiles/r06ab_solo_launch_ab.txt).
            // ffn_debug 128 / 256 force the 1- / 2-tile grid (tests, A/B)
            const int cus = cu_count();
            const long t2 = (a.M + 255) / 256, t1 = (a.M + 127) / 128;
            const double e2 = (double)t2 / (double)(((t2 + cus - 1) / cus) * cus);
            const double e1 = (double)t1 / (double)(((t1 + cus - 1) / cus) * cus);
            const bool one = (ffn_debug & 128) || (!(ffn_debug & 256) && kinet_solo_launch && e1 > 1.5 * e2);
            if (D == 128) {
                if (one) launch_pair_cfg<T, 128, 1, 8, 1>(a, s);
                else launch_pair_cfg<T, 128, 2, 8, 1>(a, s);
            } else {
                if (one) launch_pair_cfg<T, 256, 1, 8, 1>(a, s);
                else launch_pair_cfg<T, 256, 2, 8, 1>(a, s);
            }
            break;
        }
        default: return KINET_ERR_ARG;
    }
    return KINET_OK;
}

// packed[c][f][lane][j] (see include/kinet_ffn.h): f < 2KS -> W1 fragment (h-tile f / KS,
// k-step f % KS); else W2 fragment of output tile f - 2KS with the hidden index permuted to
// the phase-A accumulator order.
// kinet_bottleneck_pack: ffn_pack_kernel's fragment order from f32 weights, W3 row h scaled by
// s3[h] and W1 row n by s1[n] (FrozenBN folded) before the one rounding to T
template <typename T>
__global__ void bneck_pack_kernel(const float* __restrict__ W3, const float* __restrict__ W1,
                                  const float* __restrict__ s3, const float* __restrict__ s1, T* __restrict__ out,
                                  int D, int F, int DB) {
    const int KS = D / 32, NT = DB / 16, FR = 2 * KS + NT;
    const long total = (long)(D + DB) * F;
    for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
        const long per_chunk = (long)FR * 512;
        const int c = (int)(idx / per_chunk);
        const int rem = (int)(idx - (long)c * per_chunk);
        const int f = rem >> 9, e = rem & 511;
        const int lane = e >> 3, j = e & 7, g = lane >> 4, c16 = lane & 15;
        float v;
        if (f < 2 * KS) {
            const int ht = f / KS, ks = f - ht * KS;
            const int h = 32 * c + 16 * ht + c16;
            v = W3[(long)h * D + 32 * ks + 8 * g + j] * s3[h];
        } else {
            const int nt = f - 2 * KS;
            const int h = 32 * c + (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4));
            const int n = ffn_sigma(nt, c16);
            v = W1[(long)n * F + h] * s1[n];
        }
        out[idx] = Cvt<T>::from(v);
    }
}

template <typename T>
__global__ void ffn_pack_kernel(const T* __restrict__ W1, const T* __restrict__ W2, T* __restrict__ out, int D,
                                int F) {
    const int KS = D / 32, NT = D / 16, FR = 2 * KS + NT;
    const long total = 2L * D * F;
    for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
        const long per_chunk = (long)FR * 512;
        const int c = (int)(idx / per_chunk);
        const int rem = (int)(idx - (long)c * per_chunk);
        const int f = rem >> 9, e = rem & 511;
        const int lane = e >> 3, j = e & 7, g = lane >> 4, c16 = lane & 15;
        T v;
        if (f < 2 * KS) {
            const int ht = f / KS, ks = f - ht * KS;
            v = W1[(long)(32 * c + 16 * ht + c16) * D + 32 * ks + 8 * g + j];
        } else {
            const int nt = f - 2 * KS;
            const int h = 32 * c + (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4));
            v = W2[(long)ffn_sigma(nt, c16) * F + h];
        }
        out[idx] = v;
    }
}

template <typename T, int D>
int launch_ffn(const FfnArgs& a, hipStream_t s) {
    // persistent: one workgroup per CU walks row tiles.  Many rows: 4 waves x 32 rows (128
    // rows share each weight byte; the 2 x D/16 output tiles + 2 x D/32 x-fragments (+ the
    // next tile's prefetch) need > 256 VGPRs, so one wave per SIMD);  few rows (decoder
    // queries): 4 waves x 16 rows, so the rows spread over more CUs
    if (a.M >= 16384) {
        const int nt = (a.M + 127) / 128;
        if constexpr (FfnGeo<D>::FR % 8 == 0) {
            if (a.dbg & 2) {   // A/B knob: 4 waves x 32 rows (one wave per SIMD)
                const int n2 = (a.M + 127) / 128;
                hipLaunchKernelGGL((ffn_fused_kernel<T, D, 2, 4>), dim3(n2 < 256 ? n2 : 256), dim3(256), 0, s, a, n2);
                return KINET_OK;
            }
            if (a.dbg & 8) {   // A/B knob: 8 waves x 16 rows (the round-3 default)
                hipLaunchKernelGGL((ffn_fused_kernel<T, D, 1, 8>), dim3(nt < 256 ? nt : 256), dim3(512), 0, s, a, nt);
                return KINET_OK;
            }
            // 8 waves x 32 rows: each weight fragment feeds two MFMAs and two waves per SIMD hide
            // each other's latency (config-2 encoder FFN at batch 16: 419 vs 486 us alone, bench
            // 1267 vs 1219 frames/s, profiles/r04c_ffn_probe.log, r04c_ab_*.json)
            const int n4 = (a.M + 255) / 256;
            hipLaunchKernelGGL((ffn_fused_rt2_kernel<T, D>), dim3(n4 < 256 ? n4 : 256), dim3(512), 0, s, a, n4);
        } else {
            hipLaunchKernelGGL((ffn_fused_kernel<T, D, 2, 4>), dim3(nt < 256 ? nt : 256), dim3(256), 0, s, a, nt);
        }
    } else {
        const int nt = (a.M + 63) / 64;
        hipLaunchKernelGGL((ffn_fused_kernel<T, D, 1, 4>), dim3(nt < 256 ? nt : 256), dim3(256), 0, s, a, nt);
    }
    return KINET_OK;
}

bool al16(const void* q) { return (((uintptr_t)q) & 15u) == 0; }

}  // namespace
}  // namespace kinet

using namespace kinet;

extern "C" int kinet_ffn_set_debug(int flags) {
    const int old = ffn_debug;
    ffn_debug = flags;
    return old;
}

extern "C" int kinet_ffn_pack(const void* W1, const void* W2, void* packed, int D, int F, int dtype,
                              kinet_stream_t stream) {
    KINET_CHECK_ARG(D > 0 && D % 32 == 0 && F > 0 && F % 32 == 0, "ffn_pack: need D %% 32 == 0 and F %% 32 == 0 (D=%d F=%d)", D, F);
    KINET_CHECK_ARG(dtype == KINET_BF16 || dtype == KINET_F16, "ffn_pack: dtype must be bf16 or f16");
    const long total = 2L * D * F;
    const int grid = (int)((total + 255) / 256 < kMaxGridStride ? (total + 255) / 256 : kMaxGridStride);
    if (dtype == KINET_BF16)
        hipLaunchKernelGGL(ffn_pack_kernel<bf16_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)W1,
                           (const bf16_t*)W2, (bf16_t*)packed, D, F);
    else
        hipLaunchKernelGGL(ffn_pack_kernel<f16_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const f16_t*)W1,
                           (const f16_t*)W2, (f16_t*)packed, D, F);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_ffn_fused(const void* X, int ldx, const void* packed, const float* b1, const float* b2,
                               const float* ln_gamma, const float* ln_beta, float ln_eps, void* Y, int ldy, int M,
                               int D, int F, int dtype, kinet_stream_t stream) {
    KINET_CHECK_ARG(D == 256 || D == 288, "ffn_fused: D must be 256 or 288 (got %d)", D);
    KINET_CHECK_ARG(F > 0 && F % 32 == 0 && F <= FFN_MAX_F, "ffn_fused: F must be a multiple of 32 in [32, %d] (got %d)", FFN_MAX_F, F);
    KINET_CHECK_ARG(M >= 0 && ldx >= D && ldy >= D && ldx % 8 == 0 && ldy % 8 == 0, "ffn_fused: bad M / ldx / ldy");
    KINET_CHECK_ARG(dtype == KINET_BF16 || dtype == KINET_F16, "ffn_fused: dtype must be bf16 or f16");
    KINET_CHECK_ARG(b1 != nullptr && b2 != nullptr, "ffn_fused: b1 and b2 are required");
    KINET_CHECK_ARG((ln_gamma == nullptr) == (ln_beta == nullptr), "ffn_fused: LayerNorm needs both gamma and beta");
    KINET_CHECK_ARG(al16(X) && al16(Y) && al16(packed) && al16(b1) && al16(b2) &&
                    (ln_gamma == nullptr || (al16(ln_gamma) && al16(ln_beta))),
                    "ffn_fused: X, Y, packed weights, biases and LayerNorm params must be 16-byte aligned");
    if (M == 0) return KINET_OK;
    const long long xb = ((long long)(M - 1) * ldx + D) * 2;
    KINET_CHECK_ARG(xb < (1LL << 31), "ffn_fused: X larger than 2 GiB (split the call)");
    FfnArgs a{};
    a.X = X; a.W = packed; a.b1 = b1; a.b2 = b2; a.ln_g = ln_gamma; a.ln_b = ln_beta; a.Y = Y; a.eps = ln_eps;
    a.ldx = ldx; a.ldy = ldy; a.M = M; a.F = F;
    a.x_bytes = (int)xb;
    a.w_bytes = (int)(2LL * D * F * 2);
    const long long yb = ((long long)(M - 1) * ldy + D) * 2;
    KINET_CHECK_ARG(yb < (1LL << 31), "ffn_fused: Y larger than 2 GiB (split the call)");
    a.y_bytes = (int)yb;
    a.dbg = ffn_debug;
    hipStream_t s = (hipStream_t)stream;
    int rc;
    if (dtype == KINET_BF16) rc = D == 256 ? launch_ffn<bf16_t, 256>(a, s) : launch_ffn<bf16_t, 288>(a, s);
    else rc = D == 256 ? launch_ffn<f16_t, 256>(a, s) : launch_ffn<f16_t, 288>(a, s);
    if (rc) return rc;
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_bottleneck_pack(const float* W3, const float* W1, const float* s3, const float* s1,
                                     void* packed, int D, int F, int DB, int dtype, kinet_stream_t stream) {
    KINET_CHECK_ARG(D > 0 && D % 32 == 0 && F > 0 && F % 32 == 0 && DB > 0 && DB % 32 == 0,
                    "bottleneck_pack: need D, F, DB multiples of 32 (D=%d F=%d DB=%d)", D, F, DB);
    KINET_CHECK_ARG(dtype == KINET_BF16 || dtype == KINET_F16, "bottleneck_pack: dtype must be bf16 or f16");
    KINET_CHECK_ARG(W3 && W1 && s3 && s1 && packed, "bottleneck_pack: null pointer");
    const long total = (long)(D + DB) * F;
    const int grid = (int)((total + 255) / 256 < kMaxGridStride ? (total + 255) / 256 : kMaxGridStride);
    if (dtype == KINET_BF16)
        hipLaunchKernelGGL(bneck_pack_kernel<bf16_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream, W3, W1, s3, s1,
                           (bf16_t*)packed, D, F, DB);
    else
        hipLaunchKernelGGL(bneck_pack_kernel<f16_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream, W3, W1, s3, s1,
                           (f16_t*)packed, D, F, DB);
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}

extern "C" int kinet_bottleneck_pair(const void* X, int ldx, const void* R, const void* packed, const float* b3,
                                     const float* b1, void* Y, void* T, int M, int D, int F, int DB, int dtype,
                                     kinet_stream_t stream) {
    KINET_CHECK_ARG(D == 64 || D == 128 || D == 256, "bottleneck_pair: D must be 64, 128 or 256 (got %d)", D);
    KINET_CHECK_ARG(F == 4 * D, "bottleneck_pair: F must be 4 * D (got D=%d F=%d)", D, F);
    KINET_CHECK_ARG(DB == D || (D == 64 && DB == 128), "bottleneck_pair: DB must be D, or 128 at D = 64 (got D=%d DB=%d)", D, DB);
    KINET_CHECK_ARG(M >= 0 && ldx >= D && ldx % 8 == 0, "bottleneck_pair: bad M / ldx");
    KINET_CHECK_ARG(dtype == KINET_BF16 || dtype == KINET_F16, "bottleneck_pair: dtype must be bf16 or f16");
    KINET_CHECK_ARG(b3 && b1, "bottleneck_pair: folded BN biases of both convs are required");
    KINET_CHECK_ARG(al16(X) && al16(R) && al16(packed) && al16(Y) && al16(T) && al16(b3) && al16(b1),
                    "bottleneck_pair: tensors and BN biases must be 16-byte aligned");
    if (M == 0) return KINET_OK;
    const long long xb = ((long long)(M - 1) * ldx + D) * 2, fb = (long long)M * F * 2;
    KINET_CHECK_ARG(xb < (1LL << 31) && fb < (1LL << 31), "bottleneck_pair: tensors larger than 2 GiB (split the call)");
    PairArgs a{};
    a.X = X; a.R = R; a.W = packed; a.b3 = b3; a.b1 = b1; a.Y = Y; a.T = T;
    a.ldx = ldx; a.M = M; a.F = F;
    a.x_bytes = (int)xb;
    a.r_bytes = (int)fb;
    a.y_bytes = (int)fb;
    a.w_bytes = (int)((long long)(D + DB) * F * 2);
    a.t_bytes = (int)((long long)M * DB * 2);
    hipStream_t s = (hipStream_t)stream;
    const int rc = dtype == KINET_BF16 ? launch_pair<bf16_t>(a, D, DB, s) : launch_pair<f16_t>(a, D, DB, s);
    if (rc) return rc;
    KINET_LAUNCH_CHECK();
    return KINET_OK;
}
