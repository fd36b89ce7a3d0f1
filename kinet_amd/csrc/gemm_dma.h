// LDS-DMA staged variant of gemm.hip's gemm_kernel (included by gemm.hip after gemm_kernel,
// inside its anonymous namespace; uses ResRows / epilogue_rows from there).
//
// rocprofv3 on the register-staged kernel (3x3 conv, batch 8): SQ_WAIT_INST_LDS 21 % of wave
// cycles, MFMA busy 21 % -- the ds_write_b128 staging pass (13 cycles per wave-instruction)
// costs more LDS time per K-step than the MFMAs take.  Here the DMA writes LDS directly:
//  * one wave-instruction fills 8 consecutive 128-byte tile rows (1 KiB, lane-linear); the
//    XOR swizzle that compute() reads with is applied on the SOURCE side (lane l of a row
//    group loads logical chunk (l & 7) ^ (row & 7));
//  * a 3-slot ring: K-step kt+2 is issued right after the barrier of step kt into the slot
//    step kt-1 used; a counted `s_waitcnt vmcnt` (one step's DMA count) retires step kt while
//    kt+1 stays in flight across the raw s_barrier; the loop holds no VGPR-destination load,
//    so hipcc adds no vmcnt(0) of its own;
//  * steps past K are issued too (range check -> zeros): no conditional DMA, exact counts;
//  * 4 waves (64x128-class tiles, 2 workgroups per CU) or 8 waves (256x128 / 128x256 tiles,
//    64x64 per wave, one workgroup per CU: 3 x 48 KiB ring, the 256x132 f32 epilogue tile
//    reuses it; 256x256, 128x64 per wave: 2 x 64 KiB ring, epilogue in two row halves) --
//    the 8-wave tiles halve the LDS fragment reads per MFMA of the 4-wave 64x128 tile and
//    the L2 -> LDS bytes per flop.
#pragma once

template <int BM, int BN, int NS_>
struct DmaSmem {
    static constexpr int STAGE = (BM + BN) * ROWB;
    static constexpr int NS = NS_;
    static constexpr int EPI_LD = BN + 4;
    // the f32 epilogue tile is parked whole, or in two row halves when the whole tile would
    // not fit beside the ring (256x256)
    static constexpr int EPI_ROWS = (BM * EPI_LD * 4 <= NS * STAGE || BM * EPI_LD * 4 <= 160 * 1024) ? BM : BM / 2;
    static constexpr int EPI = EPI_ROWS * EPI_LD * 4;
    static constexpr int BYTES = (NS * STAGE > EPI) ? NS * STAGE : EPI;
};

template <int N>
__device__ __forceinline__ void gemm_wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void gemm_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <typename T, typename TO, int BM, int BN, int WGM, int WGN, bool CONV, bool LN, int NS_ = 3>
__global__ __launch_bounds__(64 * WGM * WGN, WGM * WGN == 4 ? 2 : 1) void gemm_dma_kernel(const GemmArgs p,
                                                                                        const int nNt) {
    constexpr int NW = WGM * WGN;
    static_assert(NW == 4 || NW == 8, "4 or 8 waves");
    constexpr int EPC = Mma<T>::EPC;
    constexpr int BK = ROWB / (int)sizeof(T);
    constexpr int WTM = BM / WGM, WTN = BN / WGN;   // wave tile
    constexpr int TM = WTM / 16, TN = WTN / 16;
    using SM = DmaSmem<BM, BN, NS_>;
    constexpr int STAGE = SM::STAGE;
    constexpr int NS = SM::NS;
    constexpr int EPI_LD = SM::EPI_LD;
    constexpr int EROWS = SM::EPI_ROWS;
    static_assert(NS == 2 || NS == 3, "ring of 2 or 3 slots");
    static_assert(EROWS % WTM == 0, "a wave's rows must lie in one epilogue part");
    constexpr int XS = BM / (8 * NW), WS = BN / (8 * NW);   // DMA wave-instructions per wave per K-step
    constexpr int SLOTS = XS + WS;
    static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "whole 8-row groups per wave");
    __shared__ __attribute__((aligned(16))) char lds[SM::BYTES];

    int bid = blockIdx.x;
    {
        const int nblk = gridDim.x, q = nblk >> 3, r = nblk & 7, xcd = bid & 7;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    }
    const int mt = bid / nNt, nt = bid - (bid / nNt) * nNt;
    const int m0 = p.m_begin + mt * BM, n0 = nt * BN;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % WGM, wn = wave / WGM;
    const int M = p.M, N = p.N;
    const int kbeg = p.kchunk ? (int)blockIdx.y * p.kchunk : 0;
    const int K = p.kchunk ? min(p.K, kbeg + p.kchunk) : p.K;

    constexpr unsigned OOB = 0x80000000u;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.b_bytes, 0x00020000);

    // this lane's staging rows: A row-group wave + NW*i (i < XS), B row-group wave + NW*i (i < WS),
    // row (lane >> 3) of the group, logical 16-byte chunk sch of the row
    const int rsub = lane >> 3;
    const int sch = (lane & 7) ^ rsub;            // (row & 7) == rsub: groups are 8-row aligned
    unsigned xbase[XS];
    int xih[XS], xiw[XS];
    bool xok[XS];
#pragma unroll
    for (int i = 0; i < XS; ++i) {
        const int m = m0 + (wave + NW * i) * 8 + rsub;
        xok[i] = m < M;
        if (CONV) {
            const int hw = p.Hout * p.Wout;
            const int img = m / hw;
            const int rem = m - img * hw;
            const int oh = rem / p.Wout, ow = rem - (rem / p.Wout) * p.Wout;
            xih[i] = oh * p.stride - p.pad;
            xiw[i] = ow * p.stride_w - p.pad_w;
            // element offset of the receptive field's (0, 0) tap (used only behind the bounds test)
            xbase[i] = (unsigned)img * (unsigned)(p.Hin * p.Win * p.Cin) +
                       (unsigned)((xih[i] * p.Win + xiw[i]) * p.Cin);
        } else {
            xih[i] = xiw[i] = 0;
            xbase[i] = (unsigned)m * (unsigned)p.lda;
        }
    }
    unsigned wbase[WS];
    bool wok[WS];
#pragma unroll
    for (int i = 0; i < WS; ++i) {
        const int n = n0 + (wave + NW * i) * 8 + rsub;
        wok[i] = n < N;
        wbase[i] = (unsigned)n * (unsigned)p.ldb;
    }
    const bool tap_uniform = CONV && (p.Cin % BK) == 0;
    const int nk = (K - kbeg + BK - 1) / BK;
    // channel-chunk-major, tap-minor K-step order (gemm_kernel's kmap)
    const int ntaps = CONV ? p.K / p.Cin : 1;
    const bool korder = tap_uniform && p.kchunk == 0 && ntaps > 1;
    const int nchunk = p.Cin / BK;
    auto kmap = [&](int kt) -> int {
        if (!korder || kt >= nk) return kt * BK;
        const int c = kt / ntaps, t = kt - c * ntaps;
        return (t * nchunk + c) * BK;
    };

    // DMA of K-step kt into ring slot kt % NS (offsets with bit 31 set read zeros)
    auto stage = [&](int kt) {
        char* st = lds + (kt % NS) * STAGE;
        const int k0 = kbeg + kmap(kt);
        const int k = k0 + sch * EPC;
        const unsigned kbad = k < K ? 0u : OOB;
        int kh = 0, kw = 0, dk = 0;
        if (CONV) {
            if (tap_uniform) {
                const int ks0 = __builtin_amdgcn_readfirstlane(k0);
                const int tap = ks0 / p.Cin;
                kh = tap / p.KW;
                kw = tap - kh * p.KW;
                dk = __builtin_amdgcn_readfirstlane((kh * p.Win + kw) * p.Cin + ks0 - tap * p.Cin) + sch * EPC;
            } else {
                const int tap = k / p.Cin;
                kh = tap / p.KW;
                kw = tap - kh * p.KW;
                dk = (kh * p.Win + kw) * p.Cin + k - tap * p.Cin;
            }
        }
#pragma unroll
        for (int i = 0; i < XS; ++i) {
            unsigned off, bad = kbad | (xok[i] ? 0u : OOB);
            if (CONV) {
                const bool in = (unsigned)(xih[i] + kh) < (unsigned)p.Hin && (unsigned)(xiw[i] + kw) < (unsigned)p.Win;
                bad |= in ? 0u : OOB;
                off = xbase[i] + (unsigned)dk;
            } else {
                off = xbase[i] + (unsigned)k;
            }
            dma16(ra, st + (wave + NW * i) * 8 * ROWB, (off * (unsigned)sizeof(T)) | bad);
        }
#pragma unroll
        for (int i = 0; i < WS; ++i)
            dma16(rb, st + (BM + (wave + NW * i) * 8) * ROWB,
                  ((wbase[i] + (unsigned)k) * (unsigned)sizeof(T)) | kbad | (wok[i] ? 0u : OOB));
    };

    f32x4 acc[TN][TM];
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    // The K-step's two 32-deep halves: the second half's fragments are read while the first
    // half's MFMAs run -- its TN weight fragments right at the start, its TM activation fragments
    // one by one as the first half retires each activation fragment (row-fragment-outer MFMA
    // order) -- so only the K-step's first reads wait out an LDS round trip.  Scheduling barriers
    // keep the compiler from sinking the reads back next to their uses.  Same MFMAs per
    // accumulator in the same order (bit-identical).  256x256 tiles: within noise (two waves
    // per SIMD already cover it); 256x128 / 128x256: 4-8 % faster (profiles/r06ai_gemm_dma_prefetch_ab.txt)
    auto compute = [&](int slot) {
        const char* xl = lds + slot * STAGE;
        const char* wl = xl + BM * ROWB;
        auto xfrag = [&](int kk, int t) {
            return Mma<T>::frag(*reinterpret_cast<const u32x4*>(xl + swz(wm * WTM + t * 16 + (lane & 15), kk * 4 + (lane >> 4))));
        };
        auto wfrag = [&](int kk, int t) {
            return Mma<T>::frag(*reinterpret_cast<const u32x4*>(wl + swz(wn * WTN + t * 16 + (lane & 15), kk * 4 + (lane >> 4))));
        };
        typename Mma<T>::Frag bfr[2][TM], afr[2][TN];
#pragma unroll
        for (int t = 0; t < TN; ++t) afr[0][t] = wfrag(0, t);
#pragma unroll
        for (int t = 0; t < TM; ++t) bfr[0][t] = xfrag(0, t);
#pragma unroll
        for (int t = 0; t < TN; ++t) afr[1][t] = wfrag(1, t);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int b = 0; b < TM; ++b) {
#pragma unroll
                for (int a = 0; a < TN; ++a) Mma<T>::run(acc[a][b], afr[kk][a], bfr[kk][b]);
                if (kk == 0) bfr[1][b] = xfrag(1, b);
                __builtin_amdgcn_sched_barrier(0);
            }
    };

    stage(0);
    if (NS == 3) stage(1);
    for (int kt = 0; kt < nk; ++kt) {
        gemm_wait_vmcnt<(NS - 2) * SLOTS>();   // this wave's step-kt DMA landed (kt+1 may fly)
        gemm_lds_barrier();                    // everyone's landed; everyone done with step kt-1's slot
        stage(kt + NS - 1);
        compute(kt % NS);
    }
    gemm_wait_vmcnt<0>();              // the zero-filled steps past the end
    gemm_lds_barrier();

    // ---- epilogue: residual rows in flight, park the f32 tile (or one row half of it) in
    // LDS, stream whole rows ----
    float* ep = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int h = 0; h < BM / EROWS; ++h) {
        ResRows<TO, BN, NW, EROWS> rp;
        rp.issue(p, m0, n0, h * EROWS, wave, lane);
        if (h) __syncthreads();
        if ((wm * WTM) / EROWS == h) {
#pragma unroll
            for (int a = 0; a < TN; ++a)
#pragma unroll
                for (int b = 0; b < TM; ++b) {
                    const int ml = wm * WTM - h * EROWS + b * 16 + (lane & 15);
                    const int nl = wn * WTN + a * 16 + (lane >> 4) * 4;
                    *reinterpret_cast<f32x4*>(ep + ml * EPI_LD + nl) = acc[a][b];
                }
        }
        __syncthreads();
        epilogue_rows<TO, BN, EPI_LD, NW, LN, EROWS>(p, ep, m0, n0, h * EROWS, wave, lane, rp);
    }
}
