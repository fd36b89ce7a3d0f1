// Stream-K scheduling of the 8-wave LDS-DMA GEMM / implicit-conv tiles (included by gemm.hip
// after gemm_dma.h, inside its anonymous namespace).
//
// Why: the 8-wave tiles run one workgroup per CU, so a launch of T tiles takes ceil(T / 256)
// full tile times -- 263 tiles of a layer-3 3x3 conv at batch 16 cost 2 rounds for 1.03
// rounds of work.  Here the grid is one workgroup per CU and the T x nk (tile, K-step)
// iterations are cut into equal contiguous ranges, one per workgroup (tile-major, K-minor):
//  * a workgroup's range is [tail of tile t0][whole tiles ...][head of tile t1];
//  * the TAIL segment (K-steps k0 > 0 .. nk) is always the first thing a workgroup computes:
//    it writes its f32 tile (parked in LDS, row-major) to its own workspace slot, then
//    releases flags[wg] = epoch (agent scope);
//  * the HEAD owner (K-steps 0 .. k1) is the tile's finisher: at the end of its range it
//    acquires the flags of the following workgroups covering the tile (set long before: they
//    did that segment first), adds their partials in workgroup order -- a fixed order, so the
//    result is deterministic -- and runs the fused epilogue;
//  * no workgroup waits before it has produced its own partial, so the waits form no cycle;
//    every spin is bounded.
// The epoch (one per launch on a stream's workspace) makes flags self-resetting.
#pragma once

template <typename T, typename TO, int BM, int BN, int WGM, int WGN, bool CONV, int NS>
__global__ __launch_bounds__(512, 1) void gemm_sk_kernel(const GemmArgs p, const int nNt, const int nTiles,
                                                        const int iters_per_wg, float* __restrict__ part,
                                                        unsigned* __restrict__ flags, const unsigned epoch) {
    constexpr int NW = WGM * WGN;
    static_assert(NW == 8, "8 waves");
    constexpr int EPC = Mma<T>::EPC;
    constexpr int BK = ROWB / (int)sizeof(T);
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    using SM = DmaSmem<BM, BN, NS>;
    constexpr int STAGE = SM::STAGE;
    constexpr int EPI_LD = SM::EPI_LD;
    constexpr int EROWS = SM::EPI_ROWS;
    constexpr int XS = BM / (8 * NW), WS = BN / (8 * NW);
    constexpr int SLOTS = XS + WS;
    static_assert(NS == 2 || NS == 3, "ring of 2 or 3 slots");
    static_assert(EROWS % WTM == 0, "a wave's rows must lie in one epilogue part");
    __shared__ __attribute__((aligned(16))) char lds[SM::BYTES];

    int v = blockIdx.x;   // virtual workgroup index: consecutive ranges on one XCD
    {
        const int nblk = gridDim.x, q = nblk >> 3, r = nblk & 7, xcd = v & 7;
        v = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (v >> 3);
    }
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % WGM, wn = wave / WGM;
    const int M = p.M, N = p.N, K = p.K;
    const int nk = (K + BK - 1) / BK;

    constexpr unsigned OOB = 0x80000000u;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.b_bytes, 0x00020000);
    const bool tap_uniform = CONV && (p.Cin % BK) == 0;
    const int ntaps = CONV ? p.K / p.Cin : 1;
    const bool korder = tap_uniform && ntaps > 1;   // gemm_kernel's channel-chunk-major K order
    const int nchunk = p.Cin / BK;
    auto kmap = [&](int kt) -> int {
        if (!korder || kt >= nk) return kt * BK;
        const int c = kt / ntaps, t = kt - c * ntaps;
        return (t * nchunk + c) * BK;
    };
    const int rsub = lane >> 3;
    const int sch = (lane & 7) ^ rsub;

    unsigned xbase[XS];
    int xih[XS], xiw[XS];
    bool xok[XS];
    unsigned wbase[WS];
    bool wok[WS];
    int m0 = 0, n0 = 0;
    auto setup = [&](int tile) {
        const int mt = tile / nNt, nt = tile - (tile / nNt) * nNt;
        m0 = mt * BM;
        n0 = nt * BN;
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
                xbase[i] = (unsigned)img * (unsigned)(p.Hin * p.Win * p.Cin) +
                           (unsigned)((xih[i] * p.Win + xiw[i]) * p.Cin);
            } else {
                xih[i] = xiw[i] = 0;
                xbase[i] = (unsigned)m * (unsigned)p.lda;
            }
        }
#pragma unroll
        for (int i = 0; i < WS; ++i) {
            const int n = n0 + (wave + NW * i) * 8 + rsub;
            wok[i] = n < N;
            wbase[i] = (unsigned)n * (unsigned)p.ldb;
        }
    };

    // DMA of K-step kt into ring slot kt % NS; `live` false -> zeros (no traffic), so every
    // segment issues exactly NS-1 steps ahead and the vmcnt counts stay exact
    auto stage = [&](int kt, bool live) {
        char* st = lds + (kt % NS) * STAGE;
        const int k0 = kmap(kt);
        const int k = k0 + sch * EPC;
        const unsigned kbad = (live && k < K) ? 0u : OOB;
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
    auto compute = [&](int slot) {
        const char* xl = lds + slot * STAGE;
        const char* wl = xl + BM * ROWB;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = kk * 4 + (lane >> 4);
            u32x4 bfr[TM], afr[TN];
#pragma unroll
            for (int t = 0; t < TM; ++t)
                bfr[t] = *reinterpret_cast<const u32x4*>(xl + swz(wm * WTM + t * 16 + (lane & 15), ch));
#pragma unroll
            for (int t = 0; t < TN; ++t)
                afr[t] = *reinterpret_cast<const u32x4*>(wl + swz(wn * WTN + t * 16 + (lane & 15), ch));
#pragma unroll
            for (int a = 0; a < TN; ++a)
#pragma unroll
                for (int b = 0; b < TM; ++b) Mma<T>::run(acc[a][b], afr[a], bfr[b]);
        }
    };

    const long total = (long)nTiles * nk;
    long it = (long)v * iters_per_wg;
    const long end = it + iters_per_wg < total ? it + iters_per_wg : total;
    while (it < end) {
        const int t = (int)(it / nk);
        const int k0 = (int)(it - (long)t * nk);
        const int k1 = (long)nk < k0 + (end - it) ? nk : (int)(k0 + (end - it));
        setup(t);
#pragma unroll
        for (int a = 0; a < TN; ++a)
#pragma unroll
            for (int b = 0; b < TM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
        __syncthreads();   // the previous tile's epilogue is done with the LDS
        stage(k0, true);
        if (NS == 3) stage(k0 + 1, k0 + 1 < k1);
        for (int kt = k0; kt < k1; ++kt) {
            gemm_wait_vmcnt<(NS - 2) * SLOTS>();
            gemm_lds_barrier();
            stage(kt + NS - 1, kt + NS - 1 < k1);
            compute(kt % NS);
        }
        gemm_wait_vmcnt<0>();
        gemm_lds_barrier();

        // Both kinds of segment park the f32 tile in LDS first (the accumulators die there, so the
        // hand-off code below holds no accumulator registers), one row part at a time:
        //  * tail segment: copy the part to this workgroup's workspace slot (row-major f32,
        //    coalesced), then publish the flag;
        //  * head segment: acquire the following workgroups' flags, add their parts into LDS in
        //    workgroup order, then the fused epilogue.
        const bool head = k0 == 0;
        const int nprod = head ? (int)(((long)(t + 1) * nk - 1) / iters_per_wg) - v : 0;   // partial producers
        if (nprod > 0) {
            if (tid == 0) {
                for (int w = v + 1; w <= v + nprod; ++w) {
                    for (int spin = 0; spin < (1 << 24); ++spin) {
                        if (__hip_atomic_load(flags + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) break;
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                // ONE lane polls relaxed (bounded), then one agent-scope acquire and a drain;
                // the barrier below orders every wave's plain loads after it
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        float* ep = reinterpret_cast<float*>(lds);
#pragma unroll
        for (int h = 0; h < BM / EROWS; ++h) {
            ResRows<TO, BN, NW, EROWS> rp;
            if (head) rp.issue(p, m0, n0, h * EROWS, wave, lane);
            else rp.on = false;
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
            constexpr int Q = BN / 4;   // f32x4 per tile row
            if (!head) {
                f32x4* dst = reinterpret_cast<f32x4*>(part + ((size_t)v * BM + h * EROWS) * BN);
                for (int i = tid; i < EROWS * Q; i += 64 * NW) {
                    const int r = i / Q, c = (i - r * Q) * 4;
                    dst[i] = *reinterpret_cast<const f32x4*>(ep + r * EPI_LD + c);
                }
            } else {
                for (int w = v + 1; w <= v + nprod; ++w) {
                    const f32x4* src = reinterpret_cast<const f32x4*>(part + ((size_t)w * BM + h * EROWS) * BN);
                    for (int i = tid; i < EROWS * Q; i += 64 * NW) {
                        const int r = i / Q, c = (i - r * Q) * 4;
                        *reinterpret_cast<f32x4*>(ep + r * EPI_LD + c) += src[i];
                    }
                }
                if (nprod > 0) __syncthreads();
                epilogue_rows<TO, BN, EPI_LD, NW, false, EROWS>(p, ep, m0, n0, h * EROWS, wave, lane, rp);
            }
        }
        if (!head) {
            // cdna_hip_programming.md Guideline 16 / the in-launch split-K recipe: every storing
            // wave drains, barrier, ONE lane's agent-scope release, drain again, flag
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(flags + v, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        it += k1 - k0;
    }
}
