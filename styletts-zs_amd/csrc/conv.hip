// The universal MFMA conv1d / linear of the hot path.
//
// Implicit GEMM on gfx950 matrix cores: M = output time rows, N = output channels, K = taps x
// input channels.  One 256-thread workgroup (4 waves as 2x2) owns a 128 x 128 output tile; each
// wave a 64 x 64 sub-tile = 4 x 4 accumulators of v_mfma_f32_16x16x32_bf16 (bf16 operands, fp32
// accumulate).  Two workgroups fit per CU (<= 80 KB LDS each), so one's staging/epilogue VALU
// overlaps the other's MFMAs.
//
//  * INPUT: per input-channel chunk (cic = 32|64|128) the tile's rows INCLUDING the dilation halo
//    are staged ONCE into LDS through registers, with the AdaIN/cscale prologue and the
//    activation (LeakyReLU / Snake with the hardware v_sin) applied on the way in.  Rows use a
//    16-B padded pitch (conflict-light ds_read_b128 for the A fragments).  Every tap re-reads that
//    tile at row offset tap*dil: the halo is fetched once, no separate norm/activation pass exists.
//  * WEIGHTS: pre-packed per 128-column tile as a stream of K-steps, each [128 co][32 ci] bf16 =
//    8 KB, already XOR-swizzled into the LDS image order (stzs/weights.py) so that a lane-linear
//    LDS-DMA copy (global_load_lds_dwordx4, 1 KB per wave instruction) lands a conflict-free
//    B-fragment layout.  A 3-slot ring keeps two K-steps in flight: counted s_waitcnt vmcnt + one
//    raw s_barrier per K-step, never a vmcnt(0) drain inside the K loop.
//  * EPILOGUE: accumulators go through LDS (fp32, padded rows) and leave as 16-B vectors per lane:
//    bias, activation, DiT gate, residual (optionally at t/res_tdiv = nearest-x2 shortcut), scale,
//    fp32/bf16 accumulate-input (MRF sum, EDM c_skip*x), the polyphase ConvTranspose1d scatter and
//    ReflectionPad(1,0) when ups > 0.
#include "conv_common.hpp"

int stzs_gemm_glds_launch(const stzs_conv_args& a, hipStream_t s);   // csrc/gemm.hip
int stzs_conv_x3_launch(const stzs_conv_args* a, hipStream_t s);     // csrc/convx.hip
int stzs_conv_f32_launch(const stzs_conv_args* a, hipStream_t s);    // csrc/convx.hip

namespace {

// DEEP (r05, the batch-1 split-K launches, one input-channel chunk per slice): every weight K-step of the slice is
// issued into its own LDS slot at entry, beside the staging loads, so the slice pays ONE memory latency and its K loop
// runs from LDS with no wait and no barrier (the 3-slot ring waited a fill latency every other K-step: ~0.37 us per
// K-step at batch 1).  Same K order, same combine: bit-identical to the ring form at the same slice count.
// SKE (with DEEP): the slice stores its fp32 partial tile row-major into its slab and ends; the combine and the fused
// epilogue run in splitk_epi, a second launch spread over 8 workgroups per tile (the last-arriver combine read every
// other slice's 64-KB slab through ONE workgroup: 7.5 us of a 24-us batch-1 decoder conv, tools/conv_phase.py).
// (r06) the body as an always-inlined device function of (arguments by value, split-K slice zs): conv_mfma is this
// body with zs = grid z, conv_mfma_pair two problems' bodies in one launch.
template <typename TIn, typename TOut, bool FLAT, int PACT, bool DEEP = false, bool SKE = false>
STZS_DEV void conv_body(const stzs_conv_args a, const int zs) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int cic = a.cic;
    const int pitch = cic * 2 + 16;
    const int ks = FLAT ? 1 : a.ks;
    const int rows_in = FLAT ? BT : (BT - 1) * a.stride + (ks - 1) * a.dil + 1;
    unsigned char* in_lds = smem;
    unsigned char* ring = smem + ((rows_in * pitch + 15) & ~15);
    const int nslot = DEEP ? (FLAT ? 1 : a.ks) * (cic >> 5) : NSLOT;
    float* c_sc = reinterpret_cast<float*>(ring + nslot * SLOT_BYTES);
    float* c_sh = c_sc + 128;
    float* c_al = c_sh + 128;
    float* c_ia = c_al + 128;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = wave >> 1, wc = wave & 1;
    // XCD-aware tile order (as gemm_glds): each XCD runs a contiguous range of tiles, output-channel tile fastest,
    // so the workgroups one XCD holds at a time share their staged input rows (one fabric fetch per XCD instead
    // of one per channel tile).  Same tiles, same K order: bit-identical to the linear order.
    const int gy = gridDim.y;
    const bool lin_ids = (a.flags & STZS_CONV_LINEAR_IDS) != 0;
    const int lin = lin_ids ? 0 : xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gy);
    const int by = lin_ids ? (int)blockIdx.y : lin % gy;
    const int bx = lin_ids ? (int)blockIdx.x : lin / gy;
    int bq = 0, t0 = 0;
    long row0 = 0;
    if (FLAT) {
        row0 = (long)bx * BT;
    } else {
        const int tpb = (a.T_out + BT - 1) / BT;
        bq = bx / tpb;
        t0 = (bx - bq * tpb) * BT;
    }
    const int nchunk = a.ci_pad / cic;
    const int kpc = cic >> 5;
    const int NK = nchunk * ks * kpc;
    const bf16_t* Wt = reinterpret_cast<const bf16_t*>(a.w) + (long)by * NK * (BCO * 32);
    // in-launch split-K over input-channel chunks (stzs_conv_args.splitk, grid.z slices): slice z stages and runs
    // chunks [cc_lo, cc_hi) -- K-steps [k_lo, k_hi) of the chunk-major weight stream -- and hands its fp32 partial
    // to the tile's last arriver (splitk_combine_rt), which runs the fused epilogue.  For the small grids of the
    // batch-1 front end (text-encoder k5 convs: 4 workgroups x 80 K-steps at batch 1).
    // Slice z takes chunks [z n / S, (z+1) n / S): equal slices when S divides n, otherwise sizes differing by one
    // (the decoder / predictor AdaIN convs of the batch-1 engine: 9 chunks in 3 or 4 slices)
    const int SKr = a.splitk > 1 ? a.splitk : 1;
    const int cc_lo = SKr > 1 ? zs * nchunk / SKr : 0;
    const int cc_hi = SKr > 1 ? (zs + 1) * nchunk / SKr : nchunk;
    const int k_lo = cc_lo * ks * kpc, k_hi = cc_hi * ks * kpc;

    auto fill = [&](int k) {
        const bf16_t* src = Wt + (long)k * (BCO * 32) + wave * 1024 + lane * 8;
        unsigned char* dst = ring + (DEEP ? k - k_lo : k % NSLOT) * SLOT_BYTES + wave * 2048;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 512),
                                         (__attribute__((address_space(3))) void*)(dst + 1024), 16, 0, 0);
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const TIn* X = reinterpret_cast<const TIn*>(a.x);
    const int vpr = cic >> 3;
    const int rstr = FLAT ? 1 : a.stride;
    // B-fragment LDS byte offsets inside a slot (fixed per lane): row rr, chunk (lane>>4) swizzled
    int boff[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int rr = wc * 64 + nt * 16 + (lane & 15);
        boff[nt] = rr * 64 + (((lane >> 4) ^ gswz(rr)) << 4);
    }

    CPROF_RT(15)
    CPROF(0)
    if constexpr (DEEP) {
        for (int kk = k_lo; kk < k_hi; ++kk) fill(kk);  // the whole slice (one chunk): ks x cic / 32 slots
    } else {
        fill(k_lo);
        if (k_lo + 1 < k_hi) fill(k_lo + 1);
    }
    int k = k_lo;
    for (int cc = cc_lo; cc < cc_hi; ++cc) {
        __syncthreads();
        const int nv = (a.flags & 1) ? 0 : rows_in * vpr;
        // Staging: ONE batch of SB independent 16-B loads per thread (every MRF tile fits), issued
        // BEFORE the per-chunk coefficient loads so both latencies overlap in the same wait.  Loads are
        // UNCONDITIONAL from clamped (always valid) addresses and masked afterwards (a runtime-
        // conditioned load makes hipcc drain vmcnt(0) per element).  vpr = cic/8 is a power of two
        // dividing NTHR, so a thread's channel vector cv is the same for every row it stages.
        constexpr int SB = sizeof(TIn) == 2 ? 12 : 4;
        using RawT = typename Raw<TIn>::T;
        const int lv = cic == 128 ? 4 : (cic == 64 ? 3 : 2);
        const int cv = tid & (vpr - 1);
        const int ci = cc * cic + cv * 8;
        const bool ci_ok = ci < a.Ci;
        const int cic0 = ci_ok ? ci : 0;
        const int rstep = NTHR >> lv;
        RawT raw[SB];
        bool okv[SB];
        const float invTi = 1.f / (float)a.T_in;  // (FLAT rows -> utterance, rowdiv)
        auto issue = [&](int v0) {
            const int rb = (v0 >> lv) + (tid >> lv);
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                const int r = rb + i * rstep;
                bool ok = ci_ok && r < rows_in;
                long off;
                if (FLAT) {
                    long R = row0 + r;
                    const long nR = (long)a.B * a.T_in;
                    ok = ok && R < nR;
                    R = R < nR ? R : nR - 1;
                    const long bb = rowdiv(R, a.T_in, invTi, nR < (1L << 22));
                    off = bb * a.bsx + (R - bb * a.T_in) * a.ldx + cic0;
                } else {
                    int tin = t0 * a.stride - a.pad + r;
                    ok = ok && tin >= 0 && tin < a.T_in;
                    tin = tin < 0 ? 0 : (tin >= a.T_in ? a.T_in - 1 : tin);
                    off = (long)bq * a.bsx + (long)tin * a.ldx + cic0;
                }
                okv[i] = ok;
                raw[i] = Raw<TIn>::load(X + off);
            }
        };
        if (nv > 0) issue(0);
        if (tid < cic) {
            const int cg = cc * cic + tid;
            float sc = 0.f, sh = 0.f, al = 1.f;
            if (cg < a.Ci) {
                if (a.pro_mode == STZS_PRO_ADAIN) {
                    float mu, rs;
                    if (a.pro_part) {  // statistics from the partials (stzs_conv_args.pro_part: <= 8 chunks)
                        const float2* Pp = reinterpret_cast<const float2*>(a.pro_part) + (long)bq * a.pro_nch * a.pro_ld + cg;
                        float2 pv[8];
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            if (k < a.pro_nch) pv[k] = Pp[(long)k * a.pro_ld];
                        double ssum = 0.0, qsum = 0.0;  // chunk order, as stzs_chan_stats_final's groups
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            if (k < a.pro_nch) {
                                ssum += (double)pv[k].x;
                                qsum += (double)pv[k].y;
                            }
                        stat_finish(ssum, qsum, a.pro_T, a.pro_eps, mu, rs);
                    } else {
                        mu = a.pro_mean[(long)bq * a.stat_bs + cg];
                        rs = a.pro_rstd[(long)bq * a.stat_bs + cg];
                    }
                    const float g = a.pro_gb[(long)bq * a.gb_bs + cg];
                    const float be = a.pro_gb[(long)bq * a.gb_bs + a.gb_beta_off + cg];
                    sc = (1.f + g) * rs;
                    sh = be - mu * sc;
                } else {
                    sc = a.pro_cscale;
                }
                if (a.pro_alpha) al = a.pro_alpha[cg];
            }
            c_sc[tid] = sc;
            c_sh[tid] = sh;
            c_al[tid] = al;
            c_ia[tid] = 1.f / al;
        }
        __syncthreads();
        float k_sc[8], k_sh[8], k_al[8], k_ia[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            k_sc[j] = c_sc[cv * 8 + j];
            k_sh[j] = c_sh[cv * 8 + j];
            k_al[j] = c_al[cv * 8 + j];
            k_ia[j] = c_ia[cv * 8 + j];
        }
        for (int v0 = 0; v0 < nv; v0 += SB * NTHR) {
            if (v0 > 0) issue(v0);
            const int rb = (v0 >> lv) + (tid >> lv);
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                const int r = rb + i * rstep;
                if (r >= rows_in) break;
                float f[8], o[8];
                Raw<TIn>::cvt(raw[i], f);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float y = pro_act<PACT>(f[j] * k_sc[j] + k_sh[j], a.pro_slope, k_al[j], k_ia[j]);
                    o[j] = okv[i] ? y : 0.f;
                }
                *reinterpret_cast<uint4*>(in_lds + r * pitch + cv * 16) = pack8(o);
            }
        }
        if constexpr (DEEP) waitcnt_vm(0);  // this wave's weight slots landed (the barrier publishes every wave's)
        __syncthreads();
        if (cc == cc_lo) { CPROF(1) }
        for (int tap = 0; tap < ((a.flags & 2) ? 0 : ks); ++tap) {
            const int roff = FLAT ? 0 : tap * a.dil;
            for (int kq = 0; kq < kpc; ++kq, ++k) {
                if constexpr (!DEEP) {
                    waitcnt_vm(k + 1 < k_hi ? 2 : 0);
                    __builtin_amdgcn_s_barrier();
                    if (k + 2 < k_hi) fill(k + 2);
                }
                const unsigned char* wl = ring + (DEEP ? k - k_lo : k % NSLOT) * SLOT_BYTES;
                const int kb = (kq * 32 + 8 * (lane >> 4)) * 2;
                bf16x8 af[4], bw[4];
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
                    const int r = (wt * 64 + mt * 16 + (lane & 15)) * rstr + roff;
                    af[mt] = *reinterpret_cast<const bf16x8*>(in_lds + r * pitch + kb);
                }
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) bw[nt] = *reinterpret_cast<const bf16x8*>(wl + boff[nt]);
                __builtin_amdgcn_sched_barrier(0);  // issue all 8 fragment reads before the first MFMA
#pragma unroll
                for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bw[nt], acc[mt][nt], 0, 0, 0);
            }
        }
    }

    CPROF(2)
    if constexpr (SKE) {
        // the partial tile through LDS (fp32, padded rows) to the slab [tile = by gx + bx][z][128 rows][128], valid rows only
        __syncthreads();  // every wave is past its K loop (staging / weight slots idle)
        float* ep = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    ep[(wt * 64 + mt * 16 + (lane >> 4) * 4 + r) * EP_PITCH + wc * 64 + nt * 16 + (lane & 15)] = acc[mt][nt][r];
        __syncthreads();
        const long tile = (long)by * gridDim.x + bx;
        float* slab = reinterpret_cast<float*>(a.splitk_ws) + (tile * SKr + zs) * (long)(BT * BCO);
        const long rows_left = FLAT ? (long)a.B * a.T_out - row0 : (long)(a.T_out - t0);
        const int nrow = rows_left < BT ? (int)rows_left : BT;
        for (int e = tid; e < nrow * (BCO / 4); e += NTHR) {
            const int r = e >> 5, v = e & 31;
            *reinterpret_cast<float4*>(slab + r * BCO + v * 4) = *reinterpret_cast<const float4*>(ep + r * EP_PITCH + v * 4);
        }
        CPROF(3)
        CPROF_RT(14)
        return;
    }
    if (SKr > 1 && !splitk_combine_rt<BT, DEEP ? 4 : 1>(a, acc, smem, SKr, zs)) {
        CPROF_RT(14)
        return;
    }
    CPROF(5)
    finish<TOut, FLAT>(a, acc, smem, bq, t0, row0, by);
    CPROF(6)
    CPROF_RT(14)
#ifdef STZS_CONV_PROF
    if (threadIdx.x == 0) {
        const unsigned wg_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        if (wg_ < 8192) g_cprof[wg_ * 16 + 13] = __builtin_amdgcn_s_getreg(0x14 | (3 << 11)) + 1;  // HW_REG_XCC_ID (+1)
    }
#endif
}

template <typename TIn, typename TOut, bool FLAT, int PACT, bool DEEP = false, bool SKE = false>
__global__ __launch_bounds__(NTHR, DEEP ? 1 : 2) void conv_mfma(const stzs_conv_args a) {
    conv_body<TIn, TOut, FLAT, PACT, DEEP, SKE>(a, blockIdx.z);
}

// (r06) two independent DEEP split-K convs of one shape (the prosody predictor's F0 and N branches at batch 1) in one
// launch: grid z < splitk runs problem 0's slice z, the rest problem 1's -- each workgroup the single-problem body, so
// every slab holds the bits of its own launch; splitk_epi_pair combines them.
template <typename TIn, typename TOut, int PACT>
__global__ __launch_bounds__(NTHR, 1) void conv_mfma_pair(const stzs_conv_args a0, const stzs_conv_args a1) {
    const int SK = a0.splitk;
    if ((int)blockIdx.z < SK)
        conv_body<TIn, TOut, false, PACT, true, true>(a0, blockIdx.z);
    else
        conv_body<TIn, TOut, false, PACT, true, true>(a1, (int)blockIdx.z - SK);
}

// splitk_combine with the slice count at run time (conv_mfma): the same slabs, ticket and slice-order sum, the
// slices loaded one at a time (no [SK][NV] register block).
template <int BTM, int RB>
STZS_DEV bool splitk_combine_rt(const stzs_conv_args& a, f32x4 (&acc)[BTM / 32][4], unsigned char* smem, int SK, int z) {
    constexpr int NV = BTM / 32 * 4;
    constexpr int SLAB = NV * NTHR * 16;
    const int tid = threadIdx.x;
    const long tile = blockIdx.x + (long)gridDim.x * blockIdx.y;
    unsigned char* base = reinterpret_cast<unsigned char*>(a.splitk_ws) + tile * (long)SK * SLAB;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(base, 0, SK * SLAB, 0x00020000);
#pragma unroll
    for (int i = 0; i < NV; ++i)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i >> 2][i & 3]), wr,
                                               (z * NV + i) * (NTHR * 16) + tid * 16, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    CPROF(3)
    volatile int* flag = reinterpret_cast<volatile int*>(smem);  // staging / ring idle: every wave is past its K loop
    if (tid == 0) {
        typedef __attribute__((address_space(1))) unsigned int gu32;
        gu32* ctr = (gu32*)(a.splitk_ctr + tile);
        const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == (unsigned)(SK - 1);
        if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
    }
    __syncthreads();
    CPROF(4)
    if (!*flag) return false;
#pragma unroll
    for (int i = 0; i < NV; ++i)
        acc[i >> 2][i & 3] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, i * (NTHR * 16) + tid * 16, 0, 16));
    // RB slices per round, all their loads in flight at once, summed in slice order (the same sum for every RB)
    for (int sl = 1; sl < SK; sl += RB) {
        u32x4 v[RB][NV];
#pragma unroll
        for (int j = 0; j < RB; ++j)
            if (sl + j < SK)
#pragma unroll
                for (int i = 0; i < NV; ++i)
                    v[j][i] = __builtin_amdgcn_raw_buffer_load_b128(wr, ((sl + j) * NV + i) * (NTHR * 16) + tid * 16, 0, 16);
#pragma unroll
        for (int j = 0; j < RB; ++j)
            if (sl + j < SK)
#pragma unroll
                for (int i = 0; i < NV; ++i) acc[i >> 2][i & 3] += __builtin_bit_cast(f32x4, v[j][i]);
    }
    return true;
}

// The split-K combine + fused epilogue of the SKE slices (a second launch): workgroup (bx, 8 by + cg) owns rows
// [0, 128) x columns [by 128 + 16 cg, +16) of tile (bx, by); thread (row = tid / 2, 8-column vector tid % 2) sums the
// SK slabs in slice order (the last-arriver combine's order: y is bit-identical to it), then bias, activation,
// conv-mode gate, residual (t / res_tdiv), alpha, beta * acc_in, the store, and the InstanceNorm partials of the
// stored values per 64-row half (one deterministic fp32 partial per (utterance, 64-row chunk, channel), reduced
// lanes -> waves in a fixed order).
template <typename TOut, bool FLAT>
STZS_DEV void splitk_epi_body(const stzs_conv_args a, const int SK) {
    __shared__ float red[4][2][8][2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int bx = blockIdx.x, by = blockIdx.y >> 3, cg = blockIdx.y & 7;
    const int rl = tid >> 1, cvl = tid & 1;
    int bq = 0, t0 = 0;
    long row0 = 0;
    if (FLAT) {
        row0 = (long)bx * BT;
    } else {
        const int tpb = (a.T_out + BT - 1) / BT;
        bq = bx / tpb;
        t0 = (bx - bq * tpb) * BT;
    }
    const int co = by * BCO + cg * 16 + cvl * 8;
    const bool col_ok = co < a.Co;
    const int cc = col_ok ? co : 0;
    long bb = bq, t = t0 + rl;
    bool ok = col_ok;
    if (FLAT) {
        const long R = row0 + rl;
        ok = ok && R < (long)a.B * a.T_out;
        bb = ok ? R / a.T_out : 0;
        t = ok ? R - bb * a.T_out : 0;
    } else {
        ok = ok && t < a.T_out;
    }
    const long tile = (long)by * gridDim.x + bx;
    const float* S = reinterpret_cast<const float*>(a.splitk_ws) + tile * SK * (long)(BT * BCO) + rl * BCO + cg * 16 + cvl * 8;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    float bias[8], gt[8], rr[8], ai[8];
    if (ok) {
        // residual / accumulate / bias / gate loads in flight with the slabs'
        const TOut* Rp = reinterpret_cast<const TOut*>(a.res);
        const TOut* AI = reinterpret_cast<const TOut*>(a.acc_in);
        if (a.res) {
            const long tr = a.res_tdiv == 1 ? t : (long)((int)t / a.res_tdiv);
            load8(Rp + bb * a.bsr + tr * a.ldr + cc, rr);
        }
        if (a.acc_in) load8(AI + bb * a.bsa + t * a.lda + cc, ai);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            bias[j] = a.bias ? a.bias[cc + j] : 0.f;
            gt[j] = (!FLAT && a.gate) ? a.gate[(long)bq * a.gate_bs + cc + j] : 1.f;
        }
        // slice 0, then slices 1.. in order, 4 slices' loads in flight per round
        float4 p0 = *reinterpret_cast<const float4*>(S), p1 = *reinterpret_cast<const float4*>(S + 4);
        v[0] = p0.x; v[1] = p0.y; v[2] = p0.z; v[3] = p0.w; v[4] = p1.x; v[5] = p1.y; v[6] = p1.z; v[7] = p1.w;
        for (int z = 1; z < SK; z += 4) {
            float4 q[4][2];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (z + i < SK) {
                    q[i][0] = *reinterpret_cast<const float4*>(S + (long)(z + i) * (BT * BCO));
                    q[i][1] = *reinterpret_cast<const float4*>(S + (long)(z + i) * (BT * BCO) + 4);
                }
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (z + i < SK) {
                    v[0] += q[i][0].x; v[1] += q[i][0].y; v[2] += q[i][0].z; v[3] += q[i][0].w;
                    v[4] += q[i][1].x; v[5] += q[i][1].y; v[6] += q[i][1].z; v[7] += q[i][1].w;
                }
        }
    }
    float st_s[8], st_q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) st_s[j] = st_q[j] = 0.f;
    if (ok) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float x;
            switch (a.epi_act) {  // (uniform)
                case STZS_ACT_GELU: x = epi_act<STZS_ACT_GELU>(v[j] + bias[j], a.epi_slope); break;
                case STZS_ACT_SILU: x = epi_act<STZS_ACT_SILU>(v[j] + bias[j], a.epi_slope); break;
                case STZS_ACT_LEAKY: x = epi_act<STZS_ACT_LEAKY>(v[j] + bias[j], a.epi_slope); break;
                default: x = v[j] + bias[j]; break;
            }
            if (!FLAT) x *= gt[j];
            if (a.res) x += rr[j];
            x *= a.alpha;
            if (a.acc_in) x += a.beta * ai[j];
            o[j] = x;
        }
        TOut* Y = reinterpret_cast<TOut*>(a.y) + bb * a.bsy + t * a.ldy + co;
        if constexpr (sizeof(TOut) == 2) {
            const uint4 pk = pack8(o);
            *reinterpret_cast<uint4*>(Y) = pk;
            unpack8(pk, o);  // statistics of the value as stored (bf16-rounded)
        } else {
            store8(Y, o);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            st_s[j] = o[j];
            st_q[j] = o[j] * o[j];
        }
    }
    if (FLAT || !a.stat_part) return;
    // rows of this wave: 32 per column vector (lane & 1); lanes -> wave partial, then the two waves of each 64-row half
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int m = 2; m < 64; m <<= 1) {
            st_s[j] += __shfl_xor(st_s[j], m, 64);
            st_q[j] += __shfl_xor(st_q[j], m, 64);
        }
    }
    if (lane < 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            red[wave][lane][j][0] = st_s[j];
            red[wave][lane][j][1] = st_q[j];
        }
    }
    __syncthreads();
    if (tid < 32) {
        const int half = tid >> 4, c16 = tid & 15, cv = c16 >> 3, j = c16 & 7;
        const int c = by * BCO + cg * 16 + c16;
        const int r0 = t0 + half * 64;
        if (c < a.Co && r0 < a.T_out) {
            const float ss = red[2 * half][cv][j][0] + red[2 * half + 1][cv][j][0];
            const float qq = red[2 * half][cv][j][1] + red[2 * half + 1][cv][j][1];
            const int nch = (a.T_out + 63) / 64;
            float* P = reinterpret_cast<float*>(a.stat_part) + (((long)bq * nch + r0 / 64) * a.stat_ld + c) * 2;
            P[0] = ss;
            P[1] = qq;
        }
    }
}

template <typename TOut, bool FLAT>
__global__ __launch_bounds__(NTHR) void splitk_epi(const stzs_conv_args a, int SK) {
    splitk_epi_body<TOut, FLAT>(a, SK);
}

// (r06) the combines of a conv_mfma_pair launch: grid z picks the problem
template <typename TOut>
__global__ __launch_bounds__(NTHR) void splitk_epi_pair(const stzs_conv_args a0, const stzs_conv_args a1, int SK) {
    if (blockIdx.z == 0)
        splitk_epi_body<TOut, false>(a0, SK);
    else
        splitk_epi_body<TOut, false>(a1, SK);
}

size_t lds_bytes(int rows_in, int cic, int nslot = NSLOT) {
    const size_t main = (((size_t)rows_in * (cic * 2 + 16) + 15) & ~(size_t)15) + (size_t)nslot * SLOT_BYTES + 4 * 128 * 4;
    const size_t epi = (size_t)BT * EP_PITCH * 4 + 2 * BCO * 4 + 2 * 4 * BCO * 2 * 4;
    return main > epi ? main : epi;
}

template <typename TIn, typename TOut, bool F8 = false>
int launch_dt(const stzs_conv_args& a, hipStream_t s) {
    const bool flat = (a.ks == 1 && a.stride == 1 && a.pad == 0 && a.ups == 0 && a.pro_mode == STZS_PRO_NONE &&
                       a.pro_act == STZS_ACT_NONE && a.T_in == a.T_out);
    const int rows_in = flat ? BT : (BT - 1) * a.stride + (a.ks - 1) * a.dil + 1;
    // DEEP: split-K with one input-channel chunk per slice whose K-steps all fit LDS beside the staged rows
    const int nslot_deep = (flat ? 1 : a.ks) * (a.cic >> 5);
    const bool deep = a.splitk > 1 && a.splitk == a.ci_pad / a.cic && !(a.flags & STZS_CONV_RING) &&
                      lds_bytes(rows_in, a.cic, nslot_deep) <= 160 * 1024;
    const size_t lds = lds_bytes(rows_in, a.cic, deep ? nslot_deep : NSLOT);
    if (lds > 160 * 1024) return STZS_ESHAPE;
    const unsigned gx = flat ? (unsigned)(((long)a.B * a.T_out + BT - 1) / BT)
                             : (unsigned)a.B * (unsigned)((a.T_out + BT - 1) / BT);
    dim3 grid(gx, a.co_pad / BCO);
    if (flat && a.stat_part) return STZS_EINVAL;  // fused statistics: per-utterance tiles only
    void (*k)(stzs_conv_args);
    if (F8 || (flat && sizeof(TIn) == 2 && (a.flags & STZS_CONV_A_DMA) && a.pro_cscale == 1.f))
        return stzs_gemm_glds_launch(a, s);  // (csrc/gemm.hip)
    if (a.splitk > 1) {  // conv_mfma: split over input-channel chunks (2..16 slices, at least one chunk each)
        if (F8 || a.splitk > 16 || a.splitk > a.ci_pad / a.cic || !a.splitk_ws || !a.splitk_ctr ||
            !stzs_aligned(a.splitk_ws, 16) || !stzs_aligned(a.splitk_ctr, 4))
            return STZS_EINVAL;
        grid.z = (unsigned)a.splitk;
    }
    if constexpr (F8) {
        return STZS_EDTYPE;  // (unreachable: fp8 is a pure linear)
    } else {
        // DEEP slices hand their partials to splitk_epi (vectorised epilogue, no DiT row gate) unless STZS_CONV_SK_TICKET
        const bool ske = deep && epi_vec(a) && !(flat && a.gate) && a.ups == 0 && !(a.flags & STZS_CONV_SK_TICKET);
        if (ske) {
            if (flat)
                k = conv_mfma<TIn, TOut, true, STZS_ACT_NONE, true, true>;
            else if (a.pro_act == STZS_ACT_LEAKY)
                k = conv_mfma<TIn, TOut, false, STZS_ACT_LEAKY, true, true>;
            else if (a.pro_act == STZS_ACT_SNAKE)
                k = conv_mfma<TIn, TOut, false, STZS_ACT_SNAKE, true, true>;
            else
                k = conv_mfma<TIn, TOut, false, STZS_ACT_NONE, true, true>;
            if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            hipLaunchKernelGGL(k, grid, dim3(NTHR), lds, s, a);
            STZS_LAUNCH_CHECK();
            auto ke = flat ? splitk_epi<TOut, true> : splitk_epi<TOut, false>;
            hipLaunchKernelGGL(ke, dim3(grid.x, grid.y * 8), dim3(NTHR), 0, s, a, (int)a.splitk);
            STZS_LAUNCH_CHECK();
            return STZS_OK;
        }
        if (deep) {
            if (flat)
                k = conv_mfma<TIn, TOut, true, STZS_ACT_NONE, true>;
            else if (a.pro_act == STZS_ACT_LEAKY)
                k = conv_mfma<TIn, TOut, false, STZS_ACT_LEAKY, true>;
            else if (a.pro_act == STZS_ACT_SNAKE)
                k = conv_mfma<TIn, TOut, false, STZS_ACT_SNAKE, true>;
            else
                k = conv_mfma<TIn, TOut, false, STZS_ACT_NONE, true>;
        } else if (flat)
            k = conv_mfma<TIn, TOut, true, STZS_ACT_NONE>;
        else if (a.pro_act == STZS_ACT_SNAKE)
            k = conv_mfma<TIn, TOut, false, STZS_ACT_SNAKE>;
        else if (a.pro_act == STZS_ACT_LEAKY)
            k = conv_mfma<TIn, TOut, false, STZS_ACT_LEAKY>;
        else
            k = conv_mfma<TIn, TOut, false, STZS_ACT_NONE>;
        if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k, grid, dim3(NTHR), lds, s, a);
        STZS_LAUNCH_CHECK();
        return STZS_OK;
    }
}

// (r06) two problems as ONE conv_mfma_pair + ONE splitk_epi_pair launch where each would take the DEEP split-K form with
// the splitk_epi combine on its own (not flat; the batch-1 predictor / decoder AdaIN-block convs) with the same
// prologue activation, grid, slice count and LDS; otherwise STZS_ESHAPE (nothing launched).
template <typename TIn, typename TOut>
int launch_pair_dt(const stzs_conv_args* p, hipStream_t s) {
    size_t lds = 0;
    for (int i = 0; i < 2; ++i) {
        const stzs_conv_args& a = p[i];
        const bool flat = (a.ks == 1 && a.stride == 1 && a.pad == 0 && a.ups == 0 && a.pro_mode == STZS_PRO_NONE &&
                           a.pro_act == STZS_ACT_NONE && a.T_in == a.T_out);
        const int rows_in = (BT - 1) * a.stride + (a.ks - 1) * a.dil + 1;
        const int nslot_deep = a.ks * (a.cic >> 5);
        const bool deep = !flat && a.splitk > 1 && a.splitk == a.ci_pad / a.cic && !(a.flags & STZS_CONV_RING) &&
                          lds_bytes(rows_in, a.cic, nslot_deep) <= 160 * 1024;
        const bool ske = deep && epi_vec(a) && a.ups == 0 && !(a.flags & (STZS_CONV_SK_TICKET | STZS_CONV_A_DMA));
        if (!ske || a.splitk > 16 || !a.splitk_ws || !a.splitk_ctr || !stzs_aligned(a.splitk_ws, 16) ||
            !stzs_aligned(a.splitk_ctr, 4))
            return STZS_ESHAPE;
        const size_t l = lds_bytes(rows_in, a.cic, nslot_deep);
        if (i == 0) lds = l;
        if (i == 1 && (l != lds || a.splitk != p[0].splitk || a.pro_act != p[0].pro_act || a.B != p[0].B ||
                       a.T_out != p[0].T_out || a.co_pad != p[0].co_pad))
            return STZS_ESHAPE;
    }
    const stzs_conv_args& a = p[0];
    void (*k)(stzs_conv_args, stzs_conv_args) = a.pro_act == STZS_ACT_LEAKY ? conv_mfma_pair<TIn, TOut, STZS_ACT_LEAKY>
                                               : a.pro_act == STZS_ACT_SNAKE ? conv_mfma_pair<TIn, TOut, STZS_ACT_SNAKE>
                                                                             : conv_mfma_pair<TIn, TOut, STZS_ACT_NONE>;
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    dim3 grid((unsigned)a.B * (unsigned)((a.T_out + BT - 1) / BT), a.co_pad / BCO, 2 * a.splitk);
    hipLaunchKernelGGL(k, grid, dim3(NTHR), lds, s, p[0], p[1]);
    STZS_LAUNCH_CHECK();
    hipLaunchKernelGGL(splitk_epi_pair<TOut>, dim3(grid.x, grid.y * 8, 2), dim3(NTHR), 0, s, p[0], p[1], (int)a.splitk);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

}  // namespace

int stzs_mrf_conv_launch(const stzs_conv_args& a, hipStream_t s);     // csrc/mrf.hip
int stzs_narrow_conv_launch(const stzs_conv_args& a, hipStream_t s);  // csrc/mrf.hip

namespace {

int core_checks(const stzs_conv_args* a) {
    if (!a || !a->x || !a->w || !a->y) return STZS_EINVAL;
    if (a->cic != 32 && a->cic != 64 && a->cic != 128) return STZS_EINVAL;
    if (a->B <= 0 || a->T_in <= 0 || a->T_out <= 0 || a->Ci <= 0 || a->Co <= 0 || a->ks <= 0 || a->dil <= 0 ||
        a->stride <= 0)
        return STZS_ESHAPE;
    if (a->ci_pad % a->cic || a->ci_pad < a->Ci || a->co_pad % BCO) return STZS_ESHAPE;
    if (a->splitk > 1 && (a->flags & (STZS_CONV_W_X3 | STZS_CONV_W_F32 | STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32)))
        return STZS_EINVAL;
    const int ncol = a->ups > 0 ? a->ups * a->Co : a->Co;
    if (a->co_pad < ncol) return STZS_ESHAPE;
    if (a->ldx % 8 || a->bsx % 8 || a->ldx < ((a->Ci + 7) / 8) * 8) return STZS_ESHAPE;
    if (!stzs_aligned(a->x, 16) || !stzs_aligned(a->w, 16)) return STZS_EINVAL;
    if (a->ups > 0) {
        if (a->ks != 2 || a->pad != 1 || a->stride != 1 || a->dil != 1 || a->T_out != a->T_in + 1) return STZS_ESHAPE;
        if (a->Co % 8) return STZS_ESHAPE;
        if (a->refl && a->T_final < 2) return STZS_ESHAPE;
    } else if (a->refl) {
        return STZS_EINVAL;
    }
    if (a->res && a->res_tdiv <= 0) return STZS_EINVAL;
    if (a->pro_part && (a->pro_nch < 1 || a->pro_nch > 8 || a->pro_T < 1 || a->pro_ld < a->Ci ||
                        (a->flags & (STZS_CONV_W_X3 | STZS_CONV_W_F32 | STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32 |
                                     STZS_CONV_W_FRAG32 | STZS_CONV_W_FRAG32X3 | STZS_CONV_ROWS | STZS_CONV_A_DMA))))
        return STZS_EINVAL;  // (the prologue partials: generic conv path, <= 8 chunks)
    if (a->pro_mode == STZS_PRO_ADAIN && (!a->pro_part && (!a->pro_mean || !a->pro_rstd)) ) return STZS_EINVAL;
    if (a->pro_mode == STZS_PRO_ADAIN && !a->pro_gb) return STZS_EINVAL;
    // the prologue activations: NONE, LEAKY, SNAKE only (GELU / SILU are epilogue activations); every kernel family
    // below selects its prologue template from these three
    if (a->pro_act != STZS_ACT_NONE && a->pro_act != STZS_ACT_LEAKY && a->pro_act != STZS_ACT_SNAKE) return STZS_EINVAL;
    if (a->pro_act == STZS_ACT_SNAKE && !a->pro_alpha) return STZS_EINVAL;
    if (a->stat_part && (a->ups > 0 || !epi_vec(*a) || a->stat_ld < a->Co || !stzs_aligned(a->stat_part, 8)))
        return STZS_EINVAL;
    return STZS_OK;
}

}  // namespace

// (r06) two generic-path problems in one conv_mfma_pair + splitk_epi_pair launch (stzs_conv1d_group, n = 2): each must
// pass stzs_conv1d's checks, be bf16 -> bf16 without a W_* / ROWS / A_DMA flag and take the DEEP split-K form with the
// splitk_epi combine on its own; STZS_ESHAPE otherwise (nothing launched: the caller runs them one at a time).
__attribute__((visibility("hidden"))) int stzs_conv_pair_launch(const stzs_conv_args* p, hipStream_t s) {
    constexpr int WF = STZS_CONV_W_X3 | STZS_CONV_W_F32 | STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32 | STZS_CONV_W_FRAG32 |
                       STZS_CONV_W_FRAG32X3 | STZS_CONV_ROWS | STZS_CONV_A_DMA | STZS_CONV_UPS_NOISE;
    for (int i = 0; i < 2; ++i) {
        const int rc = core_checks(&p[i]);
        if (rc != STZS_OK) return rc;
        if ((p[i].flags & WF) || p[i].in_dtype != STZS_BF16 || p[i].out_dtype != STZS_BF16) return STZS_ESHAPE;
    }
    return launch_pair_dt<bf16_t, bf16_t>(p, s);
}

// the dispatcher proper; csrc/dispatch.hip routes the register-direct MRF form before it
__attribute__((visibility("hidden"))) int stzs_conv1d_core(const stzs_conv_args* a, void* stream) {
    {
        const int rc = core_checks(a);
        if (rc != STZS_OK) return rc;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (a->in_dtype == STZS_F8) {
        const bool lin = a->ks == 1 && a->stride == 1 && a->pad == 0 && a->ups == 0 && a->T_in == a->T_out &&
                         a->pro_mode == STZS_PRO_NONE && a->pro_act == STZS_ACT_NONE && a->pro_cscale == 1.f;
        if (!lin || !(a->flags & STZS_CONV_A_DMA) || (a->flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32)))
            return STZS_EDTYPE;
        if (!a->x_scale || !a->w_scale || a->stat_part) return STZS_EINVAL;
        if (a->ci_pad % 64 || a->ldx % 16 || a->bsx % 16) return STZS_ESHAPE;
        if (a->out_dtype == STZS_BF16) return launch_dt<f8_t, bf16_t, true>(*a, s);
        if (a->out_dtype == STZS_F32) return launch_dt<f8_t, float, true>(*a, s);
        return STZS_EDTYPE;
    }
    if (a->flags & STZS_CONV_W_X3) return stzs_conv_x3_launch(a, s);    // (csrc/convx.hip)
    if (a->flags & STZS_CONV_W_F32) return stzs_conv_f32_launch(a, s);  // (csrc/convx.hip)
    if (a->flags & STZS_CONV_W_LANE16) return stzs_mrf_conv_launch(*a, s);
    if (a->flags & STZS_CONV_W_NARROW32) return stzs_narrow_conv_launch(*a, s);
    if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16) return launch_dt<bf16_t, bf16_t>(*a, s);
    if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32) return launch_dt<bf16_t, float>(*a, s);
    if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16) return launch_dt<float, bf16_t>(*a, s);
    if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F32) return launch_dt<float, float>(*a, s);
    return STZS_EDTYPE;
}

extern "C" size_t stzs_conv_splitk_workspace(int64_t rows, int32_t co_pad, int32_t splitk) {
    if (rows <= 0 || co_pad <= 0 || co_pad % BCO || (splitk != 2 && splitk != 4)) return 0;
    const int64_t tiles = (rows + 63) / 64 * (co_pad / BCO);
    return (size_t)tiles * splitk * (64 / 32 * 4) * NTHR * 16;
}

#ifdef STZS_GEMM_PROF
extern "C" int stzs_gemm_prof_conv(const stzs_conv_args* a, void* stream) { return stzs_conv1d_core(a, stream); }
#endif

#ifdef STZS_CONV_PROF
// probe build only: copy the stamps to the host (n <= 16 * 8192 words) / zero them
extern "C" int stzs_conv_prof_read(unsigned long long* host, size_t n, int zero) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_cprof)) != hipSuccess) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (host && hipMemcpy(host, p, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (zero && hipMemset(p, 0, sizeof(unsigned long long) * 16 * 8192) != hipSuccess) return -1;
    return 0;
}
#endif
