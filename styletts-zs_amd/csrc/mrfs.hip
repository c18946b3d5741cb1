// The stage-1 MRF conv (the generator's AdaINResBlock1 convs at 128 channels, one input chunk),
// warp-specialised and persistent: the same arithmetic as the register-direct mrfv_conv (csrc/mrfv.hip -- same
// staged bf16 operands, same K order per output, same epilogue and statistics partials: BIT-identical), with the
// input staging taken off the MFMA waves' critical path.
//
// Why (profiles/r04_e_mrfv_flags*.log, B = 64, stage 1): the K loop alone runs at 1 400-1 575 TF/s, but staging the
// input tile (HBM loads + AdaIN + Snake on the VALU) and the epilogue add 38-120 % on top (k3 c1: 105 us of K loop,
// 232 us in all), because every workgroup runs load -> transform -> K loop -> epilogue in sequence and three of them
// per CU do not cover one another's load latency.
//
// Form: ONE 512-thread workgroup per CU walks a contiguous range of 128-row tiles.  Waves 0-3 (consumers, one per
// SIMD) run the K loop and the epilogue of tile i from LDS buffer i & 1, each wave 32 output channels x 128 rows as
// in mrfv; waves 4-7 (producers, the SIMD partners: waves w and w + 4 share a SIMD) stage tile i + 1 into the other
// buffer meanwhile -- global loads, the per-channel AdaIN / Snake constants (in registers), the transform, the LDS
// stores.  One workgroup barrier per tile hands the buffers over.  s_waitcnt vmcnt is per wave, so the consumers'
// weight and residual loads never wait behind the producers' input loads.  The consumers stream the weight fragments
// PD K-steps ahead as mrfv does, the ring running on across tiles (every tile uses the same K-steps).
// NC = 2 (the stage-0 convs, 256 -> 256 channels): the unit of the pipeline is one (tile, 128-channel input chunk);
// each consumer wave owns 64 output channels (mrfv's wide form: bit-identical to it), accumulates chunk 0 then
// chunk 1 and runs the epilogue after chunk 1.  Producers and consumers run separate loops with the same barrier
// count, so the consumers' accumulators are not live across the producers' staging code (register pressure).
#include "common.hpp"

namespace {

constexpr int NTH = 512;
constexpr int BT = 128;
constexpr int P = 272;  // staged input row pitch, bytes (as mrfv: conflict-free ds_read_b128)

// x[0..N) summed over the 16 lanes of each DPP row (mrfv.hip row_sum16_n: the same additions in the same order)
template <int N>
STZS_DEV void row_sum16(float* x) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
}

// staged rows per 16-row pass (as mrfv sb_rows: k3 dil <= 8, k7 / k11 dil <= 5)
constexpr int sb_of(int ks) { return ks == 3 ? 9 : (ks == 7 ? 10 : 12); }

template <bool HR, bool HA, int KS, bool AL, int NC>
__global__ __launch_bounds__(NTH, 1) void mrfs_conv(const stzs_conv_args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NKC = KS * 4;              // 32-wide K-steps of one 128-channel chunk
    constexpr int SB = sb_of(KS);
    // RESW: every weight fragment of the K loop resident in registers (k3: 96 VGPRs).  Off: with the producer's and the
    // consumer's registers allocated together it spilled 28 VGPRs; the k3 K loop streams its weights like k7 / k11
    constexpr bool RESW = false;
    // streamed weights: K-steps in flight ahead of the MFMAs.  The ring slot of K-step s is s % (PD + 1) with s the
    // compile-time index within the unit, so PD + 1 must divide NKC = 4 KS for the ring to stay aligned when it runs
    // on into the next unit (register arrays need compile-time indices): PD = 3; the two-chunk form's K-step is twice
    // as long (4 fragments): PD = 1, as mrfv's wide form
    constexpr int PD = RESW ? 0 : (NC == 1 ? 3 : 1);
    static_assert(RESW || NKC % (PD + 1) == 0, "the weight ring wraps at unit boundaries");
    const int dil = a.dil;
    const int rows_in = BT + (KS - 1) * dil;
    const int buf_bytes = (rows_in * P + 15) & ~15;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool producer = wave >= 4;
    const int tpb = (a.T_out + BT - 1) / BT;
    const int ntiles = a.B * tpb;
    const int G = gridDim.x;
    const int per = (ntiles + G - 1) / G;
    const int tbeg = blockIdx.x * per;
    const int tend = min(ntiles, tbeg + per);
    // pipeline units (tile, chunk), chunk fastest; uniform per workgroup: every wave runs the same barriers
    const int nmy = tend > tbeg ? (tend - tbeg) * NC : 0;

    // ------------------------------------------------------------------ producer: stage tile `tile` into buffer b
    const int ptid = tid - 256;  // producers 0..255 (the mrfv staging thread map)
    const int cv = ptid & 15, rsub = ptid >> 4;
    auto stage = [&](int u, int b) {
        const int tile = tbeg + u / NC, cc = u % NC;
        const int bq = tile / tpb;
        const int t0 = (tile - bq * tpb) * BT;
        const bf16_t* X = reinterpret_cast<const bf16_t*>(a.x) + (long)bq * a.bsx;
        const int c = cc * 128 + cv * 8;
        const bool c_ok = c < a.Ci;
        const int cl = c_ok ? c : 0;
        const bool interior = t0 - a.pad >= 0 && t0 - a.pad + 16 * SB <= a.T_in && cc * 128 + 128 <= a.Ci;
        uint4 raw[SB];
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            int tin = t0 - a.pad + rsub + 16 * i;
            if (!interior) tin = tin < 0 ? 0 : (tin >= a.T_in ? a.T_in - 1 : tin);
            const unsigned off = (unsigned)(tin * (int)a.ldx + cl) * 2u;
            raw[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(X) + off);
        }
        // the per-channel constants of this thread's 8 channels, in registers (mrfv computes the same values into
        // LDS: sc = (1 + gamma) rstd, sh = beta - mean sc; Snake cosine form ka = sc a / pi, kb = sh a / pi, km = -1/(2a))
        f32x2 ka[4], kbv[4], ksc[4], ksh[4], km[4];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int ch = c + j;
            const bool ok = ch < a.Ci;
            float sc = 0.f, sh = 0.f;
            if (ok && a.pro_mode == STZS_PRO_ADAIN) {
                const float mu = a.pro_mean[(long)bq * a.stat_bs + ch];
                const float rs = a.pro_rstd[(long)bq * a.stat_bs + ch];
                const float gm = a.pro_gb[(long)bq * a.gb_bs + ch];
                const float be = a.pro_gb[(long)bq * a.gb_bs + a.gb_beta_off + ch];
                sc = (1.f + gm) * rs;
                sh = be - mu * sc;
            } else if (ok) {
                sc = a.pro_cscale;
            }
            const float al = ok ? a.pro_alpha[ch] : 1.f;
            const float h = 0.5f / al;
            const float w = al * 0.318309886183790672f;  // a / pi
            ka[j >> 1][j & 1] = sc * w;
            kbv[j >> 1][j & 1] = sh * w;
            ksc[j >> 1][j & 1] = sc;
            ksh[j >> 1][j & 1] = sh + h;
            km[j >> 1][j & 1] = -h;
        }
        uint32_t* rw = reinterpret_cast<uint32_t*>(raw);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                const uint32_t wv = rw[4 * i + p];
                const f32x2 x = f32x2{__uint_as_float(wv << 16), __uint_as_float(wv & 0xFFFF0000u)};
                f32x2 y = x * ksc[p] + ksh[p];
                const f32x2 t = x * ka[p] + kbv[p];
                const f32x2 cz = f32x2{__builtin_amdgcn_cosf(t.x), __builtin_amdgcn_cosf(t.y)};
                y = cz * km[p] + y;
                const int tin = t0 - a.pad + rsub + 16 * i;
                const bool ok = interior || (c_ok && tin >= 0 && tin < a.T_in);
                rw[4 * i + p] = ok ? pack2bf(y.x, y.y) : 0u;
            }
        }
        unsigned char* S = smem + b * buf_bytes;
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            const int r = rsub + 16 * i;
            if (r < rows_in) *reinterpret_cast<uint4*>(S + r * P + cv * 16) = raw[i];
        }
    };

    // ------------------------------------------------------------------ consumer state
    constexpr int NA = 2 * NC;  // A fragments (16 output channels each) per wave and K-step
    constexpr int NKT = NC * NKC;  // K-steps of a tile (the weight ring's period)
    // consumer wave: NC == 1 output channels 32 cw ..; NC == 2 (mrfv's wide map) the packed waves ow0, ow0 + 1 of
    // 128-channel tile ct
    const int ct = NC == 1 ? 0 : (wave & 3) >> 1;
    const int ow0 = NC == 1 ? (wave & 3) : (wave & 1) * 2;
    const bf16x8* Wf = reinterpret_cast<const bf16x8*>(a.w) + (long)ct * NKT * 512 + ow0 * 128 + lane;
    const int xoff0 = (lane & 15) * P + (lane >> 4) * 16;
    const int dP = dil * P;
    const int g = lane >> 4, n = lane & 15;
    const bool stat = a.stat_part != nullptr;
    const int nch = (a.T_out + 63) / 64;
    bf16_t* Y = reinterpret_cast<bf16_t*>(a.y);

    if (NC > 1 && producer) {  // ---------------------------------------- producer loop (two-chunk form)
        if (nmy > 0) stage(0, 0);
        __syncthreads();
        for (int i = 0; i < nmy; ++i) {
            if (i + 1 < nmy) stage(i + 1, (i + 1) & 1);
            __syncthreads();  // unit i + 1 staged; unit i's buffer free for unit i + 2
        }
        return;
    }
    // ------------------------------------------------------------------ consumer loop
    bf16x8 wres[RESW ? NKC : 1][NA];
    bf16x8 wf[PD + 1][NA];
    int kq = 0;  // streamed: the next K-step (mod NKT) the ring loads
    if (producer) {
    } else if constexpr (RESW) {
#pragma unroll
        for (int s = 0; s < NKC; ++s)
#pragma unroll
            for (int j = 0; j < NA; ++j) wres[s][j] = Wf[(long)s * 512 + 64 * j];
    } else {
#pragma unroll
        for (int i = 0; i < PD; ++i)
#pragma unroll
            for (int j = 0; j < NA; ++j) wf[i][j] = Wf[(long)i * 512 + 64 * j];
        kq = PD;
    }
    auto compute = [&](f32x4 (&acc)[NA][8], int u, int b) {
        const int tile = tbeg + u / NC, cc = u % NC;
        const int bq = tile / tpb;
        const int t0 = (tile - bq * tpb) * BT;
        const unsigned char* S = smem + b * buf_bytes;
        bf16x8 xf[8];
        const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
        if constexpr (NC > 1) {
            if (cc == 0) {
#pragma unroll
                for (int j = 0; j < NA; ++j)
#pragma unroll
                    for (int mt = 0; mt < 8; ++mt) acc[j][mt] = zero;
            }
        }
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) xf[mt] = *reinterpret_cast<const bf16x8*>(S + xoff0 + mt * 16 * P);
#pragma unroll
        for (int s = 0; s < NKC; ++s) {
            if constexpr (!RESW) {  // the ring runs on across units: K-step kq of this or the next unit
#pragma unroll
                for (int j = 0; j < NA; ++j) wf[(s + PD) % (PD + 1)][j] = Wf[(long)kq * 512 + 64 * j];
                kq = kq + 1 == NKT ? 0 : kq + 1;
            }
            const int sn = s + 1;
            const int offn = (sn >> 2) * dP + (sn & 3) * 64;
#pragma unroll
            for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
                for (int j = 0; j < NA; ++j) {
                    const bf16x8 wv = RESW ? wres[s][j] : wf[s % (PD + 1)][j];
                    acc[j][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, xf[mt], (NC == 1 && s == 0) ? zero : acc[j][mt], 0, 0, 0);
                }
                if (sn < NKC) xf[mt] = *reinterpret_cast<const bf16x8*>(S + xoff0 + offn + mt * 16 * P);
            }
            if constexpr (!RESW) __builtin_amdgcn_sched_group_barrier(0x020, NA, 0);  // the weight loads first
#pragma unroll
            for (int mt = 0; mt < 8; ++mt) {
                __builtin_amdgcn_sched_group_barrier(0x008, NA, 0);
                if (sn < NKC) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (cc != NC - 1) return;
        // ---- epilogue (mrfv's): lane (g, n) holds time t0 + mt 16 + n, channels co0..+7 of each 32-channel group
        const char* Rq = reinterpret_cast<const char*>(a.res) + (long)bq * a.bsr * 2;
        const char* Aq = reinterpret_cast<const char*>(a.acc_in) + (long)bq * a.bsa * 2;
#pragma unroll
        for (int sw = 0; sw < NC; ++sw) {  // (two-chunk form: the wave's two 32-channel groups one after the other)
        const int co0 = ct * 128 + (ow0 + sw) * 32 + g * 8;
        const bool col_ok = co0 < a.Co;
        const int coc = col_ok ? co0 : 0;
        float bias[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) bias[i] = a.bias ? a.bias[coc + i] : 0.f;
        // residual / accumulate rows: all 8 row tiles at once, or per 64-row half where both operands are present in
        // the two-chunk form (its 128 accumulator VGPRs leave no room for 64 more)
        constexpr int RQ = (NC > 1 && HR && HA) ? 4 : 8;
        uint4 rr[RQ], aa[RQ];
        auto load_ra = [&](int mt0) {
#pragma unroll
            for (int q = 0; q < RQ; ++q) {
                const int t = t0 + (mt0 + q) * 16 + n;
                const int tc = t < a.T_out ? t : a.T_out - 1;
                if constexpr (HR) rr[q] = *reinterpret_cast<const uint4*>(Rq + (unsigned)(tc * (int)a.ldr + coc) * 2u);
                if constexpr (HA) aa[q] = *reinterpret_cast<const uint4*>(Aq + (unsigned)(tc * (int)a.lda + coc) * 2u);
            }
        };
        if constexpr (RQ == 8) load_ra(0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if constexpr (RQ == 4) load_ra(h * 4);
            float ss[8], sq[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) ss[i] = sq[i] = 0.f;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int mt = h * 4 + m;
                const int t = t0 + mt * 16 + n;
                const bool ok = col_ok && t < a.T_out;
                float v[8];
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[nt * 4 + r] = acc[sw * 2 + nt][mt][r] + bias[nt * 4 + r];
                if constexpr (HR) {
                    float f[8];
                    unpack8(rr[RQ == 8 ? mt : m], f);
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] += f[i];
                }
                if constexpr (AL) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] *= a.alpha;
                }
                if constexpr (HA) {
                    float f[8];
                    unpack8(aa[RQ == 8 ? mt : m], f);
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] = fmaf(a.beta, f[i], v[i]);
                }
                const uint4 o = pack8(v);
                if (ok) *reinterpret_cast<uint4*>(Y + (long)bq * a.bsy + (long)t * a.ldy + coc) = o;
                if (stat && ok) {
                    float f[8];
                    unpack8(o, f);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        ss[i] += f[i];
                        sq[i] = fmaf(f[i], f[i], sq[i]);
                    }
                }
            }
            if (stat) {
                row_sum16<8>(ss);
                row_sum16<8>(sq);
                const int r0 = t0 + h * 64;
                if (n == 0 && col_ok && r0 < a.T_out) {
                    float* Pp = reinterpret_cast<float*>(a.stat_part) + (((long)bq * nch + r0 / 64) * a.stat_ld + co0) * 2;
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        Pp[2 * i] = ss[i];
                        Pp[2 * i + 1] = sq[i];
                    }
                }
            }
        }
        }
    };
    if constexpr (NC == 1) {
        // one loop for both roles (measured: with separate loops hipcc spilled 28-99 VGPRs of the k7 / k11 forms)
        if (nmy > 0 && producer) stage(0, 0);
        __syncthreads();
        for (int i = 0; i < nmy; ++i) {
            if (!producer) {
                f32x4 acc[NA][8];
                compute(acc, i, i & 1);
            } else if (i + 1 < nmy) {
                stage(i + 1, (i + 1) & 1);
            }
            __syncthreads();  // unit i + 1 staged, unit i's buffer free for unit i + 2
        }
    } else {
        __syncthreads();  // unit 0 staged
        f32x4 acc[NA][8];
#pragma unroll 1
        for (int i = 0; i < nmy; ++i) {
            compute(acc, i, i & 1);
            __syncthreads();
        }
    }
}

template <bool HR, bool HA, bool AL, int NC>
void (*pick_ks(int ks))(stzs_conv_args) {
    switch (ks) {
        case 3: return mrfs_conv<HR, HA, 3, AL, NC>;
        case 7: return mrfs_conv<HR, HA, 7, AL, NC>;
        case 11: return mrfs_conv<HR, HA, 11, AL, NC>;
        default: return nullptr;
    }
}
template <bool HR, bool HA, bool AL>
void (*pick_nc(int ks, int nc))(stzs_conv_args) {
    return nc == 1 ? pick_ks<HR, HA, AL, 1>(ks) : pick_ks<HR, HA, AL, 2>(ks);
}

}  // namespace

// internal entry (csrc/mrfv.hip stzs_mrfv_conv_launch): 1 = not this form (the caller goes on), else a status.
// Taken for STZS_CONV_MRFS: FRAG32 weights, Snake prologue, 128 -> 128 channels (stage 1) or 256 -> 256 (stage 0:
// two input chunks, one 256-channel column tile), stride 1, the dilation within the staging of its kernel width.
__attribute__((visibility("hidden"))) int stzs_mrfs_conv_launch(const stzs_conv_args& a, hipStream_t s) {
    if (!(a.flags & STZS_CONV_MRFS)) return 1;
    const int nc = a.ci_pad / 128;
    if (a.pro_act != STZS_ACT_SNAKE || (nc != 1 && nc != 2) || a.co_pad != a.ci_pad || a.cic != 128 || a.stride != 1 ||
        (a.ks != 3 && a.ks != 7 && a.ks != 11) || a.ups || a.refl || a.gate || a.epi_act != STZS_ACT_NONE ||
        a.in_dtype != STZS_BF16 || a.out_dtype != STZS_BF16 || a.splitk > 1 || a.x_scale)
        return 1;
    const int rows_in = BT + (a.ks - 1) * a.dil;
    if (rows_in > 16 * sb_of(a.ks) || !a.pro_alpha || (a.res && a.res_tdiv != 1)) return 1;
    const size_t lds = 2 * (((size_t)rows_in * P + 15) & ~(size_t)15);
    const bool R = a.res != nullptr, A = a.acc_in != nullptr, al = a.alpha != 1.f;
    void (*k)(stzs_conv_args) = R ? (A ? (al ? pick_nc<true, true, true>(a.ks, nc) : pick_nc<true, true, false>(a.ks, nc))
                                       : (al ? pick_nc<true, false, true>(a.ks, nc) : pick_nc<true, false, false>(a.ks, nc)))
                                  : (A ? (al ? pick_nc<false, true, true>(a.ks, nc) : pick_nc<false, true, false>(a.ks, nc))
                                       : (al ? pick_nc<false, false, true>(a.ks, nc) : pick_nc<false, false, false>(a.ks, nc)));
    if (!k) return 1;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const long ntiles = (long)a.B * ((a.T_out + BT - 1) / BT);
    const int G = (int)(ntiles < stzs_cu_count() ? ntiles : stzs_cu_count());  // one workgroup per CU
    hipLaunchKernelGGL(k, dim3(G), dim3(NTH), lds, s, a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
