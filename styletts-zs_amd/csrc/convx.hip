// Precise (parity) forms of the conv / linear (csrc/conv.hip's dispatcher routes STZS_CONV_W_X3 and STZS_CONV_W_F32
// weights here): conv_f32 on the fp32 MFMA, conv_x3 with split bf16 operands (three MFMA products per fp32 product),
// sharing the tile geometry and the fused epilogue of conv_common.hpp.
#include "conv_common.hpp"

namespace {

// PRECISE (parity) mode, STZS_CONV_W_F32: fp32 operands on v_mfma_f32_16x16x4_f32 (products exact in
// fp32, fp32 accumulate), libm-accurate prologue (act_apply).  Same 128 x 128 tile, 2 x 2 waves and
// accumulator layout as conv_mfma (the 16x16 C/D map is dtype-independent on gfx950), so the whole
// fused epilogue (finish) is shared.  Per 32-channel input chunk the tile rows (+ halo) are staged once
// in fp32; per tap one [128 co][32 ci] fp32 weight K-step goes through LDS.  The 16-B fragment reads keep
// conv_mfma's k geometry: lane l holds k = 8 (l >> 4) + j of its row/column, and MFMA j sums the four k
// values {8 h + j}; A and B use the same map, so the eight MFMAs of a K-step cover all 32 k exactly once.
// Not a performance path: it exists so the decoder can be run at fp32 accuracy against the oracle.
constexpr int P32 = 36;  // fp32 LDS row pitch (32 + 4 floats)
template <typename TIn, typename TOut>
__global__ __launch_bounds__(NTHR, 1) void conv_f32(const stzs_conv_args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ks = a.ks;
    const int rows_in = (BT - 1) * a.stride + (ks - 1) * a.dil + 1;
    float* xin = reinterpret_cast<float*>(smem);
    float* wl = xin + rows_in * P32;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = wave >> 1, wc = wave & 1;
    const int tpb = (a.T_out + BT - 1) / BT;
    const int bq = blockIdx.x / tpb;
    const int t0 = (blockIdx.x - bq * tpb) * BT;
    const int nchunk = a.ci_pad / 32;
    const float* Wt = reinterpret_cast<const float*>(a.w) + (long)blockIdx.y * nchunk * ks * (BCO * 32);
    const TIn* X = reinterpret_cast<const TIn*>(a.x) + (long)bq * a.bsx;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int cc = 0; cc < nchunk; ++cc) {
        __syncthreads();
        for (int v = tid; v < rows_in * 4; v += NTHR) {
            const int r = v >> 2, cv = v & 3;
            const int ci = cc * 32 + cv * 8;
            const int tin = t0 * a.stride - a.pad + r;
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = 0.f;
            if (tin >= 0 && tin < a.T_in && ci < a.Ci) {
                float f[8];
                load8(X + (long)tin * a.ldx + ci, f);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int c = ci + j;
                    if (c >= a.Ci) break;
                    float sc = a.pro_cscale, sh = 0.f;
                    if (a.pro_mode == STZS_PRO_ADAIN) {
                        const float mu = a.pro_mean[(long)bq * a.stat_bs + c];
                        const float rs = a.pro_rstd[(long)bq * a.stat_bs + c];
                        const float g = a.pro_gb[(long)bq * a.gb_bs + c];
                        const float be = a.pro_gb[(long)bq * a.gb_bs + a.gb_beta_off + c];
                        sc = (1.f + g) * rs;
                        sh = be - mu * sc;
                    }
                    o[j] = act_apply(a.pro_act, f[j] * sc + sh, a.pro_slope, a.pro_alpha ? a.pro_alpha[c] : 1.f);
                }
            }
            float* d = xin + r * P32 + cv * 8;
            *reinterpret_cast<float4*>(d) = make_float4(o[0], o[1], o[2], o[3]);
            *reinterpret_cast<float4*>(d + 4) = make_float4(o[4], o[5], o[6], o[7]);
        }
        for (int tap = 0; tap < ks; ++tap) {
            __syncthreads();  // staged rows visible; previous weight K-step consumed
            const float* src = Wt + (long)(cc * ks + tap) * (BCO * 32);
            for (int e = tid * 4; e < BCO * 32; e += NTHR * 4)
                *reinterpret_cast<float4*>(wl + (e >> 5) * P32 + (e & 31)) = *reinterpret_cast<const float4*>(src + e);
            __syncthreads();
            const int kb = 8 * (lane >> 4);
            float av[4][8], bv[4][8];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const float* p = xin + ((wt * 64 + mt * 16 + (lane & 15)) * a.stride + tap * a.dil) * P32 + kb;
#pragma unroll
                for (int j = 0; j < 8; ++j) av[mt][j] = p[j];
            }
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const float* p = wl + (wc * 64 + nt * 16 + (lane & 15)) * P32 + kb;
#pragma unroll
                for (int j = 0; j < 8; ++j) bv[nt][j] = p[j];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt][j], bv[nt][j], acc[mt][nt], 0, 0, 0);
        }
    }
    finish<TOut, false, BT>(a, acc, smem, bq, t0, 0, blockIdx.y);
}

// PRECISE mode on the bf16 matrix cores, STZS_CONV_W_X3: split-operand ("bf16x3") products.  Every fp32
// operand v is split into hi = bf16(v) and lo = bf16(v - hi) (v = hi + lo to ~2^-17 relative), and
// a*b ~= ah*bh + ah*bl + al*bh on v_mfma_f32_16x16x32_bf16 (each product exact in fp32, fp32 accumulate; the
// dropped al*bl is ~2^-16 of the rest).  Input rows are split ONCE when staged (after the libm-accurate
// AdaIN / activation prologue, in fp32); weights arrive pre-split as two K-step streams (hi, then lo) in
// conv_mfma's swizzled layout with 32-channel chunks (stzs/weights.py kstep_stream_x3).  Same 128 x 128 tile,
// 2 x 2 waves, accumulator layout and fused epilogue (finish) as conv_mfma; per K-step 3 x 16 MFMAs.
// tools/precision_probe.py: this arithmetic in every GEMM of the pipeline keeps the end-to-end log-mel L1 at
// 2.2e-4 of the fp32 oracle; ~3x the bf16 MFMA work instead of the 16x of fp32 MFMA (conv_f32).
constexpr int XSLOT_C = 2 * SLOT_BYTES;  // one K-step: hi + lo weights
constexpr int PX = 80;  // staged row pitch, bytes: 32 bf16 + 16 (conflict-light ds_read_b128) ...
constexpr int PX_TIGHT = 64;  // ... or unpadded when the padded tiles would not fit (stride-6 noise convs: 774 rows)
__host__ __device__ inline int x3_pitch(int rows_in) {
    return 2 * ((rows_in * PX + 15) & ~15) + NSLOT * XSLOT_C + 3 * 32 * 4 <= 160 * 1024 ? PX : PX_TIGHT;
}
constexpr int XSLOT = XSLOT_C;
template <typename TIn, typename TOut, int PACT, bool FLAT>
__global__ __launch_bounds__(NTHR, 2) void conv_x3(const stzs_conv_args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ks = FLAT ? 1 : a.ks;
    const int rows_in = (BT - 1) * a.stride + (ks - 1) * a.dil + 1;
    const int px = x3_pitch(rows_in);
    unsigned char* thi = smem;
    unsigned char* tlo = smem + ((rows_in * px + 15) & ~15);
    unsigned char* ring = tlo + ((rows_in * px + 15) & ~15);
    float* c_sc = reinterpret_cast<float*>(ring + NSLOT * XSLOT);
    float* c_sh = c_sc + 32;
    float* c_al = c_sh + 32;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = wave >> 1, wc = wave & 1;
    // FLAT (linears: ks 1, no prologue): 128 consecutive rows of the [B * T] row space per tile
    int bq = 0, t0 = 0;
    long row0 = 0;
    if (FLAT) {
        row0 = (long)blockIdx.x * BT;
    } else {
        const int tpb = (a.T_out + BT - 1) / BT;
        bq = blockIdx.x / tpb;
        t0 = (blockIdx.x - bq * tpb) * BT;
    }
    const int nchunk = a.ci_pad / 32;
    const int NK = nchunk * ks;
    const long stream_el = (long)(a.co_pad / BCO) * NK * (BCO * 32);  // bf16 elements of one (hi | lo) stream
    const bf16_t* Wh = reinterpret_cast<const bf16_t*>(a.w) + (long)blockIdx.y * NK * (BCO * 32);
    const TIn* X = reinterpret_cast<const TIn*>(a.x) + (FLAT ? 0 : (long)bq * a.bsx);
    const long nR = (long)a.B * a.T_in;
    const float invTi = 1.f / (float)a.T_in;  // (FLAT rows -> utterance, rowdiv)
    auto fill = [&](int k) {
        const bf16_t* src = Wh + (long)k * (BCO * 32) + wave * 1024 + lane * 8;
        unsigned char* dst = ring + (k % NSLOT) * XSLOT + wave * 2048;
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // hi, lo
            const bf16_t* sh = src + h * stream_el;
            unsigned char* dh = dst + h * SLOT_BYTES;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)sh,
                                             (__attribute__((address_space(3))) void*)dh, 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(sh + 512),
                                             (__attribute__((address_space(3))) void*)(dh + 1024), 16, 0, 0);
        }
    };
    int boff[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int rr = wc * 64 + nt * 16 + (lane & 15);
        boff[nt] = rr * 64 + (((lane >> 4) ^ gswz(rr)) << 4);
    }
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    fill(0);
    if (NK > 1) fill(1);
    int k = 0;
    for (int cc = 0; cc < nchunk; ++cc) {
        __syncthreads();  // previous chunk's tiles / constants consumed
        if (tid < 32) {   // per-channel prologue constants of this chunk (fp32, the oracle's formula)
            const int c = cc * 32 + tid;
            float sc = 0.f, sh = 0.f, al = 1.f;
            if (c < a.Ci) {
                sc = a.pro_cscale;
                if (a.pro_mode == STZS_PRO_ADAIN) {
                    const float mu = a.pro_mean[(long)bq * a.stat_bs + c];
                    const float rs = a.pro_rstd[(long)bq * a.stat_bs + c];
                    const float g = a.pro_gb[(long)bq * a.gb_bs + c];
                    const float be = a.pro_gb[(long)bq * a.gb_bs + a.gb_beta_off + c];
                    sc = (1.f + g) * rs;
                    sh = be - mu * sc;
                }
                if (a.pro_alpha) al = a.pro_alpha[c];
            }
            c_sc[tid] = sc;
            c_sh[tid] = sh;
            c_al[tid] = al;
        }
        __syncthreads();
        // staging: rows_in x 4 vectors of 8 channels, prologue in fp32, split into the hi / lo tiles
        for (int v = tid; v < rows_in * 4; v += NTHR) {
            const int r = v >> 2, cv = v & 3;
            const int ci = cc * 32 + cv * 8;
            long off;
            bool rok;
            if (FLAT) {
                const long R = row0 + r;
                const long bb = rowdiv(R, a.T_in, invTi, nR + BT < (1L << 22));
                rok = R < nR;
                off = bb * a.bsx + (R - bb * a.T_in) * a.ldx;
            } else {
                const int tin = t0 * a.stride - a.pad + r;
                rok = tin >= 0 && tin < a.T_in;
                off = (long)tin * a.ldx;
            }
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = 0.f;
            if (rok && ci < a.Ci) {
                float f[8];
                load8(X + off + ci, f);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float y = f[j] * c_sc[cv * 8 + j] + c_sh[cv * 8 + j];
                    float z = y;
                    if constexpr (PACT == STZS_ACT_SNAKE) {
                        const float al = c_al[cv * 8 + j];
                        const float sn = sinf(al * y);
                        z = y + sn * sn / al;
                    } else if constexpr (PACT == STZS_ACT_LEAKY) {
                        z = y >= 0.f ? y : y * a.pro_slope;
                    }
                    o[j] = ci + j < a.Ci ? z : 0.f;
                }
            }
            float lo[8];
            uint4 hp = pack8(o);
            float hf[8];
            unpack8(hp, hf);
#pragma unroll
            for (int j = 0; j < 8; ++j) lo[j] = o[j] - hf[j];  // exact (Sterbenz-range subtraction)
            *reinterpret_cast<uint4*>(thi + r * px + cv * 16) = hp;
            *reinterpret_cast<uint4*>(tlo + r * px + cv * 16) = pack8(lo);
        }
        __syncthreads();
        for (int tap = 0; tap < ks; ++tap, ++k) {
            waitcnt_vm(k + 1 < NK ? 4 : 0);  // this K-step's 4 LDS-DMA pieces landed (the next may fly)
            __builtin_amdgcn_s_barrier();
            if (k + 2 < NK) fill(k + 2);
            const unsigned char* wl = ring + (k % NSLOT) * XSLOT;
            const int kb = 16 * (lane >> 4);
            bf16x8 ah[4], alo[4], bh[4], bl[4];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const int r = (wt * 64 + mt * 16 + (lane & 15)) * a.stride + tap * a.dil;
                ah[mt] = *reinterpret_cast<const bf16x8*>(thi + r * px + kb);
                alo[mt] = *reinterpret_cast<const bf16x8*>(tlo + r * px + kb);
            }
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                bh[nt] = *reinterpret_cast<const bf16x8*>(wl + boff[nt]);
                bl[nt] = *reinterpret_cast<const bf16x8*>(wl + SLOT_BYTES + boff[nt]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo[mt], bh[nt], acc[mt][nt], 0, 0, 0);
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bl[nt], acc[mt][nt], 0, 0, 0);
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bh[nt], acc[mt][nt], 0, 0, 0);
                }
        }
    }
    finish<TOut, FLAT, BT>(a, acc, smem, bq, t0, row0, blockIdx.y);
}

size_t x3_lds_bytes(int rows_in) {
    const size_t main = 2 * (((size_t)rows_in * x3_pitch(rows_in) + 15) & ~(size_t)15) + NSLOT * XSLOT + 3 * 32 * 4;
    const size_t epi = (size_t)BT * EP_PITCH * 4 + 2 * BCO * 4 + 2 * 4 * BCO * 2 * 4;
    return main > epi ? main : epi;
}

}  // namespace

// internal entries (csrc/conv.hip stzs_conv1d_core, arguments validated there)
__attribute__((visibility("hidden"))) int stzs_conv_x3_launch(const stzs_conv_args* a, hipStream_t s) {
    if (a->cic != 32 || a->ci_pad % 32 || (a->flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32 | STZS_CONV_W_F32)))
        return STZS_EINVAL;
    if (a->in_dtype == STZS_F32 ? (a->ldx % 8 || a->bsx % 8) : false) return STZS_ESHAPE;
    const int rows_in = (BT - 1) * a->stride + (a->ks - 1) * a->dil + 1;
    const size_t lds = x3_lds_bytes(rows_in);
    if (lds > 160 * 1024) return STZS_ESHAPE;
    void (*k)(stzs_conv_args) = nullptr;
    const bool flat = a->ks == 1 && a->stride == 1 && a->pad == 0 && a->ups == 0 && a->pro_mode == STZS_PRO_NONE &&
                      a->pro_act == STZS_ACT_NONE && a->T_in == a->T_out && !a->stat_part;
#define STZS_X3_PICK(TI, TO)                                                                         \
    k = flat ? conv_x3<TI, TO, STZS_ACT_NONE, true>                                                  \
    : a->pro_act == STZS_ACT_SNAKE ? conv_x3<TI, TO, STZS_ACT_SNAKE, false>                      \
    : a->pro_act == STZS_ACT_LEAKY ? conv_x3<TI, TO, STZS_ACT_LEAKY, false> : conv_x3<TI, TO, STZS_ACT_NONE, false>;
    if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F32) { STZS_X3_PICK(float, float) }
    else if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16) { STZS_X3_PICK(float, bf16_t) }
    else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32) { STZS_X3_PICK(bf16_t, float) }
    else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16) { STZS_X3_PICK(bf16_t, bf16_t) }
    else return STZS_EDTYPE;
#undef STZS_X3_PICK
    if (a->pro_act != STZS_ACT_NONE && a->pro_act != STZS_ACT_LEAKY && a->pro_act != STZS_ACT_SNAKE)
        return STZS_EINVAL;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    dim3 grid(flat ? (unsigned)(((long)a->B * a->T_out + BT - 1) / BT)
                   : (unsigned)a->B * (unsigned)((a->T_out + BT - 1) / BT), a->co_pad / BCO);
    hipLaunchKernelGGL(k, grid, dim3(NTHR), lds, s, *a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

__attribute__((visibility("hidden"))) int stzs_conv_f32_launch(const stzs_conv_args* a, hipStream_t s) {
    if (a->cic != 32 || a->ci_pad % 32 || (a->flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32)))
        return STZS_EINVAL;
    const int rows_in = (BT - 1) * a->stride + (a->ks - 1) * a->dil + 1;
    const size_t main = (size_t)(rows_in + BCO) * P32 * 4;
    const size_t epi = (size_t)BT * EP_PITCH * 4 + 2 * BCO * 4 + 2 * 4 * BCO * 2 * 4;
    const size_t lds = main > epi ? main : epi;
    if (lds > 160 * 1024) return STZS_ESHAPE;
    void (*k)(stzs_conv_args) = nullptr;
    if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F32) k = conv_f32<float, float>;
    else if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16) k = conv_f32<float, bf16_t>;
    else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32) k = conv_f32<bf16_t, float>;
    else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16) k = conv_f32<bf16_t, bf16_t>;
    else return STZS_EDTYPE;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    dim3 grid((unsigned)a->B * (unsigned)((a->T_out + BT - 1) / BT), a->co_pad / BCO);
    hipLaunchKernelGGL(k, grid, dim3(NTHR), lds, s, *a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
