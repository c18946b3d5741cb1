// PRECISE-mode register-direct conv (SURVEY.md §8(a) a12 -- the generator's MRF resblock convs -- and the k3 convs of
// the decoder / predictor AdaIN residual blocks, a9, in StyleTTSZS(precise=True)): the data movement of csrc/mrfv.hip
// with the split-operand arithmetic of csrc/convx.hip conv_x3.
//
//  * fp32 activations in and out; per 128-channel input chunk the tile's rows (+ dilation halo) are loaded ONCE, put
//    through the AdaIN affine + Snake (or LeakyReLU) in fp32 and split into hi = bf16(z) and lo = bf16(z - hi), two
//    staged LDS tiles (z = hi + lo to ~2^-17 relative);
//  * the 4 waves split the 128 output channels (32 each): a wave's weights come straight from global memory into
//    VGPRs as hi and lo 16x16x32 A-fragments (STZS_CONV_W_FRAG32X3: per K-step [hl][wave][nt][lane][8], hi and lo of
//    one K-step adjacent), one K-step ahead; no weight ring, no barrier in the K loop;
//  * per K-step and wave: 8 | 4 B-fragment pairs (hi, lo) from LDS and 3 x 16 | 3 x 8 MFMAs -- every product
//    w * z as wl * zh + wh * zl + wh * zh on v_mfma_f32_16x16x32_bf16 with fp32 accumulation (the dropped wl * zl is
//    ~2^-16 of the rest).  Three times the MFMAs of the bf16 form per staged byte: the K loop carries the staging;
//  * staged rows at a 256-B pitch with the 16-B chunk of channel group c of row r at position c ^ (r & 15): the
//    ds_read_b128 B-fragment reads (16 consecutive rows x 4 channel groups per wave-instruction) are bank-conflict
//    free without padding, so a 146-row tile pair (hi + lo) takes 73 KB and two workgroups fit a CU.  Tiles whose
//    halo would exceed that (k7 d5, k11 d3 / d5) run as 64-row tiles;
//  * epilogue straight from the accumulators (lane (g, n): 8 consecutive channels of one time row, 32-B fp32 loads /
//    stores), fused InstanceNorm statistics of the stored fp32 values per 64-row chunk (the stzs_chan_stats partial
//    layout, as mrfv / conv_x3).
// The Snake uses the hardware sine on the revolution argument alpha y / 2 pi: its error (~1e-7 of |alpha y|) scales
// with |y| as the output does, i.e. fp32-level relative to z, below the split products' ~2^-17.
#include "common.hpp"

#include <type_traits>

namespace {

constexpr int NTH = 256;
constexpr int BCO = 128;
constexpr int PX = 256;  // staged row pitch, bytes (128 channels x bf16, XOR-swizzled 16-B chunks)
constexpr int NCS = 4;   // per-channel constants: sc, sh, alpha / 2 pi, 1 / alpha

// staged 16-B row vectors per thread (16 rows each): rows_in = BT + (KS - 1) dil <= 16 SB (sized per form: every
// staged vector costs its load and transform whether or not its row is used)
constexpr int sb_rows(int ks, int bt) {
    return bt == 128 ? (ks == 7 ? 10 : 9) : (ks == 3 ? 5 : (ks == 7 ? 6 : 8));
}

// x[0..N) summed over the 16 lanes of each DPP row, VALU only (the csrc/mrfv.hip reduction)
template <int N>
STZS_DEV void row_sum16_n(float* x) {
    static_assert(N >= 4, "dependent DPP steps need >= 2 independent instructions between them");
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
}

// fp32 -> (hi, lo) bf16 split of 8 values: hi = RNE bf16, lo = RNE bf16 of the exact remainder z - hi
STZS_DEV void split8(const float* z, uint4& hi, uint4& lo) {
    hi = pack8(z);
    float h[8], r[8];
    unpack8(hi, h);
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = z[i] - h[i];  // exact (Sterbenz)
    lo = pack8(r);
}

// NCH = 1: one 128-channel input chunk (the stage-1 generator convs); 0: any number (accumulators live across chunks).
// AL: the epilogue scales by a.alpha.  BT: 128 or 64 time rows per tile.
// NW (narrow, Co <= 32: conv_post 128 -> 22): the 4 waves split the tile's ROWS (32 each) and all compute output
// channels 0..31 from packed wave 0's fragments; no statistics, masked stores past Co.
template <int PACT, bool HR, bool HA, int KS, int BT, int NCH, bool AL, bool NW = false>
__global__ __launch_bounds__(NTH, 2) void mrfx_conv(const stzs_conv_args a) {
    constexpr int MT = NW ? BT / 64 : BT / 16;  // 16-row B fragments per wave
    constexpr int NKC = KS * 4;   // 32-wide K-steps per 128-channel chunk
    constexpr int SB = sb_rows(KS, BT);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int dil = a.dil;
    const int rows_in = BT + (KS - 1) * dil;
    unsigned char* const thi = smem;
    const int lo_off = rows_in * PX;
    float* cs = reinterpret_cast<float*>(smem + 2 * lo_off);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tpb = (a.T_out + BT - 1) / BT;
    const int nx = gridDim.x;
    const int lin = (a.flags & STZS_CONV_LINEAR_IDS) ? blockIdx.y * nx + blockIdx.x
                                                      : xcd_remap(blockIdx.y * nx + blockIdx.x, nx * gridDim.y);
    const int by = lin / nx, bx = lin - by * nx;  // (co tile, utterance x time tile)
    const int bq = bx / tpb;
    const int t0 = (bx - bq * tpb) * BT;
    const int nchunk = NCH ? NCH : a.ci_pad >> 7;
    // weights: [co tile][chunk][tap][kq][hl][wave][nt][lane][8] bf16 -> 1024 bf16x8 per K-step
    const bf16x8* Wf = reinterpret_cast<const bf16x8*>(a.w) + ((long)by * nchunk * NKC) * 1024 + (NW ? 0 : wave * 128) +
                       lane;
    const int wrow = NW ? wave * (BT / 4) : 0;  // this wave's first tile row
    auto wload = [&](bf16x8 (&w)[4], int kk) {  // [0, 1] hi of row tiles 0, 1; [2, 3] lo
        const bf16x8* p = Wf + (long)kk * 1024;
        w[0] = p[0];
        w[1] = p[64];
        w[2] = p[512];
        w[3] = p[576];
    };
    f32x4 acc[2][MT];
    bf16x8 wf[2][4];
    bf16x8 xh[MT], xl[MT];
    const float* X = reinterpret_cast<const float*>(a.x) + (long)bq * a.bsx;
    const int cv = tid & 15, rsub = tid >> 4;
    // the B-fragment row of lane l at tap 0 is (l & 15) (+ 16 mt): its swizzle at tap `tap` is ((l & 15) + tap dil) & 15
    const int g4 = lane >> 4;

    for (int cc = 0; cc < nchunk; ++cc) {
        const int kb = cc * NKC;
        wload(wf[0], kb);  // the chunk's first weight K-step flies during the staging
        __syncthreads();   // every wave is done reading the previous chunk's tiles and constants
        if (!(a.flags & 1)) {
            const int c = cc * 128 + cv * 8;
            const bool c_ok = c < a.Ci;  // vectors past Ci (ci_pad > Ci) are zero; weights there are 0
            const int cl = c_ok ? c : 0;
            if (tid < 128) {  // per-channel constants (fp32, the oracle's AdaIN folded into one affine)
                const int ch = cc * 128 + tid;
                const bool ok = ch < a.Ci;
                float sc = 0.f, sh = 0.f, kar = 0.f, kia = 0.f;
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
                if constexpr (PACT == STZS_ACT_SNAKE) {
                    const float al = ok ? a.pro_alpha[ch] : 1.f;
                    kar = al * 0.159154943091895336f;  // alpha / 2 pi: v_sin takes revolutions
                    kia = 1.f / al;
                }
                cs[tid] = sc;
                cs[128 + tid] = sh;
                cs[256 + tid] = kar;
                cs[384 + tid] = kia;
            }
            auto stage = [&](auto full_tag) {
                constexpr bool FULL = decltype(full_tag)::value;
                // row vectors loaded per group: all of them when the accumulators are not live (one chunk), half
                // otherwise (the multi-chunk forms stage chunk 2 beside 64 live accumulators)
                constexpr int G = NCH == 1 ? SB : (SB + 1) / 2;
                float4 raw[G][2];
                auto load_group = [&](int i0) {
#pragma unroll
                    for (int i = 0; i < G; ++i) {  // 32-bit offsets from the utterance base (SGPR)
                        if (i0 + i >= SB) break;
                        int tin = t0 - a.pad + rsub + 16 * (i0 + i);
                        if constexpr (!FULL) tin = tin < 0 ? 0 : (tin >= a.T_in ? a.T_in - 1 : tin);
                        const unsigned off = (unsigned)(tin * (int)a.ldx + cl) * 4u;
                        const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(X) + off);
                        raw[i][0] = p[0];
                        raw[i][1] = p[1];
                    }
                };
                load_group(0);
                __syncthreads();  // constants visible
                float ksc[8], ksh[8], kar[8], kia[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    ksc[j] = cs[cv * 8 + j];
                    ksh[j] = cs[128 + cv * 8 + j];
                    if constexpr (PACT == STZS_ACT_SNAKE) {
                        kar[j] = cs[256 + cv * 8 + j];
                        kia[j] = cs[384 + cv * 8 + j];
                    }
                }
                const float slope = a.pro_slope;
#pragma unroll
                for (int i = 0; i < SB; ++i) {
                    if (i > 0 && i % G == 0) load_group(i);
                    const int r = rsub + 16 * i;
                    const int ig = i % G;
                    const float xin[8] = {raw[ig][0].x, raw[ig][0].y, raw[ig][0].z, raw[ig][0].w,
                                          raw[ig][1].x, raw[ig][1].y, raw[ig][1].z, raw[ig][1].w};
                    float z[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float y = fmaf(xin[j], ksc[j], ksh[j]);
                        float v = y;
                        if constexpr (PACT == STZS_ACT_SNAKE) {
                            const float s = __builtin_amdgcn_sinf(y * kar[j]);
                            v = fmaf(s * s, kia[j], y);
                        } else if constexpr (PACT == STZS_ACT_LEAKY) {
                            v = y >= 0.f ? y : y * slope;
                        }
                        z[j] = v;
                    }
                    if constexpr (!FULL) {  // zero padding / channels past Ci
                        const int tin = t0 - a.pad + r;
                        const bool ok = c_ok && tin >= 0 && tin < a.T_in;
#pragma unroll
                        for (int j = 0; j < 8; ++j) z[j] = ok ? z[j] : 0.f;
                    }
                    uint4 hi, lo;
                    split8(z, hi, lo);
                    if (r < rows_in) {
                        const int o = r * PX + ((cv ^ (r & 15)) << 4);
                        *reinterpret_cast<uint4*>(thi + o) = hi;
                        *reinterpret_cast<uint4*>(thi + lo_off + o) = lo;
                    }
                }
            };
            const bool interior = t0 - a.pad >= 0 && t0 - a.pad + 16 * SB <= a.T_in && cc * 128 + 128 <= a.Ci;
            if (interior)
                stage(std::integral_constant<bool, true>{});
            else
                stage(std::integral_constant<bool, false>{});
        }
        __syncthreads();
        // K loop: no barrier.  K-step s = tap * 4 + kq reads input rows t + tap dil, channels kq * 32 ..
        // (the lane index laundered per chunk: otherwise hipcc hoists all NKC fragment offsets out of the chunk loop
        // of the multi-chunk forms and keeps them live -- 15-27 VGPRs spilled at k7 / k11)
        int lr = lane & 15;
        asm volatile("" : "+v"(lr));
        auto kloop = [&](auto first_tag) {
            constexpr bool FIRST = decltype(first_tag)::value;
            const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
            auto frag_off = [&](int s) {  // byte offset of this lane's B fragment (row tile 0) at K-step s
                const int tap = s >> 2, kq = s & 3;
                const int r = lr + tap * dil;
                return (wrow + r) * PX + ((((kq << 2) + g4) ^ (r & 15)) << 4);
            };
            {
                const int o = frag_off(0);
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    xh[mt] = *reinterpret_cast<const bf16x8*>(thi + o + mt * 16 * PX);
                    xl[mt] = *reinterpret_cast<const bf16x8*>(thi + lo_off + o + mt * 16 * PX);
                }
            }
#pragma unroll
            for (int s = 0; s < NKC; ++s) {
                if (s + 1 < NKC) wload(wf[(s + 1) & 1], kb + s + 1);
                const int on = s + 1 < NKC ? frag_off(s + 1) : 0;
                const bf16x8* w = wf[s & 1];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const bool z = FIRST && s == 0;
#pragma unroll
                    for (int j = 0; j < 2; ++j) {  // small products first: wl * zh, wh * zl, then wh * zh
                        acc[j][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2 + j], xh[mt], z ? zero : acc[j][mt], 0, 0, 0);
                        acc[j][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], xl[mt], acc[j][mt], 0, 0, 0);
                        acc[j][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], xh[mt], acc[j][mt], 0, 0, 0);
                    }
                    if (s + 1 < NKC) {
                        xh[mt] = *reinterpret_cast<const bf16x8*>(thi + on + mt * 16 * PX);
                        xl[mt] = *reinterpret_cast<const bf16x8*>(thi + lo_off + on + mt * 16 * PX);
                    }
                }
                if (s + 1 < NKC) {
                    __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);  // the next weight K-step's loads first
                }
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
                    if (s + 1 < NKC) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        if constexpr (NCH == 1) {
            kloop(std::integral_constant<bool, true>{});
        } else {
            if (cc == 0) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            kloop(std::integral_constant<bool, false>{});
        }
    }
    if (a.flags & 4) return;

    // ---------------- epilogue: lane (g, n): time t = t0 + mt*16 + n, channels co0 .. co0 + 7 (fp32)
    const int g = lane >> 4, n = lane & 15;
    const bool stat = a.stat_part != nullptr;
    constexpr bool TD1 = PACT == STZS_ACT_SNAKE;  // the MRF forms: res_tdiv 1 (checked by the launcher)
    const float* Rq = reinterpret_cast<const float*>(a.res) + (long)bq * a.bsr;
    const float* Aq = reinterpret_cast<const float*>(a.acc_in) + (long)bq * a.bsa;
    float* Y = reinterpret_cast<float*>(a.y) + (long)bq * a.bsy;
    const int nch = (a.T_out + 63) / 64;
    const int co0 = by * BCO + (NW ? 0 : wave * 32) + g * 8;
    const bool col_ok = co0 < a.Co;
    const int coc = col_ok ? co0 : 0;
    const int ncv = a.Co - co0 < 8 ? a.Co - co0 : 8;  // valid channels of this lane's group (NW: Co % 8 != 0)
    float bias[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) bias[i] = a.bias ? a.bias[(NW && i >= ncv) ? coc : coc + i] : 0.f;
    constexpr int MH = MT < 4 ? MT : 4;  // row tiles per epilogue pass
    constexpr int NH = MT / MH;          // (BT >= 64, not NW: 64-row halves, one statistics partial each)
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        // this half's residual / accumulate rows in flight at once (32-B fp32 row vectors)
        float4 rr[MH][2], aa[MH][2];
#pragma unroll
        for (int m = 0; m < MH; ++m) {
            const int t = t0 + wrow + (h * MH + m) * 16 + n;
            const int tc = t < a.T_out ? t : a.T_out - 1;
            if constexpr (HR) {
                const int tr = TD1 ? tc : tc / a.res_tdiv;
                const float4* p = reinterpret_cast<const float4*>(Rq + (long)tr * a.ldr + coc);
                rr[m][0] = p[0];
                rr[m][1] = p[1];
            }
            if constexpr (HA) {
                const float4* p = reinterpret_cast<const float4*>(Aq + (long)tc * a.lda + coc);
                aa[m][0] = p[0];
                aa[m][1] = p[1];
            }
        }
        float ss[8], sq[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) ss[i] = sq[i] = 0.f;
#pragma unroll
        for (int m = 0; m < MH; ++m) {
            const int mt = h * MH + m;
            const int t = t0 + wrow + mt * 16 + n;
            const bool ok = col_ok && t < a.T_out;
            float v[8];
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[nt * 4 + r] = acc[nt][mt][r] + bias[nt * 4 + r];
            if constexpr (HR) {
                const float f[8] = {rr[m][0].x, rr[m][0].y, rr[m][0].z, rr[m][0].w,
                                    rr[m][1].x, rr[m][1].y, rr[m][1].z, rr[m][1].w};
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] += f[i];
            }
            if constexpr (AL) {
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] *= a.alpha;
            }
            if constexpr (HA) {
                const float f[8] = {aa[m][0].x, aa[m][0].y, aa[m][0].z, aa[m][0].w,
                                    aa[m][1].x, aa[m][1].y, aa[m][1].z, aa[m][1].w};
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = fmaf(a.beta, f[i], v[i]);
            }
            if (ok) {
                if (!NW || ncv == 8) {
                    float4* p = reinterpret_cast<float4*>(Y + (long)t * a.ldy + coc);
                    p[0] = make_float4(v[0], v[1], v[2], v[3]);
                    p[1] = make_float4(v[4], v[5], v[6], v[7]);
                } else {
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        if (i < ncv) Y[(long)t * a.ldy + coc + i] = v[i];
                }
            }
            if (stat && ok) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    ss[i] += v[i];
                    sq[i] = fmaf(v[i], v[i], sq[i]);
                }
            }
        }
        if (!NW && stat) {
            row_sum16_n<8>(ss);
            row_sum16_n<8>(sq);
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

// ---------------------------------------------------------------------------------------------------------------
// FLAT linears of the precise pipeline (ks 1, no prologue but pro_cscale): 128 consecutive rows of the [B * T] row
// space per tile, the same split-operand K loop over 128-channel chunks (4 K-steps each), and the next chunk's fp32
// rows loaded into registers while the current chunk's K loop runs (every row a tile stages is a whole 512-B row
// piece: no halo).  Epilogue of the linears (csrc/conv_common.hpp epilogue, FLAT): bias, GELU / SiLU, the DiT gate of
// the row's utterance, residual, alpha, beta * acc_in; fp32 out.
template <int EACT, bool GATE, bool HR, bool HA>
__global__ __launch_bounds__(NTH, 2) void mrfx_lin(const stzs_conv_args a) {
    constexpr int BT = 128, MT = 8, NKC = 4, SB = 8;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* const thi = smem;
    constexpr int lo_off = BT * PX;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nx = gridDim.x;
    const int lin = (a.flags & STZS_CONV_LINEAR_IDS) ? blockIdx.y * nx + blockIdx.x
                                                      : xcd_remap(blockIdx.y * nx + blockIdx.x, nx * gridDim.y);
    const int by = lin / nx, bx = lin - by * nx;
    const long nR = (long)a.B * a.T_in;
    const long row0 = (long)bx * BT;
    const int nchunk = a.ci_pad >> 7;
    const bf16x8* Wf = reinterpret_cast<const bf16x8*>(a.w) + ((long)by * nchunk * NKC) * 1024 + wave * 128 + lane;
    auto wload = [&](bf16x8 (&w)[4], int kk) {
        const bf16x8* p = Wf + (long)kk * 1024;
        w[0] = p[0];
        w[1] = p[64];
        w[2] = p[512];
        w[3] = p[576];
    };
    const float* X = reinterpret_cast<const float*>(a.x);
    const int cv = tid & 15, rsub = tid >> 4;
    const int g4 = lane >> 4;
    // the A rows: flat row R -> utterance R / T_in, step R % T_in (any batch stride); rows past nR are clamped here and
    // zeroed in the transform
    const float invTi = 1.f / (float)a.T_in;
    unsigned xoff[SB];  // element offsets (the launcher checks B * bsx < 2^31)
#pragma unroll
    for (int i = 0; i < SB; ++i) {
        long R = row0 + rsub + 16 * i;
        R = R < nR ? R : nR - 1;
        const int q = (int)((float)(int)R * invTi);
        int qq = q, rr = (int)R - q * a.T_in;
        if (rr < 0) { --qq; rr += a.T_in; } else if (rr >= a.T_in) { ++qq; rr -= a.T_in; }
        xoff[i] = (unsigned)(qq * (int)a.bsx + rr * (int)a.ldx);
    }
    float4 raw[SB][2];
    auto load_chunk = [&](int cc) {
        const int c = cc * 128 + cv * 8;
        const int cl = c < a.Ci ? c : 0;
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            const float4* p = reinterpret_cast<const float4*>(X + xoff[i] + cl);
            raw[i][0] = p[0];
            raw[i][1] = p[1];
        }
    };
    f32x4 acc[2][MT];
    bf16x8 wf[2][4];
    bf16x8 xh[MT], xl[MT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    load_chunk(0);
    const float csc = a.pro_cscale;
    for (int cc = 0; cc < nchunk; ++cc) {
        const int kb = cc * NKC;
        wload(wf[0], kb);
        __syncthreads();  // every wave is done reading the previous chunk's tiles
        {
            const bool c_ok = cc * 128 + cv * 8 < a.Ci;
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                const int r = rsub + 16 * i;
                const bool ok = c_ok && row0 + r < nR;
                const float xin[8] = {raw[i][0].x, raw[i][0].y, raw[i][0].z, raw[i][0].w,
                                      raw[i][1].x, raw[i][1].y, raw[i][1].z, raw[i][1].w};
                float z[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) z[j] = ok ? xin[j] * csc : 0.f;
                uint4 hi, lo;
                split8(z, hi, lo);
                const int o = r * PX + ((cv ^ (r & 15)) << 4);
                *reinterpret_cast<uint4*>(thi + o) = hi;
                *reinterpret_cast<uint4*>(thi + lo_off + o) = lo;
            }
        }
        if (cc + 1 < nchunk) load_chunk(cc + 1);  // the next chunk's rows fly during this chunk's K loop
        __syncthreads();
        int lr = lane & 15;
        asm volatile("" : "+v"(lr));
        auto frag_off = [&](int s) { return lr * PX + (((s << 2) + g4) ^ lr) * 16; };
        {
            const int o = frag_off(0);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                xh[mt] = *reinterpret_cast<const bf16x8*>(thi + o + mt * 16 * PX);
                xl[mt] = *reinterpret_cast<const bf16x8*>(thi + lo_off + o + mt * 16 * PX);
            }
        }
#pragma unroll
        for (int s = 0; s < NKC; ++s) {
            if (s + 1 < NKC) wload(wf[(s + 1) & 1], kb + s + 1);
            const int on = s + 1 < NKC ? frag_off(s + 1) : 0;
            const bf16x8* w = wf[s & 1];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[j][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2 + j], xh[mt], acc[j][mt], 0, 0, 0);
                    acc[j][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], xl[mt], acc[j][mt], 0, 0, 0);
                    acc[j][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], xh[mt], acc[j][mt], 0, 0, 0);
                }
                if (s + 1 < NKC) {
                    xh[mt] = *reinterpret_cast<const bf16x8*>(thi + on + mt * 16 * PX);
                    xl[mt] = *reinterpret_cast<const bf16x8*>(thi + lo_off + on + mt * 16 * PX);
                }
            }
            if (s + 1 < NKC) __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
                if (s + 1 < NKC) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (a.flags & 4) return;

    // ---------------- epilogue: lane (g, n): flat row row0 + mt*16 + n, channels co0 .. co0 + 7 (fp32)
    const int g = lane >> 4, n = lane & 15;
    const int co0 = by * BCO + wave * 32 + g * 8;
    if (co0 >= a.Co) return;
    float bias[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) bias[i] = a.bias ? a.bias[co0 + i] : 0.f;
    const float invTo = 1.f / (float)a.T_out;
    const bool gvec = GATE && (reinterpret_cast<uintptr_t>(a.gate) & 15) == 0 && a.gate_bs % 4 == 0;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const long R = row0 + mt * 16 + n;
        if (R >= nR) continue;
        const long q = (long)(int)((float)(int)R * invTo);
        long b = q, t = R - q * a.T_out;
        if (t < 0) { --b; t += a.T_out; } else if (t >= a.T_out) { ++b; t -= a.T_out; }
        float v[8];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[nt * 4 + r] = acc[nt][mt][r] + bias[nt * 4 + r];
        if constexpr (EACT == STZS_ACT_GELU) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = 0.5f * v[i] * (1.f + erff(v[i] * 0.70710678118654752f));
        } else if constexpr (EACT == STZS_ACT_SILU) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = v[i] / (1.f + expf(-v[i]));
        }
        if constexpr (GATE) {
            const float* gp = a.gate + b * a.gate_bs + co0;
            float gv[8];
            if (gvec) {
                load8(gp, gv);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) gv[i] = gp[i];
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] *= gv[i];
        }
        if constexpr (HR) {
            float f[8];
            load8(reinterpret_cast<const float*>(a.res) + b * a.bsr + t * a.ldr + co0, f);
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] += f[i];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] *= a.alpha;
        if constexpr (HA) {
            float f[8];
            load8(reinterpret_cast<const float*>(a.acc_in) + b * a.bsa + t * a.lda + co0, f);
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = fmaf(a.beta, f[i], v[i]);
        }
        store8(reinterpret_cast<float*>(a.y) + b * a.bsy + t * a.ldy + co0, v);
    }
}

template <int EACT>
void (*pick_lin_e(bool g, bool r, bool h))(stzs_conv_args) {
    if (g) return r ? (h ? mrfx_lin<EACT, true, true, true> : mrfx_lin<EACT, true, true, false>)
                    : (h ? mrfx_lin<EACT, true, false, true> : mrfx_lin<EACT, true, false, false>);
    return r ? (h ? mrfx_lin<EACT, false, true, true> : mrfx_lin<EACT, false, true, false>)
             : (h ? mrfx_lin<EACT, false, false, true> : mrfx_lin<EACT, false, false, false>);
}
void (*pick_lin(const stzs_conv_args& a))(stzs_conv_args) {
    const bool g = a.gate != nullptr, r = a.res != nullptr, h = a.acc_in != nullptr;
    switch (a.epi_act) {
        case STZS_ACT_NONE: return pick_lin_e<STZS_ACT_NONE>(g, r, h);
        case STZS_ACT_GELU: return pick_lin_e<STZS_ACT_GELU>(g, r, h);
        case STZS_ACT_SILU: return pick_lin_e<STZS_ACT_SILU>(g, r, h);
        default: return nullptr;
    }
}

template <int PACT, bool HR, bool HA, int BT, int NCH, bool AL>
void (*pick_ks(int ks))(stzs_conv_args) {
    switch (ks) {
        case 3: return mrfx_conv<PACT, HR, HA, 3, BT, NCH, AL>;
        case 7: return mrfx_conv<PACT, HR, HA, 7, BT, NCH, AL>;
        case 11: return mrfx_conv<PACT, HR, HA, 11, BT, NCH, AL>;
        default: return nullptr;
    }
}
template <int PACT, bool HR, bool HA, int BT>
void (*pick(int ks, bool one, bool al))(stzs_conv_args) {
    if (al) return one ? pick_ks<PACT, HR, HA, BT, 1, true>(ks) : pick_ks<PACT, HR, HA, BT, 0, true>(ks);
    return one ? pick_ks<PACT, HR, HA, BT, 1, false>(ks) : pick_ks<PACT, HR, HA, BT, 0, false>(ks);
}
template <int BT>
void (*pick_form(const stzs_conv_args& a))(stzs_conv_args) {
    const bool R = a.res != nullptr, A = a.acc_in != nullptr;
    const bool one = a.ci_pad == 128;
    const bool al = a.alpha != 1.f;
    if (a.pro_act == STZS_ACT_SNAKE)
        return R ? (A ? pick<STZS_ACT_SNAKE, true, true, BT>(a.ks, one, al) : pick<STZS_ACT_SNAKE, true, false, BT>(a.ks, one, al))
                 : (A ? pick<STZS_ACT_SNAKE, false, true, BT>(a.ks, one, al) : pick<STZS_ACT_SNAKE, false, false, BT>(a.ks, one, al));
    // the AdaIN residual-block convs of the decoder / prosody predictor: k3, no accumulate input, alpha 1/sqrt 2 or 1
    if (A || a.ks != 3 || BT != 128) return nullptr;
    if (a.pro_act == STZS_ACT_LEAKY)
        return R ? (void (*)(stzs_conv_args))mrfx_conv<STZS_ACT_LEAKY, true, false, 3, 128, 0, true>
                 : (void (*)(stzs_conv_args))mrfx_conv<STZS_ACT_LEAKY, false, false, 3, 128, 0, true>;
    if (a.pro_act == STZS_ACT_NONE)
        return R ? (void (*)(stzs_conv_args))mrfx_conv<STZS_ACT_NONE, true, false, 3, 128, 0, true>
                 : (void (*)(stzs_conv_args))mrfx_conv<STZS_ACT_NONE, false, false, 3, 128, 0, true>;
    return nullptr;
}

}  // namespace

// the precise FLAT linear (ks 1): validated and launched by stzs_mrfx_conv_launch
static int mrfx_lin_launch(const stzs_conv_args& a, hipStream_t s) {
    if (a.pad || a.stride != 1 || a.T_in != a.T_out || a.pro_mode != STZS_PRO_NONE || a.pro_act != STZS_ACT_NONE ||
        a.stat_part || a.ups || a.refl || a.cic != 128 || a.ci_pad % 128 || a.Co % 8 || a.co_pad % BCO ||
        a.in_dtype != STZS_F32 || a.out_dtype != STZS_F32 || a.ldx % 8 || a.bsx % 8 || a.ldy % 8 || a.bsy % 8 ||
        (a.res && (a.ldr % 8 || a.bsr % 8 || a.res_tdiv != 1)) || (a.acc_in && (a.lda % 8 || a.bsa % 8)) ||
        (long)a.B * a.T_in >= (1L << 22) - 256 || (long)a.B * a.bsx >= (1L << 31))
        return STZS_ESHAPE;
    if (!stzs_aligned(a.x, 32) || !stzs_aligned(a.y, 32) || (a.res && !stzs_aligned(a.res, 32)) ||
        (a.acc_in && !stzs_aligned(a.acc_in, 32)))
        return STZS_EINVAL;
    void (*k)(stzs_conv_args) = pick_lin(a);
    if (!k) return STZS_EINVAL;
    const size_t lds = (size_t)2 * 128 * PX;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    dim3 grid((unsigned)(((long)a.B * a.T_in + 127) / 128), a.co_pad / BCO);
    hipLaunchKernelGGL(k, grid, dim3(NTH), lds, s, a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

// internal entry used by stzs_conv1d for STZS_CONV_W_FRAG32X3 weights (csrc/dispatch.hip)
__attribute__((visibility("hidden"))) int stzs_mrfx_conv_launch(const stzs_conv_args& a, hipStream_t s) {
    if (a.ks == 1) return mrfx_lin_launch(a, s);
    // conv_post (128 -> 22, k7, LeakyReLU(0.01), fp32 out): the narrow form, waves split the rows
    const bool narrow = a.Co <= 32 && a.ci_pad == 128 && a.ks == 7 && !a.res && !a.acc_in && !a.stat_part &&
                        a.pro_mode == STZS_PRO_NONE && a.pro_act == STZS_ACT_LEAKY && a.alpha == 1.f &&
                        128 + 6 * a.dil <= 16 * sb_rows(7, 128);
    if (a.stride != 1 || a.cic != 128 || a.ci_pad % 128 || (a.Co % 8 && !narrow) || a.co_pad % BCO || a.ups || a.refl || a.gate ||
        a.in_dtype != STZS_F32 || a.out_dtype != STZS_F32 || a.epi_act != STZS_ACT_NONE || a.ldx % 8 || a.bsx % 8 ||
        a.ldy % 8 || a.bsy % 8 || (a.res && (a.ldr % 8 || a.bsr % 8 || a.res_tdiv <= 0)) ||
        (a.acc_in && (a.lda % 8 || a.bsa % 8)) || (a.stat_part && a.stat_ld < a.Co) ||
        (a.ks != 3 && a.ks != 7 && a.ks != 11))
        return STZS_ESHAPE;
    if (!stzs_aligned(a.x, 32) || !stzs_aligned(a.y, 32) || (a.res && !stzs_aligned(a.res, 32)) ||
        (a.acc_in && !stzs_aligned(a.acc_in, 32)))
        return STZS_EINVAL;
    if (a.pro_act == STZS_ACT_SNAKE && !a.pro_alpha) return STZS_EINVAL;
    if (a.pro_act == STZS_ACT_SNAKE && a.res && a.res_tdiv != 1) return STZS_ESHAPE;  // (TD1 in the kernel)
    const int ks = a.ks;
    // 128-row tiles while the hi + lo tile pair of the halo'd rows fits two workgroups per CU, else 64-row tiles
    const int rows128 = 128 + (ks - 1) * a.dil, rows64 = 64 + (ks - 1) * a.dil;
    int bt = 0;
    if (rows128 <= 16 * sb_rows(ks, 128))
        bt = 128;
    else if (rows64 <= 16 * sb_rows(ks, 64))
        bt = 64;
    if (!bt) return STZS_ESHAPE;
    void (*k)(stzs_conv_args) = bt == 128 ? pick_form<128>(a) : pick_form<64>(a);
    if (narrow) k = mrfx_conv<STZS_ACT_LEAKY, false, false, 7, 128, 1, false, true>;
    if (!k) return STZS_ESHAPE;
    const int rows_in = bt + (ks - 1) * a.dil;
    const size_t lds = (size_t)2 * rows_in * PX + NCS * 128 * 4;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    dim3 grid((unsigned)a.B * (unsigned)((a.T_out + bt - 1) / bt), narrow ? 1u : (unsigned)(a.co_pad / BCO));
    hipLaunchKernelGGL(k, grid, dim3(NTH), lds, s, a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
