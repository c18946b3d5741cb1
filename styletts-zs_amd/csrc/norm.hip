// Normalisation statistics and row LayerNorm.
//
// stzs_chan_stats: InstanceNorm1d statistics per (b, c) over time for channels-last
// activations.  Pass 1 streams the tensor once with 16-B loads (8 channels per lane, rows split
// over the 8 row-lanes of a 256-thread block) and writes fp32 partial (sum, sumsq) per
// 256-row chunk; pass 2 combines the chunks in a fixed order in fp64 -> deterministic,
// bit-reproducible statistics (no float atomics).  HBM-bound: 1 read of the tensor.
//
// stzs_row_layernorm: one wave per row, values kept in registers, two-pass mean/variance
// (as torch.layer_norm), fused modulation  (gadd + G) * x_hat + Bt  and activation.
#include "common.hpp"
#include "rowln.hpp"

namespace {

constexpr int STAT_ROWS = 256;  // rows per partial chunk
constexpr int STAT_CG = 32;     // 8-channel vectors per block (256 channels)

template <typename T>
__global__ __launch_bounds__(256) void chan_stats_partial(const stzs_stats_args a, int nchunk) {
    __shared__ float red[8][STAT_CG * 8][2];
    const int tid = threadIdx.x, tx = tid & 31, ty = tid >> 5;
    const int chunk = blockIdx.x, b = blockIdx.y;
    const int cv = blockIdx.z * STAT_CG + tx;
    const int c = cv * 8;
    float s[8], q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
    const int r0 = chunk * STAT_ROWS, r1 = min(a.T, r0 + STAT_ROWS);
    const T* X = reinterpret_cast<const T*>(a.x) + (long)b * a.bs;
    if (c < a.C) {
        // four rows' 16-B loads in flight per pass, accumulated in row order (same sums as one row at a time)
        int r = r0 + ty;
        for (; r + 24 < r1; r += 32) {
            float v[4][8];
#pragma unroll
            for (int u = 0; u < 4; ++u) load8(X + (long)(r + 8 * u) * a.ld + c, v[u]);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    s[j] += v[u][j];
                    q[j] += v[u][j] * v[u][j];
                }
        }
        for (; r < r1; r += 8) {
            float v[8];
            load8(X + (long)r * a.ld + c, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                s[j] += v[j];
                q[j] += v[j] * v[j];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[ty][tx * 8 + j][0] = s[j];
        red[ty][tx * 8 + j][1] = q[j];
    }
    __syncthreads();
    // 256 threads: one channel of the block's 256 each
    const int cl = tid;
    const int cg = blockIdx.z * STAT_CG * 8 + cl;
    if (cg < a.C) {
        float ss = 0.f, qq = 0.f;
#pragma unroll
        for (int y = 0; y < 8; ++y) {
            ss += red[y][cl][0];
            qq += red[y][cl][1];
        }
        float* P = reinterpret_cast<float*>(a.partial);
        const long o = (((long)b * nchunk + chunk) * a.C + cg) * 2;
        P[o] = ss;
        P[o + 1] = qq;
    }
}

// pass 2: block = (utterance, 32 channels); 8 chunk groups stride over the chunks with coalesced
// 8-B (sum, sumsq) loads, fp64 sums, combined in fixed group order -> deterministic.
constexpr int FIN_CH = 32;
STZS_DEV void stats_final_body(const stzs_stats_args a, int nchunk, int b, int by) {
    __shared__ double red[8][FIN_CH][2];
    const int tid = threadIdx.x, cl = tid & (FIN_CH - 1), g = tid >> 5;
    const int c = by * FIN_CH + cl;
    double s = 0.0, q = 0.0;
    if (c < a.C) {
        const float2* P = reinterpret_cast<const float2*>(a.partial) + (long)b * nchunk * a.C + c;
        int k = g;
        for (; k + 24 < nchunk; k += 32) {  // four independent loads in flight per iteration
            float2 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = P[(long)(k + 8 * u) * a.C];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                s += (double)v[u].x;
                q += (double)v[u].y;
            }
        }
        for (; k < nchunk; k += 8) {
            const float2 v = P[(long)k * a.C];
            s += (double)v.x;
            q += (double)v.y;
        }
    }
    red[g][cl][0] = s;
    red[g][cl][1] = q;
    __syncthreads();
    if (tid < FIN_CH && c < a.C) {
        s = q = 0.0;
#pragma unroll
        for (int y = 0; y < 8; ++y) {
            s += red[y][tid][0];
            q += red[y][tid][1];
        }
        float mu, rs;
        stat_finish(s, q, a.T, a.eps, mu, rs);  // (common.hpp: the same rounding as the conv prologue's pro_part path)
        a.mean[(long)b * a.stat_bs + c] = mu;
        a.rstd[(long)b * a.stat_bs + c] = rs;
    }
}

__global__ __launch_bounds__(256) void chan_stats_final(const stzs_stats_args a, int nchunk) {
    stats_final_body(a, nchunk, blockIdx.x, blockIdx.y);
}

// (r06) up to three independent finalisations in one launch (grid z = problem): each block runs the body above for
// its own problem, so every mean / rstd has the bits of its own chan_stats_final launch
struct StatsGroup {
    stzs_stats_args a[3];
    int nchunk[3];
};
__global__ __launch_bounds__(256) void chan_stats_final_group(const StatsGroup g) {
    const int z = blockIdx.z;
    const stzs_stats_args& a = z == 0 ? g.a[0] : (z == 1 ? g.a[1] : g.a[2]);
    if ((int)blockIdx.x >= a.B || (int)blockIdx.y * FIN_CH >= a.C) return;  // (uniform per block)
    stats_final_body(a, z == 0 ? g.nchunk[0] : (z == 1 ? g.nchunk[1] : g.nchunk[2]), blockIdx.x, blockIdx.y);
}


template <typename TI, typename TO>
__global__ __launch_bounds__(256) void row_ln(const stzs_rowln_args a) {
    const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= a.R) return;
    stzs_ln::row_ln_one<TI, TO>(a, r, threadIdx.x & 63);
}

__global__ __launch_bounds__(256) void quant_rows(const stzs_quant_args a) {
    constexpr int MAXV = 4;
    const int lane = threadIdx.x & 63;
    const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= a.R) return;
    const bf16_t* X = reinterpret_cast<const bf16_t*>(a.x) + r * a.ldx;
    const int nv = a.C >> 3;
    float v[MAXV][8];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        const int vi = lane + i * 64;
        if (vi < nv) {
            load8(X + vi * 8, v[i]);
#pragma unroll
            for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[i][j]));
        }
    }
    stzs_ln::store_f8_row(reinterpret_cast<f8_t*>(a.y) + r * a.ldy, v, nv, lane, amax, a.scale + r);
}

}  // namespace

extern "C" size_t stzs_chan_stats_workspace(int B, int T, int C) {
    const int nchunk = (T + STAT_ROWS - 1) / STAT_ROWS;
    return (size_t)B * nchunk * C * 2 * sizeof(float);
}

static int chan_stats_pass1(const stzs_stats_args* a, hipStream_t s, int* nchunk_out) {
    if (a->B <= 0 || a->T <= 0 || a->C <= 0 || a->ld % 8 || a->bs % 8 || a->ld < a->C) return STZS_ESHAPE;
    if (a->C % 8) return STZS_ESHAPE;
    const int nchunk = (a->T + STAT_ROWS - 1) / STAT_ROWS;
    dim3 g1(nchunk, a->B, (a->C + STAT_CG * 8 - 1) / (STAT_CG * 8));
    if (a->dtype == STZS_BF16)
        hipLaunchKernelGGL(chan_stats_partial<bf16_t>, g1, dim3(256), 0, s, *a, nchunk);
    else if (a->dtype == STZS_F32)
        hipLaunchKernelGGL(chan_stats_partial<float>, g1, dim3(256), 0, s, *a, nchunk);
    else
        return STZS_EDTYPE;
    *nchunk_out = nchunk;
    return STZS_OK;
}

extern "C" int stzs_chan_stats_partial(const stzs_stats_args* a, void* stream) {
    if (!a || !a->x || !a->partial) return STZS_EINVAL;
    int nchunk = 0;
    const int rc = chan_stats_pass1(a, reinterpret_cast<hipStream_t>(stream), &nchunk);
    if (rc != STZS_OK) return rc;
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_chan_stats(const stzs_stats_args* a, void* stream) {
    if (!a || !a->x || !a->mean || !a->rstd || !a->partial) return STZS_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int nchunk = 0;
    const int rc = chan_stats_pass1(a, s, &nchunk);
    if (rc != STZS_OK) return rc;
    STZS_LAUNCH_CHECK();
    hipLaunchKernelGGL(chan_stats_final, dim3(a->B, (a->C + FIN_CH - 1) / FIN_CH), dim3(256), 0, s, *a, nchunk);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_chan_stats_final(const stzs_stats_args* a, int chunk_rows, void* stream) {
    if (!a || !a->mean || !a->rstd || !a->partial) return STZS_EINVAL;
    if (a->B <= 0 || a->T <= 0 || a->C <= 0 || chunk_rows <= 0) return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int nchunk = (a->T + chunk_rows - 1) / chunk_rows;
    hipLaunchKernelGGL(chan_stats_final, dim3(a->B, (a->C + FIN_CH - 1) / FIN_CH), dim3(256), 0, s, *a, nchunk);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_chan_stats_final_group(const stzs_stats_args* a, int n, int chunk_rows, void* stream) {
    if (!a || n < 1 || n > 3 || chunk_rows <= 0) return STZS_EINVAL;
    StatsGroup g = {};
    int gx = 0, gy = 0;
    for (int i = 0; i < n; ++i) {
        if (!a[i].mean || !a[i].rstd || !a[i].partial) return STZS_EINVAL;
        if (a[i].B <= 0 || a[i].T <= 0 || a[i].C <= 0) return STZS_ESHAPE;
        g.a[i] = a[i];
        g.nchunk[i] = (a[i].T + chunk_rows - 1) / chunk_rows;
        gx = a[i].B > gx ? a[i].B : gx;
        const int ny = (a[i].C + FIN_CH - 1) / FIN_CH;
        gy = ny > gy ? ny : gy;
    }
    hipLaunchKernelGGL(chan_stats_final_group, dim3(gx, gy, n), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), g);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_row_layernorm(const stzs_rowln_args* a, void* stream) {
    if (!a || !a->x || !a->y) return STZS_EINVAL;
    if (a->R <= 0 || a->C <= 0 || a->C % 8 || a->C > 2048 || a->ldx % 8 || a->ldy % 8 || a->gdiv <= 0)
        return STZS_ESHAPE;
    if ((a->G && (a->gs % 8 || !stzs_aligned(a->G, 32))) || (a->Bt && (a->bs % 8 || !stzs_aligned(a->Bt, 32))))
        return STZS_ESHAPE;  // modulation rows are read as 32-B vectors
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    dim3 g((a->R + 3) / 4);
    if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16)
        hipLaunchKernelGGL((row_ln<bf16_t, bf16_t>), g, dim3(256), 0, s, *a);
    else if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16)
        hipLaunchKernelGGL((row_ln<float, bf16_t>), g, dim3(256), 0, s, *a);
    else if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F32)
        hipLaunchKernelGGL((row_ln<float, float>), g, dim3(256), 0, s, *a);
    else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32)
        hipLaunchKernelGGL((row_ln<bf16_t, float>), g, dim3(256), 0, s, *a);
    else if (a->out_dtype == STZS_F8 && (!a->y_scale || a->ldy % 16))
        return STZS_EINVAL;
    else if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F8)
        hipLaunchKernelGGL((row_ln<float, f8_t>), g, dim3(256), 0, s, *a);
    else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F8)
        hipLaunchKernelGGL((row_ln<bf16_t, f8_t>), g, dim3(256), 0, s, *a);
    else
        return STZS_EDTYPE;
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_quant_rows(const stzs_quant_args* a, void* stream) {
    if (!a || !a->x || !a->y || !a->scale) return STZS_EINVAL;
    if (a->R <= 0 || a->C <= 0 || a->C % 8 || a->C > 2048 || a->ldx % 8 || a->ldy % 16 || a->ldy < a->C)
        return STZS_ESHAPE;
    if (!stzs_aligned(a->x, 16) || !stzs_aligned(a->y, 16)) return STZS_EINVAL;
    hipLaunchKernelGGL(quant_rows, dim3((a->R + 3) / 4), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), *a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
