// Sampler glue and small utilities + library entry points.
//   stzs_dn_cond      c = silu(pooled prompt + sigma embedding)        (adaLN-single input)
//   stzs_adaln_expand per-layer modulation = shared + table[l] (+1 on scale chunks)
//   stzs_cfg_euler    fused classifier-free guidance combine + Euler step, fp32 state
//   stzs_state_init   x0 = eps * sigma_0 for the (duplicated) CFG state
//   stzs_mean_rows    pooled style / prompt vectors
//   stzs_copy2d       strided row copy with dtype conversion (buffer assembly, no torch ops)
//   stzs_embed        token embedding rows (text front end)
#include "common.hpp"
#include "cfg.hpp"

namespace {

// c[s][r][j] = silu(pool[r][j] + temb[s][j]) for all sampler steps s at once
template <typename TO>
__global__ void dn_cond_kernel(const float* pool, const float* temb, TO* c, int R, int D, int steps) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    const long rd = (long)R * D;
    if (i >= rd * steps) return;
    const int s = (int)(i / rd);
    const long rj = i - s * rd;
    const int j = (int)(rj % D);
    const float x = pool[rj] + temb[(long)s * D + j];
    DT<TO>::st(c + i, x / (1.f + expf(-x)));
}

__global__ void adaln_expand_kernel(const float* mod, const float* table, float* out, int R, int D, int nchunk,
                                    int nlayers, unsigned mask) {
    const long W = (long)nchunk * D;
    const long n = (long)nlayers * R * W;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const long l = i / (R * W);
    const long rem = i - l * R * W;
    const long j = rem % W;
    float v = mod[rem];
    if (table) v += table[l * W + j];
    if ((mask >> (j / D)) & 1u) v += 1.f;
    out[i] = v;
}

__global__ void cfg_euler_kernel(float* x, const float* D, int B, int N, int cfg, float s, float s0, float dsig) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)B * N) return;
    const float xn = stzs_cfg_euler_elem(x[i], D[i], cfg ? D[(long)B * N + i] : 0.f, cfg, s, s0, dsig);
    x[i] = xn;
    if (cfg) x[(long)B * N + i] = xn;
}

__global__ void state_init_kernel(float* x, const float* eps, int B, int N, int cfg, float sigma) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)B * N) return;
    const float v = eps[i] * sigma;
    x[i] = v;
    if (cfg) x[(long)B * N + i] = v;
}

__global__ void mean_rows_kernel(const float* x, float* y, int B, int L, long ldx, long bsx, int c0, int C,
                                 long ldy) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)B * C) return;
    const int b = (int)(i / C), c = (int)(i - (long)b * C);
    // 8 rows' loads in flight at a time, summed in row order (the serial loop waited on each load in turn)
    const float* X = x + b * bsx + c0 + c;
    float s = 0.f;
    int l = 0;
    for (; l + 8 <= L; l += 8) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = X[(long)(l + j) * ldx];
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; l < L; ++l) s += X[(long)l * ldx];
    y[b * ldy + c] = s / L;
}

template <typename TI, typename TO>
__global__ void copy_kernel(const stzs_copy_args a) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    const long n = (long)a.B * a.R * a.C;
    if (i >= n) return;
    const long c = i % a.C;
    const long rr = (i / a.C) % a.R;
    const long b = i / ((long)a.C * a.R);
    const float v = DT<TI>::ld(reinterpret_cast<const TI*>(a.x) + b * a.bsx + rr * a.ldx + c);
    DT<TO>::st(reinterpret_cast<TO*>(a.y) + b * a.bsy + rr * a.ldy + c, v);
}

template <typename TO>
__global__ void embed_kernel(const int32_t* tok, const float* emb, TO* y, int B, int T, int D, long ldy) {
    const int t = blockIdx.x, b = blockIdx.y;
    const int id = tok[(long)b * T + t];
    const float* e = emb + (long)id * D;
    TO* o = y + ((long)b * T + t) * ldy;
    for (int c = threadIdx.x; c < D; c += 256) DT<TO>::st(o + c, e[c]);
}

inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

extern "C" int stzs_dn_cond(const float* pool, const float* temb, void* c, int R, int D, void* stream) {
    if (!pool || !temb || !c) return STZS_EINVAL;
    if (R <= 0 || D <= 0) return STZS_ESHAPE;
    hipLaunchKernelGGL(dn_cond_kernel<bf16_t>, dim3(nblk((long)R * D)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       pool, temb, reinterpret_cast<bf16_t*>(c), R, D, 1);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_dn_cond_steps(const float* pool, const float* temb, void* c, int R, int D, int steps,
                                  void* stream) {
    if (!pool || !temb || !c) return STZS_EINVAL;
    if (R <= 0 || D <= 0 || steps <= 0) return STZS_ESHAPE;
    hipLaunchKernelGGL(dn_cond_kernel<bf16_t>, dim3(nblk((long)R * D * steps)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), pool, temb, reinterpret_cast<bf16_t*>(c), R, D, steps);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_dn_cond_steps_f32(const float* pool, const float* temb, float* c, int R, int D, int steps,
                                      void* stream) {
    if (!pool || !temb || !c) return STZS_EINVAL;
    if (R <= 0 || D <= 0 || steps <= 0) return STZS_ESHAPE;
    hipLaunchKernelGGL(dn_cond_kernel<float>, dim3(nblk((long)R * D * steps)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), pool, temb, c, R, D, steps);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_adaln_expand(const float* mod, const float* table, float* out, int R, int D, int nchunk,
                                 int nlayers, unsigned scale_mask, void* stream) {
    if (!mod || !out) return STZS_EINVAL;
    if (R <= 0 || D <= 0 || nchunk <= 0 || nchunk > 32 || nlayers <= 0) return STZS_ESHAPE;
    hipLaunchKernelGGL(adaln_expand_kernel, dim3(nblk((long)nlayers * R * nchunk * D)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), mod, table, out, R, D, nchunk, nlayers, scale_mask);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_cfg_euler(float* x, const float* D, int B, int N, int cfg, float scale, float s0, float dsig,
                              void* stream) {
    if (!x || !D) return STZS_EINVAL;
    if (B <= 0 || N <= 0 || !(s0 > 0.f)) return STZS_ESHAPE;
    hipLaunchKernelGGL(cfg_euler_kernel, dim3(nblk((long)B * N)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       x, D, B, N, cfg, scale, s0, dsig);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_state_init(float* x, const float* eps, int B, int N, int cfg, float sigma, void* stream) {
    if (!x || !eps) return STZS_EINVAL;
    if (B <= 0 || N <= 0) return STZS_ESHAPE;
    hipLaunchKernelGGL(state_init_kernel, dim3(nblk((long)B * N)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), x, eps, B, N, cfg, sigma);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_mean_rows(const float* x, float* y, int B, int L, int64_t ldx, int64_t bsx, int c0, int C,
                              int64_t ldy, void* stream) {
    if (!x || !y) return STZS_EINVAL;
    if (B <= 0 || L <= 0 || C <= 0) return STZS_ESHAPE;
    hipLaunchKernelGGL(mean_rows_kernel, dim3(nblk((long)B * C)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       x, y, B, L, (long)ldx, (long)bsx, c0, C, (long)ldy);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_copy2d(const stzs_copy_args* a, void* stream) {
    if (!a || !a->x || !a->y) return STZS_EINVAL;
    if (a->B <= 0 || a->R <= 0 || a->C <= 0) return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    dim3 g(nblk((long)a->B * a->R * a->C));
    if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F32)
        hipLaunchKernelGGL((copy_kernel<float, float>), g, dim3(256), 0, s, *a);
    else if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16)
        hipLaunchKernelGGL((copy_kernel<float, bf16_t>), g, dim3(256), 0, s, *a);
    else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16)
        hipLaunchKernelGGL((copy_kernel<bf16_t, bf16_t>), g, dim3(256), 0, s, *a);
    else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32)
        hipLaunchKernelGGL((copy_kernel<bf16_t, float>), g, dim3(256), 0, s, *a);
    else
        return STZS_EDTYPE;
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_embed(const int32_t* tok, const float* emb, void* y, int B, int T, int D, int64_t ldy,
                          void* stream) {
    if (!tok || !emb || !y) return STZS_EINVAL;
    if (B <= 0 || T <= 0 || D <= 0) return STZS_ESHAPE;
    hipLaunchKernelGGL(embed_kernel<bf16_t>, dim3(T, B), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), tok, emb,
                       reinterpret_cast<bf16_t*>(y), B, T, D, (long)ldy);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_embed_f32(const int32_t* tok, const float* emb, float* y, int B, int T, int D, int64_t ldy,
                              void* stream) {
    if (!tok || !emb || !y) return STZS_EINVAL;
    if (B <= 0 || T <= 0 || D <= 0) return STZS_ESHAPE;
    hipLaunchKernelGGL(embed_kernel<float>, dim3(T, B), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), tok, emb,
                       y, B, T, D, (long)ldy);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_init(int device) {
    if (hipSetDevice(device) != hipSuccess) return STZS_EHIP;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) return STZS_EHIP;
    if (strncmp(p.gcnArchName, "gfx950", 6) != 0) return STZS_EINVAL;  // built for CDNA4 only
    return STZS_OK;
}

extern "C" int stzs_version(void) { return 1; }

extern "C" const char* stzs_strerror(int code) {
    switch (code) {
        case STZS_OK: return "ok";
        case STZS_EINVAL: return "STZS_EINVAL: invalid argument (null pointer, enum or alignment)";
        case STZS_ESHAPE: return "STZS_ESHAPE: shape or stride violation";
        case STZS_EDTYPE: return "STZS_EDTYPE: unsupported dtype combination";
        case STZS_EHIP: return "STZS_EHIP: HIP runtime error";
        default: return "unknown stzs error";
    }
}
