// LSTM recurrence of the prosody predictor: the 3 DurationEncoder
// BiLSTMs, the duration LSTM and the shared F0/N LSTM — 520 dependent steps per 5-s utterance.
//
// The input projection x W_ih^T + b is one MFMA GEMM over all steps (stzs_conv1d); this kernel
// runs only the sequential part, latency-bound by construction.  Design (weights never move):
//   * per (direction, group of <= 64 utterances) the 4H gate columns are split over P = H/32
//     workgroups; workgroup p owns hidden units [32p, 32p + 32) = 128 gate columns, and each of its
//     4 waves keeps ITS gate's 2 x (H/32) W_hh^T B-fragments in REGISTERS for the whole launch;
//   * per step: h_{t-1} [<=64 x H] (bf16) is read from a double-buffered exchange slab with
//     16-B write-through (sc1) buffer loads, all in flight at once, into an LDS A tile; 16x16x32
//     MFMAs give the gate pre-activations (8 waves: two per gate, each half of the row tiles), gates
//     meet in LDS, each of the 512 threads updates 4 (utterance, unit) cells (c in registers;
//     sigmoid / tanh from v_exp + v_rcp) and publishes its h with one 8-B write-through store
//     (data-tagged granules -- Guideline 16 R2 -- measured slower: 64 KB re-swept per step);
//   * hand-off (MI355X guide, Guideline 16 'Valid forms' table row 1): every storing wave drains
//     vmcnt(0), workgroup barrier, ONE lane adds to the direction's agent-scope arrival counter;
//     consumers poll that counter with sc1 loads, then all loads of the slab are sc1 (no fences).
//     Spins are bounded: on timeout the kernel records an error word and finishes (never hangs).
// Residency: grid = P x ndir x groups <= 64 workgroups, one per CU: always co-resident on MI355X.
// SMALL BATCHES (a group of <= TAG_ROWS utterances, bf16 mode -- configs[1] runs at batch 1): h travels as
// data-tagged granules instead (MI355X guide Guideline 16 R2, payload <= 4 KB): the cell update is mapped one GATE per
// lane (quad = unit: the g = 0 lane gathers f / g / o by DPP), and even units publish their h pair as one 8-B
// {tag = step + 1, bf16 pair} word with an agent-scope atomic store, and the consumers sweep
// the granules until every tag matches -- one fabric round trip per step instead of drain + counter + poll +
// slab load.  The granule region (the first TAG_BYTES of the workspace) starts zeroed and every call leaves it
// zeroed (the last workgroup to finish resets it), so a tag can only match a value of the current call.
// PRECISE (stzs_lstm_args.precise, the split-operand mode): h travels as hi = bf16(h) and lo = bf16(h - hi)
// (one slab row = hi[H] | lo[H]), W_hh^T as hi and lo fragments, the recurrent product is
// h_lo W_hi + h_hi W_lo + h_hi W_hi on the same MFMAs (~fp32 accuracy), the gates use libm expf / tanhf,
// and y is written in fp32.
#include "common.hpp"

namespace {

constexpr int MROWS = 64;   // utterances per group at most (4 MFMA row tiles): the slab / LDS capacity of a group
constexpr int UNITS = 32;   // hidden units per workgroup
constexpr unsigned SPIN_LIMIT = 1u << 22;
constexpr int TAG_ROWS = 2;  // groups with <= TAG_ROWS valid rows use granules (32: bench -3%, the sweep's bytes)
constexpr int TAG_BYTES = 2 * 2 * TAG_ROWS * (256 / 2) * 8;  // [dir][parity][row][H/2] u64, H <= 256

typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

STZS_DEV unsigned poll_ge(gu32* ctr, unsigned target, gu32* err, gu32* status, unsigned limit) {
    unsigned v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (v < target) {
        __builtin_amdgcn_s_sleep(1);
        v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (++spins > limit) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (status) __hip_atomic_fetch_or(status, STZS_STATUS_LSTM_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return 0;
        }
    }
    return 1;
}

// gate activations and the cell update with every rounding pinned (no contraction choice left to hipcc): the
// batch-1 cell map below computes them in other lanes and in another order than the counter form, and both must give
// the same bits (a batch of 1 == the same utterance inside a larger batch, test_latency_engine_batch_invariant)
STZS_DEV float fast_sigmoid(float x) { return __builtin_amdgcn_rcpf(__fadd_rn(1.f, __expf(-x))); }
STZS_DEV float fast_tanh(float x) { return fmaf(-2.f, __builtin_amdgcn_rcpf(__fadd_rn(1.f, __expf(2.f * x))), 1.f); }
STZS_DEV float cell_c(float ig, float fg, float tg, float c) { return fmaf(fg, c, __fmul_rn(ig, tg)); }
STZS_DEV float cell_h(float og, float c) { return __fmul_rn(og, fast_tanh(c)); }
template <int CTRL>
STZS_DEV float dpp_f(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

STZS_DEV float acc_sigmoid(float x) { return 1.f / (1.f + expf(-x)); }

// GR: utterances per group (16 / 32 / 64, lstm_group_rows: more workgroups, less MFMA / h-load / cell work per step
// and group; every row's gate chain and cell update are the same, so the result does not depend on GR)
// PAIRED launches (stzs_lstm_pair): two independent recurrences of one shape class (same H, group height,
// directions, mode; own gates, weights, T, outputs and exchange state) share the grid -- z < nz0 is the first,
// z >= nz0 the second -- so they run side by side whatever the stream / graph runtime does with concurrent branches
template <int NKS, bool PR, int GR = MROWS>
__global__ __launch_bounds__(512, 1) void lstm_xchg(const stzs_lstm_args a0, const stzs_lstm_args a1, const int nz0) {
    const bool second = (int)blockIdx.z >= nz0;  // uniform per workgroup
    const stzs_lstm_args& a = second ? a1 : a0;
    const int nz = second ? (int)gridDim.z - nz0 : nz0;  // this recurrence's groups
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int H = a.H, G4 = 4 * H;
    const int hp = H + 8;
    constexpr int NH = PR ? 2 : 1;  // slab row = hi[H] (| lo[H])
    bf16_t* As = reinterpret_cast<bf16_t*>(smem);                                   // [NH][64][hp]
    float* gs = reinterpret_cast<float*>(smem + ((NH * MROWS * hp * 2 + 15) & ~15)); // [64][4*UNITS + 4]
    __shared__ int s_ok, s_last;
    const int gp = 4 * UNITS + 4;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int gate = wave & 3, mh = wave >> 2;  // 8 waves: two per gate, each half of the row tiles
    const int p = blockIdx.x, dir = blockIdx.y, grp = (int)blockIdx.z - (second ? nz0 : 0);
    const int P = H / UNITS;
    const int b0 = grp * GR;
    const int nrows = min(GR, a.B - b0);
    const int nmt = (nrows + 15) >> 4;
    // exchange slab [group][dir][2][GR][NH H] bf16, counters [group][dir] (16 words apart)
    bf16_t* X = reinterpret_cast<bf16_t*>(reinterpret_cast<unsigned char*>(a.xchg) + TAG_BYTES) +
                ((long)(grp * a.ndir + dir) * 2) * GR * NH * H;
    const bool tagged = !PR && nrows <= TAG_ROWS;  // uniform: the group's row count
    gu64* gran = (gu64*)(a.xchg) + dir * 2 * TAG_ROWS * (H / 2);  // this direction's [parity][row][H/2] granules
    gu32* ctr = (gu32*)(a.sync) + (grp * a.ndir + dir) * 16;
    // the slab through a buffer descriptor: 16-B write-through (sc1, aux 16) stores and loads
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(X, 0, 2 * GR * NH * H * 2, 0x00020000);
    gu32* err = (gu32*)(a.sync) + 1023;
    gu32* status = (gu32*)a.status;
    const unsigned limit = a.spin_limit ? a.spin_limit : SPIN_LIMIT;

    // W_hh^T fragments of this wave's gate (g = wave) for the workgroup's 32 units, in registers
    const bf16_t* Wd = reinterpret_cast<const bf16_t*>(a.whhT) + (long)dir * (G4 / 16) * NKS * 512;
    bf16x8 bw[2][NKS], bwl[PR ? 2 : 1][PR ? NKS : 1];
    const long lo_off = (long)2 * (G4 / 16) * NKS * 512;  // PR: the lo fragments follow both directions' hi ones
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int ct = (gate * H + p * UNITS) / 16 + c;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            bw[c][ks] = *reinterpret_cast<const bf16x8*>(Wd + ((long)ct * NKS + ks) * 512 + lane * 8);
            if constexpr (PR) bwl[c][ks] = *reinterpret_cast<const bf16x8*>(Wd + lo_off + ((long)ct * NKS + ks) * 512 + lane * 8);
        }
    }
    // cells of this thread: row = tid / 8, units (tid % 8) * 4 .. +4
    constexpr int CPT = 4;
    const int crow = tid >> 3, cu0 = (tid & 7) * CPT;
    const bool cvalid = crow < nrows;
    const int cb = b0 + (cvalid ? crow : 0);
    float c[CPT];
    float c1 = 0.f;  // the tagged (batch <= 2) cell map's one cell per quad
#pragma unroll
    for (int j = 0; j < CPT; ++j) c[j] = 0.f;
    bf16_t* Y = reinterpret_cast<bf16_t*>(a.y);
    float* Yf = reinterpret_cast<float*>(a.y);
    if (tid == 0) s_ok = 1;

#ifdef STZS_LSTM_PROF
    unsigned long long pt[6] = {0, 0, 0, 0, 0, 0}, tp = 0;
#define PROF(i) if (tid == 0 && p == 0 && dir == 0) { unsigned long long n_ = __builtin_amdgcn_s_memtime(); if (i) pt[i] += n_ - tp; tp = n_; }
#else
#define PROF(i)
#endif
    for (int s = 0; s < a.T; ++s) {
        PROF(0)
        const int t = dir == 0 ? s : a.T - 1 - s;
        // gate input projections of this thread's cells (issued early, consumed after the MFMAs)
        float4 gx[4];
        float gxs = 0.f;  // tagged (batch <= 2): this lane's one gate input (the batch-1 cell map below)
        if (tagged) {
            if (tid < nrows * 128) {
                const int row = tid >> 7, u = (tid >> 2) & 31, g = tid & 3;
                gxs = a.gx[(long)(b0 + row) * a.bsg + (long)t * a.ldg + dir * G4 + g * H + p * UNITS + u];
            }
        } else {
            const float* G = a.gx + (long)cb * a.bsg + (long)t * a.ldg + dir * G4 + p * UNITS + cu0;
#pragma unroll
            for (int g = 0; g < 4; ++g) gx[g] = *reinterpret_cast<const float4*>(G + g * H);
        }
        // ---- wait for h_{s-1} from all P workgroups, stage it into the A tile ----
        if (s == 0) {
            for (int e = tid; e < NH * MROWS * hp / 8; e += 512) reinterpret_cast<uint4*>(As)[e] = make_uint4(0, 0, 0, 0);
        } else if (tagged) {
            // sweep h_{s-1}'s granules (tag s) straight into the A tile: no counter, no fence
            const gu64* src = gran + ((s - 1) & 1) * TAG_ROWS * (H / 2);
            const int ng = nrows * (H / 2);
            constexpr int GPT = (TAG_ROWS * 128 + 511) / 512;  // granules per thread, all loads in flight first
            unsigned long long xg[GPT];
#pragma unroll
            for (int i = 0; i < GPT; ++i)
                if (tid + i * 512 < ng) xg[i] = __hip_atomic_load(src + tid + i * 512, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int i = 0; i < GPT; ++i) {
                const int e = tid + i * 512;
                if (e >= ng) break;
                unsigned long long x = xg[i];
                unsigned spins = 0;
                while ((unsigned)(x >> 32) != (unsigned)s && s_ok) {
                    __builtin_amdgcn_s_sleep(1);
                    x = __hip_atomic_load(src + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (++spins > limit) {  // record, stop spinning for the rest of the call (never hang)
                        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (status) __hip_atomic_fetch_or(status, STZS_STATUS_LSTM_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        s_ok = 0;
                    }
                }
                const int r = e / (H / 2), k = (e - r * (H / 2)) * 2;
                *reinterpret_cast<unsigned*>(As + r * hp + k) = (unsigned)x;
            }
        } else {
            if (tid == 0 && s_ok) s_ok = poll_ge(ctr, (unsigned)(P * s), err, status, limit);  // after a timeout: no more spins
            PROF(1)
            __syncthreads();
            // h_{s-1}: MROWS x H bf16 = H/8 16-B words per row, all of this thread's sc1 loads in flight
            const int base = ((s - 1) & 1) * GR * NH * H * 2;
            constexpr int NWT = GR * NH * NKS * 32 / 8;        // 16-B words of h (H = 32 NKS)
            constexpr int NW = (NWT + 511) / 512;              // per thread
            // only the group's valid rows (a batch-1 group moves 1/64 of the slab); rows >= nrows of the A
            // tile stay as zeroed at s = 0 and only feed gate rows no cell reads
            const int nwt = nrows * (NH * NKS * 32 / 8);
            u32x4 v[NW];
#pragma unroll
            for (int i = 0; i < NW; ++i)  // uniform guard; the modulo keeps every address inside the rows
                if (i * 512 < nwt) v[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, base + ((tid + i * 512) % nwt) * 16, 0, 16);
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int e = tid + i * 512, r = (e * 8) / (NH * H), k = (e * 8) - r * (NH * H);
                const int hl = PR ? (k >= H) : 0;  // PR: lo half of the slab row -> the lo tile
                if (e < nwt) *reinterpret_cast<u32x4*>(As + hl * MROWS * hp + r * hp + k - hl * H) = v[i];
            }
        }
        __syncthreads();
        PROF(2)
        // ---- gates of this wave's gate g = wave for all rows: [64 x 32 units] ----
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
            const int mt = mh * 2 + mi;
            if (mt >= nmt) break;
            f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const int ao = (mt * 16 + (lane & 15)) * hp + ks * 32 + 8 * (lane >> 4);
                const bf16x8 af = *reinterpret_cast<const bf16x8*>(As + ao);
                if constexpr (PR) {  // h_lo W_hi + h_hi W_lo + h_hi W_hi (small terms first)
                    const bf16x8 afl = *reinterpret_cast<const bf16x8*>(As + MROWS * hp + ao);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl, bw[0][ks], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl, bw[1][ks], acc1, 0, 0, 0);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bwl[0][ks], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bwl[1][ks], acc1, 0, 0, 0);
                }
                acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[0][ks], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[1][ks], acc1, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = mt * 16 + (lane >> 4) * 4 + r;
                gs[row * gp + gate * UNITS + (lane & 15)] = acc0[r];
                gs[row * gp + gate * UNITS + 16 + (lane & 15)] = acc1[r];
            }
        }
        __syncthreads();
        PROF(3)
        // ---- cell update, publish h ----
        if (tagged) {
            // batch-1 cell map: lane (row, unit u, gate g) = tid (row 7 bits up, u = (tid >> 2) & 31, g = tid & 3)
            // activates ONE gate (two transcendentals instead of the counter form's ten per cell chain), the quad's
            // g = 0 lane gathers f / g / o by DPP and updates the cell; even units publish {tag, h_u, h_u+1} granules
            if (tid < nrows * 128) {
                const int row = tid >> 7, u = (tid >> 2) & 31, g = tid & 3;
                const float pre = gs[row * gp + g * UNITS + u] + gxs;
                const float act = g == 2 ? fast_tanh(pre) : fast_sigmoid(pre);
                const float fg = dpp_f<0x55>(act), gt = dpp_f<0xAA>(act), og = dpp_f<0xFF>(act);  // quad lanes 1, 2, 3
                c1 = cell_c(act, fg, gt, c1);  // (meaningful in the g = 0 lane)
                const float h = cell_h(og, c1);
                // unit u + 1's h (its g = 0 lane, 4 lanes up -- inside the same 16-lane row for the even units that
                // publish): DPP row_shl:4 instead of a ds_bpermute round trip
                const float h1 = dpp_f<0x104>(h);
                if (g == 0 && (u & 1) == 0) {
                    const unsigned pr = pack2bf(h, h1);
                    gu64* gp8 = gran + (s & 1) * TAG_ROWS * (H / 2) + row * (H / 2) + (p * UNITS + u) / 2;
                    __hip_atomic_store(gp8, ((unsigned long long)(unsigned)(s + 1) << 32) | pr, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    *reinterpret_cast<unsigned*>(Y + (long)(b0 + row) * a.bsy + (long)t * a.ldy + dir * H + p * UNITS + u) = pr;
                }
            }
            // no barrier here: the next step writes As only after every wave passed this step's post-MFMA barrier
            // (its As reads are consumed), and gs only after the next post-staging barrier
            PROF(5)
            continue;
        }
        float hv[CPT];
#pragma unroll
        for (int j = 0; j < CPT; ++j) {
            const float* gr = gs + crow * gp + cu0 + j;
            const float gi = gr[0] + gx[0][j], gf = gr[UNITS] + gx[1][j], gg = gr[2 * UNITS] + gx[2][j],
                        go = gr[3 * UNITS] + gx[3][j];
            if constexpr (PR) {
                const float ig = acc_sigmoid(gi), fg = acc_sigmoid(gf), og = acc_sigmoid(go);
                c[j] = fg * c[j] + ig * tanhf(gg);
                hv[j] = og * tanhf(c[j]);
            } else {
                const float ig = fast_sigmoid(gi), fg = fast_sigmoid(gf), og = fast_sigmoid(go);
                c[j] = cell_c(ig, fg, fast_tanh(gg), c[j]);
                hv[j] = cell_h(og, c[j]);
            }
        }
        const uint2 hb = make_uint2(pack2bf(hv[0], hv[1]), pack2bf(hv[2], hv[3]));
        if (cvalid) {
            const __attribute__((ext_vector_type(2))) unsigned int hw = {hb.x, hb.y};
            const int so = ((s & 1) * GR * NH * H + crow * NH * H + p * UNITS + cu0) * 2;
            __builtin_amdgcn_raw_buffer_store_b64(hw, xr, so, 0, 16);
            if constexpr (PR) {  // lo = bf16(h - hi) (exact difference)
                float hf[4];
#pragma unroll
                for (int j = 0; j < CPT; ++j) hf[j] = hv[j] - __uint_as_float((j & 1) ? ((j < 2 ? hb.x : hb.y) & 0xFFFF0000u)
                                                                                      : ((j < 2 ? hb.x : hb.y) << 16));
                const __attribute__((ext_vector_type(2))) unsigned int lw = {pack2bf(hf[0], hf[1]), pack2bf(hf[2], hf[3])};
                __builtin_amdgcn_raw_buffer_store_b64(lw, xr, so + H * 2, 0, 16);
            }
        }
        PROF(4)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the layer output (read by later launches only) leaves after the signal, outside the drain
        if (cvalid) {
            const long yo = (long)cb * a.bsy + (long)t * a.ldy + dir * H + p * UNITS + cu0;
            if constexpr (PR)
                *reinterpret_cast<float4*>(Yf + yo) = make_float4(hv[0], hv[1], hv[2], hv[3]);
            else
                *reinterpret_cast<uint2*>(Y + yo) = hb;
        }
        PROF(5)
    }
#ifdef STZS_LSTM_PROF
    if (tid == 0 && p == 0 && dir == 0)
        for (int i = 1; i < 6; ++i) ((unsigned long long*)a.sync)[256 + i] = pt[i];
#endif
#undef PROF
    // leave the counters zeroed for the next call: the LAST workgroup to finish (told by its add to the
    // done word) resets every arrival counter, the error word and the done word with agent-scope atomic
    // stores.  Every other workgroup's last poll returned before its done add, so nothing reads a counter
    // after its reset.  (A per-call hipMemsetAsync of the counters is NOT coherent with the pollers' sc1
    // loads when replayed from a HIP graph: measured, every replay read stale counters, tools/lstm_det.py.)
    __syncthreads();
    if (tid == 0) {
        gu32* done = (gu32*)(a.sync) + 1020;
        const unsigned nwg = gridDim.x * gridDim.y * nz;  // this recurrence's workgroups (its own done word)
        s_last = 0;
        if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nwg - 1) {
            for (unsigned i = 0; i < gridDim.y * nz; ++i)
                __hip_atomic_store((gu32*)(a.sync) + i * 16, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(err, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = 1;
        }
    }
    __syncthreads();
    if (s_last && a.B - (nz - 1) * GR <= TAG_ROWS && !PR) {  // the last group ran tagged: its granules back to zero
        gu64* g0 = (gu64*)(a.xchg);
        for (int e = tid; e < TAG_BYTES / 8; e += 512) __hip_atomic_store(g0 + e, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// zero a caller's LSTM state (the 1024 counter / error / done words of `sync` and the granule region at the start
// of `xchg`) with agent-scope atomic stores -- the same stores the kernel's own tail uses, so the reset is ordered
// and coherent with the pollers' sc1 loads under graph replay too (a memset node is not, see the kernel's tail)
__global__ __launch_bounds__(256) void lstm_state_reset(gu32* sync, gu64* gran) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < 1024) __hip_atomic_store(sync + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (gran && i < TAG_BYTES / 8) __hip_atomic_store(gran + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

extern "C" int stzs_lstm_state_reset(void* sync, void* xchg, void* stream) {
    if (!sync) return STZS_EINVAL;
    constexpr int n = 1024 > TAG_BYTES / 8 ? 1024 : TAG_BYTES / 8;
    hipLaunchKernelGGL(lstm_state_reset, dim3((n + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       (gu32*)sync, (gu64*)xchg);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

// utterances per group: 16 above 16 utterances (one MFMA row tile: the step's MFMA, h-load and cell work of a
// 16-row group; measured at B = 64 x H = 256, tools/probe/lstm_prof.py: 2.7 us per step vs 3.1 at 32 rows and 3.8 at
// 64), falling back to 32 / 64 where the grid would not stay co-resident (<= 63 groups x directions, <= 256
// workgroups).  STZS_LSTM_GROUP=32|64 caps the group (A/B switch -- the result is the same either way)
static int lstm_group_rows(int B, int H, int ndir) {
    static const int force = [] {
        const char* e = getenv("STZS_LSTM_GROUP");
        return e ? atoi(e) : 0;
    }();
    if (B <= 16) return MROWS;
    for (int gr = 16; gr < MROWS; gr *= 2) {
        const int g = (B + gr - 1) / gr;
        if (gr >= force && g * ndir <= 63 && (H / UNITS) * ndir * g <= 256) return gr;
    }
    return MROWS;
}

extern "C" size_t stzs_lstm_workspace(int B, int H, int ndir) {
    const int groups = (B + lstm_group_rows(B, H, ndir) - 1) / lstm_group_rows(B, H, ndir);
    // the small-batch granule region, then the slab (sized for the precise hi | lo rows)
    return (size_t)TAG_BYTES + (size_t)groups * ndir * 2 * lstm_group_rows(B, H, ndir) * 2 * H * sizeof(bf16_t);
}

static int lstm_check(const stzs_lstm_args* a) {
    if (!a || !a->gx || !a->whhT || !a->y || !a->xchg || !a->sync) return STZS_EINVAL;
    if (a->B <= 0 || a->T <= 0 || a->H <= 0 || a->H > 256 || a->H % UNITS || (a->ndir != 1 && a->ndir != 2))
        return STZS_ESHAPE;
    if (a->ldg % 8 || a->bsg % 8 || a->ldy % 8 || a->bsy % 8) return STZS_ESHAPE;
    const int gr = lstm_group_rows(a->B, a->H, a->ndir);
    const int groups = (a->B + gr - 1) / gr;
    if (groups * a->ndir > 63 || (a->H / UNITS) * a->ndir * groups > 256) return STZS_ESHAPE;
    if (a->precise > 1) return STZS_EINVAL;
    if (a->precise && (a->ldy % 4 || a->bsy % 4)) return STZS_ESHAPE;
    return STZS_OK;
}

// one launch of one recurrence (b == nullptr) or of two of one shape class side by side
static int lstm_launch(const stzs_lstm_args* a, const stzs_lstm_args* b, void* stream) {
    const int gr = lstm_group_rows(a->B, a->H, a->ndir);
    const int groups = (a->B + gr - 1) / gr;
    const int P = a->H / UNITS;
    if (b && P * a->ndir * 2 * groups > 256) {
        // both grids must be co-resident (one workgroup per CU); past that (e.g. B = 129: 9 groups of 16 rows, 144
        // workgroups per recurrence) the two recurrences run as two launches on the stream, one after the other --
        // the same bits as the paired launch (each recurrence's groups, gates and exchange are independent of the other)
        const int rc = lstm_launch(a, nullptr, stream);
        return rc != STZS_OK ? rc : lstm_launch(b, nullptr, stream);
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // the counters start at zero (caller-zeroed once) and every call leaves them zeroed (see the kernel's
    // tail); the caller's status word (a->status) accumulates over calls and is never cleared here
    const int hp = a->H + 8;
    const int nh = a->precise ? 2 : 1;
    const size_t lds = ((nh * MROWS * hp * 2 + 15) & ~15) + (size_t)MROWS * (4 * UNITS + 4) * 4;
    dim3 grid(P, a->ndir, b ? 2 * groups : groups);
    switch (a->H / 32) {
#define STZS_LSTM_CASE(n)                                                                                   \
    case n: {                                                                                               \
        auto k = a->precise ? (gr == 32 ? lstm_xchg<n, true, 32> : gr == 16 ? lstm_xchg<n, true, 16> : lstm_xchg<n, true>) \
                            : (gr == 32 ? lstm_xchg<n, false, 32> : gr == 16 ? lstm_xchg<n, false, 16> : lstm_xchg<n, false>); \
        if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
        hipLaunchKernelGGL(k, grid, dim3(512), lds, s, *a, b ? *b : *a, groups);                           \
        break;                                                                                              \
    }
        STZS_LSTM_CASE(1)
        STZS_LSTM_CASE(2)
        STZS_LSTM_CASE(4)
        STZS_LSTM_CASE(8)
#undef STZS_LSTM_CASE
        default: return STZS_ESHAPE;
    }
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_lstm(const stzs_lstm_args* a, void* stream) {
    const int rc = lstm_check(a);
    return rc != STZS_OK ? rc : lstm_launch(a, nullptr, stream);
}

// two independent recurrences in one launch: same B, H, directions and mode (so one group height and one
// kernel), each with its own gates / weights / T / outputs and its OWN exchange workspace and sync words
// (a->xchg != b->xchg, a->sync != b->sync); each result is the same bits as its own stzs_lstm call
extern "C" int stzs_lstm_pair(const stzs_lstm_args* a, const stzs_lstm_args* b, void* stream) {
    int rc = lstm_check(a);
    if (rc == STZS_OK) rc = lstm_check(b);
    if (rc != STZS_OK) return rc;
    if (a->B != b->B || a->H != b->H || a->ndir != b->ndir || a->precise != b->precise) return STZS_ESHAPE;
    if (a->xchg == b->xchg || a->sync == b->sync) return STZS_EINVAL;
    return lstm_launch(a, b, stream);
}
