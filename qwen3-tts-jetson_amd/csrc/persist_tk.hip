// persist_tk.hip — the Talker decode step of one slot (src/tts_transformer.cpp:1376-1512 build_step_graph, the codec
// head and the CB0 selection of :2416-2499) as ONE persistent launch of role-specialised workgroups: the design of
// persist_cp.hip (every hand-off between small disjoint role groups, tools/dev/edgebench.hip) applied to the 28-layer
// step, whose attention reads a growing HBM-resident KV cache.
//
//   role (workgroups)        per layer                                           input edge
//   O    [0, 32)             K slice w = i >> 3 (kv groups 2w, 2w + 1): the      partials 2S -> 32
//                            combine of their split partials in split order,
//                            then 128 O-projection rows (row block i & 7) over
//                            the slice's 512 columns (k_gemv's wave w sum)
//   GU   [32, 128)           x' = x + (((o0 + o1) + o2) + o3); RMSNorm(ffn_norm)  o      32 -> 96
//                            + 32 gate/up SwiGLU units
//   DN   [128, 184)          18-19 down rows + residual x'                        h      96 -> 56
//   QKV  [184, 248)          RMSNorm(attn_norm) + 64 QKV rows (4 x 16); codec     x      DN 56 -> 64
//                            head 48 rows (3 x 16) after the last layer
//   ATT  [248, 248 + 8S)     kv group g, split s: positions [64 s, 64 s + 64)     QKV    ~8 -> S per group
//                            (S = ceil(n_ctx / 64)): the chunk's partial
//   SEL  248 + 8S            CB0 selection of the next frame                      logits QKV 64 -> 1
//
// No workgroup combines the splits on its own: each O workgroup combines the two kv groups its K slice reads (k_attn's
// combine, one output per thread and group), so the attention reaches the O projection in one hand-off, not two.  The
// O projection's four per-wave K-slice sums (k_gemv<1,1,4,PRO_F16,4>: wave w reduces columns [512 w, 512 w + 512))
// are computed by four workgroups and summed by their consumers in k_gemv's order, so the step stays bit-identical.
//
// Two workgroups per CU (LDS <= 80 KB, <= 256 registers per wave): the grid of up to 505 workgroups is co-resident,
// so the attention keeps k_attn's split of 64 positions per workgroup (one chunk's body; a workgroup that ran 2-3
// chunks took 5-9 us per layer, their waves issue-bound) while the other roles keep the code-predictor frame's sizes.
// Each chunk's partial is computed with k_attn's per-split arithmetic for chunk 64 and the chunk partials are combined
// in chunk order exactly as k_attn / k_persist combine their splits, so the step is bit-identical to the launch-per-op
// graph and to k_persist<0, 64> (tests/test_gpu_persist.py).  Every row keeps the per-op GEMVs' lane split and
// reduction order.  Each workgroup holds only its role's weights (<= 160 VGPRs) or K/V rows, issued right after its
// phase for the next layer.  Contexts longer than 64 x 32 positions use k_persist<0, CH>.
#include "persist.h"
#include "persist_dev.h"
#include "select.h"

#include <algorithm>

#pragma clang fp contract(off)   // every rounding as written: bit-identical to k_gemv / k_attn / k_persist

namespace q3t {

namespace {
using namespace pdev;

constexpr int H = 1024, NH = 16, NKV = 8, D = 128, QKVN = (NH + 2 * NKV) * D, INTER = 3072, VOC = 3072;
constexpr int R = NH / NKV, CHK = 64, PSLOT = 264, MAXCH = 32;   // chunk of positions; partial granules; gpart slots
// Workgroups b and b + 256 share a CU (observed dispatch, tools/dev/cuprobe.hip; speed only, never correctness): the
// attention splits >= 1 (workgroups 256..) sit beside the down workgroups, then (splits >= 8) the O workgroups.  The
// down workgroups' weight stream (issued right after their phase) has landed long before the next attention, and
// their wait during the attention is a one-lane gate.  With the O workgroups beside the splits instead, the O
// workgroups' combine sweeps shared the CU with the partials' producers: 0.385 vs 0.376 ms at position 266, 0.392 vs
// 0.382 at 500, 0.480 vs 0.476 at 1500.  Beside the QKV workgroups, which issue the next layer's rows right at the
// QKV -> attention edge, a split's poll arrived 2.3 us late (round 4, before the gated polls).
#ifndef Q3T_TK_WPUB   // QKV phase: each wave publishes its own 16 rows (one line; 0: through LDS, wave 0 publishes all 64)
#define Q3T_TK_WPUB 1
#endif
#ifndef Q3T_TK_HOIST   // attention: the new row's K / V share read once and selected per position pass (0: read under
#define Q3T_TK_HOIST 1   // a branch in every pass)
#endif
#ifndef Q3T_TK_PUT_FIRST   // a role's publish: the other waves issue the next layer's weight prefetch only after wave 0's
#define Q3T_TK_PUT_FIRST 0   // store instruction (their loads otherwise queue ahead of it in the CU's memory pipe)
#endif
#ifndef Q3T_TK_PAIR
#define Q3T_TK_PAIR 1   // development: 0 = O, gate/up, down, QKV; 1 = down, O, gate/up, QKV (the splits beside down)
#endif
#ifndef Q3T_TK_WAIT_ATT
#define Q3T_TK_WAIT_ATT g_wait   // development: g_wait_gated
#endif
#if Q3T_TK_PAIR == 0
constexpr int OW = 0, NO = 32;       // O rows 32 (8 x 4)
constexpr int UW = 32, NU = 96;      // gate/up units 32 (2 x 16)
constexpr int DW = 128, ND = 56;     // down rows 18-19 (5 x 4)
constexpr int QW = 184, NQ = 64;     // QKV rows 64 (4 x 16); codec head rows 48 (3 x 16)
#else
constexpr int DW = 0, ND = 56;
constexpr int OW = 56, NO = 32;
constexpr int UW = 88, NU = 96;
constexpr int QW = 184, NQ = 64;
#endif
constexpr int AW = 248;              // attention workgroups (8 per split), then the selecting workgroup
constexpr int GRID_MAX = 512;        // two workgroups per CU (LDS <= 80 KB, <= 256 registers per wave)
constexpr int S_MAX = (GRID_MAX - AW - 1) / 8;
constexpr int MAXL = 32;
static_assert(NO + NU + ND + NQ == AW && QW + NQ == AW, "roles");
static_assert(NQ * 64 == QKVN && NQ * 48 == VOC && NU * 32 == INTER && NO * 32 == H && ND * 19 >= H, "role rows");

template <int CPW>
struct TLds {
    uint16_t xs[INTER];
    float xr[32];
    float red[2][4][32];   // [layer parity][wave][row]
    float outv[128];             // QKV / head / O rows staged for one whole-line publish
    double dscr[8];
    float hs[32];
    // attention
    float q_s[R][D], kn_s[D], vn_s[D];
    float wred[4][CPW][R], wsum[4][CPW][R];   // per-wave softmax max / sum per chunk
    float mch[CPW][R], lch[CPW][R];   // per-chunk max / sum (split partials)
    float ared[4][CPW][R][D];
    SelLds sel;
    PLayerW layers[MAXL];
};

template <int CPW>
struct Ctx {
    const PersistParams &p;
    TLds<CPW> &S;
    Ctl c;
    unsigned seq;
    int pos, nl;
    __device__ uint32_t tag(int ph) const { return ((seq * 1024u + (unsigned)ph) << 1) | 1u; }
};

#define PROF(ph, k)                                                                                           \
    do {                                                                                                      \
        if (X.p.prof && threadIdx.x == 0 && blockIdx.x < PROF_WG) X.p.prof[((size_t)blockIdx.x * PROF_PH + (ph)) * 4 + (k)] = wall_clock64(); \
    } while (0)

// x rows 4t..4t+3 of the layer-0 input (k_persist<0,*>'s prologue, same summation order)
__device__ __forceinline__ float4 layer0_x4(const PersistParams &p) {
    const int t = threadIdx.x;
    if (!p.gather) return ldf4(p.x_in + 4 * t);
    const GatherSum &gs = p.gs;
    uint2 hv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) hv[j] = ld8(gs.tabs[j] + (size_t)gs.tok[j] * H + 4 * t);
    const int fr = gs.frame[0];
    const float *extra = fr < gs.tr_len[0] ? gs.tr + (size_t)fr * H : gs.pad;
    const float4 ex = ldf4(extra + 4 * t);
    auto h4 = [](uint2 u) { return make_float4(h2f(u.x & 0xffff), h2f(u.x >> 16), h2f(u.y & 0xffff), h2f(u.y >> 16)); };
    float4 x = h4(hv[0]);
#pragma unroll
    for (int j = 1; j < 16; ++j) { const float4 b = h4(hv[j]); x = make_float4(x.x + b.x, x.y + b.y, x.z + b.z, x.w + b.w); }
    return make_float4(x.x + ex.x, x.y + ex.y, x.z + ex.z, x.w + ex.w);
}
// one element of the same (the O workgroups' residual rows): identical per-element summation order
__device__ __forceinline__ float layer0_x1(const PersistParams &p, int e) {
    if (!p.gather) return p.x_in[e];
    const GatherSum &gs = p.gs;
    uint16_t hv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) hv[j] = gs.tabs[j][(size_t)gs.tok[j] * H + e];
    const int fr = gs.frame[0];
    const float *extra = fr < gs.tr_len[0] ? gs.tr + (size_t)fr * H : gs.pad;
    const float ex = extra[e];
    float x = h2f(hv[0]);
#pragma unroll
    for (int j = 1; j < 16; ++j) x = x + h2f(hv[j]);
    return x + ex;
}

// ------------------------------------------------------------------ QKV rows (+ codec head after the last layer)
template <int CPW>
__device__ __forceinline__ void tk_qkv(Ctx<CPW> &X) {
    const PersistParams &p = X.p;
    TLds<CPW> &S = X.S;
    const int i = blockIdx.x - QW, t = threadIdx.x, l16 = t & 15, grp = t >> 4, nl = X.nl;
    uint4 wq[4][8];
    float4 nw;
    auto issue_qkv = [&](int l) {
        const uint16_t *W = S.layers[l].qkv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // Q3T_TK_WPUB: wave w owns rows 16w .. 16w + 15 (row 16w + 4j + lane / 16) and publishes them itself
            const int row = Q3T_TK_WPUB ? 16 * (t >> 6) + 4 * j + (grp & 3) : 16 * j + grp;
            const uint16_t *r = W + (size_t)(64 * i + row) * H + l16 * 8;
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) wq[j][tt] = ld16(r + tt * 128);
        }
        nw = ldf4(S.layers[l].attn_norm + 4 * t);
    };
    issue_qkv(0);
    for (int l = 0; l < nl; ++l) {
        const int ph = 5 * l;
        float4 x;
        if (l == 0) {
            x = layer0_x4(p);
        } else {
            uint32_t u[4];
            PROF(ph, 0);
            g_gate(p.gx + 4 * t, X.tag(5 * (l - 1) + 4), X.c);
            g_waitc<4>(p.gx + 4 * t, X.tag(5 * (l - 1) + 4), u, X.c);
            PROF(ph, 1);
            x = f4_of(u);
        }
        rms_to_f16(x, nw, p.eps, S.xs, S.dscr, nullptr);
        __syncthreads();
        float acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            acc[j] = 0.0f;
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) acc[j] = dot8(wq[j][tt], *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128), acc[j]);
        }
        if constexpr (Q3T_TK_WPUB) {
            // each wave publishes its 16 rows as one whole line (persist_cp.hip role_qkv): no barrier
            float pv = 0.0f;
            const int lane = t & 63;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float v = __shfl(group_sum<16>(acc[j]), 16 * (lane & 3));
                if ((lane >> 2) == j) pv = v;
            }
            if (lane < 16) g_put(p.gqkv + 64 * i + 16 * (t >> 6) + lane, __float_as_uint(pv), X.tag(ph));
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[j] = group_sum<16>(acc[j]);
                if (l16 == 0) S.outv[16 * j + grp] = acc[j];
            }
            __syncthreads();
            // one store instruction of wave 0 publishes the 64 rows (4 whole lines): single-lane stores from four waves
            // into shared lines make the next edge slower
            if (t < 64) g_put(p.gqkv + 64 * i + t, __float_as_uint(S.outv[t]), X.tag(ph));
        }
        PROF(ph, 2);
        if (Q3T_TK_PUT_FIRST) __syncthreads();
        if (l + 1 < nl) {
            issue_qkv(l + 1);
        } else {   // codec head rows 48i + 16j + grp
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const uint16_t *r = p.head + (size_t)(48 * i + 16 * j + grp) * H + l16 * 8;
#pragma unroll
                for (int tt = 0; tt < 8; ++tt) wq[j][tt] = ld16(r + tt * 128);
            }
            nw = ldf4(p.out_norm + 4 * t);
        }
    }
    // ---- head: RMSNorm(output_norm) -> hidden (side output, workgroup 0) -> codec head logits
    const int hph = 5 * nl;
    uint32_t u[4];
    PROF(hph, 0);
    g_waitc<4>(p.gx + 4 * t, X.tag(5 * (nl - 1) + 4), u, X.c);
    PROF(hph, 1);
    rms_to_f16(f4_of(u), nw, p.eps, S.xs, S.dscr, i == 0 ? p.hidden : nullptr);
    __syncthreads();
    float a0[3], a1[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        a0[j] = 0.0f;
        a1[j] = 0.0f;
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) a0[j] = dot8(wq[j][tt], *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128), a0[j]);
#pragma unroll
        for (int tt = 4; tt < 8; ++tt) a1[j] = dot8(wq[j][tt], *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128), a1[j]);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float lg = group_sum<16>(a0[j]) + group_sum<16>(a1[j]);
        if (l16 == 0) S.outv[16 * j + grp] = lg;
    }
    __syncthreads();
    if (t < 48) {
        g_put(p.glog + 48 * i + t, __float_as_uint(S.outv[t]), X.tag(hph));
        p.logits[48 * i + t] = S.outv[t];   // read after the launch only (host, tests)
    }
    PROF(hph, 2);
}

// ------------------------------------------------------------------ split combine + O-projection K slice (128 rows)
template <int CPW>
__device__ __forceinline__ void tk_o(Ctx<CPW> &X) {
    constexpr int CB = 8;   // chunks per poll sweep
    const PersistParams &p = X.p;
    TLds<CPW> &S = X.S;
    const int i = blockIdx.x - OW, w = i >> 3, rb = i & 7, t = threadIdx.x, lane = t & 63, wave = t >> 6, l16 = t & 15,
              grp4 = lane >> 4, nl = X.nl, nch = X.pos / CHK + 1;
    uint4 wo[8][4];
    auto issue = [&](int l) {   // row 128 rb + 32 wave + 4j + grp4, columns of K slice w (k_gemv<1,1,4,PRO_F16,4>)
        const uint16_t *W = S.layers[l].o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint16_t *r = W + (size_t)(128 * rb + 32 * wave + 4 * j + grp4) * (NH * D) + w * 512 + l16 * 8;
#pragma unroll
            for (int tt = 0; tt < 4; ++tt) wo[j][tt] = ld16(r + tt * 128);
        }
    };
    // split partials of kv groups 2w (sel 0) and 2w + 1 (sel 1): this thread's output is element t of each group
    // (head r = t >> 7, uniform over a wave; dimension t & 127: granule t of every chunk slot).  Lane j also fetches the
    // max / sum of head r (granules 256 + r, 258 + r) of chunk j & 31 of group j >> 5, so the chunk weights
    // expf(m - max), uniform over the wave, are computed once per chunk (one lane each) and read back with readlane
    const uint64_t *gp0 = p.gpart + (size_t)(2 * w) * MAXCH * PSLOT;
    const int r = t >> 7, jsel = lane >> 5, jc = lane & 31;
    const uint64_t *mlp = gp0 + (size_t)jsel * MAXCH * PSLOT + (size_t)min(jc, nch - 1) * PSLOT + R * D + r;
    issue(0);
    for (int l = 0; l < nl; ++l) {
        const int ph = 5 * l + 2;
        const uint32_t want = X.tag(5 * l + 1);
        PROF(ph, 0);
        if (nch == 1) {   // k_attn's single-split output of the two groups (granule 128 g + t: elements 2t, 2t + 1)
            uint32_t u[1];
            Q3T_TK_WAIT_ATT<1>(p.gattn + (size_t)w * 256 + t, want, u, X.c);
            PROF(ph, 1);
            *reinterpret_cast<uint32_t *>(S.xs + 2 * t) = u[0];
        } else {          // k_attn's combine in chunk order (the same expressions as its split combine)
            float lt[2] = {0.0f, 0.0f}, av[2] = {0.0f, 0.0f}, swl = 0.0f, ll = 0.0f;
            // the sweeps below behind a one-lane gate on the last chunk's partial: sweeping 18 granules per thread for
            // the whole wait stalled the co-resident attention workgroup's partial stores by up to 1.7 us
            g_gate(gp0 + (size_t)(nch - 1) * PSLOT + t, want, X.c);
            for (int c0 = 0; c0 < nch; c0 += CB) {
                const int nb = min(CB, nch - c0);
                uint64_t va[2][CB], vm = 0, vl = 0;
                unsigned it = 0;
                while (true) {   // every granule of the sweep issued before any tag is checked
                    if (c0 == 0) {
                        vm = g_ld(mlp);
                        vl = g_ld(mlp + R);
                    }
#pragma unroll
                    for (int sel = 0; sel < 2; ++sel)
#pragma unroll
                        for (int k = 0; k < CB; ++k)
                            va[sel][k] = g_ld(gp0 + (size_t)sel * MAXCH * PSLOT + (size_t)(c0 + min(k, nb - 1)) * PSLOT + t);
                    bool ok = c0 > 0 || jc >= nch || ((uint32_t)(vm >> 32) == want && (uint32_t)(vl >> 32) == want);
#pragma unroll
                    for (int sel = 0; sel < 2; ++sel)
#pragma unroll
                        for (int k = 0; k < CB; ++k) ok &= k >= nb || (uint32_t)(va[sel][k] >> 32) == want;
                    if (ok || X.c.abort) break;
                    if ((++it & 255u) == 0 && (__hip_atomic_load(X.c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
                                               it >= SPIN_LIMIT)) {
                        X.c.abort = true;
                        __hip_atomic_fetch_or(X.c.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (c0 == 0) {   // lane j: chunk j & 31 of group j >> 5.  max over the chunks: order-free (expf(m - max)
                                 // is the same for either zero sign of max), then one expf per chunk
                    PROF(ph, 1);
                    const float m = jc < nch ? __uint_as_float((uint32_t)vm) : -INFINITY;
                    ll = __uint_as_float((uint32_t)vl);
                    const float mx = group_max<32>(m);
                    swl = jc < nch ? expf(m - mx) : 0.0f;
                    PROF(200 + l, 0);   // (development timeline: chunk weights)
                }
#pragma unroll
                for (int k = 0; k < CB; ++k)
                    if (k < nb)
#pragma unroll
                        for (int sel = 0; sel < 2; ++sel) {
                            const int src = sel * 32 + c0 + k;
                            const float sw = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(swl), src));
                            lt[sel] = __fmaf_rn(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(ll), src)), sw, lt[sel]);
                            av[sel] = __fmaf_rn(__uint_as_float((uint32_t)va[sel][k]), sw, av[sel]);
                        }
            }
            PROF(200 + l, 1);   // (development timeline: wave 0's combine done)
            S.xs[t] = f2h(av[0] / lt[0]);
            S.xs[256 + t] = f2h(av[1] / lt[1]);
        }
        __syncthreads();
        PROF(ph, 3);   // (development timeline: attention combined)
        float acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc[j] = 0.0f;
#pragma unroll
            for (int tt = 0; tt < 4; ++tt) acc[j] = dot8(wo[j][tt], *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128), acc[j]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc[j] = group_sum<16>(acc[j]);
            if (l16 == 0) S.outv[32 * wave + 4 * j + grp4] = acc[j];
        }
        __syncthreads();
        // two store instructions (waves 0, 1: whole lines each) publish the slice sums of the 128 rows
        if (t < 128) g_put(p.gop + (size_t)w * H + 128 * rb + t, __float_as_uint(S.outv[t]), X.tag(ph));
        PROF(ph, 2);
        if (Q3T_TK_PUT_FIRST) __syncthreads();
        if (l + 1 < nl) issue(l + 1);
    }
}

// ------------------------------------------------------------------ RMSNorm(ffn_norm) + gate/up + SwiGLU (32 units)
template <int CPW>
__device__ __forceinline__ void tk_gu(Ctx<CPW> &X) {
    const PersistParams &p = X.p;
    TLds<CPW> &S = X.S;
    const int i = blockIdx.x - UW, t = threadIdx.x, l16 = t & 15, grp = t >> 4, nl = X.nl;
    uint4 wg[2][8], wu[2][8];
    float4 nw;
    auto issue = [&](int l) {
        const uint16_t *W = S.layers[l].gu;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int unit = 32 * i + 16 * j + grp;
            const uint16_t *r = W + (size_t)((unit >> 4) * 32 + (unit & 15)) * H + l16 * 8;
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) wg[j][tt] = ld16(r + tt * 128);
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) wu[j][tt] = ld16(r + 16 * H + tt * 128);
        }
        nw = ldf4(S.layers[l].ffn_norm + 4 * t);
    };
    issue(0);
    for (int l = 0; l < nl; ++l) {
        const int ph = 5 * l + 3;
        float4 xr;   // the residual stream entering the layer
        if (l == 0) {
            xr = layer0_x4(p);
        } else {
            uint32_t u4[4];
            g_waitc<4>(p.gx + 4 * t, X.tag(5 * (l - 1) + 4), u4, X.c);
            xr = f4_of(u4);
        }
        uint32_t u[16];   // K-slice sums o_w of rows 4t..4t+3 (w = 0..3)
        PROF(ph, 0);
        g_gate(p.gop + 4 * t, X.tag(5 * l + 2), X.c);
        if constexpr (Q3T_POLL16) g_wait16<4, 4, H>(p.gop + 4 * t, X.tag(5 * l + 2), u, X.c);
        else g_wait<16, H, 4>(p.gop + 4 * t, X.tag(5 * l + 2), u, X.c);
        PROF(ph, 1);
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {   // k_gemv's ((w0 + w1) + w2) + w3, then the residual add
            const float s = ((__uint_as_float(u[e]) + __uint_as_float(u[4 + e])) + __uint_as_float(u[8 + e])) + __uint_as_float(u[12 + e]);
            x[e] = (e == 0 ? xr.x : e == 1 ? xr.y : e == 2 ? xr.z : xr.w) + s;
        }
        rms_to_f16(make_float4(x[0], x[1], x[2], x[3]), nw, p.eps, S.xs, S.dscr, nullptr);
        __syncthreads();
        float a0[2], a1[2], b0[2], b1[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            a0[j] = a1[j] = b0[j] = b1[j] = 0.0f;
#pragma unroll
            for (int tt = 0; tt < 4; ++tt) {
                const uint4 xv = *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128);
                a0[j] = dot8(wg[j][tt], xv, a0[j]);
                b0[j] = dot8(wu[j][tt], xv, b0[j]);
            }
#pragma unroll
            for (int tt = 4; tt < 8; ++tt) {
                const uint4 xv = *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128);
                a1[j] = dot8(wg[j][tt], xv, a1[j]);
                b1[j] = dot8(wu[j][tt], xv, b1[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float ga = group_sum<16>(a0[j]) + group_sum<16>(a1[j]);
            const float ub = group_sum<16>(b0[j]) + group_sum<16>(b1[j]);
            if (l16 == 0) S.hs[16 * j + grp] = silu_f(ga) * ub;
        }
        __syncthreads();
        if (t < 16) g_put(p.gh + 16 * i + t, (uint32_t)f2h(S.hs[2 * t]) | ((uint32_t)f2h(S.hs[2 * t + 1]) << 16), X.tag(ph));
        PROF(ph, 2);
        if (Q3T_TK_PUT_FIRST) __syncthreads();
        if (l + 1 < nl) issue(l + 1);
    }
}

// ------------------------------------------------------------------ down + residual (23-24 rows)
template <int CPW>
__device__ __forceinline__ void tk_dn(Ctx<CPW> &X) {
    const PersistParams &p = X.p;
    TLds<CPW> &S = X.S;
    const int i = blockIdx.x - DW, t = threadIdx.x, lane = t & 63, wave = t >> 6, l16 = t & 15, grp4 = lane >> 4, nl = X.nl;
    const int lo = i * H / ND, n = (i + 1) * H / ND - lo;
    uint4 wd[5][6];
    auto issue = [&](int l) {   // row lo + 4j + grp4 (clamped), K slice = wave (k_gemv<1,1,4,PRO_F16,8>)
        const uint16_t *W = S.layers[l].down;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const uint16_t *r = W + (size_t)(lo + min(4 * j + grp4, n - 1)) * INTER + wave * 768 + l16 * 8;
#pragma unroll
            for (int tt = 0; tt < 6; ++tt) wd[j][tt] = ld16(r + tt * 128);
        }
    };
    issue(0);
    for (int l = 0; l < nl; ++l) {
        const int ph = 5 * l + 4;
        if (t < n) {   // x' = x + (((o0 + o1) + o2) + o3) of row lo + t (as the gate/up workgroups)
            float xr;
            if (l == 0) {
                xr = layer0_x1(p, lo + t);
            } else {
                uint32_t u1[1];
                g_wait<1>(p.gx + lo + t, X.tag(5 * (l - 1) + 4), u1, X.c);
                xr = __uint_as_float(u1[0]);
            }
            uint32_t uo[4];
            g_wait<4, H>(p.gop + lo + t, X.tag(5 * l + 2), uo, X.c);
            const float s = ((__uint_as_float(uo[0]) + __uint_as_float(uo[1])) + __uint_as_float(uo[2])) + __uint_as_float(uo[3]);
            S.xr[t] = xr + s;
        }
        uint32_t u[6];
        PROF(ph, 0);
        g_gate(p.gh + 6 * t, X.tag(5 * l + 3), X.c);
        g_waitc<6>(p.gh + 6 * t, X.tag(5 * l + 3), u, X.c);
        PROF(ph, 1);
        *reinterpret_cast<uint2 *>(S.xs + 12 * t) = make_uint2(u[0], u[1]);
        *reinterpret_cast<uint2 *>(S.xs + 12 * t + 4) = make_uint2(u[2], u[3]);
        *reinterpret_cast<uint2 *>(S.xs + 12 * t + 8) = make_uint2(u[4], u[5]);
        wave_lds_sync();   // wave w polled exactly the K slice [768 w, 768 w + 768) it multiplies
        float acc[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            acc[j] = 0.0f;
#pragma unroll
            for (int tt = 0; tt < 6; ++tt)
                acc[j] = dot8(wd[j][tt], *reinterpret_cast<const uint4 *>(S.xs + wave * 768 + l16 * 8 + tt * 128), acc[j]);
        }
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            acc[j] = group_sum<16>(acc[j]);
            if (l16 == 0) S.red[l & 1][wave][4 * j + grp4] = acc[j];
        }
        __syncthreads();
        if (t < n) {
            const float (&rd)[4][32] = S.red[l & 1];
            const float s = rd[0][t] + rd[1][t] + rd[2][t] + rd[3][t];
            g_put(p.gx + lo + t, __float_as_uint(S.xr[t] + s), X.tag(ph));
        }
        PROF(ph, 2);
        if (Q3T_TK_PUT_FIRST) __syncthreads();
        if (l + 1 < nl) issue(l + 1);
    }
}

// ------------------------------------------------------------------ attention: kv group g, split s (CPW chunks)
template <int CPW>
__device__ __forceinline__ void tk_att(Ctx<CPW> &X) {
    constexpr int NP = CPW * CHK / 16;   // position passes of 16 (16 lanes x 8 dims per position)
    const PersistParams &p = X.p;
    TLds<CPW> &S = X.S;
    const int a = blockIdx.x - AW, g = a & (NKV - 1), s = a >> 3;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, pg = t >> 4, li = t & 15, nl = X.nl, pos = X.pos;
    const int nch = pos / CHK + 1, c0 = s * CPW;
    const int myc = min(max(nch - c0, 0), CPW);   // chunks of this split in use this step
    if (myc == 0) return;                           // (uniform over the workgroup)
    const int j0 = c0 * CHK;
    const bool has_pos = pos / CHK >= c0 && pos / CHK < c0 + CPW;
    // wave v polls elements lane and lane + 64 of its head (q head 2g, q head 2g+1, k, v of group g): the pair its
    // head norm and NEOX RoPE work on (no LDS staging or barrier before the norm)
    const int gi = (wave == 0 ? g * 256 : wave == 1 ? g * 256 + D : wave == 2 ? NH * D + g * D : (NH + NKV) * D + g * D) + lane;
    uint4 kr[NP], vr[NP];
    float hn[2];
    auto issue = [&](int l) {   // this split's cached K/V rows (clamped rows re-read row pos) + head-norm weights
        const size_t o = (size_t)l * p.kv_layer + (size_t)g * p.n_ctx * D;
#pragma unroll
        for (int pi = 0; pi < NP; ++pi) {
            const int j = min(j0 + pi * 16 + pg, pos);
            kr[pi] = ld16(p.kc + o + (size_t)j * D + li * 8);
            vr[pi] = ld16(p.vc + o + (size_t)j * D + li * 8);
        }
        const float *nwv = wave == 2 ? S.layers[l].kn : S.layers[l].qn;
        hn[0] = nwv[lane];
        hn[1] = nwv[lane + 64];
    };
    const float rp0 = p.rope[(size_t)pos * D + 2 * lane], rp1 = p.rope[(size_t)pos * D + 2 * lane + 1];
    const float kq_scale = 1.0f / sqrtf((float)D);
    issue(0);
    for (int l = 0; l < nl; ++l) {
        const int ph = 5 * l + 1;
        const size_t kvo = (size_t)l * p.kv_layer + (size_t)g * p.n_ctx * D;
        float xr[2];
        {
            uint32_t u[2];
            PROF(ph, 0);
            Q3T_TK_WAIT_ATT<2, 64>(p.gqkv + gi, X.tag(5 * l), u, X.c);
            PROF(ph, 1);
            xr[0] = __uint_as_float(u[0]);
            xr[1] = __uint_as_float(u[1]);
        }
        {   // wave v: q head 0 / q head 1 / k (head norm + RoPE) / v (f16 rounding)
            const int v = wave;
            if (v == 3) {
#pragma unroll
                for (int e = 0; e < 2; ++e) S.vn_s[lane + 64 * e] = f16r(xr[e]);
            } else {
                float xx[2];
                double ss = 0.0;
#pragma unroll
                for (int e = 0; e < 2; ++e) { xx[e] = xr[e]; ss += (double)__fmul_rn(xx[e], xx[e]); }
                ss = wave_sum_d(ss);
                const float scale = 1.0f / sqrtf((float)(ss / D) + p.eps);
#pragma unroll
                for (int e = 0; e < 2; ++e) xx[e] = (xx[e] * scale) * hn[e];
                const float y0 = opaque(opaque(xx[0] * rp0) - opaque(xx[1] * rp1));   // as k_attn: three roundings
                const float y1 = opaque(opaque(xx[0] * rp1) + opaque(xx[1] * rp0));
                float *dst = v == 2 ? S.kn_s : S.q_s[v];
                dst[lane] = f16r(y0);
                dst[lane + 64] = f16r(y1);
            }
        }
        __syncthreads();
        PROF(200 + l, 0);   // (development timeline: q/k normed + RoPE)
        if (has_pos && t < D) {   // KV append at pos (read by later steps only)
            p.kc[kvo + (size_t)pos * D + t] = f2h(S.kn_s[t]);
            p.vc[kvo + (size_t)pos * D + t] = f2h(S.vn_s[t]);
        }
        float q8[R][8];
#pragma unroll
        for (int h = 0; h < R; ++h)
#pragma unroll
            for (int e = 0; e < 8; ++e) q8[h][e] = S.q_s[h][li * 8 + e];
        float sc[NP][R];
        uint32_t qp[R][4];
#pragma unroll
        for (int h = 0; h < R; ++h) pack_q8(q8[h], qp[h]);
        // the new row's K / V share, read once: the position passes then select it without a branch, so the
        // independent score chains interleave (a per-pass LDS read under a branch serialised them)
        const uint4 knp = Q3T_TK_HOIST ? pack8f(&S.kn_s[li * 8]) : make_uint4(0, 0, 0, 0);
        float vn8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) vn8[e] = Q3T_TK_HOIST ? S.vn_s[li * 8 + e] : 0.0f;
#pragma unroll
        for (int pi = 0; pi < NP; ++pi) {
            const int j = j0 + pi * 16 + pg;
            const bool ok = j <= pos;
#pragma unroll
            for (int h = 0; h < R; ++h) {
                float sv;
                if constexpr (Q3T_ATTN_DOT2 && Q3T_TK_HOIST) {
                    const uint4 kk = j == pos ? knp : kr[pi];
                    sv = score8(kk, qp[h]);
                } else if constexpr (Q3T_ATTN_DOT2) {
                    sv = score8(j == pos ? pack8f(&S.kn_s[li * 8]) : kr[pi], qp[h]);
                } else {
                    float k8[8];
                    if (j == pos) {
#pragma unroll
                        for (int e = 0; e < 8; ++e) k8[e] = S.kn_s[li * 8 + e];
                    } else {
                        const uint32_t ww[4] = {kr[pi].x, kr[pi].y, kr[pi].z, kr[pi].w};
#pragma unroll
                        for (int e = 0; e < 4; ++e) { k8[2 * e] = h2f(ww[e] & 0xffff); k8[2 * e + 1] = h2f(ww[e] >> 16); }
                    }
                    sv = 0.0f;
#pragma unroll
                    for (int e = 0; e < 8; ++e) sv = __fmaf_rn(k8[e], q8[h][e], sv);   // explicit fma: identical in k_attn
                }
                sv = group_sum<16>(sv);
                sc[pi][h] = ok ? __fmul_rn(sv, kq_scale) : -INFINITY;
            }
        }
        // per chunk cc (passes 4cc .. 4cc+3): max, then exp / sum, then P.V, each as k_attn's split of 64 positions
#pragma unroll
        for (int cc = 0; cc < CPW; ++cc)
#pragma unroll
            for (int h = 0; h < R; ++h) {
                float m = sc[4 * cc][h];
#pragma unroll
                for (int q = 1; q < 4; ++q) m = fmaxf(m, sc[4 * cc + q][h]);
                m = rows_max(m);
                if (lane == 0) S.wred[wave][cc][h] = m;
            }
        __syncthreads();
        float M[CPW][R];
#pragma unroll
        for (int cc = 0; cc < CPW; ++cc)
#pragma unroll
            for (int h = 0; h < R; ++h)
                M[cc][h] = fmaxf(fmaxf(S.wred[0][cc][h], S.wred[1][cc][h]), fmaxf(S.wred[2][cc][h], S.wred[3][cc][h]));
        if (t == 0) {
#pragma unroll
            for (int cc = 0; cc < CPW; ++cc)
#pragma unroll
                for (int h = 0; h < R; ++h) S.mch[cc][h] = M[cc][h];
        }
        PROF(200 + l, 1);   // (development timeline: scores + max done)
#pragma unroll
        for (int cc = 0; cc < CPW; ++cc) {
            float pr[4][R], ls[R];
#pragma unroll
            for (int h = 0; h < R; ++h) {
                ls[h] = 0.0f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int pi = 4 * cc + q;
                    const bool ok = j0 + pi * 16 + pg <= pos;
                    pr[q][h] = ok ? exp_sm(__fsub_rn(sc[pi][h], M[cc][h])) : 0.0f;
                    ls[h] += pr[q][h];
                }
            }
            {   // rows_sum of both heads at once: row 0 ends with head 0's (r0 + r1) + (r2 + r3), row 1 with head 1's
                const float lsum = rows_sum_pair(ls[0], ls[1]);
                if ((lane & 47) == 0) S.wsum[wave][cc][lane >> 4] = lsum;   // lanes 0, 16
            }
            float acc[R][8];
#pragma unroll
            for (int h = 0; h < R; ++h)
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[h][e] = 0.0f;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int pi = 4 * cc + q;
                const int j = j0 + pi * 16 + pg;
                const bool ok = j <= pos;
                float v8[8];
                if constexpr (Q3T_TK_HOIST) {
                    const uint32_t ww[4] = {vr[pi].x, vr[pi].y, vr[pi].z, vr[pi].w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v8[2 * e] = j == pos ? vn8[2 * e] : h2f(ww[e] & 0xffff);
                        v8[2 * e + 1] = j == pos ? vn8[2 * e + 1] : h2f(ww[e] >> 16);
                    }
                } else if (j == pos) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v8[e] = S.vn_s[li * 8 + e];
                } else {
                    const uint32_t ww[4] = {vr[pi].x, vr[pi].y, vr[pi].z, vr[pi].w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) { v8[2 * e] = h2f(ww[e] & 0xffff); v8[2 * e + 1] = h2f(ww[e] >> 16); }
                }
#pragma unroll
                for (int h = 0; h < R; ++h)
#pragma unroll
                    for (int e = 0; e < 8; e += 2)   // packed fmas (v_pk_fma_f32), the same roundings
                        fma2(pr[q][h], ok ? v8[e] : 0.0f, ok ? v8[e + 1] : 0.0f, acc[h][e], acc[h][e + 1]);
            }
            // rows_sum of the 16 accumulators as a reduce-scatter (12 row swaps in place of 32): row k ends with values
            // k, 4 + k, 8 + k, 12 + k (value n = 8 h + e), each (r0 + r1) + (r2 + r3) as rows_sum
            float v16[16], c8[8];
#pragma unroll
            for (int n = 0; n < 16; ++n) v16[n] = acc[n >> 3][n & 7];
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(v16[2 * m]), __float_as_uint(v16[2 * m + 1]), false, false);
                c8[m] = __uint_as_float((uint32_t)sw[0]) + __uint_as_float((uint32_t)sw[1]);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(c8[2 * q]), __float_as_uint(c8[2 * q + 1]), false, false);
                const float av = __uint_as_float((uint32_t)sw[0]) + __uint_as_float((uint32_t)sw[1]);
                const int n = 4 * q + (lane >> 4);
                S.ared[wave][cc][n >> 3][li * 8 + (n & 7)] = av;
            }
        }
        __syncthreads();
        PROF(200 + l, 2);   // (development timeline: P.V reduced)
        uint64_t *gout = p.gattn + (size_t)g * R * (D / 2);
        if (nch == 1) {   // one chunk: k_attn's single-split output
            if (t < R * D / 2) {
                const int h = t / (D / 2), d = 2 * (t % (D / 2));
                const float lsum = (S.wsum[0][0][h] + S.wsum[1][0][h]) + (S.wsum[2][0][h] + S.wsum[3][0][h]);
                const float a0 = (S.ared[0][0][h][d] + S.ared[1][0][h][d]) + (S.ared[2][0][h][d] + S.ared[3][0][h][d]);
                const float a1 = (S.ared[0][0][h][d + 1] + S.ared[1][0][h][d + 1]) + (S.ared[2][0][h][d + 1] + S.ared[3][0][h][d + 1]);
                g_put(gout + t, (uint32_t)f2h(a0 / lsum) | ((uint32_t)f2h(a1 / lsum) << 16), X.tag(ph));
            }
        } else {   // this split's chunk partials (acc [2][128], m [2], l [2]) in their chunk slots: the O workgroups combine
            uint64_t *gp = p.gpart + (size_t)g * MAXCH * PSLOT;
            for (int cc = 0; cc < myc; ++cc) {
                uint64_t *mine = gp + (size_t)(c0 + cc) * PSLOT;
                const int h = t / D, d = t % D;
                const float av = (S.ared[0][cc][h][d] + S.ared[1][cc][h][d]) + (S.ared[2][cc][h][d] + S.ared[3][cc][h][d]);
                g_put(mine + t, __float_as_uint(av), X.tag(ph));
                if (t < PSLOT - R * D) {
                    const int hh = t % R;
                    const float lsum = (S.wsum[0][cc][hh] + S.wsum[1][cc][hh]) + (S.wsum[2][cc][hh] + S.wsum[3][cc][hh]);
                    const float v = t < R ? S.mch[cc][hh] : t < 2 * R ? lsum : 0.0f;
                    g_put(mine + R * D + t, __float_as_uint(v), X.tag(ph));
                }
            }
        }
        PROF(ph, 2);
        // the next layer's K/V rows, a layer ahead of their use (issued once the O projection was done instead, the
        // stream landed late: 0.484 vs 0.464 ms at position 500)
        if (l + 1 < nl) issue(l + 1);
    }
}

// ------------------------------------------------------------------ CB0 selection of the next frame
template <int CPW>
__device__ __forceinline__ void tk_sel(Ctx<CPW> &X) {
    const PersistParams &p = X.p;
    TLds<CPW> &S = X.S;
    const int t = threadIdx.x, hph = 5 * X.nl;
    SelPre spre;
    if (p.sel.mode != SEL_NONE) sel_prefetch<SEL_CB0>(p.sel, 0, spre);
    // the logits are waited for even without a selection: the launch's seq bump must follow every chain workgroup's
    // start (each reads seq once, at its start)
    int tok = -1;
    // one lane sleeps until the last layer's down projection is under way (its first output granule), then the whole
    // workgroup sweeps the logits: a 3,072-granule sweep polled for the whole step slowed the workgroup sharing this
    // CU by ~5 us per phase
    if (t == 0) {
        uint32_t u1[1];
        Ctl c1 = X.c;
        for (int k = 0; k < 1 << 14 && !c1.abort; ++k) {   // bounded (~14 ms)
            const uint64_t v = g_ld(p.gh);   // gate/up output of the last layer (published before the down phase)
            if ((uint32_t)(v >> 32) == X.tag(5 * (X.nl - 1) + 3)) break;
            __builtin_amdgcn_s_sleep(32);
        }
        (void)u1;
    }
    __syncthreads();
    uint32_t u[VOC / 256];
    PROF(hph, 0);
    g_waitc<VOC / 256>(p.glog + t * (VOC / 256), X.tag(hph), u, X.c);
    PROF(hph, 1);
    if (p.sel.mode != SEL_NONE) {
        float v[SEL_VPT_MAX];
#pragma unroll
        for (int e = 0; e < SEL_VPT_MAX; ++e) v[e] = e < VOC / 256 ? __uint_as_float(u[e]) : -INFINITY;
        tok = select_token_pre<SEL_CB0>(p.sel, spre, v, S.sel);
    }
    __syncthreads();
    if (t == 0) {
        if (tok >= 0) select_commit(p.sel, 0, tok);
        // k_advance folded into the launch (every workgroup read pos / frame at its start or in layer 0, long before
        // this point; the next launch sees the stores)
        if (p.adv_pos && !(p.adv_done && p.adv_done[0] >= 0)) {
            p.adv_pos[0] += 1;
            p.adv_frame[0] += 1;
        }
        __hip_atomic_store(p.seq, X.seq + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    PROF(hph, 2);
}

template <int CPW>
__global__ void __launch_bounds__(256, 2) k_tk_roles(const PersistParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    TLds<CPW> &S = *reinterpret_cast<TLds<CPW> *>(smem);
    const int t = threadIdx.x, w = blockIdx.x;
    Ctx<CPW> X{p, S, Ctl{p.err, false}, __hip_atomic_load(p.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), p.pos[0], p.n_layers};
    if (t < p.n_layers) S.layers[t] = p.L[t];
    __syncthreads();
    const int sel_w = AW + 8 * p.roles_split;
    if (w >= OW && w < OW + NO) tk_o(X);
    else if (w >= UW && w < UW + NU) tk_gu(X);
    else if (w >= DW && w < DW + ND) tk_dn(X);
    else if (w < AW) tk_qkv(X);
    else if (w < sel_w) tk_att(X);
    else tk_sel(X);
}

template <int CPW>
size_t tk_lds() { return sizeof(TLds<CPW>); }   // <= 80 KB: two workgroups per CU

template <int CPW>
const void *tk_fn() { return reinterpret_cast<const void *>(&k_tk_roles<CPW>); }

// chunks of 64 positions per attention workgroup for a context, 0 if the role kernel does not cover it
int tk_cpw(int n_ctx) {
    const int nch = (n_ctx + CHK - 1) / CHK;
    return nch <= S_MAX && nch <= MAXCH ? 1 : 0;
}

}  // namespace

bool persist_tk_roles_supported(int n_ctx) { return tk_cpw(n_ctx) != 0; }

bool persist_tk_roles_resident(int device, int n_ctx) {
    int n_cu = 0, blocks = 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cu < 256) return false;
    const int cpw = tk_cpw(n_ctx);
    if (!cpw) return false;
    const void *k = tk_fn<1>();
    const size_t lds = tk_lds<1>();
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return false;
    // the grid (up to 505 workgroups) must be co-resident: two per CU
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k, 256, lds) == hipSuccess && blocks >= 2;
}

template <int CPW>
static bool tk_launch(PersistParams p, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        Q3T_HIP(hipFuncSetAttribute(tk_fn<CPW>(), hipFuncAttributeMaxDynamicSharedMemorySize, (int)tk_lds<CPW>()));
        attr = true;
    }
    const int nch = (p.n_ctx + CHK - 1) / CHK;
    p.roles_split = (nch + CPW - 1) / CPW;
    hipLaunchKernelGGL((k_tk_roles<CPW>), dim3(AW + 8 * p.roles_split + 1), dim3(256), tk_lds<CPW>(), s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}

bool persist_tk_roles(const PersistParams &p, hipStream_t s) {
    if (!p.L || p.n_layers <= 0 || p.n_layers > MAXL || !p.head || !p.logits || !p.hidden || !p.pos || !p.rope || !p.kc ||
        !p.vc || !p.gx || (p.gather && !(p.gs.tok && p.gs.tabs && p.gs.frame && p.gs.tr && p.gs.tr_len && p.gs.pad)) ||
        (!p.gather && !p.x_in) || (p.sel.mode != SEL_NONE && (p.sel.mode != SEL_CB0 || p.sel.V != VOC))) {
        set_error("persist_tk_roles: bad parameters");
        return false;
    }
    if (tk_cpw(p.n_ctx) != 1) { set_error("persist_tk_roles: context too long"); return false; }
    return tk_launch<1>(p, s);
}

}  // namespace q3t
