// persist.hip — the Talker decode step of one slot as ONE persistent launch (gfx950).  See persist.h for the
// hand-off protocol.  Geometry: one 256-thread workgroup per CU (256 on MI355X; the dynamic LDS request keeps it to
// one per CU); every phase's row split reproduces the launch-per-phase GEMV of gemv.hip lane for lane, so the step
// is bit-identical to enqueue_talker's 141-launch graph for chunk 64 (n_ctx <= 2048):
//   A  RMSNorm(attn_norm) + QKV          16 rows / workgroup   = k_gemv<1,1,1,PRO_RMS,8>
//   B  head norm + RoPE + KV append + split flash-decode (kv group w%8, split w/8; the last split combines) = k_attn
//   C  O-proj + residual                  4 rows / workgroup   = k_gemv<1,1,4,PRO_F16,4>
//   D  RMSNorm(ffn_norm) + gate/up + SwiGLU  12 units / wg     = k_gemv<2,1,2,PRO_RMS,4>
//   E  down + residual                    4 rows / workgroup   = k_gemv<1,1,4,PRO_F16,8>
//   head: RMSNorm(output_norm) + codec head 12 rows / wg, CB0 selection by the last workgroup (fused head select)
// Reference semantics: src/tts_transformer.cpp:1376-1512 (build_step_graph), :2416-2499 (CB0 processing).
#include "persist.h"
#include "persist_dev.h"
#include "select.h"

#include <algorithm>
#include <cstdlib>

#pragma clang fp contract(off)   // every rounding as written: bit-identical to k_attn / k_gemv

namespace q3t {

namespace {

constexpr int H = 1024, NH = 16, NKV = 8, D = 128, QKVN = (NH + 2 * NKV) * D, INTER = 3072, VOC = 3072;
constexpr int G = 256;          // workgroups (one per CU)
constexpr int MAXSPLIT = G / NKV;
constexpr int R = NH / NKV;     // q heads per kv head
constexpr int MAXL = 32;        // layers (pointer table in LDS)
constexpr int PSLOT = 264;      // granules per attention split partial: acc [2][128], m [2], l [2], pad to 4
constexpr int SELW = G - 1;     // the selecting workgroup (an attention workgroup only at 32 splits)
#ifndef Q3T_SEL_HOIST0
#define Q3T_SEL_HOIST0 1        // talker step: SELW loads the selection's per-slot inputs at launch start
#endif
#ifndef Q3T_BPROF
#define Q3T_BPROF 0             // development timeline: where phase B's mid stamp goes (0 after the q/k norm, 1 after
#endif                          // the score max, 2 after the P.V reduction; tools/dev/persist_timeline*.py)
#ifndef Q3T_NOSTREAM
#define Q3T_NOSTREAM 0          // development experiment: weight rows streamed only for the first layer (timing only)
#endif
#ifndef Q3T_SEL_HOIST1
#define Q3T_SEL_HOIST1 1        // code-predictor frame: the selectors load them at launch start
#endif

using pdev::ldgv;
using pdev::ld16;
using pdev::ldf4;
using pdev::ld8;
using pdev::g_put;
using pdev::g_ld;
using pdev::ld16_sc1;
using pdev::Ctl;
using pdev::g_wait;
using pdev::f4_of;

struct Lds {
    uint16_t xs[INTER];          // f16 activation tile of the current phase
    float xr[H];                 // x (layer input; O-proj residual)
    float xr2[H];                // x' (after attention; down-proj residual)
    float red[4][16];
    double dscr[8];
    float hs[16];
    // attention
    float raw[4 * D];            // q head 2g, q head 2g+1, k, v (raw QKV rows)
    float q_s[R][D];
    float kn_s[D], vn_s[D];
    float wred[4][R];
    float ared[4][R][D];
    float cm[R], cl[R];
    float sm[MAXSPLIT][R], sl[MAXSPLIT][R], sw[MAXSPLIT][R];
    unsigned last;
    SelLds sel;
    float pl[MAXSPLIT * 264];    // split-0 combiner: every split's partial, split order
    PLayerW layers[MAXL];
    const uint16_t *heads[16];   // code-predictor lm_heads (MODE 1)
    // (layers / heads: the pointer tables, copied once: a pointer fetched from global memory inside the chain would
    // make the next wait cover every weight stream in flight, vmcnt order)
};

__device__ __forceinline__ double block_sum_d(double v, double *scr) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = wave_sum_d(v);
    __syncthreads();
    if (lane == 0) scr[wave] = v;
    __syncthreads();
    return (scr[0] + scr[1]) + (scr[2] + scr[3]);
}

// RMSNorm of the f32 row held as thread t's elements 4t..4t+3 (K = 1024) -> f16 LDS tile; optional f32 side output
// (gemv.hip prologue: double sums, (x * scale) * w, f16 rounding)
__device__ __forceinline__ void rms_to_lds(float4 x, float4 w, float eps, Lds &S, float *side) {
    const int t = threadIdx.x;
    double ss = (double)(x.x * x.x) + (double)(x.y * x.y) + (double)(x.z * x.z) + (double)(x.w * x.w);
    ss = block_sum_d(ss, S.dscr);
    const float scale = 1.0f / sqrtf((float)(ss / H) + eps);
    const float y0 = (x.x * scale) * w.x, y1 = (x.y * scale) * w.y, y2 = (x.z * scale) * w.z, y3 = (x.w * scale) * w.w;
    if (side) *reinterpret_cast<float4 *>(side + 4 * t) = make_float4(y0, y1, y2, y3);
    uint2 h;
    h.x = (uint32_t)f2h(y0) | ((uint32_t)f2h(y1) << 16);
    h.y = (uint32_t)f2h(y2) | ((uint32_t)f2h(y3) << 16);
    *reinterpret_cast<uint2 *>(S.xs + 4 * t) = h;
}

// 16-lane-group rows over K = 1024: lane l16 holds k = l16*8 + tt*128, tt < 8 (KS = 1 / two K halves)
__device__ __forceinline__ void issue_rows_k1024(const uint16_t *W, int row, uint4 (&w)[8]) {
    const int l16 = threadIdx.x & 15;
    const uint16_t *r = W + (size_t)row * H + l16 * 8;
#pragma unroll
    for (int tt = 0; tt < 8; ++tt) w[tt] = ld16(r + tt * 128);
}
// KS = 4 rows (O: K 2048, 4 chunks of 128 per slice; down: K 3072, 6 chunks): slice = wave
template <int NC>
__device__ __forceinline__ void issue_rows_ks4(const uint16_t *W, int K, int row, uint4 (&w)[NC]) {
    const int l16 = threadIdx.x & 15, wave = threadIdx.x >> 6;
    const uint16_t *r = W + (size_t)row * K + wave * (NC * 128) + l16 * 8;
#pragma unroll
    for (int tt = 0; tt < NC; ++tt) w[tt] = ld16(r + tt * 128);
}

// MODE 0: the talker step (one pass of n_layers at p.pos[0], codec head, CB0 selection).
// MODE 1: the whole code-predictor frame (trt_code_predictor.cpp:484-600): 16 passes of the 5 layers, pass q at KV
// position q (16-position cache, always one split), pass q >= 1 ends with lm_head[q-1] + token selection by the last
// workgroup, whose token (a granule) feeds the next pass's embedding gather.  K/V rows written by an earlier pass of
// the same launch are read back by the same workgroup with sc1 loads (no stale L1 line).
// MODE 2: MODE 1 with the pass inputs of passes 1..15 read as projected f32 rows (p.xtab, the 1.7B layout).
template <int MODE, int CH>
__global__ void __launch_bounds__(256) k_persist(const PersistParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Lds &S = *reinterpret_cast<Lds *>(smem);
    constexpr int NP = CH / 16;   // positions per lane group pass (16 lanes per position, 16 positions per pass)
    const int w = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6, l16 = t & 15, grp = t >> 4;
    const int grp4 = lane >> 4;   // row of a KS = 4 GEMV
    Ctl c{p.err, false};
    const unsigned seq = __hip_atomic_load(p.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    auto TAG = [&](int ph) -> uint32_t { return ((seq * 1024u + (unsigned)ph) << 1) | 1u; };
    int pos = MODE == 0 ? p.pos[0] : 0;
    const int nsplit = MODE == 0 ? pos / CH + 1 : 1;
    const int nl = p.n_layers, npass = MODE == 0 ? 1 : 16, PPH = 5 * nl + 1;   // phases per pass
    constexpr int RPW = MODE == 0 ? 12 : 8;                                    // head rows per workgroup
    const int ag = w & (NKV - 1), as = w >> 3;   // attention role: kv group, split
    const bool att = as < nsplit;
    const bool has_pos = as == nsplit - 1;
    // code-predictor frame with the layer-0 QKV table: the 8 attention workgroups select each pass's token themselves
    // (no hand-off before the next pass's attention), workgroup 0 records it and hands it to the others (they need it
    // only for layer 0's residual row, off the chain); otherwise SELW selects and hands the token to everyone
    const bool tab = MODE >= 1 && p.qkvtab != nullptr;
    const bool selector = tab ? att : w == SELW;
    const bool committer = tab ? w == 0 : w == SELW;
    int cur_tok = MODE >= 1 ? p.gs.tok[0] : 0;   // tab: this attention workgroup's token of the previous pass
    const int pg = t >> 4, li = t & 15;          // attention: position group, 8-dim chunk

    // development timeline (p.prof): wall clock at wait start / input arrived / output published, per phase
#define PROF(ph, k)                                                                                  \
    do {                                                                                             \
        if (p.prof && t == 0) p.prof[((size_t)w * PROF_PH + (ph)) * 4 + (k)] = wall_clock64();       \
    } while (0)
    PROF(0, 3);
    uint4 wq[8], wo[4], wg[8], wu[8], wd[6], kr[NP], vr[NP];
    // issue schedule (each stream lands while the chain waits on other edges):
    //   wq(l+1) after D(l)'s input, K/V(l+1) after E(l)'s, wo(l) after A(l)'s, gate/up(l) after B(l)'s, wd(l) after C(l)'s;
    //   the attention workgroups issue wo(l) and gate/up(l) after publishing B(l) instead: a weight stream issued ahead
    //   of B's input poll, output stores and K/V append queues in front of them in the CU's memory pipeline, and B runs
    //   on those few workgroups alone (talker step 0.600 -> 0.569 ms, code-predictor frame 1.393 -> 1.366 ms, A/B)
    const int gu_unit = w * 12 + min(grp, 11);
    const int gu_row = (gu_unit >> 4) * 32 + (gu_unit & 15);
    auto issue_kv = [&](int layer, int kpos) {   // this split's cached K/V rows (clamped rows re-read row kpos)
        const size_t o = (size_t)layer * p.kv_layer + (size_t)ag * p.n_ctx * D;
        const int j0 = as * CH;
#pragma unroll
        for (int pi = 0; pi < NP; ++pi) {
            const int j = min(j0 + pi * 16 + pg, kpos);
            if constexpr (MODE >= 1) {
                kr[pi] = ld16_sc1(p.kc + o + (size_t)j * D + li * 8);
                vr[pi] = ld16_sc1(p.vc + o + (size_t)j * D + li * 8);
            } else {
                kr[pi] = ld16(p.kc + o + (size_t)j * D + li * 8);
                vr[pi] = ld16(p.vc + o + (size_t)j * D + li * 8);
            }
        }
    };
    if (t < p.n_layers) S.layers[t] = p.L[t];
    if (MODE >= 1 && t < 15) S.heads[t] = p.heads[t];
    // the selection's per-slot inputs (done, frame, seed, utterance, CB0 seen bytes) loaded before any wait, so that
    // none of these dependent loads sits between the last logits and the token
    SelPre spre;
    constexpr int SELM = MODE == 0 ? SEL_CB0 : SEL_CP;
    constexpr bool HOIST = MODE >= 1 ? Q3T_SEL_HOIST1 : Q3T_SEL_HOIST0;
    if (HOIST && p.sel.mode != SEL_NONE && selector) sel_prefetch<SELM>(p.sel, 0, spre);
    issue_rows_k1024(p.L[0].qkv, w * 16 + grp, wq);
    if (att) issue_kv(0, pos);
    float4 nwA = ldf4(p.L[0].attn_norm + 4 * t), nwD;   // attn_norm(l) / ffn_norm(l) for this thread's 4 elements
    float hn[2], rp[2];                                  // attention: head-norm weights and RoPE (cos, sin) of this lane

    __syncthreads();   // layer / head tables visible
    for (int pass = 0, ph0 = 0; pass < npass; ++pass, ph0 += PPH) {
    const bool head_here = MODE == 0 || pass > 0;
    if (MODE >= 1) pos = pass;
    for (int l = 0; l < nl; ++l) {
        const PLayerW Lw = S.layers[l];
        const bool st = !(Q3T_NOSTREAM && (pass > 0 || l > 0));
        const size_t kvo = (size_t)l * p.kv_layer + (size_t)ag * p.n_ctx * D;
        const bool from_tab = tab && l == 0 && pass >= 1;   // layer 0's QKV rows come from the table
        uint2 traw = make_uint2(0, 0);                      // from_tab: this thread's two raw QKV values
        // ================= A: x -> RMSNorm -> QKV rows
        float4 x;
        if (from_tab) {
            int tok = cur_tok;
            if (!att && pass >= 2) {
                uint32_t u1[1];
                g_wait<1>(p.gtok + pass - 1, TAG(ph0 - 1), u1, c);
                tok = min((int)u1[0], p.sel.V - 1);   // an aborted wait returns a stale payload: keep it in the table
            }
            if (att) {   // the attention operands straight from the table row (gi: B's layout of the raw row)
                const int gi = t < 128 ? ag * 256 + 2 * t : t < 192 ? NH * D + ag * D + 2 * (t - 128) : (NH + NKV) * D + ag * D + 2 * (t - 192);
                const size_t row = (size_t)(pass == 1 ? 0 : VOC + (pass - 2) * 2048) + tok;
                traw = ld8(p.qkvtab + row * QKVN + gi);
            }
            if constexpr (MODE == 2) {   // 1.7B: the projected row
                x = ldf4(p.xtab + ((size_t)(pass == 1 ? 0 : VOC + (pass - 2) * 2048) + tok) * H + 4 * t);
            } else {        // the residual row
                const uint2 hv = ld8(p.gs.tabs[pass - 1] + (size_t)tok * H + 4 * t);
                x = make_float4(h2f(hv.x & 0xffff), h2f(hv.x >> 16), h2f(hv.y & 0xffff), h2f(hv.y >> 16));
            }
        } else if (l == 0) {
            if (MODE == 0 && p.gather) {
                const GatherSum &gs = p.gs;
                const int *tk = gs.tok;
                uint2 hv[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) hv[j] = ld8(gs.tabs[j] + (size_t)tk[j] * H + 4 * t);
                const int fr = gs.frame[0];
                const float *extra = fr < gs.tr_len[0] ? gs.tr + (size_t)fr * H : gs.pad;
                const float4 ex = ldf4(extra + 4 * t);
                auto h4 = [](uint2 u) { return make_float4(h2f(u.x & 0xffff), h2f(u.x >> 16), h2f(u.y & 0xffff), h2f(u.y >> 16)); };
                x = h4(hv[0]);
#pragma unroll
                for (int j = 1; j < 16; ++j) { const float4 b = h4(hv[j]); x = make_float4(x.x + b.x, x.y + b.y, x.z + b.z, x.w + b.w); }
                x = make_float4(x.x + ex.x, x.y + ex.y, x.z + ex.z, x.w + ex.w);
            } else if (MODE == 0 || pass == 0) {
                x = ldf4(p.x_in + 4 * t);
            } else {   // code-predictor pass input: table row of the previous pass's token (pass 1: CB0)
                int tok = p.gs.tok[0];
                if (pass >= 2) {
                    uint32_t u1[1];
                    g_wait<1>(p.gtok + pass - 1, TAG(ph0 - 1), u1, c);
                    tok = min((int)u1[0], p.sel.V - 1);   // an aborted wait returns a stale payload: keep it in the table
                }
                if constexpr (MODE == 2) {
                    x = ldf4(p.xtab + ((size_t)(pass == 1 ? 0 : VOC + (pass - 2) * 2048) + tok) * H + 4 * t);
                } else {
                    const uint2 hv = ld8(p.gs.tabs[pass - 1] + (size_t)tok * H + 4 * t);
                    x = make_float4(h2f(hv.x & 0xffff), h2f(hv.x >> 16), h2f(hv.y & 0xffff), h2f(hv.y >> 16));
                }
            }
        } else {
            uint32_t u[4];
            PROF(ph0 + 5 * l + 0, 0);
            g_wait<4>(p.gx + 4 * t, TAG(ph0 + 5 * (l - 1) + 4), u, c);
            PROF(ph0 + 5 * l + 0, 1);
            x = f4_of(u);
        }
        if (att) {
            const float *nwv = wave == 2 ? Lw.kn : Lw.qn;
            hn[0] = nwv[lane];
            hn[1] = nwv[lane + 64];
            rp[0] = p.rope[(size_t)pos * D + 2 * lane];
            rp[1] = p.rope[(size_t)pos * D + 2 * lane + 1];
        }
        if (!att && st) issue_rows_ks4<4>(Lw.o, NH * D, w * 4 + grp4, wo);
        __syncthreads();
        *reinterpret_cast<float4 *>(S.xr + 4 * t) = x;
        if (!from_tab) {
        rms_to_lds(x, nwA, p.eps, S, nullptr);
        __syncthreads();
        if (l > 0) PROF(ph0 + 5 * l + 0, 3);
        {
            float acc = 0.0f;
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) acc = dot8(wq[tt], *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128), acc);
            acc = group_sum<16>(acc);
            if (l16 == 0) g_put(p.gqkv + w * 16 + grp, __float_as_uint(acc), TAG(ph0 + 5 * l + 0));
            PROF(ph0 + 5 * l + 0, 2);
        }
        }
        // code-predictor frame: the non-attention workgroups issue the next QKV (or head) rows here, as soon as A has
        // consumed the registers, instead of at D: D's input poll then no longer waits behind them (vmcnt order), and
        // they land while B runs on the attention workgroups (1.364 -> 1.336 ms per frame, A/B).  Not in the talker
        // step, whose code generation this perturbs (0.558 -> 0.586 ms).
        if constexpr (MODE >= 1) {
            if (!att && st) {
                if (l + 1 < nl) {
                    nwA = ldf4(S.layers[l + 1].attn_norm + 4 * t);
                    issue_rows_k1024(S.layers[l + 1].qkv, w * 16 + grp, wq);
                } else if (head_here) {
                    nwA = ldf4(p.out_norm + 4 * t);
                    issue_rows_k1024(S.heads[pass - 1], w * RPW + min(grp, RPW - 1), wq);
                } else if (!tab) {
                    nwA = ldf4(S.layers[0].attn_norm + 4 * t);
                    issue_rows_k1024(S.layers[0].qkv, w * 16 + grp, wq);
                }
            }
        }
        // ================= B: attention (kv group ag, split as)
        if (!att) {
            nwD = ldf4(Lw.ffn_norm + 4 * t);
            if (st) issue_rows_k1024(Lw.gu, gu_row, wg);
            if (st) issue_rows_k1024(Lw.gu, gu_row + 16, wu);
            // talker step: the down rows too (they land while the attention runs, so that D's poll does not wait
            // for them behind C; 0.570 -> 0.560 ms A/B; no gain in the code-predictor frame, whose B is short)
            if (MODE == 0 && st) issue_rows_ks4<6>(Lw.down, INTER, w * 4 + grp4, wd);
        } else {
            {
                uint32_t u[2];
                const int gi = t < 128 ? ag * 256 + 2 * t : t < 192 ? NH * D + ag * D + 2 * (t - 128) : (NH + NKV) * D + ag * D + 2 * (t - 192);
                PROF(ph0 + 5 * l + 1, 0);
                if (from_tab) { u[0] = traw.x; u[1] = traw.y; }
                else g_wait<2>(p.gqkv + gi, TAG(ph0 + 5 * l + 0), u, c);
                PROF(ph0 + 5 * l + 1, 1);
                S.raw[2 * t] = __uint_as_float(u[0]);
                S.raw[2 * t + 1] = __uint_as_float(u[1]);
            }
            __syncthreads();
            {   // wave v: q head 0 / q head 1 / k (head norm + RoPE) / v (f16 rounding)
                const int v = wave;
                if (v == 3) {
#pragma unroll
                    for (int e = 0; e < 2; ++e) S.vn_s[lane + 64 * e] = f16r(S.raw[3 * D + lane + 64 * e]);
                } else {
                    const float *src = S.raw + v * D;
                    float xx[2];
                    double ss = 0.0;
#pragma unroll
                    for (int e = 0; e < 2; ++e) { xx[e] = src[lane + 64 * e]; ss += (double)__fmul_rn(xx[e], xx[e]); }
                    ss = wave_sum_d(ss);
                    const float scale = 1.0f / sqrtf((float)(ss / D) + p.eps);
#pragma unroll
                    for (int e = 0; e < 2; ++e) xx[e] = (xx[e] * scale) * hn[e];
                    const float cs = rp[0], sn = rp[1];
                    const float y0 = opaque(opaque(xx[0] * cs) - opaque(xx[1] * sn));   // as k_attn: three roundings
                    const float y1 = opaque(opaque(xx[0] * sn) + opaque(xx[1] * cs));
                    float *dst = v == 2 ? S.kn_s : S.q_s[v];
                    dst[lane] = f16r(y0);
                    dst[lane + 64] = f16r(y1);
                }
            }
            __syncthreads();
            if (Q3T_BPROF == 0) PROF(ph0 + 5 * l + 1, 3);
            if (has_pos && t < D) {   // KV append at pos (read by later launches only)
                p.kc[kvo + (size_t)pos * D + t] = f2h(S.kn_s[t]);
                p.vc[kvo + (size_t)pos * D + t] = f2h(S.vn_s[t]);
            }
            const int j0 = as * CH;
            const float kq_scale = 1.0f / sqrtf((float)D);
            float q8[R][8];
#pragma unroll
            for (int h = 0; h < R; ++h)
#pragma unroll
                for (int e = 0; e < 8; ++e) q8[h][e] = S.q_s[h][li * 8 + e];
            float sc[NP][R];
            bool ok[NP];
            uint32_t qp[R][4];
#pragma unroll
            for (int h = 0; h < R; ++h) pack_q8(q8[h], qp[h]);
#pragma unroll
            for (int pi = 0; pi < NP; ++pi) {
                const int j = j0 + pi * 16 + pg;
                ok[pi] = j <= pos;
#pragma unroll
                for (int h = 0; h < R; ++h) {
                    float s;
                    if constexpr (Q3T_ATTN_DOT2) {
                        s = score8(j == pos ? pack8f(&S.kn_s[li * 8]) : kr[pi], qp[h]);
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
                        s = 0.0f;
#pragma unroll
                        for (int e = 0; e < 8; ++e) s = __fmaf_rn(k8[e], q8[h][e], s);   // explicit fma: identical in k_attn and persist.hip
                    }
                    s = group_sum<16>(s);
                    sc[pi][h] = ok[pi] ? __fmul_rn(s, kq_scale) : -INFINITY;
                }
            }
            float M[R], Lsum[R];
#pragma unroll
            for (int h = 0; h < R; ++h) {
                float m = sc[0][h];
#pragma unroll
                for (int pi = 1; pi < NP; ++pi) m = fmaxf(m, sc[pi][h]);
                m = rows_max(m);
                if (lane == 0) S.wred[wave][h] = m;
            }
            __syncthreads();
#pragma unroll
            for (int h = 0; h < R; ++h) M[h] = fmaxf(fmaxf(S.wred[0][h], S.wred[1][h]), fmaxf(S.wred[2][h], S.wred[3][h]));
            __syncthreads();
            if (Q3T_BPROF == 1) PROF(ph0 + 5 * l + 1, 3);
            float pr[NP][R];
#pragma unroll
            for (int h = 0; h < R; ++h) {
                float lsum = 0.0f;
#pragma unroll
                for (int pi = 0; pi < NP; ++pi) {
                    pr[pi][h] = ok[pi] ? exp_sm(__fsub_rn(sc[pi][h], M[h])) : 0.0f;
                    lsum += pr[pi][h];
                }
                lsum = rows_sum(lsum);
                if (lane == 0) S.wred[wave][h] = lsum;
            }
            float acc[R][8];
#pragma unroll
            for (int h = 0; h < R; ++h)
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[h][e] = 0.0f;
#pragma unroll
            for (int pi = 0; pi < NP; ++pi) {
                const int j = j0 + pi * 16 + pg;
                float v8[8];
                if (j == pos) {
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
                    for (int e = 0; e < 8; ++e) acc[h][e] = __fmaf_rn(pr[pi][h], ok[pi] ? v8[e] : 0.0f, acc[h][e]);
            }
#pragma unroll
            for (int h = 0; h < R; ++h)
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float a = rows_sum(acc[h][e]);
                    if (lane < 16) S.ared[wave][h][li * 8 + e] = a;
                }
            __syncthreads();
            if (Q3T_BPROF == 2) PROF(ph0 + 5 * l + 1, 3);
#pragma unroll
            for (int h = 0; h < R; ++h) Lsum[h] = (S.wred[0][h] + S.wred[1][h]) + (S.wred[2][h] + S.wred[3][h]);
            uint64_t *gout = p.gattn + (size_t)ag * R * (D / 2);
            if (nsplit == 1) {
                if (t < R * D / 2) {
                    const int h = t / (D / 2), d = 2 * (t % (D / 2));
                    const float a0 = (S.ared[0][h][d] + S.ared[1][h][d]) + (S.ared[2][h][d] + S.ared[3][h][d]);
                    const float a1 = (S.ared[0][h][d + 1] + S.ared[1][h][d + 1]) + (S.ared[2][h][d + 1] + S.ared[3][h][d + 1]);
                    g_put(gout + t, (uint32_t)f2h(a0 / Lsum[h]) | ((uint32_t)f2h(a1 / Lsum[h]) << 16), TAG(ph0 + 5 * l + 1));
                }
            } else {
                // splits >= 1 publish their partial (acc [2][128], m [2], l [2]) as granules; split 0 polls them and
                // combines in split order with k_attn's arithmetic (bit-identical), then publishes the output
                uint64_t *gp = p.gpart + (size_t)ag * MAXSPLIT * PSLOT;
                float *pl = S.pl;
                if (as > 0) {
                    uint64_t *mine = gp + (size_t)as * PSLOT;
                    {
                        const int h = t / D, d = t % D;
                        const float a = (S.ared[0][h][d] + S.ared[1][h][d]) + (S.ared[2][h][d] + S.ared[3][h][d]);
                        g_put(mine + t, __float_as_uint(a), TAG(ph0 + 5 * l + 1));
                    }
                    if (t < PSLOT - R * D) {
                        const float v = t < R ? M[t] : t < 2 * R ? Lsum[t - R] : 0.0f;
                        g_put(mine + R * D + t, __float_as_uint(v), TAG(ph0 + 5 * l + 1));
                    }
                } else {
                    {
                        const int h = t / D, d = t % D;
                        pl[t] = (S.ared[0][h][d] + S.ared[1][h][d]) + (S.ared[2][h][d] + S.ared[3][h][d]);
                        if (t < R) { pl[R * D + t] = M[t]; pl[R * D + R + t] = Lsum[t]; }
                    }
                    const int n = (nsplit - 1) * PSLOT;
                    for (int i0 = 4 * t; i0 < n; i0 += 1024) {
                        uint32_t u4[4];
                        g_wait<4>(gp + PSLOT + i0, TAG(ph0 + 5 * l + 1), u4, c);
#pragma unroll
                        for (int q = 0; q < 4; ++q) pl[PSLOT + i0 + q] = __uint_as_float(u4[q]);
                    }
                    __syncthreads();
                    if (t < R) {
                        float mx = -INFINITY;
                        for (int s2 = 0; s2 < nsplit; ++s2) mx = fmaxf(mx, pl[s2 * PSLOT + R * D + t]);
                        float lt = 0.0f;
                        for (int s2 = 0; s2 < nsplit; ++s2)
                            lt = __fmaf_rn(pl[s2 * PSLOT + R * D + R + t], expf(pl[s2 * PSLOT + R * D + t] - mx), lt);
                        S.cm[t] = mx;
                        S.cl[t] = lt;
                    }
                    __syncthreads();
                    for (int i = t; i < nsplit * R; i += 256) {
                        const int s2 = i / R, h = i % R;
                        S.sw[s2][h] = expf(pl[s2 * PSLOT + R * D + h] - S.cm[h]);
                    }
                    __syncthreads();
                    if (t < R * D / 2) {
                        const int h = t / (D / 2), d = 2 * (t % (D / 2));
                        float a2[2];
#pragma unroll
                        for (int q = 0; q < 2; ++q) {
                            float a = 0.0f;
                            for (int s2 = 0; s2 < nsplit; ++s2) a = __fmaf_rn(pl[s2 * PSLOT + h * D + d + q], S.sw[s2][h], a);
                            a2[q] = a;
                        }
                        g_put(gout + t, (uint32_t)f2h(a2[0] / S.cl[h]) | ((uint32_t)f2h(a2[1] / S.cl[h]) << 16), TAG(ph0 + 5 * l + 1));
                    }
                }
            }
        }
        PROF(ph0 + 5 * l + 1, 2);
        if (att) {   // (the streams of the other workgroups are in flight since A / B; ffn_norm too: a load issued
                     // after B's input poll would hold the attention body's K/V waits, vmcnt order)
            nwD = ldf4(Lw.ffn_norm + 4 * t);
            if (st) issue_rows_ks4<4>(Lw.o, NH * D, w * 4 + grp4, wo);
            if (st) issue_rows_k1024(Lw.gu, gu_row, wg);
            if (st) issue_rows_k1024(Lw.gu, gu_row + 16, wu);
        }
        // ================= C: O-proj + residual -> x'
        {
            uint32_t u[4];
            PROF(ph0 + 5 * l + 2, 0);
            g_wait<4>(p.gattn + 4 * t, TAG(ph0 + 5 * l + 1), u, c);
            PROF(ph0 + 5 * l + 2, 1);
            if ((MODE != 0 || att) && st) issue_rows_ks4<6>(Lw.down, INTER, w * 4 + grp4, wd);
            __syncthreads();
            *reinterpret_cast<uint4 *>(S.xs + 8 * t) = make_uint4(u[0], u[1], u[2], u[3]);
            __syncthreads();
            float acc = 0.0f;
#pragma unroll
            for (int tt = 0; tt < 4; ++tt)
                acc = dot8(wo[tt], *reinterpret_cast<const uint4 *>(S.xs + wave * 512 + l16 * 8 + tt * 128), acc);
            acc = group_sum<16>(acc);
            if (l16 == 0) S.red[wave][grp4] = acc;
            __syncthreads();
            if (t < 4) {
                const float s = S.red[0][t] + S.red[1][t] + S.red[2][t] + S.red[3][t];
                const int row = w * 4 + t;
                g_put(p.gx2 + row, __float_as_uint(S.xr[row] + s), TAG(ph0 + 5 * l + 2));
            }
            PROF(ph0 + 5 * l + 2, 2);
        }
        // ================= D: RMSNorm(ffn_norm) + gate/up + SwiGLU -> h
        {
            uint32_t u[4];
            PROF(ph0 + 5 * l + 3, 0);
            g_wait<4>(p.gx2 + 4 * t, TAG(ph0 + 5 * l + 2), u, c);
            PROF(ph0 + 5 * l + 3, 1);
            if ((MODE >= 1 && !att) || !st) {
                // (issued at A)
            } else if (l + 1 < nl) {
                nwA = ldf4(S.layers[l + 1].attn_norm + 4 * t);
                issue_rows_k1024(S.layers[l + 1].qkv, w * 16 + grp, wq);
            } else if (head_here) {
                nwA = ldf4(p.out_norm + 4 * t);
                issue_rows_k1024(MODE == 0 ? p.head : S.heads[pass - 1], w * RPW + min(grp, RPW - 1), wq);
            } else if (!tab) {   // code-predictor pass 0 (no head): the next pass's layer 0
                nwA = ldf4(S.layers[0].attn_norm + 4 * t);
                issue_rows_k1024(S.layers[0].qkv, w * 16 + grp, wq);
            }
            const float4 x2 = f4_of(u);
            __syncthreads();
            *reinterpret_cast<float4 *>(S.xr2 + 4 * t) = x2;
            rms_to_lds(x2, nwD, p.eps, S, nullptr);
            __syncthreads();
            PROF(ph0 + 5 * l + 3, 3);
            float a0 = 0.0f, a1 = 0.0f, b0 = 0.0f, b1 = 0.0f;   // gate / up, K halves 0 and 1
#pragma unroll
            for (int tt = 0; tt < 4; ++tt) {
                const uint4 xv = *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128);
                a0 = dot8(wg[tt], xv, a0);
                b0 = dot8(wu[tt], xv, b0);
            }
#pragma unroll
            for (int tt = 4; tt < 8; ++tt) {
                const uint4 xv = *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128);
                a1 = dot8(wg[tt], xv, a1);
                b1 = dot8(wu[tt], xv, b1);
            }
            a0 = group_sum<16>(a0); a1 = group_sum<16>(a1);
            b0 = group_sum<16>(b0); b1 = group_sum<16>(b1);
            if (l16 == 0 && grp < 12) S.hs[grp] = silu_f(a0 + a1) * (b0 + b1);
            __syncthreads();
            if (t < 6) g_put(p.gh + w * 6 + t, (uint32_t)f2h(S.hs[2 * t]) | ((uint32_t)f2h(S.hs[2 * t + 1]) << 16), TAG(ph0 + 5 * l + 3));
            PROF(ph0 + 5 * l + 3, 2);
        }
        // ================= E: down + residual -> x (next layer input)
        {
            uint32_t u[6];
            PROF(ph0 + 5 * l + 4, 0);
            g_wait<6>(p.gh + 6 * t, TAG(ph0 + 5 * l + 3), u, c);
            PROF(ph0 + 5 * l + 4, 1);
            if (att && l + 1 < nl) issue_kv(l + 1, pos);
            else if (att && !head_here && pass + 1 < npass) issue_kv(0, pos + 1);
            __syncthreads();
            *reinterpret_cast<uint2 *>(S.xs + 12 * t) = make_uint2(u[0], u[1]);
            *reinterpret_cast<uint2 *>(S.xs + 12 * t + 4) = make_uint2(u[2], u[3]);
            *reinterpret_cast<uint2 *>(S.xs + 12 * t + 8) = make_uint2(u[4], u[5]);
            __syncthreads();
            float acc = 0.0f;
#pragma unroll
            for (int tt = 0; tt < 6; ++tt)
                acc = dot8(wd[tt], *reinterpret_cast<const uint4 *>(S.xs + wave * 768 + l16 * 8 + tt * 128), acc);
            acc = group_sum<16>(acc);
            if (l16 == 0) S.red[wave][grp4] = acc;
            __syncthreads();
            if (t < 4) {
                const float s = S.red[0][t] + S.red[1][t] + S.red[2][t] + S.red[3][t];
                const int row = w * 4 + t;
                g_put(p.gx + row, __float_as_uint(S.xr2[row] + s), TAG(ph0 + 5 * l + 4));
            }
            PROF(ph0 + 5 * l + 4, 2);
        }
    }
    // ================= head: RMSNorm(output_norm) -> hidden (side output) -> codec head / lm_head logits -> selection
    if (head_here) {
        uint32_t u[4];
        const int hph = ph0 + 5 * nl;
        PROF(hph, 0);
        g_wait<4>(p.gx + 4 * t, TAG(ph0 + 5 * (nl - 1) + 4), u, c);
        PROF(hph, 1);
        const float4 x = f4_of(u);
        __syncthreads();
        rms_to_lds(x, nwA, p.eps, S, w == 0 ? p.hidden : nullptr);
        __syncthreads();
        // head rows are in registers now: the next pass's layer-0 streams can follow
        uint4 wh[8];
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) wh[tt] = wq[tt];
        if (MODE >= 1 && pass + 1 < npass) {
            if (!tab && Q3T_NOSTREAM == 0) {
                nwA = ldf4(S.layers[0].attn_norm + 4 * t);
                issue_rows_k1024(S.layers[0].qkv, w * 16 + grp, wq);
            }
            if (att) issue_kv(0, pos + 1);
        }
        float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) a0 = dot8(wh[tt], *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128), a0);
#pragma unroll
        for (int tt = 4; tt < 8; ++tt) a1 = dot8(wh[tt], *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128), a1);
        a0 = group_sum<16>(a0);
        a1 = group_sum<16>(a1);
        if (l16 == 0 && grp < RPW) {
            const float lg = a0 + a1;
            p.logits[w * RPW + grp] = lg;   // read after the launch only (host, tests)
            g_put(p.glog + w * RPW + grp, __float_as_uint(lg), TAG(hph));
        }
        PROF(hph, 2);
        // one fixed workgroup gathers the logits granules and selects: no arrival ticket, no store drain and no
        // reload of the logits row on the chain (the last 256 -> 1 fan-in of the step)
        if (selector) {
            int tok = -1;
            SelectSpec sp = p.sel;
            if (MODE >= 1) sp.step = pass - 1;
            const bool rec = p.prof && t == 0 && w == (tab ? 1 : SELW);   // one selector records its timeline
            if (rec) p.prof[((size_t)w * PROF_PH + hph) * 4 + 3] = wall_clock64();   // selection start
            if (sp.mode != SEL_NONE) {
                constexpr int VPT = MODE == 0 ? VOC / G : 2048 / G;
                uint32_t u[VPT];
                g_wait<VPT>(p.glog + t * VPT, TAG(hph), u, c);
                float v[SEL_VPT_MAX];
#pragma unroll
                for (int e = 0; e < SEL_VPT_MAX; ++e) v[e] = e < VPT ? __uint_as_float(u[e]) : -INFINITY;
                if (!HOIST) sel_prefetch<SELM>(sp, 0, spre);
                tok = select_token_pre<SELM>(sp, spre, v, S.sel);
            }
            if (rec) p.prof[((size_t)0 * PROF_PH + hph) * 4 + 3] = wall_clock64();   // selection end (row 0)
            if (committer && t == 0) {
                if (MODE >= 1 && pass + 1 < npass) g_put(p.gtok + pass, (uint32_t)max(tok, 0), TAG(hph));
                if (tok >= 0) select_commit(sp, 0, tok);
                if (pass + 1 == npass) __hip_atomic_store(p.seq, seq + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (MODE >= 1) cur_tok = max(tok, 0);
        }
    }
    }   // passes
}

struct StateLayout {
    size_t gx, gx2, gqkv, gattn, gh, part, gpart, gop, gtok, glog, ctr, total;
    StateLayout() {
        size_t o = 0;
        auto take = [&](size_t b) { const size_t r = o; o += (b + 255) & ~(size_t)255; return r; };
        gx = take(H * 8);
        gx2 = take(H * 8);
        gqkv = take(QKVN * 8);
        gattn = take(NH * D / 2 * 8);
        gh = take(INTER / 2 * 8);
        part = take((size_t)NKV * MAXSPLIT * R * (D + 2) * 4);
        gpart = take((size_t)NKV * MAXSPLIT * PSLOT * 8);
        gop = take((size_t)4 * H * 8);
        gtok = take(16 * 8);
        glog = take(VOC * 8);
        ctr = take(64 * 4);
        total = o;
    }
};

}  // namespace

#ifdef Q3T_DEV
static const int g_min_chunk = [] { const char *e = std::getenv("Q3T_PERSIST_CH"); return e ? std::atoi(e) : 64; }();
#else
static constexpr int g_min_chunk = 64;
#endif
size_t persist_qkv_table_rows() { return (size_t)VOC + 14 * 2048; }

int persist_chunk(int n_ctx) {
    int ch = g_min_chunk;
    while (ch * MAXSPLIT < n_ctx) ch += 64;
    return ch;
}

bool persist_supported(int hidden, int n_heads, int n_kv, int head_dim, int inter, int vocab, int n_ctx, int n_cu) {
    return hidden == H && n_heads == NH && n_kv == NKV && head_dim == D && inter == INTER && vocab == VOC && n_cu == G &&
           persist_chunk(n_ctx) <= 256;
}

size_t persist_state_bytes() { return StateLayout().total; }

static size_t persist_lds() { return std::max(sizeof(Lds), (size_t)96 * 1024); }   // > 80 KB: one workgroup per CU

bool persist_resident(int device, int n_ctx, bool cp_frame) {
    int n_cu = 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cu < G) return false;
    auto fits = [&](const void *f) {
        int blocks = 0;
        if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)persist_lds()) != hipSuccess) return false;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, f, 256, persist_lds()) == hipSuccess && blocks >= 1;
    };
    const void *k = nullptr;
    switch (persist_chunk(n_ctx)) {
        case 64: k = reinterpret_cast<const void *>(&k_persist<0, 64>); break;
        case 128: k = reinterpret_cast<const void *>(&k_persist<0, 128>); break;
        case 192: k = reinterpret_cast<const void *>(&k_persist<0, 192>); break;
        case 256: k = reinterpret_cast<const void *>(&k_persist<0, 256>); break;
        default: return false;
    }
    if (!fits(k)) return false;
    return !cp_frame || (fits(reinterpret_cast<const void *>(&k_persist<1, 16>)) &&
                         fits(reinterpret_cast<const void *>(&k_persist<2, 16>)));
}

bool persist_resident_cp(int device) {
    int n_cu = 0, blocks = 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cu < G) return false;
    for (const void *k : {reinterpret_cast<const void *>(&k_persist<1, 16>), reinterpret_cast<const void *>(&k_persist<2, 16>)}) {
        if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)persist_lds()) != hipSuccess) return false;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k, 256, persist_lds()) != hipSuccess || blocks < 1) return false;
    }
    return true;
}

void persist_carve(uint8_t *base, PersistParams &p) {
    const StateLayout L;
    p.gx = reinterpret_cast<uint64_t *>(base + L.gx);
    p.gx2 = reinterpret_cast<uint64_t *>(base + L.gx2);
    p.gqkv = reinterpret_cast<uint64_t *>(base + L.gqkv);
    p.gattn = reinterpret_cast<uint64_t *>(base + L.gattn);
    p.gh = reinterpret_cast<uint64_t *>(base + L.gh);
    p.part = reinterpret_cast<float *>(base + L.part);
    p.gpart = reinterpret_cast<uint64_t *>(base + L.gpart);
    p.gop = reinterpret_cast<uint64_t *>(base + L.gop);
    p.gtok = reinterpret_cast<uint64_t *>(base + L.gtok);
    p.glog = reinterpret_cast<uint64_t *>(base + L.glog);
    unsigned *ctr = reinterpret_cast<unsigned *>(base + L.ctr);
    p.seq = ctr;               // [0]
    p.head_ticket = ctr + 16;  // own 64-B line
    p.err = ctr + 32;
    p.ticket = ctr + 48;       // [8]
}

template <int MODE, int CH>
static bool launch_ch(const PersistParams &p, hipStream_t s) {
    const size_t lds = persist_lds();
    static bool attr = false;
    if (!attr) {
        Q3T_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_persist<MODE, CH>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr = true;
    }
    hipLaunchKernelGGL((k_persist<MODE, CH>), dim3(G), dim3(256), lds, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}

bool persist_talker_step(const PersistParams &p, hipStream_t s) {
    if (!p.L || p.n_layers <= 0 || p.n_layers > MAXL || !p.head || !p.logits || !p.hidden || !p.pos || !p.rope || !p.kc || !p.vc || !p.gx ||
        (p.gather && !(p.gs.tok && p.gs.tabs && p.gs.frame && p.gs.tr && p.gs.tr_len && p.gs.pad)) || (!p.gather && !p.x_in) ||
        (p.sel.mode != SEL_NONE && (p.sel.mode != SEL_CB0 || p.sel.V != VOC))) {
        set_error("persist_talker_step: bad parameters");
        return false;
    }
    switch (persist_chunk(p.n_ctx)) {
        case 64: return launch_ch<0, 64>(p, s);
        case 128: return launch_ch<0, 128>(p, s);
        case 192: return launch_ch<0, 192>(p, s);
        case 256: return launch_ch<0, 256>(p, s);
        default: set_error("persist_talker_step: context too long"); return false;
    }
}

bool persist_cp_frame(const PersistParams &p, hipStream_t s) {
    if (!p.L || p.n_layers <= 0 || p.n_layers > MAXL || !p.heads || !p.logits || !p.rope || !p.kc || !p.vc || !p.gx ||
        !p.x_in || !p.gs.tok || !p.gs.tabs || p.n_ctx != 16 || p.sel.mode != SEL_CP || p.sel.V != 2048) {
        set_error("persist_cp_frame: bad parameters");
        return false;
    }
    // MODE 2: the pass inputs as projected f32 rows (1.7B); its own instantiation, so the 0.6B frame's register
    // allocation does not see the branch (+22 us per frame when it did)
    return p.xtab ? launch_ch<2, 16>(p, s) : launch_ch<1, 16>(p, s);
}

}  // namespace q3t
