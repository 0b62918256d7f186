// persist_cp.hip — the code-predictor frame of one slot (src/trt_code_predictor.cpp:484-600,
// scripts/export_code_predictor.py:132-231: 16 passes of the 5-layer stack, lm_head[p-1] + token selection after pass
// p >= 1) as ONE persistent launch whose workgroups each keep ONE role for the whole frame.
//
// Why roles.  The frame is a chain of ~400 dependent hand-offs; its weights (157 MB, Infinity-Cache resident) stream
// beside the chain at no measurable cost (a build that streamed no weight rows at all ran the frame 1.25 vs 1.31 ms).
// What a hand-off costs depends on how many workgroups publish and poll it (tools/dev/edgebench.hip, 1024-granule
// vectors): 256 producers -> 256 consumers 2.57 us per edge, a chain of edges between disjoint role groups of 8-64
// workgroups 1.38 us.  persist.hip's frame runs every phase on all 256 workgroups; here each phase runs on its own
// group, so every edge has few producers and few pollers:
//
//   role (workgroups)     per layer                                     input edge (producers -> pollers)
//   QKV   [0, 64)         RMSNorm(attn_norm) + 64 QKV rows; lm_head      x      DN 56 -> 64
//                         (32 rows) after the last layer
//   ATT   [64, 72)        kv group w-64: head norm + RoPE, K/V append    QKV    8 -> 1 per group (table row at layer 0)
//                         into an LDS-resident 16-position cache,
//                         attention; every ATT workgroup selects the
//                         token of each pass (8 x the same result)
//   O     [72, 104)       32 O-projection rows + residual                attn   8 -> 32
//   GU    [104, 200)      RMSNorm(ffn_norm) + 32 gate/up SwiGLU units    x'     32 -> 96
//   DN    [200, 256)      18-19 down rows + residual                     h      96 -> 56
//
// Every row keeps persist.hip's (and the per-op GEMVs') lane split and reduction order, so the frame is bit-identical to
// the launch-per-op graph (tests/test_gpu_persist.py).  Each workgroup holds only its role's weights (<= 128 VGPRs),
// issued right after its phase for the next layer, a whole layer before they are needed.  Layer 0 of passes 1..15
// reads its raw QKV row from the per-token table (Engine::build_cp_qkv_table); pass 0's last layer stops after its
// K/V append (no head consumes its output).
#include "persist.h"
#include "persist_dev.h"
#ifdef Q3T_DEV
// development timeline: the selection's stage stamps (select.h SEL_STAMP) in phase slots 440.. of the profile rows
namespace q3t { __device__ uint64_t *g_selprof = nullptr; }
#define SEL_STAMP(k)                                                                                              \
    do {                                                                                                          \
        if (threadIdx.x == 0 && q3t::g_selprof)                                                                   \
            q3t::g_selprof[((size_t)blockIdx.x * PROF_PH + 440 + ((k) >> 2)) * 4 + ((k) & 3)] = wall_clock64();   \
    } while (0)
#endif
#include "select.h"

#pragma clang fp contract(off)   // every rounding as written: bit-identical to k_gemv / k_attn / k_persist

#ifndef Q3T_CP_SGATE   // the selection's logits poll behind the same one-lane gate
#define Q3T_CP_SGATE 1
#endif
#ifndef Q3T_CP_GATE   // polls: lane 0 of each wave gates on the wave's first granule before the sweep (talker form)
#define Q3T_CP_GATE 1
#endif
#ifndef Q3T_CP_WPUB   // QKV phase: each wave publishes its own 16 rows (one line; 0: through LDS, wave 0 publishes all 64)
#define Q3T_CP_WPUB 1
#endif
#ifndef Q3T_CP_PUT_FIRST   // a role's publish: the other waves issue the next weight prefetch only after wave 0's store
#define Q3T_CP_PUT_FIRST 1   // (their loads, 128 KB per QKV workgroup, otherwise queue ahead of it in the CU's memory pipe)
#endif
#ifndef Q3T_CP_MMS
#define Q3T_CP_MMS 16   // granule stride of the head workgroups' max / min pairs (16: a line each; 2: packed)
#endif
#ifndef Q3T_CP_RANGE
#define Q3T_CP_RANGE 1    // the head workgroups publish each 32-row block's max / min (0: the selection's own B1)
#endif
#ifndef Q3T_CP_PREDIV
#define Q3T_CP_PREDIV 1   // the head workgroups publish the rows divided by T (0: the selecting workgroups divide)
#endif
#ifndef Q3T_CP_WAIT
#define Q3T_CP_WAIT g_waitc   // contiguous granules (16-byte loads; development: g_wait_gated)
#endif

namespace q3t {

namespace {
using namespace pdev;

constexpr int H = 1024, NH = 16, NKV = 8, D = 128, QKVN = (NH + 2 * NKV) * D, INTER = 3072, VOC = 3072, CPV = 2048;
constexpr int G = 256, NLC = 5, NPASS = 16, PPH = 5 * NLC + 1, MMS = Q3T_CP_MMS;
constexpr int QW = 0, NQ = 64;      // QKV rows 64 (4 x 16) of 4096; lm_head rows 32 (2 x 16) of 2048
constexpr int AW = 64, NA = 8;      // attention of kv group w - AW, token selection
constexpr int OW = 72, NO = 32;     // O-projection rows 32 (8 x 4) of 1024
constexpr int UW = 104, NU = 96;    // gate/up SwiGLU units 32 (2 x 16) of 3072
constexpr int DW = 200, ND = 56;    // down rows 18-19 (5 x 4) of 1024
static_assert(QW + NQ == AW && AW + NA == OW && OW + NO == UW && UW + NU == DW && DW + ND == G, "roles cover the grid");
static_assert(NQ * 64 == QKVN && NQ * 32 == CPV && NO * 32 == H && NU * 32 == INTER && ND * 19 >= H, "role row counts");

struct CLds {
    uint16_t xs[INTER];          // f16 activation tile of the current phase
    float xr[32];                // residual rows of this workgroup (O / DN)
    float red[2][4][32];         // K-slice partial sums [layer parity][wave][row] (O / DN)
    float outv[64];              // QKV / head rows staged for one whole-line publish
    double dscr[8];
    float hs[32];                // SwiGLU outputs (GU)
    float q_s[2][D];
    float wred[4][2], wsum[4][2];   // per-wave softmax max / sum (apart: no barrier between them)
    float ared[4][2][D];
    uint16_t kc[NLC][16][D], vc[NLC][16][D];   // ATT: this kv group's 16-position K/V cache (f16), the whole frame
    float qn[NLC][D], kn[NLC][D];              // ATT: head-norm weights
    float rope[16][D];                         // ATT: (cos, sin) pairs of positions 0..15
    SelLds sel;
    PLayerW layers[NLC];
    const uint16_t *heads[16];
    const uint16_t *tabs[16];
};

struct Ctx {
    const PersistParams &p;
    CLds &S;
    Ctl c;
    unsigned seq;
    __device__ uint32_t tag(int ph) const { return ((seq * 1024u + (unsigned)ph) << 1) | 1u; }
};

#define PROF(ph, k)                                                                                           \
    do {                                                                                                      \
        if (X.p.prof && threadIdx.x == 0 && blockIdx.x < PROF_WG) X.p.prof[((size_t)blockIdx.x * PROF_PH + (ph)) * 4 + (k)] = wall_clock64(); \
    } while (0)

__device__ __forceinline__ int ph_of(int pass, int l, int k) { return pass * PPH + 5 * l + k; }

// ------------------------------------------------------------------ QKV rows (+ lm_head after the last layer)
__device__ __forceinline__ void role_qkv(Ctx &X) {
    const PersistParams &p = X.p;
    CLds &S = X.S;
    const int i = blockIdx.x - QW, t = threadIdx.x, l16 = t & 15, grp = t >> 4;
    const float temp = p.sel.temperature;
    const bool samp = temp > 0.0f && Q3T_CP_RANGE;
    uint4 wq[4][8];
    float4 nw;
    auto issue_qkv = [&](int l) {
        const uint16_t *W = S.layers[l].qkv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // Q3T_CP_WPUB: wave w owns rows 16w .. 16w + 15 (row 16w + 4j + lane / 16) and publishes them itself
            const int row = Q3T_CP_WPUB ? 16 * (t >> 6) + 4 * j + (grp & 3) : 16 * j + grp;
            const uint16_t *r = W + (size_t)(64 * i + row) * H + l16 * 8;
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) wq[j][tt] = ld16(r + tt * 128);
        }
        nw = ldf4(S.layers[l].attn_norm + 4 * t);
    };
    auto issue_head = [&](int pass) {   // lm_head[pass - 1]: rows 32i + 16j + grp
        const uint16_t *W = S.heads[pass - 1];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint16_t *r = W + (size_t)(32 * i + 16 * j + grp) * H + l16 * 8;
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) wq[j][tt] = ld16(r + tt * 128);
        }
        nw = ldf4(p.out_norm + 4 * t);
    };
    issue_qkv(0);
    for (int pass = 0; pass < NPASS; ++pass) {
        for (int l = pass == 0 ? 0 : 1; l < NLC; ++l) {
            const int ph = ph_of(pass, l, 0);
            float4 x;
            if (l == 0) {
                x = ldf4(p.x_in + 4 * t);   // pass 0: the talker hidden state (written before the launch)
            } else {
                uint32_t u[4];
                PROF(ph, 0);
                if (Q3T_CP_GATE) g_gate(p.gx + 4 * t, X.tag(ph_of(pass, l - 1, 4)), X.c);
                Q3T_CP_WAIT<4>(p.gx + 4 * t, X.tag(ph_of(pass, l - 1, 4)), u, X.c);
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
            if constexpr (Q3T_CP_WPUB) {
                // each wave publishes its 16 rows as one whole line: lane L < 16 takes row 4j + g (j = L / 4, g = L % 4)
                // from lane 16 g of the group that reduced it (the l16 == 0 lane, as the LDS form), no barrier
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
                // one store instruction of wave 0 publishes the 64 rows (4 whole lines): single-lane stores from four
                // waves into shared lines make the next edge slower
                if (t < 64) g_put(p.gqkv + 64 * i + t, __float_as_uint(S.outv[t]), X.tag(ph));
            }
            PROF(ph, 2);
            if (Q3T_CP_PUT_FIRST) __syncthreads();   // the publish store enters the CU's memory pipe before the prefetch
            if (l + 1 < NLC) issue_qkv(l + 1);
            else if (pass >= 1) issue_head(pass);
            else issue_qkv(1);   // pass 0 has no head; layer 0 of the next passes comes from the table
        }
        if (pass == 0) continue;
        // ---- head: RMSNorm(output_norm) -> lm_head[pass - 1] logits (granules for the selecting workgroups)
        const int hph = ph_of(pass, NLC, 0);
        uint32_t u[4];
        PROF(hph, 0);
        if (Q3T_CP_GATE) g_gate(p.gx + 4 * t, X.tag(ph_of(pass, NLC - 1, 4)), X.c);
        Q3T_CP_WAIT<4>(p.gx + 4 * t, X.tag(ph_of(pass, NLC - 1, 4)), u, X.c);
        PROF(hph, 1);
        rms_to_f16(f4_of(u), nw, p.eps, S.xs, S.dscr, nullptr);
        __syncthreads();
        float a0[2], a1[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            a0[j] = 0.0f;
            a1[j] = 0.0f;
#pragma unroll
            for (int tt = 0; tt < 4; ++tt) a0[j] = dot8(wq[j][tt], *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128), a0[j]);
#pragma unroll
            for (int tt = 4; tt < 8; ++tt) a1[j] = dot8(wq[j][tt], *reinterpret_cast<const uint4 *>(S.xs + l16 * 8 + tt * 128), a1[j]);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float lg = group_sum<16>(a0[j]) + group_sum<16>(a1[j]);
            if (l16 == 0) S.outv[16 * j + grp] = lg;
        }
        __syncthreads();
        PROF(hph, 3);   // (development timeline: head rows reduced)
        if (t < 64) {   // wave 0, ONE store instruction: lanes 0..31 publish the rows, lanes 32 / 33 (sampling) their max
                        // and finite min
            // sampling: the rows divided by T (the selection's first step, the same IEEE division) and the 32 rows'
            // max / finite min, so the selecting workgroups skip that step and its block reduction
            const float lg = S.outv[t & 31];   // lanes 32..63 hold the same rows
            const float sv = samp && Q3T_CP_PREDIV ? lg / temp : lg;
            const float mx = group_max<32>(sv), mn = -group_max<32>(sv > -INFINITY ? -sv : -INFINITY);
            if (t < 32 || (samp && t < 34))
                g_put(t < 32 ? p.glog + 32 * i + t : p.glog + CPV + MMS * i + (t - 32),
                      __float_as_uint(t < 32 ? sv : t == 32 ? mx : mn), X.tag(hph));
            if (t < 32) p.logits[32 * i + t] = lg;   // read after the launch only (host, tests)
        }
        PROF(hph, 2);
        if (Q3T_CP_PUT_FIRST) __syncthreads();
        if (pass + 1 < NPASS) issue_qkv(1);
    }
}

// ------------------------------------------------------------------ attention of one kv group + token selection
__device__ __forceinline__ void role_att(Ctx &X) {
    const PersistParams &p = X.p;
    CLds &S = X.S;
    const int g = blockIdx.x - AW, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int pg = t >> 4, li = t & 15;   // attention: position, 8-dim chunk
    // wave v takes elements lane and lane + 64 of its head (q head 2g, q head 2g+1, k, v of group g): the pair its head
    // norm and NEOX RoPE work on, polled straight from the granules (no LDS staging or barrier before the norm)
    const int hb = wave == 0 ? g * 256 : wave == 1 ? g * 256 + D : wave == 2 ? NH * D + g * D : (NH + NKV) * D + g * D;
    const int gi = hb + lane;
    for (int e = t; e < NLC * D; e += 256) {
        S.qn[e / D][e % D] = S.layers[e / D].qn[e % D];
        S.kn[e / D][e % D] = S.layers[e / D].kn[e % D];
    }
    for (int e = t; e < 16 * D; e += 256) S.rope[e / D][e % D] = p.rope[e];
    S.sel.hist[t] = 0u;   // sel_sample_range's precondition (zeroed again after every selection)
    SelPre spre;
    sel_prefetch<SEL_CP>(p.sel, 0, spre);
    int tok = p.gs.tok[0];   // CB0: the input of pass 1
    float traw[2] = {ldgv<float>(p.qkvtab + (size_t)tok * QKVN + gi), ldgv<float>(p.qkvtab + (size_t)tok * QKVN + gi + 64)};
    const float kq_scale = 1.0f / sqrtf((float)D);
    __syncthreads();
    for (int pass = 0; pass < NPASS; ++pass) {
        const int pos = pass;
        for (int l = 0; l < NLC; ++l) {
            const int ph = ph_of(pass, l, 1);
            float xr[2];
            if (pass >= 1 && l == 0) {
                xr[0] = traw[0];
                xr[1] = traw[1];
            } else {
                uint32_t u[2];
                PROF(ph, 0);
                g_wait<2, 64>(p.gqkv + gi, X.tag(ph_of(pass, l, 0)), u, X.c);
                PROF(ph, 1);
                xr[0] = __uint_as_float(u[0]);
                xr[1] = __uint_as_float(u[1]);
            }
            {   // wave v: q head 0 / q head 1 / k (head norm + RoPE, K append) / v (f16 rounding, V append)
                const int v = wave;
                if (v == 3) {
#pragma unroll
                    for (int e = 0; e < 2; ++e) S.vc[l][pos][lane + 64 * e] = f2h(xr[e]);
                } else {
                    const float *hn = v == 2 ? S.kn[l] : S.qn[l];
                    float xx[2];
                    double ss = 0.0;
#pragma unroll
                    for (int e = 0; e < 2; ++e) { xx[e] = xr[e]; ss += (double)__fmul_rn(xx[e], xx[e]); }
                    ss = wave_sum_d(ss);
                    const float scale = 1.0f / sqrtf((float)(ss / D) + p.eps);
#pragma unroll
                    for (int e = 0; e < 2; ++e) xx[e] = (xx[e] * scale) * hn[lane + 64 * e];
                    const float cs = S.rope[pos][2 * lane], sn = S.rope[pos][2 * lane + 1];
                    const float y0 = opaque(opaque(xx[0] * cs) - opaque(xx[1] * sn));   // as k_attn: three roundings
                    const float y1 = opaque(opaque(xx[0] * sn) + opaque(xx[1] * cs));
                    if (v == 2) {
                        S.kc[l][pos][lane] = f2h(y0);
                        S.kc[l][pos][lane + 64] = f2h(y1);
                    } else {
                        S.q_s[v][lane] = f16r(y0);
                        S.q_s[v][lane + 64] = f16r(y1);
                    }
                }
            }
            __syncthreads();
            if (pass == 0 && l == NLC - 1) continue;   // pass 0's last layer: only its K/V rows are ever read
            // scores of position pg (16 lanes x 8 dims), softmax over positions 0..pos, P.V (k_attn arithmetic)
            const bool ok = pg <= pos;
            float q8[2][8], k8[8], v8[8];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int e = 0; e < 8; ++e) q8[h][e] = S.q_s[h][li * 8 + e];
            const uint4 kk = *reinterpret_cast<const uint4 *>(&S.kc[l][pg][li * 8]);
            {
                const uint4 vv = *reinterpret_cast<const uint4 *>(&S.vc[l][pg][li * 8]);
                const uint32_t kw[4] = {kk.x, kk.y, kk.z, kk.w}, vw[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if constexpr (!Q3T_ATTN_DOT2) { k8[2 * e] = h2f(kw[e] & 0xffff); k8[2 * e + 1] = h2f(kw[e] >> 16); }
                    v8[2 * e] = h2f(vw[e] & 0xffff); v8[2 * e + 1] = h2f(vw[e] >> 16);
                }
            }
            float sc[2], M[2], pr[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float s = 0.0f;
                if constexpr (Q3T_ATTN_DOT2) {   // score8 (q3t_common.h), as k_attn
                    uint32_t qp[4];
                    pack_q8(q8[h], qp);
                    s = score8(kk, qp);
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) s = __fmaf_rn(k8[e], q8[h][e], s);
                }
                s = group_sum<16>(s);
                sc[h] = ok ? __fmul_rn(s, kq_scale) : -INFINITY;
                const float m = rows_max(sc[h]);
                if (lane == 0) S.wred[wave][h] = m;
            }
            __syncthreads();
#pragma unroll
            for (int h = 0; h < 2; ++h) M[h] = fmaxf(fmaxf(S.wred[0][h], S.wred[1][h]), fmaxf(S.wred[2][h], S.wred[3][h]));
#pragma unroll
            for (int h = 0; h < 2; ++h) pr[h] = ok ? exp_sm(__fsub_rn(sc[h], M[h])) : 0.0f;
            {   // rows_sum of both heads at once: row 0 ends with head 0's (r0 + r1) + (r2 + r3), row 1 with head 1's
                const float lsum = rows_sum_pair(pr[0], pr[1]);
                if ((lane & 47) == 0) S.wsum[wave][lane >> 4] = lsum;   // lanes 0, 16
            }
            {   // rows_sum of the 16 products as a reduce-scatter (persist_tk.hip): row k ends with values k, 4 + k,
                // 8 + k, 12 + k (value n = 8 h + e), each (r0 + r1) + (r2 + r3) as rows_sum
                float v16[16], c8[8];
#pragma unroll
                for (int n = 0; n < 16; n += 2) {   // packed fmas onto 0 (v_pk_fma_f32), the same roundings
                    v16[n] = v16[n + 1] = 0.0f;
                    fma2(pr[n >> 3], ok ? v8[n & 7] : 0.0f, ok ? v8[(n + 1) & 7] : 0.0f, v16[n], v16[n + 1]);
                }
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
                    S.ared[wave][n >> 3][li * 8 + (n & 7)] = av;
                }
            }
            __syncthreads();
            if (t < 128) {
                const int h = t / (D / 2), d = 2 * (t % (D / 2));
                const float lsum = (S.wsum[0][h] + S.wsum[1][h]) + (S.wsum[2][h] + S.wsum[3][h]);
                const float a0 = (S.ared[0][h][d] + S.ared[1][h][d]) + (S.ared[2][h][d] + S.ared[3][h][d]);
                const float a1 = (S.ared[0][h][d + 1] + S.ared[1][h][d + 1]) + (S.ared[2][h][d + 1] + S.ared[3][h][d + 1]);
                g_put(p.gattn + g * 128 + t, (uint32_t)f2h(a0 / lsum) | ((uint32_t)f2h(a1 / lsum) << 16), X.tag(ph));
            }
            PROF(ph, 2);
        }
        if (pass == 0) continue;
        // ---- selection of code `pass` (lm_head[pass - 1]): every ATT workgroup gathers the logits and selects (the
        // same token in all 8), so the next pass's attention starts without a token hand-off; workgroup AW commits it
        // and hands it to the O workgroups (the residual row of layer 0)
        const int hph = ph_of(pass, NLC, 0);
        const bool samp = p.sel.temperature > 0.0f;
        constexpr bool RNG = Q3T_CP_RANGE;
        const float u = uniform24(spre.seed, spre.utt, (uint64_t)spre.frame, (uint64_t)pass);   // select_token_pre's u
        uint32_t u8[8], mm[2];
        PROF(hph, 0);
        if (Q3T_CP_SGATE) g_gate(p.glog + 8 * t, X.tag(hph), X.c);
        if constexpr (Q3T_POLL16) {
            if (samp && RNG) g_wait16_pair<8, 2>(p.glog + 8 * t, p.glog + CPV + MMS * lane, X.tag(hph), u8, mm, X.c);
            else g_waitc<8>(p.glog + 8 * t, X.tag(hph), u8, X.c);
        } else {
            if (samp && RNG) g_wait_pair<8, 2>(p.glog + 8 * t, p.glog + CPV + MMS * lane, X.tag(hph), u8, mm, X.c);
            else g_wait<8>(p.glog + 8 * t, X.tag(hph), u8, X.c);
        }
        PROF(hph, 1);
        float v[SEL_VPT_MAX];
#pragma unroll
        for (int e = 0; e < SEL_VPT_MAX; ++e) v[e] = e < 8 ? __uint_as_float(u8[e]) : -INFINITY;
        SelectSpec sp = p.sel;
        sp.step = pass - 1;
        int sel;
        if (spre.done >= 0) {
            sel = -1;
        } else if (!samp) {
            sel = sel_argmax(v, CPV, 8, S.sel);
        } else if (!RNG) {
            sel = select_token_pre<SEL_CP>(sp, spre, v, S.sel);
        } else {   // the row arrives divided by T with the 64 producers' max / min (lane l: producer l)
            float mx = wave_max(__uint_as_float(mm[0])), mn = -wave_max(-__uint_as_float(mm[1]));
            if constexpr (!Q3T_CP_PREDIV) {   // the raw row: divide here (x -> x / T is monotonic, so the max / min of
                                              // the quotients are the quotients of the max / min)
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = v[e] / p.sel.temperature;
                mx = mx / p.sel.temperature;
                mn = mn / p.sel.temperature;
            }
            sel = sel_sample_range(v, CPV, 8, p.sel.top_k, u, mx, mn, S.sel);
        }
        S.sel.hist[t] = 0u;   // the next selection's range histogram (this one's bins were read before its last barrier)
        PROF(hph, 3);   // (development timeline: token selected)
        if (g == 0 && t == 0) {
            if (pass + 1 < NPASS) g_put(p.gtok + pass, (uint32_t)max(sel, 0), X.tag(hph));
            if (sel >= 0) select_commit(sp, 0, sel);
            if (pass + 1 == NPASS) __hip_atomic_store(p.seq, X.seq + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        PROF(hph, 2);
        tok = max(sel, 0);
        if (pass + 1 < NPASS) {
            const float *row = p.qkvtab + ((size_t)(VOC + (pass - 1) * CPV) + tok) * QKVN + gi;
            traw[0] = ldgv<float>(row);
            traw[1] = ldgv<float>(row + 64);
        }
    }
}

// ------------------------------------------------------------------ O-projection + residual (32 rows)
__device__ __forceinline__ void role_o(Ctx &X) {
    const PersistParams &p = X.p;
    CLds &S = X.S;
    const int i = blockIdx.x - OW, t = threadIdx.x, lane = t & 63, wave = t >> 6, l16 = t & 15, grp4 = lane >> 4;
    uint4 wo[8][4];
    auto issue = [&](int l) {   // row 32i + 4j + grp4, K slice = wave (k_gemv<1,1,4,PRO_F16,4>)
        const uint16_t *W = S.layers[l].o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint16_t *r = W + (size_t)(32 * i + 4 * j + grp4) * (NH * D) + wave * 512 + l16 * 8;
#pragma unroll
            for (int tt = 0; tt < 4; ++tt) wo[j][tt] = ld16(r + tt * 128);
        }
    };
    issue(0);
    int it = 0;   // phase executions: the parity of S.red
    for (int pass = 0; pass < NPASS; ++pass) {
        for (int l = 0; l < NLC; ++l) {
            if (pass == 0 && l == NLC - 1) continue;
            const int par = it++ & 1;
            const int ph = ph_of(pass, l, 2);
            if (t < 32) {   // the residual rows x_l[32i + t]
                const int row = 32 * i + t;
                float xr;
                if (l == 0 && pass == 0) {
                    xr = p.x_in[row];
                } else if (l == 0) {   // the table row of the previous pass's token (pass 1: CB0)
                    int tok = p.gs.tok[0];
                    if (pass >= 2) {
                        uint32_t u1[1];
                        g_wait<1>(p.gtok + pass - 1, X.tag(ph_of(pass - 1, NLC, 0)), u1, X.c);
                        tok = min((int)u1[0], p.sel.V - 1);   // an aborted wait returns a stale payload: keep it in the table
                    }
                    // 1.7B: the projected f32 row (xtab, the QKV table's row order) instead of the f16 table row
                    xr = p.xtab ? p.xtab[((size_t)(pass == 1 ? 0 : VOC + (pass - 2) * CPV) + tok) * H + row]
                                : h2f(S.tabs[pass - 1][(size_t)tok * H + row]);
                } else {
                    uint32_t u1[1];
                    g_wait<1>(p.gx + row, X.tag(ph_of(pass, l - 1, 4)), u1, X.c);
                    xr = __uint_as_float(u1[0]);
                }
                S.xr[t] = xr;
            }
            uint32_t u[4];
            PROF(ph, 0);
            if (Q3T_CP_GATE) g_gate(p.gattn + 4 * t, X.tag(ph_of(pass, l, 1)), X.c);
            Q3T_CP_WAIT<4>(p.gattn + 4 * t, X.tag(ph_of(pass, l, 1)), u, X.c);
            PROF(ph, 1);
            *reinterpret_cast<uint4 *>(S.xs + 8 * t) = make_uint4(u[0], u[1], u[2], u[3]);
            wave_lds_sync();   // wave w polled exactly the K slice [512 w, 512 w + 512) it multiplies
            float acc[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                acc[j] = 0.0f;
#pragma unroll
                for (int tt = 0; tt < 4; ++tt)
                    acc[j] = dot8(wo[j][tt], *reinterpret_cast<const uint4 *>(S.xs + wave * 512 + l16 * 8 + tt * 128), acc[j]);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                acc[j] = group_sum<16>(acc[j]);
                if (l16 == 0) S.red[par][wave][4 * j + grp4] = acc[j];
            }
            __syncthreads();
            if (t < 32) {
                const float (&rd)[4][32] = S.red[par];
                const float s = rd[0][t] + rd[1][t] + rd[2][t] + rd[3][t];
                g_put(p.gx2 + 32 * i + t, __float_as_uint(S.xr[t] + s), X.tag(ph));
            }
            PROF(ph, 2);
            if (Q3T_CP_PUT_FIRST) __syncthreads();
            const int nl = (l + 1 < NLC && !(pass == 0 && l + 1 == NLC - 1)) ? l + 1 : 0;
            if (!(pass + 1 == NPASS && l + 1 == NLC)) issue(nl);
        }
    }
}

// ------------------------------------------------------------------ RMSNorm(ffn_norm) + gate/up + SwiGLU (32 units)
__device__ __forceinline__ void role_gu(Ctx &X) {
    const PersistParams &p = X.p;
    CLds &S = X.S;
    const int i = blockIdx.x - UW, t = threadIdx.x, l16 = t & 15, grp = t >> 4;
    uint4 wg[2][8], wu[2][8];
    float4 nw;
    auto issue = [&](int l) {   // unit 32i + 16j + grp: gate row, up row 16 below (16-row interleaved blocks)
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
    for (int pass = 0; pass < NPASS; ++pass) {
        for (int l = 0; l < NLC; ++l) {
            if (pass == 0 && l == NLC - 1) continue;
            const int ph = ph_of(pass, l, 3);
            uint32_t u[4];
            PROF(ph, 0);
            if (Q3T_CP_GATE) g_gate(p.gx2 + 4 * t, X.tag(ph_of(pass, l, 2)), X.c);
            Q3T_CP_WAIT<4>(p.gx2 + 4 * t, X.tag(ph_of(pass, l, 2)), u, X.c);
            PROF(ph, 1);
            rms_to_f16(f4_of(u), nw, p.eps, S.xs, S.dscr, nullptr);
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
            if (Q3T_CP_PUT_FIRST) __syncthreads();
            const int nl = (l + 1 < NLC && !(pass == 0 && l + 1 == NLC - 1)) ? l + 1 : 0;
            if (!(pass + 1 == NPASS && l + 1 == NLC)) issue(nl);
        }
    }
}

// ------------------------------------------------------------------ down + residual (18-19 rows)
__device__ __forceinline__ void role_dn(Ctx &X) {
    const PersistParams &p = X.p;
    CLds &S = X.S;
    const int i = blockIdx.x - DW, t = threadIdx.x, lane = t & 63, wave = t >> 6, l16 = t & 15, grp4 = lane >> 4;
    const int lo = i * H / ND, n = (i + 1) * H / ND - lo;
    uint4 wd[5][6];
    auto issue = [&](int l) {   // row lo + 4j + grp4 (clamped: rows past n re-read row lo + n - 1), K slice = wave
        const uint16_t *W = S.layers[l].down;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const uint16_t *r = W + (size_t)(lo + min(4 * j + grp4, n - 1)) * INTER + wave * 768 + l16 * 8;
#pragma unroll
            for (int tt = 0; tt < 6; ++tt) wd[j][tt] = ld16(r + tt * 128);
        }
    };
    issue(0);
    int it = 0;   // phase executions: the parity of S.red
    for (int pass = 0; pass < NPASS; ++pass) {
        for (int l = 0; l < NLC; ++l) {
            if (pass == 0 && l == NLC - 1) continue;
            const int par = it++ & 1;
            const int ph = ph_of(pass, l, 4);
            if (t < n) {   // the residual rows x'_l (published a phase earlier)
                uint32_t u1[1];
                g_wait<1>(p.gx2 + lo + t, X.tag(ph_of(pass, l, 2)), u1, X.c);
                S.xr[t] = __uint_as_float(u1[0]);
            }
            uint32_t u[6];
            PROF(ph, 0);
            if (Q3T_CP_GATE) g_gate(p.gh + 6 * t, X.tag(ph_of(pass, l, 3)), X.c);
            Q3T_CP_WAIT<6>(p.gh + 6 * t, X.tag(ph_of(pass, l, 3)), u, X.c);
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
                if (l16 == 0) S.red[par][wave][4 * j + grp4] = acc[j];
            }
            __syncthreads();
            if (t < n) {
                const float (&rd)[4][32] = S.red[par];
                const float s = rd[0][t] + rd[1][t] + rd[2][t] + rd[3][t];
                g_put(p.gx + lo + t, __float_as_uint(S.xr[t] + s), X.tag(ph));
            }
            PROF(ph, 2);
            if (Q3T_CP_PUT_FIRST) __syncthreads();
            const int nl = (l + 1 < NLC && !(pass == 0 && l + 1 == NLC - 1)) ? l + 1 : 0;
            if (!(pass + 1 == NPASS && l + 1 == NLC)) issue(nl);
        }
    }
}

__global__ void __launch_bounds__(256) k_cp_roles(const PersistParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    CLds &S = *reinterpret_cast<CLds *>(smem);
    const int t = threadIdx.x, w = blockIdx.x;
    Ctx X{p, S, Ctl{p.err, false}, __hip_atomic_load(p.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
#ifdef Q3T_DEV
    if (w == 0 && t == 0) g_selprof = p.prof;
#endif
    // pointer tables in LDS: a pointer fetched from global memory inside the chain would make the next wait cover every
    // weight stream in flight (vmcnt order)
    if (t < NLC) S.layers[t] = p.L[t];
    if (t < 15) S.heads[t] = p.heads[t];
    if (t < 16) S.tabs[t] = p.gs.tabs[t];
    __syncthreads();
    if (w < AW) role_qkv(X);
    else if (w < OW) role_att(X);
    else if (w < UW) role_o(X);
    else if (w < DW) role_gu(X);
    else role_dn(X);
}

size_t cp_roles_lds() { return std::max(sizeof(CLds), (size_t)96 * 1024); }   // > 80 KB: one workgroup per CU

}  // namespace

bool persist_cp_roles_resident(int device) {
    int n_cu = 0, blocks = 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cu < G) return false;
    const void *k = reinterpret_cast<const void *>(&k_cp_roles);
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)cp_roles_lds()) != hipSuccess) return false;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k, 256, cp_roles_lds()) == hipSuccess && blocks >= 1;
}

bool persist_cp_roles(const PersistParams &p, hipStream_t s) {
    if (!p.L || p.n_layers != NLC || !p.heads || !p.logits || !p.rope || !p.x_in || !p.gs.tok || !p.gs.tabs || !p.qkvtab ||
        !p.gx || p.sel.mode != SEL_CP || p.sel.V != CPV) {
        set_error("persist_cp_roles: bad parameters");
        return false;
    }
    static bool attr = false;
    if (!attr) {
        Q3T_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_cp_roles), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)cp_roles_lds()));
        attr = true;
    }
    hipLaunchKernelGGL(k_cp_roles, dim3(G), dim3(256), cp_roles_lds(), s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}

}  // namespace q3t
