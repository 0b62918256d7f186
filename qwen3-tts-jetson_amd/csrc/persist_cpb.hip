// persist_cpb.hip — the BATCHED code-predictor frame (4..64 slots, BASELINE configs[2]) as ONE persistent launch:
// 16 passes of the 5-layer stack, lm_head[p-1] + token selection after pass p >= 1, and the next talker step's
// embedding (src/tts_transformer.cpp:2153-2340, src/trt_code_predictor.cpp:484-600,
// scripts/export_code_predictor.py:132-231).  It replaces the ~570-launch graph of decoder_stack_mm (engine.cpp) for one
// frame, and computes the same bits: every projection is that graph's MFMA tile with the same K quarters, the same
// split-K slices and the same LDS sum order (gemm_mfma.hip), every residual + RMSNorm is k_resid_norm's arithmetic, the
// attention is k_attn_small's source (attn_small.h) and the selection is k_select_embed_norm's (select.h).
//
// Work per layer for S slots in NT token tiles of 32 (NT = 1: S <= 32, NT = 2: S <= 64), one 256-thread workgroup per CU:
//
//   job              count            workgroups        tile / input (per job)                    output
//   RN_A / RN_F      1 per slot       128 + 2b          x[b] += 4 slabs; RMSNorm -> f16 row        xnA / xnF [b]
//   QKV              128 x NT         [0, 128 NT)       32 rows x 32 tokens, K 1024 (xnA 64 KB)    qkv f32
//   ATT              1 per slot       192 + b           8 kv groups (2 per wave), <= 16 positions  attn f16 [b]
//   O                32 x 4 x NT      [0, 128 NT)       32 rows x 32 tokens x K slice 512          slabO f32 [z]
//   GU               96 x NT          gj: [0, 128), odd slot wgs  64 rows (32 SwiGLU units) x 32 tokens  h f16
//   DN               32 x 4 x NT      [0, 128 NT)       32 rows x 32 tokens x K slice 768          slabD f32 [z]
//   HEAD (p >= 1)    64 x NT          [0, 64 NT)        32 rows x 32 tokens, K 1024 (final xnA)    logits f32
//   SEL  (p >= 1)    1 per slot       192 + b           top-k / argmax of the slot's row, commit; next pass's x[b]
//
// The residual stream of slot b never leaves its RN workgroup: x[b] lives in registers (4 values per thread) for the
// whole frame.  Hand-offs are MI355X_MICROARCH.md's flag form for bandwidth (hand-off table, row 1): every payload byte
// is stored with an agent-scope (sc1) store, each storing wave waits vmcnt(0), a workgroup barrier, then ONE lane
// stores the job's flag (sc1); a consumer wave polls the flags of exactly the producers whose bytes it reads (sc1
// loads) and then loads the payload with sc1 loads.  A flag carries ((seq << 10) + phase + 1): seq is bumped once per
// launch, so a flag of an earlier phase or launch never matches.  Payload buffers are single-buffered: every producer
// reaches its next write of a buffer only through a chain of jobs that needs every reader of the previous contents to
// have finished.  Every wait is bounded (persist_dev.h SPIN_LIMIT): a protocol fault ends the launch with *err set and
// the engine falls back to the launch-per-op graph, which is bit-identical.
#include "persist.h"
#include "persist_mm.h"
#include "attn_small.h"
#include "select.h"

#pragma clang fp contract(off)   // every rounding as written: bit-identical to k_gemm_mfma / k_resid_norm / k_attn_small

namespace q3t {

namespace {
using namespace pmm;

constexpr int NLC = 5, NPASS = 16, SW0 = 128;

enum Kind { K_RNA = 0, K_QKV = 1, K_ATT = 2, K_O = 3, K_RNF = 4, K_GU = 5, K_DN = 6, K_HEAD = 7 };
__device__ __forceinline__ int ph_of(int pass, int l, int k) { return pass * 48 + l * 8 + k; }

// ---------------------------------------------------------------- state block (cpb_state_bytes, zeroed once)
// xna / xnf / attn / h: f16 payloads behind flags; qkv, slo, sld, logits: {f32, tag} granules (8 B each, no flag)
struct StateLayout {
    size_t xna = 0;
    size_t xnf = xna + (size_t)SMAX * H * 2;
    size_t qkv = xnf + (size_t)SMAX * H * 2;
    size_t attn = qkv + (size_t)SMAX * QKVN * 8;
    size_t slo = attn + (size_t)SMAX * NH * D * 2;
    size_t sld = slo + (size_t)4 * SMAX * H * 8;
    size_t h = sld + (size_t)4 * SMAX * H * 8;
    size_t lg = h + (size_t)SMAX * INTER * 2;
    size_t flags = lg + (size_t)SMAX * CPV * 8;     // 8 kinds x FLAGS_PER_KIND u32
    size_t ctr = flags + 8 * FLAGS_PER_KIND * 4;    // seq, err (own lines)
    size_t total = ctr + 256;
};

struct BLds {
    // the next job's A fragments [wave][16 rt + 4c + j][lane] (LDS-DMA, issued one job ahead); once a job's MFMAs are
    // done, wave w's region holds its K-quarter partial tiles [rt][reg][lane] (f32)
    uint4 wl[4][32][64];
    SelLds sel;
    AttnSmallLds att[4];
    double dscr[4];
    int toks[16];
    PLayerW layers[NLC];
    const uint16_t *heads[16];
    const uint16_t *tabs[16];
};

// ---------------------------------------------------------------- the kernel
template <int NT>
__global__ void __launch_bounds__(256, 1) k_cpb(const CpbParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    BLds &S = *reinterpret_cast<BLds *>(smem);
    const StateLayout SL;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, w = blockIdx.x;
    Ctx X{S.wl, p.prof, Ctl{reinterpret_cast<unsigned *>(p.state + SL.ctr) + 32, false},
          __hip_atomic_load(reinterpret_cast<unsigned *>(p.state + SL.ctr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
          reinterpret_cast<unsigned *>(p.state + SL.flags),
          __builtin_amdgcn_make_buffer_rsrc(p.state, 0, (int)SL.total, BUF_RSRC), p.S};
    // GEMM jobs: 64 rows x one token tile; QKV / O / DN on [0, 64 NT), gate/up on [0, 96 NT), lm_head on [0, 32 NT)
    const int NQJ = 64 * NT, NGJ = 96 * NT, NHJ = 32 * NT;
    // slot workgroups: SW0 + 2b + hf for slot b, half hf (kv groups 4 hf .. 4 hf + 3); the even one (rn) also keeps the
    // slot's residual row, runs its norms and commits its selections
    const int sw = w - SW0;
    const bool slot = sw >= 0 && sw < 2 * p.S;
    const int b = sw >> 1, hf = sw & 1;
    const bool rn = slot && hf == 0;
    // gate/up job gj: workgroups [0, 128), then the odd slot workgroups 129, 131, ...: the residual rows' workgroups
    // (even) run the norm right before gate/up, so a gate/up job there started ~2 us after the others
    const int gj = w < SW0 ? w : (w & 1) ? SW0 + (w - SW0 - 1) / 2 : -1;
    const bool hq = w < NQJ, hg = gj >= 0 && gj < NGJ, hh = w < NHJ;
    if (t < NLC) S.layers[t] = p.L[t];
    if (t < 15) S.heads[t] = p.heads[t];
    if (t < 16) S.tabs[t] = p.tabs[t];
    if (slot && t < 16) S.toks[t] = p.sel.tokens[b * 16 + t];
    __syncthreads();

    // ---- the GEMM job sequence of this workgroup, weights issued one job ahead
    int cp = 0, cl = 0, ck = K_QKV;   // slot of the job whose weights S.wl holds (cp = NPASS: none)
    auto has = [&](int k) { return k == K_GU ? hg : k == K_HEAD ? hh : hq; };
    auto advance = [&]() {
        if (ck == K_QKV) {
            if (cp == 0 && cl == NLC - 1) { cp = 1; cl = 0; ck = K_O; }
            else ck = K_O;
        } else if (ck == K_O) ck = K_GU;
        else if (ck == K_GU) ck = K_DN;
        else if (ck == K_DN) {
            if (cl + 1 < NLC) { ++cl; ck = K_QKV; }
            else { cl = NLC; ck = K_HEAD; }
        } else { ++cp; cl = 0; ck = K_O; }
    };
    auto issue = [&]() {
        while (cp < NPASS && !has(ck)) advance();
        if (cp >= NPASS) return;
        const PLayerW &Lw = S.layers[cl < NLC ? cl : 0];
        switch (ck) {
            case K_QKV: load_w<4>(S.wl, Lw.qkv, H, 64 * (w % 64), 0); break;
            case K_O: load_w<2>(S.wl, Lw.o, NH * D, 64 * (w % 16), 512 * ((w / 16) % 4)); break;
            case K_GU: load_w<4>(S.wl, Lw.gu, H, 64 * (gj % 96), 0); break;
            case K_DN: load_w<3>(S.wl, Lw.down, INTER, 64 * (w % 16), 768 * ((w / 16) % 4)); break;
            default: load_w<4>(S.wl, S.heads[cp - 1], H, 64 * (w % 32), 0); break;
        }
    };
    auto next_job = [&]() { advance(); issue(); };
    // a slot workgroup issues the next job's weights after its next attention (the polls of the norm and attention steps
    // before it then do not queue behind 128 KB of weight DMA; O and the final norm follow with no slot work of this
    // workgroup), at the latest when that job starts
    bool pending = false;
    auto after_job = [&]() { if (slot) pending = true; else next_job(); };
    auto after_rn = [&]() { if (pending) { next_job(); pending = false; } };
    issue();

    // ---- the RN workgroups' residual row (thread t: elements 4t .. 4t+3)
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    // RMSNorm of x -> f16 row of slot b in the hand-off buffer `xo`, flag (kind, b)
    auto norm_pub = [&](const float *nw, size_t xo, int kind, uint32_t tg) {
        double ss = (double)(x.x * x.x) + (double)(x.y * x.y) + (double)(x.z * x.z) + (double)(x.w * x.w);
        ss = block_sum_d(ss, S.dscr);
        const float scale = 1.0f / sqrtf((float)(ss / H) + p.eps);
        const float4 wv = ldf4(nw + 4 * t);
        const float y0 = (x.x * scale) * wv.x, y1 = (x.y * scale) * wv.y, y2 = (x.z * scale) * wv.z, y3 = (x.w * scale) * wv.w;
        const u32x2_t hv = {(uint32_t)f2h(y0) | ((uint32_t)f2h(y1) << 16), (uint32_t)f2h(y2) | ((uint32_t)f2h(y3) << 16)};
        CPROF((int)((tg - 1u) & 1023u), 3);
        __builtin_amdgcn_raw_buffer_store_b64(hv, X.rs, (int)xo + fragoff(H / 8, b, 4 * t), 0, SC1);
        publish(X, kind, b, tg);
    };
    // x += the 4 split-K slabs of slot b (k_resid_norm<4> order): thread t polls the 16 granules of its 4 elements
    auto fold = [&](size_t slab, uint32_t tg) {
        const int ph_ = (int)((tg - 1u) & 1023u);
        (void)ph_;
        CPROF(ph_, 0);
        u32x4_t pz[8];
        poll_gran<8>(X, tg, pz, [&](u32x4_t (&r)[8]) {
#pragma unroll
            for (int z = 0; z < 4; ++z)
#pragma unroll
                for (int hh2 = 0; hh2 < 2; ++hh2)
                    r[2 * z + hh2] = __builtin_amdgcn_raw_buffer_load_b128(X.rs, (int)(slab + (((size_t)z * SMAX + b) * H + 4 * t + 2 * hh2) * 8), 0, SC1V);
        });
        CPROF(ph_, 1);
#pragma unroll
        for (int z = 0; z < 4; ++z)
            x = make_float4(x.x + __uint_as_float(pz[2 * z].x), x.y + __uint_as_float(pz[2 * z].z), x.z + __uint_as_float(pz[2 * z + 1].x),
                            x.w + __uint_as_float(pz[2 * z + 1].z));
    };

    for (int pass = 0; pass < NPASS; ++pass) {
        const int pos = slot ? p.pos[(size_t)pass * p.pos_ld + b] : 0;
        for (int l = 0; l < NLC; ++l) {
            const PLayerW &Lw = S.layers[l];
            if (pass == 0 || l >= 1) {
                // ---- RN_A: the layer's input row, normalised (pass 0 layer 0: the talker hidden state)
                if (rn) {
                    if (pass == 0 && l == 0) x = ldf4(p.x_in + (size_t)b * H + 4 * t);
                    else fold(SL.sld, X.tag(ph_of(pass, l - 1, K_DN)));
                    norm_pub(Lw.attn_norm, SL.xna, K_RNA, X.tag(ph_of(pass, l, K_RNA)));
                }
                // ---- QKV: rows 64 rp .. +63 of tile tt -> granules
                if (hq) {
                    after_rn();
                    const int rp = w % 64, tt = w / 64;
                    const int nv = min(32, p.S - 32 * tt);
                    wait_flags_wg(X, K_RNA, nv, [&](int i) { return 32 * tt + i; }, X.tag(ph_of(pass, l, K_RNA)));
                    mm_tile<4>(X, SL.xna, H / 8, 0, 32 * tt);
                    CPROF(ph_of(pass, l, K_QKV), 3);
                    epi_gran(X, SL.qkv, QKVN, 64 * rp, 32 * tt, X.tag(ph_of(pass, l, K_QKV)));
                    CPROF(ph_of(pass, l, K_QKV), 2);
                    after_job();
                }
            }
            // ---- ATT: kv group 4 hf + wave of slot b (one wave each); its cached K / V rows are loaded before the wait
            if (slot) {
                const bool tab = pass >= 1 && l == 0;
                const int g = 4 * hf + wave;
                const size_t hoff = (size_t)l * p.kv_layer + (((size_t)b * NKV + g) * 16) * D;
                AttnSmallKV kv;
                attn_small_load_kv<true>(pos, p.kc + hoff, p.vc + hoff, kv);
                AttnSmallAux aux;
                attn_small_load_aux(p.rope + (size_t)pos * D, Lw.qn, Lw.kn, aux);
                float xs[4][2];
                if (tab) {   // layer 0 of passes 1..15: the per-token table row of the previous pass's token
                    attn_small_load_qkv<false>(p.qkvtab + ((size_t)(pass == 1 ? 0 : VOC + (pass - 2) * CPV) + S.toks[pass - 1]) * QKVN,
                                               g, NH, NKV, xs);
                } else {     // the QKV jobs' granules of slot b
                    const uint32_t tg = X.tag(ph_of(pass, l, K_QKV));
                    CPROF(ph_of(pass, l, K_QKV), 0);
                    u32x4_t gq[4];   // {v, e = 0} / {v, e = 1} of q0, q1, k, v (x, y: e 0; z, w: e 1)
                    poll_gran<4>(X, tg, gq, [&](u32x4_t (&r)[4]) {
#pragma unroll
                        for (int v = 0; v < 4; ++v) {
                            const size_t o = SL.qkv + ((size_t)b * QKVN + attn_small_src(g, v, NH, NKV) + lane) * 8;
                            const u32x2_t a = __builtin_amdgcn_raw_buffer_load_b64(X.rs, (int)o, 0, SC1V);
                            const u32x2_t c = __builtin_amdgcn_raw_buffer_load_b64(X.rs, (int)(o + 64 * 8), 0, SC1V);
                            r[v] = u32x4_t{a.x, a.y, c.x, c.y};
                        }
                    });
                    CPROF(ph_of(pass, l, K_QKV), 1);
#pragma unroll
                    for (int v = 0; v < 4; ++v) { xs[v][0] = __uint_as_float(gq[v].x); xs[v][1] = __uint_as_float(gq[v].z); }
                }
                uint16_t *const ab = reinterpret_cast<uint16_t *>(p.state + SL.attn);
                attn_small_compute<true>(kv, xs, aux, g, pos, p.eps, p.kc + hoff, p.vc + hoff,
                                         [&](int e) { return ab + fragoff(NH * D / 8, b, e) / 2; }, S.att[wave]
#ifdef CPB_ATT_STAMPS   // development: stamps inside the attention, phases (pass, 5, 1 + l), column k
                                         , [&](int k) { CPROF(pass * 48 + 41 + l, k); }
#endif
                );
                CPROF(ph_of(pass, l, K_ATT), 3);
                if (!(pass == 0 && l == NLC - 1)) publish(X, K_ATT, sw, X.tag(ph_of(pass, l, K_ATT)));
                else __syncthreads();
                after_rn();
            }
            if (pass == 0 && l == NLC - 1) continue;   // pass 0's last layer: only its K/V rows are ever read
            // ---- O: split-K slab z of rows 64 rp .. +63, tile tt
            if (hq) {
                after_rn();
                const int rp = w % 16, z = (w / 16) % 4, tt = w / 64;
                const int nv = min(32, p.S - 32 * tt);
                // wave w multiplies heads 4 z + w: kv group (4 z + w) / 2, published by the slots' half (4 z + w) / 8
                // (wave 0 polls both halves' flags of the slice: 4 z + w for w < 4 spans one half)
                wait_flags_wg(X, K_ATT, nv, [&](int i) { return 2 * (32 * tt + i) + ((4 * z) >> 3); }, X.tag(ph_of(pass, l, K_ATT)));
                mm_tile<2>(X, SL.attn, NH * D / 8, 512 * z, 32 * tt);
                CPROF(ph_of(pass, l, K_O), 3);
                epi_gran(X, SL.slo + (size_t)z * SMAX * H * 8, H, 64 * rp, 32 * tt, X.tag(ph_of(pass, l, K_O)));
                CPROF(ph_of(pass, l, K_O), 2);
                after_job();
            }
            // ---- RN_F
            if (rn) {
                fold(SL.slo, X.tag(ph_of(pass, l, K_O)));
                norm_pub(Lw.ffn_norm, SL.xnf, K_RNF, X.tag(ph_of(pass, l, K_RNF)));
            }
            // ---- GU: 32 SwiGLU units (rows 64 rp .. +63, gate/up interleaved in 16-row blocks), tile tt
            if (hg) {
                after_rn();
                const int rp = gj % 96, tt = gj / 96;
                const int nv = min(32, p.S - 32 * tt);
                wait_flags_wg(X, K_RNF, nv, [&](int i) { return 32 * tt + i; }, X.tag(ph_of(pass, l, K_RNF)));
                mm_tile<4>(X, SL.xnf, H / 8, 0, 32 * tt);
                CPROF(ph_of(pass, l, K_GU), 3);
                {   // k_gemm_mfma SWIGLU epilogue per row tile: wave = (rt, q)
                    const int rt = wave >> 1, q = wave & 1, r = lane & 31, h = lane >> 5;
                    const int tok = 32 * tt + r;
                    if (tok < p.S) {
                        const int unit = 32 * rp + 16 * rt + 8 * q + 4 * h;
                        float hv[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) hv[e] = silu_f(sum4(S.wl, rt, 4 * q + e, lane)) * sum4(S.wl, rt, 4 * (q + 2) + e, lane);
                        const u32x2_t o = {(uint32_t)f2h(hv[0]) | ((uint32_t)f2h(hv[1]) << 16),
                                           (uint32_t)f2h(hv[2]) | ((uint32_t)f2h(hv[3]) << 16)};
                        __builtin_amdgcn_raw_buffer_store_b64(o, X.rs, (int)SL.h + fragoff(INTER / 8, tok, unit), 0, SC1);
                    }
                }
                publish(X, K_GU, gj, X.tag(ph_of(pass, l, K_GU)));
                after_job();
            }
            // ---- DN: split-K slab z of rows 64 rp .. +63, tile tt; wave w reads units [768 z + 192 w, +192)
            if (hq) {
                after_rn();
                const int rp = w % 16, z = (w / 16) % 4, tt = w / 64;
                // each wave waits for the 6 gate/up jobs of its own K quarter only (units [768 z + 192 w, +192)): no barrier,
                // no wave held by another quarter's late producer
                wait_flags(X, K_GU, 6, [&](int i) { return 24 * z + 6 * wave + i + 96 * tt; }, X.tag(ph_of(pass, l, K_GU)));
                mm_tile<3>(X, SL.h, INTER / 8, 768 * z, 32 * tt);
                CPROF(ph_of(pass, l, K_DN), 3);
                epi_gran(X, SL.sld + (size_t)z * SMAX * H * 8, H, 64 * rp, 32 * tt, X.tag(ph_of(pass, l, K_DN)));
                CPROF(ph_of(pass, l, K_DN), 2);
                after_job();
            }
        }
        if (pass == 0) {   // pass 1's input: the codec_embd row of CB0 (k_gather_sum, one table)
            if (rn) {
                const uint2 u = *reinterpret_cast<const uint2 *>(S.tabs[0] + (size_t)S.toks[0] * H + 4 * t);
                x = make_float4(h2f(u.x & 0xffff), h2f(u.x >> 16), h2f(u.y & 0xffff), h2f(u.y >> 16));
            }
            continue;
        }
        // ---- final RMSNorm (output_norm) -> lm_head[pass - 1] -> selection of code `pass`
        if (rn) {
            fold(SL.sld, X.tag(ph_of(pass, NLC - 1, K_DN)));
            norm_pub(p.out_norm, SL.xna, K_RNA, X.tag(ph_of(pass, NLC, K_RNA)));
        }
        if (hh) {
            after_rn();
            const int rp = w % 32, tt = w / 32;
            const int nv = min(32, p.S - 32 * tt);
            wait_flags_wg(X, K_RNA, nv, [&](int i) { return 32 * tt + i; }, X.tag(ph_of(pass, NLC, K_RNA)));
            mm_tile<4>(X, SL.xna, H / 8, 0, 32 * tt);
            CPROF(ph_of(pass, NLC, K_HEAD), 3);
            epi_gran(X, SL.lg, CPV, 64 * rp, 32 * tt, X.tag(ph_of(pass, NLC, K_HEAD)));
            CPROF(ph_of(pass, NLC, K_HEAD), 2);
            after_job();
        }
        if (slot) {   // both halves select (the same token); the even one commits it
            const uint32_t tg = X.tag(ph_of(pass, NLC, K_HEAD));
            CPROF(ph_of(pass, NLC, K_HEAD), 0);
            SelectSpec sp = p.sel;
            sp.step = pass - 1;
            SelPre pre;   // the selection's per-slot inputs (done, frame, seed, utterance) before the poll, off the chain
            sel_prefetch<SEL_CP>(sp, b, pre);
            u32x4_t lr[4];   // thread t: logits 8t .. 8t+7 (select_token's exact-width ownership, V = 2048)
            poll_gran<4>(X, tg, lr, [&](u32x4_t (&r)[4]) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    r[k] = __builtin_amdgcn_raw_buffer_load_b128(X.rs, (int)(SL.lg + ((size_t)b * CPV + 8 * t + 2 * k) * 8), 0, SC1V);
            });
            CPROF(ph_of(pass, NLC, K_HEAD), 1);
            float v[SEL_VPT_MAX];
#pragma unroll
            for (int k = 0; k < 4; ++k) { v[2 * k] = __uint_as_float(lr[k].x); v[2 * k + 1] = __uint_as_float(lr[k].z); }
#pragma unroll
            for (int e = 8; e < SEL_VPT_MAX; ++e) v[e] = -INFINITY;
            const int tok = select_token_pre<SEL_CP>(sp, pre, v, S.sel);   // -1: slot done
            if (t == 0 && tok >= 0) {
                if (rn) select_commit(sp, b, tok);
                S.toks[pass] = tok;
            }
            __syncthreads();
            CPROF(ph_of(pass, NLC, K_HEAD), 3);
            if (!rn) {
            } else if (pass + 1 < NPASS) {   // the next pass's input: code_pred.codec_embd[pass - 1] row of this token
                const uint2 u = *reinterpret_cast<const uint2 *>(S.tabs[pass] + (size_t)S.toks[pass] * H + 4 * t);
                x = make_float4(h2f(u.x & 0xffff), h2f(u.x >> 16), h2f(u.y & 0xffff), h2f(u.y >> 16));
            } else {
                if (p.talker_next) {   // the next talker step's embedding + its layer-0 RMSNorm (k_select_embed_norm, nt 16)
                    float a[4];
                    {
                        const uint2 u = *reinterpret_cast<const uint2 *>(S.tabs[0] + (size_t)S.toks[0] * H + 4 * t);
                        a[0] = h2f(u.x & 0xffff); a[1] = h2f(u.x >> 16); a[2] = h2f(u.y & 0xffff); a[3] = h2f(u.y >> 16);
                    }
#pragma unroll
                    for (int j = 1; j < 16; ++j) {
                        const uint2 u = *reinterpret_cast<const uint2 *>(S.tabs[j] + (size_t)S.toks[j] * H + 4 * t);
                        a[0] += h2f(u.x & 0xffff); a[1] += h2f(u.x >> 16); a[2] += h2f(u.y & 0xffff); a[3] += h2f(u.y >> 16);
                    }
                    const int fr = p.frame[b];
                    const float *extra = fr < p.tr_len[b] ? p.tr + (size_t)b * p.tr_ld + (size_t)fr * H : p.pad + (size_t)b * H;
                    const float4 e = ldf4(extra + 4 * t);
                    a[0] += e.x; a[1] += e.y; a[2] += e.z; a[3] += e.w;
                    const float4 xt = make_float4(a[0], a[1], a[2], a[3]);
                    *reinterpret_cast<float4 *>(p.tx + (size_t)b * H + 4 * t) = xt;
                    double ss = (double)(xt.x * xt.x) + (double)(xt.y * xt.y) + (double)(xt.z * xt.z) + (double)(xt.w * xt.w);
                    ss = block_sum_d(ss, S.dscr);
                    const float scale = 1.0f / sqrtf((float)(ss / H) + p.eps);
                    const float4 wv = ldf4(p.tnw + 4 * t);
                    const float y0 = (xt.x * scale) * wv.x, y1 = (xt.y * scale) * wv.y, y2 = (xt.z * scale) * wv.z, y3 = (xt.w * scale) * wv.w;
                    uint2 hh2;
                    hh2.x = (uint32_t)f2h(y0) | ((uint32_t)f2h(y1) << 16);
                    hh2.y = (uint32_t)f2h(y2) | ((uint32_t)f2h(y3) << 16);
                    *reinterpret_cast<uint2 *>(p.txn + (size_t)b * H + 4 * t) = hh2;
                }
            }
        }
    }
    exit_ticket(reinterpret_cast<unsigned *>(p.state + SL.ctr), X.seq);
}

size_t cpb_lds() { return std::max(sizeof(BLds), (size_t)96 * 1024); }   // > 80 KB: one workgroup per CU
static_assert(sizeof(BLds) <= 160 * 1024, "LDS");

template <int NT>
bool cpb_attr() {
    static bool done = false;
    if (!done) {
        Q3T_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_cpb<NT>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)cpb_lds()));
        done = true;
    }
    return true;
}

}  // namespace

size_t cpb_state_bytes() { return StateLayout().total; }
bool cpb_error(const uint8_t *state, hipStream_t s, bool *err) {
    unsigned e = 0;
    Q3T_HIP(hipMemcpyAsync(&e, state + StateLayout().ctr + 32 * 4, 4, hipMemcpyDeviceToHost, s));
    Q3T_HIP(hipStreamSynchronize(s));
    *err = e != 0;
    return true;
}
bool cpb_clear(uint8_t *state, hipStream_t s) {   // after a fault: zero the flags and the error word (seq kept)
    const StateLayout L;
    Q3T_HIP(hipMemsetAsync(state + L.flags, 0, L.ctr - L.flags, s));
    Q3T_HIP(hipMemsetAsync(state + L.ctr + 32 * 4, 0, 4, s));
    Q3T_HIP(hipMemsetAsync(state + L.ctr + 48 * 4, 0, 4, s));   // the exit ticket
    return true;
}

bool cpb_resident(int device) {
    int n_cu = 0, blocks = 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cu < G) return false;
    for (const void *k : {reinterpret_cast<const void *>(&k_cpb<1>), reinterpret_cast<const void *>(&k_cpb<2>)}) {
        if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)cpb_lds()) != hipSuccess) return false;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k, 256, cpb_lds()) != hipSuccess || blocks < 1) return false;
    }
    return true;
}

bool persist_cp_batched(const CpbParams &p, hipStream_t s) {
    if (!p.L || !p.heads || !p.tabs || !p.out_norm || !p.qkvtab || !p.x_in || !p.rope || !p.pos || !p.kc || !p.vc || !p.logits ||
        !p.state || p.S < 1 || p.S > SMAX || p.sel.mode != SEL_CP || p.sel.V != CPV || !p.sel.tokens ||
        (p.talker_next && !(p.tx && p.txn && p.tnw && p.tr && p.tr_len && p.frame && p.pad))) {
        set_error("persist_cp_batched: bad parameters");
        return false;
    }
    if (p.S <= 32) {
        if (!cpb_attr<1>()) return false;
        hipLaunchKernelGGL(k_cpb<1>, dim3(G), dim3(256), cpb_lds(), s, p);
    } else {
        if (!cpb_attr<2>()) return false;
        hipLaunchKernelGGL(k_cpb<2>, dim3(G), dim3(256), cpb_lds(), s, p);
    }
    Q3T_HIP(hipGetLastError());
    return true;
}

}  // namespace q3t
