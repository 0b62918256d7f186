// persist_tkb.hip — the BATCHED talker decode step (2..64 slots, BASELINE configs[2]) as ONE persistent launch: the
// 28-layer stack, the final norm (hidden-state side output), the codec head and the CB0 selection of the next frame
// (src/tts_transformer.cpp:1376-1512 build_step_graph, :2416-2499 CB0 processing).  It replaces decoder_stack_mm's
// 7 launches per layer + head + select_tokens (engine.cpp) and computes the same bits: every projection is that
// graph's MFMA tile with the same K quarters, split-K slices and LDS sum order (persist_mm.h, gemm_mfma.hip), every
// residual + RMSNorm is k_resid_norm's arithmetic, the attention is k_attn_seq's source (attn_seq.h) and the selection
// is select_tokens' (select.h).
//
// Work per layer for S slots in NT token tiles of 32, one 256-thread workgroup per CU (persist_mm.h hand-offs):
//
//   job              count            workgroups        tile / input (per job)                      output
//   RN_A / RN_F      1 per slot       128 + 2b          x[b] += 4 slabs; RMSNorm -> f16 row          xnA / xnF [b]
//   QKV              64 x NT          [0, 64 NT)        64 rows x 32 tokens, K 1024                  qkv granules
//   ATT              8 per slot       u % 256, u = 8b+g (slot b, kv head g): the whole context          attn f16
//   O                16 x 4 x NT      [0, 64 NT)        64 rows x 32 tokens x K slice 512            slabO granules
//   GU               96 x NT          gj: [0, 128), odd slot wgs  32 SwiGLU units x 32 tokens           h f16
//   DN               16 x 4 x NT      [0, 64 NT)        64 rows x 32 tokens x K slice 768            slabD granules
//   HEAD             48 x NT          [0, 48 NT)        64 rows x 32 tokens, K 1024 (final xnA)      logits granules
//   SEL              1 per slot       128 + 2b          CB0 selection of the slot (+ logits row, commit)
//
// The residual stream of slot b never leaves its RN workgroup (4 values per thread for the whole step).  The attention
// units of a workgroup run in order u = w, w + 256: K/V chunk 0 of a unit is in flight before its QKV granules are
// polled.  Every wait is bounded (persist_dev.h SPIN_LIMIT): a protocol fault ends the launch with *err set and the
// engine falls back to the launch-per-op graph, which is bit-identical.
#include "persist.h"
#include "persist_mm.h"
#include "attn_seq.h"
#include "select.h"

#pragma clang fp contract(off)   // every rounding as written: bit-identical to k_gemm_mfma / k_resid_norm / k_attn_seq

namespace q3t {

namespace {
using namespace pmm;

constexpr int NL = 28, SW0 = 128, VPT = VOC / 256;
#ifndef TKB_NB
#define TKB_NB 4   // attention K/V ring depth (chunks of 32 KB per workgroup)
#endif

enum Kind { K_RNA = 0, K_QKV = 1, K_ATT = 2, K_O = 3, K_RNF = 4, K_GU = 5, K_DN = 6, K_HEAD = 7 };
__device__ __forceinline__ int ph_of(int l, int k) { return l * 8 + k; }   // l = NL: the final norm / head

// ---------------------------------------------------------------- state block (tkb_state_bytes, zeroed once)
struct StateLayout {
    size_t xna = 0;
    size_t xnf = xna + (size_t)SMAX * H * 2;
    size_t qkv = xnf + (size_t)SMAX * H * 2;
    size_t attn = qkv + (size_t)SMAX * QKVN * 8;
    size_t slo = attn + (size_t)SMAX * NH * D * 2;
    size_t sld = slo + (size_t)4 * SMAX * H * 8;
    size_t h = sld + (size_t)4 * SMAX * H * 8;
    size_t lg = h + (size_t)SMAX * INTER * 2;
    size_t flags = lg + (size_t)SMAX * VOC * 8;     // 8 kinds x FLAGS_PER_KIND u32
    size_t ctr = flags + 8 * FLAGS_PER_KIND * 4;    // seq, err (own lines)
    size_t total = ctr + 256;
};

struct BLds {
    uint4 wl[4][32][64];   // the next job's A fragments / the K-quarter partials (persist_mm.h)
    SelLds sel;
    AttnSeqLds att;
    double dscr[4];
    PLayerW layers[NL];
};

#ifdef Q3T_DEV
#define TPROF(ph, k)                                                                                          \
    do {                                                                                                      \
        if (p.prof && threadIdx.x == 0) p.prof[((size_t)blockIdx.x * 768 + (ph)) * 4 + (k)] = wall_clock64(); \
    } while (0)
#else
#define TPROF(ph, k) ((void)0)
#endif

template <int NT>
__global__ void __launch_bounds__(256, 1) k_tkb(const TkbParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    BLds &S = *reinterpret_cast<BLds *>(smem);
    const StateLayout SL;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, w = blockIdx.x;
    Ctx X{S.wl, p.prof, Ctl{reinterpret_cast<unsigned *>(p.state + SL.ctr) + 32, false},
          __hip_atomic_load(reinterpret_cast<unsigned *>(p.state + SL.ctr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
          reinterpret_cast<unsigned *>(p.state + SL.flags),
          __builtin_amdgcn_make_buffer_rsrc(p.state, 0, (int)SL.total, BUF_RSRC), p.S};
    const int NQJ = 64 * NT, NGJ = 96 * NT, NHJ = 48 * NT;
    const int sw = w - SW0;
    const bool rn = sw >= 0 && sw < 2 * p.S && (sw & 1) == 0;   // slot b's residual row, norms and selection
    const bool slot = sw >= 0 && sw < 2 * p.S;
    const int b = sw >> 1;
    // gate/up job gj: workgroups [0, 128), then the odd slot workgroups 129, 131, ...: the residual rows' workgroups
    // (even) run the norm right before gate/up, so a gate/up job there started ~2 us after the others
    const int gj = w < SW0 ? w : (w & 1) ? SW0 + (w - SW0 - 1) / 2 : -1;
    const bool hq = w < NQJ, hg = gj >= 0 && gj < NGJ, hh = w < NHJ;
    const int nunits = NKV * p.S;
    for (int i = t; i < NL; i += 256) S.layers[i] = p.L[i];
    __syncthreads();

    // ---- the GEMM job sequence of this workgroup, weights issued one job ahead
    int cl = 0, ck = K_QKV;   // the job whose weights S.wl holds (cl = NL + 1: none)
    auto has = [&](int k) { return k == K_GU ? hg : k == K_HEAD ? hh : hq; };
    auto advance = [&]() {
        if (ck == K_QKV) ck = K_O;
        else if (ck == K_O) ck = K_GU;
        else if (ck == K_GU) ck = K_DN;
        else if (ck == K_DN) {
            if (cl + 1 < NL) { ++cl; ck = K_QKV; }
            else { cl = NL; ck = K_HEAD; }
        } else cl = NL + 1;
    };
    auto issue = [&]() {
        while (cl <= NL && !has(ck)) advance();
        if (cl > NL) return;
        const PLayerW &Lw = S.layers[cl < NL ? cl : 0];
        switch (ck) {
            case K_QKV: load_w<4>(S.wl, Lw.qkv, H, 64 * (w % 64), 0); break;
            case K_O: load_w<2>(S.wl, Lw.o, NH * D, 64 * (w % 16), 512 * ((w / 16) % 4)); break;
            case K_GU: load_w<4>(S.wl, Lw.gu, H, 64 * (gj % 96), 0); break;
            case K_DN: load_w<3>(S.wl, Lw.down, INTER, 64 * (w % 16), 768 * ((w / 16) % 4)); break;
            default: load_w<4>(S.wl, p.head, H, 64 * (w % 48), 0); break;
        }
    };
    auto next_job = [&]() { advance(); issue(); };
    // a slot workgroup issues the next job's weights after its next attention units (its norm and attention polls then
    // do not queue behind the weight DMA), at the latest when that job starts
    bool pending = false;
    auto after_job = [&]() { if (slot) pending = true; else next_job(); };
    auto flush = [&]() { if (pending) { next_job(); pending = false; } };
    issue();

    // ---- the RN workgroups' residual row (thread t: elements 4t .. 4t+3)
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    // RMSNorm of x -> f16 row of slot b (fragment order) in `xo`, flag (kind, b); side: the f32 normalised row
    auto norm_pub = [&](const float *nw, size_t xo, int kind, uint32_t tg, float *side) {
        double ss = (double)(x.x * x.x) + (double)(x.y * x.y) + (double)(x.z * x.z) + (double)(x.w * x.w);
        ss = block_sum_d(ss, S.dscr);
        const float scale = 1.0f / sqrtf((float)(ss / H) + p.eps);
        const float4 wv = ldf4(nw + 4 * t);
        const float y0 = (x.x * scale) * wv.x, y1 = (x.y * scale) * wv.y, y2 = (x.z * scale) * wv.z, y3 = (x.w * scale) * wv.w;
        if (side) *reinterpret_cast<float4 *>(side + (size_t)b * H + 4 * t) = make_float4(y0, y1, y2, y3);
        const u32x2_t hv = {(uint32_t)f2h(y0) | ((uint32_t)f2h(y1) << 16), (uint32_t)f2h(y2) | ((uint32_t)f2h(y3) << 16)};
        TPROF((int)((tg - 1u) & 1023u), 3);
        __builtin_amdgcn_raw_buffer_store_b64(hv, X.rs, (int)xo + fragoff(H / 8, b, 4 * t), 0, SC1);
        publish(X, kind, b, tg);
    };
    // x += the 4 split-K slabs of slot b (k_resid_norm<4> order)
    auto fold = [&](size_t slab, uint32_t tg) {
        TPROF((int)((tg - 1u) & 1023u), 0);
        u32x4_t pz[8];
        poll_gran<8>(X, tg, pz, [&](u32x4_t (&r)[8]) {
#pragma unroll
            for (int z = 0; z < 4; ++z)
#pragma unroll
                for (int hh2 = 0; hh2 < 2; ++hh2)
                    r[2 * z + hh2] = __builtin_amdgcn_raw_buffer_load_b128(X.rs, (int)(slab + (((size_t)z * SMAX + b) * H + 4 * t + 2 * hh2) * 8), 0, SC1V);
        });
        TPROF((int)((tg - 1u) & 1023u), 1);
#pragma unroll
        for (int z = 0; z < 4; ++z)
            x = make_float4(x.x + __uint_as_float(pz[2 * z].x), x.y + __uint_as_float(pz[2 * z].z), x.z + __uint_as_float(pz[2 * z + 1].x),
                            x.w + __uint_as_float(pz[2 * z + 1].z));
    };

    for (int l = 0; l < NL; ++l) {
        const PLayerW &Lw = S.layers[l];
        // ---- RN_A: the layer's input row, normalised (layer 0: the step's input row)
        if (rn) {
            if (l == 0) x = ldf4(p.x_in + (size_t)b * H + 4 * t);
            else fold(SL.sld, X.tag(ph_of(l - 1, K_DN)));
            norm_pub(Lw.attn_norm, SL.xna, K_RNA, X.tag(ph_of(l, K_RNA)), nullptr);
        }
        // ---- QKV: rows 64 rp .. +63 of tile tt -> granules
        if (hq) {
            flush();
            const int rp = w % 64, tt = w / 64;
            const int nv = min(32, p.S - 32 * tt);
            wait_flags_wg(X, K_RNA, nv, [&](int i) { return 32 * tt + i; }, X.tag(ph_of(l, K_RNA)));
            mm_tile<4>(X, SL.xna, H / 8, 0, 32 * tt);
            TPROF(ph_of(l, K_QKV), 3);
            epi_gran(X, SL.qkv, QKVN, 64 * rp, 32 * tt, X.tag(ph_of(l, K_QKV)));
            TPROF(ph_of(l, K_QKV), 2);
            pending = true;   // the O weights after the attention units: their polls and K/V streams go first
        }
        // ---- ATT: units u = w, w + 256 (slot u / 8, kv head u % 8), the whole context of each, in turn as one chunk
        // stream (the second unit's first chunks in flight during the first unit's tail)
        if (w < nunits) {
            const uint32_t tq = X.tag(ph_of(l, K_QKV));
            const int nu = w + G < nunits ? 2 : 1, g = w & 7;
            const int ub[2] = {w >> 3, (w + G) >> 3};
            TPROF(ph_of(l, K_QKV), 0);
            attn_seq_stream<TKB_NB>(
                nu,
                [&](int k, int &pos, uint16_t *&kc, uint16_t *&vc, const float *&rope_row) {
                    pos = p.pos[ub[k]];
                    const size_t hoff = (size_t)l * p.kv_layer + ((size_t)ub[k] * NKV + g) * p.n_ctx * D;
                    kc = p.kc + hoff;
                    vc = p.vc + hoff;
                    rope_row = p.rope + (size_t)pos * D;
                },
                Lw.qn, Lw.kn, p.eps,
                [&](int k, int v, float (&xv)[2]) {   // wave v: q head 2g + v (v < 2), k (2), v (3) of slot ub[k]
                    const int row = v < 2 ? (2 * g + v) * D : v == 2 ? (NH + g) * D : (NH + NKV + g) * D;
                    u32x4_t gq[1];
                    poll_gran<1>(X, tq, gq, [&](u32x4_t (&r)[1]) {
                        const size_t o = SL.qkv + ((size_t)ub[k] * QKVN + row + lane) * 8;
                        const u32x2_t a = __builtin_amdgcn_raw_buffer_load_b64(X.rs, (int)o, 0, SC1V);
                        const u32x2_t c = __builtin_amdgcn_raw_buffer_load_b64(X.rs, (int)(o + 64 * 8), 0, SC1V);
                        r[0] = u32x4_t{a.x, a.y, c.x, c.y};
                    });
                    if (k == 0 && v == 0) TPROF(ph_of(l, K_QKV), 1);
                    xv[0] = __uint_as_float(gq[0].x);
                    xv[1] = __uint_as_float(gq[0].z);
                },
                [&](int k, int hd, int d, float y) {   // one half of the slot's attention row, fragment order
                    __builtin_amdgcn_raw_buffer_store_b16(f2h(y), X.rs, (int)SL.attn + fragoff(NH * D / 8, ub[k], (2 * g + hd) * D + d), 0, SC1);
                },
                [&](int k) {
                    if (k == 0) TPROF(ph_of(l, K_ATT), 3);
                    publish(X, K_ATT, w + k * G, X.tag(ph_of(l, K_ATT)));
                },
                S.att);
        }
        flush();
        // ---- O: split-K slab z of rows 64 rp .. +63, tile tt: heads 4z .. 4z+3 = kv heads 2z, 2z+1 of the tile's slots
        if (hq) {
            const int rp = w % 16, z = (w / 16) % 4, tt = w / 64;
            const int nv = min(32, p.S - 32 * tt);
            // wave w multiplies head 4 z + w: the units of kv head 2 z + w / 2 of the tile's slots (its own wait, no barrier)
            wait_flags(X, K_ATT, nv, [&](int i) { return (32 * tt + i) * NKV + 2 * z + (wave >> 1); }, X.tag(ph_of(l, K_ATT)));
            mm_tile<2>(X, SL.attn, NH * D / 8, 512 * z, 32 * tt);
            TPROF(ph_of(l, K_O), 3);
            epi_gran(X, SL.slo + (size_t)z * SMAX * H * 8, H, 64 * rp, 32 * tt, X.tag(ph_of(l, K_O)));
            TPROF(ph_of(l, K_O), 2);
            after_job();
        }
        // ---- RN_F
        if (rn) {
            fold(SL.slo, X.tag(ph_of(l, K_O)));
            norm_pub(Lw.ffn_norm, SL.xnf, K_RNF, X.tag(ph_of(l, K_RNF)), nullptr);
        }
        // ---- GU: 32 SwiGLU units (rows 64 rp .. +63, gate/up interleaved in 16-row blocks), tile tt
        if (hg) {
            flush();
            const int rp = gj % 96, tt = gj / 96;
            const int nv = min(32, p.S - 32 * tt);
            wait_flags_wg(X, K_RNF, nv, [&](int i) { return 32 * tt + i; }, X.tag(ph_of(l, K_RNF)));
            mm_tile<4>(X, SL.xnf, H / 8, 0, 32 * tt);
            TPROF(ph_of(l, K_GU), 3);
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
            publish(X, K_GU, gj, X.tag(ph_of(l, K_GU)));
            after_job();
        }
        // ---- DN: split-K slab z of rows 64 rp .. +63, tile tt; wave w reads units [768 z + 192 w, +192)
        if (hq) {
            flush();
            const int rp = w % 16, z = (w / 16) % 4, tt = w / 64;
            // each wave waits for the 6 gate/up jobs of its own K quarter only (units [768 z + 192 w, +192)): no barrier,
                // no wave held by another quarter's late producer
                wait_flags(X, K_GU, 6, [&](int i) { return 24 * z + 6 * wave + i + 96 * tt; }, X.tag(ph_of(l, K_GU)));
            mm_tile<3>(X, SL.h, INTER / 8, 768 * z, 32 * tt);
            TPROF(ph_of(l, K_DN), 3);
            epi_gran(X, SL.sld + (size_t)z * SMAX * H * 8, H, 64 * rp, 32 * tt, X.tag(ph_of(l, K_DN)));
            TPROF(ph_of(l, K_DN), 2);
            after_job();
        }
    }
    // ---- final RMSNorm (output_norm, hidden-state side output) -> codec head -> CB0 selection
    if (rn) {
        fold(SL.sld, X.tag(ph_of(NL - 1, K_DN)));
        norm_pub(p.out_norm, SL.xna, K_RNA, X.tag(ph_of(NL, K_RNA)), p.hidden);
    }
    if (hh) {
        flush();
        const int rp = w % 48, tt = w / 48;
        const int nv = min(32, p.S - 32 * tt);
        wait_flags_wg(X, K_RNA, nv, [&](int i) { return 32 * tt + i; }, X.tag(ph_of(NL, K_RNA)));
        mm_tile<4>(X, SL.xna, H / 8, 0, 32 * tt);
        TPROF(ph_of(NL, K_HEAD), 3);
        epi_gran(X, SL.lg, VOC, 64 * rp, 32 * tt, X.tag(ph_of(NL, K_HEAD)));
        TPROF(ph_of(NL, K_HEAD), 2);
    }
    if (rn) {
        const uint32_t tg = X.tag(ph_of(NL, K_HEAD));
        TPROF(ph_of(NL, K_HEAD), 0);
        SelPre pre;   // the selection's per-slot inputs (done, frame, seed, seen bytes) before the poll, off the chain
        if (p.select) sel_prefetch<SEL_CB0>(p.sel, b, pre);
        u32x4_t lr[VPT / 2];   // thread t: logits VPT t .. VPT t + VPT - 1 (select_token's exact-width ownership, V = 3072)
        poll_gran<VPT / 2>(X, tg, lr, [&](u32x4_t (&r)[VPT / 2]) {
#pragma unroll
            for (int k = 0; k < VPT / 2; ++k)
                r[k] = __builtin_amdgcn_raw_buffer_load_b128(X.rs, (int)(SL.lg + ((size_t)b * VOC + VPT * t + 2 * k) * 8), 0, SC1V);
        });
        TPROF(ph_of(NL, K_HEAD), 1);
        float v[SEL_VPT_MAX];
#pragma unroll
        for (int k = 0; k < VPT / 2; ++k) { v[2 * k] = __uint_as_float(lr[k].x); v[2 * k + 1] = __uint_as_float(lr[k].z); }
#pragma unroll
        for (int e = VPT; e < SEL_VPT_MAX; ++e) v[e] = -INFINITY;
        if (p.logits) {   // the logits row, as the per-op head GEMM writes it
            float *row = p.logits + (size_t)b * VOC + VPT * t;
#pragma unroll
            for (int k = 0; k < VPT / 4; ++k) *reinterpret_cast<float4 *>(row + 4 * k) = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
        }
        if (p.select) {
            const int tok = select_token_pre<SEL_CB0>(p.sel, pre, v, S.sel);   // -1: slot done
            if (t == 0 && tok >= 0) select_commit(p.sel, b, tok);
        }
        TPROF(ph_of(NL, K_HEAD), 3);
    }
    exit_ticket(reinterpret_cast<unsigned *>(p.state + SL.ctr), X.seq);
}

size_t tkb_lds() { return std::max(sizeof(BLds), (size_t)96 * 1024); }   // > 80 KB: one workgroup per CU
static_assert(sizeof(BLds) <= 160 * 1024, "LDS");

template <int NT>
bool tkb_attr() {
    static bool done = false;
    if (!done) {
        Q3T_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_tkb<NT>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)tkb_lds()));
        done = true;
    }
    return true;
}

}  // namespace

size_t tkb_state_bytes() { return StateLayout().total; }
bool tkb_error(const uint8_t *state, hipStream_t s, bool *err) {
    unsigned e = 0;
    Q3T_HIP(hipMemcpyAsync(&e, state + StateLayout().ctr + 32 * 4, 4, hipMemcpyDeviceToHost, s));
    Q3T_HIP(hipStreamSynchronize(s));
    *err = e != 0;
    return true;
}
bool tkb_clear(uint8_t *state, hipStream_t s) {   // after a fault: zero the flags and the error word (seq kept)
    const StateLayout L;
    Q3T_HIP(hipMemsetAsync(state + L.flags, 0, L.ctr - L.flags, s));
    Q3T_HIP(hipMemsetAsync(state + L.ctr + 32 * 4, 0, 4, s));
    Q3T_HIP(hipMemsetAsync(state + L.ctr + 48 * 4, 0, 4, s));   // the exit ticket
    return true;
}

bool tkb_resident(int device) {
    int n_cu = 0, blocks = 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cu < G) return false;
    for (const void *k : {reinterpret_cast<const void *>(&k_tkb<1>), reinterpret_cast<const void *>(&k_tkb<2>)}) {
        if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tkb_lds()) != hipSuccess) return false;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k, 256, tkb_lds()) != hipSuccess || blocks < 1) return false;
    }
    return true;
}

bool persist_talker_batched(const TkbParams &p, hipStream_t s) {
    if (!p.L || p.n_layers != NL || !p.head || !p.out_norm || !p.x_in || !p.hidden || !p.rope || !p.pos || !p.kc || !p.vc ||
        p.n_ctx < 1 || !p.state || p.S < 2 || p.S > SMAX || (p.select && (p.sel.mode != SEL_CB0 || p.sel.V != VOC || !p.sel.tokens))) {
        set_error("persist_talker_batched: bad parameters");
        return false;
    }
    if (p.S <= 32) {
        if (!tkb_attr<1>()) return false;
        hipLaunchKernelGGL(k_tkb<1>, dim3(G), dim3(256), tkb_lds(), s, p);
    } else {
        if (!tkb_attr<2>()) return false;
        hipLaunchKernelGGL(k_tkb<2>, dim3(G), dim3(256), tkb_lds(), s, p);
    }
    Q3T_HIP(hipGetLastError());
    return true;
}

}  // namespace q3t
