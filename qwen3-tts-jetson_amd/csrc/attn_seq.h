// attn_seq.h — decode attention of ONE (slot, kv head) on ONE 256-thread workgroup walking the whole context
// (src/tts_transformer.cpp:1410-1475: head RMSNorm over 128 lanes, NEOX RoPE at pos, F16 KV append, softmax with scale
// 1/sqrt(D), GQA: 2 q heads per kv head).  Shared source of k_attn_seq (attn.hip, one launch per layer at >= 16 slots)
// and the persistent batched talker step (persist_tkb.hip), so both compute the same bits.
//
// The workgroup walks its context in 64-position chunks with the next NB - 1 chunks' K/V loads in flight (a register
// ring of NB chunks: k_attn_seq, two workgroups per CU, NB = 2; the persistent step, one per CU, a deeper ring -- one
// chunk in flight per CU bounded it at ~20 GB/s per CU); each wave keeps its own online-softmax state (max, sum, 8-dim accumulator per head) over its 16 positions of
// every chunk, so no barrier is taken per chunk; the four waves merge once at the end.  Scores are v_dot2_f32_f16 on the
// packed K registers against the f16-exact q, exponentials v_exp_f32 (__expf); every chunk but the last is whole (all
// 64 positions <= pos: no masks), and the new K/V row (pos) is read from LDS in place of the last chunk's loaded one.
//
// The caller supplies the raw QKV values (qkv_of: wave v < 2 q head 2g + v, v = 2 the new k, v = 3 the new v; lanes
// lane and lane + 64) -- K/V chunk 0 is in flight before it is called -- and the output store (out: one value, or with
// VEC4 four consecutive dims of threads 0..63; the per-dim arithmetic does not depend on the thread that runs it).
// (Measured and rejected: two units per workgroup with their whole chunks interleaved -- two dependency chains per wave
// -- spilled 340 B per lane inside the persistent step and ran 20 us per layer against 15 us for the two in turn.)
#pragma once
#include "kernels.h"

#include <type_traits>

#pragma clang fp contract(off)   // every rounding as written (both includers compile with contraction off too)

namespace q3t {

struct AttnSeqLds {
    float q_s[2][128];
    alignas(16) uint16_t kh_s[128];
    alignas(16) uint16_t vh_s[128];
    float wm[4][2], wl[4][2];
    float wa[4][2][128];
};

namespace aseq {
typedef unsigned int u32x4_s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16(const uint16_t *p) {
    typedef const __attribute__((address_space(1))) u32x4_s gv;
    const u32x4_s v = *(gv *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
// each converted value materialised: the consumer FMA may not absorb the conversion into a v_fma_mix_f32 (whose f16
// operands do not go through v_cvt_f32_f16: whole chunks then differed from the masked last chunk)
__device__ __forceinline__ void unpack8_cvt(const uint4 u, float (&f)[8]) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) { f[2 * e] = opaque(h2f(w[e] & 0xffff)); f[2 * e + 1] = opaque(h2f(w[e] >> 16)); }
}
}  // namespace aseq

namespace aseq {
constexpr int D = 128, R = 2, LPP = D / 8, NP = 4;   // 16 lanes per position, 4 passes of 16 positions per 64-chunk
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
struct Unit {   // one (slot, kv head): its cache, position and online-softmax state (this thread's share)
    int pos, nch;
    uint16_t *kc, *vc;
    h2_t q2[R][4];
    float m[R], l[R], acc[R][8];
};
__device__ __forceinline__ void unit_init(Unit &U, int pos, uint16_t *kc, uint16_t *vc) {
    U.pos = pos;
    U.nch = pos / 64 + 1;
    U.kc = kc;
    U.vc = vc;
}
// chunk c >= U.nch: a placeholder issue (the ring's steps past the end) -- the same load instructions, every lane on the
// cache's first 16 bytes (one line per instruction), the registers never read
__device__ __forceinline__ void issue(const Unit &U, int c, uint4 (&kr)[NP], uint4 (&vr)[NP]) {
    const int t = threadIdx.x, pg = t / LPP, li = t % LPP;
    const bool live = c < U.nch;
#pragma unroll
    for (int pi = 0; pi < NP; ++pi) {
        const int o = live ? min(c * 64 + pi * 16 + pg, U.pos) * D + li * 8 : 0;
        kr[pi] = ld16(U.kc + o);
        vr[pi] = ld16(U.vc + o);
    }
}
// head RMSNorm + NEOX RoPE of the R q heads and the new k (k_attn arithmetic); the new v f16-rounded (wave v: vector v)
template <class QkvOf>
__device__ __forceinline__ void prologue(const float *rope_row, const float *qn, const float *kn, float eps, QkvOf qkv_of,
                                         AttnSeqLds &L) {
    const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
    float x[2];
    qkv_of(v, x);
    if (v == R + 1) {
#pragma unroll
        for (int e = 0; e < 2; ++e) L.vh_s[lane + 64 * e] = f2h(x[e]);
    } else {
        const bool isk = v == R;
        const float *w = isk ? kn : qn;
        double ss = 0.0;
#pragma unroll
        for (int e = 0; e < 2; ++e) ss += (double)__fmul_rn(x[e], x[e]);
        ss = wave_sum_d(ss);
        const float scale = 1.0f / sqrtf((float)(ss / D) + eps);
#pragma unroll
        for (int e = 0; e < 2; ++e) x[e] = (x[e] * scale) * w[lane + 64 * e];
        const float c = rope_row[2 * lane], s = rope_row[2 * lane + 1];
        const float y0 = opaque(opaque(x[0] * c) - opaque(x[1] * s));
        const float y1 = opaque(opaque(x[0] * s) + opaque(x[1] * c));
        if (isk) {
            L.kh_s[lane] = f2h(y0);
            L.kh_s[lane + 64] = f2h(y1);
        } else {
            L.q_s[v][lane] = f16r(y0);
            L.q_s[v][lane + 64] = f16r(y1);
        }
    }
}
// after the barrier that follows prologue(): the KV append at pos, q as f16 pairs (f16-exact: the scores are
// v_dot2_f32_f16 straight from the K registers), the state zeroed
__device__ __forceinline__ void start(Unit &U, const AttnSeqLds &L) {
    const int t = threadIdx.x, li = t % LPP;
    if (t < D) {
        U.kc[(size_t)U.pos * D + t] = L.kh_s[t];
        U.vc[(size_t)U.pos * D + t] = L.vh_s[t];
    }
#pragma unroll
    for (int h = 0; h < R; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            U.q2[h][e].x = (_Float16)L.q_s[h][li * 8 + 2 * e];
            U.q2[h][e].y = (_Float16)L.q_s[h][li * 8 + 2 * e + 1];
        }
#pragma unroll
    for (int h = 0; h < R; ++h) {
        U.m[h] = -INFINITY;
        U.l[h] = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) U.acc[h][e] = 0.0f;
    }
}
// one chunk; LAST: positions past pos masked, a wave may hold no live position yet
// The new row (pos, in LDS since start()) stands in for the last chunk's loaded one at its use: pass (pos % 64) / 16,
// position group pos % 16 (the ring registers are only read, so the compiler keeps no copies of them)
template <bool LAST>
__device__ __forceinline__ void chunk(Unit &U, int c, const uint4 (&kr)[NP], const uint4 (&vr)[NP], const AttnSeqLds &L) {
    const int pg = threadIdx.x / LPP, li = threadIdx.x % LPP;
    uint4 kn4, vn4;
    if constexpr (LAST) {
        kn4 = *reinterpret_cast<const uint4 *>(&L.kh_s[li * 8]);
        vn4 = *reinterpret_cast<const uint4 *>(&L.vh_s[li * 8]);
    }
    auto isnew = [&](int pi) { return LAST && pi == ((U.pos & 63) >> 4) && pg == (U.pos & 15); };
    const float kq_scale = 1.0f / sqrtf((float)D);
    // the last chunk's passes past pos hold no live position for any lane: they are skipped (exactly: their scores
    // are -inf, their exponentials 0, and adding 0 leaves l and acc -- never -0 -- unchanged)
    const int npi = LAST ? ((U.pos & 63) >> 4) + 1 : NP;
    float sc[NP][R];
    bool ok[NP];
#pragma unroll
    for (int pi = 0; pi < NP; ++pi) {
        ok[pi] = !LAST || c * 64 + pi * 16 + pg <= U.pos;
        if (LAST && pi >= npi) {
#pragma unroll
            for (int h = 0; h < R; ++h) sc[pi][h] = -INFINITY;
            continue;
        }
        const uint4 kv = isnew(pi) ? kn4 : kr[pi];
        const uint32_t kw[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
        for (int h = 0; h < R; ++h) {
            float s = 0.0f;
#pragma unroll
            for (int e = 0; e < 4; ++e) s = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, kw[e]), U.q2[h][e], s, false);
            s = group_sum<LPP>(s);
            sc[pi][h] = ok[pi] ? __fmul_rn(s, kq_scale) : -INFINITY;
        }
    }
#pragma unroll
    for (int h = 0; h < R; ++h) {
        float mc = sc[0][h];
#pragma unroll
        for (int pi = 1; pi < NP; ++pi) mc = fmaxf(mc, sc[pi][h]);
        mc = rows_max(mc);                      // this wave's 16 positions of the chunk
        const float mn = fmaxf(U.m[h], mc);
        if (LAST && mn == -INFINITY) continue;  // no live position in this wave yet
        const float alpha = __expf(__fsub_rn(U.m[h], mn));
        U.l[h] *= alpha;
#pragma unroll
        for (int e = 0; e < 8; ++e) U.acc[h][e] *= alpha;
        U.m[h] = mn;
    }
#pragma unroll
    for (int pi = 0; pi < NP; ++pi) {
        if (LAST && pi >= npi) continue;
        float v8[8];
        unpack8_cvt(isnew(pi) ? vn4 : vr[pi], v8);
#pragma unroll
        for (int h = 0; h < R; ++h) {
            const float pr = ok[pi] ? __expf(__fsub_rn(sc[pi][h], U.m[h])) : 0.0f;
            U.l[h] += pr;
#pragma unroll
            for (int e = 0; e < 8; ++e) U.acc[h][e] = __fmaf_rn(pr, ok[pi] ? v8[e] : 0.0f, U.acc[h][e]);
        }
    }
}
// merge the four waves' states (LDS), then the outputs
template <bool VEC4, class Out>
__device__ __forceinline__ void finish(const Unit &U, Out out, AttnSeqLds &L) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, li = t % LPP;
#pragma unroll
    for (int h = 0; h < R; ++h) {
        const float ls = rows_sum(U.l[h]);
        if (lane == 0) { L.wm[wave][h] = U.m[h]; L.wl[wave][h] = ls; }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float a = rows_sum(U.acc[h][e]);
            if (lane < 16) L.wa[wave][h][li * 8 + e] = a;
        }
    }
    __syncthreads();
    auto merged = [&](int h, int d) {
        const float M = fmaxf(fmaxf(L.wm[0][h], L.wm[1][h]), fmaxf(L.wm[2][h], L.wm[3][h]));
        float num = 0.0f, den = 0.0f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            if (L.wm[w][h] == -INFINITY) continue;
            const float f = expf(__fsub_rn(L.wm[w][h], M));
            num = __fmaf_rn(L.wa[w][h][d], f, num);
            den = __fmaf_rn(L.wl[w][h], f, den);
        }
        return num / den;
    };
    if constexpr (VEC4) {
        if (t < 64) {
            const int h = t >> 5, d0 = (t & 31) * 4;
            float y[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) y[e] = merged(h, d0 + e);
            out(h, d0, y);
        }
    } else {
        for (int o = t; o < R * D; o += 256) out(o / D, o % D, merged(o / D, o % D));
    }
}
}  // namespace aseq

//   kc/vc: this (layer, slot, kv head)'s cache [n_ctx][128] f16 (row pos is written here); rope_row: rope + pos * 128
template <bool VEC4, int NB, class QkvOf, class Out>
__device__ __forceinline__ void attn_seq_wg(int pos, uint16_t *kc, uint16_t *vc, const float *rope_row, const float *qn,
                                            const float *kn, float eps, QkvOf qkv_of, Out out, AttnSeqLds &L) {
    using namespace aseq;
    static_assert(NB >= 2 && NB <= 4, "ring depth");
    Unit U;
    unit_init(U, pos, kc, vc);
    uint4 kq[NB][NP], vq[NB][NP];
    // every ring step issues one chunk, unconditionally (past the end: a placeholder, see issue), so every path
    // to a chunk's first use has the same NB - 1 chunks issued after it and the compiler's wait is vmcnt(8 (NB - 1)),
    // not vmcnt(0) (a conditional issue made the path without it the wait's worst case: every chunk then waited for
    // the chunks issued after it, and the ring held one chunk in flight)
#pragma unroll
    for (int c = 0; c < NB - 1; ++c) issue(U, c, kq[c], vq[c]);
    prologue(rope_row, qn, kn, eps, qkv_of, L);
    __syncthreads();
    start(U, L);
    for (int c0 = 0; c0 < U.nch; c0 += NB) {
#pragma unroll
        for (int k = 0; k < NB; ++k) {   // ring slots are compile-time: chunk c0 + k in slot k
            const int c = c0 + k;
            issue(U, c + NB - 1, kq[(k + NB - 1) % NB], vq[(k + NB - 1) % NB]);
            if (c < U.nch) {
                if (c + 1 < U.nch) chunk<false>(U, c, kq[k], vq[k], L);
                else chunk<true>(U, c, kq[k], vq[k], L);
            }
        }
    }
    finish<VEC4>(U, out, L);
}

// nu (1 or 2) units of one workgroup in turn as ONE chunk stream through the NB register ring: the second unit's first
// chunks are issued during the first unit's last chunks, so they land while it merges and publishes.  Each unit's
// arithmetic is attn_seq_wg's.  unit(k, pos, kc, vc, rope_row) describes unit k; qkv_of(k, v, x) / out(k, h, d, y)
// as attn_seq_wg's (one output dimension per thread: the merge on all four waves); done(k) runs on the whole workgroup after unit k's outputs (its publish).
template <int NB, class UnitOf, class QkvOf, class Out, class Done>
__device__ __forceinline__ void attn_seq_stream(int nu, UnitOf unit_of, const float *qn, const float *kn, float eps,
                                                QkvOf qkv_of, Out out, Done done, AttnSeqLds &L) {
    using namespace aseq;
    static_assert(NB >= 2 && NB <= 4, "ring depth");
    Unit Ud[2];   // descriptors (pos, nch, caches) of both units; the softmax state lives in U
    const float *rope[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        int pos = 0;
        uint16_t *kc = nullptr, *vc = nullptr;
        rope[k] = nullptr;
        if (k < nu) unit_of(k, pos, kc, vc, rope[k]);
        unit_init(Ud[k], pos, kc, vc);
    }
    const int n0 = Ud[0].nch, total = n0 + (nu > 1 ? Ud[1].nch : 0);
    auto issue_g = [&](int g, uint4 (&kr)[NP], uint4 (&vr)[NP]) {   // chunk g of the stream (g >= total: placeholder)
        if (g < n0 || g >= total) issue(Ud[0], g < n0 ? g : n0, kr, vr);
        else issue(Ud[1], g - n0, kr, vr);
    };
    uint4 kq[NB][NP], vq[NB][NP];
    // unconditional issues (placeholders past the stream's end): the compiler's waits count NB - 1 chunks in flight
    // (attn_seq_wg)
#pragma unroll
    for (int g = 0; g < NB - 1; ++g) issue_g(g, kq[g], vq[g]);
    Unit U = Ud[0];
    prologue(rope[0], qn, kn, eps, [&](int v, float (&x)[2]) { qkv_of(0, v, x); }, L);
    __syncthreads();
    start(U, L);
    for (int g0 = 0; g0 < total; g0 += NB) {
#pragma unroll
        for (int k = 0; k < NB; ++k) {   // ring slots are compile-time: chunk g0 + k in slot k
            const int g = g0 + k;
            issue_g(g + NB - 1, kq[(k + NB - 1) % NB], vq[(k + NB - 1) % NB]);
            if (g < total) {
                if (g == n0) {   // unit boundary: the first unit's merge, outputs and publish, the second's prologue
                    finish<false>(U, [&](int h, int d, float y) { out(0, h, d, y); }, L);
                    done(0);
                    U = Ud[1];
                    prologue(rope[1], qn, kn, eps, [&](int v, float (&x)[2]) { qkv_of(1, v, x); }, L);
                    __syncthreads();
                    start(U, L);
                }
                const int c = g < n0 ? g : g - n0;
                if (c + 1 < U.nch) chunk<false>(U, c, kq[k], vq[k], L);
                else chunk<true>(U, c, kq[k], vq[k], L);
            }
        }
    }
    finish<false>(U, [&](int h, int d, float y) { out(nu - 1, h, d, y); }, L);
    done(nu - 1);
}

}  // namespace q3t
