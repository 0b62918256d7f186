// attn.hip — decode attention of the talker (and of the code predictor when its fused O-projection prologue is not
// used): one new token per slot, Qwen3 block semantics of src/tts_transformer.cpp:1410-1475 (head RMSNorm over the
// 128 lanes, NEOX RoPE at pos, F16 KV append, flash_attn_ext with scale 1/sqrt(D), GQA head h -> kv head h/R).
//
// MI355X layout: grid (slot, kv head, split), one 256-thread workgroup per ATTN_CHUNK = 64 positions.  Every lane
// issues its K and V loads (NP x 16 B each) before anything else, so a chunk is ONE memory round trip; D/8 lanes
// per position, dot products reduced with xor butterflies.  Split partials (m, l, acc) are published with
// agent-scope (sc1) stores and an arrival ticket; the workgroup whose ticket add comes last combines them in the
// same launch (MI355X_MICROARCH.md, hand-off table row 1: sc1 stores -> vmcnt(0) -> barrier -> one agent atomic
// add; the last adder loads the partials with sc1 loads) -- no combine launch, no release/acquire cache flushes.
#include "kernels.h"
#include "attn_small.h"
#include "attn_seq.h"

#include <type_traits>

#pragma clang fp contract(off)   // every rounding as written (persist.hip reproduces this kernel bit for bit)

namespace q3t {

template <class V>
__device__ __forceinline__ V ldg_a(const void *p) {
    typedef const __attribute__((address_space(1))) V gV;
    return *(gV *)(p);
}
typedef unsigned int u32x4_a __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldg16(const uint16_t *p) {
    const u32x4_a v = ldg_a<u32x4_a>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_sc1(float *p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ float ld_sc1(const float *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void unpack8(const uint4 u, float (&f)[8]) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) { f[2 * e] = h2f(w[e] & 0xffff); f[2 * e + 1] = h2f(w[e] >> 16); }
}
// the same with each converted value materialised: the consumer FMA may not absorb the conversion into a
// v_fma_mix_f32 (whose f16 operands do not go through v_cvt_f32_f16: k_attn_seq's whole chunks then differed from
// its masked last chunk, where a select sits between the two)
__device__ __forceinline__ void unpack8_cvt(const uint4 u, float (&f)[8]) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) { f[2 * e] = opaque(h2f(w[e] & 0xffff)); f[2 * e + 1] = opaque(h2f(w[e] >> 16)); }
}

template <int D, int RMAX, int CHUNK>
__global__ void __launch_bounds__(256) k_attn(const AttnParams p) {
    constexpr int LPP = D / 8;               // lanes per position
    constexpr int PPP = 256 / LPP;           // positions per pass
    constexpr int NP = CHUNK / PPP;          // passes per chunk
    constexpr int E = D / 64;                // elements per lane in the one-wave-per-vector prologue
    const int slot = blockIdx.x, g = blockIdx.y, split = blockIdx.z;
    constexpr int R = RMAX;   // q heads per kv head
    const int pos = p.pos[slot];
    const int j0 = split * CHUNK;
    if (j0 > pos) return;
    const int nsplit = pos / CHUNK + 1;
    const bool has_pos = split == nsplit - 1;   // this chunk contains the new token
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, pg = t / LPP, li = t % LPP;

    __shared__ float q_s[RMAX][D];
    __shared__ float kn_s[D], vn_s[D];
    __shared__ float wred[4][RMAX];
    __shared__ float ared[4][RMAX][D];
    __shared__ float cm[RMAX], cl[RMAX];
    __shared__ float sm[ATTN_MAX_SPLITS][RMAX], sl[ATTN_MAX_SPLITS][RMAX], sw[ATTN_MAX_SPLITS][RMAX];
    __shared__ unsigned last_s;

    // ---- (1) this chunk's K/V rows: every load issued up front (clamped rows are masked later)
    const size_t head_off = ((size_t)slot * p.nKV + g) * p.n_ctx * D;
    uint4 kr[NP], vr[NP];
#pragma unroll
    for (int pi = 0; pi < NP; ++pi) {
        // rows past pos (masked below) re-read row pos: no HBM bytes beyond the live context (the last chunk of a
        // context at p = 266 would otherwise fetch 53 dead rows of 64)
        const int j = min(j0 + pi * PPP + pg, pos);
        kr[pi] = ldg16(p.kc + head_off + (size_t)j * D + li * 8);
        vr[pi] = ldg16(p.vc + head_off + (size_t)j * D + li * 8);
    }

    // ---- (2) head RMSNorm (double sum, ggml_rms_norm) + NEOX RoPE of the R q heads and the new k; f16-rounded
    const int QKV = (p.nH + 2 * p.nKV) * D;
    const float *qkv = p.qkv + (size_t)slot * QKV;
    const float *rope = p.rope + (size_t)pos * D;
    const int nvec = R + (has_pos ? 2 : 0);
    for (int v = wave; v < nvec; v += 4) {
        if (v == R + 1) {   // the new v row: f16-rounded, no norm
#pragma unroll
            for (int e = 0; e < E; ++e) vn_s[lane + 64 * e] = f16r(qkv[(size_t)(p.nH + p.nKV + g) * D + lane + 64 * e]);
            continue;
        }
        const bool isk = v == R;
        const float *src = isk ? qkv + (size_t)(p.nH + g) * D : qkv + (size_t)(g * R + v) * D;
        const float *w = isk ? p.kn : p.qn;
        float x[E];
        double ss = 0.0;
#pragma unroll
        for (int e = 0; e < E; ++e) { x[e] = src[lane + 64 * e]; ss += (double)__fmul_rn(x[e], x[e]); }
        ss = wave_sum_d(ss);
        const float scale = 1.0f / sqrtf((float)(ss / D) + p.eps);
#pragma unroll
        for (int e = 0; e < E; ++e) x[e] = (x[e] * scale) * w[lane + 64 * e];
        float y[E];
        if constexpr (D == 128) {
            const float c = rope[2 * lane], s = rope[2 * lane + 1];
            // every rounding explicit (no fma / fma_mix fusion): the persistent step (persist.hip) reproduces it bit for bit
            y[0] = opaque(opaque(x[0] * c) - opaque(x[1] * s));
            y[1] = opaque(opaque(x[0] * s) + opaque(x[1] * c));
        } else {
            const int i = lane & 31;
            const float c = rope[2 * i], s = rope[2 * i + 1];
            const float other = __shfl_xor(x[0], 32, 64);
            y[0] = lane < 32 ? x[0] * c - other * s : other * s + x[0] * c;
        }
        float *dst = isk ? kn_s : q_s[v];
#pragma unroll
        for (int e = 0; e < E; ++e) dst[lane + 64 * e] = f16r(y[e]);
    }
    __syncthreads();
    if (has_pos)   // KV append at pos (the only block that touches position pos)
        for (int e = t; e < D; e += 256) {
            p.kc[head_off + (size_t)pos * D + e] = f2h(kn_s[e]);
            p.vc[head_off + (size_t)pos * D + e] = f2h(vn_s[e]);
        }

    // ---- (3) scores of this lane's NP positions for the R heads
    const float kq_scale = 1.0f / sqrtf((float)D);
    float q8[RMAX][8];
#pragma unroll
    for (int h = 0; h < RMAX; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) q8[h][e] = h < R ? q_s[h][li * 8 + e] : 0.0f;
    float sc[NP][RMAX];
    bool ok[NP];
    uint32_t qp[RMAX][4];
#pragma unroll
    for (int h = 0; h < RMAX; ++h) pack_q8(q8[h], qp[h]);
    // the new row's K / V share read once and selected per pass (persist_tk.hip: a per-pass LDS read under a branch
    // serialised the independent score chains)
    const uint4 knp = pack8f(&kn_s[li * 8]);
    float vn8[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) vn8[e] = vn_s[li * 8 + e];
#pragma unroll
    for (int pi = 0; pi < NP; ++pi) {
        const int j = j0 + pi * PPP + pg;
        ok[pi] = j <= pos;
#pragma unroll
        for (int h = 0; h < RMAX; ++h) {
            float s;
            if constexpr (Q3T_ATTN_DOT2) {   // score8 (q3t_common.h): identical in every single-slot attention kernel
                const uint4 kk = j == pos ? knp : kr[pi];
                s = score8(kk, qp[h]);
            } else {
                float k8[8];
                if (j == pos) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) k8[e] = kn_s[li * 8 + e];
                } else {
                    unpack8(kr[pi], k8);
                }
                s = 0.0f;
#pragma unroll
                for (int e = 0; e < 8; ++e) s = __fmaf_rn(k8[e], q8[h][e], s);   // explicit fma: identical in k_attn and persist.hip
            }
            s = group_sum<LPP>(s);
            sc[pi][h] = ok[pi] ? __fmul_rn(s, kq_scale) : -INFINITY;
        }
    }
    // ---- (4) chunk max / exp / sum per head (xor over the position bits of the wave, then LDS over waves)
    float M[RMAX], L[RMAX];
#pragma unroll
    for (int h = 0; h < RMAX; ++h) {
        float m = sc[0][h];
#pragma unroll
        for (int pi = 1; pi < NP; ++pi) m = fmaxf(m, sc[pi][h]);
        if constexpr (LPP == 16) m = rows_max(m);
        else
#pragma unroll
            for (int o = LPP; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        if (lane == 0) wred[wave][h] = m;
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < RMAX; ++h) M[h] = fmaxf(fmaxf(wred[0][h], wred[1][h]), fmaxf(wred[2][h], wred[3][h]));
    __syncthreads();
    float pr[NP][RMAX];
#pragma unroll
    for (int h = 0; h < RMAX; ++h) {
        float l = 0.0f;
#pragma unroll
        for (int pi = 0; pi < NP; ++pi) {
            pr[pi][h] = ok[pi] ? exp_sm(__fsub_rn(sc[pi][h], M[h])) : 0.0f;
            l += pr[pi][h];
        }
        if constexpr (LPP == 16) l = rows_sum(l);
        else
#pragma unroll
            for (int o = LPP; o < 64; o <<= 1) l += __shfl_xor(l, o, 64);
        if (lane == 0) wred[wave][h] = l;
    }
    // ---- (5) P.V over this lane's positions, reduced over the position groups
    float acc[RMAX][8];
#pragma unroll
    for (int h = 0; h < RMAX; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[h][e] = 0.0f;
#pragma unroll
    for (int pi = 0; pi < NP; ++pi) {
        const int j = j0 + pi * PPP + pg;
        float v8[8];
        unpack8(vr[pi], v8);
#pragma unroll
        for (int e = 0; e < 8; ++e) v8[e] = j == pos ? vn8[e] : v8[e];
#pragma unroll
        for (int h = 0; h < RMAX; ++h)
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[h][e] = __fmaf_rn(pr[pi][h], ok[pi] ? v8[e] : 0.0f, acc[h][e]);
    }
#pragma unroll
    for (int h = 0; h < RMAX; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float a = acc[h][e];
            if constexpr (LPP == 16) a = rows_sum(a);
            else
#pragma unroll
                for (int o = LPP; o < 64; o <<= 1) a += __shfl_xor(a, o, 64);
            if (lane < LPP && h < R) ared[wave][h][li * 8 + e] = a;
        }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < RMAX; ++h) L[h] = (wred[0][h] + wred[1][h]) + (wred[2][h] + wred[3][h]);

    const int RD = R * D;
    if (nsplit == 1) {
        for (int o = t; o < RD; o += 256) {
            const int h = o / D, d = o % D;
            const float a = (ared[0][h][d] + ared[1][h][d]) + (ared[2][h][d] + ared[3][h][d]);
            p.out[(size_t)slot * p.nH * D + (size_t)(g * R + h) * D + d] = f2h(a / L[h]);
            if (p.dbg && slot == 0 && g == 5 && R == 2) p.dbg[516 + o] = a / L[h];
        }
        if (p.dbg && slot == 0 && g == 5 && R == 2 && t < D) {
            p.dbg[t] = q_s[0][t]; p.dbg[128 + t] = q_s[1 % R][t]; p.dbg[256 + t] = kn_s[t]; p.dbg[384 + t] = vn_s[t];
            if (t == 0) { p.dbg[512] = M[0]; p.dbg[513] = M[1 % R]; p.dbg[514] = L[0]; p.dbg[515] = L[1 % R]; }
        }
        return;
    }
    // ---- (6) publish the partial with sc1 stores, take a ticket; the last arrival combines
    float *part = p.part + (((size_t)slot * p.nKV + g) * p.max_splits) * R * (D + 2);
    for (int o = t; o < RD; o += 256) {
        const int h = o / D, d = o % D;
        const float a = (ared[0][h][d] + ared[1][h][d]) + (ared[2][h][d] + ared[3][h][d]);
        st_sc1(part + ((size_t)split * R + h) * (D + 2) + d, a);
    }
    if (t < R) {
        st_sc1(part + ((size_t)split * R + t) * (D + 2) + D, M[t]);
        st_sc1(part + ((size_t)split * R + t) * (D + 2) + D + 1, L[t]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned *ticket = p.ticket + (size_t)slot * p.nKV + g;
    if (t == 0) last_s = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(nsplit - 1);
    __syncthreads();
    if (!last_s) return;
    // combine (the last arrival): every partial load is issued in parallel (sc1 loads, L2-served)
    for (int i = t; i < nsplit * R; i += 256) {
        const int s = i / R, h = i % R;
        sm[s][h] = ld_sc1(part + ((size_t)s * R + h) * (D + 2) + D);
        sl[s][h] = ld_sc1(part + ((size_t)s * R + h) * (D + 2) + D + 1);
    }
    __syncthreads();
    if (t < R) {
        float mx = -INFINITY;
        for (int s = 0; s < nsplit; ++s) mx = fmaxf(mx, sm[s][t]);
        float lt = 0.0f;
        for (int s = 0; s < nsplit; ++s) lt = __fmaf_rn(sl[s][t], expf(sm[s][t] - mx), lt);
        cm[t] = mx;
        cl[t] = lt;
    }
    __syncthreads();
    for (int i = t; i < nsplit * R; i += 256) {
        const int s = i / R, h = i % R;
        sw[s][h] = expf(sm[s][h] - cm[h]);
    }
    __syncthreads();
    for (int o = t; o < RD; o += 256) {
        const int h = o / D, d = o % D;
        float a = 0.0f;
        for (int s0 = 0; s0 < nsplit; s0 += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                v[u] = s0 + u < nsplit ? ld_sc1(part + ((size_t)(s0 + u) * R + h) * (D + 2) + d) : 0.0f;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (s0 + u < nsplit) a = __fmaf_rn(v[u], sw[s0 + u][h], a);
        }
        p.out[(size_t)slot * p.nH * D + (size_t)(g * R + h) * D + d] = f2h(a / cl[h]);
    }
    if (t == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------ batched: one workgroup per
// (slot, kv head) streaming the whole context.  At 64 slots the split grid (slot x kv x 64-position split, partials,
// tickets, last-arriver combine) ran at ~2.9 TB/s; here each workgroup walks its context in 64-position chunks with
// the next chunk's K/V loads in flight (register double buffer), and each wave keeps its own online-softmax state
// (max, sum, 8-dim accumulator per head) over its 16 positions of every chunk, so no barrier is taken per chunk; the
// four waves merge once at the end.  The per-position arithmetic differs from k_attn's in summation order (dot2 pairs)
// and exponential (v_exp_f32), the rescaling order of the online softmax from the split combine (f32): the batched
// family is checked against the oracle (teacher-forced decisions), not bit for bit against the single-slot kernels.
//
// The kernel is issue-bound, not HBM-bound (one wave per SIMD saw every instruction's latency): scores are
// v_dot2_f32_f16 on the packed K registers, softmax exponentials v_exp_f32 (__expf), and every chunk but the
// last is whole (all 64 positions <= pos), so it runs without position masks, without the new-row branch and without
// the empty-wave test; the new K/V row (pos) is patched into the last chunk's registers once, from LDS (exact: the
// LDS copy is the f16 value).
#ifndef Q3T_ATTN_SEQ_MINB
#define Q3T_ATTN_SEQ_MINB 2
#endif
#ifndef Q3T_ATTN_SEQ_NB
#define Q3T_ATTN_SEQ_NB 2   // K/V ring depth (attn_seq.h)
#endif
template <int D, int R>
__global__ void __launch_bounds__(256, Q3T_ATTN_SEQ_MINB) k_attn_seq(const AttnParams p) {
    static_assert(D == 128 && R == 2, "talker heads: D 128, 2 q heads per kv head (attn_seq.h)");
    __shared__ AttnSeqLds L;
    const int slot = blockIdx.x, g = blockIdx.y, lane = threadIdx.x & 63;
    const int pos = p.pos[slot];
    const size_t head_off = ((size_t)slot * p.nKV + g) * p.n_ctx * D;
    const float *qkv = p.qkv + (size_t)slot * (p.nH + 2 * p.nKV) * D;
    attn_seq_wg<false, Q3T_ATTN_SEQ_NB>(
        pos, p.kc + head_off, p.vc + head_off, p.rope + (size_t)pos * D, p.qn, p.kn, p.eps,
        [&](int v, float (&x)[2]) {
            const float *src = v == R + 1 ? qkv + (size_t)(p.nH + p.nKV + g) * D
                             : v == R     ? qkv + (size_t)(p.nH + g) * D
                                          : qkv + (size_t)(g * R + v) * D;
            x[0] = src[lane];
            x[1] = src[lane + 64];
        },
        [&](int h, int d, float y) { p.out[(size_t)slot * p.nH * D + (size_t)(g * R + h) * D + d] = f2h(y); }, L);
}


// ------------------------------------------------------------------------------------------ batched code predictor:
// <= 16 positions, one wave per (slot, kv head) (attn_small.h, shared with the persistent batched frame)
template <int D, int R>
__global__ void __launch_bounds__(64) k_attn_small(const AttnParams p) {
    static_assert(D == 128 && R == 2, "code-predictor heads: D 128, 2 q heads per kv head");
    const int slot = blockIdx.x, g = blockIdx.y;
    __shared__ AttnSmallLds L;
    const int pos = p.pos[slot];
    const size_t head_off = ((size_t)slot * p.nKV + g) * p.n_ctx * D;
    const int QKV = (p.nH + 2 * p.nKV) * D;
    const float *qkv = p.qkv_tab ? p.qkv_tab + (p.tab_row0 + (size_t)p.tab_tok[(size_t)slot * p.tab_ld + p.tab_col]) * QKV
                                 : p.qkv + (size_t)slot * QKV;
    attn_small_wave<false>(g, pos, p.nH, p.nKV, qkv, p.qn, p.kn, p.eps, p.rope + (size_t)pos * D, p.kc + head_off,
                           p.vc + head_off, p.out + (size_t)slot * p.nH * D, L);
}

// ------------------------------------------------------------------ causal prefill attention
// build_prefill_forward_graph (src/tts_transformer.cpp:1233-1374): every prompt row of an utterance in one pass --
// q / k head RMSNorm + NEOX RoPE at the row's position, the F16 K/V rows appended to the cache, explicit KQ, scale,
// diag_mask_inf, soft_max and KQV per row.  One workgroup per (utterance, kv head) holds the utterance's <= 16 rows of
// that head group in LDS; the head-norm / RoPE prologue is k_attn's (one wave per vector, the same roundings).
// 512 threads: the 64 prologue vectors and 32 (row, head) tasks of a 16-row prompt spread over 8 waves (at one
// workgroup per kv head, 4 waves ran them as a serial chain: 16 us per layer).
__device__ __forceinline__ float tree16(const float (&v)[16]) {
    float a[8], b[4];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = v[2 * k] + v[2 * k + 1];
#pragma unroll
    for (int k = 0; k < 4; ++k) b[k] = a[2 * k] + a[2 * k + 1];
    return (b[0] + b[1]) + (b[2] + b[3]);
}
constexpr int PF_THREADS = 512;
template <int D, int R>
__global__ void __launch_bounds__(PF_THREADS) k_prefill_attn(const PrefillAttnParams p) {
    constexpr int PMAX = PREFILL_MAX_ROWS, E = D / 64, LPP = D / 8, GROUPS = PF_THREADS / LPP, NW = PF_THREADS / 64;
    static_assert(PMAX == 16, "tree16: the decode kernel's first 16 positions");
    __shared__ float q_s[PMAX][R][D];
    __shared__ float k_s[PMAX][D], v_s[PMAX][D];
    const int u = blockIdx.x, g = blockIdx.y, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int plen = p.plen, QKV = (p.nH + 2 * p.nKV) * D;
    const size_t head_off = ((size_t)p.slot[u] * p.nKV + g) * p.n_ctx * D;
    // ---- prologue: vectors (row i, v) with v < R the q heads, v == R the k row, v == R + 1 the v row; task
    // wave + NW k.  Every operand of the wave's tasks is loaded first (one memory round trip instead of one per task:
    // with one workgroup per kv head the serial loads were ~17 us of an 18 us launch)
    constexpr int MAXT = (PMAX * (R + 2) + NW - 1) / NW;
    const int ntask = plen * (R + 2);
    float xv[MAXT][E], rc[MAXT], rs[MAXT], qw[E], kw[E];
#pragma unroll
    for (int e = 0; e < E; ++e) { qw[e] = p.qn[lane + 64 * e]; kw[e] = p.kn[lane + 64 * e]; }
#pragma unroll
    for (int k = 0; k < MAXT; ++k) {
        const int task = wave + NW * k;
        rc[k] = rs[k] = 0.0f;
#pragma unroll
        for (int e = 0; e < E; ++e) xv[k][e] = 0.0f;
        if (task < ntask) {
            const int i = task / (R + 2), v = task % (R + 2);
            const float *qkv = p.qkv + (size_t)(u * plen + i) * QKV;
            const float *src = v == R + 1 ? qkv + (size_t)(p.nH + p.nKV + g) * D : v == R ? qkv + (size_t)(p.nH + g) * D : qkv + (size_t)(g * R + v) * D;
#pragma unroll
            for (int e = 0; e < E; ++e) xv[k][e] = src[lane + 64 * e];
            const float *rope = p.rope + (size_t)i * D;
            const int ri = D == 128 ? lane : (lane & 31);
            rc[k] = rope[2 * ri];
            rs[k] = rope[2 * ri + 1];
        }
    }
#pragma unroll
    for (int k = 0; k < MAXT; ++k) {
        const int task = wave + NW * k;
        if (task >= ntask) break;
        const int i = task / (R + 2), v = task % (R + 2);
        if (v == R + 1) {
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const float y = f16r(xv[k][e]);
                v_s[i][lane + 64 * e] = y;
                p.vc[head_off + (size_t)i * D + lane + 64 * e] = f2h(y);
            }
            continue;
        }
        const bool isk = v == R;
        float x[E];
        double ss = 0.0;
#pragma unroll
        for (int e = 0; e < E; ++e) { x[e] = xv[k][e]; ss += (double)__fmul_rn(x[e], x[e]); }
        ss = wave_sum_d(ss);
        const float scale = 1.0f / sqrtf((float)(ss / D) + p.eps);
#pragma unroll
        for (int e = 0; e < E; ++e) x[e] = (x[e] * scale) * (isk ? kw[e] : qw[e]);
        float y[E];
        if constexpr (D == 128) {
            const float c = rc[k], sn = rs[k];
            y[0] = opaque(opaque(x[0] * c) - opaque(x[1] * sn));
            y[1] = opaque(opaque(x[0] * sn) + opaque(x[1] * c));
        } else {
            const float c = rc[k], sn = rs[k];
            const float other = __shfl_xor(x[0], 32, 64);
            y[0] = lane < 32 ? x[0] * c - other * sn : other * sn + x[0] * c;
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const float r = f16r(y[e]);
            if (isk) {
                k_s[i][lane + 64 * e] = r;
                p.kc[head_off + (size_t)i * D + lane + 64 * e] = f2h(r);
            } else {
                q_s[i][v][lane + 64 * e] = r;
            }
        }
    }
    __syncthreads();
    // ---- attention: one LPP-lane group per (row i, head h); lane li holds dims li*8 .. li*8+7.  Row i < 16 lies in
    // the first 64-position chunk of the decode kernel, and the sums below are k_attn's reduction tree over that
    // chunk's 16 leading positions (pairs of neighbours, then pairs of pairs ...; masked positions add +0), so every
    // prefill row equals the decode step replayed at its position bit for bit.
    const float kq_scale = 1.0f / sqrtf((float)D);
    const int grp = t / LPP, li = t % LPP;
    for (int task = grp; task < plen * R; task += GROUPS) {
        const int i = task / R, h = task % R;
        float q8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) q8[e] = q_s[i][h][li * 8 + e];
        uint32_t qp[4];
        pack_q8(q8, qp);
        float sc[PMAX];
        float m = -INFINITY;
#pragma unroll
        for (int j = 0; j < PMAX; ++j) {   // rows j >= plen hold stale LDS: computed, then masked
            float d = 0.0f;
            if constexpr (Q3T_ATTN_DOT2) {
                d = score8(pack8f(&k_s[j][li * 8]), qp);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) d = __fmaf_rn(k_s[j][li * 8 + e], q8[e], d);
            }
            d = group_sum<LPP>(d);
            sc[j] = j <= i ? __fmul_rn(d, kq_scale) : -INFINITY;
            m = fmaxf(m, sc[j]);
        }
        float pj[PMAX];
#pragma unroll
        for (int j = 0; j < PMAX; ++j) pj[j] = j <= i ? exp_sm(__fsub_rn(sc[j], m)) : 0.0f;
        const float l = tree16(pj);
        uint16_t *o = p.out + (size_t)(u * plen + i) * p.nH * D + (size_t)(g * R + h) * D + li * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float pv[PMAX];
#pragma unroll
            for (int j = 0; j < PMAX; ++j)   // k_attn's fma onto 0, then + 0 from its masked passes (-0 -> +0)
                pv[j] = j <= i ? __fadd_rn(__fmaf_rn(pj[j], v_s[j][li * 8 + e], 0.0f), 0.0f) : 0.0f;
            o[e] = f2h(tree16(pv) / l);
        }
    }
}

bool prefill_attn(const PrefillAttnParams &p, hipStream_t s) {
    if (p.n_utt <= 0) return true;
    if (p.plen < 1 || p.plen > PREFILL_MAX_ROWS || p.nKV <= 0 || p.nH % p.nKV != 0 || !p.qkv || !p.slot || !p.kc || !p.vc ||
        !p.out || !p.rope) {
        set_error("prefill_attn: bad parameters");
        return false;
    }
    const dim3 grid(p.n_utt, p.nKV);
    const int R = p.nH / p.nKV;
#define Q3T_PF_LAUNCH(DD, RR) hipLaunchKernelGGL((k_prefill_attn<DD, RR>), grid, dim3(PF_THREADS), 0, s, p)
    if (p.D == 128 && R == 2) Q3T_PF_LAUNCH(128, 2);
    else if (p.D == 128 && R == 1) Q3T_PF_LAUNCH(128, 1);
    else if (p.D == 128 && R == 4) Q3T_PF_LAUNCH(128, 4);
    else if (p.D == 64 && R == 2) Q3T_PF_LAUNCH(64, 2);
    else if (p.D == 64 && R == 1) Q3T_PF_LAUNCH(64, 1);
    else if (p.D == 64 && R == 4) Q3T_PF_LAUNCH(64, 4);
    else { set_error("prefill_attn: unsupported head layout"); return false; }
#undef Q3T_PF_LAUNCH
    Q3T_HIP(hipGetLastError());
    return true;
}

bool attn_decode(const AttnParams &p, hipStream_t s) {
    if (p.small) {
        if (p.n_ctx > 16 || p.D != 128 || p.nH != 2 * p.nKV) { set_error("attn_decode: small-context attention needs n_ctx <= 16, D 128, 2 q heads per kv head"); return false; }
        hipLaunchKernelGGL((k_attn_small<128, 2>), dim3(p.S, p.nKV), dim3(64), 0, s, p);
        Q3T_HIP(hipGetLastError());
        return true;
    }
    if (p.seqk && p.D == 128 && p.nH == 2 * p.nKV) {
        hipLaunchKernelGGL((k_attn_seq<128, 2>), dim3(p.S, p.nKV), dim3(256), 0, s, p);
        Q3T_HIP(hipGetLastError());
        return true;
    }
    if (p.nH % p.nKV != 0 || p.nH / p.nKV > 4 || (p.D != 64 && p.D != 128)) {
        set_error("attn_decode: unsupported head layout");
        return false;
    }
    if ((p.chunk != 64 && p.chunk != 128) || p.max_splits * p.chunk < p.n_ctx || p.max_splits > ATTN_MAX_SPLITS || !p.part || !p.ticket) {
        set_error("attn_decode: split buffers too small");
        return false;
    }
    const dim3 grid(p.S, p.nKV, p.max_splits);
    const int R = p.nH / p.nKV;
#define Q3T_ATTN_LAUNCH(DD, RR)                                                                      \
    do {                                                                                             \
        if (p.chunk == 128) hipLaunchKernelGGL((k_attn<DD, RR, 128>), grid, dim3(256), 0, s, p);     \
        else hipLaunchKernelGGL((k_attn<DD, RR, 64>), grid, dim3(256), 0, s, p);                     \
    } while (0)
    if (p.D == 128) {
        if (R == 1) Q3T_ATTN_LAUNCH(128, 1);
        else if (R == 2) Q3T_ATTN_LAUNCH(128, 2);
        else if (R == 4) Q3T_ATTN_LAUNCH(128, 4);
        else { set_error("attn_decode: q/kv head ratio must be 1, 2 or 4"); return false; }
    } else {
        if (R == 1) Q3T_ATTN_LAUNCH(64, 1);
        else if (R == 2) Q3T_ATTN_LAUNCH(64, 2);
        else if (R == 4) Q3T_ATTN_LAUNCH(64, 4);
        else { set_error("attn_decode: q/kv head ratio must be 1, 2 or 4"); return false; }
    }
#undef Q3T_ATTN_LAUNCH
    Q3T_HIP(hipGetLastError());
    return true;
}

}  // namespace q3t
