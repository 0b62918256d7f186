// attn_small.h — the batched code predictor's attention of ONE (slot, kv head) on ONE wave: <= 16 positions
// (scripts/export_code_predictor.py:132-231 step semantics; src/tts_transformer.cpp:2153-2340 as the ggml graph).
// Shared source of k_attn_small (attn.hip, one launch per layer) and the persistent batched code-predictor frame
// (persist_cpb.hip), so both compute the same bits.
//
// The cached K/V rows do not depend on this step's QKV row, so they are loaded first; then the head RMSNorm + NEOX RoPE
// of the 2 q heads and the new k (k_attn arithmetic), the F16 KV append, scores with one lane pair per (head, position)
// over 64 dims each, the softmax per head and P.V with four output dims per lane.
//
// SC1 = false: the kernel form (plain loads; a workgroup of one wave, so __syncthreads is the LDS fence).
// SC1 = true: inside a persistent launch -- the QKV row and the cached K/V rows are read with agent-scope (sc1) loads
// (written in this launch, by other CUs or by this CU in an earlier pass: no stale L1 line), the output is stored with
// 8-byte sc1 stores, and the LDS fence is the wave's own (lgkmcnt(0) + wave barrier: every LDS word here is written and
// read by the same wave).
#pragma once
#include "kernels.h"

#pragma clang fp contract(off)   // every rounding as written (both includers compile with contraction off too)

namespace q3t {

struct AttnSmallLds {
    float q_s[2][128];
    alignas(16) uint16_t kh_s[128];
    alignas(16) uint16_t vh_s[128];
    float pr_s[2][16];
    float l_s[2];
};

namespace asm_detail {
template <bool SC1>
__device__ __forceinline__ uint4 ld_k16(const uint16_t *p) {
    if constexpr (SC1) {
        const uint64_t *q = reinterpret_cast<const uint64_t *>(p);
        const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    } else {
        typedef const __attribute__((address_space(1))) u32x4_t gv;
        const u32x4_t v = *(gv *)p;
        return make_uint4(v.x, v.y, v.z, v.w);
    }
}
template <bool SC1>
__device__ __forceinline__ uint2 ld_v8(const uint16_t *p) {
    if constexpr (SC1) {
        const uint64_t a = __hip_atomic_load(reinterpret_cast<const uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return make_uint2((uint32_t)a, (uint32_t)(a >> 32));
    } else {
        return *reinterpret_cast<const uint2 *>(p);
    }
}
template <bool SC1>
__device__ __forceinline__ float ld_f(const float *p) {
    if constexpr (SC1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
template <bool SC1>
__device__ __forceinline__ void lds_fence() {
    if constexpr (SC1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    } else {
        __syncthreads();
    }
}
// the value as rounded by the f16 conversion and back (attn.hip unpack8_cvt: the consumer fma may not absorb the
// conversion)
__device__ __forceinline__ void unpack8_cvt(const uint4 u, float (&f)[8]) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) { f[2 * e] = opaque(h2f(w[e] & 0xffff)); f[2 * e + 1] = opaque(h2f(w[e] >> 16)); }
}
}  // namespace asm_detail

// The cached K / V rows one lane needs (positions < pos; the new row comes from LDS): they do not depend on this step's
// QKV row, so a caller issues them before it waits for that row
struct AttnSmallKV {
    uint4 kr[8];
    uint2 vr[16];
};
template <bool SC1>
__device__ __forceinline__ void attn_small_load_kv(int pos, const uint16_t *kc, const uint16_t *vc, AttnSmallKV &kv) {
    using namespace asm_detail;
    constexpr int D = 128, NPOS = 16;
    const int lane = threadIdx.x & 63;
    const int sj = (lane >> 1) & 15, sk = lane & 1, vd = (lane & 31) * 4;
    const int jk = min(sj, max(pos - 1, 0));
#pragma unroll
    for (int e = 0; e < 8; ++e) kv.kr[e] = ld_k16<SC1>(kc + (size_t)jk * D + sk * 64 + e * 8);
#pragma unroll
    for (int j = 0; j < NPOS; ++j) {
        const int jv = min(j, max(pos - 1, 0));
        kv.vr[j] = ld_v8<SC1>(vc + (size_t)jv * D + vd);
    }
}

// the lane's per-layer / per-position operands: RoPE (cos, sin) of its dimension pair, q / k head-norm weights
struct AttnSmallAux {
    float c, sn, qw0, qw1, kw0, kw1;
};
__device__ __forceinline__ void attn_small_load_aux(const float *rope_row, const float *qn, const float *kn, AttnSmallAux &a) {
    const int lane = threadIdx.x & 63;
    a.c = rope_row[2 * lane];
    a.sn = rope_row[2 * lane + 1];
    a.qw0 = qn[lane];
    a.qw1 = qn[lane + 64];
    a.kw0 = kn[lane];
    a.kw1 = kn[lane + 64];
}

// lane's share of the raw QKV values of kv group g: xs[v][e] = element lane + 64 e of q head 2g (v 0), q head 2g+1 (1),
// k (2), v (3) of the slot's Q | K | V row ((nH + 2 nKV) * D f32: the QKV projection, or the per-token table row)
__device__ __forceinline__ int attn_small_src(int g, int v, int nH, int nKV) {
    constexpr int D = 128, R = 2;
    return v < R ? (g * R + v) * D : v == R ? (nH + g) * D : (nH + nKV + g) * D;
}
template <bool SC1>
__device__ __forceinline__ void attn_small_load_qkv(const float *qkv, int g, int nH, int nKV, float (&xs)[4][2]) {
    using namespace asm_detail;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const float *src = qkv + attn_small_src(g, v, nH, nKV);
        xs[v][0] = ld_f<SC1>(src + lane);
        xs[v][1] = ld_f<SC1>(src + lane + 64);
    }
}

// One (slot, kv head g) of the code predictor's attention at position pos (< 16), 2 q heads of D = 128, from the cached
// rows `kv` (attn_small_load_kv) and the raw QKV values `xs` (attn_small_load_qkv).
//   kc/vc: this (layer, slot, kv head)'s cache [16][D] f16; dst_of(e): where halves e .. e+3 (e a multiple of 4) of the
//   slot's attention row [nH * D] f16 go
struct AttnNoStamp {   // development timeline hook of attn_small_compute (persist_cpb.hip stamps)
    __device__ void operator()(int) const {}
};
template <bool SC1, class Dst, class Stamp = AttnNoStamp>
__device__ __forceinline__ void attn_small_compute(AttnSmallKV &kvr, const float (&xs)[4][2], const AttnSmallAux &aux, int g,
                                                   int pos, float eps, uint16_t *kc, uint16_t *vc, Dst dst_of,
                                                   AttnSmallLds &L, Stamp stamp = Stamp()) {
    using namespace asm_detail;
    constexpr int D = 128, R = 2, NPOS = 16;
    const int lane = threadIdx.x & 63;
    // score lanes: head sh, position sj, K half sk (64 dims); P.V lanes: head vh, dims vd .. vd+3
    const int sh = lane >> 5, sj = (lane >> 1) & 15, sk = lane & 1;
    const int vh = lane >> 5, vd = (lane & 31) * 4;
    uint4 (&kr)[8] = kvr.kr;
    uint2 (&vr)[NPOS] = kvr.vr;
    // head RMSNorm + NEOX RoPE of the 2 q heads and the new k, the new v f16-rounded (k_attn arithmetic)
    const float c = aux.c, sn = aux.sn;
#pragma unroll
    for (int v = 0; v < R + 1; ++v) {
        const float w0 = v == R ? aux.kw0 : aux.qw0, w1 = v == R ? aux.kw1 : aux.qw1;
        double ss = (double)__fmul_rn(xs[v][0], xs[v][0]) + (double)__fmul_rn(xs[v][1], xs[v][1]);
        ss = wave_sum_d(ss);
        const float scale = 1.0f / sqrtf((float)(ss / D) + eps);
        const float x0 = (xs[v][0] * scale) * w0, x1 = (xs[v][1] * scale) * w1;
        const float y0 = opaque(opaque(x0 * c) - opaque(x1 * sn));
        const float y1 = opaque(opaque(x0 * sn) + opaque(x1 * c));
        if (v == R) {
            L.kh_s[lane] = f2h(y0);
            L.kh_s[lane + 64] = f2h(y1);
        } else {
            L.q_s[v][lane] = f16r(y0);
            L.q_s[v][lane + 64] = f16r(y1);
        }
    }
    L.vh_s[lane] = f2h(xs[R + 1][0]);
    L.vh_s[lane + 64] = f2h(xs[R + 1][1]);
    stamp(0);
    lds_fence<SC1>();
    stamp(1);
    kc[(size_t)pos * D + lane] = L.kh_s[lane];
    kc[(size_t)pos * D + lane + 64] = L.kh_s[lane + 64];
    vc[(size_t)pos * D + lane] = L.vh_s[lane];
    vc[(size_t)pos * D + lane + 64] = L.vh_s[lane + 64];
    // scores: the new row from LDS, cached rows from registers
    if (sj == pos) {
#pragma unroll
        for (int e = 0; e < 8; ++e) kr[e] = *reinterpret_cast<const uint4 *>(&L.kh_s[sk * 64 + e * 8]);
    }
    float s = 0.0f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        float k8[8];
        unpack8_cvt(kr[e], k8);
#pragma unroll
        for (int u = 0; u < 8; ++u) s = __fmaf_rn(k8[u], L.q_s[sh][sk * 64 + e * 8 + u], s);
    }
    s += __shfl_xor(s, 1);
    const float kq_scale = 1.0f / sqrtf((float)D);
    const float sc = sj <= pos ? __fmul_rn(s, kq_scale) : -INFINITY;
    const float mx = group_max<32>(sc);
    const float pv = sj <= pos ? expf(__fsub_rn(sc, mx)) : 0.0f;
    const float lsum = group_sum<32>(sk == 0 ? pv : 0.0f);
    if (sk == 0) L.pr_s[sh][sj] = pv;
    if ((lane & 31) == 0) L.l_s[sh] = lsum;
    stamp(2);
    lds_fence<SC1>();
    stamp(3);
    // P.V: the new row from LDS
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NPOS; ++j) {   // positions 0..pos in order (a guard, not a break: j stays a constant, vr in registers)
        if (j <= pos) {
            const uint2 u = j == pos ? *reinterpret_cast<const uint2 *>(&L.vh_s[vd]) : vr[j];
            const float pj = L.pr_s[vh][j];
            acc[0] = __fmaf_rn(pj, h2f(u.x & 0xffff), acc[0]);
            acc[1] = __fmaf_rn(pj, h2f(u.x >> 16), acc[1]);
            acc[2] = __fmaf_rn(pj, h2f(u.y & 0xffff), acc[2]);
            acc[3] = __fmaf_rn(pj, h2f(u.y >> 16), acc[3]);
        }
    }
    const float l = L.l_s[vh];
    uint2 o;
    o.x = (uint32_t)f2h(acc[0] / l) | ((uint32_t)f2h(acc[1] / l) << 16);
    o.y = (uint32_t)f2h(acc[2] / l) | ((uint32_t)f2h(acc[3] / l) << 16);
    uint16_t *dst = dst_of((g * R + vh) * D + vd);
    if constexpr (SC1) {
        __hip_atomic_store(reinterpret_cast<uint64_t *>(dst), ((uint64_t)o.y << 32) | o.x, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *reinterpret_cast<uint2 *>(dst) = o;
    }
}

template <bool SC1>
__device__ __forceinline__ void attn_small_wave(int g, int pos, int nH, int nKV, const float *qkv, const float *qn,
                                                const float *kn, float eps, const float *rope_row, uint16_t *kc,
                                                uint16_t *vc, uint16_t *out, AttnSmallLds &L) {
    AttnSmallKV kv;
    attn_small_load_kv<SC1>(pos, kc, vc, kv);
    float xs[4][2];
    attn_small_load_qkv<SC1>(qkv, g, nH, nKV, xs);
    AttnSmallAux aux;
    attn_small_load_aux(rope_row, qn, kn, aux);
    attn_small_compute<SC1>(kv, xs, aux, g, pos, eps, kc, vc, [&](int e) { return out + e; }, L);
}

}  // namespace q3t
