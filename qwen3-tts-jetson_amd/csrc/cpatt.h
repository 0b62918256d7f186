// cpatt.h — the code predictor's attention for one new token over its <= 16-position F16 cache, computed by EVERY
// workgroup that needs the attention output (device code shared by gemv.hip's PRO_CPATT prologue and persist.hip's
// code-predictor frame, so both produce the same bits).  Semantics: scripts/export_code_predictor.py:132-231 /
// src/tts_transformer.cpp:1514-1827 step graph: q / k head RMSNorm (double sums), NEOX RoPE from the host (cos, sin)
// table, f16-rounded q / k / v, softmax(q k^T / sqrt(D)) with expf, f16-rounded output [16 heads][128].
//
// Register layout of the raw QKV row: thread t holds elements i*1024 + 4t .. +3 (i < 4): q head t/32, q head 8 + t/32,
// k head t/32, v head t/32, dims 4(t%32) .. +3 -- one head per 32-lane half-wave.
#pragma once
#include "kernels.h"

namespace q3t {

constexpr int CPA_POS = 16, CPA_NKV = 8, CPA_NH = 16, CPA_D = 128;
constexpr size_t CPA_LDS = (size_t)CPA_NH * CPA_D * 2 + (size_t)CPA_POS * CPA_NKV * CPA_D * 2 + CPA_NKV * CPA_D * 2 +
                           CPA_NH * CPA_POS * 4 + CPA_NH * 4;
constexpr size_t CPA_LDS_VL = CPA_LDS + (size_t)CPA_POS * CPA_NKV * CPA_D * 2;   // + the V cache staged in LDS (VL)

struct CpAttRegs {
    float4 raw[4], qn, kn, rc[2];
    uint4 kk[8], vv[16];
    int pos;
};

template <class V>
__device__ __forceinline__ V cpa_ldg(const void *p) {
    typedef const __attribute__((address_space(1))) V gV;
    return *(gV *)(p);
}
// SC1: agent-scope loads (two 8-B halves) -- cache rows written earlier in the same launch by another workgroup
template <bool SC1>
__device__ __forceinline__ uint4 cpa_ld16(const uint16_t *p) {
    if constexpr (SC1) {
        uint64_t *q = reinterpret_cast<uint64_t *>(const_cast<uint16_t *>(p));
        const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    } else {
        const u32x4_t v = cpa_ldg<u32x4_t>(p);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
}
__device__ __forceinline__ float4 cpa_ldf4(const float *p) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v v = cpa_ldg<f4v>(p);
    return make_float4(v.x, v.y, v.z, v.w);
}

// the cached K / V rows of the slot ([8 kv][16 pos][128] f16 each; all 16 positions, masked later).
// VL = false: V as the P.V owner's 16 rows in registers (vv[0..15]); VL = true: V in K's chunk layout (vv[0..7]), to be
// staged in LDS by cpatt_stage_kv (half the registers: the persistent frame holds them across phases)
template <bool SC1, bool VL = false>
__device__ __forceinline__ void cpatt_issue_kv(const uint16_t *kc, const uint16_t *vc, CpAttRegs &a) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 8; ++i) {   // K chunk c = i*256 + t: [j][g][d0..d0+7], j = c/128, g = (c/16)%8, d0 = 8(c%16)
        const int c = i * 256 + t, j = c >> 7, g = (c >> 4) & 7, d0 = (c & 15) * 8;
        a.kk[i] = cpa_ld16<SC1>(kc + ((size_t)g * CPA_POS + j) * CPA_D + d0);
        if constexpr (VL) a.vv[i] = cpa_ld16<SC1>(vc + ((size_t)g * CPA_POS + j) * CPA_D + d0);
    }
    if constexpr (!VL) {
        const int h = t >> 4, g = h >> 1, d0 = (t & 15) * 8;   // P.V ownership: head h, dims d0 .. d0+7
#pragma unroll
        for (int j = 0; j < CPA_POS; ++j) a.vv[j] = cpa_ld16<SC1>(vc + ((size_t)g * CPA_POS + j) * CPA_D + d0);
    }
}
// the cached K rows (and with VL the V rows) of every position except pos -> the LDS scratch; the caller orders these
// writes before cpatt_compute's reads with a workgroup barrier
template <bool VL>
__device__ __forceinline__ void cpatt_stage_kv(const CpAttRegs &a, int pos, uint8_t *scratch) {
    const int t = threadIdx.x;
    uint16_t *kf = reinterpret_cast<uint16_t *>(scratch) + CPA_NH * CPA_D;
    uint16_t *vf = reinterpret_cast<uint16_t *>(scratch + CPA_LDS);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int c = i * 256 + t, j = c >> 7;
        if (j != pos) {
            *reinterpret_cast<uint4 *>(kf + (size_t)c * 8) = a.kk[i];
            if constexpr (VL) *reinterpret_cast<uint4 *>(vf + (size_t)c * 8) = a.vv[i];
        }
    }
}
// head-norm weights and the RoPE (cos, sin) pairs of position pos
__device__ __forceinline__ void cpatt_issue_par(const float *qn, const float *kn, const float *rope, int pos, CpAttRegs &a) {
    const int l = threadIdx.x & 31;
    a.pos = pos;
    a.qn = cpa_ldf4(qn + 4 * l);
    a.kn = cpa_ldf4(kn + 4 * l);
    const float *rp = rope + (size_t)pos * CPA_D + 8 * (l & 15);
    a.rc[0] = cpa_ldf4(rp);
    a.rc[1] = cpa_ldf4(rp + 4);
}
__device__ __forceinline__ uint2 cpa_pack4(float a, float b, float c, float d) {
    uint2 h;
    h.x = (uint32_t)f2h(a) | ((uint32_t)f2h(b) << 16);
    h.y = (uint32_t)f2h(c) | ((uint32_t)f2h(d) << 16);
    return h;
}
__device__ __forceinline__ void cpa_store8(uint16_t *p, uint2 v, bool sc1) {
    if (sc1) {   // write-through: read by other workgroups of the same launch in later passes
        __hip_atomic_store(reinterpret_cast<uint64_t *>(p), ((uint64_t)v.y << 32) | v.x, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *reinterpret_cast<uint2 *>(p) = v;
    }
}

// the attention output of the new token -> xrow (LDS f16 [16][128]).  kc_w / vc_w: the slot's cache where this
// workgroup appends the new K / V row at a.pos (null: no append); valid = false zeroes the output (padding slot).
// scratch: CPA_LDS bytes of LDS (VL: CPA_LDS_VL, the cached rows already staged by cpatt_stage_kv<true>).  Ends with a
// workgroup barrier.  V read from LDS or from registers: the same values, so VL changes no bit of the result.
template <bool SC1_STORE, bool VL = false>
__device__ __forceinline__ void cpatt_compute(const CpAttRegs &a, float eps, uint16_t *kc_w, uint16_t *vc_w, bool valid,
                                              uint16_t *xrow, uint8_t *scratch) {
#pragma clang fp contract(off)   // every rounding as written: the same bits in every translation unit
    const int t = threadIdx.x, l = t & 31, hw = t >> 5;
    uint16_t *qf = reinterpret_cast<uint16_t *>(scratch);                  // [16][128]
    uint16_t *kf = qf + CPA_NH * CPA_D;                                    // [16 pos][8][128]
    uint16_t *vcur = kf + CPA_POS * CPA_NKV * CPA_D;                       // [8][128]
    float *sc = reinterpret_cast<float *>(vcur + CPA_NKV * CPA_D);         // [16][16]
    float *lsum = sc + CPA_NH * CPA_POS;                                   // [16]
    const uint16_t *vf = reinterpret_cast<const uint16_t *>(scratch + CPA_LDS);   // VL: [16 pos][8][128]
    const int pos = a.pos;
    // ---- head RMSNorm (q heads hw, 8+hw; k head hw) + NEOX RoPE, f16-rounded
    float y[3][4];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float4 v = a.raw[i];
        const float x[4] = {v.x, v.y, v.z, v.w};
        double ss = (double)(x[0] * x[0]) + (double)(x[1] * x[1]) + (double)(x[2] * x[2]) + (double)(x[3] * x[3]);
        ss += dpp_d<DPP_XOR1>(ss);   // all-reduce over the 32-lane half-wave that holds this head
        ss += dpp_d<DPP_XOR2>(ss);
        ss += dpp_d<DPP_HALF_MIRROR>(ss);
        ss += dpp_d<DPP_MIRROR>(ss);
        ss += xrow16_d(ss);
        const float scale = 1.0f / sqrtf((float)(ss / CPA_D) + eps);
        const float4 w = i < 2 ? a.qn : a.kn;
        const float w4[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) y[i][e] = (x[e] * scale) * w4[e];
    }
    const float cs[8] = {a.rc[0].x, a.rc[0].y, a.rc[0].z, a.rc[0].w, a.rc[1].x, a.rc[1].y, a.rc[1].z, a.rc[1].w};
    const bool lo = l < 16;   // dims 4l.. < 64 pair with the partner lane's dims + 64
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float o4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float mine = y[i][e], other = xrow16(mine);
            const float c = cs[2 * e], s = cs[2 * e + 1];
            o4[e] = f16r(lo ? mine * c - other * s : other * s + mine * c);
        }
        const uint2 hv = cpa_pack4(o4[0], o4[1], o4[2], o4[3]);
        if (i < 2) *reinterpret_cast<uint2 *>(qf + (i * 8 + hw) * CPA_D + 4 * l) = hv;
        else {
            *reinterpret_cast<uint2 *>(kf + ((size_t)pos * CPA_NKV + hw) * CPA_D + 4 * l) = hv;
            if (valid && kc_w) cpa_store8(kc_w + ((size_t)hw * CPA_POS + pos) * CPA_D + 4 * l, hv, SC1_STORE);
        }
    }
    {
        const float4 v = a.raw[3];
        const uint2 hv = cpa_pack4(v.x, v.y, v.z, v.w);
        *reinterpret_cast<uint2 *>(vcur + hw * CPA_D + 4 * l) = hv;
        if (valid && vc_w) cpa_store8(vc_w + ((size_t)hw * CPA_POS + pos) * CPA_D + 4 * l, hv, SC1_STORE);
    }
    if constexpr (!VL) cpatt_stage_kv<false>(a, pos, scratch);
    __syncthreads();
    // ---- scores: thread = (head h, position j)
    {
        const int h = t >> 4, j = t & 15, g = h >> 1;
        const uint16_t *qh = qf + h * CPA_D, *kj = kf + ((size_t)j * CPA_NKV + g) * CPA_D;
        float acc = 0.0f;
        // chunk order rotated by j: the 16 lanes of a head read 16 different 16-B chunks of their 2-KB-strided K
        // rows (no LDS bank conflicts)
#pragma unroll
        for (int c = 0; c < CPA_D / 8; ++c) {
            const int d = ((c + j) & (CPA_D / 8 - 1)) * 8;
            acc = dot8(*reinterpret_cast<const uint4 *>(qh + d), *reinterpret_cast<const uint4 *>(kj + d), acc);
        }
        const float s = j <= pos ? acc * (1.0f / sqrtf((float)CPA_D)) : -INFINITY;
        float m = s;
        m = group_max<16>(m);
        const float e = j <= pos ? expf(s - m) : 0.0f;
        const float ls = group_sum<16>(e);
        sc[h * CPA_POS + j] = e;
        if (j == 0) lsum[h] = ls;
    }
    __syncthreads();
    // ---- P.V: thread = (head h, dims d0 .. d0+7)
    {
        const int h = t >> 4, g = h >> 1, d0 = (t & 15) * 8;
        float acc[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.0f;
        const uint4 ucur = *reinterpret_cast<const uint4 *>(vcur + g * CPA_D + d0);
#pragma unroll
        for (int j = 0; j < CPA_POS; ++j) {
            const bool use = j <= pos;
            uint4 u;
            if constexpr (VL) u = j == pos ? ucur : *reinterpret_cast<const uint4 *>(vf + ((size_t)j * CPA_NKV + g) * CPA_D + d0);
            else u = j == pos ? ucur : a.vv[j];
            const float pj = use ? sc[h * CPA_POS + j] : 0.0f;
            const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float lo2 = use ? h2f(w[e] & 0xffff) : 0.0f, hi2 = use ? h2f(w[e] >> 16) : 0.0f;
                acc[2 * e] += pj * lo2;
                acc[2 * e + 1] += pj * hi2;
            }
        }
        const float inv = lsum[h];
        uint4 o;
        o.x = (uint32_t)f2h(acc[0] / inv) | ((uint32_t)f2h(acc[1] / inv) << 16);
        o.y = (uint32_t)f2h(acc[2] / inv) | ((uint32_t)f2h(acc[3] / inv) << 16);
        o.z = (uint32_t)f2h(acc[4] / inv) | ((uint32_t)f2h(acc[5] / inv) << 16);
        o.w = (uint32_t)f2h(acc[6] / inv) | ((uint32_t)f2h(acc[7] / inv) << 16);
        if (!valid) o = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4 *>(xrow + h * CPA_D + d0) = o;
    }
    __syncthreads();   // scratch reuse by the next slot / the caller's own barrier protocol
}

}  // namespace q3t
