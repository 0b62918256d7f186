// q3t_common.h — shared device/host helpers for the MI355X (gfx950) Qwen3-TTS decode path.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <string>

namespace q3t {

// thread-local last error (q3t_last_error in the C ABI)
void set_error(const std::string &msg);
const std::string &last_error();

#define Q3T_HIP(call)                                                                                   \
    do {                                                                                                \
        hipError_t e__ = (call);                                                                        \
        if (e__ != hipSuccess) {                                                                        \
            ::q3t::set_error(std::string(#call) + ": " + hipGetErrorString(e__) + " @" + __FILE__ + ":" + \
                             std::to_string(__LINE__));                                                 \
            return false;                                                                               \
        }                                                                                               \
    } while (0)

constexpr int WAVE = 64;

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ float h2f(uint16_t h) { return __half2float(__ushort_as_half(h)); }
__device__ __forceinline__ uint16_t f2h(float f) { return __half_as_ushort(__float2half_rn(f)); }
__device__ __forceinline__ float f16r(float f) { return __half2float(__float2half_rn(f)); }

// an f32 value the compiler must materialise as rounded: blocks fusing the producing op with its consumer (e.g. a
// mul-sub followed by an f16 conversion becoming ONE v_fma_mixlo_f16, which rounds once instead of three times)
__device__ __forceinline__ float opaque(float x) {
    asm volatile("" : "+v"(x));
    return x;
}

// 8 f16 (one uint4) dot 8 f16 -> f32 accumulate (v_dot2_f32_f16: exact f16 products, f32 sums)
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float dot8(const uint4 &a, const uint4 &b, float acc) {
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, a.x), __builtin_bit_cast(half2_t, b.x), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, a.y), __builtin_bit_cast(half2_t, b.y), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, a.z), __builtin_bit_cast(half2_t, b.z), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, a.w), __builtin_bit_cast(half2_t, b.w), acc, false);
    return acc;
}
__device__ __forceinline__ float score8(const uint4 &k, const uint32_t (&qp)[4]) {
    return dot8(k, make_uint4(qp[0], qp[1], qp[2], qp[3]), 0.0f);
}

// ---------------------------------------------------------------- decode-attention score / softmax arithmetic
// One lane's share of a q.k score: 8 dims, k as packed f16 (the cache's own bits), q as 4 packed f16 pairs (q is
// f16-rounded before the scores, so the packing is exact), summed by v_dot2_f32_f16 onto 0 in dim order (dot8).
// Every single-slot attention kernel (k_attn, k_prefill_attn, persist.hip, persist_tk.hip, persist_cp.hip) scores and
// exponentiates with these two functions, so the persistent kernels stay bit-identical to the launch-per-op graph.
#ifndef Q3T_ATTN_DOT2
#define Q3T_ATTN_DOT2 1
#endif
__device__ __forceinline__ uint32_t pk_f16x2(float a, float b) {   // exact for f16-representable a, b
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
}
__device__ __forceinline__ void pack_q8(const float (&q8)[8], uint32_t (&qp)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) qp[e] = pk_f16x2(q8[2 * e], q8[2 * e + 1]);
}
__device__ __forceinline__ uint4 pack8f(const float *x) {   // 8 f16-exact floats -> packed f16
    return make_uint4(pk_f16x2(x[0], x[1]), pk_f16x2(x[2], x[3]), pk_f16x2(x[4], x[5]), pk_f16x2(x[6], x[7]));
}
// the softmax exponential of (score - max) <= 0: v_exp_f32 on x * log2(e)
__device__ __forceinline__ float exp_sm(float x) { return Q3T_ATTN_DOT2 ? __expf(x) : expf(x); }

// two fmas as one v_pk_fma_f32 (each lane element is the IEEE fma of its pair: bit-identical to two __fmaf_rn)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
#ifndef Q3T_PK_FMA
#define Q3T_PK_FMA 1
#endif
__device__ __forceinline__ void fma2(float a, float b0, float b1, float &c0, float &c1) {
    if constexpr (Q3T_PK_FMA) {
        const f32x2_t r = __builtin_elementwise_fma(f32x2_t{a, a}, f32x2_t{b0, b1}, f32x2_t{c0, c1});
        c0 = r.x;
        c1 = r.y;
    } else {
        c0 = __fmaf_rn(a, b0, c0);
        c1 = __fmaf_rn(a, b1, c1);
    }
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// 16-byte load through a global (address space 1) pointer: global_load_dwordx4, never a flat load (a flat load counts
// in both vmcnt and lgkmcnt, so its waits also drain the LDS traffic around it)
__device__ __forceinline__ uint4 ldg16(const void *p) {
    typedef const __attribute__((address_space(1))) u32x4_t gv;
    const u32x4_t v = *(gv *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
// 16-byte streaming load of once-read weights (non-temporal policy, microarch 'nt-weights')
__device__ __forceinline__ uint4 ld_nt16(const void *ptr) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(ptr));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// ---------------------------------------------------------------- wave-level reductions (gfx950)
// DPP row ops (VALU, no LDS round trip) inside 16-lane rows; v_permlane16/32_swap (CDNA4) across rows.  The generic
// __shfl_xor lowers to ds_bpermute_b32 (an LDS-crossbar round trip per step), measured ~0.9 us for a 6-step wave
// reduction on the selection path -- too slow for the latency-bound decode chain.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const unsigned lo = dpp_u<CTRL>((unsigned)u), hi = dpp_u<CTRL>((unsigned)(u >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;
// value of the same lane in the partner row (lane ^ 16) / partner half (lane ^ 32)
__device__ __forceinline__ unsigned xrow16_u(unsigned v) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return ((threadIdx.x >> 4) & 1) ? (unsigned)r[0] : (unsigned)r[1];
}
__device__ __forceinline__ unsigned xrow32_u(unsigned v) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return ((threadIdx.x >> 5) & 1) ? (unsigned)r[0] : (unsigned)r[1];
}
__device__ __forceinline__ float xrow16(float v) { return __builtin_bit_cast(float, xrow16_u(__builtin_bit_cast(unsigned, v))); }
__device__ __forceinline__ float xrow32(float v) { return __builtin_bit_cast(float, xrow32_u(__builtin_bit_cast(unsigned, v))); }
__device__ __forceinline__ double xrow16_d(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    return __builtin_bit_cast(double, ((uint64_t)xrow16_u((unsigned)(u >> 32)) << 32) | xrow16_u((unsigned)u));
}
__device__ __forceinline__ double xrow32_d(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    return __builtin_bit_cast(double, ((uint64_t)xrow32_u((unsigned)(u >> 32)) << 32) | xrow32_u((unsigned)u));
}

template <int W>
__device__ __forceinline__ float group_sum(float v) {   // all-reduce inside aligned groups of W lanes
    static_assert(W == 4 || W == 8 || W == 16 || W == 32 || W == 64, "group width");
    v += dpp_f<DPP_XOR1>(v);
    v += dpp_f<DPP_XOR2>(v);
    if constexpr (W >= 8) v += dpp_f<DPP_HALF_MIRROR>(v);
    if constexpr (W >= 16) v += dpp_f<DPP_MIRROR>(v);
    if constexpr (W >= 32) v += xrow16(v);
    if constexpr (W >= 64) v += xrow32(v);
    return v;
}
template <int W>
__device__ __forceinline__ float group_max(float v) {
    v = fmaxf(v, dpp_f<DPP_XOR1>(v));
    v = fmaxf(v, dpp_f<DPP_XOR2>(v));
    if constexpr (W >= 8) v = fmaxf(v, dpp_f<DPP_HALF_MIRROR>(v));
    if constexpr (W >= 16) v = fmaxf(v, dpp_f<DPP_MIRROR>(v));
    if constexpr (W >= 32) v = fmaxf(v, xrow16(v));
    if constexpr (W >= 64) v = fmaxf(v, xrow32(v));
    return v;
}
__device__ __forceinline__ float wave_max(float v) { return group_max<64>(v); }
__device__ __forceinline__ float wave_sum(float v) { return group_sum<64>(v); }
__device__ __forceinline__ double wave_sum_d(double v) {
    v += dpp_d<DPP_XOR1>(v);
    v += dpp_d<DPP_XOR2>(v);
    v += dpp_d<DPP_HALF_MIRROR>(v);
    v += dpp_d<DPP_MIRROR>(v);
    v += xrow16_d(v);
    v += xrow32_d(v);
    return v;
}
// sum / max over the lanes {l, l^16, l^32, l^48} (same position in the 4 rows), result in every lane
__device__ __forceinline__ float rows_sum(float v) { v += xrow16(v); return v + xrow32(v); }
__device__ __forceinline__ float rows_max(float v) { v = fmaxf(v, xrow16(v)); return fmaxf(v, xrow32(v)); }
// rows_sum of two values in one pass: row 0 (and 2) ends with a's (r0 + r1) + (r2 + r3), row 1 (and 3) with b's
__device__ __forceinline__ float rows_sum_pair(float a, float b) {
    const auto s = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b), false, false);
    const float c = __builtin_bit_cast(float, (unsigned)s[0]) + __builtin_bit_cast(float, (unsigned)s[1]);
    return c + xrow32(c);
}
__device__ __forceinline__ double rows_sum_d(double v) { v += xrow16_d(v); return v + xrow32_d(v); }

// wave inclusive scan (row_shr DPP within rows, row_bcast15/31 across rows: the GCN scan idiom)
__device__ __forceinline__ unsigned wave_scan_incl_u(unsigned v) {
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}
__device__ __forceinline__ float wave_scan_incl_f(float v) {
    v += dpp_f<0x111>(v);
    v += dpp_f<0x112>(v);
    v += dpp_f<0x114>(v);
    v += dpp_f<0x118>(v);
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x143, 0xC, 0xF, false));
    return v;
}

// splitmix64 finaliser; uniform in [0,1) with 24 bits (identical to oracle q3o_uniform)
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ float uniform24(uint64_t seed, uint64_t utt, uint64_t frame, uint64_t cb) {
    const uint64_t h = mix64(mix64(seed ^ (utt * 0xD1B54A32D192ED03ull)) + frame * 16ull + cb);
    return (float)(h >> 40) * (1.0f / 16777216.0f);
}

// ggml_vec_gelu_f32 with the F16 lookup (GGML_GELU_FP16) [ggml-upstream]
__device__ __forceinline__ float gelu_ggml(float x) {
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    const float v = f16r(x);
    const float g = 0.5f * v * (1.0f + tanhf(0.79788456080286535587989211986876f * v * (1.0f + 0.044715f * v * v)));
    return f16r(g);
}
__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

}  // namespace q3t
