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

// 8 f16 (one uint4) dot 8 f16 -> f32 accumulate (v_dot2_f32_f16: exact f16 products, f32 sums)
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float dot8(const uint4 &a, const uint4 &b, float acc) {
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, a.x), __builtin_bit_cast(half2_t, b.x), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, a.y), __builtin_bit_cast(half2_t, b.y), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, a.z), __builtin_bit_cast(half2_t, b.z), acc, false);
    acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, a.w), __builtin_bit_cast(half2_t, b.w), acc, false);
    return acc;
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// 16-byte streaming load of once-read weights (non-temporal policy, microarch 'nt-weights')
__device__ __forceinline__ uint4 ld_nt16(const void *ptr) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(ptr));
    return make_uint4(v.x, v.y, v.z, v.w);
}

template <int W>
__device__ __forceinline__ float group_sum(float v) {   // xor-butterfly inside aligned groups of W lanes
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, W);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
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
