// kernels.hip — hand-written gfx950 (CDNA4) kernels of the per-frame decode path.
//
// Numerics follow the reference CPU path (GGML_CUDA=OFF): f16 weights exactly as stored in the GGUF, every
// matmul input activation rounded to f16 (ggml mul_mat converts src1 to vec_dot_type F16), products
// accumulated in f32 (v_dot2_f32_f16: exact f16 products), F16 KV cache, f32 norms/softmax/residuals.
#include "kernels.h"

#include <algorithm>

namespace q3t {

// ======================================================================================= token selection
// One 1024-thread block per slot; logits staged in LDS (V <= 4096).
constexpr int SEL_T = 1024;
struct SelScratch {
    float v[4096];
    unsigned hist[256];
    float fred[16];
    int ired[16];
    unsigned ures[4];
};

__device__ __forceinline__ uint32_t fkey(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float keyf(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
__device__ float block_max_f(float v, SelScratch &S) {
    v = wave_max(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) S.fred[wave] = v;
    __syncthreads();
    float m = -INFINITY;
    for (int w = 0; w < SEL_T / 64; ++w) m = fmaxf(m, S.fred[w]);
    return m;
}
__device__ float block_sum_f(float v, SelScratch &S) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) S.fred[wave] = v;
    __syncthreads();
    float t = 0.0f;
    for (int w = 0; w < SEL_T / 64; ++w) t += S.fred[w];
    return t;
}
// first index of the maximum (strict '>' scan of tts_transformer.cpp:2051-2061)
__device__ int block_argmax_first(const float *v, int n, SelScratch &S) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < n; i += SEL_T)
        if (v[i] > bv || (v[i] == bv && i < bi)) { bv = v[i]; bi = i; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) { S.fred[wave] = bv; S.ired[wave] = bi; }
    __syncthreads();
    bv = S.fred[0]; bi = S.ired[0];
    for (int w = 1; w < SEL_T / 64; ++w)
        if (S.fred[w] > bv || (S.fred[w] == bv && S.ired[w] < bi)) { bv = S.fred[w]; bi = S.ired[w]; }
    return bi == 0x7fffffff ? 0 : bi;
}
// k-th largest value of v[0..n) by 4-pass MSB radix select on order-preserving keys
__device__ float block_kth_largest(const float *v, int n, int k, SelScratch &S) {
    uint32_t prefix = 0, pmask = 0;
    int kk = k;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = threadIdx.x; i < 256; i += SEL_T) S.hist[i] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += SEL_T) {
            const uint32_t key = fkey(v[i]);
            if ((key & pmask) == prefix) atomicAdd(&S.hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            // lane l owns digits 255-4l .. 252-4l (descending)
            const int l = threadIdx.x;
            unsigned c[4], loc = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) { c[t] = S.hist[255 - 4 * l - t]; loc += c[t]; }
            unsigned incl = loc;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned y = __shfl_up(incl, o, 64);
                if (l >= o) incl += y;
            }
            unsigned cum = incl - loc;   // count of keys with a larger digit than this lane's first digit
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (cum < (unsigned)kk && (unsigned)kk <= cum + c[t]) {
                    S.ures[0] = (unsigned)(255 - 4 * l - t);
                    S.ures[1] = cum;
                }
                cum += c[t];
            }
        }
        __syncthreads();
        const uint32_t d = S.ures[0];
        kk -= (int)S.ures[1];
        prefix |= d << shift;
        pmask |= 255u << shift;
        __syncthreads();
    }
    return keyf(prefix);
}
// temperature -> top-k (< thr => -inf, ties survive) -> keep_id restored -> exp -> inverse CDF with u
__device__ int block_sample(float *v, int n, float temperature, int top_k, float u, int keep_id, SelScratch &S) {
    for (int i = threadIdx.x; i < n; i += SEL_T) v[i] = v[i] / temperature;
    __syncthreads();
    const float keep_v = keep_id >= 0 ? v[keep_id] : 0.0f;
    if (top_k > 0 && top_k < n) {
        const float thr = block_kth_largest(v, n, top_k, S);
        for (int i = threadIdx.x; i < n; i += SEL_T) if (v[i] < thr) v[i] = -INFINITY;
        __syncthreads();
    }
    if (keep_id >= 0 && threadIdx.x == 0) v[keep_id] = keep_v;
    __syncthreads();
    float m = -INFINITY;
    for (int i = threadIdx.x; i < n; i += SEL_T) m = fmaxf(m, v[i]);
    m = block_max_f(m, S);
    // contiguous ownership so the prefix runs in index order
    const int ept = (n + SEL_T - 1) / SEL_T;
    const int i0 = threadIdx.x * ept, i1 = min(n, i0 + ept);
    float loc = 0.0f;
    for (int i = i0; i < i1; ++i) { const float e = expf(v[i] - m); v[i] = e; loc += e; }
    // block exclusive scan of loc
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const float y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    __syncthreads();
    if (lane == 63) S.fred[wave] = incl;
    if (threadIdx.x == 0) S.ures[2] = 0x7fffffffu;
    __syncthreads();
    float wpre = 0.0f, total = 0.0f;
    for (int w = 0; w < SEL_T / 64; ++w) { if (w < wave) wpre += S.fred[w]; total += S.fred[w]; }
    const float target = u * total;
    float cum = wpre + incl - loc;
    int found = 0x7fffffff;
    for (int i = i0; i < i1; ++i) {
        cum += v[i];
        if (cum >= target && v[i] > 0.0f) { found = i; break; }
    }
    if (found != 0x7fffffff) atomicMin(reinterpret_cast<int *>(&S.ures[2]), found);
    __syncthreads();
    const int r = (int)S.ures[2];
    return r == 0x7fffffff ? n - 1 : r;
}


// ---------------------------------------------------------------- CB0 selection (tts_transformer.cpp:2417-2499)
__global__ void __launch_bounds__(SEL_T) k_cb0(const Cb0Params p) {
    __shared__ SelScratch S;
    const int s = blockIdx.x;
    if (p.done[s] >= 0) return;
    const int V = p.V, EOS = p.eos;
    const int frame = p.frame[s];
    const float *lg = p.logits + (size_t)s * V;
    const uint8_t *seen = p.seen + (size_t)s * V;
    float m = -INFINITY;
    for (int i = threadIdx.x; i < V; i += SEL_T) {
        float v = lg[i];
        if (i >= V - 1024 && i != EOS) v = -INFINITY;                         // :2418-2422
        if (p.rep != 1.0f && seen[i]) v = v > 0.0f ? v / p.rep : v * p.rep;  // :2425-2435
        S.v[i] = v;
        m = fmaxf(m, v);
    }
    m = block_max_f(m, S);
    const int ntok = p.n_tokens[s];
    const int expected = max(20, ntok * 4);                                    // :2439-2445
    if (threadIdx.x == 0) {
        if (frame >= expected) {
            const float ramp = fminf(1.0f, (float)(frame - expected) / (float)expected);
            S.v[EOS] += ramp * ((m + 5.0f) - S.v[EOS]);
        }
        if (frame < p.force_frames[s]) S.v[EOS] = -INFINITY;
    }
    __syncthreads();
    const bool masked = frame < p.force_frames[s];
    int tok;
    if (p.temperature <= 0.0f) tok = block_argmax_first(S.v, V, S);
    else tok = block_sample(S.v, V, p.temperature, p.top_k, uniform24(p.seed, p.utt[s], (uint64_t)frame, 0), masked ? -1 : EOS, S);
    if (tok == EOS) {
        if (threadIdx.x == 0) { p.done[s] = frame; p.token[s * 16] = tok; }
        return;
    }
    if (threadIdx.x == 0) {
        p.token[s * 16] = tok;
        p.seen[(size_t)s * V + tok] = 1;
        if (frame < p.max_len) p.codes[((size_t)s * p.max_len + frame) * p.ncb] = tok;
    }
    if (p.x_next) {
        const uint16_t *row = p.next_table + (size_t)tok * p.H;
        for (int h = threadIdx.x; h < p.H; h += SEL_T) p.x_next[(size_t)s * p.H + h] = h2f(row[h]);
    }
}
bool cb0_select(const Cb0Params &p, hipStream_t s) {
    if (p.V > 4096) { set_error("cb0_select: vocab > 4096"); return false; }
    hipLaunchKernelGGL(k_cb0, dim3(p.S), dim3(SEL_T), 0, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}

// ---------------------------------------------------------------- code-predictor token + next-pass gather
__global__ void __launch_bounds__(SEL_T) k_cpsel(const CpSelParams p) {
    __shared__ SelScratch S;
    const int s = blockIdx.x;
    if (p.done[s] >= 0) return;
    const int V = p.V, frame = p.frame[s];
    for (int i = threadIdx.x; i < V; i += SEL_T) S.v[i] = p.logits[(size_t)s * V + i];
    __syncthreads();
    int tok;
    if (p.temperature <= 0.0f) tok = block_argmax_first(S.v, V, S);
    else tok = block_sample(S.v, V, p.temperature, p.top_k, uniform24(p.seed, p.utt[s], (uint64_t)frame, (uint64_t)p.step + 1), -1, S);
    if (threadIdx.x == 0) {
        p.tokens[s * 16 + p.step + 1] = tok;
        if (frame < p.max_len) p.codes[((size_t)s * p.max_len + frame) * p.ncb + p.step + 1] = tok;
    }
    if (p.next_table) {
        const uint16_t *row = p.next_table + (size_t)tok * p.H;
        for (int h = threadIdx.x; h < p.H; h += SEL_T) p.x_next[(size_t)s * p.H + h] = h2f(row[h]);
    }
}
bool cp_select(const CpSelParams &p, hipStream_t s) {
    if (p.V > 4096) { set_error("cp_select: vocab > 4096"); return false; }
    hipLaunchKernelGGL(k_cpsel, dim3(p.S), dim3(SEL_T), 0, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}

// ---------------------------------------------------------------- step embedding (tts_transformer.cpp:2529-2553)
__global__ void __launch_bounds__(256) k_step_embd(const StepEmbdParams p) {
    const int s = blockIdx.x;
    const int *tk = p.tokens + s * 16;
    const int frame = p.frame[s];
    const float *tr = frame < p.trailing_len[s] ? p.trailing + ((size_t)s * p.max_trailing + frame) * p.H : p.tts_pad + (size_t)s * p.H;
    for (int h = threadIdx.x; h < p.H; h += 256) {
        float e = h2f(p.codec_embd[(size_t)tk[0] * p.H + h]);
        for (int c = 1; c < p.ncb; ++c) e += h2f(p.cp_embd[c - 1][(size_t)tk[c] * p.H + h]);
        e += tr[h];
        p.out[(size_t)s * p.H + h] = e;
    }
}
bool step_embd(const StepEmbdParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_step_embd, dim3(p.S), dim3(256), 0, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}

__global__ void k_advance(int *pos, int *frame, int S) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < S) { pos[s] += 1; frame[s] += 1; }
}
bool advance(int *pos, int *frame, int S, hipStream_t s) {
    hipLaunchKernelGGL(k_advance, dim3((S + 63) / 64), dim3(64), 0, s, pos, frame, S);
    Q3T_HIP(hipGetLastError());
    return true;
}

__global__ void k_rows_recipe(const RowRecipe *rec, int H) {
    const RowRecipe R = rec[blockIdx.x];
    for (int h = threadIdx.x; h < H; h += blockDim.x) {
        float v = 0.0f;
        bool first = true;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            if (!R.t[t].ptr) continue;
            const float x = R.t[t].is_f16 ? h2f(reinterpret_cast<const uint16_t *>(R.t[t].ptr)[h])
                                          : reinterpret_cast<const float *>(R.t[t].ptr)[h];
            v = first ? x : v + x;
            first = false;
        }
        R.out[h] = v;
    }
}
bool rows_recipe(const RowRecipe *recipe_dev, int n_rows, int H, hipStream_t s) {
    if (n_rows <= 0) return true;
    hipLaunchKernelGGL(k_rows_recipe, dim3(n_rows), dim3(256), 0, s, recipe_dev, H);
    Q3T_HIP(hipGetLastError());
    return true;
}


// ---------------------------------------------------------------- trt_cuda_kernels.cu drop-ins
__global__ void k_f32_to_f16(const float *in, uint16_t *out, int n) {
    const int i = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i + 3 < n) {
        const float4 v = *reinterpret_cast<const float4 *>(in + i);
        out[i] = f2h(v.x); out[i + 1] = f2h(v.y); out[i + 2] = f2h(v.z); out[i + 3] = f2h(v.w);
    } else {
        for (int j = i; j < n; ++j) out[j] = f2h(in[j]);
    }
}
__global__ void __launch_bounds__(SEL_T) k_argmax_f32(const float *in, int32_t *out, int n) {
    __shared__ SelScratch S;
    const int r = block_argmax_first(in, n, S);
    if (threadIdx.x == 0) *out = r;
}
__global__ void k_embed_lookup(const int32_t *tok, const float *table, float *out, int dim) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < dim) out[i] = table[(size_t)(*tok) * dim + i];
}
__global__ void __launch_bounds__(SEL_T) k_sample_topk_f32(const float *logits, const float *rand_val, int32_t *out,
                                                            float temperature, int top_k, int n) {
    __shared__ SelScratch S;
    for (int i = threadIdx.x; i < n; i += SEL_T) S.v[i] = logits[i];
    __syncthreads();
    const int r = block_sample(S.v, n, temperature, top_k, *rand_val, -1, S);
    if (threadIdx.x == 0) *out = r;
}
void launch_f32_to_f16(const float *in, uint16_t *out, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_f32_to_f16, dim3((n + 1023) / 1024), dim3(256), 0, s, in, out, n);
}
void launch_argmax_f32(const float *in, int32_t *out, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_argmax_f32, dim3(1), dim3(SEL_T), 0, s, in, out, n);
}
void launch_embed_lookup(const int32_t *tok, const float *table, float *out, int dim, hipStream_t s) {
    hipLaunchKernelGGL(k_embed_lookup, dim3((dim + 255) / 256), dim3(256), 0, s, tok, table, out, dim);
}
void launch_sample_topk_f32(const float *logits, const float *rand_val, int32_t *out, float temperature, int top_k, int n,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_sample_topk_f32, dim3(1), dim3(SEL_T), 0, s, logits, rand_val, out, temperature, top_k, n);
}

}  // namespace q3t
