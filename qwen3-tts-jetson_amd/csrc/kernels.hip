// kernels.hip — hand-written gfx950 (CDNA4) kernels of the per-frame decode path.
//
// Numerics follow the reference CPU path (GGML_CUDA=OFF): f16 weights exactly as stored in the GGUF, every
// matmul input activation rounded to f16 (ggml mul_mat converts src1 to vec_dot_type F16), products
// accumulated in f32 (v_dot2_f32_f16: exact f16 products), F16 KV cache, f32 norms/softmax/residuals.
#include "kernels.h"
#include "select.h"

#include <algorithm>

namespace q3t {

// ======================================================================================= token selection
__global__ void __launch_bounds__(256) k_select(const SelectSpec sp, const float *logits) {
    __shared__ SelLds S;
    select_slot<false>(sp, logits + (size_t)blockIdx.x * sp.V, blockIdx.x, S);
}
bool select_tokens(const SelectSpec &sp, const float *logits, int S, hipStream_t s) {
    if (sp.V > 256 * SEL_VPT_MAX || sp.V <= 0) { set_error("select: vocab must be in (0, 4096]"); return false; }
    if (S <= 0) return true;
    hipLaunchKernelGGL(k_select, dim3(S), dim3(256), 0, s, sp, logits);
    Q3T_HIP(hipGetLastError());
    return true;
}

// GatherSum rows materialised (batched path: the matrix-core GEMM has no gather prologue).  Same order of the f32
// sums as gemv.hip's issue_x_gather, so both paths see bit-identical activation rows.
template <int NT>
__global__ void __launch_bounds__(256) k_gather_sum(const GatherSum gs, int K, float *out, int ldo) {
    const int b = blockIdx.x;
    for (int k = threadIdx.x * 4; k < K; k += 1024) {   // K > 1024 (1.7B talker rows): one 1024-wide chunk per pass
    const uint16_t *row[NT];
    const float *extra = nullptr;
    if constexpr (NT == 1) {
        row[0] = gs.tab0 + (size_t)gs.tok[(size_t)b * gs.tok_ld + gs.tok_col0] * K;
    } else {
        const int *tk = gs.tok + (size_t)b * gs.tok_ld;
#pragma unroll
        for (int j = 0; j < NT; ++j) row[j] = gs.tabs[j] + (size_t)tk[j] * K;
        const int fr = gs.frame[b];
        extra = fr < gs.tr_len[b] ? gs.tr + (size_t)b * gs.tr_ld + (size_t)fr * K : gs.pad + (size_t)b * K;
    }
    float a[4];
    {
        const uint2 u = *reinterpret_cast<const uint2 *>(row[0] + k);
        a[0] = h2f(u.x & 0xffff); a[1] = h2f(u.x >> 16); a[2] = h2f(u.y & 0xffff); a[3] = h2f(u.y >> 16);
    }
#pragma unroll
    for (int j = 1; j < NT; ++j) {
        const uint2 u = *reinterpret_cast<const uint2 *>(row[j] + k);
        a[0] += h2f(u.x & 0xffff); a[1] += h2f(u.x >> 16); a[2] += h2f(u.y & 0xffff); a[3] += h2f(u.y >> 16);
    }
    if constexpr (NT > 1) {
        const float4 e = *reinterpret_cast<const float4 *>(extra + k);
        a[0] += e.x; a[1] += e.y; a[2] += e.z; a[3] += e.w;
    }
    *reinterpret_cast<float4 *>(out + (size_t)b * ldo + k) = make_float4(a[0], a[1], a[2], a[3]);
    }
}
bool gather_sum(const GatherSum &gs, int nt, int S, int K, float *out, int ldo, hipStream_t s) {
    if (K % 4 != 0 || (nt != 1 && nt != 16)) { set_error("gather_sum: unsupported shape"); return false; }
    if (S <= 0) return true;
    if (nt == 1) hipLaunchKernelGGL(k_gather_sum<1>, dim3(S), dim3(256), 0, s, gs, K, out, ldo);
    else hipLaunchKernelGGL(k_gather_sum<16>, dim3(S), dim3(256), 0, s, gs, K, out, ldo);
    Q3T_HIP(hipGetLastError());
    return true;
}

// a slot whose utterance ended (done >= 0) stays where it is: its position never runs past the context reserved
// for it, however long the other slots (or a continuous-batching queue) keep the frame loop going
__global__ void k_advance(int *pos, int *frame, const int *done, int S) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < S && !(done && done[s] >= 0)) { pos[s] += 1; frame[s] += 1; }
}
bool advance(int *pos, int *frame, const int *done, int S, hipStream_t s) {
    hipLaunchKernelGGL(k_advance, dim3((S + 63) / 64), dim3(64), 0, s, pos, frame, done, S);
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
__global__ void __launch_bounds__(256) k_argmax_f32(const float *in, int32_t *out, int n) {
    __shared__ SelLds S;
    if (n <= 256 * SEL_VPT_MAX) {
        float v[SEL_VPT_MAX];
        const int vpt = (n + 255) / 256;
        sel_load<false>(in, n, vpt, v);
        const int r = sel_argmax(v, n, vpt, S);
        if (threadIdx.x == 0) *out = r;
        return;
    }
    // any n (the reference wrapper accepts any length): strided scan, lowest index wins ties
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < n; i += 256)
        if (in[i] > bv || bi == 0x7fffffff) { bv = in[i]; bi = i; }
    sel_pair_reduce(bv, bi);
    if ((threadIdx.x & 63) == 0) { S.fred[threadIdx.x >> 6] = bv; S.ired[threadIdx.x >> 6] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w)
            if (S.fred[w] > S.fred[0] || (S.fred[w] == S.fred[0] && S.ired[w] < S.ired[0])) { S.fred[0] = S.fred[w]; S.ired[0] = S.ired[w]; }
        *out = S.ired[0] == 0x7fffffff ? 0 : S.ired[0];
    }
}
__global__ void k_embed_lookup(const int32_t *tok, const float *table, float *out, int dim) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < dim) out[i] = table[(size_t)(*tok) * dim + i];
}
__global__ void __launch_bounds__(256) k_sample_topk_f32(const float *logits, const float *rand_val, int32_t *out,
                                                          float temperature, int top_k, int n) {
    __shared__ SelLds S;
    float v[SEL_VPT_MAX];
    const int vpt = (n + 255) / 256;
    sel_load<false>(logits, n, vpt, v);
    const int r = temperature <= 0.0f ? sel_argmax(v, n, vpt, S) : sel_sample(v, n, vpt, temperature, top_k, *rand_val, -1, S);
    if (threadIdx.x == 0) *out = r;
}
void launch_f32_to_f16(const float *in, uint16_t *out, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_f32_to_f16, dim3((n + 1023) / 1024), dim3(256), 0, s, in, out, n);
}
void launch_argmax_f32(const float *in, int32_t *out, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_argmax_f32, dim3(1), dim3(256), 0, s, in, out, n);
}
void launch_embed_lookup(const int32_t *tok, const float *table, float *out, int dim, hipStream_t s) {
    hipLaunchKernelGGL(k_embed_lookup, dim3((dim + 255) / 256), dim3(256), 0, s, tok, table, out, dim);
}
void launch_sample_topk_f32(const float *logits, const float *rand_val, int32_t *out, float temperature, int top_k, int n,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_sample_topk_f32, dim3(1), dim3(256), 0, s, logits, rand_val, out, temperature, top_k, n);
}

// ------------------------------------------------------------------------------------------ batched residual + norm
// one workgroup per token; thread t owns elements 4t .. 4t+3 (H <= 1024).  Partial slabs are added in slice order;
// the RMS sum runs in double over the block (gemv.hip / gemm_mfma.hip prologue numerics).  KS (the slab count) is a
// template argument so the x and slab loads issue back to back: with a runtime count each sat in its own branch and
// waited for its own round trip.
// Workgroups past the S token rows only prefetch (ResidNorm::prefetch): global->LDS dword loads, one per 128-B line
// of the next projection's weights, which leave no register to wait on; the lines land in the Infinity Cache.
constexpr int RN_PF_LINES = 2;   // prefetched lines per thread
template <int KS>
__global__ void __launch_bounds__(256) k_resid_norm(const ResidNorm r) {
    __shared__ double scr[4];
    const int b = blockIdx.x, t = threadIdx.x, k = 4 * t;
    if (b >= r.S) {
        __shared__ uint32_t sink[256];
        const size_t lines = r.prefetch_bytes / 128, nthr = (size_t)(gridDim.x - r.S) * 256;
#pragma unroll
        for (int q = 0; q < RN_PF_LINES; ++q) {
            const size_t line = (size_t)q * nthr + (size_t)(b - r.S) * 256 + t;
            if (line < lines)
                __builtin_amdgcn_global_load_lds(static_cast<const uint8_t *>(r.prefetch) + line * 128,
                                                 (__attribute__((address_space(3))) void *)sink, 4, 0, 0);
        }
        return;
    }
    const bool ok = k < r.H;
    const size_t o = (size_t)b * r.H + (ok ? k : 0);
    float4 x = *reinterpret_cast<const float4 *>((r.xin ? r.xin : r.x) + o);
    float4 pz[KS > 0 ? KS : 1];
#pragma unroll
    for (int z = 0; z < KS; ++z) pz[z] = *reinterpret_cast<const float4 *>(r.parts + (size_t)z * r.S * r.H + o);
#pragma unroll
    for (int z = 0; z < KS; ++z) x = make_float4(x.x + pz[z].x, x.y + pz[z].y, x.z + pz[z].z, x.w + pz[z].w);
    if (!ok) x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok && (KS > 0 || (r.xin && r.xin != r.x))) *reinterpret_cast<float4 *>(r.x + o) = x;
    double ss = (double)(x.x * x.x) + (double)(x.y * x.y) + (double)(x.z * x.z) + (double)(x.w * x.w);
    ss = wave_sum_d(ss);
    if ((t & 63) == 0) scr[t >> 6] = ss;
    __syncthreads();
    ss = (scr[0] + scr[1]) + (scr[2] + scr[3]);
    if (!ok) return;
    const float scale = 1.0f / sqrtf((float)(ss / r.H) + r.eps);
    const float4 w = *reinterpret_cast<const float4 *>(r.nw + k);
    const float y0 = (x.x * scale) * w.x, y1 = (x.y * scale) * w.y, y2 = (x.z * scale) * w.z, y3 = (x.w * scale) * w.w;
    if (r.side) *reinterpret_cast<float4 *>(r.side + o) = make_float4(y0, y1, y2, y3);
    uint2 h;
    h.x = (uint32_t)f2h(y0) | ((uint32_t)f2h(y1) << 16);
    h.y = (uint32_t)f2h(y2) | ((uint32_t)f2h(y3) << 16);
    *reinterpret_cast<uint2 *>(r.xn + o) = h;
}
__global__ void __launch_bounds__(256) k_select_embed_norm(const SelectSpec sp, const float *logits, const EmbedNorm en) {
    __shared__ SelLds S;
    __shared__ double scr[4];
    __shared__ int stok;
    const int b = blockIdx.x, t = threadIdx.x, k = 4 * t;
    const int tok = select_token<false>(sp, logits + (size_t)b * sp.V, b, S);
    if (t == 0) {
        if (tok >= 0) select_commit(sp, b, tok);
        stok = tok;
    }
    __syncthreads();
    const int sel_col = sp.mode == SEL_CB0 ? 0 : sp.step + 1;   // the column this launch selected
    const GatherSum &gs = en.gs;
    auto token = [&](int col) {   // finished slots (no selection) keep the token already in the table
        const int tt = gs.tok[(size_t)b * gs.tok_ld + col];   // loaded unconditionally: no branch around the load
        return col == sel_col && stok >= 0 ? stok : tt;
    };
    const bool ok = k < en.H;
    const int kk = ok ? k : 0;
    float a[4];
    {
        const uint16_t *r0 = en.nt == 1 ? gs.tab0 + (size_t)token(gs.tok_col0) * en.H : gs.tabs[0] + (size_t)token(0) * en.H;
        const uint2 u = *reinterpret_cast<const uint2 *>(r0 + kk);
        a[0] = h2f(u.x & 0xffff); a[1] = h2f(u.x >> 16); a[2] = h2f(u.y & 0xffff); a[3] = h2f(u.y >> 16);
    }
    if (en.nt == 16) {
#pragma unroll   // the 15 token loads, then the 15 row loads, each group in flight together
        for (int j = 1; j < 16; ++j) {
            const uint2 u = *reinterpret_cast<const uint2 *>(gs.tabs[j] + (size_t)token(j) * en.H + kk);
            a[0] += h2f(u.x & 0xffff); a[1] += h2f(u.x >> 16); a[2] += h2f(u.y & 0xffff); a[3] += h2f(u.y >> 16);
        }
        const int fr = gs.frame[b];
        const float *extra = fr < gs.tr_len[b] ? gs.tr + (size_t)b * gs.tr_ld + (size_t)fr * en.H : gs.pad + (size_t)b * en.H;
        const float4 e = *reinterpret_cast<const float4 *>(extra + kk);
        a[0] += e.x; a[1] += e.y; a[2] += e.z; a[3] += e.w;
    }
    float4 x = ok ? make_float4(a[0], a[1], a[2], a[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
    const size_t o = (size_t)b * en.H + kk;
    if (ok) *reinterpret_cast<float4 *>(en.x + o) = x;
    double ss = (double)(x.x * x.x) + (double)(x.y * x.y) + (double)(x.z * x.z) + (double)(x.w * x.w);
    ss = wave_sum_d(ss);
    if ((t & 63) == 0) scr[t >> 6] = ss;
    __syncthreads();
    ss = (scr[0] + scr[1]) + (scr[2] + scr[3]);
    if (!ok) return;
    const float scale = 1.0f / sqrtf((float)(ss / en.H) + en.eps);
    const float4 w = *reinterpret_cast<const float4 *>(en.nw + k);
    const float y0 = (x.x * scale) * w.x, y1 = (x.y * scale) * w.y, y2 = (x.z * scale) * w.z, y3 = (x.w * scale) * w.w;
    uint2 h;
    h.x = (uint32_t)f2h(y0) | ((uint32_t)f2h(y1) << 16);
    h.y = (uint32_t)f2h(y2) | ((uint32_t)f2h(y3) << 16);
    *reinterpret_cast<uint2 *>(en.xn + o) = h;
}
bool select_embed_norm(const SelectSpec &sp, const float *logits, const EmbedNorm &en, int S, hipStream_t s) {
    if (sp.V > 256 * SEL_VPT_MAX || sp.V <= 0) { set_error("select: vocab must be in (0, 4096]"); return false; }
    if (en.H > 1024 || en.H % 4 != 0 || !en.x || !en.xn || !en.nw || (en.nt != 1 && en.nt != 16) ||
        (en.nt == 1 && !en.gs.tab0) || (en.nt == 16 && !(en.gs.tabs && en.gs.frame && en.gs.tr_len && en.gs.pad)) ||
        !en.gs.tok) {
        set_error("select_embed_norm: bad parameters");
        return false;
    }
    if (S <= 0) return true;
    hipLaunchKernelGGL(k_select_embed_norm, dim3(S), dim3(256), 0, s, sp, logits, en);
    Q3T_HIP(hipGetLastError());
    return true;
}

bool resid_norm(const ResidNorm &r, hipStream_t s) {
    if (r.S <= 0) return true;
    if (r.H > 1024 || r.H % 4 != 0 || !r.x || !r.nw || !r.xn || (r.parts && (r.ksplit < 1 || r.ksplit > 4))) {
        set_error("resid_norm: unsupported shape");
        return false;
    }
    const size_t pf_lines = r.prefetch ? r.prefetch_bytes / 128 : 0;
    const unsigned pf_wgs = (unsigned)std::min<size_t>((pf_lines + 256 * RN_PF_LINES - 1) / (256 * RN_PF_LINES), 1024);
    const dim3 grid((unsigned)r.S + pf_wgs);
    switch (r.parts ? r.ksplit : 0) {
        case 0: hipLaunchKernelGGL(k_resid_norm<0>, grid, dim3(256), 0, s, r); break;
        case 1: hipLaunchKernelGGL(k_resid_norm<1>, grid, dim3(256), 0, s, r); break;
        case 2: hipLaunchKernelGGL(k_resid_norm<2>, grid, dim3(256), 0, s, r); break;
        case 3: hipLaunchKernelGGL(k_resid_norm<3>, grid, dim3(256), 0, s, r); break;
        default: hipLaunchKernelGGL(k_resid_norm<4>, grid, dim3(256), 0, s, r); break;
    }
    Q3T_HIP(hipGetLastError());
    return true;
}

}  // namespace q3t
