// kernels.hip — hand-written gfx950 (CDNA4) kernels of the per-frame decode path.
//
// Numerics follow the reference CPU path (GGML_CUDA=OFF): f16 weights exactly as stored in the GGUF, every
// matmul input activation rounded to f16 (ggml mul_mat converts src1 to vec_dot_type F16), products
// accumulated in f32 (v_dot2_f32_f16: exact f16 products), F16 KV cache, f32 norms/softmax/residuals.
#include "kernels.h"

#include <algorithm>

namespace q3t {

// ======================================================================================= block reductions
__device__ __forceinline__ double block_sum_d(double v, double *scratch /*>= 4*/) {
    v = wave_sum_d(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if (lane == 0) scratch[wave] = v;
    __syncthreads();
    double t = 0.0;
    for (int w = 0; w < nw; ++w) t += scratch[w];
    return t;
}

// ======================================================================================= GEMV
// Block = 256 threads = 16 row-groups of 16 lanes.  A row-group streams one weight row with 16-B loads
// (256 contiguous bytes per group per step), the activation tile sits in LDS as f16, BT batch columns are
// held in registers.  KS = 4 splits K over the 4 waves (small-N GEMMs still fill >= 256 workgroups).
template <int RPG, int BT, int KS, int PRO>
__global__ void __launch_bounds__(256) k_gemv(const GemvParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int K = p.K, N = p.N;
    const int Kp = (K + 127) & ~127;
    uint16_t *xs = reinterpret_cast<uint16_t *>(smem);
    float *red = reinterpret_cast<float *>(smem + (size_t)BT * Kp * 2);
    double *dscr = reinterpret_cast<double *>(red + 4 * 4 * RPG * BT);
    const int tid = threadIdx.x;
    const int b0 = blockIdx.y * BT;
    const int nb = min(BT, p.B - b0);

    // ---------------- stage the activation rows (prologue fused)
    for (int b = 0; b < BT; ++b) {
        uint16_t *xr = xs + (size_t)b * Kp;
        if (b >= nb) {
            for (int k = tid * 8; k < Kp; k += 2048) *reinterpret_cast<uint4 *>(xr + k) = make_uint4(0, 0, 0, 0);
            continue;
        }
        const int src_row = p.x_idx ? p.x_idx[b0 + b] : (b0 + b);
        if constexpr (PRO == PRO_F16) {
            const uint16_t *src = reinterpret_cast<const uint16_t *>(p.x) + (size_t)src_row * p.ldx;
            for (int k = tid * 8; k < Kp; k += 2048)
                *reinterpret_cast<uint4 *>(xr + k) = k < K ? *reinterpret_cast<const uint4 *>(src + k) : make_uint4(0, 0, 0, 0);
        } else {
            const float *src = reinterpret_cast<const float *>(p.x) + (size_t)src_row * p.ldx;
            float scale = 1.0f, mean = 0.0f;
            if constexpr (PRO == PRO_RMS) {
                double ss = 0.0;
                for (int k = tid; k < K; k += 256) { const float v = src[k]; ss += (double)(v * v); }
                ss = block_sum_d(ss, dscr);
                const float m = (float)(ss / K);
                scale = 1.0f / sqrtf(m + p.eps);
            } else if constexpr (PRO == PRO_LN) {
                double s1 = 0.0;
                for (int k = tid; k < K; k += 256) s1 += (double)src[k];
                s1 = block_sum_d(s1, dscr);
                mean = (float)(s1 / K);
                double s2 = 0.0;
                for (int k = tid; k < K; k += 256) { const float d = src[k] - mean; s2 += (double)(d * d); }
                s2 = block_sum_d(s2, dscr);
                const float var = (float)(s2 / K);
                scale = 1.0f / sqrtf(var + p.eps);
            }
            for (int k = tid; k < Kp; k += 256) {
                float y = 0.0f;
                if (k < K) {
                    const float v = src[k];
                    if constexpr (PRO == PRO_RMS) y = (v * scale) * p.nw[k];
                    else if constexpr (PRO == PRO_LN) y = ((v - mean) * scale) * p.nw[k] + p.nb[k];
                    else y = v;
                    if (p.side_out && blockIdx.x == 0) p.side_out[(size_t)(b0 + b) * K + k] = y;
                }
                xr[k] = f2h(y);
            }
        }
    }
    __syncthreads();

    // ---------------- stream the weight rows
    const int lane = tid & 63, wave = tid >> 6, l16 = lane & 15, grp = lane >> 4;
    int g, rows_pb, rstride, kbeg, kend;
    if constexpr (KS == 1) {
        g = wave * 4 + grp; rows_pb = 16 * RPG; rstride = 16; kbeg = 0; kend = Kp;
    } else {
        g = grp; rows_pb = 4 * RPG; rstride = 4;
        const int Kq = ((Kp / 128 + 3) / 4) * 128;
        kbeg = wave * Kq; kend = min(Kp, kbeg + Kq);
    }
    const int row0 = blockIdx.x * rows_pb + g;
    float acc[RPG][BT];
    const uint16_t *wrow[RPG];
#pragma unroll
    for (int i = 0; i < RPG; ++i) {
        const int r = min(row0 + i * rstride, N - 1);
        wrow[i] = p.W + (size_t)r * K;
#pragma unroll
        for (int b = 0; b < BT; ++b) acc[i][b] = 0.0f;
    }
#pragma unroll 2
    for (int k = kbeg + l16 * 8; k < kend; k += 128) {
        uint4 w[RPG];
#pragma unroll
        for (int i = 0; i < RPG; ++i)
            w[i] = k < K ? ld_nt16(wrow[i] + k) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int b = 0; b < BT; ++b) {
            const uint4 xv = *reinterpret_cast<const uint4 *>(xs + (size_t)b * Kp + k);
#pragma unroll
            for (int i = 0; i < RPG; ++i) acc[i][b] = dot8(w[i], xv, acc[i][b]);
        }
    }
#pragma unroll
    for (int i = 0; i < RPG; ++i)
#pragma unroll
        for (int b = 0; b < BT; ++b) acc[i][b] = group_sum<16>(acc[i][b]);
    if constexpr (KS == 4) {
        if (l16 == 0)
#pragma unroll
            for (int i = 0; i < RPG; ++i)
#pragma unroll
                for (int b = 0; b < BT; ++b) red[((wave * 4 + grp) * RPG + i) * BT + b] = acc[i][b];
        __syncthreads();
        if (wave != 0) return;
#pragma unroll
        for (int i = 0; i < RPG; ++i)
#pragma unroll
            for (int b = 0; b < BT; ++b) {
                float s = 0.0f;
#pragma unroll
                for (int w2 = 0; w2 < 4; ++w2) s += red[((w2 * 4 + grp) * RPG + i) * BT + b];
                acc[i][b] = s;
            }
    }

    // ---------------- epilogue: lane l16 writes batch column l16
#pragma unroll
    for (int bi = 0; bi < BT; ++bi) {
        if (bi != l16 || bi >= nb) continue;
        const int bb = b0 + bi;
        const size_t orow = (size_t)bb * p.orow_mul + p.orow_add;
        if (p.act == ACT_SWIGLU) {
            if constexpr (RPG == 2) {
                const int unit = blockIdx.x * 16 + g;
                if (unit < N / 2) {
                    const float h = silu_f(acc[0][bi]) * acc[1][bi];
                    if (p.out_f16) p.out_f16[orow * p.ldo + unit] = f2h(h);
                    else p.out_f32[orow * p.ldo + unit] = h;
                }
            }
            continue;
        }
#pragma unroll
        for (int i = 0; i < RPG; ++i) {
            const int r = row0 + i * rstride;
            if (r >= N) continue;
            float v = acc[i][bi];
            if (p.bias) v += p.bias[r];
            if (p.act == ACT_SILU) v = silu_f(v);
            else if (p.act == ACT_GELU) v = gelu_ggml(v);
            if (p.scale) v *= p.scale[r];
            if (p.resid) v = p.resid[(size_t)bb * p.ldr + r] + v;
            if (p.aux) v = p.aux[(size_t)bb * p.lda + r] + v;
            if (p.out_f16) p.out_f16[orow * p.ldo + r] = f2h(v);
            else p.out_f32[orow * p.ldo + r] = v;
        }
    }
}

template <int RPG, int BT, int KS>
static void launch_gemv_pro(const GemvParams &p, dim3 grid, size_t lds, hipStream_t s) {
    switch (p.pro) {
        case PRO_F16: hipLaunchKernelGGL((k_gemv<RPG, BT, KS, PRO_F16>), grid, dim3(256), lds, s, p); break;
        case PRO_F32: hipLaunchKernelGGL((k_gemv<RPG, BT, KS, PRO_F32>), grid, dim3(256), lds, s, p); break;
        case PRO_RMS: hipLaunchKernelGGL((k_gemv<RPG, BT, KS, PRO_RMS>), grid, dim3(256), lds, s, p); break;
        default: hipLaunchKernelGGL((k_gemv<RPG, BT, KS, PRO_LN>), grid, dim3(256), lds, s, p); break;
    }
}
template <int BT>
static bool launch_gemv_bt(const GemvParams &p, hipStream_t s) {
    const int Kp = (p.K + 127) & ~127;
    const int gy = (p.B + BT - 1) / BT;
    int rpg = 1, ks = 1;
    if (p.act == ACT_SWIGLU) rpg = 2;
    else if ((long)((p.N + 15) / 16) * gy < 256) ks = 4;
    const int rows_pb = (ks == 1 ? 16 : 4) * rpg;
    const dim3 grid((p.N + rows_pb - 1) / rows_pb, gy);
    const size_t lds = (size_t)BT * Kp * 2 + 4 * 4 * rpg * BT * 4 + 8 * sizeof(double);
    if (rpg == 2) launch_gemv_pro<2, BT, 1>(p, grid, lds, s);
    else if (ks == 4) launch_gemv_pro<1, BT, 4>(p, grid, lds, s);
    else launch_gemv_pro<1, BT, 1>(p, grid, lds, s);
    return true;
}
bool gemv(const GemvParams &p, hipStream_t s) {
    if (p.B <= 0 || p.N <= 0) return true;
    if (p.K % 8 != 0 || (p.act == ACT_SWIGLU && p.N % 32 != 0)) {
        set_error("gemv: unsupported shape N=" + std::to_string(p.N) + " K=" + std::to_string(p.K));
        return false;
    }
    if ((p.K + 127) / 128 * 128 * 2 > 48 * 1024) { set_error("gemv: K too large for the LDS tile"); return false; }
    // batch tile: up to 8 activation rows in LDS as f16, capped at 48 KB of LDS
    int bt = p.B == 1 ? 1 : p.B == 2 ? 2 : p.B <= 4 ? 4 : 8;
    const int Kp = (p.K + 127) / 128 * 128;
    while (bt > 1 && (size_t)Kp * 2 * bt > 48 * 1024) bt /= 2;
    if (bt == 1) launch_gemv_bt<1>(p, s);
    else if (bt == 2) launch_gemv_bt<2>(p, s);
    else if (bt == 4) launch_gemv_bt<4>(p, s);
    else launch_gemv_bt<8>(p, s);
    Q3T_HIP(hipGetLastError());
    return true;
}

// ======================================================================================= attention (decode)
// grid (slot, kv_head, split).  16 (D=128) or 8 (D=64) lanes per key position, 16-B K/V loads.
template <int D>
__global__ void __launch_bounds__(256) k_attn(const AttnParams p) {
    constexpr int LPP = D / 8;
    constexpr int PPI = 256 / LPP;
    const int slot = blockIdx.x, kvh = blockIdx.y, split = blockIdx.z;
    const int R = p.nH / p.nKV;
    const int pos = p.pos[slot];
    const int j0 = split * ATTN_CHUNK;
    if (j0 > pos) return;
    const int j1 = min(j0 + ATTN_CHUNK, pos + 1);
    const bool last = pos < j0 + ATTN_CHUNK;

    __shared__ float q_s[4][D];
    __shared__ float kn_s[D], vn_s[D];
    __shared__ float sc[4][ATTN_CHUNK];
    __shared__ float red[PPI][4][D];
    __shared__ float mstat[4], lstat[4];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int QKV = (p.nH + 2 * p.nKV) * D;
    const float *qkv = p.qkv + (size_t)slot * QKV;
    const float *rope = p.rope + (size_t)pos * D;

    // ---- head RMSNorm (sum in double, ggml_rms_norm) + NEOX RoPE, one wave per vector
    const int nvec = R + (last ? 1 : 0);
    for (int v = wave; v < nvec; v += 4) {
        const bool isk = (v == R);
        const float *src = isk ? qkv + (size_t)(p.nH + kvh) * D : qkv + (size_t)(kvh * R + v) * D;
        const float *w = isk ? p.kn : p.qn;
        constexpr int E = D / 64;
        float x[E];
        double ss = 0.0;
#pragma unroll
        for (int t = 0; t < E; ++t) { x[t] = src[lane + 64 * t]; ss += (double)(x[t] * x[t]); }
        ss = wave_sum_d(ss);
        const float scale = 1.0f / sqrtf((float)(ss / D) + p.eps);
#pragma unroll
        for (int t = 0; t < E; ++t) x[t] = (x[t] * scale) * w[lane + 64 * t];
        float y[E];
        if constexpr (D == 128) {
            const float c = rope[2 * lane], s = rope[2 * lane + 1];
            y[0] = x[0] * c - x[1] * s;
            y[1] = x[0] * s + x[1] * c;
        } else {
            const int i = lane & 31;
            const float c = rope[2 * i], s = rope[2 * i + 1];
            const float other = __shfl_xor(x[0], 32, 64);
            y[0] = lane < 32 ? x[0] * c - other * s : other * s + x[0] * c;
        }
        float *dst = isk ? kn_s : q_s[v];
#pragma unroll
        for (int t = 0; t < E; ++t) dst[lane + 64 * t] = f16r(y[t]);
    }
    if (last)
        for (int e = tid; e < D; e += 256) vn_s[e] = f16r(qkv[(size_t)(p.nH + p.nKV + kvh) * D + e]);
    __syncthreads();
    const size_t head_off = ((size_t)slot * p.nKV + kvh) * p.n_ctx * D;
    if (last)
        for (int e = tid; e < D; e += 256) {
            p.kc[head_off + (size_t)pos * D + e] = f2h(kn_s[e]);
            p.vc[head_off + (size_t)pos * D + e] = f2h(vn_s[e]);
        }

    // ---- scores for j in [j0, j1)
    const uint16_t *kb = p.kc + head_off, *vb = p.vc + head_off;
    const int pg = tid / LPP, li = tid % LPP;
    const float kq_scale = 1.0f / sqrtf((float)D);
    for (int j = j0 + pg; j < j1; j += PPI) {
        float k8[8];
        if (j == pos) {
#pragma unroll
            for (int e = 0; e < 8; ++e) k8[e] = kn_s[li * 8 + e];
        } else {
            const uint4 u = *reinterpret_cast<const uint4 *>(kb + (size_t)j * D + li * 8);
            const uint16_t *hv = reinterpret_cast<const uint16_t *>(&u);
#pragma unroll
            for (int e = 0; e < 8; ++e) k8[e] = h2f(hv[e]);
        }
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            if (h >= R) break;
            float s = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) s += k8[e] * q_s[h][li * 8 + e];
            s = group_sum<LPP>(s);
            if (li == 0) sc[h][j - j0] = s * kq_scale;
        }
    }
    __syncthreads();
    // ---- chunk softmax statistics
    const int n = j1 - j0;
    for (int h = wave; h < R; h += 4) {
        float m = -INFINITY;
        for (int j = lane; j < n; j += 64) m = fmaxf(m, sc[h][j]);
        m = wave_max(m);
        float l = 0.0f;
        for (int j = lane; j < n; j += 64) { const float e = expf(sc[h][j] - m); sc[h][j] = e; l += e; }
        l = wave_sum(l);
        if (lane == 0) { mstat[h] = m; lstat[h] = l; }
    }
    __syncthreads();
    // ---- P.V
    float acc[4][8];
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[h][e] = 0.0f;
    for (int j = j0 + pg; j < j1; j += PPI) {
        float v8[8];
        if (j == pos) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v8[e] = vn_s[li * 8 + e];
        } else {
            const uint4 u = *reinterpret_cast<const uint4 *>(vb + (size_t)j * D + li * 8);
            const uint16_t *hv = reinterpret_cast<const uint16_t *>(&u);
#pragma unroll
            for (int e = 0; e < 8; ++e) v8[e] = h2f(hv[e]);
        }
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            if (h >= R) break;
            const float pr = sc[h][j - j0];
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[h][e] += pr * v8[e];
        }
    }
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) red[pg][h][li * 8 + e] = acc[h][e];
    __syncthreads();
    for (int o = tid; o < R * D; o += 256) {
        const int h = o / D, d = o % D;
        float s = 0.0f;
        for (int g2 = 0; g2 < PPI; ++g2) s += red[g2][h][d];
        const int hq = kvh * R + h;
        if (gridDim.z == 1) {
            p.out[(size_t)slot * p.nH * D + (size_t)hq * D + d] = f2h(s / lstat[h]);
        } else {
            float *pp = p.part + (((size_t)slot * p.nH + hq) * p.max_splits + split) * (D + 2);
            pp[d] = s;
            if (d == 0) { pp[D] = mstat[h]; pp[D + 1] = lstat[h]; }
        }
    }
}

template <int D>
__global__ void __launch_bounds__(D) k_attn_combine(const AttnParams p) {
    const int slot = blockIdx.x, hq = blockIdx.y, d = threadIdx.x;
    const int ns = p.pos[slot] / ATTN_CHUNK + 1;
    const float *pp = p.part + ((size_t)slot * p.nH + hq) * p.max_splits * (D + 2);
    float M = -INFINITY;
    for (int s = 0; s < ns; ++s) M = fmaxf(M, pp[s * (D + 2) + D]);
    float L = 0.0f, a = 0.0f;
    for (int s = 0; s < ns; ++s) {
        const float w = expf(pp[s * (D + 2) + D] - M);
        L += pp[s * (D + 2) + D + 1] * w;
        a += pp[s * (D + 2) + d] * w;
    }
    p.out[(size_t)slot * p.nH * D + (size_t)hq * D + d] = f2h(a / L);
}

bool attn_decode(const AttnParams &p, hipStream_t s) {
    if (p.nH % p.nKV != 0 || p.nH / p.nKV > 4 || (p.D != 64 && p.D != 128)) {
        set_error("attn_decode: unsupported head layout");
        return false;
    }
    const dim3 grid(p.S, p.nKV, p.max_splits);
    if (p.D == 128) hipLaunchKernelGGL(k_attn<128>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(k_attn<64>, grid, dim3(256), 0, s, p);
    if (p.max_splits > 1) {
        const dim3 g2(p.S, p.nH);
        if (p.D == 128) hipLaunchKernelGGL(k_attn_combine<128>, g2, dim3(128), 0, s, p);
        else hipLaunchKernelGGL(k_attn_combine<64>, g2, dim3(64), 0, s, p);
    }
    Q3T_HIP(hipGetLastError());
    return true;
}

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
