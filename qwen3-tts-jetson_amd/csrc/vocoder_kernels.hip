// vocoder_kernels.hip — gfx950 kernels of the Qwen3-TTS tokenizer decoder (src/audio_tokenizer_decoder.cpp:375-802).
// Activations are time-major [T][C] f32; every conv input is rounded to f16 (ggml im2col F16) and fed to
// v_mfma_f32_32x32x16_f16 with f16 weights (exact products, f32 accumulation).
#include "vocoder_kernels.h"

#include <algorithm>

namespace q3t {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

// ======================================================================================= implicit-GEMM conv
// y[m*so + ob][co] = act( bias[co] + resid + sum_j sum_ci W_j[co][ci] * f16( snake(x[m + dj][ci]) ) )
// Tile 64 (m) x 64 (co); 4 waves as 2 x 2 of 32 x 32; K-chunk = 32 input channels.
constexpr int CT_M = 64, CT_N = 64, CT_K = 32, CT_LD = CT_K + 8;   // LDS row: 32 f16 + 16 B pad

__device__ __forceinline__ float conv_act(float v, int act) {
    if (act == 1) return tanhf(v);
    if (act == 2) return fmaxf(v, 0.0f);
    if (act == 3) return tanhf(fmaxf(v, 0.0f));
    return v;
}
constexpr int CT_MAXWIN = CT_M + 64;

__global__ void __launch_bounds__(256) k_conv(const ConvParams p) {
    __shared__ __attribute__((aligned(16))) uint16_t xs[CT_MAXWIN * CT_LD];
    __shared__ __attribute__((aligned(16))) uint16_t ws[CONV_MAX_TAPS * CT_N * CT_LD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.x * CT_M, co0 = blockIdx.y * CT_N;
    const int win = CT_M + p.dmax - p.dmin;
    f32x16_t acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
    const int r = lane & 31, h = lane >> 5;
    for (int c0 = 0; c0 < p.C_in; c0 += CT_K) {
        // ---- stage the input window: f16 rows as they are (snake applied by snake_f16), or snake + f16 rounding here
        if (p.xh) {
            for (int e = tid; e < win * (CT_K / 8); e += 256) {
                const int row = e / (CT_K / 8), c8 = (e % (CT_K / 8)) * 8;
                const int i = m0 + p.dmin + row;
                uint4 u = make_uint4(0, 0, 0, 0);
                if (i >= 0 && i < p.T_in && c0 + c8 < p.C_in) {
                    if ((p.C_in & 7) == 0) {
                        u = *reinterpret_cast<const uint4 *>(p.xh + (size_t)i * p.C_in + c0 + c8);
                    } else {   // narrow channel counts (tiny test configs): element-wise, zero past C_in
                        uint16_t t8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                        for (int q = 0; q < 8; ++q) if (c0 + c8 + q < p.C_in) t8[q] = p.xh[(size_t)i * p.C_in + c0 + c8 + q];
                        u = *reinterpret_cast<const uint4 *>(t8);
                    }
                }
                *reinterpret_cast<uint4 *>(xs + row * CT_LD + c8) = u;
            }
        } else
        for (int e = tid; e < win * (CT_K / 4); e += 256) {
            const int row = e / (CT_K / 4), cq = (e % (CT_K / 4)) * 4;
            const int i = m0 + p.dmin + row;
            float v[4] = {0.f, 0.f, 0.f, 0.f};
            if (i >= 0 && i < p.T_in) {
                const int ci = c0 + cq;
                if (ci + 3 < p.C_in && (p.C_in & 3) == 0) {
                    const float4 u = *reinterpret_cast<const float4 *>(p.x + (size_t)i * p.C_in + ci);
                    v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
                } else {
                    for (int q = 0; q < 4; ++q) if (ci + q < p.C_in) v[q] = p.x[(size_t)i * p.C_in + ci + q];
                }
                if (p.snake_a) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (ci + q < p.C_in) {
                            const float sn = sinf(v[q] * p.snake_a[ci + q]);
                            v[q] = v[q] + (sn * sn) * p.snake_ib[ci + q];
                        }
                    }
                }
            }
            uint16_t *d = xs + row * CT_LD + cq;
            d[0] = f2h(v[0]); d[1] = f2h(v[1]); d[2] = f2h(v[2]); d[3] = f2h(v[3]);
        }
        // ---- stage the weight tiles of every tap: [tap][co][32 ci]
        for (int e = tid; e < p.n_taps * CT_N * (CT_K / 8); e += 256) {
            const int j = e / (CT_N * (CT_K / 8)), rem = e % (CT_N * (CT_K / 8));
            const int co = rem / (CT_K / 8), c8 = (rem % (CT_K / 8)) * 8;
            uint4 u = make_uint4(0, 0, 0, 0);
            const int gco = co0 + co, gci = c0 + c8;
            if (gco < p.C_out) {
                const uint16_t *w = p.taps[j].w + (size_t)gco * p.C_in + gci;
                if (gci + 7 < p.C_in && (p.C_in & 7) == 0) u = *reinterpret_cast<const uint4 *>(w);
                else {
                    uint16_t t8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                    for (int q = 0; q < 8; ++q) if (gci + q < p.C_in) t8[q] = w[q];
                    u = *reinterpret_cast<const uint4 *>(t8);
                }
            }
            *reinterpret_cast<uint4 *>(ws + (j * CT_N + co) * CT_LD + c8) = u;
        }
        __syncthreads();
        for (int j = 0; j < p.n_taps; ++j) {
            const int arow = wm * 32 + r + (p.taps[j].dj - p.dmin);
            const uint16_t *ab = xs + arow * CT_LD + 8 * h;
            const uint16_t *bb = ws + (j * CT_N + wn * 32 + r) * CT_LD + 8 * h;
#pragma unroll
            for (int kk = 0; kk < CT_K; kk += 16) {
                const half8_t a = *reinterpret_cast<const half8_t *>(ab + kk);
                const half8_t b = *reinterpret_cast<const half8_t *>(bb + kk);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
            }
        }
        __syncthreads();
    }
    // ---- epilogue (C/D map: col = lane & 31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5))
    const int co = co0 + wn * 32 + (lane & 31);
    if (co >= p.C_out) return;
    const float b = p.bias ? p.bias[co] : 0.0f;
    const float sa = p.y16_a ? p.y16_a[co] : 0.0f, sib = p.y16_a ? p.y16_ib[co] : 0.0f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
        const int m = m0 + wm * 32 + row;
        if (m >= p.M) continue;
        const size_t t = (size_t)m * p.so + p.ob;
        const int ldy = p.ldy ? p.ldy : p.C_out;
        float v = acc[reg] + b;
        if (p.resid) v = p.resid[t * ldy + co] + v;
        v = conv_act(v, p.act);
        if (p.y) p.y[t * ldy + co] = v;
        if (p.y16) {
            float z = v;
            if (p.y16_a) {
                const float sn = sinf(z * sa);
                z = z + (sn * sn) * sib;
            }
            p.y16[t * p.C_out + co] = f2h(z);
        }
    }
}

// ======================================================================================= multi-tile implicit-GEMM conv
// The decoder convs are tall-skinny GEMMs: M = time (up to ~1M rows), N = C_out (96..1536), K = taps x C_in.  One
// workgroup computes MT = 128*RB rows x NT output channels: every wave owns 32*RB rows x NT columns (RB x NT/32
// v_mfma_f32_32x32x16_f16 accumulators), so each B fragment (weights) read from LDS feeds RB MFMAs and each A fragment
// (input rows) NT/32.  Per 32-channel K chunk the input window (MT + tap span rows) and the chunk's weights of every
// tap are staged once in LDS (~79 KB at NT 96: two workgroups per CU, one staging while the other multiplies).
// Input: f16 rows (snake already applied).  Epilogue: bias, residual, tanh, f32 and/or f16(snake_next) outputs.
constexpr int MT_KC = 32, MT_LDK = MT_KC + 8;   // LDS row: 32 f16 + 16 B pad (conflict-free ds_read_b128)

template <int RB, int NT>
__global__ void __launch_bounds__(256, 2) k_conv_mt(const ConvParams p) {
    constexpr int MT = 128 * RB, CB = NT / 32;
    extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
    // the tap table in LDS: indexing the by-value kernel argument with a runtime tap index makes the compiler copy
    // the whole ConvParams to scratch memory
    __shared__ const uint16_t *tapw[CONV_MAX_TAPS];
    __shared__ int tapdj[CONV_MAX_TAPS];
    const int win = MT + p.dmax - p.dmin;
    uint16_t *xs = sm;                          // [win][MT_LDK]
    uint16_t *ws = sm + (size_t)win * MT_LDK;   // [taps][NT][MT_LDK]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int j = 0; j < CONV_MAX_TAPS; ++j)
        if (tid == j) { tapw[j] = p.taps[j].w; tapdj[j] = p.taps[j].dj; }
    __syncthreads();
    const int m0 = blockIdx.x * MT, co0 = blockIdx.y * NT;
    const int r = lane & 31, h = lane >> 5;
    f32x16_t acc[RB][CB];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
    // x window staged through registers one chunk ahead (chunk c+1's loads in flight while chunk c multiplies);
    // the chunk's weights (L2-resident: every workgroup reads the same ones) are loaded all at once and stored
    constexpr int XR = (MT + 64) * (MT_KC / 8) / 256;              // window rows <= MT + 64
    constexpr int WR = (CONV_MAX_TAPS * NT * (MT_KC / 8) + 255) / 256;
    const int nx = win * (MT_KC / 8), nw = p.n_taps * NT * (MT_KC / 8);
    uint4 xr[XR];
#define Q3T_CONV_XLOAD(C0)                                                                                            \
    do {                                                                                                              \
        _Pragma("unroll") for (int q = 0; q < XR; ++q) {                                                              \
            const int e = tid + q * 256, row = e >> 2, c8 = (e & 3) * 8, i = m0 + p.dmin + row;                       \
            const bool in = e < nx && i >= 0 && i < p.T_in;                                                           \
            const int ic = min(max(i, 0), p.T_in - 1);                                                                \
            const uint4 u = ldg16(p.xh + (size_t)ic * p.C_in + (C0) + c8);                                           \
            xr[q] = in ? u : make_uint4(0, 0, 0, 0);                                                                  \
        }                                                                                                             \
    } while (0)
    Q3T_CONV_XLOAD(0);
    for (int c0 = 0; c0 < p.C_in; c0 += MT_KC) {
#pragma unroll
        for (int q = 0; q < XR; ++q) {
            const int e = tid + q * 256;
            if (e < nx) *reinterpret_cast<uint4 *>(xs + (e >> 2) * MT_LDK + (e & 3) * 8) = xr[q];
        }
        // (no register array here: the compiler kept one in scratch memory; the loads of the unrolled loop still issue
        // ahead of their LDS stores)
#pragma unroll
        for (int q = 0; q < WR; ++q) {
            const int e = min(tid + q * 256, nw - 1);
            const int j = e / (NT * 4), rem = e - j * (NT * 4), co = rem >> 2, c8 = (rem & 3) * 8;
            const uint4 u = ldg16(tapw[j] + (size_t)(co0 + co) * p.C_in + c0 + c8);
            if (tid + q * 256 < nw) *reinterpret_cast<uint4 *>(ws + (j * NT + co) * MT_LDK + c8) = u;
        }
        __syncthreads();
        if (c0 + MT_KC < p.C_in) Q3T_CONV_XLOAD(c0 + MT_KC);
        for (int j = 0; j < p.n_taps; ++j) {
            const uint16_t *ab = xs + (wave * 32 * RB + r + (tapdj[j] - p.dmin)) * MT_LDK + 8 * h;
            const uint16_t *bb = ws + (j * NT + r) * MT_LDK + 8 * h;
#pragma unroll
            for (int kk = 0; kk < MT_KC; kk += 16) {
                half8_t a[RB], b[CB];
#pragma unroll
                for (int i = 0; i < RB; ++i) a[i] = *reinterpret_cast<const half8_t *>(ab + i * 32 * MT_LDK + kk);
#pragma unroll
                for (int c = 0; c < CB; ++c) b[c] = *reinterpret_cast<const half8_t *>(bb + c * 32 * MT_LDK + kk);
#pragma unroll
                for (int i = 0; i < RB; ++i)
#pragma unroll
                    for (int c = 0; c < CB; ++c) acc[i][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[c], acc[i][c], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    // ---- epilogue through LDS (the staging area is free now): each wave transposes one 32-row slice of its tile
    // (C/D map: col = lane & 31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)) so that every lane then owns 4 consecutive
    // channels of a row: 16-B residual loads / f32 stores and 8-B f16 stores instead of one instruction per element
    constexpr int ELD = NT + 4;   // f32 row stride of the transposed slice
    float *es = reinterpret_cast<float *>(sm) + wave * 32 * ELD;
#pragma unroll
    for (int i = 0; i < RB; ++i) {
#pragma unroll
        for (int c = 0; c < CB; ++c)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg)
                es[((reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)) * ELD + c * 32 + (lane & 31)] = acc[i][c][reg];
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the slice is in LDS (one wave writes and reads it)
        __builtin_amdgcn_wave_barrier();
        constexpr int Q = NT / 4;             // channel quads per row
#pragma unroll 4
        for (int k = 0; k < 32 * Q / 64; ++k) {
            const int e = lane + 64 * k, row = e / Q, q4 = (e % Q) * 4;
            const int m = m0 + wave * 32 * RB + i * 32 + row;
            if (m >= p.M) continue;
            const size_t t = (size_t)m * p.so + p.ob, o = t * (p.ldy ? p.ldy : p.C_out) + co0 + q4;
            const size_t o16 = t * p.C_out + co0 + q4;
            const float4 a = *reinterpret_cast<const float4 *>(es + row * ELD + q4);
            float v[4] = {a.x, a.y, a.z, a.w};
            if (p.bias) {
                const float4 b = *reinterpret_cast<const float4 *>(p.bias + co0 + q4);
                v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
            }
            if (p.resid) {
                const float4 rr = *reinterpret_cast<const float4 *>(p.resid + o);
                v[0] = rr.x + v[0]; v[1] = rr.y + v[1]; v[2] = rr.z + v[2]; v[3] = rr.w + v[3];
            }
            if (p.act) {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = conv_act(v[q], p.act);
            }
            if (p.y) *reinterpret_cast<float4 *>(p.y + o) = make_float4(v[0], v[1], v[2], v[3]);
            if (p.y16) {
                float z[4] = {v[0], v[1], v[2], v[3]};
                if (p.y16_a) {   // the k_snake_f16 expression, term for term
                    const float4 sa = *reinterpret_cast<const float4 *>(p.y16_a + co0 + q4);
                    const float4 sb = *reinterpret_cast<const float4 *>(p.y16_ib + co0 + q4);
                    const float av[4] = {sa.x, sa.y, sa.z, sa.w}, bv[4] = {sb.x, sb.y, sb.z, sb.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float sn = sinf(z[q] * av[q]);
                        z[q] = z[q] + (sn * sn) * bv[q];
                    }
                }
                uint2 hv;
                hv.x = (uint32_t)f2h(z[0]) | ((uint32_t)f2h(z[1]) << 16);
                hv.y = (uint32_t)f2h(z[2]) | ((uint32_t)f2h(z[3]) << 16);
                *reinterpret_cast<uint2 *>(p.y16 + o16) = hv;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

template <int RB, int NT>
static bool launch_mt(const ConvParams &p, hipStream_t s) {
    constexpr int MT = 128 * RB;
    // staging area (input window + the chunk's weights of every tap), reused by the epilogue's transposed slices
    const size_t lds = std::max(((size_t)(MT + p.dmax - p.dmin) + (size_t)p.n_taps * NT) * MT_LDK * 2,
                                (size_t)4 * 32 * (NT + 4) * 4);
    static bool attr = false;
    if (!attr) {
        Q3T_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_conv_mt<RB, NT>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
        attr = true;
    }
    const dim3 grid((p.M + MT - 1) / MT, p.C_out / NT);
    hipLaunchKernelGGL((k_conv_mt<RB, NT>), grid, dim3(256), lds, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}

bool conv(const ConvParams &p, hipStream_t s) {
    if (p.M <= 0) return true;
    if (p.n_taps < 1 || p.n_taps > CONV_MAX_TAPS || p.dmax - p.dmin > CT_MAXWIN - CT_M) {
        set_error("conv: unsupported tap layout");
        return false;
    }
    const int NT = p.C_out % 96 == 0 ? 96 : p.C_out % 64 == 0 ? 64 : 0;
    if (p.xh && NT && p.C_in % MT_KC == 0 && (p.y || p.y16)) {
        // RB 2 (256-row tiles) unless that leaves fewer than two workgroups per CU to fill the chip
        const long tiles256 = (long)((p.M + 255) / 256) * (p.C_out / NT);
        const bool big = tiles256 >= 512;
        if (NT == 96) return big ? launch_mt<2, 96>(p, s) : launch_mt<1, 96>(p, s);
        return big ? launch_mt<2, 64>(p, s) : launch_mt<1, 64>(p, s);
    }
    if (!p.y && !p.y16) { set_error("conv: no output"); return false; }
    const dim3 grid((p.M + CT_M - 1) / CT_M, (p.C_out + CT_N - 1) / CT_N);
    hipLaunchKernelGGL(k_conv, grid, dim3(256), 0, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}

__global__ void __launch_bounds__(256) k_snake_f16(const float *x, const float *a, const float *ib, uint16_t *out, int64_t n4, int C) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const int c = (int)((i * 4) % C);
    const float4 v = reinterpret_cast<const float4 *>(x)[i];
    float y[4] = {v.x, v.y, v.z, v.w};
    if (a) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {   // the k_conv staging expression, term for term
            const float sn = sinf(y[q] * a[c + q]);
            y[q] = y[q] + (sn * sn) * ib[c + q];
        }
    }
    uint2 h;
    h.x = (uint32_t)f2h(y[0]) | ((uint32_t)f2h(y[1]) << 16);
    h.y = (uint32_t)f2h(y[2]) | ((uint32_t)f2h(y[3]) << 16);
    reinterpret_cast<uint2 *>(out)[i] = h;
}
bool snake_f16(const float *x, const float *a, const float *ib, uint16_t *out, int64_t T, int C, hipStream_t s) {
    if (C % 4 != 0) { set_error("snake_f16: C % 4 != 0"); return false; }
    if ((T * C) % 4 != 0) { set_error("snake_f16: T * C % 4 != 0"); return false; }
    const int64_t n4 = T * C / 4;
    if (n4 <= 0) return true;
    hipLaunchKernelGGL(k_snake_f16, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, x, a, ib, out, n4, C);
    Q3T_HIP(hipGetLastError());
    return true;
}

// ======================================================================================= depthwise causal conv
// y[t][c] = b[c] + sum_j w[c][j] * f16(x[t + j - (K-1)][c])      (ggml_pad_ext + ggml_conv_1d_dw, im2col F16)
__global__ void __launch_bounds__(256) k_dwconv(const float *x, const uint16_t *w, const float *b, float *y, int T, int C, int K) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)T * C) return;
    const int t = (int)(idx / C), c = (int)(idx % C);
    float acc = 0.0f;
    for (int j = 0; j < K; ++j) {
        const int i = t + j - (K - 1);
        if (i >= 0) acc += h2f(w[(size_t)c * K + j]) * f16r(x[(size_t)i * C + c]);
    }
    y[idx] = acc + b[c];
}
bool dwconv(const float *x, const uint16_t *w, const float *b, float *y, int T, int C, int K, hipStream_t s) {
    const size_t n = (size_t)T * C;
    if (!n) return true;
    hipLaunchKernelGGL(k_dwconv, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, w, b, y, T, C, K);
    Q3T_HIP(hipGetLastError());
    return true;
}

// ======================================================================================= pre-transformer attention
// causal softmax attention over F frames (apply_pre_tfm_layer, audio_tokenizer_decoder.cpp:412-456): NEOX RoPE
// (theta 1e4) on q,k, f32 scores (ggml mul_mat of two F32 tensors: no rounding), output rounded to f16.
// grid (query tiles of 16, heads); 16 lanes per query row, 4 keys / 4 dims per lane.
__global__ void __launch_bounds__(256) k_attn_prefill(const float *qkv, const float *rope, uint16_t *out, int F, int nH) {
    constexpr int D = 64, QT = 16, KT = 64;
    __shared__ float qs[QT][D];
    __shared__ float ks[KT][D + 1];
    __shared__ float vs[KT][D + 1];
    __shared__ float ps[QT][KT];
    const int h = blockIdx.y, q0 = blockIdx.x * QT;
    const int tid = threadIdx.x, qi = tid / 16, l16 = tid % 16;
    const int LD = 3 * nH * D;
    auto rope_load = [&](const float *src, int pos, int e) -> float {
        // NEOX pair (e, e+32)
        const int i = e & 31;
        const float c = rope[(size_t)pos * D + 2 * i], sn = rope[(size_t)pos * D + 2 * i + 1];
        const float x0 = src[i], x1 = src[i + 32];
        return e < 32 ? x0 * c - x1 * sn : x0 * sn + x1 * c;
    };
    for (int e = tid; e < QT * D; e += 256) {
        const int qq = e / D, d = e % D, pos = q0 + qq;
        qs[qq][d] = pos < F ? rope_load(qkv + (size_t)pos * LD + h * D, pos, d) : 0.0f;
    }
    float m = -INFINITY, l = 0.0f, acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int qpos = q0 + qi;
    const float scale = 1.0f / sqrtf((float)D);
    const int kend = min(F, q0 + QT);
    for (int k0 = 0; k0 < kend; k0 += KT) {
        __syncthreads();
        for (int e = tid; e < KT * D; e += 256) {
            const int kk = e / D, d = e % D, pos = k0 + kk;
            const float *row = qkv + (size_t)pos * LD;
            ks[kk][d] = pos < F ? rope_load(row + nH * D + h * D, pos, d) : 0.0f;
            vs[kk][d] = pos < F ? row[2 * nH * D + h * D + d] : 0.0f;
        }
        __syncthreads();
        float s[4];
        float mt = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int kk = l16 * 4 + t, kpos = k0 + kk;
            float d = 0.0f;
#pragma unroll 16
            for (int e = 0; e < D; ++e) d += ks[kk][e] * qs[qi][e];
            s[t] = (kpos <= qpos && kpos < F) ? d * scale : -INFINITY;
            mt = fmaxf(mt, s[t]);
        }
        mt = group_max<16>(mt);
        const float mn = fmaxf(m, mt);
        const float corr = (m == -INFINITY) ? 0.0f : expf(m - mn);
        float ls = 0.0f;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float pv = (s[t] == -INFINITY) ? 0.0f : expf(s[t] - mn);
            ps[qi][l16 * 4 + t] = pv;
            ls += pv;
        }
        ls = group_sum<16>(ls);
        l = l * corr + ls;
        m = mn;
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] *= corr;
        __syncthreads();
        for (int kk = 0; kk < KT; ++kk) {
            const float pv = ps[qi][kk];
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] += pv * vs[kk][l16 * 4 + t];
        }
    }
    if (qpos < F) {
        const float inv = 1.0f / l;
#pragma unroll
        for (int t = 0; t < 4; ++t) out[(size_t)qpos * nH * D + h * D + l16 * 4 + t] = f2h(acc[t] * inv);
    }
}
bool attn_prefill(const float *qkv, const float *rope, uint16_t *out, int F, int nH, int D, hipStream_t s) {
    if (D != 64) { set_error("attn_prefill: head_dim must be 64"); return false; }
    if (F <= 0) return true;
    hipLaunchKernelGGL(k_attn_prefill, dim3((F + 15) / 16, nH), dim3(256), 0, s, qkv, rope, out, F, nH);
    Q3T_HIP(hipGetLastError());
    return true;
}

// codes [F][ncb] -> per-codebook index columns [ncb][F]
__global__ void k_codes_cols(const int32_t *codes, int *cols, int F, int ncb) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < F * ncb) cols[(i % ncb) * F + i / ncb] = codes[i];
}
bool codes_cols(const int32_t *codes, int *cols, int F, int ncb, hipStream_t s) {
    if (F <= 0) return true;
    hipLaunchKernelGGL(k_codes_cols, dim3((F * ncb + 255) / 256), dim3(256), 0, s, codes, cols, F, ncb);
    Q3T_HIP(hipGetLastError());
    return true;
}

}  // namespace q3t
