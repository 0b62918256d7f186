// vocoder_kernels.hip — gfx950 kernels of the Qwen3-TTS tokenizer decoder (src/audio_tokenizer_decoder.cpp:375-802).
// Activations are time-major [T][C] f32; every conv input is rounded to f16 (ggml im2col F16) and fed to
// v_mfma_f32_32x32x16_f16 with f16 weights (exact products, f32 accumulation).
#include "vocoder_kernels.h"

#include <algorithm>
#include <cstdlib>

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
    if (act == 4) return gelu_ggml(v);
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
    const int ldy = p.ldy ? p.ldy : p.C_out;
    const size_t ub = blockIdx.z;   // utterance
    const float *px = p.x ? p.x + ub * p.xbs * p.C_in : nullptr;
    const uint16_t *pxh = p.xh ? p.xh + ub * p.xbs * p.C_in : nullptr;
    float *py = p.y ? p.y + ub * p.ybs * ldy : nullptr;
    const float *pres = p.resid ? p.resid + ub * p.ybs * ldy : nullptr;
    uint16_t *py16 = p.y16 ? p.y16 + ub * p.ybs * p.C_out : nullptr;
    f32x16_t acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
    const int r = lane & 31, h = lane >> 5;
    for (int c0 = 0; c0 < p.C_in; c0 += CT_K) {
        // ---- stage the input window: f16 rows as they are (snake applied by snake_f16), or snake + f16 rounding here
        if (pxh) {
            for (int e = tid; e < win * (CT_K / 8); e += 256) {
                const int row = e / (CT_K / 8), c8 = (e % (CT_K / 8)) * 8;
                const int i = m0 + p.dmin + row;
                uint4 u = make_uint4(0, 0, 0, 0);
                if (i >= 0 && i < p.T_in && c0 + c8 < p.C_in) {
                    if ((p.C_in & 7) == 0) {
                        u = *reinterpret_cast<const uint4 *>(pxh + (size_t)i * p.C_in + c0 + c8);
                    } else {   // narrow channel counts (tiny test configs): element-wise, zero past C_in
                        uint16_t t8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                        for (int q = 0; q < 8; ++q) if (c0 + c8 + q < p.C_in) t8[q] = pxh[(size_t)i * p.C_in + c0 + c8 + q];
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
                    const float4 u = *reinterpret_cast<const float4 *>(px + (size_t)i * p.C_in + ci);
                    v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
                } else {
                    for (int q = 0; q < 4; ++q) if (ci + q < p.C_in) v[q] = px[(size_t)i * p.C_in + ci + q];
                }
                if (p.snake_a) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (ci + q < p.C_in) {
                            v[q] = snake_apply(v[q], p.snake_a[ci + q], p.snake_ib[ci + q]);
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
        float v = acc[reg] + b;
        if (p.scale) v *= p.scale[co];
        if (pres) v = pres[t * ldy + co] + v;
        v = conv_act(v, p.act);
        if (py) py[t * ldy + co] = v;
        if (py16) {
            float z = v;
            if (p.y16_a) {
                z = snake_apply(z, sa, sib);
            }
            py16[t * p.C_out + co] = f2h(z);
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

// TW: most taps the variant stages per chunk (1, 3 or 7): the chunk's weights go through TW*NT*4/256 registers per
// thread, loaded one chunk ahead like the input window.  1-tap variants (RB 1) also load their residual rows before
// the main loop, so the epilogue's f32 reads are in flight while the GEMM runs (these convs are bound by that traffic).
// ACT: 0 = no activation code in the epilogue (the decoder's convs), -1 = p.act at run time
// Tile of a workgroup: (row tile, channel tile, output phase of a transposed conv).  With xcd (ConvParams::xcd_tiles)
// the n = channel tiles x phases that read one row tile's input rows run on one XCD and are dispatched together --
// workgroup L (x fastest, then y, then z) runs on XCD L % 8; it takes row tile 8 (L / (8 n)) + L % 8 and
// (channel tile, phase) number (L / 8) % n -- so those rows are fetched once into that XCD's L2 and hit there for the
// others (in grid order they ran on other XCDs, at other times).  A bijection on each utterance's tiles (the last
// group of < 8 row tiles likewise); the arithmetic of a tile does not depend on it.
__device__ __forceinline__ void conv_tile(bool xcd, int nz, int &mt, int &ct, int &phi) {
    mt = blockIdx.x;
    ct = blockIdx.y;
    phi = blockIdx.z % nz;
    const int gx = gridDim.x, gy = gridDim.y, n = gy * nz;
    if (!xcd || n <= 1) return;
    const int L = (phi * gy + ct) * gx + mt, grp = L / (8 * n), rem = min(8, gx - 8 * grp), r = L - grp * 8 * n;
    mt = 8 * grp + r % rem;
    const int cz = r / rem;
    ct = cz % gy;
    phi = cz / gy;
}

template <int RB, int NT, int MINB, int TW, int ACT>
__global__ void __launch_bounds__(256, MINB) k_conv_mt(const ConvParams p) {
    constexpr int MT = 128 * RB, CB = NT / 32;
    extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
    // the tap table in LDS: indexing the by-value kernel argument with a runtime tap index makes the compiler copy
    // the whole ConvParams to scratch memory
    __shared__ const uint16_t *tapw[CONV_MAX_TAPS];
    __shared__ int tapdj[CONV_MAX_TAPS];
    // launch geometry of this workgroup's conv: the params' own, or output phase blockIdx.z of a transposed conv
    int n_taps = p.n_taps, dmin = p.dmin, dmax = p.dmax, M = p.M, so = p.so, ob = p.ob;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nz = p.ct_st ? p.ct_st : 1;
    const int ubi = blockIdx.z / nz;   // utterance; blockIdx.z % nz = output phase of a transposed conv
    const size_t ub = ubi;
    const int ldy = p.ldy ? p.ldy : p.C_out;
    const uint16_t *pxh = p.xh + ub * p.xbs * p.C_in;
    float *py = p.y ? p.y + ub * p.ybs * ldy : nullptr;
    const float *pres = p.resid ? p.resid + ub * p.ybs * ldy : nullptr;
    uint16_t *py16 = p.y16 ? p.y16 + ub * p.ybs * p.C_out : nullptr;
    int mt, ct, phi;
    conv_tile(p.xcd_tiles != 0, nz, mt, ct, phi);
    if (p.ct_st) {
        const int st = p.ct_st, k0 = (phi + p.ct_trim) % st;
        n_taps = 0;
        for (int k = k0; k < p.ct_k && n_taps < CONV_MAX_TAPS; k += st) {
            const int dj = (phi + p.ct_trim - k) / st;
            if (tid == n_taps) { tapw[n_taps] = p.ct_w + (size_t)k * p.C_out * p.C_in; tapdj[n_taps] = dj; }
            dmin = n_taps == 0 ? dj : min(dmin, dj);
            dmax = n_taps == 0 ? dj : max(dmax, dj);
            ++n_taps;
        }
        M = (p.T_out - phi + st - 1) / st;
        so = st;
        ob = phi;
    } else {
#pragma unroll
        for (int j = 0; j < CONV_MAX_TAPS; ++j)
            if (tid == j) { tapw[j] = p.taps[j].w; tapdj[j] = p.taps[j].dj; }
    }
    const int m0 = mt * MT, co0 = ct * NT;
    if (m0 >= M || n_taps == 0) return;   // (uniform per workgroup: shorter phases of a transposed conv)
    __syncthreads();
    const int win = MT + dmax - dmin;
    uint16_t *xs = sm;                          // [win][MT_LDK]
    uint16_t *ws = sm + (size_t)win * MT_LDK;   // [taps][NT][MT_LDK]
    const int r = lane & 31, h = lane >> 5;
    f32x16_t acc[RB][CB];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
    // x window and the chunk's weights (L2-resident: every workgroup reads the same ones) staged through registers one
    // chunk ahead: chunk c+1's loads are in flight while chunk c multiplies
    constexpr int XR = (MT + 64) * (MT_KC / 8) / 256;              // window rows <= MT + 64
    constexpr int WR = (TW * NT * (MT_KC / 8) + 255) / 256;
    const int nx = win * (MT_KC / 8), nw = n_taps * NT * (MT_KC / 8);
    constexpr int Q = NT / 4;             // channel quads per row (epilogue)
    constexpr int EK = 32 * Q / 64;       // epilogue iterations per 32-row slice
    constexpr bool RP = TW == 1 && RB == 1;
    // weights through registers one chunk ahead, except where that would spill (256-row x 96-channel 7-tap tiles:
    // 96 accumulator + 44 weight + 20 window registers): there the chunk's weights are loaded and stored at once
    constexpr bool WPF = !(TW == 7 && RB == 2 && NT == 96);
    float4 rres[RP ? EK : 1];
    if constexpr (RP) {
        if (pres) {
#pragma unroll
            for (int k = 0; k < EK; ++k) {
                const int e = lane + 64 * k, row = e / Q, q4 = (e % Q) * 4;
                const int m = min(m0 + wave * 32 + row, M - 1);
                rres[k] = *reinterpret_cast<const float4 *>(pres + ((size_t)m * so + ob) * ldy + co0 + q4);
            }
        }
    }
    uint4 xr[XR], wr[WPF ? WR : 1];
#define Q3T_CONV_WLOAD(C0)                                                                                            \
    do {                                                                                                              \
        if (Q3T_DEV_SKIP(1)) break;                                                                                   \
        _Pragma("unroll") for (int q = 0; q < WR; ++q) {                                                              \
            const int e = min(tid + q * 256, nw - 1);                                                                 \
            const int j = e / (NT * 4), rem = e - j * (NT * 4), co = rem >> 2, c8 = (rem & 3) * 8;                   \
            wr[q] = ldg16(tapw[j] + (size_t)(co0 + co) * p.C_in + (C0) + c8);                                        \
        }                                                                                                             \
    } while (0)
#ifdef Q3T_DEV
#define Q3T_DEV_SKIP(bit) (p.dev_skip & (bit))
#else
#define Q3T_DEV_SKIP(bit) false
#endif
#define Q3T_CONV_XLOAD(C0)                                                                                            \
    do {                                                                                                              \
        if (Q3T_DEV_SKIP(2)) break;                                                                                   \
        _Pragma("unroll") for (int q = 0; q < XR; ++q) {                                                              \
            const int e = tid + q * 256, row = e >> 2, c8 = (e & 3) * 8, i = m0 + dmin + row;                       \
            const bool in = e < nx && i >= 0 && i < p.T_in;                                                           \
            const int ic = min(max(i, 0), p.T_in - 1);                                                                \
            const uint4 u = ldg16(pxh + (size_t)ic * p.C_in + (C0) + c8);                                           \
            xr[q] = in ? u : make_uint4(0, 0, 0, 0);                                                                  \
        }                                                                                                             \
    } while (0)
    Q3T_CONV_XLOAD(0);
    if constexpr (WPF) Q3T_CONV_WLOAD(0);
    for (int c0 = 0; c0 < p.C_in; c0 += MT_KC) {
#pragma unroll
        for (int q = 0; q < XR; ++q) {
            const int e = tid + q * 256;
            if (e < nx) *reinterpret_cast<uint4 *>(xs + (e >> 2) * MT_LDK + (e & 3) * 8) = xr[q];
        }
        if constexpr (WPF) {
#pragma unroll
            for (int q = 0; q < WR; ++q) {
                const int e = tid + q * 256;
                if (e < nw) {
                    const int j = e / (NT * 4), rem = e - j * (NT * 4), co = rem >> 2, c8 = (rem & 3) * 8;
                    *reinterpret_cast<uint4 *>(ws + (j * NT + co) * MT_LDK + c8) = wr[q];
                }
            }
        } else if (!Q3T_DEV_SKIP(1)) {
#pragma unroll
            for (int q = 0; q < WR; ++q) {
                const int e = min(tid + q * 256, nw - 1);
                const int j = e / (NT * 4), rem = e - j * (NT * 4), co = rem >> 2, c8 = (rem & 3) * 8;
                const uint4 u = ldg16(tapw[j] + (size_t)(co0 + co) * p.C_in + c0 + c8);
                if (tid + q * 256 < nw) *reinterpret_cast<uint4 *>(ws + (j * NT + co) * MT_LDK + c8) = u;
            }
        }
        __syncthreads();
        if (c0 + MT_KC < p.C_in) {
            Q3T_CONV_XLOAD(c0 + MT_KC);
            if constexpr (WPF) Q3T_CONV_WLOAD(c0 + MT_KC);
        }
        for (int j = 0; j < n_taps; ++j) {
            const uint16_t *ab = xs + (wave * 32 * RB + r + (tapdj[j] - dmin)) * MT_LDK + 8 * h;
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
    // the epilogue's per-channel operands of this tile, once in LDS (after the four slices): bias, scale,
    // exp(alpha) and exp(-beta) of the next SnakeBeta
    float *prm = reinterpret_cast<float *>(sm) + 4 * 32 * ELD;
    if (Q3T_DEV_SKIP(4)) {   // keep the accumulators live without the epilogue
        float z = 0.0f;
#pragma unroll
        for (int i = 0; i < RB; ++i)
#pragma unroll
            for (int c = 0; c < CB; ++c) z += acc[i][c][0];
        if (z == 12345.678f && py16) py16[0] = 0;
        return;
    }
    if (tid < NT) {
        const int co = co0 + tid;
        prm[tid] = p.bias ? p.bias[co] : 0.0f;
        prm[NT + tid] = p.scale ? p.scale[co] : 1.0f;
        prm[2 * NT + tid] = p.y16_a ? p.y16_a[co] : 0.0f;
        prm[3 * NT + tid] = p.y16_a ? p.y16_ib[co] : 0.0f;
    }
    __syncthreads();
    constexpr int UF = RP ? EK : 4;
#pragma unroll
    for (int i = 0; i < RB; ++i) {
#pragma unroll
        for (int c = 0; c < CB; ++c)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg)
                es[((reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)) * ELD + c * 32 + (lane & 31)] = acc[i][c][reg];
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the slice is in LDS (one wave writes and reads it)
        __builtin_amdgcn_wave_barrier();
#pragma unroll UF
        for (int k = 0; k < EK; ++k) {
            const int e = lane + 64 * k, row = e / Q, q4 = (e % Q) * 4;
            const int m = m0 + wave * 32 * RB + i * 32 + row;
            if (m >= M) continue;
            const size_t t = (size_t)m * so + ob, o = t * ldy + co0 + q4;
            const size_t o16 = t * p.C_out + co0 + q4;
            const float4 a = *reinterpret_cast<const float4 *>(es + row * ELD + q4);
            float v[4] = {a.x, a.y, a.z, a.w};
            if (p.bias) {
                const float4 b = *reinterpret_cast<const float4 *>(prm + q4);
                v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
            }
            if (p.scale) {
                const float4 g = *reinterpret_cast<const float4 *>(prm + NT + q4);
                v[0] *= g.x; v[1] *= g.y; v[2] *= g.z; v[3] *= g.w;
            }
            if (pres) {
                float4 rr;
                if constexpr (RP) rr = rres[k];
                else rr = *reinterpret_cast<const float4 *>(pres + o);
                v[0] = rr.x + v[0]; v[1] = rr.y + v[1]; v[2] = rr.z + v[2]; v[3] = rr.w + v[3];
            }
            if constexpr (ACT != 0) {
                if (p.act) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[q] = conv_act(v[q], p.act);
                }
            }
            if (py) *reinterpret_cast<float4 *>(py + o) = make_float4(v[0], v[1], v[2], v[3]);
            if (py16) {
                float z[4] = {v[0], v[1], v[2], v[3]};
                if (p.y16_a) {   // the k_snake_f16 expression, term for term
                    const float4 sa = *reinterpret_cast<const float4 *>(prm + 2 * NT + q4);
                    const float4 sb = *reinterpret_cast<const float4 *>(prm + 3 * NT + q4);
                    const float av[4] = {sa.x, sa.y, sa.z, sa.w}, bv[4] = {sb.x, sb.y, sb.z, sb.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) z[q] = snake_apply(z[q], av[q], bv[q]);
                }
                uint2 hv;
                hv.x = (uint32_t)f2h(z[0]) | ((uint32_t)f2h(z[1]) << 16);
                hv.y = (uint32_t)f2h(z[2]) | ((uint32_t)f2h(z[3]) << 16);
                *reinterpret_cast<uint2 *>(py16 + o16) = hv;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ======================================================================================= pipelined multi-tap conv
// k_conv_mt's 256-row x NT-channel tile of a stride-1 multi-tap conv (the residual units' dilated 7-tap convs of the
// wide decoder blocks), the same MFMA fragments in the same (K chunk, tap, k) order -- so the same bits -- with its
// K-chunk staging moved off the critical path: the input window and the chunk's weights of every tap go straight to
// LDS by buffer-load-to-LDS DMA (no registers, no synchronous weight load: k_conv_mt's 7-tap tile loaded its weights
// at the top of each chunk and waited for them, since registering them one chunk ahead spilled), into two stages, so
// chunk c + 1 lands while chunk c multiplies.  One workgroup per CU (2 x 64 KB of stages).
//   stage: window rows [320][4 x 16 B] (rows past the window, before the sequence or past T_in: zeros from the
//   buffer's range check), weights [tap][NT][4 x 16 B] padded to 44 KB; 16-byte slot q of row r sits at slot
//   q ^ ((r >> 2) & 3) (conflict-free ds_read_b128 fragment reads without row padding: a DMA fills 1 KB contiguously)
// Every thread issues exactly 16 DMA instructions per stage (5 window, 11 weight; placeholders out of range), so the
// wait for the previous stage is vmcnt(16).
// stage geometry of k_conv_pd<RB, NT, TAPS>: window rows 128 RB + 64, weights TAPS x NT rows, both in 1 KB DMA pieces
// spread over the 4 waves (7 taps x 96 channels: 44 KB)
template <int RB, int NT, int TAPS> struct PdGeom {
    static constexpr int XROWS = 128 * RB + 64, XSLOTS = XROWS * 4, WSLOTS = (TAPS * NT * 4 + 255) / 256 * 256;
    static constexpr int STAGE = (XSLOTS + WSLOTS) * 16;
    static constexpr int XI = XSLOTS / 256, WI = WSLOTS / 256;   // DMA instructions per thread and stage
    static_assert(XSLOTS % 256 == 0 && 2 * STAGE <= 160 * 1024, "stages");
};
constexpr unsigned PD_OOB = 0x7ffffff0u;   // a buffer offset past every range: the DMA writes zeros

// TAPS = 7: a stride-1 conv (taps [tap][C_out][C_in] consecutive); TAPS = 2: one launch over every output phase of a
// transposed conv (grid z = utterance x phase, k_conv_mt's ct_* geometry: phase phi's taps k = k0 + j st, input rows
// m + (phi + trim - k) / st, output rows st m + phi)
template <int RB, int NT, int TAPS, int ACT>
__global__ void __launch_bounds__(256, 1) k_conv_pd(const ConvParams p) {
    constexpr int MT = 128 * RB, CB = NT / 32;
    using Gm = PdGeom<RB, NT, TAPS>;
    constexpr int PD_XSLOTS = Gm::XSLOTS, PD_STAGE = Gm::STAGE, PD_XI = Gm::XI, PD_WI = Gm::WI;
    extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int n_taps = p.n_taps, dmin = p.dmin, dmax = p.dmax, M = p.M, so = 1, ob = 0;
    int dj[TAPS];
    size_t wofs[TAPS];   // tap j's weight block, elements past the buffer base
    const uint16_t *wbase = p.taps[0].w;
    size_t wbytes = (size_t)n_taps * p.C_out * p.C_in * 2;
    const int nz = TAPS == 2 ? p.ct_st : 1;
    const size_t ub = blockIdx.z / nz;
    int mt, ct, phi;
    conv_tile(p.xcd_tiles != 0, nz, mt, ct, phi);
    if constexpr (TAPS == 2) {
        const int st = p.ct_st, k0 = (phi + p.ct_trim) % st, d0 = (phi + p.ct_trim - k0) / st;
        n_taps = min(TAPS, (p.ct_k - k0 + st - 1) / st);
#pragma unroll
        for (int j = 0; j < TAPS; ++j) { dj[j] = d0 - j; wofs[j] = (size_t)(k0 + j * st) * p.C_out * p.C_in; }
        dmin = d0 - (n_taps - 1);
        dmax = d0;
        M = (p.T_out - phi + st - 1) / st;
        so = st;
        ob = phi;
        wbase = p.ct_w;
        wbytes = (size_t)p.ct_k * p.C_out * p.C_in * 2;
    } else {
#pragma unroll
        for (int j = 0; j < TAPS; ++j) { dj[j] = p.taps[j].dj; wofs[j] = (size_t)j * p.C_out * p.C_in; }
    }
    const int ldy = p.ldy ? p.ldy : p.C_out;
    const uint16_t *pxh = p.xh + ub * p.xbs * p.C_in;
    float *py = p.y ? p.y + ub * p.ybs * ldy : nullptr;
    const float *pres = p.resid ? p.resid + ub * p.ybs * ldy : nullptr;
    uint16_t *py16 = p.y16 ? p.y16 + ub * p.ybs * p.C_out : nullptr;
    const int m0 = mt * MT, co0 = ct * NT;
    if (m0 >= M || n_taps <= 0) return;   // (uniform per workgroup: shorter phases of a transposed conv)
    const int win = MT + dmax - dmin;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(pxh), 0,
                                                                        (int)((size_t)p.T_in * p.C_in * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(wbase), 0, (int)wbytes, 0x00020000);
    typedef __attribute__((address_space(3))) void lds_t;
    // this thread's DMA sources of the tile at K chunk 0 (instruction k of wave w fills slots [(4k + w) * 64, +64) of
    // its region; lane l slot (4k + w) * 64 + l); a chunk adds 2 c0 bytes through the scalar offset, so a DMA costs no
    // vector instruction.  Out of range (rows outside the window / sequence, taps past n_taps): PD_OOB, the buffer's
    // range check writes zeros (it holds with the scalar offset added too: PD_OOB + 2 c0 < 2^32)
    constexpr int ND = PD_XI + PD_WI;
    unsigned voff[ND];
#pragma unroll
    for (int k = 0; k < PD_XI; ++k) {
        const int P = (4 * k + wave) * 64 + lane, row = P >> 2, q = (P & 3) ^ ((row >> 2) & 3);
        const int i = m0 + dmin + row;
        voff[k] = row < win && i >= 0 && i < p.T_in ? (unsigned)(((size_t)i * p.C_in + 8 * q) * 2) : PD_OOB;
    }
#pragma unroll
    for (int k = 0; k < PD_WI; ++k) {
        const int P = (4 * k + wave) * 64 + lane, j = P / (NT * 4), rem = P - j * (NT * 4), co = rem >> 2;
        const int q = (rem & 3) ^ ((co >> 2) & 3);
        size_t wj = 0;
#pragma unroll
        for (int jj = 0; jj < TAPS; ++jj) wj = jj == j ? wofs[jj] : wj;
        voff[PD_XI + k] = j < n_taps ? (unsigned)((wj + (size_t)(co0 + co) * p.C_in + 8 * q) * 2) : PD_OOB;
    }
// (the voffset argument as int: an unsigned one made the host pass drop the kernel stubs without a diagnostic)
#define PD_DMA(k, st, c0)                                                                                              \
    do {                                                                                                              \
        uint8_t *base_ = reinterpret_cast<uint8_t *>(sm) + (st) * PD_STAGE;                                           \
        if ((k) < PD_XI)                                                                                              \
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_t *)(base_ + (4 * (k) + wave) * 1024), 16, (int)voff[k], 2 * (c0), 0, 0); \
        else                                                                                                          \
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_t *)(base_ + PD_XSLOTS * 16 + (4 * ((k) - PD_XI) + wave) * 1024), \
                                                     16, (int)voff[k], 2 * (c0), 0, 0);                                    \
    } while (0)
    const int r = lane & 31, h = lane >> 5;
    f32x16_t acc[RB][CB];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
    const int nch = p.C_in / MT_KC;
#pragma unroll
    for (int k = 0; k < ND; ++k) PD_DMA(k, 0, 0);
    for (int c = 0; c < nch; ++c) {
        // chunk c's DMAs (issued during chunk c - 1's MFMAs) have landed for every thread; a bare barrier
        // (__syncthreads' fence adds nothing here)
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        const bool nxt = c + 1 < nch;
        const uint8_t *xs = reinterpret_cast<const uint8_t *>(sm) + (c & 1) * PD_STAGE;
        const uint8_t *ws = xs + PD_XSLOTS * 16;
        // the 7 taps x 2 k-steps as one straight-line sequence, each step's fragments read one step ahead into the
        // other register set (one wave per SIMD cannot hide an LDS round trip per step otherwise); the MFMA order is
        // k_conv_mt's (tap, k-step, row tile, channel tile)
        constexpr int NSTEP = 2 * TAPS;   // (every phase has TAPS taps: pd_ok)
        half8_t a[2][RB], b[2][CB];
        auto frag = [&](int st, half8_t (&av)[RB], half8_t (&bv)[CB]) {
            const int j = st >> 1, q = h + 2 * (st & 1);
            const int arow = wave * 32 * RB + r + (dj[j] - dmin);
#pragma unroll
            for (int i = 0; i < RB; ++i) {
                const int row = arow + 32 * i;
                av[i] = *reinterpret_cast<const half8_t *>(xs + row * 64 + ((q ^ ((row >> 2) & 3)) * 16));
            }
#pragma unroll
            for (int cc = 0; cc < CB; ++cc) {
                const int co = cc * 32 + r;
                bv[cc] = *reinterpret_cast<const half8_t *>(ws + (j * NT + co) * 64 + ((q ^ ((co >> 2) & 3)) * 16));
            }
        };
        frag(0, a[0], b[0]);
#pragma unroll
        for (int st = 0; st < NSTEP; ++st) {
            if (st + 1 < NSTEP) frag(st + 1, a[(st + 1) & 1], b[(st + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);   // the reads stay ahead of this step's MFMAs (the scheduler sank them)
            // chunk c + 1's DMAs into the other stage (read by chunk c - 1, released by its trailing barrier), four
            // per step among the first steps' MFMAs: their issue hides in the MFMA shadow and they land long before
            // chunk c ends
            if (nxt) {
#pragma unroll
                for (int k = 4 * st; k < 4 * st + 4; ++k)
                    if (k < ND) PD_DMA(k, (c + 1) & 1, (c + 1) * MT_KC);
            }
#pragma unroll
            for (int i = 0; i < RB; ++i)
#pragma unroll
                for (int cc = 0; cc < CB; ++cc)
                    acc[i][cc] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[st & 1][i], b[st & 1][cc], acc[i][cc], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // stage c & 1 is chunk c + 2's DMA target
    }
    // ---- epilogue: k_conv_mt's (transposed slices through LDS, 4 channels per lane)
    constexpr int ELD = NT + 4, Q = NT / 4, EK = 32 * Q / 64;
    float *es = reinterpret_cast<float *>(sm) + wave * 32 * ELD;
    float *prm = reinterpret_cast<float *>(sm) + 4 * 32 * ELD;
    if (tid < NT) {
        const int co = co0 + tid;
        prm[tid] = p.bias ? p.bias[co] : 0.0f;
        prm[NT + tid] = p.scale ? p.scale[co] : 1.0f;
        prm[2 * NT + tid] = p.y16_a ? p.y16_a[co] : 0.0f;
        prm[3 * NT + tid] = p.y16_a ? p.y16_ib[co] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RB; ++i) {
#pragma unroll
        for (int cc = 0; cc < CB; ++cc)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg)
                es[((reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)) * ELD + cc * 32 + (lane & 31)] = acc[i][cc][reg];
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
#pragma unroll 4
        for (int k = 0; k < EK; ++k) {
            const int e = lane + 64 * k, row = e / Q, q4 = (e % Q) * 4;
            const int m = m0 + wave * 32 * RB + i * 32 + row;
            if (m >= M) continue;
            const size_t t = (size_t)m * so + ob, o = t * ldy + co0 + q4;
            const size_t o16 = t * p.C_out + co0 + q4;
            const float4 a = *reinterpret_cast<const float4 *>(es + row * ELD + q4);
            float v[4] = {a.x, a.y, a.z, a.w};
            if (p.bias) {
                const float4 b = *reinterpret_cast<const float4 *>(prm + q4);
                v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
            }
            if (p.scale) {
                const float4 g = *reinterpret_cast<const float4 *>(prm + NT + q4);
                v[0] *= g.x; v[1] *= g.y; v[2] *= g.z; v[3] *= g.w;
            }
            if (pres) {
                const float4 rr = *reinterpret_cast<const float4 *>(pres + o);
                v[0] = rr.x + v[0]; v[1] = rr.y + v[1]; v[2] = rr.z + v[2]; v[3] = rr.w + v[3];
            }
            if constexpr (ACT != 0) {
                if (p.act) {
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq) v[qq] = conv_act(v[qq], p.act);
                }
            }
            if (py) *reinterpret_cast<float4 *>(py + o) = make_float4(v[0], v[1], v[2], v[3]);
            if (py16) {
                float z[4] = {v[0], v[1], v[2], v[3]};
                if (p.y16_a) {
                    const float4 sa = *reinterpret_cast<const float4 *>(prm + 2 * NT + q4);
                    const float4 sb = *reinterpret_cast<const float4 *>(prm + 3 * NT + q4);
                    const float av[4] = {sa.x, sa.y, sa.z, sa.w}, bv[4] = {sb.x, sb.y, sb.z, sb.w};
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq) z[qq] = snake_apply(z[qq], av[qq], bv[qq]);
                }
                uint2 hv;
                hv.x = (uint32_t)f2h(z[0]) | ((uint32_t)f2h(z[1]) << 16);
                hv.y = (uint32_t)f2h(z[2]) | ((uint32_t)f2h(z[3]) << 16);
                *reinterpret_cast<uint2 *>(py16 + o16) = hv;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Q3T_CONV_PD=0 keeps the multi-tap convs on k_conv_mt (A/B and the bit-exactness test; read at every launch)
static bool conv_xcd_tiles() {   // Q3T_CONV_XCD=0: the conv tiles in plain grid order (A/B)
    const char *e = std::getenv("Q3T_CONV_XCD");
    return !e || std::atoi(e) != 0;
}
static bool conv_pd_ct() {   // Q3T_CONV_PD_CT=0 keeps the transposed convs on k_conv_mt (A/B)
    const char *e = std::getenv("Q3T_CONV_PD_CT");
    return !e || std::atoi(e) != 0;
}
static int conv_pd_minc() {   // Q3T_CONV_PD_MINC: smallest C_in of a 7-tap conv on k_conv_pd (A/B; default 192)
    const char *e = std::getenv("Q3T_CONV_PD_MINC");
    return e ? std::atoi(e) : 192;
}
static int conv_pd_mode() {   // 0 off, 1 256-row tiles, 2 512-row tiles
    const char *e = std::getenv("Q3T_CONV_PD");
    return e ? std::atoi(e) : 2;
}
// k_conv_pd's preconditions: a stride-1 7-tap conv whose taps are consecutive [tap][C_out][C_in] blocks, and 32-bit buffer
// offsets below the out-of-range marker
static bool pd_ok(const ConvParams &p) {
    if (p.ct_st)   // transposed: kernel 2 st, so every output phase has exactly 2 taps
        return p.ct_k == 2 * p.ct_st && p.C_in % MT_KC == 0 && (size_t)p.T_in * p.C_in * 2 < PD_OOB &&
               (size_t)p.ct_k * p.C_out * p.C_in * 2 < PD_OOB;
    if (p.so != 1 || p.ob != 0 || p.n_taps != CONV_MAX_TAPS || p.dmax - p.dmin > 64) return false;
    for (int j = 1; j < p.n_taps; ++j)
        if (p.taps[j].w != p.taps[0].w + (size_t)j * p.C_out * p.C_in) return false;
    return (size_t)p.T_in * p.C_in * 2 < PD_OOB && (size_t)p.n_taps * p.C_out * p.C_in * 2 < PD_OOB;
}

template <int RB, int NT, int TAPS = CONV_MAX_TAPS>
static bool launch_pd(const ConvParams &p, hipStream_t s) {
    constexpr int lds = 2 * PdGeom<RB, NT, TAPS>::STAGE;
    static bool attr = false;
    if (!attr) {
        Q3T_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_conv_pd<RB, NT, TAPS, 0>), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        Q3T_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_conv_pd<RB, NT, TAPS, -1>), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        attr = true;
    }
    const dim3 grid((p.M + 128 * RB - 1) / (128 * RB), p.C_out / NT, (p.ct_st ? p.ct_st : 1) * p.nb);
    if (p.act) hipLaunchKernelGGL((k_conv_pd<RB, NT, TAPS, -1>), grid, dim3(256), lds, s, p);
    else hipLaunchKernelGGL((k_conv_pd<RB, NT, TAPS, 0>), grid, dim3(256), lds, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}

template <int RB, int NT, int MINB, int TW, int ACT>
static bool launch_mt2(const ConvParams &p, hipStream_t s) {
    constexpr int MT = 128 * RB;
    // staging area (input window + the chunk's weights of every tap), reused by the epilogue's transposed slices
    // (transposed launches: p.n_taps / dmin / dmax carry the largest tap count and span over the phases)
    const size_t lds = std::max(((size_t)(MT + p.dmax - p.dmin) + (size_t)p.n_taps * NT) * MT_LDK * 2,
                                (size_t)4 * 32 * (NT + 4) * 4 + (size_t)4 * NT * 4);
    static bool attr = false;
    if (!attr) {
        Q3T_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_conv_mt<RB, NT, MINB, TW, ACT>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
        attr = true;
    }
    const dim3 grid((p.M + MT - 1) / MT, p.C_out / NT, (p.ct_st ? p.ct_st : 1) * p.nb);
    hipLaunchKernelGGL((k_conv_mt<RB, NT, MINB, TW, ACT>), grid, dim3(256), lds, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}
template <int RB, int NT, int MINB, int TW>
static bool launch_mt1(const ConvParams &p, hipStream_t s) {
    return p.act ? launch_mt2<RB, NT, MINB, TW, -1>(p, s) : launch_mt2<RB, NT, MINB, TW, 0>(p, s);
}
template <int RB, int NT, int MINB = 2>
static bool launch_mt(const ConvParams &p, hipStream_t s) {
    if constexpr (MINB == 3) {   // the 1-tap narrow-channel variant only
        return launch_mt1<RB, NT, MINB, 1>(p, s);
    } else {
        if (p.n_taps <= 1) return launch_mt1<RB, NT, MINB, 1>(p, s);
        if (p.n_taps <= 3) return launch_mt1<RB, NT, MINB, 3>(p, s);
        return launch_mt1<RB, NT, MINB, 7>(p, s);
    }
}

#ifdef Q3T_DEV
// development builds: Q3T_CONV_VARIANT picks another tile shape for the multi-tap convs (tools/dev experiments)
static const int g_conv_variant = [] { const char *e = std::getenv("Q3T_CONV_VARIANT"); return e ? std::atoi(e) : 0; }();
#else
static constexpr int g_conv_variant = 0;
#endif

#ifdef Q3T_DEV
static const int g_conv_skip = [] { const char *e = std::getenv("Q3T_CONV_SKIP"); return e ? std::atoi(e) : 0; }();
#endif

bool conv(const ConvParams &pin, hipStream_t s) {
#ifdef Q3T_DEV
    ConvParams p = pin;
    if (p.n_taps > 1) p.dev_skip = g_conv_skip;
#else
    const ConvParams &p = pin;
#endif
    if (p.ct_st) {   // one launch over every output phase (multi-tile kernel only)
        const int NT = p.C_out % 96 == 0 ? 96 : p.C_out % 64 == 0 ? 64 : 0;
        if (!p.xh || !NT || p.C_in % MT_KC != 0 || p.ct_k > p.ct_st * CONV_MAX_TAPS) {
            set_error("conv: unsupported transposed launch");
            return false;
        }
        if (p.nb <= 0) return true;
        if (p.nb > 1 && (p.xbs < p.T_in || p.ybs < p.T_out)) { set_error("conv: bad utterance strides"); return false; }
        ConvParams q = p;
        q.xcd_tiles = conv_xcd_tiles();
        q.M = (p.T_out + p.ct_st - 1) / p.ct_st;   // phase 0 has the most rows
        q.n_taps = (p.ct_k + p.ct_st - 1) / p.ct_st;
        q.dmin = 0;
        q.dmax = q.n_taps - 1;                      // taps of one phase are consecutive input rows
        if (q.M <= 0) return true;
        const long tiles256 = (long)((q.M + 255) / 256) * (p.C_out / NT) * p.ct_st * p.nb;
        // the pipelined kernel (512-row tiles, both taps of a phase per K chunk) where a tile has 24+ K chunks (per launch
        // at 512 frames: C_in 1536 116 -> 94 us, 768 162 -> 157; 384 209 -> 201; 192 275 -> 288 us)
        if (tiles256 >= 512 && p.C_in >= 768 && conv_pd_mode() == 2 && pd_ok(q) && conv_pd_ct())
            return NT == 96 ? launch_pd<4, 96, 2>(q, s) : launch_pd<4, 64, 2>(q, s);
        if (NT == 96) return tiles256 >= 512 ? launch_mt<2, 96>(q, s) : launch_mt<1, 96>(q, s);
        return tiles256 >= 512 ? launch_mt<2, 64>(q, s) : launch_mt<1, 64>(q, s);
    }
    if (p.M <= 0 || p.nb <= 0) return true;
    if (p.nb > 1 && (p.xbs < p.T_in || p.ybs <= 0)) { set_error("conv: bad utterance strides"); return false; }
    if (p.n_taps < 1 || p.n_taps > CONV_MAX_TAPS || p.dmax - p.dmin > CT_MAXWIN - CT_M) {
        set_error("conv: unsupported tap layout");
        return false;
    }
    const int NT = p.C_out % 96 == 0 ? 96 : p.C_out % 64 == 0 ? 64 : 0;
    if (p.xh && NT && p.C_in % MT_KC == 0 && (p.y || p.y16)) {
        // RB 2 (256-row tiles) unless that leaves fewer than two workgroups per CU to fill the chip.  1-tap convs over
        // narrow channel counts are bound by their epilogue traffic (f32 residual in, f32 + f16 out): 128-row tiles
        // at three workgroups per CU keep more of it in flight
        const long tiles256 = (long)((p.M + 255) / 256) * (p.C_out / NT) * p.nb;
        const bool big = tiles256 >= 512;
        ConvParams q = p;
        q.xcd_tiles = conv_xcd_tiles();
        if (big && p.n_taps == 1 && p.C_in <= 192) return NT == 96 ? launch_mt<1, 96, 3>(q, s) : launch_mt<1, 64, 3>(q, s);
        if (g_conv_variant && big && p.n_taps > 1) {
            switch (g_conv_variant) {
                case 1: return NT == 96 ? launch_mt1<1, 96, 2, 7>(p, s) : launch_mt1<1, 64, 2, 7>(p, s);
                case 2: return launch_mt1<2, 32, 3, 7>(p, s);
                case 3: return launch_mt1<4, 32, 2, 7>(p, s);
                case 4: return NT == 96 ? launch_mt1<4, 96, 1, 7>(p, s) : launch_mt1<4, 64, 1, 7>(p, s);
                default: break;
            }
        }
        // the pipelined kernel for the wide blocks' 7-tap convs (512 frames, per launch: C_in 768 191 -> 125 us, 384
        // 278 -> 207 us, 192 301 -> 256 us with 512-row tiles; 256-row tiles: 135 / 202 us, and no gain at 192)
        const int pm = conv_pd_mode();
        if (big && p.n_taps > 3 && p.C_in >= conv_pd_minc() && pd_ok(p)) {
            if (pm == 1) return NT == 96 ? launch_pd<2, 96>(q, s) : launch_pd<2, 64>(q, s);
            if (pm == 2) return NT == 96 ? launch_pd<4, 96>(q, s) : launch_pd<4, 64>(q, s);
        }
        if (NT == 96) return big ? launch_mt<2, 96>(q, s) : launch_mt<1, 96>(q, s);
        return big ? launch_mt<2, 64>(q, s) : launch_mt<1, 64>(q, s);
    }
    if (!p.y && !p.y16) { set_error("conv: no output"); return false; }
    const dim3 grid((p.M + CT_M - 1) / CT_M, (p.C_out + CT_N - 1) / CT_N, p.nb);
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
        for (int q = 0; q < 4; ++q) y[q] = snake_apply(y[q], a[c + q], ib[c + q]);
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

// ======================================================================================= row norm -> f16
__global__ void __launch_bounds__(256) k_norm_f16(const float *x, const float *w, const float *b, float eps, int mode,
                                                  uint16_t *out, int C) {
    __shared__ double scr[4];
    const int t = blockIdx.x, tid = threadIdx.x, k = 4 * tid;
    const bool ok = k < C;
    const float *row = x + (size_t)t * C;
    const float4 v = ok ? *reinterpret_cast<const float4 *>(row + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    auto block_sum = [&](double d) {
        d = wave_sum_d(d);
        __syncthreads();
        if ((tid & 63) == 0) scr[tid >> 6] = d;
        __syncthreads();
        return (scr[0] + scr[1]) + (scr[2] + scr[3]);
    };
    float y[4] = {v.x, v.y, v.z, v.w};
    if (mode == 0) {
        const double ss = block_sum((double)(v.x * v.x) + (double)(v.y * v.y) + (double)(v.z * v.z) + (double)(v.w * v.w));
        const float scale = 1.0f / sqrtf((float)(ss / C) + eps);
        if (!ok) return;
        const float4 g = *reinterpret_cast<const float4 *>(w + k);
        y[0] = (y[0] * scale) * g.x; y[1] = (y[1] * scale) * g.y; y[2] = (y[2] * scale) * g.z; y[3] = (y[3] * scale) * g.w;
    } else {
        const double s1 = block_sum((double)v.x + (double)v.y + (double)v.z + (double)v.w);
        const float mean = (float)(s1 / C);
        const float dx = v.x - mean, dy = v.y - mean, dz = v.z - mean, dw = v.w - mean;
        const double s2 = block_sum(ok ? (double)(dx * dx) + (double)(dy * dy) + (double)(dz * dz) + (double)(dw * dw) : 0.0);
        const float scale = 1.0f / sqrtf((float)(s2 / C) + eps);
        if (!ok) return;
        const float4 g = *reinterpret_cast<const float4 *>(w + k), c = *reinterpret_cast<const float4 *>(b + k);
        y[0] = (dx * scale) * g.x + c.x; y[1] = (dy * scale) * g.y + c.y;
        y[2] = (dz * scale) * g.z + c.z; y[3] = (dw * scale) * g.w + c.w;
    }
    uint2 hv;
    hv.x = (uint32_t)f2h(y[0]) | ((uint32_t)f2h(y[1]) << 16);
    hv.y = (uint32_t)f2h(y[2]) | ((uint32_t)f2h(y[3]) << 16);
    *reinterpret_cast<uint2 *>(out + (size_t)t * C + k) = hv;
}
bool norm_f16(const float *x, const float *w, const float *b, float eps, int mode, uint16_t *out, int T, int C,
              hipStream_t s) {
    if (C % 4 != 0 || C > 1024 || (mode == 1 && !b)) { set_error("norm_f16: unsupported shape"); return false; }
    if (T <= 0) return true;
    hipLaunchKernelGGL(k_norm_f16, dim3(T), dim3(256), 0, s, x, w, b, eps, mode, out, C);
    Q3T_HIP(hipGetLastError());
    return true;
}

// ======================================================================================= single-channel output conv
// one workgroup per 256 outputs: the input rows [t0 - (K-1), t0 + 256) staged once in LDS, one output per thread
constexpr int CO1_T = 256, CO1_MAXC = 104, CO1_MAXK = 8;
__global__ void __launch_bounds__(256) k_conv_out1(const uint16_t *xh, const uint16_t *w, const float *bias, float *y,
                                                   int T, int C, int K) {
    // f16 x f16 products (exact in f32) as v_dot2_f32_f16 pairs into four independent f32 accumulators: the
    // single-accumulator f32 chain (h2f per element, 1,344 dependent FMAs per sample) ran at 1.3 TB/s
    typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
    // input rows at a stride of C + 8 halves: lane l reads row l + j, so at a stride of C = 96 halves (192 B) 16 lanes'
    // 16-byte reads fell on 4 bank groups (4-way conflicts); C + 8 (208 B) puts them on 16 distinct ones
    __shared__ __attribute__((aligned(16))) uint16_t xs[(CO1_T + CO1_MAXK) * (CO1_MAXC + 8)];
    __shared__ __attribute__((aligned(16))) uint16_t ws[CO1_MAXK * CO1_MAXC];
    const int t0 = blockIdx.x * CO1_T, tid = threadIdx.x;
    xh += (size_t)blockIdx.y * T * C;   // utterance
    y += (size_t)blockIdx.y * T;
    const int rows = CO1_T + K - 1, c8n = C / 8, XLD = C + 8;
    for (int e = tid; e < rows * c8n; e += 256) {
        const int r = e / c8n, c8 = (e % c8n) * 8, i = t0 - (K - 1) + r;
        const uint4 u = (i >= 0 && i < T) ? ldg16(xh + (size_t)i * C + c8) : make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4 *>(xs + r * XLD + c8) = u;
    }
    for (int e = tid; e < K * C; e += 256) ws[e] = w[e];
    __syncthreads();
    const int t = t0 + tid;
    if (t >= T) return;
    float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int j = 0; j < K; ++j) {
        const uint16_t *xr = xs + (tid + j) * XLD;
        const uint16_t *wr = ws + j * C;
        for (int c = 0; c < C; c += 8) {
            const uint4 u = *reinterpret_cast<const uint4 *>(xr + c);
            const uint4 v = *reinterpret_cast<const uint4 *>(wr + c);
            a[0] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, u.x), __builtin_bit_cast(h2_t, v.x), a[0], false);
            a[1] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, u.y), __builtin_bit_cast(h2_t, v.y), a[1], false);
            a[2] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, u.z), __builtin_bit_cast(h2_t, v.z), a[2], false);
            a[3] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, u.w), __builtin_bit_cast(h2_t, v.w), a[3], false);
        }
    }
    y[t] = tanhf(((a[0] + a[1]) + (a[2] + a[3])) + bias[0]);
}
bool conv_out1(const uint16_t *xh, const uint16_t *w, const float *bias, float *y, int T, int C, int K, hipStream_t s,
               int nb) {
    if (C % 8 != 0 || C > CO1_MAXC || K > CO1_MAXK) { set_error("conv_out1: unsupported shape"); return false; }
    if (T <= 0 || nb <= 0) return true;
    hipLaunchKernelGGL(k_conv_out1, dim3((T + CO1_T - 1) / CO1_T, nb), dim3(256), 0, s, xh, w, bias, y, T, C, K);
    Q3T_HIP(hipGetLastError());
    return true;
}

// ======================================================================================= depthwise causal conv
// y[t][c] = b[c] + sum_j w[c][j] * f16(x[t + j - (K-1)][c])      (ggml_pad_ext + ggml_conv_1d_dw, im2col F16)
__global__ void __launch_bounds__(256) k_dwconv(const float *x, const uint16_t *w, const float *b, float *y, int T, int C, int K) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)T * C) return;
    x += (size_t)blockIdx.y * T * C;   // utterance
    y += (size_t)blockIdx.y * T * C;
    const int t = (int)(idx / C), c = (int)(idx % C);
    float acc = 0.0f;
    for (int j = 0; j < K; ++j) {
        const int i = t + j - (K - 1);
        if (i >= 0) acc += h2f(w[(size_t)c * K + j]) * f16r(x[(size_t)i * C + c]);
    }
    y[idx] = acc + b[c];
}
bool dwconv(const float *x, const uint16_t *w, const float *b, float *y, int T, int C, int K, hipStream_t s, int nb) {
    const size_t n = (size_t)T * C;
    if (!n || nb <= 0) return true;
    hipLaunchKernelGGL(k_dwconv, dim3((unsigned)((n + 255) / 256), nb), dim3(256), 0, s, x, w, b, y, T, C, K);
    Q3T_HIP(hipGetLastError());
    return true;
}

// ======================================================================================= pre-transformer attention
// causal softmax attention over F frames (apply_pre_tfm_layer, audio_tokenizer_decoder.cpp:412-456): NEOX RoPE
// (theta 1e4) on q,k, f32 scores (ggml mul_mat of two F32 tensors: no rounding), output rounded to f16.
// Two launches: RoPE applied once, in place, to the q and k columns of the qkv rows (the attention then streams plain
// rows); then one workgroup per (32 queries, head) walks 64-key chunks: K/V chunk in LDS via coalesced float4 loads,
// 16 lanes per query (4 keys each for the scores, 4 dims each for P.V), online softmax within the 16-lane group.
__global__ void k_rope_qk(float *qkv, const float *rope, int F, int nH) {
    constexpr int D = 64;
    const int idx = blockIdx.x * 256 + threadIdx.x;   // (pos, q/k, head, pair)
    const int total = F * 2 * nH * 32;
    if (idx >= total) return;
    const int i = idx & 31, hh = (idx >> 5) % (2 * nH), pos = idx / (64 * nH);
    float *x = qkv + ((size_t)blockIdx.y * F + pos) * 3 * nH * D + hh * D;   // utterance y; hh < nH: q head, else k
    const float c = rope[(size_t)pos * D + 2 * i], sn = rope[(size_t)pos * D + 2 * i + 1];
    const float x0 = x[i], x1 = x[i + 32];
    x[i] = x0 * c - x1 * sn;
    x[i + 32] = x0 * sn + x1 * c;
}

__global__ void __launch_bounds__(512) k_attn_prefill(const float *qkv, uint16_t *out, int F, int nH) {
    // 512 threads: 16 lanes per query (4 keys each for the scores, 4 dims each for P.V).  With 8 lanes per query (256
    // threads, one workgroup per CU at F = 512) the longest query block's 8 chunks ran 59 us per layer.
    constexpr int D = 64, QT = 32, KT = 64, KP = D + 4, LQ = 16;
    __shared__ __attribute__((aligned(16))) float ks[KT * KP];
    __shared__ __attribute__((aligned(16))) float vs[KT * KP];
    __shared__ float ps[QT][KT + 1];
    const int h = blockIdx.y, q0 = blockIdx.x * QT;
    const int tid = threadIdx.x, qi = tid / LQ, g = tid % LQ;
    const int LD = 3 * nH * D;
    qkv += (size_t)blockIdx.z * F * LD;   // utterance
    out += (size_t)blockIdx.z * F * nH * D;
    const int qpos = q0 + qi;
    float q[D];
    {
        const float *src = qkv + (size_t)min(qpos, F - 1) * LD + h * D;
#pragma unroll
        for (int d = 0; d < D; d += 4) {
            const float4 v = *reinterpret_cast<const float4 *>(src + d);
            q[d] = v.x; q[d + 1] = v.y; q[d + 2] = v.z; q[d + 3] = v.w;
        }
    }
    float m = -INFINITY, l = 0.0f, acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const float scale = 0.125f;   // 1 / sqrt(64)
    const int kend = min(F, q0 + QT);
    // chunk: 64 keys x 64 dims of K and V, 2 float4 per thread per tensor, loaded into registers one chunk ahead (the
    // chunk loop is serial per workgroup and the longest query block runs 8 chunks: the load latency was exposed once
    // per chunk).  Unconditional loads (rows clamped, zeroed past F at the LDS store) keep one chunk in flight at the
    // compiler's waits.
    float4 kr4[2], vr4[2];
    auto kv_load = [&](int k0) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = (u * 512 + tid) * 4, kk = e / D, d = e % D, pos = min(k0 + kk, F - 1);
            const float *row = qkv + (size_t)pos * LD;
            kr4[u] = *reinterpret_cast<const float4 *>(row + nH * D + h * D + d);
            vr4[u] = *reinterpret_cast<const float4 *>(row + 2 * nH * D + h * D + d);
        }
    };
    kv_load(0);
    for (int k0 = 0; k0 < kend; k0 += KT) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = (u * 512 + tid) * 4, kk = e / D, d = e % D;
            const bool in = k0 + kk < F;
            *reinterpret_cast<float4 *>(ks + kk * KP + d) = in ? kr4[u] : make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4 *>(vs + kk * KP + d) = in ? vr4[u] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        __syncthreads();
        kv_load(min(k0 + KT, kend - 1));   // the next chunk (past the last: the last rows again, never stored)
        float sc[4], mt = -INFINITY;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int kk = g + LQ * i, kpos = k0 + kk;
            const float *kr = ks + kk * KP;
            float dsum = 0.0f;
#pragma unroll
            for (int d = 0; d < D; d += 4) {
                const float4 kv = *reinterpret_cast<const float4 *>(kr + d);
                dsum += q[d] * kv.x + q[d + 1] * kv.y + q[d + 2] * kv.z + q[d + 3] * kv.w;
            }
            sc[i] = (kpos <= qpos && kpos < F) ? dsum * scale : -INFINITY;
            mt = fmaxf(mt, sc[i]);
        }
#pragma unroll
        for (int o = 1; o < LQ; o <<= 1) mt = fmaxf(mt, __shfl_xor(mt, o));
        const float mn = fmaxf(m, mt);
        const float corr = m == -INFINITY ? 0.0f : expf(m - mn);
        float ls = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float pv = sc[i] == -INFINITY ? 0.0f : expf(sc[i] - mn);
            ps[qi][g + LQ * i] = pv;
            ls += pv;
        }
#pragma unroll
        for (int o = 1; o < LQ; o <<= 1) ls += __shfl_xor(ls, o);
        l = l * corr + ls;
        m = mn;
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] *= corr;
        __syncthreads();
        const int kn = min(KT, kend - k0);
        for (int kk = 0; kk < kn; ++kk) {
            const float pv = ps[qi][kk];
            const float4 a = *reinterpret_cast<const float4 *>(vs + kk * KP + g * 4);
            acc[0] += pv * a.x; acc[1] += pv * a.y; acc[2] += pv * a.z; acc[3] += pv * a.w;
        }
    }
    if (qpos < F) {
        const float inv = 1.0f / l;
        uint2 o;
        o.x = (uint32_t)f2h(acc[0] * inv) | ((uint32_t)f2h(acc[1] * inv) << 16);
        o.y = (uint32_t)f2h(acc[2] * inv) | ((uint32_t)f2h(acc[3] * inv) << 16);
        *reinterpret_cast<uint2 *>(out + (size_t)qpos * nH * D + h * D + g * 4) = o;
    }
}
bool attn_prefill(float *qkv, const float *rope, uint16_t *out, int F, int nH, int D, hipStream_t s, int nb) {
    if (D != 64) { set_error("attn_prefill: head_dim must be 64"); return false; }
    if (F <= 0 || nb <= 0) return true;
    hipLaunchKernelGGL(k_rope_qk, dim3((F * 2 * nH * 32 + 255) / 256, nb), dim3(256), 0, s, qkv, rope, F, nH);
    Q3T_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_attn_prefill, dim3((F + 31) / 32, nH, nb), dim3(512), 0, s, qkv, out, F, nH);
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
