// vocoder_resunit.hip — one decoder residual unit of the 96-channel block as ONE launch (gfx950):
//
//   h  = f16( snake2( conv7_dil(xh) + b1 ) )        xh = f16(snake1(x)), written by the previous launch's epilogue
//   x' = x + ( conv1(h) + b2 )                       f32 residual stream (in place), optional (the block's last unit
//   y16 = f16( snake_next(x') )                      feeds only the next conv's f16 input)
//
// (src/audio_tokenizer_decoder.cpp:551-579, the ResidualUnit of every decoder block).  The unfused form is two
// k_conv_mt launches; between them the f16 h tensor (2 B x 96 per row, ~190 MB at 512 frames) goes to HBM and back.
// Here a workgroup computes the 7-tap conv of its 256 rows exactly as k_conv_mt<2, 96> does (same K-chunk order, same
// MFMA fragments, same epilogue expression), leaves h in LDS, and runs the 1-tap conv on it from LDS with the
// 1-tap kernel's K order: the result is bit-identical to the two launches.
#include "vocoder_kernels.h"

#include <algorithm>

namespace q3t {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

constexpr int C = 96, CB = C / 32, RB = 2, MT = 128 * RB, KC = 32, LDK = KC + 8, TAPS = 7;
constexpr int HLD = C + 8;   // h tile / k1 weight rows in LDS: 96 f16 + 16 B pad (conflict-free ds_read_b128)
constexpr int ELD = C + 4;   // f32 row stride of an epilogue's transposed slice
constexpr int MAXWIN = MT + 6 * 9 + 8;

}  // namespace

__global__ void __launch_bounds__(256, 2) k_resunit96(const ResUnitParams p) {
    extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, hh = lane >> 5;
    const size_t ub = blockIdx.z;
    const int T = p.T, m0 = blockIdx.x * MT, dil = p.dil, dmin = -6 * dil;
    if (m0 >= T) return;
    const uint16_t *pxh = p.xh + ub * p.bs * C;
    const float *pres = p.x + ub * p.bs * C;
    float *py = p.y ? p.y + ub * p.bs * C : nullptr;
    uint16_t *py16 = p.y16 + ub * p.bs * C;
    const int win = MT - dmin;
    uint16_t *xs = sm;                        // [win][LDK]
    uint16_t *ws = sm + (size_t)win * LDK;    // [7][96][LDK]
    f32x16_t acc[RB][CB];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
    // ---------------- the 7-tap conv (k_conv_mt<2, 96, 2, 7, 0>'s loop: window through registers one chunk ahead,
    // the chunk's weights loaded and stored at once)
    constexpr int XR = (MT + 64) * (KC / 8) / 256;
    constexpr int WR = (TAPS * C * (KC / 8) + 255) / 256;
    const int nx = win * (KC / 8), nw = TAPS * C * (KC / 8);
    uint4 xr[XR];
    auto xload = [&](int c0) {
#pragma unroll
        for (int q = 0; q < XR; ++q) {
            const int e = tid + q * 256, row = e >> 2, c8 = (e & 3) * 8, i = m0 + dmin + row;
            const bool in = e < nx && i >= 0 && i < T;
            const int ic = min(max(i, 0), T - 1);
            const uint4 u = ldg16(pxh + (size_t)ic * C + c0 + c8);
            xr[q] = in ? u : make_uint4(0, 0, 0, 0);
        }
    };
    xload(0);
    for (int c0 = 0; c0 < C; c0 += KC) {
#pragma unroll
        for (int q = 0; q < XR; ++q) {
            const int e = tid + q * 256;
            if (e < nx) *reinterpret_cast<uint4 *>(xs + (e >> 2) * LDK + (e & 3) * 8) = xr[q];
        }
#pragma unroll
        for (int q = 0; q < WR; ++q) {
            const int e = min(tid + q * 256, nw - 1);
            const int j = e / (C * 4), rem = e - j * (C * 4), co = rem >> 2, c8 = (rem & 3) * 8;
            const uint4 u = ldg16(p.w1 + (size_t)j * C * C + (size_t)co * C + c0 + c8);
            if (tid + q * 256 < nw) *reinterpret_cast<uint4 *>(ws + (j * C + co) * LDK + c8) = u;
        }
        __syncthreads();
        if (c0 + KC < C) xload(c0 + KC);
        for (int j = 0; j < TAPS; ++j) {
            const uint16_t *ab = xs + (wave * 32 * RB + r + j * dil) * LDK + 8 * hh;   // tap j: input row m + j*dil - 6*dil
            const uint16_t *bb = ws + (j * C + r) * LDK + 8 * hh;
#pragma unroll
            for (int kk = 0; kk < KC; kk += 16) {
                half8_t a[RB], b[CB];
#pragma unroll
                for (int i = 0; i < RB; ++i) a[i] = *reinterpret_cast<const half8_t *>(ab + i * 32 * LDK + kk);
#pragma unroll
                for (int c = 0; c < CB; ++c) b[c] = *reinterpret_cast<const half8_t *>(bb + c * 32 * LDK + kk);
#pragma unroll
                for (int i = 0; i < RB; ++i)
#pragma unroll
                    for (int c = 0; c < CB; ++c) acc[i][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[c], acc[i][c], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    // ---------------- h = f16(snake2(acc + b1)) into LDS [MT][HLD]; the k1 weights [96][HLD] behind it
    uint16_t *hs = sm;                        // [MT][HLD]
    uint16_t *w2s = sm + (size_t)MT * HLD;    // [96][HLD]
    {
        float bc[CB], ac[CB], ic[CB];
#pragma unroll
        for (int c = 0; c < CB; ++c) {   // this lane's column of each 32-column block
            const int co = c * 32 + r;
            bc[c] = p.b1[co];
            ac[c] = p.a2[co];
            ic[c] = p.ib2[co];
        }
#pragma unroll
        for (int i = 0; i < RB; ++i)
#pragma unroll
            for (int c = 0; c < CB; ++c)
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    const int row = wave * 32 * RB + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * hh;
                    const float z = acc[i][c][reg] + bc[c];
                    hs[(size_t)row * HLD + c * 32 + r] = f2h(snake_apply(z, ac[c], ic[c]));
                }
        for (int e = tid; e < C * (C / 8); e += 256) {
            const int co = e / (C / 8), c8 = (e % (C / 8)) * 8;
            *reinterpret_cast<uint4 *>(w2s + (size_t)co * HLD + c8) = ldg16(p.w2 + (size_t)co * C + c8);
        }
    }
    __syncthreads();
    // ---------------- the 1-tap conv from LDS: K chunks of 32 in order, as k_conv_mt<1, 96, 3, 1, 0>
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
#pragma unroll
    for (int c0 = 0; c0 < C; c0 += KC) {
        const uint16_t *ab = hs + (size_t)(wave * 32 * RB + r) * HLD + c0 + 8 * hh;
        const uint16_t *bb = w2s + (size_t)r * HLD + c0 + 8 * hh;
#pragma unroll
        for (int kk = 0; kk < KC; kk += 16) {
            half8_t a[RB], b[CB];
#pragma unroll
            for (int i = 0; i < RB; ++i) a[i] = *reinterpret_cast<const half8_t *>(ab + (size_t)i * 32 * HLD + kk);
#pragma unroll
            for (int c = 0; c < CB; ++c) b[c] = *reinterpret_cast<const half8_t *>(bb + (size_t)c * 32 * HLD + kk);
#pragma unroll
            for (int i = 0; i < RB; ++i)
#pragma unroll
                for (int c = 0; c < CB; ++c) acc[i][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[c], acc[i][c], 0, 0, 0);
        }
    }
    __syncthreads();   // h / weights no longer read: the area takes the epilogue's transposed slices
    // ---------------- x' = x + (acc + b2), f32 out (optional) and f16 snake_next(x'): k_conv_mt's epilogue
    float *es = reinterpret_cast<float *>(sm) + wave * 32 * ELD;
    float *prm = reinterpret_cast<float *>(sm) + 4 * 32 * ELD;
    if (tid < C) {
        prm[tid] = p.b2[tid];
        prm[2 * C + tid] = p.an[tid];
        prm[3 * C + tid] = p.ibn[tid];
    }
    __syncthreads();
    constexpr int Q = C / 4, EK = 32 * Q / 64;
#pragma unroll
    for (int i = 0; i < RB; ++i) {
#pragma unroll
        for (int c = 0; c < CB; ++c)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg)
                es[((reg & 3) + 8 * (reg >> 2) + 4 * hh) * ELD + c * 32 + r] = acc[i][c][reg];
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the slice is in LDS (one wave writes and reads it)
        __builtin_amdgcn_wave_barrier();
#pragma unroll 4
        for (int k = 0; k < EK; ++k) {
            const int e = lane + 64 * k, row = e / Q, q4 = (e % Q) * 4;
            const int m = m0 + wave * 32 * RB + i * 32 + row;
            if (m >= T) continue;
            const size_t o = (size_t)m * C + q4;
            const float4 a = *reinterpret_cast<const float4 *>(es + row * ELD + q4);
            float v[4] = {a.x, a.y, a.z, a.w};
            const float4 b = *reinterpret_cast<const float4 *>(prm + q4);
            v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
            const float4 rr = *reinterpret_cast<const float4 *>(pres + o);
            v[0] = rr.x + v[0]; v[1] = rr.y + v[1]; v[2] = rr.z + v[2]; v[3] = rr.w + v[3];
            if (py) *reinterpret_cast<float4 *>(py + o) = make_float4(v[0], v[1], v[2], v[3]);
            float z[4] = {v[0], v[1], v[2], v[3]};
            const float4 sa = *reinterpret_cast<const float4 *>(prm + 2 * C + q4);
            const float4 sb = *reinterpret_cast<const float4 *>(prm + 3 * C + q4);
            const float av[4] = {sa.x, sa.y, sa.z, sa.w}, bv[4] = {sb.x, sb.y, sb.z, sb.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) z[q] = snake_apply(z[q], av[q], bv[q]);
            uint2 hv;
            hv.x = (uint32_t)f2h(z[0]) | ((uint32_t)f2h(z[1]) << 16);
            hv.y = (uint32_t)f2h(z[2]) | ((uint32_t)f2h(z[3]) << 16);
            *reinterpret_cast<uint2 *>(py16 + o) = hv;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

bool resunit96(const ResUnitParams &p, hipStream_t s) {
    if (p.T <= 0 || p.nb <= 0) return true;
    if (!p.xh || !p.x || !p.y16 || !p.w1 || !p.b1 || !p.a2 || !p.ib2 || !p.w2 || !p.b2 || !p.an || !p.ibn || p.dil < 1 ||
        6 * p.dil > MAXWIN - MT - 8 || (p.nb > 1 && p.bs < p.T)) {
        set_error("resunit96: bad parameters");
        return false;
    }
    const size_t lds = std::max({(size_t)(MT + 6 * p.dil + TAPS * C) * LDK * 2, (size_t)(MT + C) * HLD * 2,
                                 (size_t)4 * 32 * ELD * 4 + (size_t)4 * C * 4});
    static bool attr = false;
    if (!attr) {
        Q3T_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_resunit96), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    128 * 1024));
        attr = true;
    }
    const dim3 grid((p.T + MT - 1) / MT, 1, p.nb);
    hipLaunchKernelGGL(k_resunit96, grid, dim3(256), lds, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}

}  // namespace q3t
