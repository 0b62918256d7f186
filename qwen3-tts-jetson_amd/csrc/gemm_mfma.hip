// gemm_mfma.hip — batched decode projections on the gfx950 matrix cores (B >= Q3T_MFMA_MIN_B tokens).
//
// Y[b][n] = epilogue( W[n][:] . f16(prologue(X[b][:])) ) for up to 64 tokens per workgroup, W f16 [N][K] row-major
// exactly as in the GGUF.  The same GemvParams as the weight-streaming GEMV (gemv.hip); gemv() routes here when the
// batch is wide enough that the vector path's per-token FMAs and per-tile weight re-reads dominate (SURVEY §8(d):
// B = 64 concurrent utterances, BASELINE configs[2]).
//
// Tiling (one workgroup per 32 weight rows x 64 tokens, 4 waves = 4 K-quarters):
//   - v_mfma_f32_32x32x16_f16, A = the weight tile (32 rows), B = the activation tile (32 tokens), one or two token
//     tiles sharing every A fragment.  f16 x f16 products are exact and accumulate in f32: the numerics of the
//     vector path (and of ggml's f16 vec_dot) up to summation order.
//   - K permutation: lane (r, h) loads 64 contiguous bytes (32 halves) of row r per 64-wide K chunk and feeds
//     halves [8j, 8j+8) to k-step j.  A dot product may visit K in any order as long as both operands use the same
//     bijection, so A and B fragments are both plain 64-B row segments: full 128-B lines per lane pair, no shuffles.
//   - Every weight load of the lane (the HBM stream) is issued first, straight-line.
//   - Prologues: PRO_F16 reads f16 activation rows (optional row gather x_idx) from global memory in the same
//     fragment shape, issued a few chunks ahead; PRO_F32 / PRO_RMS / PRO_LN build the f16 activation tile in LDS
//     (norm sums in double, like gemv.hip), row stride K + 8 halves so ds_read_b128 is conflict-free.
//   - The 4 K-quarter partial tiles are summed through LDS; each wave then runs the epilogue of a quarter of the
//     tile (bias, activation, scale, residual, aux, SwiGLU pairs, f16/f32 stores of 4 consecutive rows).
#include "kernels.h"

#include <algorithm>

#include <cstdlib>

namespace q3t {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_g __attribute__((ext_vector_type(4)));
typedef float f32x4_g __attribute__((ext_vector_type(4)));

namespace {
template <class V>
__device__ __forceinline__ V gld(const void *p) {
    typedef const __attribute__((address_space(1))) V gV;
    return *(gV *)(p);
}
__device__ __forceinline__ uint4 gld16(const void *p) {
    const u32x4_g v = gld<u32x4_g>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 gldf4(const void *p) {
    const f32x4_g v = gld<f32x4_g>(p);
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ half8_t as_h8(const uint4 &u) { return __builtin_bit_cast(half8_t, u); }
}  // namespace

constexpr int MM_ROWS = 32;   // weight rows per workgroup (tokens: TT x 32)

// Split-K launches in XCD-aware tile order.  Workgroups are dispatched round-robin over the 8 XCDs (workgroup L on XCD
// L % 8), each with its own L2.  In grid order every XCD runs tiles of every K slice, so each XCD fetches the whole
// activation block (8 copies per launch: 1.42x the algorithmic bytes of the O / down projections at 64 slots).  Here
// the XCDs sharing K slice z = j % ks split that slice's (row, token) tiles between them, so each XCD fetches 1 / ks
// of the activations while every weight tile is still read once (its two token tiles stay adjacent on one XCD).
// Tiles and their arithmetic are unchanged.  Falls back to grid order when the grid does not divide.  Opt-in
// (GemvParams::xcd_slices): at 64 slots it cut the down projection's FETCH from 266 to 200 MB per step for +0.8 % of
// step time; on the O projection too it cost +3 % (1.65 vs 1.60 ms), so only the down projection uses it.
struct TileIdx { int x, y, z; };
__device__ __forceinline__ TileIdx splitk_tile() {
    const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
    TileIdx r{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
    const int pairs = gx * gy, share = 8 / gz;   // XCDs per K slice
    if (gz < 2 || 8 % gz != 0 || pairs % share != 0) return r;
    const int L = (int)blockIdx.x + gx * ((int)blockIdx.y + gy * (int)blockIdx.z);
    const int j = L & 7, i = L >> 3, per = pairs / share;
    const int pidx = (j / gz) * per + i;   // this XCD's i-th (row, token) pair of slice j % gz
    r.z = j % gz;
    r.x = pidx / gy;
    r.y = pidx % gy;
    return r;
}

// epilogue shared by the kernels: acc register i of lane (r, h) = tile row (i & 3) + 8 (i >> 2) + 4h, token r;
// sumf(tt, i) returns the K-summed value of register i of token tile tt for this lane
template <bool SWIGLU, int TT, class SumF>
__device__ __forceinline__ void mm_epilogue(const GemvParams &p, int wave, int lane, int r, int h, int row0, int t0,
                                            int nt, SumF sumf, int slab = 0) {
    const bool vec_ok = (p.ldo & 3) == 0;
    if constexpr (SWIGLU) {
        // combos (tt, q), q in {0, 1}: gate registers 4q..4q+3, up registers 4(q+2)..: unit = row0/2 + 8q + 4h + e
        if (wave < TT * 2) {
            const int tt = wave >> 1, q = wave & 1;
            const int tl = tt * 32 + r;
            if (tl < nt) {
                const int tok = t0 + tl;
                const size_t orow = (size_t)tok * p.orow_mul + p.orow_add;
                const int unit = row0 / 2 + 8 * q + 4 * h;
                float hv[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) hv[e] = silu_f(sumf(tt, 4 * q + e)) * sumf(tt, 4 * (q + 2) + e);
                if (p.out_f16) {
                    if (vec_ok) {
                        uint2 o;
                        o.x = (uint32_t)f2h(hv[0]) | ((uint32_t)f2h(hv[1]) << 16);
                        o.y = (uint32_t)f2h(hv[2]) | ((uint32_t)f2h(hv[3]) << 16);
                        *reinterpret_cast<uint2 *>(p.out_f16 + orow * p.ldo + unit) = o;
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) p.out_f16[orow * p.ldo + unit + e] = f2h(hv[e]);
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) p.out_f32[orow * p.ldo + unit + e] = hv[e];
                }
            }
        }
    } else if (p.parts) {   // split-K slab: raw partial sums of this K slice, [z][token][n]
        for (int combo = wave; combo < TT * 4; combo += (int)(blockDim.x >> 6)) {
            const int tt = combo >> 2, q = combo & 3;
            const int tl = tt * 32 + r;
            if (tl >= nt) continue;
            const int tok = t0 + tl;
            const int n0 = row0 + 8 * q + 4 * h;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = sumf(tt, 4 * q + e);
            *reinterpret_cast<float4 *>(p.parts + ((size_t)slab * p.B + tok) * p.N + n0) = make_float4(v[0], v[1], v[2], v[3]);
        }
    } else {
        for (int combo = wave; combo < TT * 4; combo += (int)(blockDim.x >> 6)) {
            const int tt = combo >> 2, q = combo & 3;
            const int tl = tt * 32 + r;
            if (tl >= nt) continue;
            const int tok = t0 + tl;
            const size_t orow = (size_t)tok * p.orow_mul + p.orow_add;
            const int n0 = row0 + 8 * q + 4 * h;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = sumf(tt, 4 * q + e);
            float bb[4] = {0.f, 0.f, 0.f, 0.f}, sc[4] = {1.f, 1.f, 1.f, 1.f}, rs[4] = {0.f, 0.f, 0.f, 0.f}, ax[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (p.bias) bb[e] = p.bias[n0 + e];
                if (p.scale) sc[e] = p.scale[n0 + e];
                if (p.resid) rs[e] = p.resid[(size_t)tok * p.ldr + n0 + e];
                if (p.aux) ax[e] = p.aux[(size_t)tok * p.lda + n0 + e];
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float x = v[e];
                if (p.bias) x += bb[e];
                if (p.act == ACT_SILU) x = silu_f(x);
                else if (p.act == ACT_GELU) x = gelu_ggml(x);
                if (p.scale) x *= sc[e];
                if (p.resid) x = rs[e] + x;
                if (p.aux) x = ax[e] + x;
                v[e] = x;
            }
            if (p.out_f16) {
                if (vec_ok) {
                    uint2 o;
                    o.x = (uint32_t)f2h(v[0]) | ((uint32_t)f2h(v[1]) << 16);
                    o.y = (uint32_t)f2h(v[2]) | ((uint32_t)f2h(v[3]) << 16);
                    *reinterpret_cast<uint2 *>(p.out_f16 + orow * p.ldo + n0) = o;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) p.out_f16[orow * p.ldo + n0 + e] = f2h(v[e]);
                }
            } else if (vec_ok) {
                *reinterpret_cast<float4 *>(p.out_f32 + orow * p.ldo + n0) = make_float4(v[0], v[1], v[2], v[3]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) p.out_f32[orow * p.ldo + n0 + e] = v[e];
            }
        }
    }
}

template <int PRO, int NCH, int TT, bool SWIGLU>
__global__ void __launch_bounds__(256, 1) k_gemm_mfma(const GemvParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr bool kLds = PRO != PRO_F16;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int K = NCH * 256;
    if (PRO == PRO_F16 && (int)blockIdx.x >= p.N / MM_ROWS) {
        // prefetch workgroup (GemvParams::prefetch): global->LDS dword loads, nothing to wait on
        const int ntx = p.N / MM_ROWS;
        const size_t lines = p.prefetch_bytes / 128, nthr = (size_t)(gridDim.x - ntx) * 256;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const size_t line = (size_t)q * nthr + (size_t)(blockIdx.x - ntx) * 256 + tid;
            if (line < lines)
                __builtin_amdgcn_global_load_lds(static_cast<const uint8_t *>(p.prefetch) + line * 128,
                                                 (__attribute__((address_space(3))) void *)smem, 4, 0, 0);
        }
        return;
    }
    const TileIdx ti = PRO == PRO_F16 && p.parts && p.xcd_slices ? splitk_tile() : TileIdx{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
    const int row0 = ti.x * MM_ROWS;
    const int t0 = ti.y * (TT * 32);
    const int nt = min(TT * 32, p.B - t0);
    const int kw0 = wave * (NCH * 64);   // first K index of this wave's quarter

    // every weight load of the lane: row row0 + r, k = kw0 + 64c + 32h .. +31.  Issued right after the first
    // activation loads (whose addresses must not wait behind them: vmcnt retires in issue order)
    uint4 wr[NCH][4];
    // f16 rows may be one K slice of a split-K launch (grid z): the weight row stride is the full K
    const int kz = PRO == PRO_F16 ? ti.z * K : 0;
    const uint16_t *wp = p.W + (size_t)(row0 + r) * (PRO == PRO_F16 ? p.K : K) + kz + kw0 + h * 32;
    const bool dbg_now = p.dbg & 2, dbg_nox = p.dbg & 1;
    auto issue_w = [&]() {
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) wr[c][j] = dbg_now ? make_uint4(j, c, 0, 0) : gld16(wp + c * 64 + j * 8);
    };

    f32x16_t acc[TT];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[tt][i] = 0.0f;

    if constexpr (kLds) {
        // ---------------- (2a) activation tile in LDS: 16 tokens per wave, f16 rows of K + 8 halves
        constexpr int KP = NCH * 256 + 8;
        uint16_t *xs = reinterpret_cast<uint16_t *>(smem);
        const float *X = reinterpret_cast<const float *>(p.x);
        float4 nwv[NCH], nbv[NCH];
        if constexpr (PRO == PRO_RMS || PRO == PRO_LN) {
#pragma unroll
            for (int it = 0; it < NCH; ++it) {
                nwv[it] = gldf4(p.nw + it * 256 + lane * 4);
                nbv[it] = PRO == PRO_LN ? gldf4(p.nb + it * 256 + lane * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        // rows in groups of 4, two groups in flight (L2-served); the weight stream (HBM) is issued behind the first
        // two groups so that their norms do not wait for it (vmcnt retires in issue order)
        float4 xa[4][4][NCH];
        auto issue_x = [&](int g) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int tl = wave * 16 + g * 4 + q;
                const float *row = X + (size_t)(t0 + min(tl, nt - 1)) * p.ldx;
#pragma unroll
                for (int it = 0; it < NCH; ++it) xa[g][q][it] = dbg_nox ? make_float4(q, it, 1.f, 0.f) : gldf4(row + it * 256 + lane * 4);
            }
        };
        issue_x(0);
        issue_x(1);
        __builtin_amdgcn_sched_barrier(0);
        issue_w();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if (g >= 1 && g + 1 < 4) {
                __builtin_amdgcn_sched_barrier(0);
                issue_x(g + 1);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int tl = wave * 16 + g * 4 + q;
                float4 (&xvq)[NCH] = xa[g][q];
                const bool valid = tl < nt;
                float scale = 1.0f, mean = 0.0f;
                if constexpr (PRO == PRO_RMS) {
                    double ss = 0.0;
#pragma unroll
                    for (int it = 0; it < NCH; ++it) {
                        const float4 v = xvq[it];
                        ss += (double)(v.x * v.x) + (double)(v.y * v.y) + (double)(v.z * v.z) + (double)(v.w * v.w);
                    }
                    ss = wave_sum_d(ss);
                    scale = 1.0f / sqrtf((float)(ss / K) + p.eps);
                } else if constexpr (PRO == PRO_LN) {
                    double s1 = 0.0;
#pragma unroll
                    for (int it = 0; it < NCH; ++it) {
                        const float4 v = xvq[it];
                        s1 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
                    }
                    s1 = wave_sum_d(s1);
                    mean = (float)(s1 / K);
                    double s2 = 0.0;
#pragma unroll
                    for (int it = 0; it < NCH; ++it) {
                        const float4 v = xvq[it];
                        const float dx = v.x - mean, dy = v.y - mean, dz = v.z - mean, dw = v.w - mean;
                        s2 += (double)(dx * dx) + (double)(dy * dy) + (double)(dz * dz) + (double)(dw * dw);
                    }
                    s2 = wave_sum_d(s2);
                    scale = 1.0f / sqrtf((float)(s2 / K) + p.eps);
                }
                const bool side = valid && blockIdx.x == 0;
#pragma unroll
                for (int it = 0; it < NCH; ++it) {
                    const int k = it * 256 + lane * 4;
                    const float4 v = xvq[it];
                    float y[4] = {v.x, v.y, v.z, v.w};
                    if constexpr (PRO == PRO_RMS || PRO == PRO_LN) {
                        const float w4[4] = {nwv[it].x, nwv[it].y, nwv[it].z, nwv[it].w};
                        const float c4[4] = {nbv[it].x, nbv[it].y, nbv[it].z, nbv[it].w};
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            if constexpr (PRO == PRO_RMS) y[e] = (y[e] * scale) * w4[e];
                            else y[e] = ((y[e] - mean) * scale) * w4[e] + c4[e];
                        }
                    }
                    if (side && p.raw_out) *reinterpret_cast<float4 *>(p.raw_out + (size_t)(t0 + tl) * K + k) = v;
                    if (side && p.side_out)
                        *reinterpret_cast<float4 *>(p.side_out + (size_t)(t0 + tl) * K + k) = make_float4(y[0], y[1], y[2], y[3]);
                    uint2 hv;
                    hv.x = valid ? ((uint32_t)f2h(y[0]) | ((uint32_t)f2h(y[1]) << 16)) : 0u;
                    hv.y = valid ? ((uint32_t)f2h(y[2]) | ((uint32_t)f2h(y[3]) << 16)) : 0u;
                    *reinterpret_cast<uint2 *>(xs + (size_t)tl * KP + k) = hv;
                }
            }
        }
        __syncthreads();
        // ---------------- (3a) MFMA over the wave's K quarter, B fragments from LDS
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const half8_t a = as_h8(wr[c][j]);
#pragma unroll
                for (int tt = 0; tt < TT; ++tt) {
                    const half8_t b = *reinterpret_cast<const half8_t *>(xs + (size_t)(tt * 32 + r) * KP + kw0 + c * 64 + h * 32 + j * 8);
                    acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[tt], 0, 0, 0);
                }
            }
        __syncthreads();   // the reduction below reuses the LDS tile
    } else {
        // ---------------- (2b)+(3b) f16 activation rows from global memory in fragment shape, MM_XD chunks ahead
        const uint16_t *xrow[TT];
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
            const int tok = t0 + min(tt * 32 + r, nt - 1);
            const int src = p.x_idx ? p.x_idx[tok] : tok;
            xrow[tt] = reinterpret_cast<const uint16_t *>(p.x) + (size_t)src * p.ldx + kz + kw0 + h * 32;
        }
        // one ring for both operands: chunk c = 4 weight loads + 4 TT activation loads, XD chunks in flight
        constexpr int XD = NCH < (TT == 2 ? 3 : 4) ? NCH : (TT == 2 ? 3 : 4);
        uint4 xr[NCH][TT][4];
        auto issue_chunk = [&](int c) {
#pragma unroll
            for (int j = 0; j < 4; ++j) wr[c][j] = dbg_now ? make_uint4(j, c, 0, 0) : gld16(wp + c * 64 + j * 8);
#pragma unroll
            for (int tt = 0; tt < TT; ++tt)
#pragma unroll
                for (int j = 0; j < 4; ++j) xr[c][tt][j] = dbg_nox ? make_uint4(j, tt, c, 0) : gld16(xrow[tt] + c * 64 + j * 8);
        };
#pragma unroll
        for (int c = 0; c < XD; ++c) issue_chunk(c);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            // pinned schedule: chunk c + XD is issued, then chunk c's MFMAs run (left alone, the scheduler
            // interleaves loads with MFMAs and keeps only ~2 in flight)
            __builtin_amdgcn_sched_barrier(0);
            if (c + XD < NCH) issue_chunk(c + XD);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const half8_t a = as_h8(wr[c][j]);
#pragma unroll
                for (int tt = 0; tt < TT; ++tt) acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, as_h8(xr[c][tt][j]), acc[tt], 0, 0, 0);
            }
        }
    }

    // ---------------- (4) sum the 4 K-quarters through LDS: red[wave][tt][reg][lane]
    float *red = reinterpret_cast<float *>(smem);
#pragma unroll
    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[((wave * TT + tt) * 16 + i) * 64 + lane] = acc[tt][i];
    __syncthreads();

    // ---------------- (5) epilogue
    auto sum4 = [&](int tt, int i) {
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < 4; ++w) v += red[((w * TT + tt) * 16 + i) * 64 + lane];
        return v;
    };
    mm_epilogue<SWIGLU, TT>(p, wave, lane, r, h, row0, t0, nt, sum4, ti.z);
}

// ------------------------------------------------------------------------------------------ norm prologues, 16 waves
// PRO_F32 / PRO_RMS / PRO_LN at K <= 1024: the per-token norm is a chain of dependent VALU work (double sums, wave
// reductions) that one wave per SIMD cannot hide (measured: ~12 us of a 17 us launch at B = 64 with no loads at all).
// 1024 threads spread it over 16 waves (4 tokens each, issued together); K splits into 64-wide chunks, one per wave
// (K / 64 waves take part in the MFMA phase), summed through LDS.
template <int PRO, int NCH, int TT, bool SWIGLU>
__global__ void __launch_bounds__(1024, 1) k_gemm_mfma_norm(const GemvParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int K = NCH * 256, NCHK = K / 64, KP = K + 8;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int row0 = blockIdx.x * MM_ROWS;
    const int t0 = blockIdx.y * (TT * 32);
    const int nt = min(TT * 32, p.B - t0);
    const bool mma = wave < NCHK;
    const bool dbg_now = p.dbg & 2, dbg_nox = p.dbg & 1;
    uint16_t *xs = reinterpret_cast<uint16_t *>(smem);
    const float *X = reinterpret_cast<const float *>(p.x);
    // (1) the wave's 2 TT activation rows, all in flight; then its weight chunk
    constexpr int TPW = 2 * TT;   // tokens per wave (TT * 32 tokens over 16 waves)
    float4 xa[TPW][NCH];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const float *row = X + (size_t)(t0 + min(wave * TPW + q, nt - 1)) * p.ldx;
#pragma unroll
        for (int it = 0; it < NCH; ++it) xa[q][it] = dbg_nox ? make_float4(q, it, 1.f, 0.f) : gldf4(row + it * 256 + lane * 4);
    }
    uint4 wr[4];
    {
        const uint16_t *wp = p.W + (size_t)(row0 + r) * K + (mma ? wave : 0) * 64 + h * 32;
#pragma unroll
        for (int j = 0; j < 4; ++j) wr[j] = dbg_now ? make_uint4(j, 1, 0, 0) : gld16(wp + j * 8);
    }
    __builtin_amdgcn_sched_barrier(0);
    // (2) norms -> f16 rows in LDS
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int tl = wave * TPW + q;
        const bool valid = tl < nt;
        float scale = 1.0f, mean = 0.0f;
        if constexpr (PRO == PRO_RMS) {
            double ss = 0.0;
#pragma unroll
            for (int it = 0; it < NCH; ++it) {
                const float4 v = xa[q][it];
                ss += (double)(v.x * v.x) + (double)(v.y * v.y) + (double)(v.z * v.z) + (double)(v.w * v.w);
            }
            ss = wave_sum_d(ss);
            scale = 1.0f / sqrtf((float)(ss / K) + p.eps);
        } else if constexpr (PRO == PRO_LN) {
            double s1 = 0.0;
#pragma unroll
            for (int it = 0; it < NCH; ++it) {
                const float4 v = xa[q][it];
                s1 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
            }
            s1 = wave_sum_d(s1);
            mean = (float)(s1 / K);
            double s2 = 0.0;
#pragma unroll
            for (int it = 0; it < NCH; ++it) {
                const float4 v = xa[q][it];
                const float dx = v.x - mean, dy = v.y - mean, dz = v.z - mean, dw = v.w - mean;
                s2 += (double)(dx * dx) + (double)(dy * dy) + (double)(dz * dz) + (double)(dw * dw);
            }
            s2 = wave_sum_d(s2);
            scale = 1.0f / sqrtf((float)(s2 / K) + p.eps);
        }
        const bool side = valid && blockIdx.x == 0;
#pragma unroll
        for (int it = 0; it < NCH; ++it) {
            const int k = it * 256 + lane * 4;
            const float4 v = xa[q][it];
            float y[4] = {v.x, v.y, v.z, v.w};
            if constexpr (PRO == PRO_RMS || PRO == PRO_LN) {
                const float4 w4 = gldf4(p.nw + k);
                const float4 c4 = PRO == PRO_LN ? gldf4(p.nb + k) : make_float4(0.f, 0.f, 0.f, 0.f);
                const float wv[4] = {w4.x, w4.y, w4.z, w4.w}, cv[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if constexpr (PRO == PRO_RMS) y[e] = (y[e] * scale) * wv[e];
                    else y[e] = ((y[e] - mean) * scale) * wv[e] + cv[e];
                }
            }
            if (side && p.raw_out) *reinterpret_cast<float4 *>(p.raw_out + (size_t)(t0 + tl) * K + k) = v;
            if (side && p.side_out)
                *reinterpret_cast<float4 *>(p.side_out + (size_t)(t0 + tl) * K + k) = make_float4(y[0], y[1], y[2], y[3]);
            uint2 hv;
            hv.x = valid ? ((uint32_t)f2h(y[0]) | ((uint32_t)f2h(y[1]) << 16)) : 0u;
            hv.y = valid ? ((uint32_t)f2h(y[2]) | ((uint32_t)f2h(y[3]) << 16)) : 0u;
            *reinterpret_cast<uint2 *>(xs + (size_t)tl * KP + k) = hv;
        }
    }
    __syncthreads();
    // (3) MFMA over this wave's 64-wide K chunk
    f32x16_t acc[TT];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[tt][i] = 0.0f;
    if (mma) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const half8_t a = as_h8(wr[j]);
#pragma unroll
            for (int tt = 0; tt < TT; ++tt) {
                const half8_t b = *reinterpret_cast<const half8_t *>(xs + (size_t)(tt * 32 + r) * KP + wave * 64 + h * 32 + j * 8);
                acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[tt], 0, 0, 0);
            }
        }
    }
    __syncthreads();   // the reduction reuses the activation tile
    float *red = reinterpret_cast<float *>(smem);
    if (mma)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt)
#pragma unroll
            for (int i = 0; i < 16; ++i) red[((wave * TT + tt) * 16 + i) * 64 + lane] = acc[tt][i];
    __syncthreads();
    auto sum_k = [&](int tt, int i) {
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < NCHK; ++w) v += red[((w * TT + tt) * 16 + i) * 64 + lane];
        return v;
    };
    mm_epilogue<SWIGLU, TT>(p, wave, lane, r, h, row0, t0, nt, sum_k);
}

// ------------------------------------------------------------------------------------------ split-K, f16 rows
// PRO_F16 projections whose epilogue is linear and lands in place on the residual stream (O-proj, down-proj:
// out = x + scale * (W.h + bias)): grid z splits K into 256-wide slices (one 64-wide chunk per wave), so N = 1024
// projections fill 256-384 workgroups instead of 32; each slice adds its scaled partial with a no-return f32 atomic
// (bias once, by slice 0).  The sum order of the slices is unspecified: the residual stream is reproducible to f32
// rounding, not bitwise, on this path.
template <int TT>
__global__ void __launch_bounds__(256, 2) k_gemm_mfma_splitk(const GemvParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int K = p.K;
    const int row0 = blockIdx.x * MM_ROWS;
    const int t0 = blockIdx.y * (TT * 32);
    const int nt = min(TT * 32, p.B - t0);
    const int k0 = blockIdx.z * 256 + wave * 64 + h * 32;
    const bool dbg_now = p.dbg & 2, dbg_nox = p.dbg & 1;
    const uint16_t *xrow[TT];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
        const int tok = t0 + min(tt * 32 + r, nt - 1);
        const int src = p.x_idx ? p.x_idx[tok] : tok;
        xrow[tt] = reinterpret_cast<const uint16_t *>(p.x) + (size_t)src * p.ldx + k0;
    }
    uint4 wr[4], xr[TT][4];
    const uint16_t *wp = p.W + (size_t)(row0 + r) * K + k0;
#pragma unroll
    for (int j = 0; j < 4; ++j) wr[j] = dbg_now ? make_uint4(j, 1, 0, 0) : gld16(wp + j * 8);
#pragma unroll
    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int j = 0; j < 4; ++j) xr[tt][j] = dbg_nox ? make_uint4(j, tt, 1, 0) : gld16(xrow[tt] + j * 8);
    f32x16_t acc[TT];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[tt][i] = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const half8_t a = as_h8(wr[j]);
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, as_h8(xr[tt][j]), acc[tt], 0, 0, 0);
    }
    float *red = reinterpret_cast<float *>(smem);
#pragma unroll
    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[((wave * TT + tt) * 16 + i) * 64 + lane] = acc[tt][i];
    __syncthreads();
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
        const int combo = wave + 4 * cc;
        if (combo >= TT * 4) break;
        const int tt = combo >> 2, q = combo & 3;
        const int tl = tt * 32 + r;
        if (tl >= nt) continue;
        const int tok = t0 + tl;
        const size_t orow = (size_t)tok * p.orow_mul + p.orow_add;
        const int n0 = row0 + 8 * q + 4 * h;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float v = 0.0f;
#pragma unroll
            for (int w = 0; w < 4; ++w) v += red[((w * TT + tt) * 16 + 4 * q + e) * 64 + lane];
            if (p.bias && blockIdx.z == 0) v += p.bias[n0 + e];
            if (p.scale) v *= p.scale[n0 + e];
            unsafeAtomicAdd(p.out_f32 + orow * p.ldo + n0 + e, v);
        }
    }
}

// ------------------------------------------------------------------------------------------ host dispatch
static int g_mfma_min_b = [] {
    const char *e = std::getenv("Q3T_MFMA_MIN_B");
    return e ? std::atoi(e) : 4;
}();
int gemm_mfma_min_batch() { return g_mfma_min_b <= 0 ? (1 << 30) : g_mfma_min_b; }
void gemm_mfma_set_min_batch(int b) { g_mfma_min_b = b; }

static int nch_of(int K) {
    switch (K) {
        case 256: return 1;
        case 512: return 2;
        case 1024: return 4;
        case 2048: return 8;
        case 3072: return 12;
        default: return 0;
    }
}

bool gemm_mfma_supported(const GemvParams &p) {
    if (((p.family_b > 0 ? p.family_b : p.B) < gemm_mfma_min_batch() && !p.force_mm) || p.sel.mode != SEL_NONE || p.N % MM_ROWS != 0) return false;
    const int nch = nch_of(p.K);
    if (!nch) return false;
    const bool swiglu = p.act == ACT_SWIGLU;
    if (swiglu && p.pro != PRO_RMS && !(p.pro == PRO_F16 && nch <= 4 && !p.x_idx)) return false;
    if (p.parts) {   // split-K slabs: f16 rows, no epilogue, K slices of 256-multiples
        const int nk = p.ksplit > 0 && nch % p.ksplit == 0 ? nch / p.ksplit : 0;
        if (p.pro != PRO_F16 || swiglu || !(nk == 1 || nk == 2 || nk == 3 || nk == 4 || nk == 8 || nk == 12) ||
            p.N % 4 != 0)
            return false;
    }
    const uintptr_t xa = reinterpret_cast<uintptr_t>(p.x);
    switch (p.pro) {
        case PRO_F16: return (xa & 15) == 0 && p.ldx % 8 == 0;
        case PRO_F32: case PRO_RMS: case PRO_LN:
            return nch <= 4 && (xa & 15) == 0 && p.ldx % 4 == 0 && !p.x_idx;
        default: return false;   // gather / fused-attention prologues stay on the vector path
    }
}

// split-K with f32 atomics onto the residual: measured slower at B = 64 (the atomic traffic of 256-384 workgroups x
// 2048 adds costs ~20 us), so off unless Q3T_MFMA_SPLITK=1
// (development builds only: make DEV=1)
static bool g_splitk = [] {
#ifdef Q3T_DEV
    const char *e = std::getenv("Q3T_MFMA_SPLITK");
    return e ? std::atoi(e) != 0 : false;
#else
    return false;
#endif
}();
// 32-token tiles per workgroup (TT) : 1 = 32 tokens (more workgroups, weights re-read from L2 per token block),
// 2 = 64 tokens; Q3T_MFMA_TT (development builds)
static int g_tt = [] {
#ifdef Q3T_DEV
    const char *e = std::getenv("Q3T_MFMA_TT");
    return e && std::atoi(e) == 2 ? 2 : 1;
#else
    return 1;
#endif
}();

static bool set_lds(const void *fn, size_t lds, bool &done) {
    if (!done) {
        Q3T_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        done = true;
    }
    return true;
}

// f16 rows, one workgroup per 32 rows x 64 tokens over all of K (4 waves = 4 K-quarters)
template <int NCH, int TT, bool SW>
static bool launch_f16_sw(const GemvParams &p, hipStream_t s) {
    const size_t lds = (size_t)4 * TT * 16 * 64 * 4;
    static bool attr = false;
    if (!set_lds(reinterpret_cast<const void *>(&k_gemm_mfma<PRO_F16, NCH, TT, SW>), lds, attr)) return false;
    const unsigned gy = (unsigned)((p.B + TT * 32 - 1) / (TT * 32));
    // prefetch workgroups only on a one-row, unsplit grid (their index is blockIdx.x past the row tiles)
    const size_t pf_lines = p.prefetch && !p.parts && gy == 1 ? p.prefetch_bytes / 128 : 0;
    const unsigned pf_wgs = (unsigned)std::min<size_t>((pf_lines + 511) / 512, 1024);
    const dim3 grid((unsigned)(p.N / MM_ROWS) + pf_wgs, gy, (unsigned)(p.parts ? p.ksplit : 1));
    hipLaunchKernelGGL((k_gemm_mfma<PRO_F16, NCH, TT, SW>), grid, dim3(256), lds, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}
template <int NCH, int TT>
static bool launch_f16(const GemvParams &p, hipStream_t s) {
    if constexpr (NCH <= 4) {
        if (p.act == ACT_SWIGLU) return launch_f16_sw<NCH, TT, true>(p, s);
    }
    return launch_f16_sw<NCH, TT, false>(p, s);
}
// f16 rows, split-K in 256-wide slices with atomic accumulation onto the residual stream
template <int TT>
static bool launch_splitk(const GemvParams &p, hipStream_t s) {
    const size_t lds = (size_t)4 * TT * 16 * 64 * 4;
    const dim3 grid((unsigned)(p.N / MM_ROWS), (unsigned)((p.B + TT * 32 - 1) / (TT * 32)), (unsigned)(p.K / 256));
    hipLaunchKernelGGL((k_gemm_mfma_splitk<TT>), grid, dim3(256), lds, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}
// f32 rows with a norm prologue (16 waves)
template <int PRO, int NCH, int TT, bool SW>
static bool launch_norm(const GemvParams &p, hipStream_t s) {
    const size_t xt = (size_t)TT * 32 * (NCH * 256 + 8) * 2, red = (size_t)(NCH * 4) * TT * 16 * 64 * 4;
    const size_t lds = xt > red ? xt : red;
    static bool attr = false;
    if (!set_lds(reinterpret_cast<const void *>(&k_gemm_mfma_norm<PRO, NCH, TT, SW>), lds, attr)) return false;
    const dim3 grid((unsigned)(p.N / MM_ROWS), (unsigned)((p.B + TT * 32 - 1) / (TT * 32)));
    hipLaunchKernelGGL((k_gemm_mfma_norm<PRO, NCH, TT, SW>), grid, dim3(1024), lds, s, p);
    Q3T_HIP(hipGetLastError());
    return true;
}
template <int PRO, int NCH, int TT>
static bool launch_norm_sw(const GemvParams &p, hipStream_t s) {
    if constexpr (PRO == PRO_RMS) {
        if (p.act == ACT_SWIGLU) return launch_norm<PRO, NCH, TT, true>(p, s);
    }
    return launch_norm<PRO, NCH, TT, false>(p, s);
}
template <int PRO>
static bool launch_norm_nch(const GemvParams &p, hipStream_t s) {
    const bool two = g_tt == 2 && p.B > 32;
    switch (nch_of(p.K)) {
        case 1: return two ? launch_norm_sw<PRO, 1, 2>(p, s) : launch_norm_sw<PRO, 1, 1>(p, s);
        case 2: return two ? launch_norm_sw<PRO, 2, 2>(p, s) : launch_norm_sw<PRO, 2, 1>(p, s);
        default: return two ? launch_norm_sw<PRO, 4, 2>(p, s) : launch_norm_sw<PRO, 4, 1>(p, s);
    }
}
template <int NCH>
static bool launch_f16_tt(const GemvParams &p, hipStream_t s) {
    return (p.mm_tt ? p.mm_tt : g_tt) == 2 && p.B > 32 ? launch_f16<NCH, 2>(p, s) : launch_f16<NCH, 1>(p, s);
}

bool gemm_mfma(const GemvParams &p, hipStream_t s) {
    switch (p.pro) {
        case PRO_F16: {
            const bool linear_inplace = p.act == ACT_NONE && !p.out_f16 && p.out_f32 && p.resid == p.out_f32 &&
                                        p.ldr == p.ldo && !p.aux && p.K % 256 == 0;
            if (g_splitk && linear_inplace && !p.parts) return g_tt == 2 && p.B > 32 ? launch_splitk<2>(p, s) : launch_splitk<1>(p, s);
            const int nch = nch_of(p.K) / (p.parts ? p.ksplit : 1);
            switch (nch) {
                case 1: return launch_f16_tt<1>(p, s);
                case 2: return launch_f16_tt<2>(p, s);
                case 3: return launch_f16_tt<3>(p, s);
                case 4: return launch_f16_tt<4>(p, s);
                case 8: return launch_f16_tt<8>(p, s);
                default: return launch_f16_tt<12>(p, s);
            }
        }
        case PRO_F32: return launch_norm_nch<PRO_F32>(p, s);
        case PRO_RMS: return launch_norm_nch<PRO_RMS>(p, s);
        default: return launch_norm_nch<PRO_LN>(p, s);
    }
}

}  // namespace q3t
