// gemv_kernel.h — the weight-streaming GEMV of the decode path (gfx950): the kernel and its launch templates, included
// by the gemv_inst_*.hip translation units that instantiate them (split for parallel compilation) and by gemv.hip.
//
// y[b][n] = epilogue( W[n][:] . f16(prologue(x[b][:])) ), W f16 row-major [N][K] exactly as stored in the GGUF.
// Numerics follow the reference CPU path (GGML_CUDA=OFF): the matmul input activation is rounded to f16 (ggml
// mul_mat converts src1 to vec_dot_type F16), products are exact f16 x f16 (v_dot2_f32_f16) accumulated in f32,
// RMSNorm / LayerNorm sums in double (ggml_compute_forward_rms_norm_f32 / norm_f32) [ggml-upstream].
//
// Batch-1 decode is latency-bound, not bandwidth-bound: a 4-12 MB GEMV is ONE memory round trip per lane, so the
// kernel is built around issuing every load it will ever need up front, in this order, in straight-line code:
//   1. the activation rows (f32 / f16), the norm weights and the epilogue operands;
//   2. every weight load of the lane (NL x RPG 16-B loads), then the gathered table rows (their addresses need
//      the scalar token loads);
//   3. the prologue math (RMSNorm / LayerNorm) waits only for (1) (partial vmcnt) while (2) is in flight, stages the
//      f16 activation tile in LDS, and the dot products then consume the weight registers.
// Block = 256 threads = 16 row-groups of 16 lanes; KS in {1,2,4} splits K over waves so that small-N GEMVs still
// launch >= Q3T_GEMV_MIN_BLOCKS workgroups (default 256: one per CU; measured faster than 512 for the RMS
// prologue shapes, tools/dev/kbench).  Large-K or wide-batch calls
// (prefill, vocoder) take the streaming loop (NL = 0).
#pragma once
#include "kernels.h"
#include "select.h"
#include "cpatt.h"

#include <cstdlib>

#ifndef Q3T_GEMV_NT
#define Q3T_GEMV_NT 0   // 1: non-temporal weight loads (the compiler then waits vmcnt(0) for every earlier load)
#endif

namespace q3t {

// global-address-space loads (never flat).  Through native clang vector types: an address-space-qualified
// HIP_vector_type struct is copied through a generic reference and comes back as a flat load.
template <class V>
__device__ __forceinline__ V ldg_v(const void *p) {
    typedef const __attribute__((address_space(1))) V gV;
    return *(gV *)(p);
}
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldg(const uint4 *p) { const u32x4_t v = ldg_v<u32x4_t>(p); return make_uint4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ uint2 ldg(const uint2 *p) { const u32x2_t v = ldg_v<u32x2_t>(p); return make_uint2(v.x, v.y); }
__device__ __forceinline__ float4 ldg(const float4 *p) { const f32x4_t v = ldg_v<f32x4_t>(p); return make_float4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ float ldg(const float *p) { return ldg_v<float>(p); }
__device__ __forceinline__ uint4 ld_w(const uint16_t *p) {
#if Q3T_GEMV_NT
    return ld_nt16(p);
#else
    return ldg(reinterpret_cast<const uint4 *>(p));
#endif
}
__device__ __forceinline__ float4 f4_zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ float4 f4_add(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 h4_to_f4(uint2 u) {
    return make_float4(h2f(u.x & 0xffff), h2f(u.x >> 16), h2f(u.y & 0xffff), h2f(u.y >> 16));
}

// f32 activation row b -> registers: element k = t*1024 + tid*4 + e, t < 4 (K <= 4096).  Loads are unconditional
// (out-of-range chunks re-read element 0) so the compiler can count them; mask_x zeroes the invalid chunks later.
__device__ __forceinline__ void issue_x_plain(const GemvParams &p, int b, float4 (&r)[4]) {
    const int tid = threadIdx.x, K = p.K, xt = (K + 1023) >> 10;
    const int row = p.x_idx ? p.x_idx[b] : b;
    const float *src = reinterpret_cast<const float *>(p.x) + (size_t)row * p.ldx;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int k = t * 1024 + tid * 4;
        r[t] = ldg(reinterpret_cast<const float4 *>(src + ((t < xt && k < K) ? k : 0)));
    }
}
__device__ __forceinline__ void mask_x(int K, bool valid, float4 (&r)[4]) {
    const int xt = (K + 1023) >> 10;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int k = t * 1024 + (int)threadIdx.x * 4;
        if (!(valid && t < xt && k < K)) r[t] = f4_zero();
    }
}
// GatherSum rows (K <= 1024: element k = tid*4 + e), NT = 1 (one table row: code-predictor pass input,
// trt_code_predictor.cpp:552-592) or 16 (codec_embd + 15 code-predictor tables + trailing/pad: the talker step
// embedding, tts_transformer.cpp:2529-2553), summed left to right in f32.  Tokens and table pointers are uniform
// scalar loads; every row load is issued before any sum.
template <int NT>
__device__ __forceinline__ void issue_x_gather(const GemvParams &p, int b, float4 (&r)[4], int tok_sel = -1) {
    const GatherSum &gs = p.gs;
    const int tid = threadIdx.x, K = p.K;
    const uint16_t *row[NT];
    const float *extra = nullptr;
    if constexpr (NT == 1) {
        row[0] = gs.tab0 + (size_t)(tok_sel >= 0 ? tok_sel : gs.tok[(size_t)b * gs.tok_ld + gs.tok_col0]) * K;
    } else {
        const int *tk = gs.tok + (size_t)b * gs.tok_ld;   // the 16 codes of the frame, [S][16]
#pragma unroll
        for (int j = 0; j < NT; ++j) row[j] = gs.tabs[j] + (size_t)tk[j] * K;
        const int fr = gs.frame[b];
        extra = fr < gs.tr_len[b] ? gs.tr + (size_t)b * gs.tr_ld + (size_t)fr * K : gs.pad + (size_t)b * K;
    }
    const int k = tid * 4;
    const bool ok = k < K;
    const int kk = ok ? k : 0;
    uint2 hv[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) hv[j] = ldg(reinterpret_cast<const uint2 *>(row[j] + kk));
    float4 ex = f4_zero();
    if constexpr (NT > 1) ex = ldg(reinterpret_cast<const float4 *>(extra + kk));
    float4 a = h4_to_f4(hv[0]);
#pragma unroll
    for (int j = 1; j < NT; ++j) a = f4_add(a, h4_to_f4(hv[j]));
    if constexpr (NT > 1) a = f4_add(a, ex);
    r[0] = a;   // masked by mask_x
    r[1] = r[2] = r[3] = f4_zero();
}

template <int XB>
__device__ __forceinline__ void block_sum_dn(double (&v)[XB], double *scr /* [4][XB] */) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < XB; ++q) v[q] = wave_sum_d(v[q]);
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < XB; ++q) scr[wave * XB + q] = v[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < XB; ++q) v[q] = (scr[q] + scr[XB + q]) + (scr[2 * XB + q] + scr[3 * XB + q]);
}


// ------------------------------------------------------------------------------------------ PRO_CPATT prologue
// Code-predictor attention for one slot, recomputed by every O-projection workgroup (<= 16 positions: 64 KB of
// F16 K/V, L2-resident) so the separate attention launch and its kernel boundary disappear.  The arithmetic is
// cpatt.h's, shared with the persistent code-predictor frame (persist.hip).
__device__ __forceinline__ void cpatt_issue(const GemvParams &p, int b, CpAttRegs &a) {
    const CpAttnSrc &A = p.att;
    const int t = threadIdx.x;
    const float *row = A.qkv + (size_t)b * A.ld;
#pragma unroll
    for (int i = 0; i < 4; ++i) a.raw[i] = ldg(reinterpret_cast<const float4 *>(row + i * 1024 + t * 4));
    cpatt_issue_par(A.qn, A.kn, A.rope, A.pos[b], a);
    const size_t slot = (size_t)b * CPA_NKV * CPA_POS * CPA_D;
    cpatt_issue_kv<false>(A.kc + slot, A.vc + slot, a);
}
__device__ __forceinline__ void cpatt_finish(const GemvParams &p, int b, bool valid, CpAttRegs &a, uint16_t *xrow,
                                             uint8_t *scratch) {
    const CpAttnSrc &A = p.att;
    const size_t slot = (size_t)b * CPA_NKV * CPA_POS * CPA_D;
    const bool w = blockIdx.x == 0;   // one workgroup appends the new K / V rows
    cpatt_compute<false>(a, A.eps, w ? A.kc + slot : nullptr, w ? A.vc + slot : nullptr, valid, xrow, scratch);
}

template <int RPG, int BT, int KS, int PRO, int NL>
__global__ void __launch_bounds__(256) k_gemv(const GemvParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int GPB = 16 / KS;   // row-groups per block
    constexpr int WPS = 4 / KS;    // waves per K slice
    constexpr bool kSelG = PRO == PRO_SEL_G1;
    constexpr bool kGather = PRO == PRO_RMS_G1 || PRO == PRO_RMS_G16 || kSelG;
    constexpr bool kRms = PRO == PRO_RMS || kGather;
    constexpr bool kAtt = PRO == PRO_CPATT;
    constexpr bool kF32 = PRO != PRO_F16 && !kAtt;
    constexpr int NT = PRO == PRO_RMS_G16 ? 16 : 1;
    constexpr int XB = BT <= 2 ? BT : 1;          // f32 activation rows held in registers at once
    constexpr bool kXh = PRO == PRO_F16 && NL > 0;   // f16 activation rows prefetched into registers (K <= 4096,
    constexpr int XHN = NL >= 24 ? 3 : 2;             // NL 24: K <= 6144)
    const int K = p.K, N = p.N;
    const int Kp = (K + 127) & ~127;
    uint16_t *xs = reinterpret_cast<uint16_t *>(smem);
    float *red = reinterpret_cast<float *>(smem + (size_t)BT * Kp * 2);
    double *dscr = reinterpret_cast<double *>(red + 16 * RPG * BT);
    uint8_t *att_lds = reinterpret_cast<uint8_t *>(dscr + 8);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, grp = lane >> 4;
    const int b0 = blockIdx.y * BT;
    const int nb = min(BT, p.B - b0);

    // ---------------- rows and K slice of this lane
    const int kslice = wave / WPS, g = (wave % WPS) * 4 + grp;
    const int Kq = ((Kp / 128 + KS - 1) / KS) * 128;
    const int kbeg = kslice * Kq, kend = min(Kp, kbeg + Kq);
    int rows[RPG];
    bool unit_ok = true;
    const int unit = blockIdx.x * GPB + g;
    if constexpr (RPG == 2) {
        // SwiGLU: gate/up interleaved in 16-row blocks: unit u -> gate row (u/16)*32 + u%16, up row +16
        unit_ok = unit < N / 2;
        const int u = min(unit, N / 2 - 1);
        rows[0] = (u >> 4) * 32 + (u & 15);
        rows[1] = rows[0] + 16;
    } else {
#pragma unroll
        for (int i = 0; i < RPG; ++i) rows[i] = blockIdx.x * GPB * RPG + g + i * GPB;
    }
    const uint16_t *wrow[RPG];
#pragma unroll
    for (int i = 0; i < RPG; ++i) wrow[i] = p.W + (size_t)min(rows[i], N - 1) * K;

    // ---------------- (1) activation rows of the first chunk, norm weights, epilogue operands
    float4 r[XB][4];
    float4 nwv[4], nbv[4];
    uint4 xh[kXh ? BT : 1][XHN];
    if constexpr (kF32 && !kGather) {
#pragma unroll
        for (int q = 0; q < XB; ++q) issue_x_plain(p, b0 + min(q, nb - 1), r[q]);
    }
    CpAttRegs ar;
    if constexpr (kAtt) cpatt_issue(p, b0, ar);
    // PRO_SEL_G1: the first slot's logits row, ahead of the weight stream (vmcnt retires in issue order)
    float selv[kSelG ? SEL_VPT_MAX : 1];
    if constexpr (kSelG) sel_load_exact<8>(p.sel_logits + (size_t)b0 * p.sel.V, selv);   // V = 2048 (gemv() checks)
    if constexpr (kXh) {
#pragma unroll
        for (int b = 0; b < BT; ++b) {
            const int src_row = b < nb ? (p.x_idx ? p.x_idx[b0 + b] : b0 + b) : 0;
            const uint16_t *src = reinterpret_cast<const uint16_t *>(p.x) + (size_t)src_row * p.ldx;
#pragma unroll
            for (int t = 0; t < XHN; ++t) {
                const int k = tid * 8 + t * 2048;
                xh[b][t] = ldg(reinterpret_cast<const uint4 *>(src + ((b < nb && k < K) ? k : 0)));
            }
        }
    }
    if constexpr (kRms || PRO == PRO_LN) {
        const int xt = (K + 1023) >> 10;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int k = t * 1024 + tid * 4;
            const int kk = (t < xt && k < K) ? k : 0;   // used only where k < K
            nwv[t] = ldg(reinterpret_cast<const float4 *>(p.nw + kk));
            if constexpr (PRO == PRO_LN) nbv[t] = ldg(reinterpret_cast<const float4 *>(p.nb + kk));
            else nbv[t] = f4_zero();
        }
    }
    // epilogue operands of the (row, batch column) this lane writes: lane l16 writes column l16
    float e_bias[RPG], e_scale[RPG], e_res[RPG], e_aux[RPG];
    {
        const int bb = b0 + min(l16, nb - 1);
#pragma unroll
        for (int i = 0; i < RPG; ++i) {
            // unconditional loads (null operands read a valid dummy word): the compiler can then wait exactly
            const int rr = min(rows[i], N - 1);
            const float *dummy = reinterpret_cast<const float *>(p.W);
            const float vb = ldg(p.bias ? p.bias + rr : dummy);
            const float vs = ldg(p.scale ? p.scale + rr : dummy);
            const float vr = ldg(p.resid ? p.resid + (size_t)bb * p.ldr + rr : dummy);
            const float va = ldg(p.aux ? p.aux + (size_t)bb * p.lda + rr : dummy);
            e_bias[i] = vb;   // used only under the same conditions in the epilogue
            e_scale[i] = vs;
            e_res[i] = vr;
            e_aux[i] = va;
        }
    }

    __builtin_amdgcn_sched_barrier(0);   // keep the issue order: (1) before (2), no math hoisted above the weights

    // ---------------- (2) every weight load of this lane, then the gathered rows
    uint4 wv[NL > 0 ? NL : 1][RPG];
    if constexpr (NL > 0) {
#pragma unroll
        for (int t = 0; t < NL; ++t) {
            const int k = kbeg + l16 * 8 + t * 128;
            const bool ok = k < kend && k < K;
            // unconditional (invalid slots re-read column 0, finite f16 weights): exact vmcnt for the prologue;
            // slots k >= kend are skipped by the dot loop, k in [K, Kp) cannot occur (K % 8 == 0 and lanes step 8)
#pragma unroll
            for (int i = 0; i < RPG; ++i) wv[t][i] = ld_w(wrow[i] + (ok ? k : 0));
        }
    }
    // PRO_SEL_G1: every workgroup selects the tokens of its slots while its weights stream (uniform per workgroup,
    // identical in every workgroup: same inputs, same code); workgroup x = 0 records them
    int *sel_tok = reinterpret_cast<int *>(att_lds + (kSelG ? sizeof(SelLds) : 0));
    if constexpr (kSelG) {
        __builtin_amdgcn_sched_barrier(0);
        SelLds &SL = *reinterpret_cast<SelLds *>(att_lds);
        for (int b = 0; b < nb; ++b) {
            const int s = b0 + b;
            if (b > 0) sel_load_exact<8>(p.sel_logits + (size_t)s * p.sel.V, selv);
            const int tok = select_token_regs<SEL_CP>(p.sel, selv, s, SL);
            if (tok >= 0 && blockIdx.x == 0 && tid == 0) select_commit(p.sel, s, tok);
            if (tid == 0) sel_tok[b] = tok;
            __syncthreads();
        }
    }
    if constexpr (kGather) {
#pragma unroll
        for (int q = 0; q < XB; ++q) issue_x_gather<NT>(p, b0 + min(q, nb - 1), r[q], kSelG ? sel_tok[min(q, nb - 1)] : -1);
    }

    __builtin_amdgcn_sched_barrier(0);

    // ---------------- (3) prologue: f16 activation tile in LDS
    if constexpr (kAtt) {
        for (int b = 0; b < BT; ++b) {
            if (b > 0) cpatt_issue(p, b0 + min(b, nb - 1), ar);
            cpatt_finish(p, b0 + min(b, nb - 1), b < nb, ar, xs + (size_t)b * Kp, att_lds);
        }
    } else if constexpr (!kF32) {
        if constexpr (kXh) {
#pragma unroll
            for (int b = 0; b < BT; ++b)
#pragma unroll
                for (int t = 0; t < XHN; ++t) {
                    const int k = tid * 8 + t * 2048;
                    if (k < Kp)
                        *reinterpret_cast<uint4 *>(xs + (size_t)b * Kp + k) = (b < nb && k < K) ? xh[b][t] : make_uint4(0, 0, 0, 0);
                }
        } else {
            // unrolled over the tile's rows: every row's loads are in flight before the first LDS store
#pragma unroll
            for (int b = 0; b < BT; ++b) {
                uint16_t *xr = xs + (size_t)b * Kp;
                const int src_row = b < nb ? (p.x_idx ? p.x_idx[b0 + b] : b0 + b) : 0;
                const uint16_t *src = reinterpret_cast<const uint16_t *>(p.x) + (size_t)src_row * p.ldx;
#pragma unroll 2
                for (int k = tid * 8; k < Kp; k += 2048)
                    *reinterpret_cast<uint4 *>(xr + k) =
                        (b < nb && k < K) ? ldg(reinterpret_cast<const uint4 *>(src + k)) : make_uint4(0, 0, 0, 0);
            }
        }
    } else {
        // rows bb + XB.. are loaded while rows bb.. reduce (one row's load latency per tile instead of one per row)
        float4 rn[BT > XB ? XB : 1][4];
        for (int bb = 0; bb < BT; bb += XB) {
            if (BT > XB && bb + XB < BT)
#pragma unroll
                for (int q = 0; q < XB; ++q) {
                    const int b = bb + XB + q;
                    if constexpr (kGather) issue_x_gather<NT>(p, b0 + min(b, nb - 1), rn[q], kSelG ? sel_tok[min(b, nb - 1)] : -1);
                    else issue_x_plain(p, b0 + min(b, nb - 1), rn[q]);
                }
#pragma unroll
            for (int q = 0; q < XB; ++q) mask_x(K, bb + q < nb, r[q]);
            float scale[XB], mean[XB];
#pragma unroll
            for (int q = 0; q < XB; ++q) { scale[q] = 1.0f; mean[q] = 0.0f; }
            if constexpr (kRms) {
                double ss[XB];
#pragma unroll
                for (int q = 0; q < XB; ++q) {
                    ss[q] = 0.0;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const float4 v = r[q][t];
                        ss[q] += (double)(v.x * v.x) + (double)(v.y * v.y) + (double)(v.z * v.z) + (double)(v.w * v.w);
                    }
                }
                block_sum_dn<XB>(ss, dscr);
#pragma unroll
                for (int q = 0; q < XB; ++q) scale[q] = 1.0f / sqrtf((float)(ss[q] / K) + p.eps);
            } else if constexpr (PRO == PRO_LN) {
                double s1[XB];
#pragma unroll
                for (int q = 0; q < XB; ++q) {
                    s1[q] = 0.0;
#pragma unroll
                    for (int t = 0; t < 4; ++t) s1[q] += (double)r[q][t].x + (double)r[q][t].y + (double)r[q][t].z + (double)r[q][t].w;
                }
                block_sum_dn<XB>(s1, dscr);
                double s2[XB];
#pragma unroll
                for (int q = 0; q < XB; ++q) {
                    mean[q] = (float)(s1[q] / K);
                    s2[q] = 0.0;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int k = t * 1024 + tid * 4;
                        if (k < K) {
                            const float4 v = r[q][t];
                            const float dx = v.x - mean[q], dy = v.y - mean[q], dz = v.z - mean[q], dw = v.w - mean[q];
                            s2[q] += (double)(dx * dx) + (double)(dy * dy) + (double)(dz * dz) + (double)(dw * dw);
                        }
                    }
                }
                block_sum_dn<XB>(s2, dscr);
#pragma unroll
                for (int q = 0; q < XB; ++q) scale[q] = 1.0f / sqrtf((float)(s2[q] / K) + p.eps);
            }
#pragma unroll
            for (int q = 0; q < XB; ++q) {
                const int b = bb + q;
                uint16_t *xr = xs + (size_t)b * Kp;
                const bool side = b < nb && blockIdx.x == 0;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int k = t * 1024 + tid * 4;
                    if (k >= Kp) continue;
                    const float4 v = r[q][t];
                    float y[4] = {v.x, v.y, v.z, v.w};
                    if (k < K) {
                        if (side && p.raw_out) *reinterpret_cast<float4 *>(p.raw_out + (size_t)(b0 + b) * K + k) = v;
                        if constexpr (kRms || PRO == PRO_LN) {
                            const float w4[4] = {nwv[t].x, nwv[t].y, nwv[t].z, nwv[t].w};
                            const float c4[4] = {nbv[t].x, nbv[t].y, nbv[t].z, nbv[t].w};
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                if constexpr (kRms) y[e] = (y[e] * scale[q]) * w4[e];
                                else y[e] = ((y[e] - mean[q]) * scale[q]) * w4[e] + c4[e];
                            }
                        }
                        if (side && p.side_out)
                            *reinterpret_cast<float4 *>(p.side_out + (size_t)(b0 + b) * K + k) = make_float4(y[0], y[1], y[2], y[3]);
                    } else {
                        y[0] = y[1] = y[2] = y[3] = 0.0f;
                    }
                    uint2 h;
                    h.x = (uint32_t)f2h(y[0]) | ((uint32_t)f2h(y[1]) << 16);
                    h.y = (uint32_t)f2h(y[2]) | ((uint32_t)f2h(y[3]) << 16);
                    *reinterpret_cast<uint2 *>(xr + k) = h;
                }
            }
            if constexpr (BT > XB) {
#pragma unroll
                for (int q = 0; q < XB; ++q)
#pragma unroll
                    for (int t = 0; t < 4; ++t) r[q][t] = rn[q][t];
            }
        }
    }
    __syncthreads();

    // ---------------- (4) dot products
    float acc[RPG][BT];
#pragma unroll
    for (int i = 0; i < RPG; ++i)
#pragma unroll
        for (int b = 0; b < BT; ++b) acc[i][b] = 0.0f;
    if constexpr (NL > 0) {
#pragma unroll
        for (int t = 0; t < NL; ++t) {
            const int k = kbeg + l16 * 8 + t * 128;
            if (k < kend && k < K) {
#pragma unroll
                for (int b = 0; b < BT; ++b) {
                    const uint4 xv = *reinterpret_cast<const uint4 *>(xs + (size_t)b * Kp + k);
#pragma unroll
                    for (int i = 0; i < RPG; ++i) acc[i][b] = dot8(wv[t][i], xv, acc[i][b]);
                }
            }
        }
    } else {
#pragma unroll 2
        for (int k = kbeg + l16 * 8; k < kend; k += 128) {
            uint4 w[RPG];
#pragma unroll
            for (int i = 0; i < RPG; ++i) w[i] = k < K ? ld_w(wrow[i] + k) : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int b = 0; b < BT; ++b) {
                const uint4 xv = *reinterpret_cast<const uint4 *>(xs + (size_t)b * Kp + k);
#pragma unroll
                for (int i = 0; i < RPG; ++i) acc[i][b] = dot8(w[i], xv, acc[i][b]);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < RPG; ++i)
#pragma unroll
        for (int b = 0; b < BT; ++b) acc[i][b] = group_sum<16>(acc[i][b]);
    if constexpr (KS > 1) {
        if (l16 == 0)
#pragma unroll
            for (int i = 0; i < RPG; ++i)
#pragma unroll
                for (int b = 0; b < BT; ++b) red[((kslice * GPB + g) * RPG + i) * BT + b] = acc[i][b];
        __syncthreads();
        if (kslice == 0)
#pragma unroll
            for (int i = 0; i < RPG; ++i)
#pragma unroll
                for (int b = 0; b < BT; ++b) {
                    float s = 0.0f;
#pragma unroll
                    for (int q = 0; q < KS; ++q) s += red[((q * GPB + g) * RPG + i) * BT + b];
                    acc[i][b] = s;
                }
    }
    constexpr bool kSel = RPG == 1 && PRO == PRO_RMS;   // head GEMVs may select the token in the same launch
    const bool sel = kSel && p.sel.mode != SEL_NONE;

    // ---------------- (5) epilogue: lane l16 of each group writes batch column l16
    if (kslice == 0) {
#pragma unroll
        for (int bi = 0; bi < BT; ++bi) {
            if (bi != l16 || bi >= nb) continue;
            const int bb = b0 + bi;
            const size_t orow = (size_t)bb * p.orow_mul + p.orow_add;
            if (p.act == ACT_SWIGLU) {
                if constexpr (RPG == 2) {
                    if (unit_ok) {
                        const float h = silu_f(acc[0][bi]) * acc[1][bi];
                        if (p.out_f16) p.out_f16[orow * p.ldo + unit] = f2h(h);
                        else p.out_f32[orow * p.ldo + unit] = h;
                    }
                }
                continue;
            }
#pragma unroll
            for (int i = 0; i < RPG; ++i) {
                const int rr = rows[i];
                if (rr >= N) continue;
                float v = acc[i][bi];
                if (p.bias) v += e_bias[i];
                if (p.act == ACT_SILU) v = silu_f(v);
                else if (p.act == ACT_GELU) v = gelu_ggml(v);
                if (p.scale) v *= e_scale[i];
                if (p.resid) v = e_res[i] + v;
                if (p.aux) v = e_aux[i] + v;
                if (p.out_f16) p.out_f16[orow * p.ldo + rr] = f2h(v);
                else if (sel) __hip_atomic_store(p.out_f32 + orow * p.ldo + rr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else p.out_f32[orow * p.ldo + rr] = v;
            }
        }
    }

    // ---------------- (6) fused token selection: sc1 logits stores -> vmcnt(0) -> barrier -> one agent-scope ticket
    // add per workgroup; the last adder loads the logits with sc1 loads and selects (MI355X_MICROARCH.md, hand-off
    // table row 1).
    if constexpr (kSel) {
        if (sel) {
            SelLds &S = *reinterpret_cast<SelLds *>(att_lds);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0)
                S.last = __hip_atomic_fetch_add(p.sel.ticket + blockIdx.y, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                         gridDim.x - 1;
            __syncthreads();
            if (S.last) {
                for (int b = 0; b < nb; ++b) {
                    select_slot<true>(p.sel, p.out_f32 + (size_t)(b0 + b) * p.ldo, b0 + b, S);
                    __syncthreads();
                }
                if (tid == 0) __hip_atomic_store(p.sel.ticket + blockIdx.y, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------ host dispatch
template <int RPG, int BT, int KS, int PRO, int NL>
void launch_one(const GemvParams &p, dim3 grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((k_gemv<RPG, BT, KS, PRO, NL>), grid, dim3(256), lds, s, p);
}
template <int RPG, int BT, int KS, int PRO>
void launch_nl(const GemvParams &p, int nl, dim3 grid, size_t lds, hipStream_t s) {
    if constexpr (BT <= 2) {
        if (nl == 2) return launch_one<RPG, BT, KS, PRO, 2>(p, grid, lds, s);
        if (nl == 4) return launch_one<RPG, BT, KS, PRO, 4>(p, grid, lds, s);
        if (nl == 8) return launch_one<RPG, BT, KS, PRO, 8>(p, grid, lds, s);
    }
    // single-row K <= 2048 per lane slice (the 1.7B talker's 2,048-wide QKV / gate-up / O rows): every weight load up front
    if constexpr (BT == 1 && (PRO == PRO_RMS || PRO == PRO_F16 || PRO == PRO_F32))
        if (nl == 16) return launch_one<RPG, BT, KS, PRO, 16>(p, grid, lds, s);
    if constexpr (BT == 1 && PRO == PRO_F16)   // (the 1.7B down projection: K 6,144 in two slices of 3,072)
        if (nl == 24) return launch_one<RPG, BT, KS, PRO, 24>(p, grid, lds, s);
    launch_one<RPG, BT, KS, PRO, 0>(p, grid, lds, s);
}
template <int RPG, int BT, int KS>
void launch_pro(const GemvParams &p, int nl, dim3 grid, size_t lds, hipStream_t s) {
    if constexpr (RPG == 2) {
        launch_nl<2, BT, KS, PRO_RMS>(p, nl, grid, lds, s);
    } else {
        switch (p.pro) {
            case PRO_F16: launch_nl<1, BT, KS, PRO_F16>(p, nl, grid, lds, s); break;
            case PRO_F32: launch_nl<1, BT, KS, PRO_F32>(p, nl, grid, lds, s); break;
            case PRO_RMS: launch_nl<1, BT, KS, PRO_RMS>(p, nl, grid, lds, s); break;
            case PRO_RMS_G1: launch_nl<1, BT, KS, PRO_RMS_G1>(p, nl, grid, lds, s); break;
            case PRO_RMS_G16: launch_nl<1, BT, KS, PRO_RMS_G16>(p, nl, grid, lds, s); break;
            case PRO_SEL_G1: launch_nl<1, BT, KS, PRO_SEL_G1>(p, nl, grid, lds, s); break;
            case PRO_CPATT: launch_nl<1, BT, KS, PRO_CPATT>(p, nl, grid, lds, s); break;
            default: launch_nl<1, BT, KS, PRO_LN>(p, nl, grid, lds, s); break;
        }
    }
}

}  // namespace q3t
