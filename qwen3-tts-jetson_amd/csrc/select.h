// select.h — token selection of the decode path on one 256-thread workgroup (device code, included by the kernel
// translation units).  Thread t owns the contiguous indices [t*vpt, t*vpt + vpt), vpt = ceil(V / 256) <= 16, in
// registers.
//
//   argmax         first maximum (strict '>' scan, src/tts_transformer.cpp:2051-2061)
//   top-k sampling /T -> top-k with `< thr -> -inf` so ties survive (:2456-2464), the kept id restored (EOS,
//                  :2466-2470), exp(v - max), inverse CDF with u * total (:2474-2495; CP: trt_cuda_kernels.cu:120-183).
//                  Default: sel_topk_fast -- three workgroup barriers (row max / min, a 256-bin range histogram, the
//                  <= 128 entries at or above the boundary bin gathered in index order); the boundary-bin entries are
//                  ranked among themselves, so the survivors are exactly {v >= k-th largest} (+ the kept id).  Its CDF
//                  total adds the survivors' exponentials two per lane and scans across one wave, in index order: the
//                  same set and order as the reference's sequential loop, but not the same f32 rounding of the running
//                  sum as the general path (per-thread sums in index order, then the waves), so a row whose u * total
//                  falls within an ulp-level distance of a CDF boundary can pick a neighbouring token on the two paths
//                  (checked against the reference semantics within 1e-4 of the CDF: tests/test_gpu_select.py,
//                  test_gpu_parity.py::test_cb0_select_kept_eos).  Degenerate rows (no finite range, fewer than k finite
//                  values, more than 128 entries at or above the boundary bin) take the general path: k-th largest by a
//                  range histogram + candidate ranking, or a 3-pass radix select on order-preserving keys (11/11/10-bit
//                  digits), then the thread-order inverse-CDF scan.
//   CB0 processing control-range mask, repetition penalty over the seen set, EOS ramp, bench EOS mask
//                  (src/tts_transformer.cpp:2416-2445)
#pragma once
#include "kernels.h"

namespace q3t {

constexpr int SEL_VPT_MAX = 16;   // V <= 4096

#ifndef SEL_STAMP
#define SEL_STAMP(k) ((void)0)   // development hook (tools/dev/selbench.hip): stage timestamps of one selection
#endif

constexpr int SEL_CAND = 256;     // boundary-bin candidate list of the top-k threshold search

struct alignas(16) SelLds {
    unsigned hist[4096];
    uint32_t cand[SEL_CAND];
    unsigned ncand;
    float fred[4];
    int ired[4];
    unsigned ures[4];
    unsigned sres[2];
    float wsum[4];
    float rmax[4], rmin[4];   // sel_kth_largest_range's wave max / min (apart from fred: CB0's block max reads fred
                              // right before it, so its first barrier is not needed)
    unsigned fcnt[4];         // sel_topk_fast: entries per wave (the entries overlay hist[1024..2047])
    unsigned last;
};

__device__ __forceinline__ uint32_t sel_fkey(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float sel_keyf(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
__device__ __forceinline__ float sel_block_max(float v, SelLds &S) {
    v = wave_max(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) S.fred[wave] = v;
    __syncthreads();
    return fmaxf(fmaxf(S.fred[0], S.fred[1]), fmaxf(S.fred[2], S.fred[3]));
}

// (value, index) max with lowest-index tie break over the whole wave (DPP in rows, permlane swaps across rows)
template <int CTRL>
__device__ __forceinline__ void sel_pair_step(float &bv, int &bi) {
    const float ov = dpp_f<CTRL>(bv);
    const int oi = (int)dpp_u<CTRL>((unsigned)bi);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
}
__device__ __forceinline__ void sel_pair_reduce(float &bv, int &bi) {
    sel_pair_step<DPP_XOR1>(bv, bi);
    sel_pair_step<DPP_XOR2>(bv, bi);
    sel_pair_step<DPP_HALF_MIRROR>(bv, bi);
    sel_pair_step<DPP_MIRROR>(bv, bi);
    float ov = xrow16(bv);
    int oi = (int)xrow16_u((unsigned)bi);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    ov = xrow32(bv);
    oi = (int)xrow32_u((unsigned)bi);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
}

// first index of the maximum
__device__ __forceinline__ int sel_argmax(const float (&v)[SEL_VPT_MAX], int n, int vpt, SelLds &S) {
    const int t = threadIdx.x;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) {
        const int i = t * vpt + e;
        if (e < vpt && i < n && (v[e] > bv || bi == 0x7fffffff)) { bv = v[e]; bi = i; }
    }
    // NaN-free inputs: strict '>' keeps the first index of a tie inside the thread; across threads the lower index wins
    sel_pair_reduce(bv, bi);
    const int lane = t & 63, wave = t >> 6;
    __syncthreads();
    if (lane == 0) { S.fred[wave] = bv; S.ired[wave] = bi; }
    __syncthreads();
    bv = S.fred[0];
    bi = S.ired[0];
#pragma unroll
    for (int w = 1; w < 4; ++w)
        if (S.fred[w] > bv || (S.fred[w] == bv && S.ired[w] < bi)) { bv = S.fred[w]; bi = S.ired[w]; }
    return bi == 0x7fffffff ? 0 : bi;
}

// block inclusive scan over 256 threads (in thread order) of a per-thread count; returns the exclusive prefix,
// *total = the block total
__device__ __forceinline__ unsigned sel_scan_u(unsigned loc, unsigned *total, SelLds &S) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned incl = wave_scan_incl_u(loc);
    __syncthreads();
    if (lane == 63) S.ures[wave] = incl;
    __syncthreads();
    unsigned pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) { if (w < wave) pre += S.ures[w]; tot += S.ures[w]; }
    *total = tot;
    return pre + incl - loc;
}

// one MSB radix pass over the keys matching (prefix, pmask): finds the digit (bits [shift, shift+bits)) that holds the
// kk-th largest key; returns the number of matching keys with a larger digit through *above
__device__ __forceinline__ uint32_t sel_radix_pass(const uint32_t (&keys)[SEL_VPT_MAX], int n, int vpt, uint32_t prefix,
                                                   uint32_t pmask, int shift, int bits, int kk, unsigned *above, SelLds &S) {
    const int t = threadIdx.x, nb = 1 << bits, bpt = nb / 256;
    const uint32_t dmask = (uint32_t)nb - 1u;
    for (int i = t * 4; i < nb; i += 1024) *reinterpret_cast<uint4 *>(&S.hist[i]) = make_uint4(0, 0, 0, 0);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e)
        if (e < vpt && t * vpt + e < n && (keys[e] & pmask) == prefix) atomicAdd(&S.hist[(keys[e] >> shift) & dmask], 1u);
    __syncthreads();
    // thread t owns digits nb-1-t*bpt .. nb-bpt-t*bpt (descending; contiguous 16-B reads)
    unsigned c[16], loc = 0;
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
        uint4 h4 = make_uint4(0, 0, 0, 0);
        if (q4 * 4 < bpt) h4 = *reinterpret_cast<const uint4 *>(&S.hist[nb - t * bpt - 4 - q4 * 4]);
        c[q4 * 4 + 0] = h4.w; c[q4 * 4 + 1] = h4.z; c[q4 * 4 + 2] = h4.y; c[q4 * 4 + 3] = h4.x;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) { if (q >= bpt) c[q] = 0; loc += c[q]; }
    unsigned tot;
    unsigned cum = sel_scan_u(loc, &tot, S);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        if (q < bpt && cum < (unsigned)kk && (unsigned)kk <= cum + c[q]) {
            S.sres[0] = (unsigned)(nb - 1 - t * bpt - q);
            S.sres[1] = cum;
        }
        cum += c[q];
    }
    if (t == 0) S.ncand = 0;
    __syncthreads();
    *above = S.sres[1];
    return S.sres[0];
}

// k-th largest value (1-based k) of v[0..n): one 12-bit MSB histogram pass (4096 bins: sign, exponent, 3 mantissa
// bits), then an exact rank among the few keys of the boundary bin (LDS candidate list); a boundary bin with more
// than SEL_CAND keys (degenerate inputs) falls back to two more 10-bit radix passes.
__device__ __forceinline__ float sel_kth_largest(const float (&v)[SEL_VPT_MAX], int n, int vpt, int k, SelLds &S) {
    const int t = threadIdx.x;
    uint32_t keys[SEL_VPT_MAX];
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) keys[e] = (e < vpt && t * vpt + e < n) ? sel_fkey(v[e]) : 0u;
    unsigned above;
    const uint32_t d0 = sel_radix_pass(keys, n, vpt, 0u, 0u, 20, 12, k, &above, S);
    uint32_t prefix = d0 << 20, pmask = 0xFFFu << 20;
    int kk = k - (int)above;
    // candidates of the boundary bin
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e)
        if (e < vpt && t * vpt + e < n && (keys[e] & pmask) == prefix) {
            const unsigned i = atomicAdd(&S.ncand, 1u);
            if (i < SEL_CAND) S.cand[i] = keys[e];
        }
    __syncthreads();
    const unsigned nc = S.ncand;
    if (nc <= 64) {
        // one wave ranks the candidates with readlane broadcasts (no LDS round trips in the loop)
        if (t < 64) {
            const uint32_t me = t < (int)nc ? S.cand[t] : 0u;
            unsigned gt = 0, eq = 0;
            for (unsigned j = 0; j < nc; ++j) {
                const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)me, (int)j);
                gt += o > me;
                eq += o == me;
            }
            if (t < (int)nc && gt < (unsigned)kk && (unsigned)kk <= gt + eq) S.sres[0] = me;   // same key for all writers
        }
        __syncthreads();
        const uint32_t r = S.sres[0];
        __syncthreads();
        return sel_keyf(r);
    }
    if (nc <= SEL_CAND) {
        if (t < (int)nc) {
            const uint32_t me = S.cand[t];
            unsigned gt = 0, eq = 0;
#pragma unroll 8
            for (unsigned j = 0; j < nc; ++j) { const uint32_t o = S.cand[j]; gt += o > me; eq += o == me; }
            if (gt < (unsigned)kk && (unsigned)kk <= gt + eq) S.sres[0] = me;
        }
        __syncthreads();
        const uint32_t r = S.sres[0];
        __syncthreads();
        return sel_keyf(r);
    }
    const uint32_t d1 = sel_radix_pass(keys, n, vpt, prefix, pmask, 10, 10, kk, &above, S);
    prefix |= d1 << 10;
    pmask |= 0x3FFu << 10;
    kk -= (int)above;
    const uint32_t d2 = sel_radix_pass(keys, n, vpt, prefix, pmask, 0, 10, kk, &above, S);
    return sel_keyf(prefix | d2);
}

// k-th largest value (1-based k < n) through ONE 256-bin histogram of the value range [min, max] of the finite
// values (bin = floor((v - min) * 256 / (max - min)), monotonic in v, so the boundary bin holds the k-th largest),
// scanned by a single wave; then the exact rank among the boundary bin's keys (LDS candidate list, as above).
// Degenerate rows (max == min, non-finite range, > SEL_CAND keys in the boundary bin) take sel_kth_largest.
// *vmax = the row maximum (exact, so the caller's softmax needs no second block reduction).
__device__ __forceinline__ float sel_kth_largest_range(const float (&v)[SEL_VPT_MAX], int n, int vpt, int k, float *vmax, SelLds &S) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    float mx = -INFINITY, mn = INFINITY;
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e)
        if (e < vpt && t * vpt + e < n) {
            mx = fmaxf(mx, v[e]);
            if (v[e] > -INFINITY) mn = fminf(mn, v[e]);
        }
    // (no barrier ahead of these writes: rmax / rmin / hist are read only inside this call, and every caller runs a
    // workgroup barrier between two selections)
    S.hist[t] = 0u;   // 256 bins, one per thread
    mx = wave_max(mx);
    mn = -wave_max(-mn);
    if (lane == 0) { S.rmax[wave] = mx; S.rmin[wave] = mn; }
    __syncthreads();
    mx = fmaxf(fmaxf(S.rmax[0], S.rmax[1]), fmaxf(S.rmax[2], S.rmax[3]));
    mn = fminf(fminf(S.rmin[0], S.rmin[1]), fminf(S.rmin[2], S.rmin[3]));
    SEL_STAMP(1);
    *vmax = mx;
    const float range = mx - mn;
    if (!(range > 0.0f) || !(range < INFINITY)) return sel_kth_largest(v, n, vpt, k, S);   // uniform
    const float scale = 256.0f / range;
    int dig[SEL_VPT_MAX];
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) {
        dig[e] = -1;
        if (e < vpt && t * vpt + e < n && v[e] > -INFINITY) {
            dig[e] = min(255, (int)((v[e] - mn) * scale));
            atomicAdd(&S.hist[dig[e]], 1u);
        }
    }
    __syncthreads();
    SEL_STAMP(2);
    if (wave == 0) {
        // lane l owns bins 255-4l .. 252-4l (descending), so the inclusive lane scan counts keys from the top
        const uint4 h4 = *reinterpret_cast<const uint4 *>(&S.hist[252 - 4 * lane]);
        const unsigned c[4] = {h4.w, h4.z, h4.y, h4.x};
        const unsigned loc = c[0] + c[1] + c[2] + c[3];
        const unsigned incl = wave_scan_incl_u(loc);
        const unsigned total = (unsigned)__builtin_amdgcn_readlane((int)incl, 63);
        unsigned cum = incl - loc;
        if (lane == 0) { S.ncand = 0; S.sres[0] = 0xFFFFFFFFu; }
        if (total >= (unsigned)k) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (cum < (unsigned)k && (unsigned)k <= cum + c[q]) { S.sres[0] = 255 - 4 * lane - q; S.sres[1] = cum; }
                cum += c[q];
            }
        }
    }
    __syncthreads();
    SEL_STAMP(3);
    const unsigned bstar = S.sres[0];
    if (bstar == 0xFFFFFFFFu) return -INFINITY;   // fewer than k finite values: the k-th largest is -inf
    const int kk = k - (int)S.sres[1];
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e)
        if (dig[e] == (int)bstar) {
            const unsigned i = atomicAdd(&S.ncand, 1u);
            if (i < SEL_CAND) S.cand[i] = sel_fkey(v[e]);
        }
    __syncthreads();
    SEL_STAMP(4);
    const unsigned nc = S.ncand;
    if (nc > SEL_CAND) return sel_kth_largest(v, n, vpt, k, S);   // uniform
    if (nc <= 64) {
        if (t < 64) {
            const uint32_t me = t < (int)nc ? S.cand[t] : 0u;
            unsigned gt = 0, eq = 0;
            for (unsigned j = 0; j < nc; ++j) {
                const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)me, (int)j);
                gt += o > me;
                eq += o == me;
            }
            if (t < (int)nc && gt < (unsigned)kk && (unsigned)kk <= gt + eq) S.sres[0] = me;
        }
    } else if (t < (int)nc) {
        const uint32_t me = S.cand[t];
        unsigned gt = 0, eq = 0;
#pragma unroll 8
        for (unsigned j = 0; j < nc; ++j) { const uint32_t o = S.cand[j]; gt += o > me; eq += o == me; }
        if (gt < (unsigned)kk && (unsigned)kk <= gt + eq) S.sres[0] = me;
    }
    __syncthreads();
    SEL_STAMP(5);
    return sel_keyf(S.sres[0]);   // (sres is written again only by the next selection, behind the caller's barrier)
}

// Top-k sampling in three workgroup barriers (v already divided by T; returns the token, or -2 when the row needs the
// general path below: a degenerate value range, fewer than k finite values, or more than SEL_FAST_CAP entries at or above
// the boundary bin; the condition is uniform over the workgroup).
//   B1  row max / min of the finite values (the range histogram's bounds, and the softmax max)
//   B2  256-bin range histogram (sel_kth_largest_range's bins); every wave then scans it itself: boundary bin b*, count
//       above it
//   B3  each wave writes its entries with bin >= b* (and the kept id) in index order into its own LDS region
// then EVERY wave, redundantly (so no barrier hands the token over): loads the <= 128 entries two per lane in index order,
// ranks the boundary-bin entries among themselves (an entry survives iff fewer than k - above of them are larger: the
// same set as `v >= k-th largest`), exp(v - max), a wave scan of the survivors' exps in index order (two per lane), total
// = the last lane's sum, and the first index whose cumulative sum reaches u * total.
// RANGE: the caller passes the row max and finite min (mx, mn; computed by the logits' producers) and has zeroed
// S.hist[0..255] behind a workgroup barrier that follows the previous selection: B1 is skipped.
constexpr int SEL_FAST_CAP = 128;
template <bool RANGE = false>
__device__ __forceinline__ int sel_topk_fast(const float (&v)[SEL_VPT_MAX], int n, int vpt, int k, float u, int keep_id, SelLds &S,
                                             float mx = -INFINITY, float mn = INFINITY) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if constexpr (!RANGE) {
#pragma unroll
        for (int e = 0; e < SEL_VPT_MAX; ++e)
            if (e < vpt && t * vpt + e < n) {
                mx = fmaxf(mx, v[e]);
                if (v[e] > -INFINITY) mn = fminf(mn, v[e]);
            }
        S.hist[t] = 0u;
        mx = wave_max(mx);
        mn = -wave_max(-mn);
        if (lane == 0) { S.rmax[wave] = mx; S.rmin[wave] = mn; }
        __syncthreads();   // B1
        SEL_STAMP(10);
        mx = fmaxf(fmaxf(S.rmax[0], S.rmax[1]), fmaxf(S.rmax[2], S.rmax[3]));
        mn = fminf(fminf(S.rmin[0], S.rmin[1]), fminf(S.rmin[2], S.rmin[3]));
    }
    const float range = mx - mn;
    if (!(range > 0.0f) || !(range < INFINITY)) return -2;
    const float scale = 256.0f / range;
    int dig[SEL_VPT_MAX];
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) {
        dig[e] = -1;
        if (e < vpt && t * vpt + e < n && v[e] > -INFINITY) {
            dig[e] = min(255, (int)((v[e] - mn) * scale));
            atomicAdd(&S.hist[dig[e]], 1u);
        }
    }
    __syncthreads();   // B2
    SEL_STAMP(11);
    unsigned bstar, above;
    {   // lane l owns bins 255-4l .. 252-4l (descending): the inclusive lane scan counts keys from the top
        const uint4 h4 = *reinterpret_cast<const uint4 *>(&S.hist[252 - 4 * lane]);
        const unsigned c[4] = {h4.w, h4.z, h4.y, h4.x};
        const unsigned loc = c[0] + c[1] + c[2] + c[3];
        const unsigned incl = wave_scan_incl_u(loc);
        if ((unsigned)__builtin_amdgcn_readlane((int)incl, 63) < (unsigned)k) return -2;   // < k finite values
        unsigned cum = incl - loc, mb = 0, ma = 0;
        bool hit = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (cum < (unsigned)k && (unsigned)k <= cum + c[q]) { hit = true; mb = 255 - 4 * lane - q; ma = cum; }
            cum += c[q];
        }
        const int src = __builtin_ctzll(__ballot(hit));
        bstar = (unsigned)__builtin_amdgcn_readlane((int)mb, src);
        above = (unsigned)__builtin_amdgcn_readlane((int)ma, src);
    }
    SEL_STAMP(12);
    // entries: bin >= b*, or the kept id (its value competes for the threshold like any other and survives anyway)
    uint2 *ent = reinterpret_cast<uint2 *>(&S.hist[1024]) + SEL_FAST_CAP * wave;
    unsigned cnt = 0;
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) {
        const int i = t * vpt + e;
        if (e < vpt && i < n && (dig[e] >= (int)bstar || i == keep_id)) ++cnt;
    }
    const unsigned cincl = wave_scan_incl_u(cnt);
    const unsigned wtot = (unsigned)__builtin_amdgcn_readlane((int)cincl, 63);
    if (wtot <= (unsigned)SEL_FAST_CAP) {
        unsigned pos = cincl - cnt;
#pragma unroll
        for (int e = 0; e < SEL_VPT_MAX; ++e) {
            const int i = t * vpt + e;
            if (e < vpt && i < n && (dig[e] >= (int)bstar || i == keep_id))
                ent[pos++] = make_uint2(__float_as_uint(v[e]), (uint32_t)i | (dig[e] == (int)bstar ? 0x80000000u : 0u));
        }
    }
    if (lane == 0) S.fcnt[wave] = wtot;
    __syncthreads();   // B3
    SEL_STAMP(13);
    const unsigned c0 = S.fcnt[0], c1 = S.fcnt[1], c2 = S.fcnt[2], c3 = S.fcnt[3];
    const unsigned ns = c0 + c1 + c2 + c3;
    if (ns > (unsigned)SEL_FAST_CAP) return -2;   // (also covers one wave over its region: ns >= that wave's count)
    float ev[2];
    uint32_t ei[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const unsigned j = 2 * lane + s;
        ev[s] = -INFINITY;
        ei[s] = 0x7fffffffu;
        if (j < ns) {
            const unsigned r = j < c0 ? 0u : j < c0 + c1 ? 1u : j < c0 + c1 + c2 ? 2u : 3u;
            const unsigned off = j - (r >= 1 ? c0 : 0u) - (r >= 2 ? c1 : 0u) - (r >= 3 ? c2 : 0u);
            const uint2 q = reinterpret_cast<const uint2 *>(&S.hist[1024])[SEL_FAST_CAP * r + off];
            ev[s] = __uint_as_float(q.x);
            ei[s] = q.y;
        }
    }
    SEL_STAMP(14);
    // boundary-bin entries: rank among themselves
    const unsigned kk = (unsigned)k - above;
    unsigned gt[2] = {0u, 0u};
#pragma unroll
    for (int so = 0; so < 2; ++so) {
        uint64_t m = __ballot((ei[so] & 0x80000000u) && ei[so] != 0x7fffffffu);
        while (m) {
            const int j = __builtin_ctzll(m);
            m &= m - 1;
            const float o = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ev[so]), j));
            gt[0] += o > ev[0];
            gt[1] += o > ev[1];
        }
    }
    SEL_STAMP(15);
    float p[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const bool valid = ei[s] != 0x7fffffffu;
        const bool cand = valid && (ei[s] & 0x80000000u);
        const bool keep = valid && (int)(ei[s] & 0x7fffffffu) == keep_id;
        const bool surv = valid && (keep || !cand || gt[s] < kk);
        p[s] = surv ? expf(ev[s] - mx) : 0.0f;
    }
    const float loc = p[0] + p[1];
    const float incl = wave_scan_incl_f(loc);
    const float total = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, incl), 63));
    const float target = u * total;
    const float cum0 = (incl - loc) + p[0], cum1 = cum0 + p[1];
    const bool f0 = cum0 >= target && p[0] > 0.0f, f1 = cum1 >= target && p[1] > 0.0f;
    const uint64_t fm = __ballot(f0 || f1);
    SEL_STAMP(16);
    if (fm == 0) return n - 1;
    const int src = __builtin_ctzll(fm);
    const uint32_t pick = f0 ? ei[0] : ei[1];
    return (int)((uint32_t)__builtin_amdgcn_readlane((int)pick, src) & 0x7fffffffu);
}

// temperature -> top-k -> keep_id restored -> exp -> inverse CDF with u (v is modified)
__device__ __forceinline__ int sel_sample(float (&v)[SEL_VPT_MAX], int n, int vpt, float temperature, int top_k, float u, int keep_id,
                          SelLds &S) {
    const int t = threadIdx.x;
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e)
        if (e < vpt) v[e] = v[e] / temperature;
    // the kept logit (after /T) is restored after top-k by its owner thread
    const int keep_owner = keep_id >= 0 ? keep_id / vpt : -1;
    float keep_v = 0.0f;
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e)
        if (t == keep_owner && t * vpt + e == keep_id) keep_v = v[e];
    float m = -INFINITY;
    const bool topk = top_k > 0 && top_k < n;
#ifndef Q3T_SEL_GENERAL
    if (topk) {
        const int r = sel_topk_fast(v, n, vpt, top_k, u, keep_id, S);
        if (r != -2) return r;
        __syncthreads();   // (uniform) the waves may still read this selection's histogram
    }
#endif
    if (topk) {
        // the row max survives the threshold and bounds the restored kept logit: it is the softmax max as well
        const float thr = sel_kth_largest_range(v, n, vpt, top_k, &m, S);
#pragma unroll
        for (int e = 0; e < SEL_VPT_MAX; ++e)
            if (v[e] < thr) v[e] = -INFINITY;
    }
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e)
        if (t == keep_owner && t * vpt + e == keep_id) v[e] = keep_v;
    if (!topk) {
#pragma unroll
        for (int e = 0; e < SEL_VPT_MAX; ++e)
            if (e < vpt && t * vpt + e < n) m = fmaxf(m, v[e]);
        m = sel_block_max(m, S);
    }
    float loc = 0.0f;
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) {
        const bool in = e < vpt && t * vpt + e < n;
        v[e] = in ? expf(v[e] - m) : 0.0f;
        loc += v[e];
    }
    SEL_STAMP(6);
    // block exclusive scan of the per-thread sums (index order)
    const int lane = t & 63, wave = t >> 6;
    const float incl = wave_scan_incl_f(loc);
    // (wsum / ures[0] are last read behind a barrier of this selection's threshold search, or of the previous selection)
    if (lane == 63) S.wsum[wave] = incl;
    if (t == 0) S.ures[0] = 0x7fffffffu;
    __syncthreads();
    SEL_STAMP(7);
    float wpre = 0.0f, total = 0.0f;
#pragma unroll
    for (int w = 0; w < 4; ++w) { if (w < wave) wpre += S.wsum[w]; total += S.wsum[w]; }
    const float target = u * total;
    float cum = wpre + incl - loc;
    int found = 0x7fffffff;
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) {
        if (found != 0x7fffffff || e >= vpt) continue;
        cum += v[e];
        if (cum >= target && v[e] > 0.0f) found = t * vpt + e;
    }
    if (found != 0x7fffffff) atomicMin(reinterpret_cast<int *>(&S.ures[0]), found);
    __syncthreads();
    SEL_STAMP(8);
    const int r = (int)S.ures[0];
    return r == 0x7fffffff ? n - 1 : r;
}

// top-k sampling of a row already divided by T whose max / finite min the producers computed (the code-predictor role
// kernel's heads): sel_topk_fast<true>, or sel_sample at T = 1 (x / 1 = x exactly) for the rows it does not take.
// Precondition as sel_topk_fast<true>: S.hist[0..255] zeroed behind a barrier after the previous selection.
__device__ __forceinline__ int sel_sample_range(float (&v)[SEL_VPT_MAX], int n, int vpt, int top_k, float u, float mx, float mn,
                                                SelLds &S) {
    if (top_k > 0 && top_k < n) {
        const int r = sel_topk_fast<true>(v, n, vpt, top_k, u, -1, S, mx, mn);
        if (r != -2) return r;
        __syncthreads();   // (uniform) the waves may still read this selection's histogram
    }
    return sel_sample(v, n, vpt, 1.0f, top_k, u, -1, S);
}

// load one slot's logits row into the owner registers (SC1: agent-scope loads of a row published in this launch)
template <bool SC1>
__device__ __forceinline__ void sel_load(const float *row, int n, int vpt, float (&v)[SEL_VPT_MAX]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) {
        const int i = t * vpt + e;
        const bool in = e < vpt && i < n;
        if constexpr (SC1) v[e] = in ? __hip_atomic_load(row + (in ? i : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : -INFINITY;
        else v[e] = in ? row[i] : -INFINITY;
    }
}
// the same for the vocabularies of the decode path (V = 2048: vpt 8, V = 3072: vpt 12, n == 256 vpt): 16-byte
// loads, all issued before any is consumed
template <int VPT>
__device__ __forceinline__ void sel_load_exact(const float *row, float (&v)[SEL_VPT_MAX]) {
    static_assert(VPT % 4 == 0 && VPT <= SEL_VPT_MAX, "vpt");
    const float4 *r4 = reinterpret_cast<const float4 *>(row + threadIdx.x * VPT);
    float4 q[VPT / 4];
#pragma unroll
    for (int i = 0; i < VPT / 4; ++i) q[i] = r4[i];
#pragma unroll
    for (int i = 0; i < VPT / 4; ++i) { v[4 * i] = q[i].x; v[4 * i + 1] = q[i].y; v[4 * i + 2] = q[i].z; v[4 * i + 3] = q[i].w; }
#pragma unroll
    for (int e = VPT; e < SEL_VPT_MAX; ++e) v[e] = -INFINITY;
}

// Per-slot selection inputs that do not depend on the logits (done flag, frame, seed, utterance id, CB0 prompt
// length / EOS mask / seen bytes of this thread's indices).  A kernel that knows its slot early loads them before
// it waits for the logits, so none of these dependent global loads sits on the chain after the logits arrive.
struct SelPre {
    int done, frame, n_tokens, force;
    uint64_t seed, utt;
    uint32_t seen[SEL_VPT_MAX / 4];   // CB0 seen flags of this thread's indices, byte e of the thread in byte e % 4 of word e / 4
};
template <int MODE>
__device__ __forceinline__ void sel_prefetch(const SelectSpec &sp, int s, SelPre &q) {
    const int t = threadIdx.x, V = sp.V, vpt = (V + 255) / 256;
    q.done = sp.done[s];
    q.frame = sp.frame[s] + sp.frame_offset;
    q.seed = sp.seed_dev ? *sp.seed_dev : sp.seed;
    q.utt = sp.utt[s];
    q.n_tokens = 0;
    q.force = 0;
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX / 4; ++e) q.seen[e] = 0;
    if constexpr (MODE == SEL_CB0) {
        q.n_tokens = sp.n_tokens[s];
        q.force = sp.force_frames[s];
        if (sp.rep != 1.0f) {
            const uint8_t *seen = sp.seen + (size_t)s * V;
            if (V % 1024 == 0) {   // vpt % 4 == 0 and every index in range: whole words (the row is 4-byte aligned)
                const uint32_t *sw = reinterpret_cast<const uint32_t *>(seen + (size_t)t * vpt);
#pragma unroll
                for (int e = 0; e < SEL_VPT_MAX / 4; ++e)
                    if (4 * e < vpt) q.seen[e] = sw[e];
            } else {
#pragma unroll
                for (int e = 0; e < SEL_VPT_MAX; ++e) {
                    const int i = t * vpt + e;
                    if (e < vpt && i < V) q.seen[e >> 2] |= (uint32_t)seen[i] << (8 * (e & 3));
                }
            }
        }
    }
}

// Calling rule of every selection entry point (select_token_pre / select_token_regs / select_token / select_slot,
// sel_sample, sel_sample_range): the workgroup runs a barrier between two selections, and SelLds is not aliased by LDS
// the caller writes in between.  The selection writes its histogram, candidate list and per-wave slots without a
// leading barrier (the previous selection's readers are behind the caller's barrier); all current callers (gemv_kernel.h's
// kSel / kSelG loops, kernels.hip, k_tk_roles, k_cp_roles, k_persist) keep the rule.
// the token of a slot from its prefetched inputs (uniform over the workgroup), or -1 if the slot is done; no side
// effects.  MODE: SEL_CB0 / SEL_CP at compile time (the code-predictor path carries none of the CB0 rules)
template <int MODE>
__device__ __forceinline__ int select_token_pre(const SelectSpec &sp, const SelPre &q, float (&v)[SEL_VPT_MAX], SelLds &S) {
    if (q.done >= 0) return -1;   // uniform over the workgroup
    const int t = threadIdx.x, V = sp.V, vpt = (V + 255) / 256;
    const int frame = q.frame;
    int keep = -1;
    float u;
    if constexpr (MODE == SEL_CB0) {
        const int EOS = sp.eos;
        float m = -INFINITY;
#pragma unroll
        for (int e = 0; e < SEL_VPT_MAX; ++e) {
            const int i = t * vpt + e;
            if (e >= vpt || i >= V) continue;
            float x = v[e];
            if (i >= V - 1024 && i != EOS) x = -INFINITY;                          // :2418-2422
            if (sp.rep != 1.0f && ((q.seen[e >> 2] >> (8 * (e & 3))) & 0xffu)) x = x > 0.0f ? x / sp.rep : x * sp.rep;  // :2425-2435
            v[e] = x;
            m = fmaxf(m, x);
        }
        m = sel_block_max(m, S);
        const int expected = max(20, q.n_tokens * 4);                              // :2439-2445
        const bool masked = frame < q.force;
#pragma unroll
        for (int e = 0; e < SEL_VPT_MAX; ++e) {
            if (t * vpt + e != EOS || e >= vpt) continue;
            if (frame >= expected) {
                const float ramp = fminf(1.0f, (float)(frame - expected) / (float)expected);
                v[e] += ramp * ((m + 5.0f) - v[e]);
            }
            if (masked) v[e] = -INFINITY;
        }
        keep = masked ? -1 : EOS;
        u = uniform24(q.seed, q.utt, (uint64_t)frame, 0);
    } else {
        u = uniform24(q.seed, q.utt, (uint64_t)frame, (uint64_t)sp.step + 1);
    }
    return sp.temperature <= 0.0f ? sel_argmax(v, V, vpt, S) : sel_sample(v, V, vpt, sp.temperature, sp.top_k, u, keep, S);
}

// the token of slot s (uniform over the workgroup), or -1 if the slot is done; no side effects
// select_token on a row already loaded into the owner registers (sel_load): lets a kernel issue the logits loads
// ahead of its weight stream
// MODE: SEL_CB0 / SEL_CP at compile time, or SEL_NONE to dispatch on sp.mode
template <int MODE = SEL_NONE>
__device__ __forceinline__ int select_token_regs(const SelectSpec &sp, float (&v)[SEL_VPT_MAX], int s, SelLds &S) {
    if constexpr (MODE == SEL_NONE) {
        return sp.mode == SEL_CB0 ? select_token_regs<SEL_CB0>(sp, v, s, S) : select_token_regs<SEL_CP>(sp, v, s, S);
    } else {
        SelPre q;
        sel_prefetch<MODE>(sp, s, q);
        return select_token_pre<MODE>(sp, q, v, S);
    }
}

// agent-scope (sc1) loads of a row published in this launch, exact widths: unconditional, all issued first
template <int VPT>
__device__ __forceinline__ void sel_load_exact_sc1(const float *row, float (&v)[SEL_VPT_MAX]) {
    const float *r = row + threadIdx.x * VPT;
#pragma unroll
    for (int e = 0; e < VPT; ++e) v[e] = __hip_atomic_load(r + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int e = VPT; e < SEL_VPT_MAX; ++e) v[e] = -INFINITY;
}

template <bool SC1>
__device__ __forceinline__ int select_token(const SelectSpec &sp, const float *row, int s, SelLds &S) {
    float v[SEL_VPT_MAX];
    if (sp.V == 2048) {
        if constexpr (SC1) sel_load_exact_sc1<8>(row, v);
        else sel_load_exact<8>(row, v);
    } else if (sp.V == 3072) {
        if constexpr (SC1) sel_load_exact_sc1<12>(row, v);
        else sel_load_exact<12>(row, v);
    } else {
        sel_load<SC1>(row, sp.V, (sp.V + 255) / 256, v);
    }
    return select_token_regs(sp, v, s, S);
}

// the side effects of a selected token (thread 0 of ONE workgroup per slot): frame codes, EOS, seen set
__device__ __forceinline__ void select_commit(const SelectSpec &sp, int s, int tok) {
    const int frame = sp.frame[s] + sp.frame_offset;
    if (sp.mode == SEL_CB0) {
        sp.tokens[s * 16] = tok;
        if (tok == sp.eos) { sp.done[s] = frame; return; }
        sp.seen[(size_t)s * sp.V + tok] = 1;
        if (frame < sp.max_len) sp.codes[((size_t)s * sp.max_len + frame) * sp.ncb] = tok;
    } else {
        sp.tokens[s * 16 + sp.step + 1] = tok;
        if (frame < sp.max_len) sp.codes[((size_t)s * sp.max_len + frame) * sp.ncb + sp.step + 1] = tok;
    }
}

// select the token of slot s from its logits row and record it (SelectSpec semantics, kernels.h)
template <bool SC1>
__device__ __forceinline__ void select_slot(const SelectSpec &sp, const float *row, int s, SelLds &S) {
    const int tok = select_token<SC1>(sp, row, s, S);
    if (tok >= 0 && threadIdx.x == 0) select_commit(sp, s, tok);
}

}  // namespace q3t
