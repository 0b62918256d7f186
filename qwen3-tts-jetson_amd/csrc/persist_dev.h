// persist_dev.h — device helpers shared by the persistent kernels (persist.hip: the talker step and the 1.7B /
// fallback code-predictor frame; persist_cp.hip: the role-specialised code-predictor frame): global loads that never
// lower to flat loads, the {payload, tag} granule hand-off (one 8-byte agent-scope store, polled with agent-scope
// loads until every tag matches; MI355X_MICROARCH.md hand-off rows), the bounded wait and the RMSNorm prologue.
#pragma once
#include "kernels.h"

namespace q3t {
namespace pdev {

constexpr unsigned SPIN_LIMIT = 1u << 21;   // polls before a hand-off wait gives up (sets *err)

template <class V>
__device__ __forceinline__ V ldgv(const void *p) {
    typedef const __attribute__((address_space(1))) V gV;
    return *(gV *)(p);
}
__device__ __forceinline__ uint4 ld16(const void *p) {
    const u32x4_t v = ldgv<u32x4_t>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 ldf4(const float *p) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v v = ldgv<f4v>(p);
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ld8(const void *p) {
    typedef unsigned u2v __attribute__((ext_vector_type(2)));
    const u2v v = ldgv<u2v>(p);
    return make_uint2(v.x, v.y);
}

// ---------------------------------------------------------------- granules
__device__ __forceinline__ void g_put(uint64_t *p, uint32_t payload, uint32_t tag) {
    __hip_atomic_store(p, ((uint64_t)tag << 32) | payload, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t g_ld(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint4 ld16_sc1(const uint16_t *p) {   // 16 B as two agent-scope (L1-bypassing) 8-B loads
    uint64_t *q = reinterpret_cast<uint64_t *>(const_cast<uint16_t *>(p));
    const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}

struct Ctl {
    unsigned *err;
    bool abort;
};

// spin until granules base[(i / RUN) * STRIDE + i % RUN], i in [0, N), all carry `tag`; payloads to out.  Bounded:
// after SPIN_LIMIT polls (or once any workgroup has flagged a timeout) the wait gives up, sets *err and lets the launch
// drain.
template <int N, int STRIDE = 1, int RUN = 1>
__device__ __forceinline__ void g_wait(const uint64_t *base, uint32_t tag, uint32_t (&out)[N], Ctl &c) {
    uint64_t v[N];
    unsigned it = 0;
    while (true) {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = g_ld(base + (i / RUN) * STRIDE + i % RUN);
        bool ok = true;
#pragma unroll
        for (int i = 0; i < N; ++i) ok &= (uint32_t)(v[i] >> 32) == tag;
        if (ok || c.abort) break;
        ++it;
        if ((it & 255u) == 0) {
            if (__hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || it >= SPIN_LIMIT) {
                c.abort = true;
                __hip_atomic_fetch_or(c.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
#ifndef Q3T_POLL_SLEEP
#define Q3T_POLL_SLEEP 1
#endif
        if constexpr (Q3T_POLL_SLEEP > 0) __builtin_amdgcn_s_sleep(Q3T_POLL_SLEEP);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = (uint32_t)v[i];
}

// ---------------------------------------------------------------- 16-byte poll loads
// Two granules per global_load_dwordx4 sc1 (each 8-byte half was written by ONE 8-byte sc1 store and is checked against
// its own tag, so a pair torn between its halves only costs another poll).  The M loads of one poll and their
// s_waitcnt vmcnt(0) are ONE asm statement: the compiler cannot place a read or a copy of a destination register between
// a load and its wait, whatever the register pressure.  (Q3T_POLL16=0: the 8-byte atomic loads of g_wait.)
#ifndef Q3T_POLL16
#define Q3T_POLL16 1
#endif
template <int M>
__device__ __forceinline__ void ld16_sc1_batch(const uint64_t *const (&a)[M], u32x4_t (&r)[M]) {
    if constexpr (M == 1)
        asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(r[0]) : "v"(a[0]) : "memory");
    else if constexpr (M == 2)
        asm volatile("global_load_dwordx4 %0, %2, off sc1\n\tglobal_load_dwordx4 %1, %3, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(r[0]), "=&v"(r[1]) : "v"(a[0]), "v"(a[1]) : "memory");
    else if constexpr (M == 3)
        asm volatile("global_load_dwordx4 %0, %3, off sc1\n\tglobal_load_dwordx4 %1, %4, off sc1\n\tglobal_load_dwordx4 %2, %5, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]) : "v"(a[0]), "v"(a[1]), "v"(a[2]) : "memory");
    else if constexpr (M == 4)
        asm volatile("global_load_dwordx4 %0, %4, off sc1\n\tglobal_load_dwordx4 %1, %5, off sc1\n\tglobal_load_dwordx4 %2, %6, off sc1\n\tglobal_load_dwordx4 %3, %7, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]) : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]) : "memory");
    else if constexpr (M == 5)
        asm volatile("global_load_dwordx4 %0, %5, off sc1\n\tglobal_load_dwordx4 %1, %6, off sc1\n\tglobal_load_dwordx4 %2, %7, off sc1\n\tglobal_load_dwordx4 %3, %8, off sc1\n\tglobal_load_dwordx4 %4, %9, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]) : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]) : "memory");
    else if constexpr (M == 6)
        asm volatile("global_load_dwordx4 %0, %6, off sc1\n\tglobal_load_dwordx4 %1, %7, off sc1\n\tglobal_load_dwordx4 %2, %8, off sc1\n\tglobal_load_dwordx4 %3, %9, off sc1\n\tglobal_load_dwordx4 %4, %10, off sc1\n\tglobal_load_dwordx4 %5, %11, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]) : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]) : "memory");
    else if constexpr (M == 8)
        asm volatile("global_load_dwordx4 %0, %8, off sc1\n\tglobal_load_dwordx4 %1, %9, off sc1\n\tglobal_load_dwordx4 %2, %10, off sc1\n\tglobal_load_dwordx4 %3, %11, off sc1\n\tglobal_load_dwordx4 %4, %12, off sc1\n\tglobal_load_dwordx4 %5, %13, off sc1\n\tglobal_load_dwordx4 %6, %14, off sc1\n\tglobal_load_dwordx4 %7, %15, off sc1\n\ts_waitcnt vmcnt(0)" : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7]) : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]) : "memory");
    else static_assert(M == 0, "ld16_sc1_batch: unsupported count");
}
// g_wait over RUNS runs of RUN contiguous granules (RUN even, 16-B aligned), run k at base + k * STRIDE
template <int RUNS, int RUN, int STRIDE = 0>
__device__ __forceinline__ void g_wait16(const uint64_t *base, uint32_t tag, uint32_t (&out)[RUNS * RUN], Ctl &c) {
    static_assert(RUN % 2 == 0, "pairs");
    constexpr int M = RUNS * RUN / 2;
    u32x4_t r[M];
    unsigned it = 0;
    while (true) {
        const uint64_t *a[M];
#pragma unroll
        for (int k = 0; k < RUNS; ++k)
#pragma unroll
            for (int j = 0; j < RUN / 2; ++j) a[k * (RUN / 2) + j] = base + k * STRIDE + 2 * j;
        ld16_sc1_batch<M>(a, r);
        bool ok = true;
#pragma unroll
        for (int m = 0; m < M; ++m) ok &= r[m].y == tag && r[m].w == tag;
        if (ok || c.abort) break;
        ++it;
        if ((it & 255u) == 0) {
            if (__hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || it >= SPIN_LIMIT) {
                c.abort = true;
                __hip_atomic_fetch_or(c.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        if constexpr (Q3T_POLL_SLEEP > 0) __builtin_amdgcn_s_sleep(Q3T_POLL_SLEEP);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
        out[2 * m] = r[m].x;
        out[2 * m + 1] = r[m].z;
    }
}
// g_wait_pair with 16-byte loads: N contiguous granules at a and M at b (both even, 16-B aligned)
template <int N, int M2>
__device__ __forceinline__ void g_wait16_pair(const uint64_t *a, const uint64_t *b, uint32_t tag, uint32_t (&oa)[N], uint32_t (&ob)[M2],
                                              Ctl &c) {
    static_assert(N % 2 == 0 && M2 % 2 == 0, "pairs");
    constexpr int M = (N + M2) / 2;
    u32x4_t r[M];
    unsigned it = 0;
    while (true) {
        const uint64_t *ad[M];
#pragma unroll
        for (int j = 0; j < N / 2; ++j) ad[j] = a + 2 * j;
#pragma unroll
        for (int j = 0; j < M2 / 2; ++j) ad[N / 2 + j] = b + 2 * j;
        ld16_sc1_batch<M>(ad, r);
        bool ok = true;
#pragma unroll
        for (int m = 0; m < M; ++m) ok &= r[m].y == tag && r[m].w == tag;
        if (ok || c.abort) break;
        ++it;
        if ((it & 255u) == 0) {
            if (__hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || it >= SPIN_LIMIT) {
                c.abort = true;
                __hip_atomic_fetch_or(c.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        if constexpr (Q3T_POLL_SLEEP > 0) __builtin_amdgcn_s_sleep(Q3T_POLL_SLEEP);
    }
#pragma unroll
    for (int m = 0; m < N / 2; ++m) { oa[2 * m] = r[m].x; oa[2 * m + 1] = r[m].z; }
#pragma unroll
    for (int m = 0; m < M2 / 2; ++m) { ob[2 * m] = r[N / 2 + m].x; ob[2 * m + 1] = r[N / 2 + m].z; }
}
// the contiguous form of g_wait: N granules at base (16-B aligned)
template <int N>
__device__ __forceinline__ void g_waitc(const uint64_t *base, uint32_t tag, uint32_t (&out)[N], Ctl &c) {
    if constexpr (Q3T_POLL16 && N % 2 == 0) g_wait16<1, N>(base, tag, out, c);
    else g_wait<N>(base, tag, out, c);
}

// g_wait over two granule runs a[0..N) and b[0..M) in one poll loop (one round trip per poll for both)
template <int N, int M>
__device__ __forceinline__ void g_wait_pair(const uint64_t *a, const uint64_t *b, uint32_t tag, uint32_t (&oa)[N], uint32_t (&ob)[M],
                                            Ctl &c) {
    uint64_t v[N + M];
    unsigned it = 0;
    while (true) {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = g_ld(a + i);
#pragma unroll
        for (int i = 0; i < M; ++i) v[N + i] = g_ld(b + i);
        bool ok = true;
#pragma unroll
        for (int i = 0; i < N + M; ++i) ok &= (uint32_t)(v[i] >> 32) == tag;
        if (ok || c.abort) break;
        ++it;
        if ((it & 255u) == 0) {
            if (__hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || it >= SPIN_LIMIT) {
                c.abort = true;
                __hip_atomic_fetch_or(c.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        if constexpr (Q3T_POLL_SLEEP > 0) __builtin_amdgcn_s_sleep(Q3T_POLL_SLEEP);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) oa[i] = (uint32_t)v[i];
#pragma unroll
    for (int i = 0; i < M; ++i) ob[i] = (uint32_t)v[N + i];
}

// g_gate: lane 0 of each wave polls one granule alone (one 8-B load per poll) until it carries `tag`.  g_wait_gated:
// g_wait behind the gate on the wave's first granule: lane 0 first polls it alone, then the wave sweeps all N.  For long waits of many granules per thread, whose sweeps would otherwise flood
// the CU's memory path for the whole wait (a co-resident workgroup's stores then stalled for ~230 us).
__device__ __forceinline__ void g_gate(const uint64_t *g, uint32_t tag, Ctl &c) {
    if ((threadIdx.x & 63) == 0) {
        unsigned it = 0;
        while (!c.abort && (uint32_t)(g_ld(g) >> 32) != tag) {
            if ((++it & 255u) == 0 && (__hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
                                       it >= SPIN_LIMIT)) {
                c.abort = true;
                __hip_atomic_fetch_or(c.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    c.abort = __shfl(c.abort ? 1 : 0, 0) != 0;
}
template <int N, int STRIDE = 1, int RUN = 1>
__device__ __forceinline__ void g_wait_gated(const uint64_t *base, uint32_t tag, uint32_t (&out)[N], Ctl &c) {
    g_gate(base, tag, c);
    g_wait<N, STRIDE, RUN>(base, tag, out, c);
}

// LDS written by this wave, then read by this wave only: the wave's own LDS traffic drained, no workgroup barrier
// (the slowest wave's poll no longer holds the others' dot products).  Q3T_WAVE_SYNC=0: a workgroup barrier.
#ifndef Q3T_WAVE_SYNC
#define Q3T_WAVE_SYNC 1
#endif
__device__ __forceinline__ void wave_lds_sync() {
    if constexpr (Q3T_WAVE_SYNC) {
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
    } else {
        __syncthreads();
    }
}

__device__ __forceinline__ float4 f4_of(const uint32_t (&u)[4]) {
    return make_float4(__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3]));
}


// block sum of one double per thread ((w0 + w1) + (w2 + w3) of the wave sums).  ONE barrier: the caller guarantees a
// workgroup barrier between consecutive calls (the role kernels' f16 tile barrier after every RMSNorm), so no wave can
// overwrite scr while another still reads the previous sums.
__device__ __forceinline__ double block_sum_d(double v, double *scr) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = wave_sum_d(v);
    if (lane == 0) scr[wave] = v;
    __syncthreads();
    return (scr[0] + scr[1]) + (scr[2] + scr[3]);
}

// RMSNorm of the f32 row held as thread t's elements 4t..4t+3 (K = 1024) -> f16 tile xs; optional f32 side output
// (gemv.hip prologue: double sums, (x * scale) * w, f16 rounding).  The caller runs a workgroup barrier before xs is
// read and before the next call (block_sum_d).
__device__ __forceinline__ void rms_to_f16(float4 x, float4 w, float eps, uint16_t *xs, double *dscr, float *side) {
    const int t = threadIdx.x;
    double ss = (double)(x.x * x.x) + (double)(x.y * x.y) + (double)(x.z * x.z) + (double)(x.w * x.w);
    ss = block_sum_d(ss, dscr);
    const float scale = 1.0f / sqrtf((float)(ss / 1024) + eps);
    const float y0 = (x.x * scale) * w.x, y1 = (x.y * scale) * w.y, y2 = (x.z * scale) * w.z, y3 = (x.w * scale) * w.w;
    if (side) *reinterpret_cast<float4 *>(side + 4 * t) = make_float4(y0, y1, y2, y3);
    uint2 h;
    h.x = (uint32_t)f2h(y0) | ((uint32_t)f2h(y1) << 16);
    h.y = (uint32_t)f2h(y2) | ((uint32_t)f2h(y3) << 16);
    *reinterpret_cast<uint2 *>(xs + 4 * t) = h;
}

}  // namespace pdev
}  // namespace q3t
