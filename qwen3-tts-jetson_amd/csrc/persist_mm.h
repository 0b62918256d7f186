// persist_mm.h — the batched persistent launches' shared device machinery (persist_cpb.hip: the code-predictor frame,
// persist_tkb.hip: the talker step), 0.6B shapes, 1..64 slots:
//   - hand-offs: flags (sc1 payload stores, every storing wave's vmcnt(0), a workgroup barrier, one lane's sc1 flag
//     store; consumers poll with sc1 loads, then load the payload with sc1 loads) and {f32, tag} granules (one 8-byte
//     sc1 store, polled until every tag matches), both MI355X_MICROARCH.md hand-off table rows; bounded waits
//   - the MFMA tile job: 2 row tiles of 32 rows x one 32-token tile with k_gemm_mfma's numerics (gemm_mfma.hip): weights
//     DMA'd into LDS one job ahead, activations from hand-off buffers in B-fragment order, 4 K quarters summed in LDS
//   - the granule epilogue
#pragma once
#include "persist_dev.h"

namespace q3t {
namespace pmm {
using namespace pdev;

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

constexpr int H = 1024, NH = 16, NKV = 8, D = 128, QKVN = (NH + 2 * NKV) * D, INTER = 3072, CPV = 2048, VOC = 3072;
constexpr int G = 256, SMAX = 64;
constexpr int BUF_RSRC = 0x00020000;   // buffer resource word 3 (gfx9 family)
constexpr int SC1 = 16;                // buffer instruction cache policy: sc1
constexpr int SC1V = SC1 | (int)0x80000000u;   // sc1, volatile (a poll's load is re-issued every iteration)
constexpr int FLAGS_PER_KIND = 512;   // flag words per hand-off kind

// The f16 activation buffers behind flags (xna, xnf, attn, h) are kept in the MFMA B-fragment order of their consumers:
// 16-byte chunk k8 (halves 8 k8 .. 8 k8 + 7) of token tok at ((tok / 32 * kch + k8) * 32 + tok % 32) * 16 bytes, kch =
// K / 8.  A consumer wave's load instruction for chunk column (c, j) then reads two runs of 32 consecutive chunks (whole
// 64-byte sectors) instead of one 16-byte piece of 64 different sectors: sc1 loads are not merged in L1, so the
// row-major order moved every activation byte four times over the CU's L2 path.
__device__ __forceinline__ int fragoff(int kch, int tok, int k) {   // byte offset of half k of token tok (8-byte stores: k % 4 == 0)
    return (((tok >> 5) * kch + (k >> 3)) * 32 + (tok & 31)) * 16 + (k & 7) * 2;
}

struct Ctx {
    uint4 (*wl)[32][64];         // LDS: [wave][A slot][lane] (the next job's weight fragments / the K-quarter partials)
    uint64_t *prof;              // development timeline (null = off)
    Ctl c;
    unsigned seq;
    unsigned *flags;             // [kind][FLAGS_PER_KIND]
    __amdgpu_buffer_rsrc_t rs;   // the whole state block
    int S_;                      // slots
    __device__ uint32_t tag(int ph) const { return (seq << 10) + (unsigned)ph + 1u; }
    __device__ unsigned *flag(int kind, int j) const { return flags + kind * FLAGS_PER_KIND + j; }
};

// ---------------------------------------------------------------- flag polls
// every lane i < n of the wave polls flag idx(i); the wave leaves once all carry `tag` (bounded)
#ifdef Q3T_DEV
// development timeline (Q3T_PERSIST_PROF): thread 0 of each workgroup stamps phase ph, k = 0 wait start, 1 data ready,
// 2 published, 3 computed; [workgroup][768 phases][4] s_memrealtime (100 MHz)
#define CPROF(ph, k)                                                                                          \
    do {                                                                                                      \
        if (X.prof && threadIdx.x == 0) X.prof[((size_t)blockIdx.x * 768 + (ph)) * 4 + (k)] = wall_clock64(); \
    } while (0)
#else
#define CPROF(ph, k) ((void)0)
#endif
template <class Idx>
__device__ __forceinline__ void wait_flags(Ctx &X, int kind, int n, Idx idx, uint32_t tag) {
    const int lane = threadIdx.x & 63;
    const int ph_ = (int)((tag - 1u) & 1023u);
    (void)ph_;
    CPROF(ph_, 0);
    const unsigned *f0 = X.flags + kind * FLAGS_PER_KIND;
    const unsigned *fa = f0 + idx(lane < n ? lane : 0);
    const unsigned *fb = f0 + idx(lane + 64 < n ? lane + 64 : 0);
    unsigned it = 0;
    while (true) {
        bool ok = true;
        if (lane < n) ok &= __hip_atomic_load(fa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tag;
        if (lane + 64 < n) ok &= __hip_atomic_load(fb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tag;
        if (__all(ok) || X.c.abort) break;
        ++it;
        if ((it & 255u) == 0) {
            if (__hip_atomic_load(X.c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || it >= SPIN_LIMIT) {
                X.c.abort = true;
                __hip_atomic_fetch_or(X.c.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_s_sleep(1);
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);   // the payload loads stay behind the poll
    CPROF(ph_, 1);
}

// the same for a whole workgroup: wave 0 polls every flag, the others load after the barrier it then joins (the polling
// traffic of one wave instead of four)
template <class Idx>
__device__ __forceinline__ void wait_flags_wg(Ctx &X, int kind, int n, Idx idx, uint32_t tag) {
    if (threadIdx.x < 64) wait_flags(X, kind, n, idx, tag);
    __syncthreads();
}

// publish: every storing wave drains its sc1 stores, then one lane signals for the workgroup
__device__ __forceinline__ void publish(Ctx &X, int kind, int j, uint32_t tag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(X.flag(kind, j), tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    CPROF((int)((tag - 1u) & 1023u), 2);
}

// the launch's LAST workgroup to finish bumps seq (ctr[0]; an exit ticket in ctr[48]): every workgroup has read seq by
// then, whatever order the workgroups were dispatched in.  Every workgroup runs it, idle ones included
__device__ __forceinline__ void exit_ticket(unsigned *ctr, unsigned seq) {
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned *done = ctr + 48;
        if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctr, seq + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// spin until every granule a lane loads (issue(r) fills r) carries `tag` (bounded, as wait_flags)
template <int M, class Issue>
__device__ __forceinline__ void poll_gran(Ctx &X, uint32_t tag, u32x4_t (&r)[M], Issue issue) {
    unsigned it = 0;
    // gate: lane 0 alone polls its own granules first, so the wave's full sweeps start once the data is arriving
    if ((threadIdx.x & 63) == 0) {
        while (true) {
            issue(r);
            bool ok = true;
#pragma unroll
            for (int m = 0; m < M; ++m) ok &= r[m].y == tag && r[m].w == tag;
            if (ok || X.c.abort) break;
            if ((++it & 255u) == 0 && (__hip_atomic_load(X.c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || it >= SPIN_LIMIT)) {
                X.c.abort = true;
                __hip_atomic_fetch_or(X.c.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    X.c.abort = __shfl(X.c.abort ? 1 : 0, 0) != 0;
    it = 0;
    while (true) {
        issue(r);
        bool ok = true;
#pragma unroll
        for (int m = 0; m < M; ++m) ok &= r[m].y == tag && r[m].w == tag;
        if (__all(ok) || X.c.abort) break;
        ++it;
        if ((it & 255u) == 0) {
            if (__hip_atomic_load(X.c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || it >= SPIN_LIMIT) {
                X.c.abort = true;
                __hip_atomic_fetch_or(X.c.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// ---------------------------------------------------------------- MFMA tile job (gemm_mfma.hip k_gemm_mfma numerics)
// A job is RT = 2 row tiles of 32 rows (64 rows) x one 32-token tile: both row tiles share every activation fragment, so
// the activation rows every job pulls through the fabric (the sc1 hand-off reads, which bound these phases) are half
// those of 32-row jobs.  Per row tile the arithmetic is k_gemm_mfma's: A = W[row0 + 32 rt + r][k], B = X[token][k] for
// lane (r = lane & 31, h = lane >> 5), k = kq + 64c + 32h + 8j, wave w owning the K quarter kq = kbase + 64 NCH w, the
// MFMA chain in (c, j) order, the 4 quarters summed through LDS in wave order.
constexpr int RT = 2;
constexpr int RS = 68;   // row stride (floats) of the K-quarter partial tiles in LDS: the epilogue's 16-byte token-quad
                         // reads then fall on all 64 banks
template <int NCH>
__device__ __forceinline__ void load_w(uint4 (*wl)[32][64], const uint16_t *W, int ldw, int row0, int kbase) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
#ifdef CPB_EXP_NOW   // timing experiment (development variant builds): no weight loads
    return;
#endif
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const uint16_t *p = W + (size_t)(row0 + 32 * rt + r) * ldw + kbase + wave * (NCH * 64) + h * 32;
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_global_load_lds(p + c * 64 + j * 8, (__attribute__((address_space(3))) void *)&wl[wave][16 * rt + 4 * c + j][0],
                                                 16, 0, 0);
    }
}

// B fragments of tokens t0 + r: sc1 loads of the hand-off buffer at byte offset xoff (fragment order, kch chunks per
// token; the columns of tokens >= S read unwritten chunks and are never stored), then the MFMA chains; the K-quarter
// partials land in the wave's LDS region (its A slots, consumed)
template <int NCH>
__device__ __forceinline__ void mm_tile(Ctx &X, size_t xoff, int kch, int kbase, int t0) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
    u32x4_t xb[4 * NCH];
    const int off = (int)xoff + fragoff(kch, t0 + r, kbase + wave * (NCH * 64) + h * 32);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#ifdef CPB_EXP_NOX   // timing experiment (development variant builds): no activation loads
            xb[4 * c + j] = u32x4_t{(unsigned)off, 0u, 0u, 0u};
#else
            xb[4 * c + j] = __builtin_amdgcn_raw_buffer_load_b128(X.rs, off + (c * 8 + j) * 512, 0, SC1);
#endif
        }
    f32x16_t acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[rt][i] = 0.0f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's weight DMA (and the B fragments) have landed
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const half8_t bf = __builtin_bit_cast(half8_t, xb[4 * c + j]);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
                acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8_t, X.wl[wave][16 * rt + 4 * c + j][lane]), bf,
                                                                 acc[rt], 0, 0, 0);
        }
    // every A slot this wave reads has been read (the MFMAs consumed them): the region takes the partials
    float *red = reinterpret_cast<float *>(&X.wl[wave][0][0]);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[(rt * 16 + i) * RS + lane] = acc[rt][i];
    __syncthreads();
}
// register i of row tile rt, lane `src`, summed over the 4 K quarters in wave order (k_gemm_mfma sum4)
__device__ __forceinline__ float sum4(const uint4 (*wl)[32][64], int rt, int i, int src) {
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += reinterpret_cast<const float *>(&wl[w][0][0])[(rt * 16 + i) * RS + src];
    return v;
}

// granule epilogue (QKV rows, split-K slabs, lm_head logits): {f32, tag} granules out[tok][row0 ..] with 8-byte sc1
// stores (MI355X_MICROARCH.md handoff-1to1: the payload carries its own tag, no drain and no flag).  Thread t takes job
// row rho = t % 64 and the token quads 4 (t / 64) and 4 (t / 64) + 16: per wave 16-byte LDS reads of four tokens (8
// reads instead of 32 scalar ones: the epilogue is latency-bound at one wave per SIMD), and every store instruction
// writes 64 consecutive rows of one token (512 contiguous bytes).  Register i of lane (r, h) holds tile row
// (i & 3) + 8 (i >> 2) + 4h of token r, so row rr of a tile is register (rr & 3) + 4 (rr >> 3) of half (rr >> 2) & 1.
__device__ __forceinline__ void epi_gran(Ctx &X, size_t obase, int ldo, int row0, int t0, uint32_t tag) {
    const int t = threadIdx.x, rho = t & 63, tq = t >> 6;
    const int rt = rho >> 5, rr = rho & 31;
    const int src4 = ((rt * 16 + (rr & 3) + 4 * (rr >> 3)) * RS + 32 * ((rr >> 2) & 1)) / 4 + tq;   // 16-byte units
    uint4 q[2][4];   // all eight reads first (one LDS round trip), then the sums
#pragma unroll
    for (int hq = 0; hq < 2; ++hq)
#pragma unroll
        for (int w = 0; w < 4; ++w) q[hq][w] = (&X.wl[w][0][0])[src4 + 4 * hq];
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {
        const int r0 = 4 * tq + 16 * hq;
        float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};   // k_gemm_mfma sum4: ((0 + q0) + q1) + q2) + q3
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            v[0] += __uint_as_float(q[hq][w].x); v[1] += __uint_as_float(q[hq][w].y);
            v[2] += __uint_as_float(q[hq][w].z); v[3] += __uint_as_float(q[hq][w].w);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {   // tokens S .. 63 too (rows of the SMAX-row buffer nobody reads): no branches
            const u32x2_t g = {__float_as_uint(v[u]), tag};
            __builtin_amdgcn_raw_buffer_store_b64(g, X.rs, (int)(obase + ((size_t)(t0 + r0 + u) * ldo + row0 + rho) * 8), 0, SC1);
        }
    }
    __syncthreads();   // the LDS region is the next job's DMA target
}


}  // namespace pmm
}  // namespace q3t
