// dev microbenchmark: the price of one all-to-all granule hand-off inside a persistent launch (256 workgroups x 256
// threads, one per CU), as a chain of R rounds with no body: round r, every producing workgroup publishes its slice of
// an NG-granule vector {payload, tag r}, every workgroup gathers the whole vector, then round r + 1.  Time per round
// = the edge (last publish -> every consumer has seen it) + producer skew.  Variants (argv[1]):
//   0  current protocol: 256 producers x 4 granules, each thread polls 4 granules, s_sleep(1) between polls
//   1  polls pipelined: a second sweep issued before the first one is checked
//   2  64 producers x 16 granules (whole 128-B lines per producer)
//   3  8 producers x 128 granules (the attention -> O-projection edge)
//   4  one wave per workgroup polls (16 granules per lane), the others wait at a barrier
//   5  no s_sleep between polls
//   6  256 producers, consumers poll a per-producer-line layout (each producer's 4 granules padded to 128 B)
//   7  current protocol, consumers poll only the 4 granules of... (control: 2 granules per thread, NG 512)
// Every wait is bounded (an abort word; the launch drains).  Build: hipcc --offload-arch=gfx950 -O3 edgebench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ void g_put(uint64_t *p, uint32_t payload, uint32_t tag) {
    __hip_atomic_store(p, ((uint64_t)tag << 32) | payload, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t g_ld(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr unsigned LIMIT = 1u << 22;

template <int N, int SLEEP, int STRIDE>
__device__ __forceinline__ bool wait_n(const uint64_t *base, uint32_t tag, uint32_t *out, unsigned *err) {
    uint64_t v[N];
    unsigned it = 0;
    while (true) {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = g_ld(base + i * STRIDE);
        bool ok = true;
#pragma unroll
        for (int i = 0; i < N; ++i) ok &= (uint32_t)(v[i] >> 32) >= tag;
        if (ok) break;
        if ((++it & 255u) == 0 && (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || it > LIMIT)) {
            __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        if constexpr (SLEEP > 0) __builtin_amdgcn_s_sleep(SLEEP);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = (uint32_t)v[i];
    return true;
}

// pipelined: two sweeps in flight
template <int N>
__device__ __forceinline__ bool wait_pipe(const uint64_t *base, uint32_t tag, uint32_t *out, unsigned *err) {
    uint64_t a[N], b[N];
#pragma unroll
    for (int i = 0; i < N; ++i) a[i] = g_ld(base + i);
    __builtin_amdgcn_s_sleep(8);
    unsigned it = 0;
    while (true) {
#pragma unroll
        for (int i = 0; i < N; ++i) b[i] = g_ld(base + i);
        bool ok = true;
#pragma unroll
        for (int i = 0; i < N; ++i) ok &= (uint32_t)(a[i] >> 32) >= tag;
        if (ok) {
#pragma unroll
            for (int i = 0; i < N; ++i) out[i] = (uint32_t)a[i];
            return true;
        }
        __builtin_amdgcn_s_sleep(8);
#pragma unroll
        for (int i = 0; i < N; ++i) a[i] = g_ld(base + i);
        ok = true;
#pragma unroll
        for (int i = 0; i < N; ++i) ok &= (uint32_t)(b[i] >> 32) >= tag;
        if (ok) {
#pragma unroll
            for (int i = 0; i < N; ++i) out[i] = (uint32_t)b[i];
            return true;
        }
        if ((++it & 127u) == 0 && (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || it > LIMIT)) {
            __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

template <int V>
__global__ void __launch_bounds__(256) k_edge(uint64_t *buf, unsigned *err, int rounds, unsigned tag0, float *sink) {
    extern __shared__ uint32_t lds[];
    const int w = blockIdx.x, t = threadIdx.x;
    float acc = 0.0f;
    for (int r = 0; r < rounds; ++r) {
        const uint32_t tag = ((tag0 + (unsigned)r) << 1) | 1u;
        uint64_t *g = buf + (size_t)(V == 9 ? r % 5 : (r & 1)) * 8192;   // two buffers alternate (a round's gather never meets the next round's publish)
        uint32_t u[16];
        bool ok = true;
        if constexpr (V == 0 || V == 1 || V == 4 || V == 5) {
            if (t < 4) g_put(g + w * 4 + t, (uint32_t)(w * 4 + t + r), tag);
            if constexpr (V == 0) ok = wait_n<4, 1, 1>(g + 4 * t, tag, u, err);
            if constexpr (V == 5) ok = wait_n<4, 0, 1>(g + 4 * t, tag, u, err);
            if constexpr (V == 1) ok = wait_pipe<4>(g + 4 * t, tag, u, err);
            if constexpr (V == 4) {
                if (t < 64) ok = wait_n<16, 1, 1>(g + 16 * t, tag, u, err);
                __syncthreads();
                if (t < 64) for (int i = 0; i < 16; ++i) lds[16 * t + i] = u[i];
                __syncthreads();
                for (int i = 0; i < 4; ++i) u[i] = lds[4 * t + i];
            }
        } else if constexpr (V == 2) {
            if (w < 64 && t < 16) g_put(g + w * 16 + t, (uint32_t)(w * 16 + t + r), tag);
            ok = wait_n<4, 1, 1>(g + 4 * t, tag, u, err);
        } else if constexpr (V == 3) {
            if (w < 8 && t < 128) g_put(g + w * 128 + t, (uint32_t)(w * 128 + t + r), tag);
            ok = wait_n<4, 1, 1>(g + 4 * t, tag, u, err);
        } else if constexpr (V == 6) {
            // each producer's 4 granules in its own 128-B line (stride 16 granules): 4 KB... 32 KB vector
            if (t < 4) g_put(g + w * 16 + t, (uint32_t)(w * 4 + t + r), tag);
            ok = wait_n<4, 1, 1>(g + 16 * t, tag, u, err);   // thread t reads producer t's line
        } else if constexpr (V >= 100) {
            constexpr int P = V - 100, GP = 1024 / P;
            if (w < P && t < GP) g_put(g + w * GP + t, (uint32_t)(w * GP + t + r), tag);
            ok = wait_n<4, 1, 1>(g + 4 * t, tag, u, err);
        } else if constexpr (V == 9 || V == 10) {
            // role-specialised chain: 5 roles on disjoint workgroups (QKV 64, attention 8, O 32, gate/up 64, down 64);
            // round r: role r%5 publishes its slice, role (r+1)%5 gathers the whole vector (V 10: 128 x 2 roles)
            constexpr int NR = 5;
            const int st0[NR] = {0, 64, 72, 104, 168};
            const int sz[NR] = {64, 8, 32, 64, 64};
            int role = -1;
            for (int k = 0; k < NR; ++k) if (w >= st0[k] && w < st0[k] + sz[k]) role = k;
            const int k = r % NR, kc = (k + 1) % NR;
            if (role == k) {
                const int GP = 1024 / sz[k], i = w - st0[k];
                if (t < GP) g_put(g + i * GP + t, (uint32_t)(i * GP + t + r), tag);
            } else if (role == kc) {
                ok = wait_n<4, 1, 1>(g + 4 * t, tag, u, err);
            } else {
                u[0] = u[1] = 0;
            }
        } else if constexpr (V == 7) {
            if (t < 2) g_put(g + w * 2 + t, (uint32_t)(w * 2 + t + r), tag);
            ok = wait_n<2, 1, 1>(g + 2 * t, tag, u, err);
        }
        if (!ok) break;
        acc += __uint_as_float(u[0] & 0x3fffffff) + __uint_as_float(u[1] & 0x3fffffff);
    }
    if (acc == 1234.5f) sink[w * 256 + t] = acc;
}

template <int V>
static double run(uint64_t *buf, unsigned *err, float *sink, int rounds, unsigned &tag0) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_edge<V>), hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    hipLaunchKernelGGL(k_edge<V>, dim3(256), dim3(256), 96 * 1024, 0, buf, err, 50, tag0, sink);   // warm
    tag0 += 50;
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(k_edge<V>, dim3(256), dim3(256), 96 * 1024, 0, buf, err, rounds, tag0, sink);
    tag0 += rounds;
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    unsigned e = 0;
    CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    if (e) { printf("variant %d: a wait gave up\n", V); exit(1); }
    return ms * 1e3 / rounds;
}

int main(int argc, char **argv) {
    int rounds = argc > 1 ? atoi(argv[1]) : 2000;
    uint64_t *buf;
    unsigned *err;
    float *sink;
    CK(hipMalloc(&buf, 5 * 8192 * 8));
    CK(hipMemset(buf, 0, 5 * 8192 * 8));
    CK(hipMalloc(&err, 256));
    CK(hipMemset(err, 0, 256));
    CK(hipMalloc(&sink, 256 * 256 * 4));
    unsigned tag0 = 1;
    for (int rep = 0; rep < 2; ++rep) {
        printf("v0 current (256 prod x4, poll 4, sleep1): %.3f us/round\n", run<0>(buf, err, sink, rounds, tag0));
        printf("v1 pipelined polls:                       %.3f us/round\n", run<1>(buf, err, sink, rounds, tag0));
        printf("v2 64 producers x 16 (whole lines):       %.3f us/round\n", run<2>(buf, err, sink, rounds, tag0));
        printf("v3 8 producers x 128:                     %.3f us/round\n", run<3>(buf, err, sink, rounds, tag0));
        printf("v4 one polling wave (16/lane):            %.3f us/round\n", run<4>(buf, err, sink, rounds, tag0));
        printf("v5 no sleep:                              %.3f us/round\n", run<5>(buf, err, sink, rounds, tag0));
        printf("v6 per-producer lines (32 KB sweep):      %.3f us/round\n", run<6>(buf, err, sink, rounds, tag0));
        printf("v7 256 prod x2, poll 2:                   %.3f us/round\n", run<7>(buf, err, sink, rounds, tag0));
        printf("v9 role chain 64/8/32/64/64:             %.3f us/round\n", run<9>(buf, err, sink, rounds, tag0));
        printf("P=128 x 8:                                %.3f us/round\n", run<228>(buf, err, sink, rounds, tag0));
        printf("P=64 x 16:                                %.3f us/round\n", run<164>(buf, err, sink, rounds, tag0));
        printf("P=32 x 32:                                %.3f us/round\n", run<132>(buf, err, sink, rounds, tag0));
        printf("P=16 x 64:                                %.3f us/round\n", run<116>(buf, err, sink, rounds, tag0));
        printf("P=8 x 128:                                %.3f us/round\n", run<108>(buf, err, sink, rounds, tag0));
    }
    return 0;
}
