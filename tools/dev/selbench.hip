// dev microbenchmark: the code-predictor token selection (select.h, SEL_CP: /T, top-50 threshold, exp, inverse CDF)
// on one 256-thread workgroup, R selections back to back inside one launch; s_memtime stamps between the stages of the
// first few selections (thread 0).  Build: hipcc --offload-arch=gfx950 -O3 -I../../qwen3-tts-jetson_amd/csrc selbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
__device__ long long g_stamp[16];
__device__ int g_stamp_on;
#define SEL_STAMP(k) do { if (g_stamp_on && threadIdx.x == 0) g_stamp[k] = wall_clock64(); } while (0)
#include "select.h"
using namespace q3t;

__global__ void __launch_bounds__(256) k_sel(const float *lg, int R, float T, int topk, long long *stamps, int *out) {
    __shared__ SelLds S;
    const int t = threadIdx.x;
    long long t0 = wall_clock64();
    int acc = 0;
    for (int r = 0; r < R; ++r) {
        float v[SEL_VPT_MAX];
#pragma unroll
        for (int e = 0; e < SEL_VPT_MAX; ++e) v[e] = e < 8 ? lg[(r & 15) * 2048 + t * 8 + e] : -INFINITY;
        const float u = uniform24(1, 0, (uint64_t)r, 3);
        if (t == 0) { g_stamp_on = r == R - 1; if (r == R - 1) g_stamp[0] = wall_clock64(); }
        __syncthreads();
        const int tok = sel_sample(v, 2048, 8, T, topk, u, -1, S);
        if (t == 0 && r == R - 1) g_stamp[9] = wall_clock64();
        acc += tok;
    }
    long long t1 = wall_clock64();
    if (t == 0) { stamps[0] = t1 - t0; out[0] = acc; }
}

int main(int argc, char **argv) {
    const int R = 2000;
    std::vector<float> h(16 * 2048);
    uint32_t z = 7;
    for (auto &x : h) {   // roughly normal logits, scale 4
        float s = 0;
        for (int k = 0; k < 4; ++k) { z = z * 1664525u + 1013904223u; s += (z >> 8) * (1.0f / 16777216.0f) - 0.5f; }
        x = s * 4.0f * 1.7f;
    }
    float *d; long long *st; int *o;
    hipMalloc(&d, h.size() * 4); hipMalloc(&st, 64); hipMalloc(&o, 64);
    hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep)
        for (float T : {0.9f}) {
            hipLaunchKernelGGL(k_sel, dim3(1), dim3(256), 0, 0, d, R, T, 50, st, o);
            long long c; hipMemcpy(&c, st, 8, hipMemcpyDeviceToHost);
            printf("T=%.1f top-50: %.3f us per selection (wall clock 100 MHz)\n", T, c / 100.0 / R);
            long long sv[16];
            hipMemcpyFromSymbol(sv, HIP_SYMBOL(g_stamp), sizeof sv);
            printf("   stages (us from start): minmax %.2f hist %.2f bin %.2f cand %.2f rank %.2f exp %.2f scan %.2f pick %.2f end %.2f\n",
                   (sv[1] - sv[0]) / 100.0, (sv[2] - sv[0]) / 100.0, (sv[3] - sv[0]) / 100.0, (sv[4] - sv[0]) / 100.0,
                   (sv[5] - sv[0]) / 100.0, (sv[6] - sv[0]) / 100.0, (sv[7] - sv[0]) / 100.0, (sv[8] - sv[0]) / 100.0, (sv[9] - sv[0]) / 100.0);
        }
    return 0;
}
