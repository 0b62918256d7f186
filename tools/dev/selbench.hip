// dev microbenchmark: token selection (select.h sel_sample: /T, top-k threshold, exp, inverse CDF) on one 256-thread
// workgroup, R selections back to back inside one launch, over 64 logits rows of different shapes (normal, heavy
// outliers, quantised ties, masked -inf ranges) with and without a kept id.  Prints the time per selection and writes
// every token to OUT (binary) so that two builds can be compared token for token:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../qwen3-tts-jetson_amd/csrc [-DQ3T_SEL_GENERAL] selbench.hip
//   selbench V OUT
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
__device__ long long g_stamp[32];
__device__ int g_stamp_on;
#define SEL_STAMP(k) do { if (g_stamp_on && threadIdx.x == 0) g_stamp[k] = wall_clock64(); } while (0)
#include "select.h"
using namespace q3t;

constexpr int NROW = 64;

template <int VPT>
__global__ void __launch_bounds__(256) k_sel(const float *lg, int V, int R, int topk, long long *clk, int *out, int kind, int stamp_r) {
    __shared__ SelLds S;
    const int t = threadIdx.x;
    long long t0 = wall_clock64();
    for (int r = 0; r < R; ++r) {
        float v[SEL_VPT_MAX];
        const float *row = lg + (size_t)(kind < 0 ? r % NROW : (r % 8) * 8 + (kind & 7)) * V;
#pragma unroll
        for (int e = 0; e < SEL_VPT_MAX; ++e) v[e] = e < VPT ? row[t * VPT + e] : -INFINITY;
        const float u = uniform24(1, 0, (uint64_t)r, 3);
        const float T = (r & 4) ? 0.9f : 0.7f;
        const int keep = (r % 3 == 0) ? V - 1 - (r % 7) * 131 : -1;
        if (t == 0) g_stamp_on = r == (stamp_r < 0 ? R - 1 : stamp_r);
        __syncthreads();
        SEL_STAMP(0);
        const int tok = kind == 99 ? (int)(v[0] + v[VPT - 1]) : sel_sample(v, V, VPT, T, topk, u, keep, S);   // 99: loop floor
        SEL_STAMP(17);
        if (t == 0) out[r] = tok;
    }
    long long t1 = wall_clock64();
    if (t == 0) clk[0] = t1 - t0;
}

int main(int argc, char **argv) {
    const int V = argc > 1 ? atoi(argv[1]) : 2048;
    const char *outp = argc > 2 && argv[2][0] != '-' ? argv[2] : nullptr;
    const int kind = argc > 3 ? atoi(argv[3]) : -1;
    const int stamp_r = argc > 4 ? atoi(argv[4]) : -1;   // selection whose stages are stamped (0: cold caches)
    const int R = 4096;
    std::vector<float> h((size_t)NROW * V);
    uint32_t z = 7;
    auto rnd = [&]() { z = z * 1664525u + 1013904223u; return (z >> 8) * (1.0f / 16777216.0f); };
    for (int r = 0; r < NROW; ++r) {
        float *x = &h[(size_t)r * V];
        for (int i = 0; i < V; ++i) {   // roughly normal, scale 4
            float s = 0;
            for (int k = 0; k < 4; ++k) s += rnd() - 0.5f;
            x[i] = s * 4.0f * 1.7f;
        }
        const int kind = r % 8;
        if (kind == 1) for (int k = 0; k < 3; ++k) x[(int)(rnd() * V)] += 80.0f;            // far outliers
        if (kind == 2) for (int i = 0; i < V; ++i) x[i] = std::floor(x[i] * 2.0f) * 0.5f;   // ties
        if (kind == 3) for (int i = V - 1024; i < V; ++i) if (i != V - 3) x[i] = -INFINITY; // CB0-like mask
        if (kind == 4) for (int i = 0; i < V; ++i) x[i] = std::floor(x[i] * 0.25f);         // heavy ties
        if (kind == 5) for (int i = 0; i < V; ++i) x[i] *= 0.05f;                          // flat
        if (kind == 6) { for (int i = 0; i < V; ++i) x[i] = -INFINITY; for (int k = 0; k < 30; ++k) x[(int)(rnd() * V)] = rnd(); }  // < k finite
        if (kind == 7) x[5] = 1e30f;                                                      // huge range
    }
    float *d; long long *clk; int *o;
    (void)hipMalloc(&d, h.size() * 4); (void)hipMalloc(&clk, 64); (void)hipMalloc(&o, R * 4);
    (void)hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    std::vector<int> tok(R);
    for (int rep = 0; rep < 2; ++rep) {
        if (V == 2048) hipLaunchKernelGGL(k_sel<8>, dim3(1), dim3(256), 0, 0, d, V, R, 50, clk, o, kind, stamp_r);
        else hipLaunchKernelGGL(k_sel<12>, dim3(1), dim3(256), 0, 0, d, V, R, 50, clk, o, kind, stamp_r);
        long long c;
        (void)hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(tok.data(), o, R * 4, hipMemcpyDeviceToHost);
        printf("V=%d kind %d top-50: %.3f us per selection (wall clock 100 MHz)\n", V, kind, c / 100.0 / R);
        long long sv[32];
        (void)hipMemcpyFromSymbol(sv, HIP_SYMBOL(g_stamp), sizeof sv);
        printf("   last selection, us from start:");
        for (int k = 1; k < 18; ++k) if (sv[k] >= sv[0] && sv[k] - sv[0] < 100000) printf(" [%d] %.2f", k, (sv[k] - sv[0]) / 100.0);
        printf("\n");
        (void)hipMemset(clk, 0, 8);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), std::vector<long long>(32, 0).data(), 256);
    }
    if (outp) {
        FILE *f = fopen(outp, "wb");
        fwrite(tok.data(), 4, R, f);
        fclose(f);
    }
    return 0;
}
