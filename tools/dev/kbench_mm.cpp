// dev microbenchmark of the batched matrix-core GEMM (gemm_mfma.hip) on the decode shapes at B tokens, with the
// debug knobs that drop the activation or the weight loads (GemvParams::dbg) to see which stream bounds a shape.
// Build: make -C tools/dev kbench_mm    Run: tools/dev/_build/kbench_mm [B]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "kernels.h"

using namespace q3t;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
static hipStream_t st;
__global__ void k_empty(int *p) { if (p && threadIdx.x == 999) p[0] = 1; }

template <class T>
T *dev(size_t n, float fill) {
    T *p = nullptr;
    CK(hipMalloc(&p, n * sizeof(T)));
    std::vector<T> h(n);
    uint32_t z = 12345;
    for (size_t i = 0; i < n; ++i) {
        z = z * 1664525u + 1013904223u;
        const float v = ((z >> 9) * (1.0f / 8388608.0f) - 0.5f) * 2.0f * fill;
        if constexpr (sizeof(T) == 2) { _Float16 hv = (_Float16)v; h[i] = *reinterpret_cast<T *>(&hv); }
        else h[i] = v;
    }
    CK(hipMemcpy(p, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
    return p;
}
static double time_graph(int reps, const std::function<bool(int)> &fn, int iters = 20) {
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < reps; ++i) if (!fn(i)) { printf("launch failed: %s\n", last_error().c_str()); exit(1); }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st)); CK(hipStreamSynchronize(st));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a, st));
    for (int i = 0; i < iters; ++i) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st)); CK(hipEventSynchronize(b));
    float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
    hipGraphExecDestroy(ge); hipGraphDestroy(g);
    return ms * 1e3 / (iters * reps);
}

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 64;
    CK(hipSetDevice(0));
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    gemm_mfma_set_min_batch(1);
    const int NC = 28;
    for (int wg : {1, 256, 1024}) {   // floor: an empty kernel per graph node
        const double us = time_graph(NC, [&](int) { hipLaunchKernelGGL(k_empty, dim3(wg), dim3(256), 0, st, nullptr); return true; });
        printf("empty kernel, %4d workgroups: %6.2f us per graph node\n", wg, us);
    }
    float *x = dev<float>((size_t)B * 4096, 1.0f), *nw = dev<float>(4096, 1.0f);
    float *out = dev<float>((size_t)B * 8192, 0.0f), *resid = dev<float>((size_t)B * 4096, 1.0f);
    uint16_t *xh = dev<uint16_t>((size_t)B * 4096, 1.0f), *oh = dev<uint16_t>((size_t)B * 8192, 0.0f);
    float *parts = dev<float>((size_t)4 * B * 8192, 0.0f);
    struct Shape { const char *name; int N, K, pro, act, ks = 0; };
    const Shape shapes[] = {{"qkv  N4096 K1024 RMS", 4096, 1024, PRO_RMS, ACT_NONE},
                            {"gu   N6144 K1024 RMS+SwiGLU", 6144, 1024, PRO_RMS, ACT_SWIGLU},
                            {"o    N1024 K2048 F16+res", 1024, 2048, PRO_F16, ACT_NONE},
                            {"down N1024 K3072 F16+res", 1024, 3072, PRO_F16, ACT_NONE},
                            {"head N2048 K1024 RMS", 2048, 1024, PRO_RMS, ACT_NONE},
                            {"qkv  N4096 K1024 F16", 4096, 1024, PRO_F16, ACT_NONE},
                            {"gu   N6144 K1024 F16+SwiGLU", 6144, 1024, PRO_F16, ACT_SWIGLU},
                            {"qkv  N4096 K1024 F16 split-K 2", 4096, 1024, PRO_F16, ACT_NONE, 2},
                            {"qkv  N4096 K1024 F16 split-K 4", 4096, 1024, PRO_F16, ACT_NONE, 4},
                            {"o    N1024 K2048 F16 split-K 4", 1024, 2048, PRO_F16, ACT_NONE, 4},
                            {"down N1024 K3072 F16 split-K 4", 1024, 3072, PRO_F16, ACT_NONE, 4}};
    for (const Shape &sh : shapes) {
        std::vector<uint16_t *> W(NC);
        for (int c = 0; c < NC; ++c) W[c] = dev<uint16_t>((size_t)sh.N * sh.K, 0.05f);
        for (int dbg : {0, 3}) {
            const double us = time_graph(NC, [&](int i) {
                GemvParams p;
                p.W = W[i % NC]; p.N = sh.N; p.K = sh.K; p.B = B; p.pro = sh.pro; p.act = sh.act; p.dbg = dbg;
                p.nw = nw; p.eps = 1e-6f;
                if (sh.pro == PRO_F16) {
                    p.x = xh; p.ldx = sh.K;
                    if (sh.N == 1024 && !sh.ks) { p.resid = resid; p.ldr = sh.N; p.out_f32 = resid; }
                    if (sh.ks) { p.parts = parts; p.ksplit = sh.ks; }
                }
                else { p.x = x; p.ldx = sh.K; }
                if (sh.act == ACT_SWIGLU) { p.out_f16 = oh; p.ldo = sh.N / 2; }
                else { if (!p.out_f32) p.out_f32 = out; p.ldo = sh.N; }
                return gemv(p, st);
            });
            const double gbs = (double)sh.N * sh.K * 2 / (us * 1e-6) / 1e9;
            printf("mfma %-28s B=%d dbg=%d (%s): %7.2f us  W %6.0f GB/s\n", sh.name, B, dbg,
                   dbg == 0 ? "full" : dbg == 1 ? "no X loads" : dbg == 2 ? "no W loads" : "no loads", us, gbs);
        }
        for (auto *w : W) hipFree(w);
    }
    printf("done\n");
    return 0;
}
