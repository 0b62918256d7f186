// dev microbenchmark of single decode-path kernels (links the in-tree libq3t.so; runs on one MI355X).
// Each case is captured into a hipGraph of `reps` back-to-back launches over rotating weight copies (so the
// weights stream from HBM like the 28-layer talker, not from the 256 MB Infinity Cache) and timed with events.
// Build: make -C tools/dev kbench    Run: tools/dev/_build/kbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "kernels.h"
#include "select.h"

using namespace q3t;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static hipStream_t st;

template <class T>
T *dev(size_t n, float fill = 0.01f) {
    T *p = nullptr;
    CK(hipMalloc(&p, n * sizeof(T)));
    std::vector<T> h(n);
    uint32_t z = 12345;
    for (size_t i = 0; i < n; ++i) {
        z = z * 1664525u + 1013904223u;
        const float v = ((z >> 9) * (1.0f / 8388608.0f) - 0.5f) * 2.0f * fill;
        if constexpr (sizeof(T) == 2) {
            _Float16 hv = (_Float16)v;
            h[i] = *reinterpret_cast<T *>(&hv);
        } else if constexpr (std::is_same<T, float>::value) {
            h[i] = v + (fill == 0.0f ? 0.0f : 0.0f);
        } else {
            h[i] = (T)(z % 7);
        }
    }
    CK(hipMemcpy(p, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
    return p;
}

// time `reps` launches of fn(i) captured in one graph; returns us per launch
static double time_graph(int reps, const std::function<bool(int)> &fn, int iters = 20) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < reps; ++i)
        if (!fn(i)) { printf("launch failed: %s\n", last_error().c_str()); exit(1); }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, st));
    for (int i = 0; i < iters; ++i) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    return ms * 1e3 / (iters * reps);
}

__global__ void k_empty(int *p) { if (p && threadIdx.x == 12345) p[0] = 1; }

// piecewise s_memtime profile of the sampling path (thread 0 records)
__global__ void __launch_bounds__(256) k_sel_prof(const float *lg, int n, float T, int topk, long long *out) {
    __shared__ SelLds S;
    const int vpt = (n + 255) / 256;
    long long ts[8];
    ts[0] = __builtin_amdgcn_s_memtime();
    float v[SEL_VPT_MAX];
    sel_load<false>(lg, n, vpt, v);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    ts[1] = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) v[e] = v[e] / T;
    ts[2] = __builtin_amdgcn_s_memtime();
    float thr = -INFINITY;
    float vmx; if (topk > 0) thr = sel_kth_largest_range(v, n, vpt, topk, &vmx, S);
    ts[3] = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) if (v[e] < thr) v[e] = -INFINITY;
    float m = -INFINITY;
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) if (e < vpt) m = fmaxf(m, v[e]);
    m = sel_block_max(m, S);
    ts[4] = __builtin_amdgcn_s_memtime();
    float loc = 0.0f;
#pragma unroll
    for (int e = 0; e < SEL_VPT_MAX; ++e) { v[e] = e < vpt ? expf(v[e] - m) : 0.0f; loc += v[e]; }
    ts[5] = __builtin_amdgcn_s_memtime();
    unsigned tot;
    const unsigned pre = sel_scan_u((unsigned)(loc * 1000.0f), &tot, S);
    ts[6] = __builtin_amdgcn_s_memtime();
    const int r = sel_argmax(v, n, vpt, S);
    ts[7] = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        for (int i = 0; i < 8; ++i) out[i] = ts[i];
        out[8] = r + pre;
    }
}

int main(int argc, char **argv) {
    CK(hipSetDevice(0));
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int H = 1024, QKV = 4096, I = 3072, NC = 28;
    if (argc > 1 && std::string(argv[1]) == "attn_seq") {
        // ---- batched decode attention (k_attn_seq: one workgroup per (slot, kv head)), 8 rotating cache copies:
        // fixed cost (prologue, wave merge) vs per-chunk cost from a sweep over positions and slot counts
        const int n_ctx = 1024, NCA = 8;
        for (int S : {16, 32, 64}) {
            float *qkv = dev<float>((size_t)S * QKV, 1.0f), *qn = dev<float>(128, 1.0f), *kn = dev<float>(128, 1.0f);
            float *rope = dev<float>((size_t)n_ctx * 128, 1.0f);
            int *pos = dev<int>(S);
            const size_t kvl = (size_t)S * 8 * n_ctx * 128;
            uint16_t *kc = dev<uint16_t>(kvl * NCA, 0.5f), *vc = dev<uint16_t>(kvl * NCA, 0.5f);
            uint16_t *ao = dev<uint16_t>((size_t)S * 2048, 0.0f);
            for (int P : {0, 63, 127, 266, 511, 1000}) {
                std::vector<int> pv(S, P);
                CK(hipMemcpy(pos, pv.data(), S * 4, hipMemcpyHostToDevice));
                const double us = time_graph(NCA, [&](int i) {
                    AttnParams a;
                    a.qkv = qkv; a.qn = qn; a.kn = kn; a.eps = 1e-6f; a.rope = rope; a.pos = pos;
                    a.kc = kc + (i % NCA) * kvl; a.vc = vc + (i % NCA) * kvl;
                    a.n_ctx = n_ctx; a.S = S; a.nH = 16; a.nKV = 8; a.D = 128; a.max_splits = 1; a.seqk = true; a.out = ao;
                    return attn_decode(a, st);
                });
                const double mb = (double)S * (P + 1) * 8 * 128 * 2 * 2 / 1e6;
                printf("attn_seq S %2d pos %4d: %7.2f us  KV %6.2f MB  %6.0f GB/s\n", S, P, us, mb, mb / us * 1e3);
            }
            hipFree(qkv); hipFree(qn); hipFree(kn); hipFree(rope); hipFree(pos); hipFree(kc); hipFree(vc); hipFree(ao);
        }
        return 0;
    }
    // ---- launch floor
    for (int blocks : {256, 512, 1024}) {
        const double us = time_graph(100, [&](int) { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, st, nullptr); return true; });
        printf("empty kernel %4d blocks: %.2f us/launch\n", blocks, us);
    }
    // ---- GEMV shapes of one decoder layer, 28 rotating weight copies (887 MB-like streaming)
    float *x = dev<float>((size_t)8 * 4096, 1.0f), *nw = dev<float>(4096, 1.0f);
    float *out = dev<float>((size_t)8 * 8192, 0.0f), *resid = dev<float>((size_t)8 * 4096, 1.0f);
    uint16_t *xh = dev<uint16_t>((size_t)8 * 4096, 1.0f), *oh = dev<uint16_t>((size_t)8 * 8192, 0.0f);
    struct Shape { const char *name; int N, K, pro, act; };
    const Shape shapes[] = {{"qkv  N4096 K1024 RMS", QKV, H, PRO_RMS, ACT_NONE},
                            {"gu   N6144 K1024 RMS+SwiGLU", 2 * I, H, PRO_RMS, ACT_SWIGLU},
                            {"o    N1024 K2048 F16+res", H, 2048, PRO_F16, ACT_NONE},
                            {"down N1024 K3072 F16+res", H, I, PRO_F16, ACT_NONE},
                            {"head N2048 K1024 RMS", 2048, H, PRO_RMS, ACT_NONE}};
    std::vector<int> mbs = {256, 512, 1024};
    for (const Shape &sh : shapes) {
        std::vector<uint16_t *> W(NC);
        for (int c = 0; c < NC; ++c) W[c] = dev<uint16_t>((size_t)sh.N * sh.K, 0.05f);
        for (int B : {1, 2, 8}) {
            for (int mb : mbs) {
                gemv_set_min_blocks(mb);
                const double us = time_graph(NC, [&](int i) {
                    GemvParams p;
                    p.W = W[i % NC]; p.N = sh.N; p.K = sh.K; p.B = B; p.pro = sh.pro; p.act = sh.act;
                    p.nw = nw; p.eps = 1e-6f;
                    if (sh.pro == PRO_F16) { p.x = xh; p.ldx = sh.K; p.resid = resid; p.ldr = sh.N; }
                    else { p.x = x; p.ldx = sh.K; }
                    if (sh.act == ACT_SWIGLU) { p.out_f16 = oh; p.ldo = sh.N / 2; }
                    else { p.out_f32 = out; p.ldo = sh.N; }
                    return gemv(p, st);
                });
                const double gbs = (double)sh.N * sh.K * 2 / (us * 1e-6) / 1e9;
                printf("gemv %-28s B=%d min_blocks %4d: %6.2f us  %7.0f GB/s\n", sh.name, B, mb, us, gbs);
            }
        }
        for (auto *w : W) hipFree(w);
    }
    gemv_set_min_blocks(512);
    // ---- decode attention (talker layout, 28 layers of cache)
    {
        const int n_ctx = 4200, S = 1;
        float *qkv = dev<float>((size_t)S * QKV, 1.0f), *qn = dev<float>(128, 1.0f), *kn = dev<float>(128, 1.0f);
        float *rope = dev<float>((size_t)n_ctx * 128, 1.0f);
        const int max_splits = (n_ctx + ATTN_CHUNK - 1) / ATTN_CHUNK;
        float *part = dev<float>((size_t)S * 16 * max_splits * 130, 0.0f);
        unsigned *ticket = dev<unsigned>((size_t)S * 8);
        CK(hipMemset(ticket, 0, S * 8 * 4));
        std::vector<int> pv(S);
        int *pos = dev<int>(S);
        const size_t kvl = (size_t)S * 8 * n_ctx * 128;
        uint16_t *kc = dev<uint16_t>(kvl * NC, 0.5f), *vc = dev<uint16_t>(kvl * NC, 0.5f);
        uint16_t *ao = dev<uint16_t>((size_t)S * 2048, 0.0f);
        for (int P : {16, 63, 64, 100, 266, 600, 1500, 4100}) {
            for (int s = 0; s < S; ++s) pv[s] = P;
            CK(hipMemcpy(pos, pv.data(), S * 4, hipMemcpyHostToDevice));
            const double us = time_graph(NC, [&](int i) {
                AttnParams a;
                a.qkv = qkv; a.qn = qn; a.kn = kn; a.eps = 1e-6f; a.rope = rope; a.pos = pos;
                a.kc = kc + (i % NC) * kvl; a.vc = vc + (i % NC) * kvl;
                a.n_ctx = n_ctx; a.S = S; a.nH = 16; a.nKV = 8; a.D = 128; a.max_splits = max_splits; a.part = part; a.ticket = ticket; a.out = ao;
                return attn_decode(a, st);
            });
            printf("attn_decode pos %5d: %6.2f us/layer (KV %.2f MB)\n", P, us, (double)(P + 1) * 8 * 128 * 2 * 2 / 1e6);
        }
    }
    // ---- selection kernels
    {
        const int S = 1;
        float *lg = dev<float>((size_t)S * 3072, 4.0f);
        int *tokens = dev<int>((size_t)S * 16), *frame = dev<int>(S), *done = dev<int>(S);
        CK(hipMemset(done, 0xff, S * 4));
        int32_t *codes = dev<int32_t>((size_t)S * 64 * 16);
        uint64_t *utt = dev<uint64_t>(S);
        uint8_t *seen = dev<uint8_t>((size_t)S * 3072);
        CK(hipMemset(seen, 0, 3072));
        int *ntok = dev<int>(S), *force = dev<int>(S);
        for (int mode : {SEL_CP, SEL_CB0}) {
            for (int variant = 0; variant < 3; ++variant) {
                const float T = variant == 0 ? 0.0f : 0.9f;
                const int topk = variant == 2 ? 0 : 50;
                SelectSpec sp;
                sp.mode = mode; sp.V = mode == SEL_CP ? 2048 : 3072; sp.tokens = tokens; sp.codes = codes; sp.max_len = 64;
                sp.frame = frame; sp.done = done; sp.temperature = T; sp.top_k = topk; sp.seed = 1; sp.utt = utt;
                sp.seen = seen; sp.n_tokens = ntok; sp.force_frames = force;
                const double us = time_graph(15, [&](int i) { sp.step = i % 15; return select_tokens(sp, lg, S, st); });
                printf("select %s T=%.1f top_k=%d: %.2f us\n", mode == SEL_CP ? "cp " : "cb0", T, topk, us);
            }
        }
    }
    {
        float *lg = dev<float>(4096, 4.0f);
        long long *o = dev<long long>(16);
        std::vector<long long> h(16);
        for (int n : {2048, 3072})
            for (int topk : {0, 50}) {
                for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k_sel_prof, dim3(1), dim3(256), 0, st, lg, n, 0.9f, topk, o);
                CK(hipStreamSynchronize(st));
                CK(hipMemcpy(h.data(), o, 16 * 8, hipMemcpyDeviceToHost));
                printf("sel_prof n=%d topk=%d (s_memtime ticks): load %lld div %lld kth %lld max %lld exp %lld scan %lld argmax %lld\n", n, topk,
                       h[1] - h[0], h[2] - h[1], h[3] - h[2], h[4] - h[3], h[5] - h[4], h[6] - h[5], h[7] - h[6]);
            }
    }
    printf("done\n");
    return 0;
}
