// dev probe: which workgroups of a 2-per-CU persistent grid share a CU (HW_ID + XCC_ID per workgroup).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
__global__ void __launch_bounds__(256, 2) k_probe(unsigned *out, int lds_words) {
    extern __shared__ unsigned lds[];
    if (threadIdx.x == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        out[blockIdx.x * 2] = hw;
        out[blockIdx.x * 2 + 1] = xcc;
        lds[0] = hw;
    }
    // stay resident for a while so the whole grid is co-resident
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < 20000) __builtin_amdgcn_s_sleep(10);
    if (threadIdx.x == 1 && lds[0] == 12345) out[0] = 0;
}
int main() {
    const int n = 512;
    unsigned *d;
    hipMalloc(&d, n * 8);
    hipFuncSetAttribute((const void *)k_probe, hipFuncAttributeMaxDynamicSharedMemorySize, 70 * 1024);
    hipLaunchKernelGGL(k_probe, dim3(n), dim3(256), 70 * 1024, 0, d, 0);
    std::vector<unsigned> h(n * 2);
    hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost);
    std::map<unsigned, std::vector<int>> cu;
    for (int b = 0; b < n; ++b) {
        const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
        const unsigned key = (xcc << 16) | (hw & 0xff00) | ((hw >> 13) & 7) << 4 | ((hw >> 12) & 1);   // xcc, cu, se, sh
        cu[key].push_back(b);
    }
    printf("distinct CUs: %zu\n", cu.size());
    int shown = 0, same256 = 0, pairs = 0;
    for (auto &kv : cu) {
        if (kv.second.size() == 2) { ++pairs; if (kv.second[1] - kv.second[0] == 256) ++same256; }
        if (shown < 24) { printf("cu %08x:", kv.first); for (int b : kv.second) printf(" %d", b); printf("\n"); ++shown; }
    }
    printf("pairs %d, pairs (b, b+256): %d\n", pairs, same256);
    for (int b = 0; b < 16; ++b) printf("wg %d hw %08x xcc %u\n", b, h[2 * b], h[2 * b + 1]);
    return 0;
}
