// probe: is __builtin_amdgcn_fdot2 (v_dot2_f32_f16) exact (exact f16 products, f32 sums)?
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__global__ void k(const __half* a, const __half* b, float* o1, float* o2, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x; if (i >= n) return;
  h2 x = {(_Float16)a[2*i], (_Float16)a[2*i+1]}, y = {(_Float16)b[2*i], (_Float16)b[2*i+1]};
  float c = 1.0f / 3.0f;
  o1[i] = __builtin_amdgcn_fdot2(x, y, c, false);
  o2[i] = fmaf(__half2float(a[2*i+1]), __half2float(b[2*i+1]), fmaf(__half2float(a[2*i]), __half2float(b[2*i]), c));
}
int main() {
  const int n = 1 << 20;
  __half *a, *b; float *o1, *o2;
  hipMallocManaged(&a, 2*n*2); hipMallocManaged(&b, 2*n*2); hipMallocManaged(&o1, n*4); hipMallocManaged(&o2, n*4);
  srand(1);
  for (int i = 0; i < 2*n; ++i) { a[i] = __float2half((rand()/(float)RAND_MAX - 0.5f) * 4); b[i] = __float2half((rand()/(float)RAND_MAX - 0.5f) * 4); }
  k<<<n/256, 256>>>(a, b, o1, o2, n); hipDeviceSynchronize();
  double mx = 0; int neq = 0;
  for (int i = 0; i < n; ++i) { double d = fabs((double)o1[i] - o2[i]) / (fabs(o2[i]) + 1e-3); if (d > mx) mx = d; neq += o1[i] != o2[i]; }
  printf("fdot2 vs fma chain: max rel diff %.3e, differing %d / %d\n", mx, neq, n);
  return 0;
}
