// Latency of the fp64 bias-correction pows the Adam / CQL-loss kernels compute
// (1 - beta^t in double, as torch does in Python floats): one workgroup, one
// lane computes `n` dependent-free pows; timed with HIP events over many
// launches against the same kernel with n = 0.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

__global__ void powk(const long long* step, double* out, int n) {
  if (threadIdx.x != 0) return;
  const long long t = *step + 1;
  double acc = 0.0;
  for (int i = 0; i < n; ++i) acc += 1.0 - pow(i & 1 ? 0.999 : 0.9, (double)(t + i));
  out[0] = acc;
}

int main() {
  long long* step;
  double* out;
  hipMalloc(&step, 8);
  hipMalloc(&out, 8);
  hipMemset(step, 0, 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int n : {0, 1, 2, 4, 8}) {
    for (int i = 0; i < 100; ++i) powk<<<1, 64>>>(step, out, n);
    hipEventRecord(e0);
    const int reps = 2000;
    for (int i = 0; i < reps; ++i) powk<<<1, 64>>>(step, out, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("{\"pows\": %d, \"us_per_launch\": %.3f}\n", n, 1000.f * ms / reps);
  }
  return 0;
}
