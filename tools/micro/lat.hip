// Latency microbenchmark (diagnostic): one wave, dependent chains of LDS / global / readlane / ballot ops,
// timed with s_memtime. Prints cycles per op.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define N 1024
__global__ void lat(const int* g, long* out, int* sink) {
  __shared__ int s[N];
  __shared__ long sl[N];
  const int lane = threadIdx.x;
  for (int i = lane; i < N; i += 64) { s[i] = (i * 17 + 5) & (N - 1); sl[i] = i * 3; }
  __syncthreads();
  int p = lane & 1;
  long t0, t1;
  // 1. LDS dependent chain
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) p = s[p];
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = (t1 - t0);
  // 2. global dependent chain (small array -> L2/L1 hits)
  int q = lane & 1;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) q = g[q];
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[1] = (t1 - t0);
  // 3. uniform LDS chain read into scalar (readfirstlane)
  int u = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) u = __builtin_amdgcn_readfirstlane(s[u]);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[2] = (t1 - t0);
  // 4. ballot + ctz chain over LDS data (probe-like)
  int j = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) {
    const uint64_t b = __ballot(sl[(j + lane) & (N - 1)] >= (long)(j * 3 + 7));
    j = (j + (b ? __builtin_ctzll(b) : 1)) & 511;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[3] = (t1 - t0);
  // 5. readlane chain
  int r = lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) r = __builtin_amdgcn_readlane(r + lane, (r & 63));
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[4] = (t1 - t0);
  // 6. s_memtime back to back
  t0 = __builtin_amdgcn_s_memtime();
  long acc = 0;
  for (int i = 0; i < 256; i++) acc += __builtin_amdgcn_s_memtime();
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[5] = (t1 - t0);
  // 7. barrier cost (one wave only here)
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) __syncthreads();
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[6] = (t1 - t0);
  sink[lane] = p + q + u + j + r + (int)acc;
}
// barrier cost with 8 waves
__global__ void bar8(long* out) {
  long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) __syncthreads();
  long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[7] = t1 - t0;
}
int main() {
  int *g, *sink; long* out;
  hipMalloc(&g, 4096 * 4); hipMalloc(&sink, 256 * 4); hipMalloc(&out, 16 * 8);
  int h[4096];
  for (int i = 0; i < 4096; i++) h[i] = (i * 17 + 5) & 1023;
  hipMemcpy(g, h, sizeof h, hipMemcpyHostToDevice);
  for (int it = 0; it < 3; it++) {
    hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, g, out, sink);
    hipLaunchKernelGGL(bar8, dim3(1), dim3(512), 0, 0, out);
    hipDeviceSynchronize();
  }
  long o[16];
  hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost);
  const char* names[] = {"lds_chain", "global_chain", "lds_uniform_readfirstlane", "ballot_probe_lds", "readlane_chain",
                         "s_memtime", "barrier_1wave", "barrier_8waves"};
  for (int i = 0; i < 8; i++) printf("%-28s %8.1f cycles/op\n", names[i], o[i] / 256.0);
  return 0;
}
