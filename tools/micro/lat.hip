// Latency microbenchmark (diagnostic): one wave, dependent chains of LDS / global / readlane / ballot ops,
// timed with s_memtime. Prints cycles per op.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define N 1024
__global__ void lat(const int* g, long* out, int* sink, int* wsink) {
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
  // 8. dependent global load chain where each step first stores 4 words (other lines): load-after-store wait
  int q2 = lane & 1;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) {
    wsink[(i & 15) * 256 + lane] = q2;
    wsink[4096 + (i & 15) * 256 + lane] = q2;
    wsink[8192 + (i & 15) * 256 + lane] = q2;
    wsink[12288 + (i & 15) * 256 + lane] = q2;
    q2 = g[q2];
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[8] = (t1 - t0);
  // 9. same chain, stores replaced by LDS stores
  int q3 = lane & 1;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) {
    s[(i & 7) * 64 + lane] = q3;
    q3 = g[q3];
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[9] = (t1 - t0);
  // 10. one-lane global store then dependent load chain (lane 0 stores only)
  int q4 = lane & 1;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) {
    if (lane == 0) wsink[(i & 15) * 16] = q4;
    q4 = g[q4];
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[10] = (t1 - t0);
  sink[lane] = p + q + u + j + r + (int)acc + q2 + q3 + q4;
}
// barrier cost with 8 waves
__global__ void bar8(long* out) {
  long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) __syncthreads();
  long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[7] = t1 - t0;
}
int main() {
  int *g, *sink, *wsink; long* out;
  hipMalloc(&g, 4096 * 4); hipMalloc(&sink, 256 * 4); hipMalloc(&out, 16 * 8);
  hipMalloc(&wsink, 16384 * 4);
  hipMemset(out, 0, 16 * 8);
  int h[4096];
  for (int i = 0; i < 4096; i++) h[i] = (i * 17 + 5) & 1023;
  hipMemcpy(g, h, sizeof h, hipMemcpyHostToDevice);
  for (int it = 0; it < 3; it++) {
    hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, g, out, sink, wsink);
    hipLaunchKernelGGL(bar8, dim3(1), dim3(512), 0, 0, out);
    hipDeviceSynchronize();
  }
  long o[16];
  hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost);
  const char* names[] = {"lds_chain", "global_chain", "lds_uniform_readfirstlane", "ballot_probe_lds", "readlane_chain",
                         "s_memtime", "barrier_1wave", "barrier_8waves", "global_chain_after_4_stores",
                         "global_chain_after_lds_store", "global_chain_after_lane0_store"};
  for (int i = 0; i < 11; i++) printf("%-28s %8.1f cycles/op\n", names[i], o[i] / 256.0);
  return 0;
}
