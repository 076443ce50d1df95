// Issue-cost microbenchmark (diagnostic): one wave alone; cycles per instruction for SALU, VALU, v_readlane /
// v_writelane pairs, taken scalar branches, and s_memtime. Timed with s_memtime over 256-iteration loops.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void issue(long* out, int* sink) {
  long t0, t1;
  int x = threadIdx.x;
  // 1. 16 dependent SALU adds per iteration
  t0 = __builtin_amdgcn_s_memtime();
  int s = 1;
  for (int i = 0; i < 256; i++) {
    asm volatile(
        "s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n"
        "s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n"
        "s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n"
        "s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n"
        : "+s"(s)
        :
        : "scc");
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  // 2. 16 independent VALU adds per iteration
  int v0 = x, v1 = x + 1, v2 = x + 2, v3 = x + 3;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) {
    asm volatile(
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
        : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[1] = t1 - t0;
  // 3. 8 v_writelane + 8 v_readlane per iteration (SGPR spill / reload pattern)
  int w = 0, r0 = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) {
    asm volatile(
        "v_writelane_b32 %0, %1, 0\n v_writelane_b32 %0, %1, 1\n v_writelane_b32 %0, %1, 2\n v_writelane_b32 %0, %1, 3\n"
        "v_writelane_b32 %0, %1, 4\n v_writelane_b32 %0, %1, 5\n v_writelane_b32 %0, %1, 6\n v_writelane_b32 %0, %1, 7\n"
        "s_nop 4\n"
        "v_readlane_b32 %1, %0, 0\n v_readlane_b32 %1, %0, 1\n v_readlane_b32 %1, %0, 2\n v_readlane_b32 %1, %0, 3\n"
        "v_readlane_b32 %1, %0, 4\n v_readlane_b32 %1, %0, 5\n v_readlane_b32 %1, %0, 6\n v_readlane_b32 %1, %0, 7\n"
        : "+v"(w), "+s"(r0)
        :
        : "scc");
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[2] = t1 - t0;
  // 4. 8 taken unconditional scalar branches per iteration
  int c = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) {
    asm volatile(
        "s_branch 1f\n 1:\n s_branch 2f\n 2:\n s_branch 3f\n 3:\n s_branch 4f\n 4:\n"
        "s_branch 5f\n 5:\n s_branch 6f\n 6:\n s_branch 7f\n 7:\n s_branch 8f\n 8:\n"
        "s_add_u32 %0, %0, 1\n"
        : "+s"(c)
        :
        : "scc");
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[3] = t1 - t0;
  // 5. 4 taken conditional branches, each over 8 s_nop, per iteration
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) {
    asm volatile(
        "s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 1f\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n 1:\n"
        "s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 2f\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n 2:\n"
        "s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 3f\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n 3:\n"
        "s_cmp_eq_u32 %0, %0\n s_cbranch_scc1 4f\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n 4:\n"
        "s_add_u32 %0, %0, 1\n"
        : "+s"(c)
        :
        : "scc");
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[4] = t1 - t0;
  // 6. s_memtime back to back with the wait for each
  t0 = __builtin_amdgcn_s_memtime();
  long acc = 0;
  for (int i = 0; i < 256; i++) acc += __builtin_amdgcn_s_memtime();
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[5] = t1 - t0;
  sink[threadIdx.x] = s + v0 + v1 + v2 + v3 + w + r0 + c + (int)acc;
}

int main() {
  long* out;
  int* sink;
  (void)hipMalloc(&out, 16 * sizeof(long));
  (void)hipMalloc(&sink, 64 * sizeof(int));
  for (int it = 0; it < 3; it++) {
    hipLaunchKernelGGL(issue, dim3(1), dim3(64), 0, 0, out, sink);
    (void)hipDeviceSynchronize();
  }
  long o[16];
  (void)hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost);
  const char* names[] = {"salu_dep (per instr)", "valu_indep (per instr)", "writelane+readlane (per instr)",
                         "s_branch taken (per branch)", "s_cbranch_scc1 taken over 8 nops (per branch)",
                         "s_memtime+wait"};
  const double per[] = {256.0 * 16, 256.0 * 16, 256.0 * 16, 256.0 * 8, 256.0 * 4, 256.0};
  for (int i = 0; i < 6; i++) printf("%-48s %8.1f cycles\n", names[i], o[i] / per[i]);
  return 0;
}
