// Back-to-back issue cost of the bf16 MFMA shapes the Q-net could use, one wave per SIMD
// (gfx950): 8 independent accumulators per wave, cycles per instruction from s_memtime
// relative to the 32x32x16 loop (32 cycles, MI355X_MICROARCH.md constants table).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define ACC8(T) T c0{}, c1{}, c2{}, c3{}, c4{}, c5{}, c6{}, c7{}
// the 8 MFMAs of one iteration as one asm block: no compiler register shuffles in the loop
#define STEP8(INS, A, B)                                                                        \
  asm volatile(INS " %0, %8, %9, %0\n" INS " %1, %8, %9, %1\n" INS " %2, %8, %9, %2\n" INS     \
               " %3, %8, %9, %3\n" INS " %4, %8, %9, %4\n" INS " %5, %8, %9, %5\n" INS        \
               " %6, %8, %9, %6\n" INS " %7, %8, %9, %7\n"                                     \
               : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7) \
               : "v"(A), "v"(B));

template <int MODE>
__global__ __launch_bounds__(64) void k(float* out, unsigned long long* cyc, int iters) {
  const int l = threadIdx.x;
  bf16x8 a, b;
  s16x4 a4, b4;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.001f * (l + j)); b[j] = (__bf16)(0.002f * (l - j)); }
  for (int j = 0; j < 4; ++j) { a4[j] = (short)(l + j); b4[j] = (short)(l * 3 + j); }
  float s = 0;
  unsigned long long t0 = 0, t1 = 0;
  if constexpr (MODE == 0) {
    ACC8(f32x16);
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) { STEP8("v_mfma_f32_32x32x16_bf16", a, b) }
    t1 = __builtin_amdgcn_s_memtime();
    s = c0[l & 15] + c1[1] + c2[2] + c3[3] + c4[4] + c5[5] + c6[6] + c7[7];
  } else if constexpr (MODE == 1) {
    ACC8(f32x4);
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) { STEP8("v_mfma_f32_16x16x32_bf16", a, b) }
    t1 = __builtin_amdgcn_s_memtime();
    s = c0[l & 3] + c1[1] + c2[2] + c3[3] + c4[0] + c5[1] + c6[2] + c7[3];
  } else if constexpr (MODE == 2) {
    ACC8(f32x4);
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) { STEP8("v_mfma_f32_16x16x16_bf16", a4, b4) }
    t1 = __builtin_amdgcn_s_memtime();
    s = c0[l & 3] + c1[1] + c2[2] + c3[3] + c4[0] + c5[1] + c6[2] + c7[3];
  } else {  // 16 independent 4x4x4 blocks: the Q-net's layer-2 tail candidate
    ACC8(f32x4);
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) { STEP8("v_mfma_f32_4x4x4_16b_bf16", a4, b4) }
    t1 = __builtin_amdgcn_s_memtime();
    s = c0[l & 3] + c1[1] + c2[2] + c3[3] + c4[0] + c5[1] + c6[2] + c7[3];
  }
  out[blockIdx.x * 64 + l] = s;
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int blocks = 256 * 4, iters = 2048;
  float* out; unsigned long long* cyc;
  (void)hipMalloc(&out, blocks * 64 * 4);
  (void)hipMalloc(&cyc, blocks * 8);
  static unsigned long long h[blocks];
  const char* names[4] = {"32x32x16_bf16", "16x16x32_bf16", "16x16x16bf16_1k", "4x4x4_16b_bf16"};
  double ref = 0;
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
      if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int b = 0; b < blocks; ++b) avg += h[b];
    avg /= blocks * 8.0 * iters;
    if (mode == 0) ref = avg;
    printf("%-18s %.3f ticks per MFMA = %.1f cycles (32x32x16 := 32)\n", names[mode], avg, 32.0 * avg / ref);
  }
  return 0;
}
