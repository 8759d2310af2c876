// Numerics probe of the two bf16 MFMAs the Q-net forwards use: one wave per
// case runs ONE v_mfma_f32_16x16x32_bf16 (or v_mfma_f32_32x32x16_bf16) on logical row-major operands
// A [M][K] bf16, B [K][N] bf16, C [M][N] fp32 and writes D [M][N]. tools/mfma_numerics.py crafts the
// operands on the host and fits the accumulation rule against the outputs.
//
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/micro/libmfma_numerics.so tools/micro/mfma_numerics.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// 16x16x32: lane l holds A row l % 16, k = 8 (l / 16) + j; B column l % 16, the same k; D column
// l % 16, rows 4 (l / 16) + i.
__global__ __launch_bounds__(64) void mfma16_probe(const __bf16* A, const __bf16* B, const float* C, float* D,
                                                   int n) {
  const int c = blockIdx.x, l = threadIdx.x;
  if (c >= n) return;
  const __bf16* a = A + (size_t)c * 16 * 32;
  const __bf16* b = B + (size_t)c * 32 * 16;
  bf16x8 av, bv;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    av[j] = a[(l % 16) * 32 + 8 * (l / 16) + j];
    bv[j] = b[(8 * (l / 16) + j) * 16 + l % 16];
  }
  f32x4 cv;
#pragma unroll
  for (int i = 0; i < 4; ++i) cv[i] = C[(size_t)c * 256 + (4 * (l / 16) + i) * 16 + l % 16];
  const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, cv, 0, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; ++i) D[(size_t)c * 256 + (4 * (l / 16) + i) * 16 + l % 16] = d[i];
}

// 32x32x16: lane l holds A row l % 32, k = 8 (l / 32) + j; B column l % 32, the same k; D column
// l % 32, rows 8 (i / 4) + 4 (l / 32) + i % 4.
__global__ __launch_bounds__(64) void mfma32_probe(const __bf16* A, const __bf16* B, const float* C, float* D,
                                                   int n) {
  const int c = blockIdx.x, l = threadIdx.x;
  if (c >= n) return;
  const __bf16* a = A + (size_t)c * 32 * 16;
  const __bf16* b = B + (size_t)c * 16 * 32;
  bf16x8 av, bv;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    av[j] = a[(l % 32) * 16 + 8 * (l / 32) + j];
    bv[j] = b[(8 * (l / 32) + j) * 32 + l % 32];
  }
  f32x16 cv;
#pragma unroll
  for (int i = 0; i < 16; ++i) cv[i] = C[(size_t)c * 1024 + (8 * (i / 4) + 4 * (l / 32) + i % 4) * 32 + l % 32];
  const f32x16 d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, cv, 0, 0, 0);
#pragma unroll
  for (int i = 0; i < 16; ++i) D[(size_t)c * 1024 + (8 * (i / 4) + 4 * (l / 32) + i % 4) * 32 + l % 32] = d[i];
}

extern "C" int mfma_probe(int form, const void* A, const void* B, const void* C, void* D, int n) {
  if (n <= 0) return 0;
  if (form == 16)
    hipLaunchKernelGGL(mfma16_probe, dim3(n), dim3(64), 0, 0, (const __bf16*)A, (const __bf16*)B, (const float*)C,
                       (float*)D, n);
  else if (form == 32)
    hipLaunchKernelGGL(mfma32_probe, dim3(n), dim3(64), 0, 0, (const __bf16*)A, (const __bf16*)B, (const float*)C,
                       (float*)D, n);
  else
    return -1;
  if (hipGetLastError() != hipSuccess) return -2;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}
