// Operand layout probe of v_mfma_f32_4x4x4_16b_bf16 (gfx950), checked on the host against the
// layout the Q-net's layer-2 tail assumes: block b = lane / 4; A[i][k] of block b in lane 4b + i
// (element k), B[k][j] in lane 4b + j (element k), D[i][j] in register i of lane 4b + j.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstring>

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

static inline short bf16_bits(float f) {  // exact for the small integers used here
  unsigned u;
  memcpy(&u, &f, 4);
  return (short)(u >> 16);
}

__global__ void probe(const s16x4* a, const s16x4* b, f32x4* d) {
  const int l = threadIdx.x;
  d[l] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a[l], b[l], f32x4{0, 0, 0, 0}, 0, 0, 0);
}

int main() {
  s16x4 ha[64], hb[64];
  float A[16][4][4], B[16][4][4];  // [block][i][k], [block][k][j]
  for (int l = 0; l < 64; ++l)
    for (int k = 0; k < 4; ++k) {
      const float av = (float)((l * 7 + k * 3) % 11 - 5), bv = (float)((l * 5 + k * 13) % 9 - 4);
      ha[l][k] = bf16_bits(av);
      hb[l][k] = bf16_bits(bv);
      A[l / 4][l % 4][k] = av;
      B[l / 4][k][l % 4] = bv;
    }
  s16x4 *da, *db;
  f32x4* dd;
  (void)hipMalloc(&da, sizeof(ha));
  (void)hipMalloc(&db, sizeof(hb));
  (void)hipMalloc(&dd, 64 * sizeof(f32x4));
  (void)hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
  (void)hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dd);
  f32x4 hd[64];
  (void)hipMemcpy(hd, dd, sizeof(hd), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      float ref = 0;
      for (int k = 0; k < 4; ++k) ref += A[l / 4][i][k] * B[l / 4][k][l % 4];
      if (hd[l][i] != ref) ++bad;
    }
  printf("4x4x4_16b_bf16 layout (A lane 4b+i, B lane 4b+j, D reg i of lane 4b+j): %s (%d of 256 differ)\n",
         bad ? "MISMATCH" : "ok", bad);
  return bad ? 1 : 0;
}
