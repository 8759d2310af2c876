// Issue cost of the 32x32 multiplies Philox4x32-10 needs, on one SIMD (gfx950).
// 8 independent chains per lane, each iteration one mulhi/mullo pair or one mad_u64_u32 per
// chain; cycles per wave-instruction from s_memtime over the loop (1 wave per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(64) void k(unsigned* out, unsigned long long* cyc, int iters) {
  unsigned a[8], b[8];
  for (int j = 0; j < 8; ++j) { a[j] = threadIdx.x * 2654435761u + j; b[j] = j * 40503u + 1; }
  const unsigned m = 0xD2511F53u;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (MODE == 0) {  // mul_lo + mul_hi
        unsigned lo, hi;
        asm volatile("v_mul_lo_u32 %0, %2, %3\n v_mul_hi_u32 %1, %2, %3" : "=&v"(lo), "=&v"(hi) : "v"(a[j]), "s"(m));
        a[j] = hi ^ b[j];
        b[j] = lo;
      } else if (MODE == 1) {  // one mad_u64_u32
        unsigned long long p;
        asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, 0" : "=&v"(p) : "v"(a[j]), "s"(m) : "s100", "s101");
        a[j] = static_cast<unsigned>(p >> 32) ^ b[j];
        b[j] = static_cast<unsigned>(p);
      } else {  // reference: fp64 add chain
        double x = __builtin_bit_cast(double, (static_cast<unsigned long long>(a[j]) << 32) | b[j]);
        asm volatile("v_add_f64 %0, %0, %0" : "+v"(x));
        unsigned long long u = __builtin_bit_cast(unsigned long long, x);
        a[j] = static_cast<unsigned>(u >> 32) ^ b[j];
        b[j] = static_cast<unsigned>(u);
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned s = 0;
  for (int j = 0; j < 8; ++j) s ^= a[j] ^ b[j];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int blocks = 256 * 4, iters = 4096;
  unsigned* out; unsigned long long* cyc;
  hipMalloc(&out, blocks * 64 * 4);
  hipMalloc(&cyc, blocks * 8);
  unsigned long long h[blocks];
  const char* names[3] = {"mul_lo+mul_hi (2 instr)", "mad_u64_u32 (1 instr)", "v_add_f64 (+2 xor, ref)"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int b = 0; b < blocks; ++b) avg += h[b];
    avg /= blocks;
    // s_memtime ticks at the shader clock on gfx950 (MI355X_MICROARCH.md constants table)
    printf("%-26s %.2f cycles per chain-iteration (8 chains x %d iters), %.2f per wave-instr\n", names[mode],
           avg / (8.0 * iters), iters, avg / (8.0 * iters) / (mode == 0 ? 2 : 1));
  }
  return 0;
}
