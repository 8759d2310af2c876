// Issue cost of the VALU instructions the env step is made of, on one SIMD (gfx950): 8
// independent chains per lane, one wave per SIMD, s_memtime ticks per wave-instruction,
// printed relative to v_add_u32 (the full-rate 32-bit op). Decides which rewrites of the fp64
// step / Philox can pay (tools/micro/intmul.hip measured the multiplies alone).
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN8(INS, T, ...)                                                   \
  _Pragma("unroll") for (int j = 0; j < 8; ++j) asm volatile(INS : "+v"(x[j]) : __VA_ARGS__);

template <int MODE>
__global__ __launch_bounds__(64) void k(unsigned long long* out, unsigned long long* cyc, int iters) {
  unsigned long long t0 = 0, t1 = 0, s = 0;
  if constexpr (MODE < 8 || MODE >= 16) {  // 32-bit chains
    unsigned x[8];
    for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 2654435761u + j;
    const unsigned m = 0xD2511F53u;
    unsigned long long msk = __builtin_amdgcn_read_exec() >> (threadIdx.x & 1);  // a lane mask in an SGPR pair
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
      if (MODE == 0) { CHAIN8("v_add_u32 %0, %0, %1", unsigned, "s"(m)) }
      if (MODE == 1) { CHAIN8("v_add_f32 %0, %0, %1", unsigned, "s"(m)) }
      if (MODE == 2) { CHAIN8("v_mul_lo_u32 %0, %0, %1", unsigned, "s"(m)) }
      if (MODE == 3) { CHAIN8("v_mul_hi_u32 %0, %0, %1", unsigned, "s"(m)) }
      if (MODE == 4) { CHAIN8("v_xor_b32 %0, %0, %1", unsigned, "s"(m)) }
      if (MODE == 5) { CHAIN8("v_cndmask_b32 %0, %0, %1, vcc", unsigned, "v"(m)) }
      if (MODE == 6) { CHAIN8("v_fma_f32 %0, %0, %1, %0", unsigned, "s"(m)) }
      if (MODE == 7) { CHAIN8("v_mul_u32_u24 %0, %0, %1", unsigned, "s"(m)) }
      if (MODE == 16) { CHAIN8("v_cndmask_b32_e64 %0, %0, %1, s[40:41]", unsigned, "v"(m)) }
      if (MODE == 17) { CHAIN8("v_cndmask_b32_e64 %0, %1, %0, vcc", unsigned, "v"(m)) }
      if (MODE == 18) { CHAIN8("v_cndmask_b32_e32 %0, %1, %0, vcc", unsigned, "v"(m)) }
      if (MODE == 19) { CHAIN8("v_cndmask_b32_e64 %0, %0, %1, vcc", unsigned, "v"(m)) }
    }
    t1 = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < 8; ++j) s ^= x[j];
  } else {  // 64-bit chains
    unsigned long long x[8];
    for (int j = 0; j < 8; ++j) x[j] = (threadIdx.x * 2654435761ull + j) | 0x3ff0000000000000ull;
    const unsigned long long m = 0x3ff0000000000001ull;
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
      if (MODE == 8) { CHAIN8("v_add_f64 %0, %0, %1", unsigned long long, "s"(m)) }
      if (MODE == 9) { CHAIN8("v_mul_f64 %0, %0, %1", unsigned long long, "s"(m)) }
      if (MODE == 10) { CHAIN8("v_fma_f64 %0, %0, %1, %0", unsigned long long, "s"(m)) }
      if (MODE == 11) { CHAIN8("v_lshl_add_u64 %0, %0, 3, %0", unsigned long long, "s"(m)) }
      if (MODE == 12) { CHAIN8("v_mov_b64 %0, %0", unsigned long long, "s"(m)) }
      if (MODE == 13) { CHAIN8("v_pk_add_f32 %0, %0, %1", unsigned long long, "s"(m)) }
      if (MODE == 14) { CHAIN8("v_pk_fma_f32 %0, %0, %1, %0", unsigned long long, "s"(m)) }
      if (MODE == 15) { CHAIN8("v_cmp_lt_f64 vcc, %0, %1", unsigned long long, "s"(m)) }
    }
    t1 = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < 8; ++j) s ^= x[j];
  }
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
double run(unsigned long long* out, unsigned long long* cyc, int blocks, int iters, unsigned long long* h) {
  // throughput: wave-instructions per SIMD per ns over the whole chip, from HIP events
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double wave_instr_per_simd = static_cast<double>(blocks) * 8.0 * iters / 1024.0;
  return ms * 1e6 / wave_instr_per_simd;  // ns per wave-instruction per SIMD
}

int main() {
  const int iters = 4096;
  unsigned long long *out, *cyc;
  const int max_blocks = 1024 * 8;
  hipMalloc(&out, max_blocks * 64 * 8);
  hipMalloc(&cyc, max_blocks * 8);
  static unsigned long long h[max_blocks];
  const char* names[20] = {"v_add_u32", "v_add_f32", "v_mul_lo_u32", "v_mul_hi_u32", "v_xor_b32",
                           "v_cndmask_b32", "v_fma_f32", "v_mul_u32_u24", "v_add_f64", "v_mul_f64",
                           "v_fma_f64", "v_lshl_add_u64", "v_mov_b64", "v_pk_add_f32", "v_pk_fma_f32",
                           "v_cmp_lt_f64", "v_cndmask_e64 s40", "v_cndmask_e64 vcc", "v_cndmask_e32 m,x", "v_cndmask_e64 x,m"};
  for (int wps : {8}) {
    const int blocks = 1024 * wps;  // 64-thread blocks: wps waves per SIMD
    double r[20];
    r[0] = run<0>(out, cyc, blocks, iters, h);  r[1] = run<1>(out, cyc, blocks, iters, h);
    r[2] = run<2>(out, cyc, blocks, iters, h);  r[3] = run<3>(out, cyc, blocks, iters, h);
    r[4] = run<4>(out, cyc, blocks, iters, h);  r[5] = run<5>(out, cyc, blocks, iters, h);
    r[6] = run<6>(out, cyc, blocks, iters, h);  r[7] = run<7>(out, cyc, blocks, iters, h);
    r[8] = run<8>(out, cyc, blocks, iters, h);  r[9] = run<9>(out, cyc, blocks, iters, h);
    r[10] = run<10>(out, cyc, blocks, iters, h); r[11] = run<11>(out, cyc, blocks, iters, h);
    r[12] = run<12>(out, cyc, blocks, iters, h); r[13] = run<13>(out, cyc, blocks, iters, h);
    r[14] = run<14>(out, cyc, blocks, iters, h); r[15] = run<15>(out, cyc, blocks, iters, h);
    r[16] = run<16>(out, cyc, blocks, iters, h); r[17] = run<17>(out, cyc, blocks, iters, h);
    r[18] = run<18>(out, cyc, blocks, iters, h); r[19] = run<19>(out, cyc, blocks, iters, h);
    for (int m = 0; m < 20; ++m)
      printf("waves/SIMD %d  %-16s %.3f ns per wave-instr per SIMD, %.2f x v_add_u32\n", wps, names[m], r[m],
             r[m] / r[0]);
  }
  return 0;
}
