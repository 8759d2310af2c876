// Does fp64 vector arithmetic share the matrix pipe with bf16 MFMAs on gfx950? (round 6)
//
// One block per CU, 8 waves = 2 per SIMD. Waves 0-3 ("matrix waves") run a loop of
// v_mfma_f32_32x32x16_bf16 on 8 independent accumulators; waves 4-7 ("vector waves") run, by mode,
//   0: nothing (exit at once)
//   1: v_fma_f32 on 8 independent chains
//   2: v_fma_f64 on 8 independent chains
//   3: v_add_f64 / v_mul_f64 mix on 8 independent chains (the env step's common ops)
// and the same vector loops with the matrix waves idle (matrix_waves false), for their rate alone.
// Each wave reports its s_memtime cycles; the matrix waves' cycles per MFMA (32 alone = the pipe)
// and the vector waves' cycles per instruction say which units the two streams share.
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/mfma_fp64_share tools/micro/mfma_fp64_share.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMfmaIters = 4096;  // x 8 MFMAs per matrix wave
constexpr int kVecIters = 4096;   // x 8 instructions per vector wave (x 4 per mode-3 step)

template <int MODE, bool MATRIX = true>
__global__ __launch_bounds__(512) void probe(const float* in, float* out, unsigned long long* cyc, int vec_iters) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float x = in[threadIdx.x];
  unsigned long long t0 = 0, t1 = 0;
  if (wave < 4) {
    if (!MATRIX) return;
    bf16x8 a, b;
    for (int k = 0; k < 8; ++k) {
      a[k] = static_cast<__bf16>(x * (k + 1));
      b[k] = static_cast<__bf16>(x - k);
    }
    f32x16 c[8];
    for (int j = 0; j < 8; ++j)
      for (int k = 0; k < 16; ++k) c[j][k] = 0.0f;
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kMfmaIters; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c[j], 0, 0, 0);
    }
    t1 = __builtin_amdgcn_s_memtime();
    float s = 0.0f;
    for (int j = 0; j < 8; ++j) s += c[j][lane & 15];
    out[blockIdx.x * 512 + threadIdx.x] = s;
  } else if (MODE != 0) {
    t0 = __builtin_amdgcn_s_memtime();
    if constexpr (MODE == 1) {
      float v[8];
      for (int j = 0; j < 8; ++j) v[j] = x + j;
      for (int it = 0; it < vec_iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = __builtin_fmaf(v[j], 0.999f, 0.001f);
      }
      float s = 0.0f;
      for (int j = 0; j < 8; ++j) s += v[j];
      out[blockIdx.x * 512 + threadIdx.x] = s;
    } else {
      double v[8];
      for (int j = 0; j < 8; ++j) v[j] = static_cast<double>(x) + j;
      for (int it = 0; it < vec_iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if constexpr (MODE == 2)
            v[j] = __builtin_fma(v[j], 0.999, 0.001);
          else
            v[j] = (j & 1) ? v[j] * 0.999 : v[j] + 0.001;
        }
      }
      double s = 0.0;
      for (int j = 0; j < 8; ++j) s += v[j];
      out[blockIdx.x * 512 + threadIdx.x] = static_cast<float>(s);
    }
    t1 = __builtin_amdgcn_s_memtime();
  }
  if (lane == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

template <int MODE, bool MATRIX = true>
static void run(const float* din, float* dout, unsigned long long* dcyc, int blocks, const char* name, int vec_iters) {
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL((probe<MODE, MATRIX>), dim3(blocks), dim3(512), 0, 0, din, dout, dcyc, vec_iters);
    (void)hipDeviceSynchronize();
  }
  std::vector<unsigned long long> c(blocks * 8);
  (void)hipMemcpy(c.data(), dcyc, c.size() * sizeof(c[0]), hipMemcpyDeviceToHost);
  double m = 0, v = 0;
  for (int b = 0; b < blocks; ++b)
    for (int w = 0; w < 8; ++w) (w < 4 ? m : v) += static_cast<double>(c[b * 8 + w]);
  m /= 4.0 * blocks;
  v /= 4.0 * blocks;
  std::printf("{\"matrix_waves\": %s, \"vector_waves\": \"%s\", \"vec_iters\": %d, \"matrix_cycles_per_mfma\": %.2f, "
              "\"vector_cycles_per_instr\": %.2f, \"matrix_wave_cycles\": %.0f, \"vector_wave_cycles\": %.0f}\n",
              MATRIX ? "true" : "false", name, vec_iters, m / (8.0 * kMfmaIters), MODE ? v / (8.0 * vec_iters) : 0.0, m, v);
}

int main() {
  const int blocks = 256;
  float *din, *dout;
  unsigned long long* dcyc;
  (void)hipMalloc(&din, 512 * sizeof(float));
  (void)hipMalloc(&dout, blocks * 512 * sizeof(float));
  (void)hipMalloc(&dcyc, blocks * 8 * sizeof(unsigned long long));
  std::vector<float> h(512);
  for (int i = 0; i < 512; ++i) h[i] = 0.001f * (i % 97) + 0.5f;
  (void)hipMemcpy(din, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice);
  run<0>(din, dout, dcyc, blocks, "none", kVecIters);
  for (int vi : {kVecIters, 4 * kVecIters}) {
    run<1>(din, dout, dcyc, blocks, "fma_f32", vi);
    run<2>(din, dout, dcyc, blocks, "fma_f64", vi);
    run<3>(din, dout, dcyc, blocks, "add_mul_f64", vi);
    run<1, false>(din, dout, dcyc, blocks, "fma_f32", vi);
    run<2, false>(din, dout, dcyc, blocks, "fma_f64", vi);
    run<3, false>(din, dout, dcyc, blocks, "add_mul_f64", vi);
  }
  return 0;
}
