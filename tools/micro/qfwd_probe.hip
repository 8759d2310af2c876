// Cycles per Q-net forward (qnet_forward_swp: since ABI 19 the 16x16x32 forward, 14 x 32 + 212 x 16
// = 3,840 matrix-pipe cycles; built against the ABI-18 source it is the 32x32 forward, 132 x 32 =
// 4,224) with one or two Q-net waves per SIMD and nothing else on the CU. The "mfma_tflops" and
// "mfma_cycles_per_forward" fields count the 32x32 forward's 4,224 cycles of work for both, so
// compare wall times. s_memtime around `iters` forwards per wave; weights and a 64-env observation
// tile per wave in LDS, as in the kernel.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//         -o tools/micro/qfwd_probe tools/micro/qfwd_probe.hip && tools/micro/qfwd_probe
#include "../../merging-gym_amd/csrc/merging_hip.hip"

#include <cstdio>
#include <vector>

namespace {
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void qfwd_probe(const uint8_t* net, int iters, unsigned long long* cyc,
                                                         float* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_net[kQNetBytes];
  __shared__ __attribute__((aligned(16))) float tile[64 * WAVES * kObs];
  qnet_to_lds(net, lds_net);
  for (int j = threadIdx.x; j < 64 * WAVES * kObs; j += blockDim.x) tile[j] = 0.01f * ((j * 37) % 101) - 0.5f;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float acc = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    float q[8];
    qnet_forward_swp(lds_net, tile, wave * 64, (it & 1) != 0, q);
    acc += q[0] + q[1] + q[2] + q[3] + q[4];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * WAVES + wave] = t1 - t0;
}

// the same 132 MFMAs per "forward" with register operands only (8 independent accumulators, no
// LDS, no VALU): the matrix pipe's sustained rate when nothing else runs
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void mfma_only_probe(const uint8_t* net, int iters, unsigned long long* cyc,
                                                              float* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = static_cast<__bf16>(0.001f * (lane + j));
    b[j] = static_cast<__bf16>(0.002f * (lane - j));
  }
  f32x16 c[8] = {};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 132; ++k) c[k & 7] = mfma32(a, b, c[k & 7]);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
  for (int k = 0; k < 8; ++k) acc += c[k][lane & 15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * WAVES + wave] = t1 - t0;
  (void)net;
}

// the same matrix-pipe work (132 x 32x32x16 = 264 x 16x16x32 FLOPs) as 16x16x32 MFMAs, 8 independent
// accumulators: does the smaller shape sustain a higher rate (clock) on all SIMDs?
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void mfma16_only_probe(const uint8_t* net, int iters, unsigned long long* cyc,
                                                                float* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = static_cast<__bf16>(0.001f * (lane + j));
    b[j] = static_cast<__bf16>(0.002f * (lane - j));
  }
  f32x4v c[8] = {};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 264; ++k) c[k & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[k & 7], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
  for (int k = 0; k < 8; ++k) acc += c[k][lane & 3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * WAVES + wave] = t1 - t0;
  (void)net;
}

template <int WAVES, int MODE = 0>  // MODE 0: qnet_forward_swp, 1: 32x32x16 only, 2: 16x16x32 only
void run(const uint8_t* dnet, int blocks, int iters) {
  unsigned long long* dcyc;
  float* dout;
  (void)hipMalloc(&dcyc, sizeof(unsigned long long) * blocks * WAVES);
  (void)hipMalloc(&dout, sizeof(float) * blocks * 64 * WAVES);
  for (int rep = 0; rep < 3; ++rep) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    if (MODE == 1)
      hipLaunchKernelGGL(mfma_only_probe<WAVES>, dim3(blocks), dim3(64 * WAVES), 0, 0, dnet, iters, dcyc, dout);
    else if (MODE == 2)
      hipLaunchKernelGGL(mfma16_only_probe<WAVES>, dim3(blocks), dim3(64 * WAVES), 0, 0, dnet, iters, dcyc, dout);
    else
      hipLaunchKernelGGL(qfwd_probe<WAVES>, dim3(blocks), dim3(64 * WAVES), 0, 0, dnet, iters, dcyc, dout);
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(blocks * WAVES);
    (void)hipMemcpy(c.data(), dcyc, c.size() * sizeof(c[0]), hipMemcpyDeviceToHost);
    double mean = 0;
    for (auto v : c) mean += static_cast<double>(v);
    mean /= c.size();
    const double flops = 2.0 * 132 * 32 * 32 * 16 * blocks * WAVES * iters;  // executed MFMA flops
    std::printf("{\"kernel\": \"%s\", \"waves_per_block\": %d, \"blocks\": %d, \"iters\": %d, "
                "\"cycles_per_forward\": %.0f, \"mfma_cycles_per_forward\": 4224, \"wall_ms\": %.3f, "
                "\"mfma_tflops\": %.1f, \"clock_ghz\": %.2f}\n",
                MODE == 1 ? "mfma_32x32x16_only" : MODE == 2 ? "mfma_16x16x32_only" : "qnet_forward_swp", WAVES, blocks,
                iters, mean / iters, ms,
                flops / (ms * 1e-3) / 1e12, mean / (ms * 1e-3) / 1e9);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  (void)hipFree(dcyc);
  (void)hipFree(dout);
}
}  // namespace

int main() {
  std::vector<uint16_t> h(kQNetBytes / 2);
  for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint16_t>(0x3C00 + (i * 7919) % 512);  // small bf16
  uint8_t* dnet;
  (void)hipMalloc(&dnet, kQNetBytes);
  (void)hipMemcpy(dnet, h.data(), kQNetBytes, hipMemcpyHostToDevice);
  run<4>(dnet, 256, 2000);  // one Q-net wave per SIMD, one block per CU
  run<8>(dnet, 256, 2000);  // two per SIMD
  run<4>(dnet, 512, 2000);  // one per SIMD, two blocks per CU if they fit
  run<4, 1>(dnet, 256, 2000);  // MFMAs alone, one wave per SIMD
  run<8, 1>(dnet, 256, 2000);  // two per SIMD
  run<4, 2>(dnet, 256, 2000);  // the same FLOPs as 16x16x32 MFMAs
  run<8, 2>(dnet, 256, 2000);
  (void)hipFree(dnet);
  return 0;
}
