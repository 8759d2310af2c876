// The config-5 ego forward (qnet32_forward: 64 envs, all 32x32x16, 132 MFMAs = 4,224 matrix-pipe
// cycles) with one, two and three Q-net waves per SIMD and nothing else on the CU: how much of the
// matrix pipe one wave's in-order issue leaves idle (round 6).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//         -o tools/micro/qfwd32_waves tools/micro/qfwd32_waves.hip && tools/micro/qfwd32_waves
#include "../../merging-gym_amd/csrc/merging_hip.hip"

#include <cstdio>
#include <vector>

namespace {
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void probe(const uint8_t* net, int iters, unsigned long long* cyc, float* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_net[kQ32NetBytes];
  __shared__ __attribute__((aligned(16))) float tile[64 * WAVES * kObs];
  for (int j = threadIdx.x; j < kQ32NetBytes / 16; j += blockDim.x)
    reinterpret_cast<f32x4*>(lds_net)[j] = reinterpret_cast<const f32x4*>(net)[j];
  for (int j = threadIdx.x; j < 64 * WAVES * kObs; j += blockDim.x) tile[j] = 0.01f * ((j * 37) % 101) - 0.5f;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float acc = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    float q[8];
    qnet32_forward(lds_net, tile, wave * 64, (it & 1) != 0, q);
    acc += q[0] + q[1] + q[2] + q[3] + q[4];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * WAVES + wave] = t1 - t0;
}

template <int WAVES>
void run(const uint8_t* dnet, int iters) {
  const int blocks = 256;
  unsigned long long* dcyc;
  float* dout;
  (void)hipMalloc(&dcyc, sizeof(unsigned long long) * blocks * WAVES);
  (void)hipMalloc(&dout, sizeof(float) * blocks * 64 * WAVES);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(probe<WAVES>, dim3(blocks), dim3(64 * WAVES), 0, 0, dnet, iters, dcyc, dout);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> c(blocks * WAVES);
    (void)hipMemcpy(c.data(), dcyc, c.size() * sizeof(c[0]), hipMemcpyDeviceToHost);
    double mean = 0;
    for (auto v : c) mean += static_cast<double>(v);
    mean /= c.size();
    std::printf("{\"forward\": \"qnet32_forward (64 envs)\", \"q_waves_per_simd\": %d, \"cycles_per_forward_per_wave\": %.0f, "
                "\"simd_cycles_per_64_envs\": %.0f, \"mfma_pipe_cycles\": 4224}\n",
                WAVES / 4, mean / iters, mean / iters / (WAVES / 4));
  }
  (void)hipFree(dcyc);
  (void)hipFree(dout);
}
}  // namespace

int main() {
  std::vector<uint16_t> h(kQ32NetBytes / 2);
  for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint16_t>(0x3C00 + (i * 7919) % 512);
  uint8_t* dnet;
  (void)hipMalloc(&dnet, kQ32NetBytes);
  (void)hipMemcpy(dnet, h.data(), kQ32NetBytes, hipMemcpyHostToDevice);
  run<4>(dnet, 2000);
  run<8>(dnet, 2000);
  run<12>(dnet, 1500);
  (void)hipFree(dnet);
  return 0;
}
