// Timing A/B of VERDICT r05 item 3: the 16x16 forward's layer 1 on v_mfma_f32_16x16x32_bf16 (K = 16 of
// 32 used, lanes 32-63 of the input operand zero) with the accumulator layout already equal to layer
// 2's B operand -- no v_permlane16_swap -- against the shipped qnet_mlp (layer 1 on 32x32x16, one
// permlane16_swap per register pair). Cycles per forward (s_memtime) with one or two Q-net waves per
// SIMD, nothing else on the CU, as tools/micro/qfwd_probe.hip. Timing only: the variant's weights
// are the packed net's bytes read in the variant's pattern (two 16-B layer-1 reads per k-block), so
// its Q values are not a forward's.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//         -o tools/micro/qfwd_l1x16 tools/micro/qfwd_l1x16.hip && tools/micro/qfwd_l1x16
#ifndef MG_SRC
#include "../../merging-gym_amd/csrc/merging_hip.hip"
#else
#include MG_SRC  // an edited copy of the source (tools/micro/qfwd_ablate.sh: the forward's parts removed)
#endif

#include <cstdio>
#include <vector>

namespace {

// qnet_mlp<D, 4> with layer 1 as 2 x 4 16x16x32 MFMAs per k-block (hidden tiles 2 kb, 2 kb + 1 x env
// tiles 0..3); env tile t's layer-2 operand = the ReLU pairs of its two layer-1 tiles, in place.
template <int D, class Src>
__device__ __forceinline__ void qnet_mlp_l1x16(const Src& src, const bf16x8 (&xt)[4], float (&q)[8]) {
  bf16x8 ring[D];
#pragma unroll
  for (int s = 0; s < D; ++s) ring[s] = src(s);
  auto take = [&](int s) __attribute__((always_inline)) {
    const bf16x8 f = ring[s % D];
    if (s + D < kQFrags) ring[s % D] = src(s + D);
    return f;
  };
  const f32x4 z4 = {};
  f32x4 c[2][4];
  auto layer1 = [&](int s) __attribute__((always_inline)) {
    const bf16x8 a0 = take(s);
    const bf16x8 a1 = src(s);  // the second hidden tile's fragment (one more 16-B LDS read)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      c[0][t] = mfma16(a0, xt[t], z4);
      c[1][t] = mfma16(a1, xt[t], z4);
    }
  };
  uint32_t nx[16];  // nx[4 t + d]: dword d of env tile t's layer-2 B operand
  auto relu_d = [&](int d) __attribute__((always_inline)) {  // d = 4 t + 2 m + p
    const int t = d >> 2, m = (d >> 1) & 1, p = d & 1;
    return relu_pair(c[m][t][2 * p], c[m][t][2 * p + 1]);
  };
  auto operands = [&](bf16x8 (&hb)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 4; ++t) hb[t] = __builtin_bit_cast(bf16x8, u32x4{nx[4 * t], nx[4 * t + 1], nx[4 * t + 2], nx[4 * t + 3]});
  };
  layer1(0);
#pragma unroll
  for (int d = 0; d < 16; ++d) nx[d] = relu_d(d);
  bf16x8 hb[4];
  operands(hb);
  f32x4 acc2[kQT2][4];
  auto slot = [&](f32x4& acc, const bf16x8& a, const bf16x8& b, bool zero) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    acc = mfma16(a, b, zero ? z4 : acc);
  };
  int s = 1;
#pragma unroll
  for (int kb = 0; kb < kQT1 - 1; ++kb) {
    layer1(s++);
#pragma unroll
    for (int t2 = 0; t2 < kQT2; ++t2) {
      const bf16x8 a2 = take(s++);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        slot(acc2[t2][t], a2, hb[t], kb == 0);
        // the next k-block's 16 ReLU pairs behind row tiles 1..4 (no swaps)
        if (t2 >= 1 && t2 <= 4) nx[4 * (t2 - 1) + t] = relu_d(4 * (t2 - 1) + t);
      }
    }
    operands(hb);
  }
  f32x4 acc3[4] = {z4, z4, z4, z4};
  uint32_t b3[2][4][4];
  auto pairs3 = [&](int t2, int t) __attribute__((always_inline)) {
    const int buf = (t2 >> 1) & 1, d = 2 * (t2 & 1);
    b3[buf][t][d] = relu_pair(acc2[t2][t][0], acc2[t2][t][1]);
    b3[buf][t][d + 1] = relu_pair(acc2[t2][t][2], acc2[t2][t][3]);
  };
  auto layer2 = [&](int t2, int p) __attribute__((always_inline)) {
    const bf16x8 a2 = take(s++);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      slot(acc2[t2][t], a2, hb[t], false);
      if (p >= 0) pairs3(p, t);
    }
  };
  auto layer3 = [&](int k3, int p) __attribute__((always_inline)) {
    const bf16x8 a3 = take(s++);
    const int buf = k3 & 1;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (2 * k3 + 1 >= kQT2) b3[buf][t][2] = b3[buf][t][3] = 0u;
      const bf16x8 b = __builtin_bit_cast(bf16x8, u32x4{b3[buf][t][0], b3[buf][t][1], b3[buf][t][2], b3[buf][t][3]});
      slot(acc3[t], a3, b, k3 == 0);
      if (p >= 0) pairs3(p, t);
    }
  };
  layer2(0, -1);
  layer2(1, 0);
  layer2(2, 1);
  layer3(0, 2);
  layer2(3, -1);
  layer2(4, 3);
  layer3(1, 4);
  layer2(5, -1);
  layer2(6, 5);
  layer3(2, 6);
  layer3(3, -1);
  qnet_gather_q(acc3, q);
}

// env tile t's layer-1 B operand: lanes 0-31 the features of env 16 t + (lane & 15), k-half (lane >> 4);
// lanes 32-63 zero (K 16..31 of the 16x16x32 MFMA)
__device__ __forceinline__ bf16x8 l1x16_input(const float* tile, int row0, int t, bool swap) {
  const int lane = threadIdx.x & 63;
  const bf16x8 x = qnet_input(tile + (row0 + 16 * t + (lane & 15)) * kObs, swap, (lane >> 4) & 1);
  return lane < 32 ? x : bf16x8{};
}

// weights from registers: the fragment index picks one of four (timing only: no LDS reads)
struct QSrcReg {
  bf16x8 r[4];
  __device__ __forceinline__ bf16x8 operator()(int s) const {
    bf16x8 v = r[s & 3];
    asm volatile("" : "+v"(v));  // opaque: no two fragments are the same value (no MFMA is merged)
    return v;
  }
};

template <int WAVES, int MODE>  // MODE 0: shipped qnet_forward_swp; 1: the layer-1 16x16x32 variant;
                                // 2 / 3 / 4: the shipped forward with 3 / 4 / 6 fragments in flight;
                                // 5: the shipped forward with its weights in registers
__global__ __launch_bounds__(64 * WAVES) void probe(const uint8_t* net, int iters, unsigned long long* cyc, float* out) {
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
    const bool swap = (it & 1) != 0;
    if constexpr (MODE == 0) {
      qnet_forward_swp(lds_net, tile, wave * 64, swap, q);
    } else if constexpr (MODE == 5) {
      const int r = lane & 31, h = lane >> 5;
      QSrcReg src;
#pragma unroll
      for (int j = 0; j < 4; ++j) src.r[j] = *reinterpret_cast<const bf16x8*>(lds_net + 1024 * j + 16 * lane);
      qnet_mlp<2>(src, qnet_input(tile + (wave * 64 + r) * kObs, swap, h),
                  qnet_input(tile + (wave * 64 + 32 + r) * kObs, swap, h), q);
    } else if constexpr (MODE >= 2) {
      constexpr int D = MODE == 2 ? 3 : MODE == 3 ? 4 : 6;
      const int r = lane & 31, h = lane >> 5;
      qnet_mlp<D>(qnet_lds(lds_net), qnet_input(tile + (wave * 64 + r) * kObs, swap, h),
                  qnet_input(tile + (wave * 64 + 32 + r) * kObs, swap, h), q);
    } else {
      bf16x8 xt[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) xt[t] = l1x16_input(tile, wave * 64, t, swap);
      qnet_mlp_l1x16<kQLdsAhead>(qnet_lds(lds_net), xt, q);
    }
    acc += q[0] + q[1] + q[2] + q[3] + q[4];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * WAVES + wave] = t1 - t0;
}

template <int WAVES, int MODE>
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
    hipLaunchKernelGGL((probe<WAVES, MODE>), dim3(blocks), dim3(64 * WAVES), 0, 0, dnet, iters, dcyc, dout);
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(blocks * WAVES);
    (void)hipMemcpy(c.data(), dcyc, c.size() * sizeof(c[0]), hipMemcpyDeviceToHost);
    double mean = 0;
    for (auto v : c) mean += static_cast<double>(v);
    mean /= c.size();
    std::printf("{\"forward\": \"%s\", \"q_waves_per_simd\": %d, \"blocks\": %d, \"iters\": %d, "
                "\"cycles_per_forward\": %.0f, \"mfma_pipe_cycles\": %d, \"wall_ms\": %.3f}\n",
                MODE == 0 ? "shipped (layer 1 32x32x16 + permlane16_swap), 2 fragments ahead"
                : MODE == 1 ? "layer 1 16x16x32, no swaps"
                : MODE == 2 ? "shipped, 3 ahead" : MODE == 3 ? "shipped, 4 ahead"
                : MODE == 4 ? "shipped, 6 ahead" : "shipped, weights in registers",
                WAVES / 4, blocks, iters, mean / iters, MODE == 1 ? 4288 : 3840, ms);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  (void)hipFree(dcyc);
  (void)hipFree(dout);
}
}  // namespace

int main(int argc, char** argv) {
  if (argc > 1) {  // ablation binaries: the shipped forward (and with register weights), one and two waves
    std::vector<uint16_t> h(kQNetBytes / 2);
    for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint16_t>(0x3C00 + (i * 7919) % 512);
    uint8_t* dnet;
    (void)hipMalloc(&dnet, kQNetBytes);
    (void)hipMemcpy(dnet, h.data(), kQNetBytes, hipMemcpyHostToDevice);
    std::printf("{\"variant\": \"%s\"}\n", argv[1]);
    run<4, 0>(dnet, 256, 2000);
    run<4, 5>(dnet, 256, 2000);
    run<8, 0>(dnet, 256, 2000);
    run<8, 5>(dnet, 256, 2000);
    (void)hipFree(dnet);
    return 0;
  }
  std::vector<uint16_t> h(kQNetBytes / 2);
  for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint16_t>(0x3C00 + (i * 7919) % 512);  // small bf16
  uint8_t* dnet;
  (void)hipMalloc(&dnet, kQNetBytes);
  (void)hipMemcpy(dnet, h.data(), kQNetBytes, hipMemcpyHostToDevice);
  run<4, 0>(dnet, 256, 2000);
  run<4, 1>(dnet, 256, 2000);
  run<8, 0>(dnet, 256, 2000);
  run<8, 1>(dnet, 256, 2000);
  run<4, 2>(dnet, 256, 2000);
  run<4, 3>(dnet, 256, 2000);
  run<4, 4>(dnet, 256, 2000);
  run<8, 2>(dnet, 256, 2000);
  run<8, 3>(dnet, 256, 2000);
  run<4, 0>(dnet, 256, 2000);
  (void)hipFree(dnet);
  return 0;
}
