// Feasibility probe: two 32-env forwards (the shipped qnet_mlp<D, 2> body, unit by unit) software-
// pipelined half a forward apart in ONE wave, so each one's fill, drain and layer transitions
// overlap the other's MFMAs -- what a second Q-net wave per SIMD gives (round 6: one forward alone
// keeps the matrix pipe ~52 % busy, two waves ~95 %; profiles/r06/ab/r06h_qfwd_ring_depth.txt).
// Cycles per 64 envs (two 32-env forwards) against the shipped NC 4 forward, one and two waves per SIMD.
// Timing and a bit check: the pipelined forwards' Q rows must equal qnet_mlp<D, 2>'s.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//         -o tools/micro/qfwd_pipe2 tools/micro/qfwd_pipe2.hip && tools/micro/qfwd_pipe2
#include "../../merging-gym_amd/csrc/merging_hip.hip"

#include <cstdio>
#include <vector>

namespace {

constexpr int kUnits = 62;  // units of one 32-env forward (see Fwd2::unit)
constexpr int kHalfU = 31;

// The shipped qnet_mlp<D, 2> split into 62 units in its own order: U0 layer 1 of k-block 0; U1 its
// ReLU pairs, swaps and layer-2 operands; then per k-block kb = 0..5 a layer-1 unit (k-block kb + 1)
// and seven row-tile units (2 MFMAs each, with the ReLU pairs behind row tiles 1-2 and the swaps
// behind 5, as qnet_mlp places them for nc = 2) -- the last one also forms the next operands; then
// the tail (layer 2 of k-block 6 with layer 3 interleaved, 11 units) and the gather.
template <int D, class Src>
struct Fwd2 {
  bf16x8 ring[D];
  f32x16 c0;
  uint32_t nx[8];
  bf16x8 hb[2];
  f32x4 acc2[kQT2][2];
  f32x4 acc3[2];
  uint32_t b3[2][2][4];

  __device__ __forceinline__ bf16x8 take(const Src& src, int s) {
    const bf16x8 f = ring[s % D];
    if (s + D < kQFrags) ring[s % D] = src(s + D);
    return f;
  }
  __device__ __forceinline__ void operands() {
#pragma unroll
    for (int t = 0; t < 2; ++t) hb[t] = __builtin_bit_cast(bf16x8, u32x4{nx[4 * t], nx[4 * t + 1], nx[4 * t + 2], nx[4 * t + 3]});
  }
  __device__ __forceinline__ uint32_t relu_d(int d) { return relu_pair(c0[2 * d], c0[2 * d + 1]); }
  __device__ __forceinline__ void slot(f32x4& acc, const bf16x8& a, const bf16x8& b, bool zero) {
    __builtin_amdgcn_sched_barrier(0);
    const f32x4 z4 = {};
    acc = mfma16(a, b, zero ? z4 : acc);
  }
  __device__ __forceinline__ void pairs3(int t2, int t) {
    const int buf = (t2 >> 1) & 1, d = 2 * (t2 & 1);
    b3[buf][t][d] = relu_pair(acc2[t2][t][0], acc2[t2][t][1]);
    b3[buf][t][d + 1] = relu_pair(acc2[t2][t][2], acc2[t2][t][3]);
  }
  // fragment index consumed first by unit u (the take order of qnet_mlp)
  static constexpr int frag_of(int u) {
    return u == 0 ? 0 : u == 1 ? -1 : u < 50 ? ((u - 2) / 8) * 8 + 1 + (u - 2) % 8 : u < 61 ? 49 + (u - 50) : -1;
  }
  __device__ __forceinline__ void unit(const Src& src, int u, bf16x8 xb0, float (&q)[8]) {
    const f32x16 z16 = {};
    if (u == 0) {
#pragma unroll
      for (int s = 0; s < D; ++s) ring[s] = src(s);
      const bf16x8 a1 = take(src, 0);
      c0 = mfma32(a1, xb0, z16);
    } else if (u == 1) {
#pragma unroll
      for (int d = 0; d < 8; ++d) nx[d] = relu_d(d);
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) permlane16_swap(nx[qd], nx[4 + qd]);
      operands();
    } else if (u < 50) {
      const int kb = (u - 2) / 8, r = (u - 2) % 8;
      const int s = kb * 8 + 1 + r;
      if (r == 0) {
        const bf16x8 a1 = take(src, s);
        c0 = mfma32(a1, xb0, z16);
      } else {
        const int t2 = r - 1;
        const bf16x8 a2 = take(src, s);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          slot(acc2[t2][t], a2, hb[t], kb == 0);
          if (t2 >= 1 && t2 <= 2) nx[4 * (t2 - 1) + t] = relu_d(4 * (t2 - 1) + t);
          if (t2 == 5) {
            permlane16_swap(nx[t], nx[4 + t]);
            permlane16_swap(nx[2 + t], nx[6 + t]);
          }
        }
        if (t2 == 1) {  // the remaining pairs of the two tiles' halves (qnet_mlp: t < 4 at row tiles 1, 2)
          nx[2] = relu_d(2);
          nx[3] = relu_d(3);
        }
        if (t2 == 2) {
          nx[6] = relu_d(6);
          nx[7] = relu_d(7);
        }
        if (t2 == 6) operands();
      }
    } else if (u < 61) {
      const int k = u - 50;  // the tail: layer2(0,-1) layer2(1,0) layer2(2,1) layer3(0,2) layer2(3,-1)
                             // layer2(4,3) layer3(1,4) layer2(5,-1) layer2(6,5) layer3(2,6) layer3(3,-1)
      constexpr int kind[11] = {2, 2, 2, 3, 2, 2, 3, 2, 2, 3, 3};
      constexpr int idx[11] = {0, 1, 2, 0, 3, 4, 1, 5, 6, 2, 3};
      constexpr int prv[11] = {-1, 0, 1, 2, -1, 3, 4, -1, 5, 6, -1};
      const int s = 49 + k;
      if (kind[k] == 2) {
        const int t2 = idx[k], p = prv[k];
        const bf16x8 a2 = take(src, s);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          slot(acc2[t2][t], a2, hb[t], false);
          if (p >= 0) pairs3(p, t);
        }
      } else {
        const int k3 = idx[k], p = prv[k];
        const bf16x8 a3 = take(src, s);
        const int buf = k3 & 1;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if (2 * k3 + 1 >= kQT2) b3[buf][t][2] = b3[buf][t][3] = 0u;
          const bf16x8 b = __builtin_bit_cast(bf16x8, u32x4{b3[buf][t][0], b3[buf][t][1], b3[buf][t][2], b3[buf][t][3]});
          slot(acc3[t], a3, b, k3 == 0);
          if (p >= 0) pairs3(p, t);
        }
      }
    } else {
      const f32x4 z4 = {};
      f32x4 a4[4] = {acc3[0], acc3[1], z4, z4};
      qnet_gather_q(a4, q);
    }
  }
};

__device__ __forceinline__ bf16x8 input32(const float* tile, int row0, bool swap) {
  const int lane = threadIdx.x & 63;
  return qnet_input(tile + (row0 + (lane & 31)) * kObs, swap, lane >> 5);
}

// MODE 0: shipped NC 4 forward (64 envs); 1: shipped NC 2 forward twice (2 x 32 envs); 2: two NC 2
// forwards pipelined half a forward apart (2 x 32 envs per iteration, the pipeline primed once)
template <int WAVES, int MODE>
__global__ __launch_bounds__(64 * WAVES) void probe(const uint8_t* net, int iters, unsigned long long* cyc, float* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_net[kQNetBytes];
  __shared__ __attribute__((aligned(16))) float tile[64 * WAVES * kObs];
  qnet_to_lds(net, lds_net);
  for (int j = threadIdx.x; j < 64 * WAVES * kObs; j += blockDim.x) tile[j] = 0.01f * ((j * 37) % 101) - 0.5f;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row0 = wave * 64;
  float acc = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if constexpr (MODE == 0) {
    for (int it = 0; it < iters; ++it) {
      float q[8];
      qnet_forward_swp(lds_net, tile, row0, (it & 1) != 0, q);
      acc += q[0] + q[1] + q[2] + q[3] + q[4];
    }
  } else if constexpr (MODE == 1) {
    for (int it = 0; it < iters; ++it) {
      float q[8];
      const bool sw = (it & 1) != 0;
      qnet_mlp<kQLdsAhead, 2>(qnet_lds(lds_net), input32(tile, row0, sw), input32(tile, row0, sw), q);
      acc += q[0] + q[1] + q[2] + q[3] + q[4];
      qnet_mlp<kQLdsAhead, 2>(qnet_lds(lds_net), input32(tile, row0 + 32, sw), input32(tile, row0 + 32, sw), q);
      acc += q[0] + q[1] + q[2] + q[3] + q[4];
    }
  } else {
    using F = Fwd2<kQLdsAhead, QSrcLds>;
    F A, B;
    const QSrcLds srcA = qnet_lds(lds_net), srcB = qnet_lds(lds_net);
    float qa[8], qb[8];
    bf16x8 xa = input32(tile, row0, false), xb = input32(tile, row0 + 32, false);
    // prime: A's first half alone
#pragma unroll
    for (int u = 0; u < kHalfU; ++u) A.unit(srcA, u, xa, qa);
    for (int it = 0; it < iters; ++it) {
      const bool sw = (it & 1) != 0;
      xb = input32(tile, row0 + 32, sw);
#pragma unroll
      for (int u = 0; u < kHalfU; ++u) {  // A's second half beside B's first
        __builtin_amdgcn_sched_barrier(0);
        A.unit(srcA, kHalfU + u, xa, qa);
        __builtin_amdgcn_sched_barrier(0);
        B.unit(srcB, u, xb, qb);
      }
      acc += qa[0] + qa[1] + qa[2] + qa[3] + qa[4];
      xa = input32(tile, row0, !sw);
#pragma unroll
      for (int u = 0; u < kHalfU; ++u) {  // B's second half beside A's next first half
        __builtin_amdgcn_sched_barrier(0);
        B.unit(srcB, kHalfU + u, xb, qb);
        __builtin_amdgcn_sched_barrier(0);
        A.unit(srcA, u, xa, qa);
      }
      acc += qb[0] + qb[1] + qb[2] + qb[3] + qb[4];
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * WAVES + wave] = t1 - t0;
}

// bit check: one pipelined pair against qnet_mlp<D, 2> on the same inputs
__global__ __launch_bounds__(64) void check(const uint8_t* net, float* out_ref, float* out_pipe) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_net[kQNetBytes];
  __shared__ __attribute__((aligned(16))) float tile[64 * kObs];
  qnet_to_lds(net, lds_net);
  for (int j = threadIdx.x; j < 64 * kObs; j += blockDim.x) tile[j] = 0.013f * ((j * 41) % 97) - 0.4f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  float q[8];
  qnet_mlp<kQLdsAhead, 2>(qnet_lds(lds_net), input32(tile, 0, false), input32(tile, 0, false), q);
  for (int j = 0; j < 8; ++j) out_ref[lane * 16 + j] = q[j];
  qnet_mlp<kQLdsAhead, 2>(qnet_lds(lds_net), input32(tile, 32, false), input32(tile, 32, false), q);
  for (int j = 0; j < 8; ++j) out_ref[lane * 16 + 8 + j] = q[j];
  using F = Fwd2<kQLdsAhead, QSrcLds>;
  F A, B;
  const QSrcLds src = qnet_lds(lds_net);
  float qa[8], qb[8];
  const bf16x8 xa = input32(tile, 0, false), xb = input32(tile, 32, false);
#pragma unroll
  for (int u = 0; u < kHalfU; ++u) A.unit(src, u, xa, qa);
#pragma unroll
  for (int u = 0; u < kHalfU; ++u) {
    A.unit(src, kHalfU + u, xa, qa);
    B.unit(src, u, xb, qb);
  }
#pragma unroll
  for (int u = 0; u < kHalfU; ++u) B.unit(src, kHalfU + u, xb, qb);
  for (int j = 0; j < 8; ++j) {
    out_pipe[lane * 16 + j] = qa[j];
    out_pipe[lane * 16 + 8 + j] = qb[j];
  }
}

template <int WAVES, int MODE>
void run(const uint8_t* dnet, int blocks, int iters) {
  unsigned long long* dcyc;
  float* dout;
  (void)hipMalloc(&dcyc, sizeof(unsigned long long) * blocks * WAVES);
  (void)hipMalloc(&dout, sizeof(float) * blocks * 64 * WAVES);
  for (int rep = 0; rep < 2; ++rep) {
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
    std::printf("{\"forward\": \"%s\", \"q_waves_per_simd\": %d, \"cycles_per_64_envs\": %.0f, \"wall_ms\": %.3f}\n",
                MODE == 0 ? "shipped NC4" : MODE == 1 ? "shipped NC2 x 2" : "NC2 x 2 pipelined half a forward apart",
                WAVES / 4, mean / iters, ms);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  (void)hipFree(dcyc);
  (void)hipFree(dout);
}
}  // namespace

int main() {
  std::vector<uint16_t> h(kQNetBytes / 2);
  for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint16_t>(0x3C00 + (i * 7919) % 512);
  uint8_t* dnet;
  (void)hipMalloc(&dnet, kQNetBytes);
  (void)hipMemcpy(dnet, h.data(), kQNetBytes, hipMemcpyHostToDevice);
  float *r, *p;
  (void)hipMalloc(&r, 64 * 16 * 4);
  (void)hipMalloc(&p, 64 * 16 * 4);
  hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, dnet, r, p);
  std::vector<float> hr(64 * 16), hp(64 * 16);
  (void)hipMemcpy(hr.data(), r, hr.size() * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hp.data(), p, hp.size() * 4, hipMemcpyDeviceToHost);
  int same = 0;
  for (int i = 0; i < 64 * 16; ++i) same += (reinterpret_cast<uint32_t&>(hr[i]) == reinterpret_cast<uint32_t&>(hp[i]));
  std::printf("{\"bit_check\": \"%d of %d Q values equal\"}\n", same, 64 * 16);
  run<4, 0>(dnet, 256, 1000);
  run<4, 1>(dnet, 256, 1000);
  run<4, 2>(dnet, 256, 1000);
  run<8, 0>(dnet, 256, 1000);
  run<8, 2>(dnet, 256, 1000);
  (void)hipFree(dnet);
  return 0;
}
