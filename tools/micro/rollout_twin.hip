// The memory ceiling for mg_rollout_random's access pattern on gfx950 (round 4).
//
// twin    : rollout_kernel<true>'s loads and stores with a few arithmetic instructions in place of
//           the physics: the env's seven state arrays read once and written once per launch, then
//           per step t the observation rows of slice t staged per wave through LDS and written as
//           16-byte non-temporal stores (2,560 B per wave-step), the f32x2 rewards and the u32 step
//           record (non-temporal). 52 + 100 / T bytes per env-step, T = 16: 58.25 B.
// direct  : the same, observation rows stored straight from registers (five f32x2 per lane).
// twin2   : twin with two envs per lane: 5,120-byte observation pieces per wave-step.
// stream  : float4 non-temporal stores of the same total bytes, contiguous, one per thread.
//
// hipcc --offload-arch=gfx950 -O3 -o rollout_twin rollout_twin.hip && ./rollout_twin [n_envs] [T] [reps]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

constexpr int kBlock = 256, kObs = 10;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct Arrays {
  double *p1, *v1, *p2, *v2, *r1, *r2;
  uint16_t* tf;
  float* obs;  // [T, n, 10]
  float* rew;  // [T, n, 2]
  uint32_t* flags;  // [T, n]
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool DIRECT>
__global__ __launch_bounds__(kBlock) void twin(Arrays A, int64_t n, int T) {
  __shared__ __attribute__((aligned(16))) float tile[kBlock * kObs];
  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock, i = base + tid;
  const int64_t wbase = base + (tid & ~63);
  if (i >= n) return;  // n is a multiple of 256 here
  double p1 = A.p1[i], v1 = A.v1[i], p2 = A.p2[i], v2 = A.v2[i], r1 = A.r1[i], r2 = A.r2[i];
  uint16_t tf = A.tf[i];
  for (int t = 0; t < T; ++t) {
    const int64_t row = static_cast<int64_t>(t) * n + i;
    v1 += 0.2; v2 -= 0.2; p1 += v1; p2 += v2; r1 += 0.5; r2 -= 0.5;
    tf = static_cast<uint16_t>(tf + 1);
    float o[kObs];
#pragma unroll
    for (int j = 0; j < kObs; ++j) o[j] = static_cast<float>(j & 1 ? p1 - p2 : v1 + j);
    __builtin_nontemporal_store(f32x2{static_cast<float>(r1), static_cast<float>(r2)},
                                reinterpret_cast<f32x2*>(A.rew) + row);
    __builtin_nontemporal_store(static_cast<uint32_t>(tf) * 0x01010101u, A.flags + row);
    if constexpr (DIRECT) {
      f32x2* d = reinterpret_cast<f32x2*>(A.obs + row * kObs);
#pragma unroll
      for (int j = 0; j < kObs / 2; ++j) __builtin_nontemporal_store(f32x2{o[2 * j], o[2 * j + 1]}, d + j);
    } else {
      float* w = tile + (tid & ~63) * kObs;
      f32x2* t2 = reinterpret_cast<f32x2*>(w + lane * kObs);
#pragma unroll
      for (int j = 0; j < kObs / 2; ++j) t2[j] = f32x2{o[2 * j], o[2 * j + 1]};
      wave_sync();
      f32x4* d4 = reinterpret_cast<f32x4*>(A.obs + (static_cast<int64_t>(t) * n + wbase) * kObs);
      const f32x4* s4 = reinterpret_cast<const f32x4*>(w);
      const f32x4 a = s4[lane], b = s4[64 + lane], c = s4[128 + (lane & 31)];
      __builtin_nontemporal_store(a, d4 + lane);
      __builtin_nontemporal_store(b, d4 + 64 + lane);
      if (lane < 32) __builtin_nontemporal_store(c, d4 + 128 + lane);
      wave_sync();
    }
  }
  A.p1[i] = p1; A.v1[i] = v1; A.p2[i] = p2; A.v2[i] = v2; A.r1[i] = r1; A.r2[i] = r2; A.tf[i] = tf;
}

// twin2: two envs per lane (envs wbase + lane and wbase + 64 + lane of a 128-env wave piece), so a
// wave writes 5,120 contiguous bytes of observations per step instead of 2,560 (the pattern an
// ILP-2 rollout would have)
__global__ __launch_bounds__(kBlock) void twin2(Arrays A, int64_t n, int T) {
  __shared__ __attribute__((aligned(16))) float tile[2 * kBlock * kObs];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t wbase = static_cast<int64_t>(blockIdx.x) * 2 * kBlock + wave * 128;
  double p1[2], v1[2], r1[2], p2[2], v2[2], r2[2];
  uint16_t tf[2];
  for (int j = 0; j < 2; ++j) {
    const int64_t i = wbase + 64 * j + lane;
    p1[j] = A.p1[i]; v1[j] = A.v1[i]; r1[j] = A.r1[i]; p2[j] = A.p2[i]; v2[j] = A.v2[i]; r2[j] = A.r2[i];
    tf[j] = A.tf[i];
  }
  float* w = tile + wave * 128 * kObs;
  for (int t = 0; t < T; ++t) {
    for (int j = 0; j < 2; ++j) {
      const int64_t i = wbase + 64 * j + lane, row = static_cast<int64_t>(t) * n + i;
      v1[j] += 0.2; p1[j] += v1[j]; r1[j] += 0.5;
      __builtin_nontemporal_store(f32x2{static_cast<float>(r1[j]), static_cast<float>(p1[j])},
                                  reinterpret_cast<f32x2*>(A.rew) + row);
      __builtin_nontemporal_store(static_cast<uint32_t>(t) * 0x01010101u, A.flags + row);
      f32x2* t2 = reinterpret_cast<f32x2*>(w + (64 * j + lane) * kObs);
#pragma unroll
      for (int q = 0; q < kObs / 2; ++q) t2[q] = f32x2{static_cast<float>(p1[j]) + q, static_cast<float>(v1[j]) - q};
    }
    wave_sync();
    f32x4* d4 = reinterpret_cast<f32x4*>(A.obs + (static_cast<int64_t>(t) * n + wbase) * kObs);
    const f32x4* s4 = reinterpret_cast<const f32x4*>(w);
#pragma unroll
    for (int q = 0; q < 5; ++q) __builtin_nontemporal_store(s4[64 * q + lane], d4 + 64 * q + lane);
    wave_sync();
  }
  for (int j = 0; j < 2; ++j) {
    const int64_t i = wbase + 64 * j + lane;
    A.p1[i] = p1[j]; A.v1[i] = v1[j]; A.r1[i] = r1[j] + tf[j];
    A.p2[i] = p2[j] + 1.0; A.v2[i] = v2[j] - 1.0; A.r2[i] = r2[j] * 0.5; A.tf[i] = static_cast<uint16_t>(tf[j] + T);
  }
}

__global__ __launch_bounds__(kBlock) void stream(f32x4* dst, int64_t n4) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n4) __builtin_nontemporal_store(f32x4{1.f, 2.f, 3.f, static_cast<float>(i)}, dst + i);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : (1 << 20);
  const int T = argc > 2 ? std::atoi(argv[2]) : 16;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 50;
  Arrays A;
  double* st[6];
  for (auto& p : st) {
    CHECK(hipMalloc(&p, n * 8));
    CHECK(hipMemset(p, 0, n * 8));
  }
  A.p1 = st[0]; A.v1 = st[1]; A.p2 = st[2]; A.v2 = st[3]; A.r1 = st[4]; A.r2 = st[5];
  CHECK(hipMalloc(&A.tf, n * 2));
  CHECK(hipMalloc(&A.obs, n * T * kObs * 4));
  CHECK(hipMalloc(&A.rew, n * T * 8));
  CHECK(hipMalloc(&A.flags, n * T * 4));
  const double bytes = (52.0 + 100.0 / T) * n * T;
  const int64_t n4 = static_cast<int64_t>(bytes / 16);
  f32x4* big;
  CHECK(hipMalloc(&big, n4 * 16));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const dim3 grid(static_cast<unsigned>((n + kBlock - 1) / kBlock));
  for (int variant = 0; variant < 4; ++variant) {
    auto launch = [&]() {
      if (variant == 0) hipLaunchKernelGGL(twin<false>, grid, dim3(kBlock), 0, 0, A, n, T);
      else if (variant == 1) hipLaunchKernelGGL(twin<true>, grid, dim3(kBlock), 0, 0, A, n, T);
      else if (variant == 2) hipLaunchKernelGGL(twin2, dim3(static_cast<unsigned>(n / (2 * kBlock))), dim3(kBlock), 0, 0, A, n, T);
      else hipLaunchKernelGGL(stream, dim3(static_cast<unsigned>((n4 + kBlock - 1) / kBlock)), dim3(kBlock), 0, 0, big, n4);
    };
    for (int w = 0; w < 10; ++w) launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const char* name[] = {"twin", "direct", "twin2", "stream"};
    std::printf("{\"variant\": \"%s\", \"envs\": %lld, \"T\": %d, \"us_per_launch\": %.1f, \"us_per_step\": %.2f, "
                "\"TBps_at_%.2fB\": %.3f}\n",
                name[variant], static_cast<long long>(n), T, ms * 1e3, ms * 1e3 / T, 52.0 + 100.0 / T,
                bytes / (ms * 1e-3) / 1e12);
  }
  return 0;
}
