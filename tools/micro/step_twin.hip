// The memory ceiling for mg_step_random's exact access pattern on gfx950.
//
// twin    : step_kernel's loads and stores (six f64 + one u16 state array read and written, two
//           i8 action arrays, f32x2 reward, two u8 flag arrays, the obs tile staged through LDS
//           and written as 16-byte stores), non-temporal output stores as built, and about ten
//           arithmetic instructions in place of the physics. 152 B per env.
// twin_s  : the same with every store a plain store (no non-temporal hint).
// twin_p  : twin with the four byte outputs (a1, a2, done, collision) as one interleaved u32.
// mix     : float4 streaming kernel with the same 50 : 102 read : write bytes (contiguous).
// copy    : float4 copy, 1 : 1 (MI355X_MICROARCH.md's 6.29 TB/s figure).
//
// hipcc --offload-arch=gfx950 -O3 -o step_twin step_twin.hip && ./step_twin [n_envs] [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int kBlock = 256, kObs = 10;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <bool NT, class T>
__device__ __forceinline__ void st(T* p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}

struct Arrays {
  double *p1, *v1, *p2, *v2, *r1, *r2;
  uint16_t* tf;
  int8_t *a1, *a2;
  float* rew;
  uint8_t *done, *coll;
  float* obs;
};

template <bool NT, bool PACK>
__global__ __launch_bounds__(kBlock) void twin(Arrays A, int64_t n, uint32_t k) {
  __shared__ __attribute__((aligned(16))) float tile[kBlock * kObs];
  const int tid = threadIdx.x;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock, i = base + tid;
  float o[kObs];
  if (i < n) {
    double p1 = A.p1[i], v1 = A.v1[i], p2 = A.p2[i], v2 = A.v2[i], r1 = A.r1[i], r2 = A.r2[i];
    uint16_t tf = A.tf[i];
    const uint32_t h = (static_cast<uint32_t>(i) * 2654435761u) ^ k;
    const int a1 = h % 5, a2 = (h >> 8) % 5;
    if (!PACK) {
      st<NT>(A.a1 + i, static_cast<int8_t>(a1));
      st<NT>(A.a2 + i, static_cast<int8_t>(a2));
    }
    v1 += 0.2 * a1; v2 += 0.2 * a2; p1 += v1; p2 += v2; r1 += 0.5; r2 -= 0.5;
    const bool done = (tf & 0x1FFF) > 2500;
    tf = done ? 0 : static_cast<uint16_t>(tf + 1);
    for (int j = 0; j < kObs; ++j) o[j] = static_cast<float>(j & 1 ? p1 - p2 : v1 + j);
    st<NT>(reinterpret_cast<f32x2*>(A.rew) + i, f32x2{static_cast<float>(r1), static_cast<float>(r2)});
    if (PACK) {  // the four byte outputs interleaved: one u32 per env
      st<NT>(reinterpret_cast<uint32_t*>(A.a1) + i, static_cast<uint32_t>(a1) | (a2 << 8) |
                                                        (static_cast<uint32_t>(done) << 16) |
                                                        (static_cast<uint32_t>(p1 == p2) << 24));
    } else {
      st<NT>(A.done + i, static_cast<uint8_t>(done));
      st<NT>(A.coll + i, static_cast<uint8_t>(p1 == p2));
    }
    A.p1[i] = p1; A.v1[i] = v1; A.p2[i] = p2; A.v2[i] = v2; A.r1[i] = r1; A.r2[i] = r2; A.tf[i] = tf;
  }
  // obs: rows staged through LDS, written as 16-byte stores (step_kernel's store_obs_tile)
  float2* t2 = reinterpret_cast<float2*>(tile + tid * kObs);
  for (int j = 0; j < kObs / 2; ++j) t2[j] = make_float2(o[2 * j], o[2 * j + 1]);
  __syncthreads();
  const int64_t rem = n - base;
  const int nrows = rem < kBlock ? static_cast<int>(rem) : kBlock;
  const int n4 = nrows * kObs / 4;
  f32x4* d4 = reinterpret_cast<f32x4*>(A.obs + base * kObs);
  const f32x4* s4 = reinterpret_cast<const f32x4*>(tile);
  for (int j = tid; j < n4; j += kBlock) st<NT>(d4 + j, s4[j]);
}

// twin_aos: the same bytes with the six f64 state values of an env as one 48-byte record
// (p1, v1, p2, v2, r1, r2), read and written by each wave as 3 KB of consecutive bytes: lane l
// moves 16-byte piece l + 64 j (j = 0..2) of the wave's 64 records through LDS (3 dwordx4 loads
// and stores per lane, one sequential stream instead of six strided ones). tf stays a u16 array.
template <bool NT>
__global__ __launch_bounds__(kBlock) void twin_aos(double* rec, Arrays A, int64_t n, uint32_t k) {
  __shared__ __attribute__((aligned(16))) float tile[kBlock * kObs];
  __shared__ __attribute__((aligned(16))) double srec[kBlock * 6];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock, i = base + tid;
  const int64_t wbase = base + 64 * w;
  f32x4* g4 = reinterpret_cast<f32x4*>(rec + wbase * 6);
  f32x4* l4 = reinterpret_cast<f32x4*>(srec + 64 * w * 6);
  const bool full = wbase + 64 <= n;
  if (full) {
    const f32x4 x0 = g4[lane], x1 = g4[lane + 64], x2 = g4[lane + 128];
    l4[lane] = x0; l4[lane + 64] = x1; l4[lane + 128] = x2;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  float o[kObs];
  double* r = srec + tid * 6;
  double p1 = r[0], v1 = r[1], p2 = r[2], v2 = r[3], r1 = r[4], r2 = r[5];
  uint16_t tf = i < n ? A.tf[i] : 0;
  const uint32_t h = (static_cast<uint32_t>(i) * 2654435761u) ^ k;
  const int a1 = h % 5, a2 = (h >> 8) % 5;
  v1 += 0.2 * a1; v2 += 0.2 * a2; p1 += v1; p2 += v2; r1 += 0.5; r2 -= 0.5;
  const bool done = (tf & 0x1FFF) > 2500;
  tf = done ? 0 : static_cast<uint16_t>(tf + 1);
  for (int j = 0; j < kObs; ++j) o[j] = static_cast<float>(j & 1 ? p1 - p2 : v1 + j);
  if (i < n) {
    st<NT>(reinterpret_cast<f32x2*>(A.rew) + i, f32x2{static_cast<float>(r1), static_cast<float>(r2)});
    st<NT>(reinterpret_cast<uint32_t*>(A.a1) + i, static_cast<uint32_t>(a1) | (a2 << 8) |
                                                      (static_cast<uint32_t>(done) << 16) |
                                                      (static_cast<uint32_t>(p1 == p2) << 24));
    A.tf[i] = tf;
  }
  r[0] = p1; r[1] = v1; r[2] = p2; r[3] = v2; r[4] = r1; r[5] = r2;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  if (full) {
    g4[lane] = l4[lane]; g4[lane + 64] = l4[lane + 64]; g4[lane + 128] = l4[lane + 128];
  }
  float2* t2 = reinterpret_cast<float2*>(tile + tid * kObs);
  for (int j = 0; j < kObs / 2; ++j) t2[j] = make_float2(o[2 * j], o[2 * j + 1]);
  __syncthreads();
  const int64_t rem = n - base;
  const int nrows = rem < kBlock ? static_cast<int>(rem) : kBlock;
  const int n4 = nrows * kObs / 4;
  f32x4* d4 = reinterpret_cast<f32x4*>(A.obs + base * kObs);
  const f32x4* s4 = reinterpret_cast<const f32x4*>(tile);
  for (int j = tid; j < n4; j += kBlock) st<NT>(d4 + j, s4[j]);
}

// Reads nr float4 and writes nw float4 per "unit"; units spread over a grid-stride loop.
__global__ __launch_bounds__(256) void mix(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                           int64_t nr4, int64_t nw4) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  for (int64_t j = g; j < nr4; j += stride) acc += src[j];
  for (int64_t j = g; j < nw4; j += stride) dst[j] = acc + static_cast<float>(j);
}

__global__ __launch_bounds__(256) void copy4(const f32x4* __restrict__ src, f32x4* __restrict__ dst, int64_t n4) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g < n4) dst[g] = src[g];
}

template <class F>
static float time_us(F launch, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < 50; ++r) launch(r);
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch(r);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipGetLastError());
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : (1 << 20);
  const int reps = argc > 2 ? std::atoi(argv[2]) : 1000;
  Arrays A;
  auto alloc = [](auto*& p, size_t bytes) { CHECK(hipMalloc(&p, bytes)); CHECK(hipMemset(p, 0, bytes)); };
  alloc(A.p1, n * 8); alloc(A.v1, n * 8); alloc(A.p2, n * 8); alloc(A.v2, n * 8);
  alloc(A.r1, n * 8); alloc(A.r2, n * 8); alloc(A.tf, n * 2); alloc(A.a1, n * 4); alloc(A.a2, n);
  alloc(A.rew, n * 8); alloc(A.done, n); alloc(A.coll, n); alloc(A.obs, n * 40);
  double* rec;
  alloc(rec, n * 48);
  const double bytes = 152.0 * n;
  const unsigned grid = static_cast<unsigned>((n + kBlock - 1) / kBlock);
  for (int rep = 0; rep < 2; ++rep) {
    float us = time_us([&](int r) { hipLaunchKernelGGL((twin<true, false>), dim3(grid), dim3(kBlock), 0, 0, A, n, r); }, reps);
    std::printf("twin   (NT outputs)  n=%lld: %8.2f us  %6.3f TB/s  (152 B/env)\n", (long long)n, us, bytes / us / 1e6);
    us = time_us([&](int r) { hipLaunchKernelGGL((twin<true, true>), dim3(grid), dim3(kBlock), 0, 0, A, n, r); }, reps);
    std::printf("twin_p (NT, packed u32 bytes): %8.2f us  %6.3f TB/s\n", us, bytes / us / 1e6);
    us = time_us([&](int r) { hipLaunchKernelGGL((twin<false, false>), dim3(grid), dim3(kBlock), 0, 0, A, n, r); }, reps);
    std::printf("twin_s (plain)               : %8.2f us  %6.3f TB/s\n", us, bytes / us / 1e6);
    us = time_us([&](int r) { hipLaunchKernelGGL((twin_aos<true>), dim3(grid), dim3(kBlock), 0, 0, rec, A, n, r); }, reps);
    std::printf("twin_aos (48-B state records): %8.2f us  %6.3f TB/s\n", us, bytes / us / 1e6);
  }
  float us;

  const int64_t nr4 = 50 * n / 16, nw4 = 102 * n / 16;
  f32x4 *src, *dst;
  alloc(src, nr4 * 16 > nw4 * 16 ? nr4 * 16 : nw4 * 16);
  alloc(dst, nw4 * 16 > nr4 * 16 ? nw4 * 16 : nr4 * 16);
  for (unsigned g : {1024u, 2048u, 4096u, 8192u}) {
    us = time_us([&](int) { hipLaunchKernelGGL(mix, dim3(g), dim3(256), 0, 0, src, dst, nr4, nw4); }, reps);
    std::printf("mix 50:102 grid %5u: %8.2f us  %6.3f TB/s\n", g, us, (nr4 + nw4) * 16.0 / us / 1e6);
  }
  const int64_t c4 = 76 * n / 16;  // 76 B read + 76 B written per env = 152 B
  us = time_us([&](int) { hipLaunchKernelGGL(copy4, dim3((c4 + 255) / 256), dim3(256), 0, 0, src, dst, c4); }, reps);
  std::printf("copy 1:1 (152 B/env)         : %8.2f us  %6.3f TB/s\n", us, 2.0 * c4 * 16 / us / 1e6);
  return 0;
}
