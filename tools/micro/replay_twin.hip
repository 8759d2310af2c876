// The memory ceiling for mg_replay_store's access pattern on gfx950.
//
// A store of a [T, N] trajectory reads, per transition, the 40-B observation row (the step's s'
// and, carried in registers, the next step's s), the interleaved flags word (a, done), the f32
// reward and 1/8 B of won bits, and writes one 88-B row [s, a, r, s'] (DESIGN.md "Replay
// memory": 137 algorithmic bytes per transition with the done rows' terminal observations).
//
// twin     : replay_write_kernel's structure (one block per 256 envs x 2 steps, the obs row of
//            step t kept as step t+1's s, the next row prefetched, rows gathered in an LDS tile,
//            written as 16-B non-temporal stores) with every transition kept and ring position
//            t*N + i: no scan launches, no wrap, no terminal rows.
// twin_nobar: the same with each wave writing its own 64 rows (its own contiguous run), so no
//            block barrier sits between a step's loads and its stores.
// mix      : a contiguous float4 stream with the same 49 : 88 read : write bytes, each block
//            reading its chunk and then writing its chunk (the store's shape without the rows).
// mix_il   : the same bytes interleaved per thread (one read, then its share of writes).
// rd / wr  : the read half alone, the write half alone (non-temporal float4 stores).
//
// hipcc --offload-arch=gfx950 -O3 -o replay_twin replay_twin.hip && ./replay_twin [n_envs] [T] [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int kObs = 10, kRow = 22, kRBlock = 256, kChunk = 2;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <class T>
__device__ __forceinline__ void st_nt(T* p, T v) { __builtin_nontemporal_store(v, p); }

__device__ __forceinline__ void load_row10(const float* src, float (&v)[kObs]) {
  const f32x2* s2 = reinterpret_cast<const f32x2*>(src);
#pragma unroll
  for (int k = 0; k < kObs / 2; ++k) {
    const f32x2 a = s2[k];
    v[2 * k] = a[0];
    v[2 * k + 1] = a[1];
  }
}

struct In {
  const float* obs;        // [T, n, 10]
  const float* obs_first;  // [n, 10]
  const uint8_t* flags;    // [T, n, 4]: a, _, done, _
  const float* reward;     // [T, n]
  const uint64_t* won;     // [T, n / 64]
  int64_t n;
  int T;
};

// WAVE_RUNS: each wave writes its own 64 rows; otherwise the block's 256 rows go out as one run.
template <bool WAVE_RUNS>
__global__ __launch_bounds__(kRBlock) void twin(const In X, float* rows) {
  __shared__ __attribute__((aligned(16))) float tile[kRBlock * kRow];
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kRBlock + threadIdx.x;
  const int t0 = blockIdx.y * kChunk, t1 = t0 + kChunk < X.T ? t0 + kChunk : X.T;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float s[kObs], o[kObs];
  load_row10(t0 == 0 ? X.obs_first + i * kObs : X.obs + ((t0 - 1) * X.n + i) * kObs, s);
  load_row10(X.obs + (t0 * X.n + i) * kObs, o);
  for (int t = t0; t < t1; ++t) {
    const int64_t row = static_cast<int64_t>(t) * X.n + i;
    float on[kObs];
    if (t + 1 < t1) load_row10(X.obs + (row + X.n) * kObs, on);
    const uint64_t w = X.won[row >> 6];
    const uint32_t fl = reinterpret_cast<const uint32_t*>(X.flags)[row];
    const float r = X.reward[row];
    // keep every transition, but make the won word and flags feed the row so they are loaded
    const float a = static_cast<float>(static_cast<int8_t>(fl & 0xff)) + (((w >> lane) & 1) ? 1e-30f : 0.0f);
    float* d = tile + threadIdx.x * kRow;
#pragma unroll
    for (int k = 0; k < kObs; ++k) {
      d[k] = s[k];
      d[kObs + 2 + k] = ((fl >> 16) & 0xff) ? o[k] * 1.0f : o[k];
    }
    d[kObs] = a;
    d[kObs + 1] = r;
    if constexpr (WAVE_RUNS) {
      __builtin_amdgcn_wave_barrier();
      // 64 rows = 1,408 floats = 352 float4 from this wave's quarter of the tile
      const f32x2* s2 = reinterpret_cast<const f32x2*>(tile + 64 * wave * kRow);
      f32x4* d4 = reinterpret_cast<f32x4*>(rows + (row - lane) * kRow);  // 16-B aligned: 64 rows
      for (int k = lane; k < 64 * kRow / 4; k += 64) {
        const f32x2 lo = s2[2 * k], hi = s2[2 * k + 1];
        st_nt(d4 + k, f32x4{lo[0], lo[1], hi[0], hi[1]});
      }
      __builtin_amdgcn_wave_barrier();
    } else {
      __syncthreads();
      const f32x2* s2 = reinterpret_cast<const f32x2*>(tile);
      f32x4* d4 = reinterpret_cast<f32x4*>(rows + (row - threadIdx.x) * kRow);
      for (int k = threadIdx.x; k < kRBlock * kRow / 4; k += kRBlock) {
        const f32x2 lo = s2[2 * k], hi = s2[2 * k + 1];
        st_nt(d4 + k, f32x4{lo[0], lo[1], hi[0], hi[1]});
      }
      __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < kObs; ++k) s[k] = o[k];
#pragma unroll
    for (int k = 0; k < kObs; ++k) o[k] = on[k];
  }
}

// Each block reads its nr float4 chunk, then writes its nw float4 chunk.
__global__ __launch_bounds__(256) void mix(const f32x4* __restrict__ src, f32x4* __restrict__ dst, int64_t cr,
                                           int64_t cw, int64_t nr4, int64_t nw4) {
  const int64_t r0 = blockIdx.x * cr, w0 = blockIdx.x * cw;
  f32x4 acc = {0, 0, 0, 0};
  for (int64_t j = r0 + threadIdx.x; j < r0 + cr && j < nr4; j += 256) acc += src[j];
  for (int64_t j = w0 + threadIdx.x; j < w0 + cw && j < nw4; j += 256) st_nt(dst + j, acc + static_cast<float>(j));
}

// Per thread: one float4 read, then its share of the writes (88 / 49 of them on average).
__global__ __launch_bounds__(256) void mix_il(const f32x4* __restrict__ src, f32x4* __restrict__ dst, int64_t nr4,
                                              int64_t nw4) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (g >= nr4) return;
  const f32x4 v = src[g];
  const int64_t w0 = g * nw4 / nr4, w1 = (g + 1) * nw4 / nr4;
  for (int64_t j = w0; j < w1; ++j) st_nt(dst + j, v + static_cast<float>(j));
}

__global__ __launch_bounds__(256) void rd(const f32x4* __restrict__ src, f32x4* __restrict__ dst, int64_t nr4) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (g >= nr4) return;
  const f32x4 v = src[g];
  if (v[0] == 12345.0f) dst[g] = v;  // never taken: keeps the load
}

__global__ __launch_bounds__(256) void wr(f32x4* __restrict__ dst, int64_t nw4) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (g < nw4) st_nt(dst + g, f32x4{1.0f, 2.0f, 3.0f, static_cast<float>(g)});
}

template <class F>
static float time_us(F launch, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < 5; ++r) launch();
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipGetLastError());
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : (1 << 20);
  const int T = argc > 2 ? std::atoi(argv[2]) : 16;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 50;
  if (n % 256 || T % kChunk) { std::printf("n must be a multiple of 256 and T of %d\n", kChunk); return 1; }
  const int64_t M = n * T;  // transitions
  In X;
  X.n = n;
  X.T = T;
  float *obs, *obs_first, *reward, *rows;
  uint8_t* flags;
  uint64_t* won;
  CHECK(hipMalloc(&obs, M * kObs * 4));
  CHECK(hipMalloc(&obs_first, n * kObs * 4));
  CHECK(hipMalloc(&flags, M * 4));
  CHECK(hipMalloc(&reward, M * 4));
  CHECK(hipMalloc(&won, M / 8));
  CHECK(hipMalloc(&rows, M * kRow * 4));
  CHECK(hipMemset(obs, 0, M * kObs * 4));
  CHECK(hipMemset(obs_first, 0, n * kObs * 4));
  CHECK(hipMemset(flags, 0, M * 4));
  CHECK(hipMemset(reward, 0, M * 4));
  CHECK(hipMemset(won, 0, M / 8));
  X.obs = obs;
  X.obs_first = obs_first;
  X.flags = flags;
  X.reward = reward;
  X.won = won;
  // algorithmic bytes as bench.py's replay leg counts them for a store with no done rows:
  // obs 40 + flags 4 + won 1/4 + reward 4 + row 88 per transition, obs_first 40 per env
  const double rbytes = M * (40.0 + 4.0 + 0.25 + 4.0), wbytes = M * 88.0, fbytes = n * 40.0;
  const double bytes = rbytes + wbytes + fbytes;
  const dim3 grid(static_cast<unsigned>(n / kRBlock), static_cast<unsigned>(T / kChunk));
  std::printf("n=%lld T=%d transitions=%lld  algorithmic %.3f GB (read %.3f, write %.3f)\n", (long long)n, T,
              (long long)M, bytes / 1e9, (rbytes + fbytes) / 1e9, wbytes / 1e9);
  for (int rep = 0; rep < 2; ++rep) {
    float us = time_us([&] { hipLaunchKernelGGL(twin<false>, grid, dim3(kRBlock), 0, 0, X, rows); }, reps);
    std::printf("twin       (block runs)      : %8.2f us  %6.3f TB/s  %.3f of 8\n", us, bytes / us / 1e6,
                bytes / us / 8e6);
    us = time_us([&] { hipLaunchKernelGGL(twin<true>, grid, dim3(kRBlock), 0, 0, X, rows); }, reps);
    std::printf("twin_nobar (wave runs)       : %8.2f us  %6.3f TB/s  %.3f of 8\n", us, bytes / us / 1e6,
                bytes / us / 8e6);
  }
  const int64_t nr4 = static_cast<int64_t>((rbytes + fbytes) / 16), nw4 = static_cast<int64_t>(wbytes / 16);
  f32x4* dst = reinterpret_cast<f32x4*>(rows);
  f32x4* big;  // a separate read buffer of the read half's size
  CHECK(hipMalloc(&big, nr4 * 16));
  CHECK(hipMemset(big, 0, nr4 * 16));
  const f32x4* src = big;
  for (int64_t blocks : {8192ll, 32768ll, 131072ll}) {
    const int64_t cr = (nr4 + blocks - 1) / blocks, cw = (nw4 + blocks - 1) / blocks;
    float us = time_us(
        [&] { hipLaunchKernelGGL(mix, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, 0, src, dst, cr, cw, nr4, nw4); },
        reps);
    std::printf("mix 49:88 blocks %6lld       : %8.2f us  %6.3f TB/s  %.3f of 8\n", (long long)blocks, us,
                (nr4 + nw4) * 16.0 / us / 1e6, (nr4 + nw4) * 16.0 / us / 8e6);
  }
  float us = time_us(
      [&] { hipLaunchKernelGGL(mix_il, dim3(static_cast<unsigned>((nr4 + 255) / 256)), dim3(256), 0, 0, src, dst, nr4, nw4); },
      reps);
  std::printf("mix_il (interleaved)         : %8.2f us  %6.3f TB/s  %.3f of 8\n", us, (nr4 + nw4) * 16.0 / us / 1e6,
              (nr4 + nw4) * 16.0 / us / 8e6);
  const float ur = time_us(
      [&] { hipLaunchKernelGGL(rd, dim3(static_cast<unsigned>((nr4 + 255) / 256)), dim3(256), 0, 0, src, dst, nr4); }, reps);
  std::printf("read half alone              : %8.2f us  %6.3f TB/s\n", ur, nr4 * 16.0 / ur / 1e6);
  const float uw = time_us(
      [&] { hipLaunchKernelGGL(wr, dim3(static_cast<unsigned>((nw4 + 255) / 256)), dim3(256), 0, 0, dst, nw4); }, reps);
  std::printf("write half alone             : %8.2f us  %6.3f TB/s\n", uw, nw4 * 16.0 / uw / 1e6);
  std::printf("read + write halves in sequence: %8.2f us  %6.3f TB/s  %.3f of 8\n", ur + uw,
              (nr4 + nw4) * 16.0 / (ur + uw) / 1e6, (nr4 + nw4) * 16.0 / (ur + uw) / 8e6);
  return 0;
}
