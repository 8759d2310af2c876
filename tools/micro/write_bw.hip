// Store-only streaming bandwidth on gfx950: the ceiling of a write-dominated kernel such as the
// fused rollout (58 B written per env-step against 6 B read). float4 stores over a buffer far
// past the 256 MB Infinity Cache, plain and non-temporal, grid-stride, several grid sizes; a
// float4 copy of the same bytes for reference.
//   hipcc --offload-arch=gfx950 -O3 -o write_bw write_bw.hip && ./write_bw [MiB] [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void fill(f32x4* d, size_t n4, float v) {
  const f32x4 x = {v, v + 1.f, v + 2.f, v + 3.f};
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += gridDim.x * 256ull) {
    if constexpr (NT) __builtin_nontemporal_store(x, d + i); else d[i] = x;
  }
}

__global__ __launch_bounds__(256) void copy(const f32x4* s, f32x4* d, size_t n4) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += gridDim.x * 256ull) d[i] = s[i];
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? std::atoll(argv[1]) : 1024;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 50;
  const size_t bytes = mib << 20, n4 = bytes / 16;
  f32x4 *a, *b;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMemset(a, 0, bytes));
  CHECK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int grid : {8192, 16384, 65536, static_cast<int>(n4 / 256)}) {
    for (int mode = 0; mode < 3; ++mode) {
      auto launch = [&](int r) {
        if (mode == 0) hipLaunchKernelGGL(fill<false>, dim3(grid), dim3(256), 0, 0, a, n4, float(r));
        if (mode == 1) hipLaunchKernelGGL(fill<true>, dim3(grid), dim3(256), 0, 0, a, n4, float(r));
        if (mode == 2) hipLaunchKernelGGL(copy, dim3(grid), dim3(256), 0, 0, b, a, n4);
      };
      for (int r = 0; r < 5; ++r) launch(r);
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) launch(r);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / reps;
      const double moved = (mode == 2 ? 2.0 : 1.0) * bytes;
      const char* names[3] = {"fill (plain stores)", "fill (NT stores)", "copy (read + write)"};
      std::printf("grid %6d  %-22s %8.1f us  %.3f TB/s (%zu MiB written)\n", grid, names[mode], us,
                  moved / (us * 1e-6) / 1e12, mib);
    }
  }
  return 0;
}
