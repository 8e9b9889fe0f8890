// Practical ceiling of the pull's memory pattern on MI355X: random whole-row
// gathers OR-reduced per receiver, without the engine's probes, column ids or
// bookkeeping.  Each wave takes receivers one at a time; a receiver ORs DEG
// rows picked at random (uniform, or degree-weighted like a Chung-Lu gamma =
// 2.5 overlay with hubs scattered by a bijective hash) and writes its result
// row.  Rows of 512 B (W = 64, C4/C5) and 64 B (W = 8, the 512-message shard).
//
// build:  hipcc -O3 --offload-arch=gfx950 gather_ceiling.hip -o gather_ceiling
// run:    ./gather_ceiling            (one JSON line per variant)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef uint64_t u64;
struct __attribute__((aligned(16))) u64x2 { u64 x, y; };

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ u64 mix(u64 z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// row picked for arc j: uniform, or i = n * u^3 (P(i) ~ i^(-2/3), the Chung-Lu
// weight of gamma = 2.5) relabelled by an odd multiplier mod 2^log2n
__device__ __forceinline__ int64_t pick(u64 j, int log2n, int skew) {
  const u64 n = 1ull << log2n;
  const u64 h = mix(j * 0x9e3779b97f4a7c15ull + 12345);
  if (!skew) return (int64_t)(h & (n - 1));
  const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
  u64 i = (u64)((double)n * u * u * u);
  if (i >= n) i = n - 1;
  return (int64_t)(((i + 1) * 0x9e3779b97f4a7c15ull) & (n - 1));
}

// W words per row; LPR = W / 2 lanes per row, RPI = 64 / LPR rows per
// wave-instruction, RIF instructions in flight per lane
template <int W, int RIF, int DEG>
__global__ __launch_bounds__(256) void k_gather(const u64* __restrict__ table, u64* __restrict__ out,
                                                int64_t receivers, int log2n, int skew) {
  constexpr int LPR = W / 2, RPI = 64 / LPR;
  const int lane = threadIdx.x & 63, g = lane / LPR, lw = lane % LPR;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wave; r < receivers; r += waves) {
    u64x2 acc = {0, 0};
    for (int k0 = 0; k0 < DEG; k0 += RIF * RPI) {
      u64x2 v[RIF];
#pragma unroll
      for (int q = 0; q < RIF; ++q) {
        const int k = k0 + g + q * RPI;
        v[q] = u64x2{0, 0};
        if (k < DEG) {
          const int64_t row = pick((u64)r * DEG + k, log2n, skew);
          v[q] = *reinterpret_cast<const u64x2*>(table + row * W + lw * 2);
        }
      }
#pragma unroll
      for (int q = 0; q < RIF; ++q) {
        acc.x |= v[q].x;
        acc.y |= v[q].y;
      }
    }
#pragma unroll
    for (int s = LPR; s < 64; s <<= 1) {
      acc.x |= __shfl_xor(acc.x, s);
      acc.y |= __shfl_xor(acc.y, s);
    }
    if (g == 0) *reinterpret_cast<u64x2*>(out + (r & ((1ll << log2n) - 1)) * W + lw * 2) = acc;
  }
}

__global__ void k_fill(u64* t, int64_t words) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x)
    t[i] = mix((u64)i);
}

template <int W, int RIF, int DEG>
static void run(const char* name, u64* table, u64* out, int log2n, int skew, int64_t receivers, int cus) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int grid = cus * 8;   // 32 waves per CU
  hipLaunchKernelGGL((k_gather<W, RIF, DEG>), dim3(grid), dim3(256), 0, 0, table, out, receivers, log2n, skew);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int it = 0; it < 3; ++it) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_gather<W, RIF, DEG>), dim3(grid), dim3(256), 0, 0, table, out, receivers, log2n, skew);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double rows = (double)receivers * DEG;
  const double rbytes = rows * 8.0 * W, wbytes = (double)receivers * 8.0 * W;
  printf("{\"variant\": \"%s\", \"row_bytes\": %d, \"rows_per_receiver\": %d, \"rows_in_flight\": %d, "
         "\"skew\": %d, \"rows\": %.0f, \"ms\": %.3f, \"row_GBs\": %.1f, \"rows_per_s_G\": %.2f, "
         "\"read_plus_write_GBs\": %.1f}\n",
         name, 8 * W, DEG, RIF, skew, rows, best, rbytes / best / 1e6, rows / best / 1e6,
         (rbytes + wbytes) / best / 1e6);
  fflush(stdout);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int log2n = 24;   // 2^24 rows, as C4
  u64 *table = nullptr, *out = nullptr;
  const int64_t words = (1ll << log2n) * 64;   // 8 GiB at W = 64
  CHECK(hipMalloc(&table, words * 8));
  CHECK(hipMalloc(&out, words * 8));
  hipLaunchKernelGGL(k_fill, dim3(cus * 8), dim3(256), 0, 0, table, words);
  CHECK(hipDeviceSynchronize());
  const int64_t recv = 1ll << 24;   // 16 M receivers x 16 rows = 268 M rows (a C4 dense round)
  run<64, 4, 16>("W64 uniform", table, out, log2n, 0, recv, cus);
  run<64, 4, 16>("W64 chung-lu", table, out, log2n, 1, recv, cus);
  run<64, 2, 16>("W64 uniform rif2", table, out, log2n, 0, recv, cus);
  run<64, 8, 16>("W64 uniform rif8", table, out, log2n, 0, recv, cus);
  run<8, 3, 16>("W8 uniform", table, out, log2n, 0, recv, cus);
  run<8, 3, 16>("W8 chung-lu", table, out, log2n, 1, recv, cus);
  CHECK(hipFree(table));
  CHECK(hipFree(out));
  return 0;
}
