// fetch_calib.hip -- what rocprofv3's FETCH_SIZE reports on gfx950 for the
// engine's access widths (MI355X_MICROARCH.md: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
// Each kernel is one dispatch with a known number of distinct 128-B lines
// touched in a 4 GiB buffer (far past the 256 MiB Infinity Cache), so every
// access misses L2 and the L3; FETCH_SIZE per dispatch / lines touched gives
// the bytes the counter books per missed line for that access width.
//   stream16   1 GiB, 16 B per lane, coalesced (guide: reported at 1/2)
//   rand1      2^24 random lines, one 1-byte load each (the line-mask probe)
//   rand8      2^24 random lines, one 8-byte load each (the activity-bit probe)
//   row64      2^24 random 64-B rows (4 lanes x 16 B: half a line; the W = 8 shard rows)
//   line128    2^24 random lines, the whole 128-B line (8 lanes x 16 B)
//   row512     2^22 random 512-B rows (32 lanes x 16 B: 4 lines each)
// hipcc --offload-arch=gfx950 -O3 fetch_calib.hip -o fetch_calib
// rocprofv3 --pmc FETCH_SIZE --output-format csv -d out -o calib -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u64 mix(u64 x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void k_stream16(const u64x2* __restrict__ p, int64_t n, u64* __restrict__ sink) {
  u64x2 acc = {0, 0};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc |= p[i];
  if ((acc.x | acc.y) == 0x123456789ull) sink[0] = acc.x;
}

// one access per random line; `width` bytes at the start of the line
template <int WIDTH>
__global__ void k_rand(const uint8_t* __restrict__ p, int64_t nlines_buf, int64_t n, u64 seed, u64* __restrict__ sink) {
  u64 acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t line = (int64_t)(mix(seed + (u64)i) % (u64)nlines_buf);
    const uint8_t* q = p + line * 128;
    if constexpr (WIDTH == 1) acc += q[0];
    else acc += *reinterpret_cast<const u64*>(q);
  }
  if (acc == 0x123456789ull) sink[0] = acc;
}

// GROUP lanes x 16 B per random item (8: one 128-B line, 32: a 512-B row)
template <int GROUP>
__global__ void k_rand_rows(const uint8_t* __restrict__ p, int64_t nitems_buf, int64_t n, u64 seed,
                            u64* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int g = lane / GROUP, lw = lane % GROUP;
  constexpr int PER_WAVE = 64 / GROUP;
  u64x2 acc = {0, 0};
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave * PER_WAVE + g; i < n; i += nwaves * PER_WAVE) {
    const int64_t item = (int64_t)(mix(seed + (u64)i) % (u64)nitems_buf);
    acc |= *reinterpret_cast<const u64x2*>(p + item * (16 * GROUP) + lw * 16);
  }
  if ((acc.x | acc.y) == 0x123456789ull) sink[0] = acc.x;
}

// the line-mask round's pattern: GROUP lanes read a random 128-B line of the
// big buffer (a row piece) and lane 0 of the group probes one random byte of a
// small table (the nibble array, 8 MiB at C4: past one XCD's L2, inside the
// Infinity Cache).  FETCH_SIZE minus k_rand_rows<8>'s for the same count is
// what the probes cost at the memory-side counters.
__global__ void k_rows_probe(const uint8_t* __restrict__ p, int64_t nitems_buf, const uint8_t* __restrict__ tab,
                             int64_t tab_lines, int64_t n, u64 seed, u64* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int g = lane / 8, lw = lane % 8;
  u64x2 acc = {0, 0};
  u64 t = 0;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave * 8 + g; i < n; i += nwaves * 8) {
    const u64 h = mix(seed + (u64)i);
    acc |= *reinterpret_cast<const u64x2*>(p + (int64_t)(h % (u64)nitems_buf) * 128 + lw * 16);
    if (lw == 0) t += tab[(int64_t)((h >> 32) % (u64)tab_lines) * 128 + (h & 127)];
  }
  if ((acc.x | acc.y | t) == 0x123456789ull) sink[0] = acc.x;
}

int main() {
  const size_t bytes = size_t(4) << 30;
  uint8_t* buf = nullptr;
  u64* sink = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) {
    fprintf(stderr, "hipMalloc failed\n");
    return 1;
  }
  hipMemset(buf, 1, bytes);
  hipDeviceSynchronize();
  const int grid = 256 * 16, block = 256;
  const int64_t lines = (int64_t)(bytes / 128);
  // dispatch order (the CSV lists them in this order)
  hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(block), 0, 0, (const u64x2*)buf, (int64_t)((size_t(1) << 30) / 16), sink);
  hipLaunchKernelGGL(k_rand<1>, dim3(grid), dim3(block), 0, 0, buf, lines, int64_t(1) << 24, 11ull, sink);
  hipLaunchKernelGGL(k_rand<8>, dim3(grid), dim3(block), 0, 0, buf, lines, int64_t(1) << 24, 22ull, sink);
  hipLaunchKernelGGL(k_rand_rows<4>, dim3(grid), dim3(block), 0, 0, buf, lines, int64_t(1) << 24, 55ull, sink);
  hipLaunchKernelGGL(k_rand_rows<8>, dim3(grid), dim3(block), 0, 0, buf, lines, int64_t(1) << 24, 33ull, sink);
  hipLaunchKernelGGL(k_rand_rows<32>, dim3(grid), dim3(block), 0, 0, buf, (int64_t)(bytes / 512), int64_t(1) << 22,
                     44ull, sink);
  // an 8 MiB table (65536 lines) at the end of the buffer, probed 2^24 times
  // with 1-byte loads, twice (the second pass finds it warm in the Infinity
  // Cache): counted per probe if the memory-side counters see L3 hits
  const int64_t tab_lines = 65536;
  const uint8_t* tab = buf + bytes - tab_lines * 128;
  hipLaunchKernelGGL(k_rand<1>, dim3(grid), dim3(block), 0, 0, tab, tab_lines, int64_t(1) << 24, 66ull, sink);
  hipLaunchKernelGGL(k_rand<1>, dim3(grid), dim3(block), 0, 0, tab, tab_lines, int64_t(1) << 24, 77ull, sink);
  // rows alone, then rows with a probe of the table each (the line-mask round)
  hipLaunchKernelGGL(k_rand_rows<8>, dim3(grid), dim3(block), 0, 0, buf, lines - tab_lines, int64_t(1) << 24, 88ull,
                     sink);
  hipLaunchKernelGGL(k_rows_probe, dim3(grid), dim3(block), 0, 0, buf, lines - tab_lines, tab, tab_lines,
                     int64_t(1) << 24, 99ull, sink);
  if (hipDeviceSynchronize() != hipSuccess) {
    fprintf(stderr, "kernel failed\n");
    return 1;
  }
  printf("expected bytes touched: stream16 %zu, rand1 %lld lines, rand8 %lld lines, row64 (first half of) %lld lines, line128 %lld lines, "
         "row512 %lld rows (x4 lines); then rand1 on an 8 MiB table x2, line128 alone and with a table probe each, "
         "%lld each\n",
         size_t(1) << 30, 1ll << 24, 1ll << 24, 1ll << 24, 1ll << 24, 1ll << 22, 1ll << 24);
  hipFree(buf);
  hipFree(sink);
  return 0;
}
