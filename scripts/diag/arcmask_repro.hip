// Standalone reproducer for the k_arcmask store finding (DESIGN.md §3.7;
// VERDICT r1 item 7): per-arc activity mask words, one 64-arc word per ballot,
// AM_WORDS ballots per wave, written by four store patterns and compared with a
// host reference over random inputs.
//   K0  lane 0 stores each ballot as it is formed (the engine's form)
//   K1  the four ballots selected into lanes 0-3 by chained ternaries, one store
//   K2  the four ballots selected by a dynamic register-array index, one store
//   K3  the four ballots staged through LDS by lane 0, read back by lanes 0-3, one store
//   K4  K2 with an `s_nop 4` after each ballot (does padding alone fix it?)
//   K5  K2 with each ballot's condition materialised in a VGPR behind an asm
//       barrier before the ballot
// build: hipcc -O3 --offload-arch=gfx950 arcmask_repro.hip -o arcmask_repro
// run:   ./arcmask_repro [log2_words] [trials]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned long long u64;
constexpr int AM_WORDS = 4;
constexpr int BLOCK = 256, WAVES = 4;

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                        \
    }                                                                                 \
  } while (0)

template <int VAR>
__global__ __launch_bounds__(BLOCK) void k_mask(const int32_t* __restrict__ gcol, const u64* __restrict__ abits,
                                                u64* __restrict__ amask, int64_t nnz) {
  const int lane = threadIdx.x & 63;
  const int64_t k0 = ((int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6)) * AM_WORDS;
  if (k0 * 64 >= nnz) return;
  int32_t u[AM_WORDS];
#pragma unroll
  for (int q = 0; q < AM_WORDS; ++q) {
    const int64_t e = (k0 + q) * 64 + lane;
    u[q] = e < nnz ? gcol[e] : -1;
  }
  u64 w[AM_WORDS];
#pragma unroll
  for (int q = 0; q < AM_WORDS; ++q) w[q] = u[q] >= 0 ? abits[u[q] >> 6] : 0ull;
  if constexpr (VAR == 0) {
#pragma unroll
    for (int q = 0; q < AM_WORDS; ++q) {
      const u64 m = __ballot(u[q] >= 0 && ((w[q] >> (u[q] & 63)) & 1ull));
      if (lane == 0 && (k0 + q) * 64 < nnz) amask[k0 + q] = m;
    }
  } else {
    u64 m[AM_WORDS];
    if constexpr (VAR == 4) {
#pragma unroll
      for (int q = 0; q < AM_WORDS; ++q) {
        m[q] = __ballot(u[q] >= 0 && ((w[q] >> (u[q] & 63)) & 1ull));
        asm volatile("s_nop 4" ::: "memory");
      }
    } else if constexpr (VAR == 5) {
#pragma unroll
      for (int q = 0; q < AM_WORDS; ++q) {
        int c = (u[q] >= 0 && ((w[q] >> (u[q] & 63)) & 1ull)) ? 1 : 0;
        asm volatile("" : "+v"(c));
        m[q] = __ballot(c != 0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < AM_WORDS; ++q) m[q] = __ballot(u[q] >= 0 && ((w[q] >> (u[q] & 63)) & 1ull));
    }
    u64 sel = 0;
    if constexpr (VAR == 1) {
      sel = lane == 0 ? m[0] : lane == 1 ? m[1] : lane == 2 ? m[2] : m[3];
    } else if constexpr (VAR == 2 || VAR == 4 || VAR == 5) {
      sel = m[lane & (AM_WORDS - 1)];
    } else {
      __shared__ u64 stage[WAVES][AM_WORDS];
      const int wib = threadIdx.x >> 6;
      if (lane == 0)
#pragma unroll
        for (int q = 0; q < AM_WORDS; ++q) stage[wib][q] = m[q];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane < AM_WORDS) sel = stage[wib][lane];
    }
    if (lane < AM_WORDS && (k0 + lane) * 64 < nnz) amask[k0 + lane] = sel;
  }
}

static uint64_t rng(uint64_t& s) {
  s += 0x9E3779B97F4A7C15ull;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  const int lw = argc > 1 ? atoi(argv[1]) : 22;
  const int trials = argc > 2 ? atoi(argv[2]) : 4;
  const int64_t words = 1ll << lw, n = 1 << 24;
  constexpr int NV = 6;
  long bad[NV] = {0, 0, 0, 0, 0, 0};
  int32_t* d_gcol;
  u64 *d_abits, *d_mask;
  CHECK(hipMalloc(&d_gcol, words * 64 * 4));
  CHECK(hipMalloc(&d_abits, n / 64 * 8));
  CHECK(hipMalloc(&d_mask, words * 8));
  std::vector<int32_t> gcol(words * 64);
  std::vector<u64> abits(n / 64), ref(words), got(words);
  uint64_t s = 12345;
  for (int t = 0; t < trials; ++t) {
    const int64_t nnz = words * 64 - (int64_t)(rng(s) % 64);   // a ragged last word
    for (auto& c : gcol) c = (int32_t)(rng(s) % n);
    const uint64_t dens = rng(s) % 4;   // 1/16 .. all active
    for (auto& b : abits) {
      b = rng(s);
      for (uint64_t k = 0; k < dens; ++k) b &= rng(s);
      if (dens == 3 && (rng(s) & 1)) b = ~0ull;
    }
    for (int64_t k = 0; k < words; ++k) {
      u64 m = 0;
      for (int l = 0; l < 64; ++l) {
        const int64_t e = k * 64 + l;
        if (e < nnz && ((abits[gcol[e] >> 6] >> (gcol[e] & 63)) & 1ull)) m |= 1ull << l;
      }
      ref[k] = m;
    }
    CHECK(hipMemcpy(d_gcol, gcol.data(), words * 64 * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_abits, abits.data(), n / 64 * 8, hipMemcpyHostToDevice));
    const dim3 grid((unsigned)((words + WAVES * AM_WORDS - 1) / (WAVES * AM_WORDS)));
    for (int var = 0; var < NV; ++var) {
      CHECK(hipMemset(d_mask, 0xA5, words * 8));
      switch (var) {
        case 0: hipLaunchKernelGGL(k_mask<0>, grid, dim3(BLOCK), 0, 0, d_gcol, d_abits, d_mask, nnz); break;
        case 1: hipLaunchKernelGGL(k_mask<1>, grid, dim3(BLOCK), 0, 0, d_gcol, d_abits, d_mask, nnz); break;
        case 2: hipLaunchKernelGGL(k_mask<2>, grid, dim3(BLOCK), 0, 0, d_gcol, d_abits, d_mask, nnz); break;
        case 3: hipLaunchKernelGGL(k_mask<3>, grid, dim3(BLOCK), 0, 0, d_gcol, d_abits, d_mask, nnz); break;
        case 4: hipLaunchKernelGGL(k_mask<4>, grid, dim3(BLOCK), 0, 0, d_gcol, d_abits, d_mask, nnz); break;
        default: hipLaunchKernelGGL(k_mask<5>, grid, dim3(BLOCK), 0, 0, d_gcol, d_abits, d_mask, nnz); break;
      }
      CHECK(hipGetLastError());
      CHECK(hipMemcpy(got.data(), d_mask, words * 8, hipMemcpyDeviceToHost));
      long b = 0;
      for (int64_t k = 0; k < words; ++k) {
        if (got[k] != ref[k]) {
          // forensics: is the wrong word the mask of another word of the wave,
          // or this word's mask with another word's bitmap words, or with the
          // load's ADDRESS still in the register (a load consumed early)?
          const int64_t k0 = k - k % AM_WORDS;
          int other = -1, wsrc = -1, addr = 0, diffl = 0;
          for (int q = 0; q < AM_WORDS; ++q)
            if (k0 + q != k && got[k] == ref[k0 + q]) other = q;
          u64 ma = 0;
          for (int l = 0; l < 64; ++l) {
            const int64_t e = k * 64 + l;
            if (e >= nnz) continue;
            const u64 av = (u64)(((uint32_t)gcol[e] >> 3) & 0x1ffffff8u);
            if ((av >> (gcol[e] & 63)) & 1ull) ma |= 1ull << l;
          }
          addr = got[k] == ma;
          for (int q = 0; q < AM_WORDS; ++q) {
            u64 mq = 0;
            for (int l = 0; l < 64; ++l) {
              const int64_t e = k * 64 + l, eq = (k0 + q) * 64 + l;
              if (e >= nnz || eq >= nnz) continue;
              if ((abits[gcol[eq] >> 6] >> (gcol[e] & 63)) & 1ull) mq |= 1ull << l;
            }
            if (k0 + q != k && got[k] == mq) wsrc = q;
          }
          diffl = __builtin_popcountll(got[k] ^ ref[k]);
          if (b < 2)
            printf("  trial %d K%d word %lld (q %lld): got %016llx ref %016llx  bits differ %d, other-word %d, "
                   "w-of-word %d, address-as-data %d\n", t, var, (long long)k, (long long)(k % AM_WORDS), got[k],
                   ref[k], diffl, other, wsrc, addr);
          ++b;
        }
      }
      bad[var] += b;
    }
    printf("trial %d: %lld words, density class %llu: bad K0 %ld K1 %ld K2 %ld K3 %ld K4 %ld K5 %ld\n", t,
           (long long)words, (unsigned long long)dens, bad[0], bad[1], bad[2], bad[3], bad[4], bad[5]);
    fflush(stdout);
  }
  CHECK(hipFree(d_gcol));
  CHECK(hipFree(d_abits));
  CHECK(hipFree(d_mask));
  printf("total bad words: K0 %ld K1 %ld K2 %ld K3 %ld K4 %ld K5 %ld\n", bad[0], bad[1], bad[2], bad[3], bad[4],
         bad[5]);
  long any = 0;
  for (int v = 0; v < NV; ++v) any += bad[v];
  return any ? 1 : 0;
}
