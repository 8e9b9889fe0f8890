// bitcount.hip -- per-message coverage and forwards of a finished run
// (DESIGN.md §3.6), the pass gp_finalize_messages makes
// over every Message-List:
//   coverage[m] = #vertices holding m
//   forwards[m] = sum of deg(v) over the holders v of m (no liveness: by
//                 forward-once every holder sent m once to each of its links,
//                 Peer.py:402-404)
//
// A per-bit loop costs 64 adds per 8-B word and made this pass VALU-bound
// (12.4 ms for C4's 8 GiB of rows).  Here each lane owns one word position w
// of the rows and counts its 64 bit-columns bit-sliced (Harley-Seal carry-save
// adders): 8 rows at a time go through a CSA tree into "ones / twos / fours"
// planes plus 8 planes of eights, ~15 VALU ops per word instead of 64+, so the
// pass runs at the rate the rows stream in.  The planes are expanded into
// per-bit counts (and added to LDS) only when they fill (2047 rows) or, for
// the weighted sum, when the weight changes: the rows are visited in order of
// (degree, vertex) -- keys sorted once per overlay -- so a wave sees long runs
// of equal weight and flushes count x deg once per run.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <rocprim/device/device_radix_sort.hpp>

#include "gp_internal.h"

namespace gp {

constexpr int BC_BLOCK = 256;
constexpr int BC_WAVES = BC_BLOCK / 64;
constexpr int BC_MAXCNT = 2047;   // what ones/twos/fours + 8 planes of eights can hold
constexpr uint8_t BC_SLOT_NONE = 0xFF;

struct BitcountArgs {
  const u64* slot[3];               // Message-List slots; row v = slot[sp[v]][v] (sp 0xFF: empty; 2: parked)
  const uint8_t* __restrict__ sp;
  const u64* __restrict__ keys;     // [count] sorted (deg << 32 | v), or null: position = vertex, unweighted
  int64_t count;
  const u64* __restrict__ dcount;   // k_bitcount_tail: the count lives on the device (else null)
  uint32_t* __restrict__ part;      // [gridDim.x][2][W * 64] per-block counts / weighted sums
};

__device__ __forceinline__ void csa(u64& h, u64& l, u64 a, u64 b, u64 c) {
  const u64 u = a ^ b;
  h = (a & b) | (u & c);
  l = u ^ c;
}

template <int W, bool KEYED>
__global__ __launch_bounds__(BC_BLOCK) void k_bitcount(BitcountArgs a) {
  constexpr int RPI = 64 / W;   // rows per wave-instruction: lane = (row slot q, word w)
  constexpr int M = W * 64;
  __shared__ uint32_t lc[M];            // [bit][word]: lanes of one instruction hit distinct banks
  __shared__ uint32_t ls[KEYED ? M : 1];
  for (int t = threadIdx.x; t < M; t += BC_BLOCK) {
    lc[t] = 0u;
    if (KEYED) ls[t] = 0u;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int w = lane % W, q = lane / W;
  const int64_t nw = (int64_t)gridDim.x * BC_WAVES;
  const int64_t wid = (int64_t)blockIdx.x * BC_WAVES + wib;
  const int64_t per = ((a.count + nw - 1) / nw + RPI - 1) / RPI * RPI;
  const int64_t p0 = std::min(a.count, wid * per), p1 = std::min(a.count, p0 + per);

  u64 o1 = 0, o2 = 0, o4 = 0, e[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = 0;
  int held = 0;          // rows in the planes (uniform within a row slot)
  uint32_t cur_d = 0;    // their weight
  auto flush = [&]() {
#pragma unroll 4
    for (int b = 0; b < 64; ++b) {
      uint32_t hi = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) hi |= (uint32_t)((e[j] >> b) & 1ull) << j;
      const uint32_t cnt = (uint32_t)((o1 >> b) & 1ull) + 2u * (uint32_t)((o2 >> b) & 1ull) +
                           4u * (uint32_t)((o4 >> b) & 1ull) + 8u * hi;
      if (cnt) {
        atomicAdd(&lc[b * W + w], cnt);
        if (KEYED) atomicAdd(&ls[b * W + w], cnt * cur_d);
      }
    }
    o1 = o2 = o4 = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = 0;
    held = 0;
  };

  // Software pipeline, one memory latency per 8 rows: iteration i issues the
  // slot bytes of group i + 1 (its keys arrived during iteration i - 1), the
  // keys of group i + 2 and the rows of group i together, then waits once.
  // A group is the next <= 8 positions of this lane slot with equal weight.
  struct Group {
    int64_t p;        // first position
    int32_t v[8];     // vertices (k < K)
    int K;            // rows in the group (0: past the range)
    uint32_t d;       // their weight
  };
  auto keys_at = [&](int64_t pp, u64* kk) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t pk = pp + (int64_t)k * RPI;
      kk[k] = (KEYED && pk < p1) ? a.keys[pk] : ~0ull;
    }
  };
  auto make_group = [&](int64_t pp, const u64* kk) {
    Group g;
    g.p = pp;
    if (pp >= p1) {
      g.K = 0;
      g.d = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) g.v[k] = 0;
      return g;
    }
    if constexpr (KEYED) {
      g.d = (uint32_t)(kk[0] >> 32);
      g.K = 1;
      bool run = true;
#pragma unroll
      for (int k = 1; k < 8; ++k) {   // the leading rows of the same weight (keys are sorted)
        run = run && kk[k] != ~0ull && (uint32_t)(kk[k] >> 32) == g.d;
        g.K += run ? 1 : 0;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) g.v[k] = (int32_t)(uint32_t)kk[k];
    } else {
      g.d = 0;
      g.K = (int)std::min<int64_t>(8, (p1 - pp + RPI - 1) / RPI);
#pragma unroll
      for (int k = 0; k < 8; ++k) g.v[k] = (int32_t)(pp + (int64_t)k * RPI);
    }
    return g;
  };
  auto slots_of = [&](const Group& g, uint32_t* sl) {
#pragma unroll
    for (int k = 0; k < 8; ++k) sl[k] = k < g.K ? (uint32_t)a.sp[g.v[k]] : (uint32_t)BC_SLOT_NONE;
  };

  u64 kk[8];
  keys_at(p0 + q, kk);
  Group ga = make_group(p0 + q, kk);
  uint32_t sa[8];
  slots_of(ga, sa);
  int64_t pb = ga.p + (int64_t)ga.K * RPI;
  keys_at(pb, kk);
  while (__any(ga.K > 0)) {
    if (ga.K > 0) {
      const Group gb = make_group(pb, kk);
      uint32_t sb[8];
      slots_of(gb, sb);
      pb = gb.p + (int64_t)gb.K * RPI;
      keys_at(pb, kk);   // group i + 2
      if (KEYED ? (held > 0 && (ga.d != cur_d || held + 8 > BC_MAXCNT)) : (held + 8 > BC_MAXCNT)) flush();
      cur_d = ga.d;
      u64 x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        x[k] = sa[k] != BC_SLOT_NONE ? a.slot[sa[k]][(int64_t)ga.v[k] * W + w] : 0ull;
      u64 t2a, t2b, t4a, t4b, t8;
      csa(t2a, o1, o1, x[0], x[1]);
      csa(t2b, o1, o1, x[2], x[3]);
      csa(t4a, o2, o2, t2a, t2b);
      csa(t2a, o1, o1, x[4], x[5]);
      csa(t2b, o1, o1, x[6], x[7]);
      csa(t4b, o2, o2, t2a, t2b);
      csa(t8, o4, o4, t4a, t4b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const u64 cj = e[j] & t8;
        e[j] ^= t8;
        t8 = cj;
      }
      held += 8;   // capacity bookkeeping: at most 8 rows entered
      ga = gb;
#pragma unroll
      for (int k = 0; k < 8; ++k) sa[k] = sb[k];
    }
  }
  if (held > 0) flush();
  __syncthreads();
  uint32_t* out = a.part + (size_t)blockIdx.x * 2 * M;
  for (int t = threadIdx.x; t < M; t += BC_BLOCK) {
    out[t] = lc[t];
    out[M + t] = KEYED ? ls[t] : 0u;
  }
}

// Unweighted count at W = 64 (coverage of a churn run: every row, in vertex
// order).  Lean enough for 8 waves per SIMD: a wave walks 16 consecutive
// vertices per step, their 16 slot bytes are two 8-B loads made wave-uniform
// (so each row's slot pointer is a scalar select) and issued one step ahead,
// and the 16 rows (8 KB per wave) go in flight together.  k_bitcount kept
// 4 KB in flight at 4 waves per SIMD and read C5's 32 GiB at 2.7 TB/s.
__device__ __forceinline__ u64 sp_word(const uint8_t* __restrict__ sp, int64_t v, int64_t count) {
  if (v + 8 <= count) return *reinterpret_cast<const u64*>(sp + v);
  u64 w = ~0ull;   // past the range: empty rows
  for (int k = 0; k < 8; ++k)
    if (v + k < count) w = (w & ~(0xFFull << (8 * k))) | ((u64)sp[v + k] << (8 * k));
  return w;
}
__global__ __launch_bounds__(BC_BLOCK) void k_bitcount_lin(BitcountArgs a) {
  constexpr int W = 64, M = W * 64;
  __shared__ uint32_t lc[M];
  for (int t = threadIdx.x; t < M; t += BC_BLOCK) lc[t] = 0u;
  __syncthreads();
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int64_t nw = (int64_t)gridDim.x * BC_WAVES;
  const int64_t wid = (int64_t)blockIdx.x * BC_WAVES + wib;
  const int64_t groups = (a.count + 15) / 16;
  const int64_t per = (groups + nw - 1) / nw;
  const int64_t g0 = std::min(groups, wid * per), g1 = std::min(groups, g0 + per);
  u64 o1 = 0, o2 = 0, o4 = 0, e[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = 0;
  int held = 0;
  auto flush = [&]() {
#pragma unroll 4
    for (int b = 0; b < 64; ++b) {
      uint32_t hi = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) hi |= (uint32_t)((e[j] >> b) & 1ull) << j;
      const uint32_t cnt = (uint32_t)((o1 >> b) & 1ull) + 2u * (uint32_t)((o2 >> b) & 1ull) +
                           4u * (uint32_t)((o4 >> b) & 1ull) + 8u * hi;
      if (cnt) atomicAdd(&lc[b * W + lane], cnt);
    }
    o1 = o2 = o4 = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = 0;
    held = 0;
  };
  auto add8 = [&](const u64* x) {
    u64 t2a, t2b, t4a, t4b, t8;
    csa(t2a, o1, o1, x[0], x[1]);
    csa(t2b, o1, o1, x[2], x[3]);
    csa(t4a, o2, o2, t2a, t2b);
    csa(t2a, o1, o1, x[4], x[5]);
    csa(t2b, o1, o1, x[6], x[7]);
    csa(t4b, o2, o2, t2a, t2b);
    csa(t8, o4, o4, t4a, t4b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const u64 cj = e[j] & t8;
      e[j] ^= t8;
      t8 = cj;
    }
  };
  u64 s0 = 0, s1 = 0;
  if (g0 < g1) {
    s0 = sp_word(a.sp, g0 * 16, a.count);
    s1 = sp_word(a.sp, g0 * 16 + 8, a.count);
  }
  for (int64_t g = g0; g < g1; ++g) {
    const u64 c0 = (u64)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)s0) |
                   ((u64)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(s0 >> 32)) << 32);
    const u64 c1 = (u64)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)s1) |
                   ((u64)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(s1 >> 32)) << 32);
    if (g + 1 < g1) {   // the next step's slot bytes, in flight with this step's rows
      s0 = sp_word(a.sp, (g + 1) * 16, a.count);
      s1 = sp_word(a.sp, (g + 1) * 16 + 8, a.count);
    }
    const int64_t v0 = g * 16;
    u64 x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t sl = (uint32_t)(((k < 8 ? c0 : c1) >> (8 * (k & 7))) & 0xFFull);
      x[k] = sl != BC_SLOT_NONE ? a.slot[sl][(v0 + k) * W + lane] : 0ull;
    }
    if (held + 16 > BC_MAXCNT) flush();
    add8(x);
    add8(x + 8);
    held += 16;
  }
  if (held > 0) flush();
  __syncthreads();
  uint32_t* out = a.part + (size_t)blockIdx.x * 2 * M;
  for (int t = threadIdx.x; t < M; t += BC_BLOCK) {
    out[t] = lc[t];
    out[M + t] = 0u;
  }
}

// cov / fwd += the per-block partials; blockIdx.y takes one slice of the blocks
__global__ void k_bitcount_reduce(const uint32_t* __restrict__ part, int32_t nblocks, int32_t M,
                                  u64* __restrict__ cov, u64* __restrict__ fwd) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M) return;
  const int per = (nblocks + (int)gridDim.y - 1) / (int)gridDim.y;
  const int b0 = (int)blockIdx.y * per, b1 = std::min(nblocks, b0 + per);
  u64 c = 0, f = 0;
  for (int b = b0; b < b1; ++b) {
    c += part[(size_t)b * 2 * M + t];
    if (fwd) f += part[(size_t)b * 2 * M + M + t];
  }
  const int m = (t % (M / 64)) * 64 + t / (M / 64);   // partials are [bit][word]
  if (c) atomicAdd(&cov[m], c);
  if (fwd && f) atomicAdd(&fwd[m], f);
}

// the high-degree tail of the (degree, vertex) order: degrees there are nearly
// all distinct, so the planes would flush after every row.  Each set bit goes
// straight into the block's LDS counters (4 rows per lane slot in flight), one
// global atomic per (message, block) at the end.
template <int W, bool WEIGHTED>
__global__ __launch_bounds__(BC_BLOCK) void k_bitcount_tail(BitcountArgs a, int64_t begin, u64* __restrict__ cov,
                                                            u64* __restrict__ fwd) {
  constexpr int RPI = 64 / W;
  constexpr int M = W * 64;
  __shared__ uint32_t lc[M];   // [bit][word]: lanes of one instruction hit distinct banks
  __shared__ uint32_t ls[M];   // sums < arcs < 2^32 (checked by the launcher)
  for (int t = threadIdx.x; t < M; t += BC_BLOCK) lc[t] = ls[t] = 0u;
  __syncthreads();
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int w = lane % W, q = lane / W;
  constexpr int U = 4;
  const int64_t count = a.dcount ? (int64_t)*a.dcount : a.count;
  const int64_t step = (int64_t)gridDim.x * BC_WAVES * RPI;
  for (int64_t p = begin + ((int64_t)blockIdx.x * BC_WAVES + wib) * RPI + q; p < count; p += U * step) {
    u64 key[U];
#pragma unroll
    for (int u = 0; u < U; ++u) key[u] = p + u * step < count ? a.keys[p + u * step] : ~0ull;
    uint32_t sl[U];
#pragma unroll
    for (int u = 0; u < U; ++u) sl[u] = key[u] != ~0ull ? (uint32_t)a.sp[(uint32_t)key[u]] : (uint32_t)BC_SLOT_NONE;
    u64 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      x[u] = sl[u] != BC_SLOT_NONE ? a.slot[sl[u]][(int64_t)(uint32_t)key[u] * W + w] : 0ull;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t d = (uint32_t)(key[u] >> 32);
      u64 xx = x[u];
      while (xx) {
        const int b = __ffsll((long long)xx) - 1;
        xx &= xx - 1;
        atomicAdd(&lc[b * W + w], 1u);
        if (WEIGHTED) atomicAdd(&ls[b * W + w], d);
      }
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < M; t += BC_BLOCK) {
    const int m = (t % W) * 64 + t / W;
    if (lc[t]) atomicAdd(&cov[m], (u64)lc[t]);
    if (WEIGHTED && ls[t]) atomicAdd(&fwd[m], (u64)ls[t]);
  }
}

__global__ void k_bc_keys(const int32_t* __restrict__ deg, int64_t n, u64* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) keys[i] = ((u64)(uint32_t)std::max(deg[i], 0) << 32) | (u64)(uint32_t)i;
}

// rows of degree above this go to k_bitcount_tail
constexpr int32_t BC_TAIL_DEG = 256;

void bitcount_free(Ctx* c) {
  c->bc_split = 0;
  dfree(&c->d_fin_comp);
  dfree(&c->d_fin_list);
  c->fin_comp_rows = 0;
  dfree(&c->d_bc_keys);
  dfree(&c->d_bc_part);
  c->bc_part_words = 0;
}

// (degree, vertex) keys of the owned vertices, once per overlay / partition
static int bc_keys(Ctx* c) {
  if (c->d_bc_keys) return 0;
  const int64_t n = c->nloc();
  // owned vertices of degree <= BC_TAIL_DEG come first in the sorted order
  int64_t split = 0;
  for (int64_t i = 0; i < n; ++i) split += c->h_deg_out[(size_t)(c->vbegin + i)] <= BC_TAIL_DEG;
  c->bc_split = split;
  u64* tmp_keys = nullptr;
  void* tmp = nullptr;
  GP_TRY(dalloc(&c->d_bc_keys, (size_t)std::max<int64_t>(n, 1)));
  if (n == 0) return 0;
  GP_TRY(dalloc(&tmp_keys, (size_t)n));
  hipLaunchKernelGGL(k_bc_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, c->d_deg_out, n,
                     tmp_keys);
  size_t tb = 0;
  hipError_t e = rocprim::radix_sort_keys(nullptr, tb, tmp_keys, c->d_bc_keys, (size_t)n, 0, 64, c->stream);
  if (e == hipSuccess) e = hipMalloc(&tmp, std::max<size_t>(tb, 16));
  if (e == hipSuccess) e = rocprim::radix_sort_keys(tmp, tb, tmp_keys, c->d_bc_keys, (size_t)n, 0, 64, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (tmp) (void)hipFree(tmp);
  dfree(&tmp_keys);
  if (e != hipSuccess) {
    dfree(&c->d_bc_keys);
    return set_error(GP_EHIP, std::string("bitcount keys: ") + hipGetErrorString(e));
  }
  return 0;
}

template <int W>
static void launch_bitcount_w(Ctx* c, BitcountArgs a, bool weighted, int nblocks) {
  if (W == 64 && !weighted)   // (grid: nblocks, sized by the caller to the resident blocks)
    hipLaunchKernelGGL(k_bitcount_lin, dim3(nblocks), dim3(BC_BLOCK), 0, c->stream, a);
  else if (weighted)
    hipLaunchKernelGGL((k_bitcount<W, true>), dim3(nblocks), dim3(BC_BLOCK), 0, c->stream, a);
  else
    hipLaunchKernelGGL((k_bitcount<W, false>), dim3(nblocks), dim3(BC_BLOCK), 0, c->stream, a);
}

// coverage (and, weighted, degree-weighted forwards) of the owned vertices'
// Message-Lists into cov / fwd [W * 64] (overwritten)
int bitcount_messages(Ctx* c, bool weighted, u64* cov, u64* fwd) {
  const int W = c->words, M = W * 64;
  int64_t n = c->nloc();
  if (weighted && (u64)c->nnz_l >= (1ull << 32))
    return set_error(GP_EINVAL, "bitcount: per-block weighted sums are 32-bit (arcs < 2^32)");
  GP_TRY(unalias(c, false));   // (this pass reads every row, complete ones too)
  if (weighted) GP_TRY(bc_keys(c));
  const int64_t n_all = n;
  if (weighted) n = c->bc_split;   // the tail is counted by k_bitcount_tail
  const int64_t rows_per_block = (int64_t)BC_WAVES * 512;
  int64_t cap = (int64_t)c->cu_count * 8;
  if (W == 64 && !weighted) {   // one wave of resident blocks: equal chunks leave no tail
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_bitcount_lin, BC_BLOCK, 0) == hipSuccess &&
        per_cu > 0)
      cap = (int64_t)c->cu_count * per_cu;
  }
  const int nblocks = (int)std::max<int64_t>(1, std::min<int64_t>((n + rows_per_block - 1) / rows_per_block, cap));
  const size_t need = (size_t)nblocks * 2 * (size_t)M;
  if (need > c->bc_part_words) {
    GP_TRY(dalloc(&c->d_bc_part, need));
    c->bc_part_words = need;
  }
  BitcountArgs a{};
  a.slot[0] = c->d_slot[0];
  a.slot[1] = c->d_slot[1];
  a.slot[2] = c->d_slot[2];
  a.sp = c->d_sp;
  a.keys = weighted ? c->d_bc_keys : nullptr;
  a.count = n;
  a.part = c->d_bc_part;
  switch (W) {
    case 1: launch_bitcount_w<1>(c, a, weighted, nblocks); break;
    case 2: launch_bitcount_w<2>(c, a, weighted, nblocks); break;
    case 4: launch_bitcount_w<4>(c, a, weighted, nblocks); break;
    case 8: launch_bitcount_w<8>(c, a, weighted, nblocks); break;
    case 16: launch_bitcount_w<16>(c, a, weighted, nblocks); break;
    case 32: launch_bitcount_w<32>(c, a, weighted, nblocks); break;
    case 64: launch_bitcount_w<64>(c, a, weighted, nblocks); break;
    default: return set_error(GP_EINVAL, "unsupported word count");
  }
  GP_HIP(hipMemsetAsync(cov, 0, (size_t)M * 8, c->stream));
  if (weighted) GP_HIP(hipMemsetAsync(fwd, 0, (size_t)M * 8, c->stream));
  const int slices = std::max(1, std::min(nblocks / 16, 64));
  hipLaunchKernelGGL(k_bitcount_reduce, dim3((unsigned)((M + 255) / 256), (unsigned)slices), dim3(256), 0, c->stream,
                     c->d_bc_part, nblocks, M, cov, weighted ? fwd : nullptr);
  if (weighted && n_all > n) {
    a.count = n_all;
    const int tb = (int)std::max<int64_t>(1, std::min<int64_t>((n_all - n + 255) / 256, (int64_t)c->cu_count * 2));
    switch (W) {
      case 1: hipLaunchKernelGGL((k_bitcount_tail<1, true>), dim3(tb), dim3(BC_BLOCK), 0, c->stream, a, n, cov, fwd); break;
      case 2: hipLaunchKernelGGL((k_bitcount_tail<2, true>), dim3(tb), dim3(BC_BLOCK), 0, c->stream, a, n, cov, fwd); break;
      case 4: hipLaunchKernelGGL((k_bitcount_tail<4, true>), dim3(tb), dim3(BC_BLOCK), 0, c->stream, a, n, cov, fwd); break;
      case 8: hipLaunchKernelGGL((k_bitcount_tail<8, true>), dim3(tb), dim3(BC_BLOCK), 0, c->stream, a, n, cov, fwd); break;
      case 16: hipLaunchKernelGGL((k_bitcount_tail<16, true>), dim3(tb), dim3(BC_BLOCK), 0, c->stream, a, n, cov, fwd); break;
      case 32: hipLaunchKernelGGL((k_bitcount_tail<32, true>), dim3(tb), dim3(BC_BLOCK), 0, c->stream, a, n, cov, fwd); break;
      default: hipLaunchKernelGGL((k_bitcount_tail<64, true>), dim3(tb), dim3(BC_BLOCK), 0, c->stream, a, n, cov, fwd); break;
    }
  }
  GP_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// Finalize through the component targets.  A vertex whose Message-List holds
// as many messages as its component has this run (seenpop == done_at, lost
// messages already dropped from both) holds exactly the
// component's mask row cmask[midx[v]]: every message it can hold originated in
// its weakly connected component.  So
//   coverage[m] = sum_K full_K * bit(cmask[K], m) + (the other rows)
//   forwards[m] = sum_K degsum_K * bit(cmask[K], m) + (the other rows, weighted)
// with full_K / degsum_K the number / degree sum of the complete vertices of
// component K.  One pass over 4-B per-vertex words replaces the pass over the
// rows; only incomplete, non-empty rows are still counted bit by bit (a C4 run
// ends with none, a churn run with the vertices crashes cut off).
// grid-stride over 64-vertex chunks per wave; a wave keeps the running count
// and degree sum of one component (the giant one, in practice) in registers
// and adds them once at the end -- per-chunk atomics on that one address were
// 0.5 M same-address adds at C4 (3.2 ms); other components add per chunk.
// First pass (list null): component sums + the number of incomplete rows;
// second pass (only when few): list them.
__global__ __launch_bounds__(BC_BLOCK) void k_fin_scan(const uint32_t* __restrict__ seenpop,
                                                       const uint32_t* __restrict__ done_at,
                                                       const int32_t* __restrict__ midx,
                                                       const int32_t* __restrict__ deg, int64_t n,
                                                       u64* __restrict__ comp_cnt, u64* __restrict__ comp_deg,
                                                       u64* __restrict__ list, u64* __restrict__ list_n) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * BC_WAVES;
  int32_t kr = -1;       // the wave's running component
  u64 rc = 0, rd = 0;    // its count and degree sum (wave-uniform)
  u64 npart = 0;         // incomplete rows seen by the wave
  for (int64_t base = ((int64_t)blockIdx.x * BC_WAVES + (threadIdx.x >> 6)) * 64; base < n; base += nwaves * 64) {
    const int64_t v = base + lane;
    bool full = false, part = false;
    int32_t k = -1;
    u64 d = 0;
    if (v < n) {
      const uint32_t pop = seenpop[v];
      if (pop) {
        k = midx[v];
        d = (u64)(uint32_t)max(deg[v], 0);
        full = k >= 0 && pop == done_at[v];
        part = !full;
      }
    }
    u64 fm = __ballot(full);
    if (kr < 0 && fm) kr = __shfl(k, __ffsll((long long)fm) - 1);
    while (fm) {
      const int leader = __ffsll((long long)fm) - 1;
      const int32_t kl = __shfl(k, leader);
      const bool mine = full && k == kl;
      const u64 mm = __ballot(mine);
      u64 ds = mine ? d : 0ull;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) ds += __shfl_xor(ds, o);
      if (list) {   // second pass: the component sums are in already
      } else if (kl == kr) {
        rc += (u64)__popcll(mm);
        rd += ds;
      } else if (lane == leader) {
        atomicAdd(&comp_cnt[kl], (u64)__popcll(mm));
        atomicAdd(&comp_deg[kl], ds);
      }
      fm &= ~mm;
    }
    const u64 pm = __ballot(part);
    if (list && pm) {   // second pass: few incomplete rows, list them
      const int first = __ffsll((long long)pm) - 1;
      u64 at = 0;
      if (lane == first) at = atomicAdd(list_n, (u64)__popcll(pm));
      at = __shfl(at, first);
      if (part) list[at + (u64)__popcll(pm & ((1ull << lane) - 1ull))] = (d << 32) | (u64)(uint32_t)v;
    }
    npart += (u64)__popcll(pm);
  }
  if (!list) {   // first pass: count the incomplete rows, one atomic per block
    __shared__ u64 bsum[BC_WAVES];
    if (lane == 0) bsum[threadIdx.x >> 6] = npart;
    __syncthreads();
    if (threadIdx.x == 0) {
      u64 t = 0;
      for (int k = 0; k < BC_WAVES; ++k) t += bsum[k];
      if (t) atomicAdd(list_n, t);
    }
    if (kr >= 0 && lane == 0) {
      atomicAdd(&comp_cnt[kr], rc);
      atomicAdd(&comp_deg[kr], rd);
    }
  }
}

// coverage / forwards of the complete vertices: message m = 64 w + b over the
// component rows (overwrites cov, and fwd when given)
__global__ void k_fin_comp(const u64* __restrict__ cmask, int32_t K, int32_t W, const u64* __restrict__ comp_cnt,
                           const u64* __restrict__ comp_deg, u64* __restrict__ cov, u64* __restrict__ fwd) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= W * 64) return;
  const int w = t / 64, b = t % 64;
  u64 c = 0, f = 0;
  for (int32_t r = 0; r < K; ++r) {
    if ((cmask[(size_t)r * W + w] >> b) & 1ull) {
      c += comp_cnt[r];
      f += comp_deg[r];
    }
  }
  cov[t] = c;
  if (fwd) fwd[t] = f;
}

int finalize_by_components(Ctx* c, bool weighted, u64* cov, u64* fwd) {
  const int W = c->words, M = W * 64;
  const int64_t n = c->nloc();
  const int32_t K = std::max(c->cmask_rows, 1);
  hipStream_t s = c->stream;
  if (weighted && (u64)c->nnz_l >= (1ull << 32))
    return set_error(GP_EINVAL, "finalize: per-block weighted sums are 32-bit (arcs < 2^32)");
  if (!c->d_fin_comp || c->fin_comp_rows < K) {
    GP_TRY(dalloc(&c->d_fin_comp, 2 * (size_t)K + 1));
    c->fin_comp_rows = K;
  }
  u64* comp_cnt = c->d_fin_comp;
  u64* comp_deg = c->d_fin_comp + K;
  u64* list_n = c->d_fin_comp + 2 * (size_t)K;
  GP_HIP(hipMemsetAsync(c->d_fin_comp, 0, (2 * (size_t)K + 1) * 8, s));
  const dim3 sg((unsigned)std::max<int64_t>(1, std::min<int64_t>((n + BC_BLOCK - 1) / BC_BLOCK,
                                                                   (int64_t)c->cu_count * 8)));
  if (n > 0)
    hipLaunchKernelGGL(k_fin_scan, sg, dim3(BC_BLOCK), 0, s, c->d_seenpop, c->d_done_at, c->d_midx, c->d_deg_out, n,
                       comp_cnt, comp_deg, (u64*)nullptr, list_n);
  u64 incomplete = 0;
  GP_TRY(copy_sync(c, &incomplete, list_n, 8, hipMemcpyDeviceToHost));
  // many incomplete rows (churn: crashes cut messages off, so nobody completes
  // its component): the bit-sliced pass over every row is the cheaper way
  if ((int64_t)incomplete * 32 > n) return bitcount_messages(c, weighted, cov, fwd);
  hipLaunchKernelGGL(k_fin_comp, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, c->d_cmask, c->cmask_rows, W,
                     comp_cnt, comp_deg, cov, weighted ? fwd : nullptr);
  GP_HIP(hipGetLastError());
  if (incomplete == 0) return 0;
  if (!c->d_fin_list) GP_TRY(dalloc(&c->d_fin_list, (size_t)std::max<int64_t>(n, 1)));
  GP_HIP(hipMemsetAsync(list_n, 0, 8, s));
  hipLaunchKernelGGL(k_fin_scan, sg, dim3(BC_BLOCK), 0, s, c->d_seenpop, c->d_done_at, c->d_midx, c->d_deg_out, n,
                     comp_cnt, comp_deg, c->d_fin_list, list_n);
  BitcountArgs a{};
  a.slot[0] = c->d_slot[0];
  a.slot[1] = c->d_slot[1];
  a.slot[2] = c->d_slot[2];
  a.sp = c->d_sp;
  a.keys = c->d_fin_list;
  a.count = n;
  a.dcount = list_n;
  const dim3 g((unsigned)std::max(1, c->cu_count * 2));
#define GP_FIN_TAIL(WW)                                                                                 \
  if (weighted) hipLaunchKernelGGL((k_bitcount_tail<WW, true>), g, dim3(BC_BLOCK), 0, s, a, 0, cov, fwd); \
  else hipLaunchKernelGGL((k_bitcount_tail<WW, false>), g, dim3(BC_BLOCK), 0, s, a, 0, cov, fwd);
  switch (W) {
    case 1: GP_FIN_TAIL(1) break;
    case 2: GP_FIN_TAIL(2) break;
    case 4: GP_FIN_TAIL(4) break;
    case 8: GP_FIN_TAIL(8) break;
    case 16: GP_FIN_TAIL(16) break;
    case 32: GP_FIN_TAIL(32) break;
    case 64: GP_FIN_TAIL(64) break;
    default: return set_error(GP_EINVAL, "unsupported word count");
  }
#undef GP_FIN_TAIL
  GP_HIP(hipGetLastError());
  return 0;
}

}  // namespace gp
