// graph_build.hip -- device-side Chung-Lu power-law overlay builder.
//
// The reference's intent is a degree-weighted ("power-law") neighbour choice
// (demonstrate_powerlaw.py:19-35 weights peers by their current degree;
// Seed.py:151-185 is a broken rank-weighted attempt).  For the throughput
// configs (BASELINE.json C3-C5) the overlay is a Chung-Lu graph whose expected
// degrees follow w_i ∝ (i+1)^(-1/(gamma-1)), built here in O(n + nnz):
//   1. host: integer Vose alias table over q_i = max(1, floor(2^32 (i+1)^-alpha))
//   2. device: E = floor(dbar*n/2) candidate edges, endpoints by alias sampling
//      from counter-based splitmix draws; ids relabelled by a random permutation
//   3. device: both arc directions as u64 keys (dst<<32 | src), radix sort,
//      unique (drops multi-edges), self-loops dropped -> in-CSR.
// Everything is integer arithmetic, so the CPU oracle reproduces the CSR bit for
// bit (oracle/gossip_oracle.c: or_chung_lu).
#include <hip/hip_runtime.h>

#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "gp_internal.h"

namespace gp {

typedef unsigned long long u64;
constexpr u64 SENTINEL = ~0ull;

struct AliasTable {
  std::vector<uint64_t> prob;    // accept threshold in [0, T]
  std::vector<int32_t> alias;
  uint64_t total = 0;            // T
};

// integer Vose alias table (deterministic: stacks filled in index order)
static void build_alias(int64_t n, double gamma, AliasTable& t) {
  const double alpha = 1.0 / (gamma - 1.0);
  std::vector<uint64_t> q((size_t)n);
  // the weights in parallel (one pow per vertex: most of a 2^24 build's host
  // time); integer sums, so the total is the same in any order
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(16, n >> 16));
  std::vector<uint64_t> part((size_t)nt, 0);
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t) {
    pool.emplace_back([&, t]() {
      const int64_t i0 = n * t / nt, i1 = n * (t + 1) / nt;
      uint64_t sum = 0;
      for (int64_t i = i0; i < i1; ++i) {
        const double w = std::ldexp(std::pow((double)(i + 1), -alpha), 32);
        uint64_t qi = (uint64_t)std::floor(w);
        if (qi < 1) qi = 1;
        q[(size_t)i] = qi;
        sum += qi;
      }
      part[(size_t)t] = sum;
    });
  }
  for (auto& th : pool) th.join();
  uint64_t T = 0;
  for (uint64_t x : part) T += x;
  t.total = T;
  t.prob.assign((size_t)n, T);
  t.alias.resize((size_t)n);
  std::vector<uint64_t> p((size_t)n);
  std::vector<int32_t> small, large;
  small.reserve((size_t)n);
  large.reserve((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    p[(size_t)i] = q[(size_t)i] * (uint64_t)n;
    t.alias[(size_t)i] = (int32_t)i;
    if (p[(size_t)i] < T) small.push_back((int32_t)i);
    else large.push_back((int32_t)i);
  }
  while (!small.empty() && !large.empty()) {
    const int32_t s = small.back();
    small.pop_back();
    const int32_t l = large.back();
    large.pop_back();
    t.prob[(size_t)s] = p[(size_t)s];
    t.alias[(size_t)s] = l;
    p[(size_t)l] -= T - p[(size_t)s];
    if (p[(size_t)l] < T) small.push_back(l);
    else large.push_back(l);
  }
  // leftovers keep prob = T (always accept); with exact integers they hold T
}

__device__ __forceinline__ int32_t alias_pick(const uint64_t* __restrict__ prob,
                                              const int32_t* __restrict__ alias, uint64_t n,
                                              uint64_t T, u64 r_slot, u64 r_coin) {
  const uint64_t i = below(r_slot, n);
  const uint64_t x = below(r_coin, T);
  return x < prob[i] ? (int32_t)i : alias[i];
}

__global__ void k_relabel_keys(u64* __restrict__ keys, int64_t n, u64 key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) keys[i] = ((draw(key, (u64)i) >> 32) << 32) | (u64)i;
}
__global__ void k_relabel_scatter(const u64* __restrict__ sorted, int32_t* __restrict__ new_id, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) new_id[(uint32_t)sorted[k]] = (int32_t)k;
}

__global__ void k_gen_edges(u64* __restrict__ keys, int64_t E, const uint64_t* __restrict__ prob,
                            const int32_t* __restrict__ alias, const int32_t* __restrict__ new_id,
                            uint64_t n, uint64_t T, u64 key) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const u64 b = 4ull * (u64)e;
  const int32_t u = alias_pick(prob, alias, n, T, draw(key, b + 0), draw(key, b + 1));
  const int32_t v = alias_pick(prob, alias, n, T, draw(key, b + 2), draw(key, b + 3));
  if (u == v) {
    keys[2 * e] = SENTINEL;
    keys[2 * e + 1] = SENTINEL;
    return;
  }
  const u64 a = (u64)(uint32_t)new_id[u], c = (u64)(uint32_t)new_id[v];
  keys[2 * e] = (a << 32) | c;
  keys[2 * e + 1] = (c << 32) | a;
}

// row_ptr from sorted unique keys (row = high 32 bits) and col = low 32 bits
__global__ void k_csr_from_keys(const u64* __restrict__ keys, int64_t A, int64_t n,
                                int64_t* __restrict__ row_ptr, int32_t* __restrict__ col) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > A) return;
  const int64_t prev = i > 0 ? (int64_t)(keys[i - 1] >> 32) : -1;
  const int64_t cur = i < A ? (int64_t)(keys[i] >> 32) : n;
  for (int64_t x = prev + 1; x <= cur && x <= n; ++x) row_ptr[x] = i;
  if (i < A) col[i] = (int32_t)(uint32_t)keys[i];
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

int build_chung_lu(Ctx* c, int64_t n, double dbar, double gamma, uint64_t seed) {
  hipStream_t s = c->stream;
  AliasTable at;
  build_alias(n, gamma, at);
  const int64_t E = (int64_t)std::floor(dbar * (double)n / 2.0);
  const int64_t K = 2 * E;

  DevBuf d_prob, d_alias, d_newid, d_ka, d_kb, d_tmp, d_cnt;
  GP_HIP(hipMalloc(&d_prob.p, (size_t)n * 8));
  GP_HIP(hipMalloc(&d_alias.p, (size_t)n * 4));
  GP_HIP(hipMalloc(&d_newid.p, (size_t)n * 4));
  const size_t kbytes = (size_t)std::max<int64_t>(std::max<int64_t>(K, n), 1) * 8;
  GP_HIP(hipMalloc(&d_ka.p, kbytes));
  GP_HIP(hipMalloc(&d_kb.p, kbytes));
  GP_HIP(hipMalloc(&d_cnt.p, 16));
  GP_HIP(hipMemcpyAsync(d_prob.p, at.prob.data(), (size_t)n * 8, hipMemcpyHostToDevice, s));
  GP_HIP(hipMemcpyAsync(d_alias.p, at.alias.data(), (size_t)n * 4, hipMemcpyHostToDevice, s));
  u64* ka = (u64*)d_ka.p;
  u64* kb = (u64*)d_kb.p;

  // temp storage sized for the largest sort / select
  size_t tmp_sort = 0, tmp_uniq = 0;
  GP_HIP(rocprim::radix_sort_keys(nullptr, tmp_sort, ka, kb, (size_t)std::max<int64_t>(K, n), 0, 64, s));
  GP_HIP(rocprim::unique(nullptr, tmp_uniq, kb, ka, (size_t*)d_cnt.p, (size_t)std::max<int64_t>(K, 1),
                         rocprim::equal_to<u64>(), s));
  const size_t tmp_bytes = std::max<size_t>(std::max(tmp_sort, tmp_uniq), 16);
  GP_HIP(hipMalloc(&d_tmp.p, tmp_bytes));

  // 1. random relabel: sort (hash32(i) << 32 | i)
  const u64 krel = stream_key(seed, STREAM_RELABEL);
  hipLaunchKernelGGL(k_relabel_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ka, n, krel);
  size_t tb = tmp_bytes;
  GP_HIP(rocprim::radix_sort_keys(d_tmp.p, tb, ka, kb, (size_t)n, 0, 64, s));
  hipLaunchKernelGGL(k_relabel_scatter, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, kb,
                     (int32_t*)d_newid.p, n);
  GP_HIP(hipGetLastError());

  // 2. candidate edges -> arc keys
  const u64 kedge = stream_key(seed, STREAM_EDGE);
  int64_t A = 0;
  if (E > 0) {
    hipLaunchKernelGGL(k_gen_edges, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, ka, E,
                       (const uint64_t*)d_prob.p, (const int32_t*)d_alias.p, (const int32_t*)d_newid.p,
                       (uint64_t)n, at.total, kedge);
    GP_HIP(hipGetLastError());
    tb = tmp_bytes;
    GP_HIP(rocprim::radix_sort_keys(d_tmp.p, tb, ka, kb, (size_t)K, 0, 64, s));
    tb = tmp_bytes;
    GP_HIP(rocprim::unique(d_tmp.p, tb, kb, ka, (size_t*)d_cnt.p, (size_t)K, rocprim::equal_to<u64>(), s));
    size_t nuniq = 0;
    GP_HIP(hipMemcpyAsync(&nuniq, d_cnt.p, sizeof(size_t), hipMemcpyDeviceToHost, s));
    GP_HIP(hipStreamSynchronize(s));
    A = (int64_t)nuniq;
    if (A > 0) {
      u64 last = 0;
      GP_TRY(copy_sync(c, &last, ka + (A - 1), 8, hipMemcpyDeviceToHost));
      if (last == SENTINEL) --A;
    }
  }
  c->n = n;
  c->nnz = A;
  c->directed = 0;
  GP_TRY(dalloc(&c->d_row_ptr, (size_t)n + 1));
  GP_TRY(dalloc(&c->d_col, (size_t)A));
  hipLaunchKernelGGL(k_csr_from_keys, dim3((unsigned)((A + 1 + 255) / 256)), dim3(256), 0, s, ka, A, n,
                     c->d_row_ptr, c->d_col);
  GP_HIP(hipGetLastError());
  GP_HIP(hipStreamSynchronize(s));
  dfree(&c->d_out_row_ptr);
  dfree(&c->d_out_col);
  return 0;
}

// gather order: each in-list re-sorted by the neighbour's in-degree, largest
// first (stable: ties keep ascending ids).  Hubs hold most messages earliest,
// so the early-exit pull covers a vertex's missing set after fewer rows.
// gather order: every in-list sorted by neighbour in-degree, descending (ties
// keep the id order: the radix sort is stable).  Arc-parallel: the owner of
// arc j comes from a max-scan of the segment heads (a thread per vertex walked
// a hub's 318 K arcs alone: 113 ms at C4, 383 ms at C5).
__global__ void k_seg_heads(const int64_t* __restrict__ rp, int32_t* __restrict__ seg, int64_t n) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n && rp[v] < rp[v + 1]) seg[rp[v]] = (int32_t)v;
}
__global__ void k_gorder_keys(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                              const int32_t* __restrict__ seg, u64* __restrict__ keys, int32_t* __restrict__ vals,
                              int64_t A) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= A) return;
  const int32_t u = col[j];
  const uint32_t d = (uint32_t)(rp[u + 1] - rp[u]);
  keys[j] = ((u64)(uint32_t)seg[j] << 32) | (u64)(0xFFFFFFFFu - d);
  vals[j] = u;
}

int build_gather_order(Ctx* c) {
  hipStream_t s = c->stream;
  const int64_t A = c->nnz;
  GP_TRY(dalloc(&c->d_gcol, (size_t)std::max<int64_t>(A, 1)));
  if (A == 0) return 0;
  DevBuf ka, kb, va, seg, tmp;
  GP_HIP(hipMalloc(&ka.p, (size_t)A * 8));
  GP_HIP(hipMalloc(&kb.p, (size_t)A * 8));
  GP_HIP(hipMalloc(&va.p, (size_t)A * 4));
  GP_HIP(hipMalloc(&seg.p, (size_t)A * 4));
  GP_HIP(hipMemsetAsync(seg.p, 0, (size_t)A * 4, s));
  hipLaunchKernelGGL(k_seg_heads, dim3((unsigned)((c->n + 255) / 256)), dim3(256), 0, s, c->d_row_ptr,
                     (int32_t*)seg.p, c->n);
  size_t tb = 0, ts = 0;
  int32_t* owner = (int32_t*)kb.p;   // the scan's output; kb is free until the sort
  GP_HIP(rocprim::inclusive_scan(nullptr, ts, (int32_t*)seg.p, owner, (size_t)A,
                                 rocprim::maximum<int32_t>(), s));
  GP_HIP(rocprim::radix_sort_pairs(nullptr, tb, (u64*)ka.p, (u64*)kb.p, (int32_t*)va.p, c->d_gcol, (size_t)A,
                                   0, 64, s));
  GP_HIP(hipMalloc(&tmp.p, std::max<size_t>(std::max(tb, ts), 16)));
  GP_HIP(rocprim::inclusive_scan(tmp.p, ts, (int32_t*)seg.p, owner, (size_t)A,
                                 rocprim::maximum<int32_t>(), s));
  hipLaunchKernelGGL(k_gorder_keys, dim3((unsigned)((A + 255) / 256)), dim3(256), 0, s, c->d_row_ptr, c->d_col,
                     (const int32_t*)owner, (u64*)ka.p, (int32_t*)va.p, A);
  GP_HIP(hipGetLastError());
  GP_HIP(rocprim::radix_sort_pairs(tmp.p, tb, (u64*)ka.p, (u64*)kb.p, (int32_t*)va.p, c->d_gcol, (size_t)A,
                                   0, 64, s));
  GP_HIP(hipStreamSynchronize(s));
  return 0;
}

// degree-split rounds: per vertex, the length of the prefix
// of its gather-ordered in-list whose senders have in-degree >= T (the order is
// by that in-degree, descending, so the prefix is exactly those arcs).  One
// thread per vertex, binary search over its segment.
__global__ void k_prehi(const int64_t* __restrict__ rp, const int32_t* __restrict__ gcol, int64_t n, int32_t T,
                        int32_t* __restrict__ prehi) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  int64_t lo = rp[v], hi = rp[v + 1];   // first j in [lo, hi) with deg(gcol[j]) < T
  const int64_t b = lo;
  while (lo < hi) {
    const int64_t mid = lo + (hi - lo) / 2;
    const int32_t u = gcol[mid];
    if (rp[u + 1] - rp[u] >= (int64_t)T) lo = mid + 1;
    else hi = mid;
  }
  prehi[v] = (int32_t)(lo - b);
}

int build_prehi(Ctx* c, int32_t T) {
  if (c->d_prehi && c->prehi_deg == T) return 0;
  GP_TRY(dalloc(&c->d_prehi, (size_t)std::max<int64_t>(c->n, 1)));
  if (c->n > 0)
    hipLaunchKernelGGL(k_prehi, dim3((unsigned)((c->n + 255) / 256)), dim3(256), 0, c->stream, c->d_row_ptr,
                       c->d_gcol, c->n, T, c->d_prehi);
  GP_HIP(hipGetLastError());
  c->prehi_deg = T;
  return 0;
}

}  // namespace gp
