// setup.hip -- once per overlay and per message table, outside the timed
// step: weakly connected components and per-vertex targets (done_at, the
// component message masks), the hub table, spread keys for the message order
// (DESIGN.md §3.4, §3.8), run-state allocation, and the C-ABI entry points
// that configure a context (include/gossip_capi.h).
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gp_device.h"
#include "xplan.h"

namespace gp {

// ---------------------------------------------------------------------------
// weakly connected components (union-find, hook larger root under smaller,
// so the label of a component is its smallest vertex id).  A vertex holding
// every message injected in its component can never receive anything new:
// done_at[v] = #messages originating in comp(v) lets E_r skip it entirely.
__device__ __forceinline__ int32_t cc_parent(const int32_t* p, int32_t x) {
  return __hip_atomic_load(p + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ int32_t cc_find(int32_t* __restrict__ parent, int32_t x) {
  int32_t p = cc_parent(parent, x);
  while (p != x) {
    const int32_t g = cc_parent(parent, p);
    if (g != p) __hip_atomic_store(parent + x, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x = p;
    p = g;
  }
  return x;
}
__global__ void k_cc_init(int32_t* __restrict__ parent, int64_t n) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) parent[v] = (int32_t)v;
}
// Weakly connected components, Afforest-style (Sutton, Ben-Nun, Barak, IPDPS'18):
// link every vertex to its first CC_SAMPLE in-neighbours, compress, find the
// component most vertices already sit in (the giant one of a power-law overlay)
// from a sample, and link the remaining arcs only of vertices outside it.  The
// old per-vertex union over whole in-lists left one thread walking a hub's
// 318 K arcs (217 ms at C4, 581 ms at C5).  Labels are the component's minimum
// vertex id either way (links always hook the larger root under the smaller).
constexpr int CC_SAMPLE = 2;
__device__ void cc_link(int32_t* __restrict__ parent, int32_t a, int32_t b) {
  while (true) {
    a = cc_find(parent, a);
    b = cc_find(parent, b);
    if (a == b) return;
    if (a < b) {
      const int32_t t = a;
      a = b;
      b = t;
    }
    if (atomicCAS(parent + a, a, b) == a) return;
  }
}
__global__ void k_cc_sample_link(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                 int32_t* __restrict__ parent, int64_t n, int32_t r) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  const int64_t j = rp[v] + r;
  if (j < rp[v + 1]) cc_link(parent, (int32_t)v, col[j]);
}
// the remaining arcs (from CC_SAMPLE on) of vertices outside component `skip`
// (-1: of every vertex -- directed overlays, whose in-lists alone do not carry
// a skipped vertex's out-arcs).  Hubs sit in the giant component and skip.
__global__ void k_cc_rest(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                          int32_t* __restrict__ parent, int64_t n, int32_t skip) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  const int64_t b = rp[v] + CC_SAMPLE, e = rp[v + 1];
  if (b >= e) return;
  if (skip >= 0 && cc_find(parent, (int32_t)v) == skip) return;
  for (int64_t j = b; j < e; ++j) cc_link(parent, (int32_t)v, col[j]);
}
__global__ void k_cc_compress(int32_t* __restrict__ parent, int64_t n) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) parent[v] = cc_find(parent, (int32_t)v);
}
__global__ void k_cc_gather(const int32_t* __restrict__ parent, int64_t n, int32_t k, uint64_t seed,
                            int32_t* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= k) return;
  u64 z = seed + (u64)(t + 1) * 0x9E3779B97F4A7C15ull;   // splitmix64 sample positions
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  out[t] = parent[(int64_t)(((unsigned __int128)z * (unsigned __int128)(u64)n) >> 64)];
}
__global__ void k_cc_final(int32_t* __restrict__ parent, int64_t n) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) parent[v] = cc_find(parent, (int32_t)v);
}
__global__ void k_count_origins(const int32_t* __restrict__ origin, const uint32_t* __restrict__ gcnt,
                                int64_t groups, const int32_t* __restrict__ comp, uint32_t* __restrict__ cnt) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < groups) atomicAdd(cnt + comp[origin[k]], gcnt[k]);
}
__global__ void k_done_at(const int32_t* __restrict__ comp, const uint32_t* __restrict__ cnt,
                          uint32_t* __restrict__ done_at, int64_t n) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) done_at[v] = cnt[comp[v]];
}
__global__ void k_degree(const int64_t* __restrict__ rp, int32_t* __restrict__ deg, int64_t n) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) deg[v] = (int32_t)(rp[v + 1] - rp[v]);
}

// spread keys (gp_spread_keys): out[k] = sum over the in-list of vtx[k] of
// val[u] (val null: the degree of u).  One wave per listed vertex, grid-stride
// over the list; hubs' lists are long, so lanes stride their arcs.
__global__ __launch_bounds__(BLOCK) void k_nbsum(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                 const u64* __restrict__ val, const int32_t* __restrict__ vtx,
                                                 int64_t cnt, u64* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (BLOCK / 64);
  for (int64_t k = (int64_t)blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6); k < cnt; k += nw) {
    const int64_t v = vtx ? vtx[k] : k;
    const int64_t b = rp[v], e = rp[v + 1];
    u64 s = 0;
    for (int64_t j = b + lane; j < e; j += 64) {
      const int32_t u = col[j];
      s += val ? val[u] : (u64)(rp[u + 1] - rp[u]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0) out[k] = s;
  }
}


int build_hubs(Ctx* c) {
  c->h_hub_items.clear();
  std::vector<int32_t> hubs, ptr;
  const int64_t thr = c->cfg.hub_threshold;
  if (!c->h_row_ptr.empty()) {
    for (int64_t v = 0; v < c->nloc(); ++v) {   // owned local ids
      const int64_t b = c->h_row_ptr[v], e = c->h_row_ptr[v + 1];
      if (e - b <= thr) continue;
      ptr.push_back((int32_t)c->h_hub_items.size());
      for (int64_t j = b; j < e; j += thr)
        c->h_hub_items.push_back(HubItem{(int32_t)v, (int32_t)hubs.size(), j, std::min(e, j + thr)});
      hubs.push_back((int32_t)v);
    }
  }
  ptr.push_back((int32_t)c->h_hub_items.size());
  c->n_hubs = (int64_t)hubs.size();
  c->n_hub_items = (int64_t)c->h_hub_items.size();
  GP_TRY(dalloc(&c->d_hub_items, c->h_hub_items.size()));
  GP_TRY(dalloc(&c->d_hubs, hubs.size()));
  GP_TRY(dalloc(&c->d_hub_item_ptr, ptr.size()));
  GP_TRY(dalloc(&c->d_hub_pnz, c->h_hub_items.size()));
  GP_TRY(dalloc(&c->d_hub_done, std::max<size_t>(hubs.size(), 1)));
  GP_HIP(hipMemsetAsync(c->d_hub_done, 0, std::max<size_t>(hubs.size(), 1) * 4, c->stream));
  c->hub_epoch = 0;
  if (!c->h_hub_items.empty())
    GP_TRY(copy_sync(c, c->d_hub_items, c->h_hub_items.data(), c->h_hub_items.size() * sizeof(HubItem),
                     hipMemcpyHostToDevice));
  if (!hubs.empty())
    GP_TRY(copy_sync(c, c->d_hubs, hubs.data(), hubs.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  GP_TRY(copy_sync(c, c->d_hub_item_ptr, ptr.data(), ptr.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  if (c->words > 0) GP_TRY(dalloc(&c->d_hub_partial, c->h_hub_items.size() * (size_t)c->words));
  return 0;
}

static void free_state(Ctx* c);

// nranks == 1: the whole overlay, local ids = global ids.  nranks > 1: the
// context keeps its owned slice plus ghosts (partition.hip: localize), once
// per overlay -- the global CSR is dropped afterwards.
static int set_partition(Ctx* c, int32_t rank, int32_t nranks) {
  if (nranks < 1 || rank < 0 || rank >= nranks) return set_error(GP_EINVAL, "bad rank/nranks");
  if (c->local && (rank != c->rank || nranks != c->nranks))
    return set_error(GP_ESTATE, "a partitioned context keeps its partition: reload the overlay to change it");
  if (c->local) return 0;
  if (nranks > 1 && c->directed)
    return set_error(GP_EINVAL, "vertex partitions need an undirected overlay (ghost rows are in-neighbours)");
  c->rank = rank;
  c->nranks = nranks;
  c->h_bounds = partition_bounds(c->n, nranks, c->cfg.partition_by_arcs,
                                 c->h_row_ptr.size() == (size_t)c->n + 1 ? c->h_row_ptr.data() : nullptr);
  c->vbegin = c->h_bounds[(size_t)rank];
  c->vend = c->h_bounds[(size_t)rank + 1];
  c->n_alloc = c->n;
  c->base_nv = c->n;
  if (nranks > 1) {   // local ids from here on: the message table must be set again
    free_state(c);
    GP_TRY(localize(c));
  }
  return build_hubs(c);
}

// the slot buffers S[0], S[1] and the push accumulator are one allocation
// (free_rows / alloc_state): a degree-split round addresses accumulator rows
// as rows of the round's slot buffer (driver.hip launch_expand, acc_row)
static void free_rows(Ctx* c) {
  dfree(&c->d_rows);
  c->d_slot[0] = c->d_slot[1] = c->d_acc = nullptr;
}

static void free_state(Ctx* c) {
  dfree(&c->d_slot[2]);
  c->park_failed = false;
  free_rows(c);
  for (int k = 0; k < 2; ++k) {
    dfree(&c->d_frx[k]);
    dfree(&c->d_fpop[k]);
  }
  dfree(&c->d_sp); dfree(&c->d_ws);
  dfree(&c->d_ulist[0]); dfree(&c->d_ulist[1]);
  c->ulist_valid = false;
  dfree(&c->d_seenpop); dfree(&c->d_first); dfree(&c->d_digest);
  dfree(&c->d_state); dfree(&c->d_miss); dfree(&c->d_deg_live); dfree(&c->d_cand);
  dfree(&c->d_det_big); dfree(&c->d_det_pre); dfree(&c->d_det_live); dfree(&c->d_det_cur); dfree(&c->d_det_base);
  dfree(&c->d_msg_cov); dfree(&c->d_reports); dfree(&c->d_abits); dfree(&c->d_dbits); dfree(&c->d_lm); dfree(&c->d_lmw[0]); dfree(&c->d_lmw[1]); dfree(&c->d_sbits); dfree(&c->d_amask); dfree(&c->d_cml[0]); dfree(&c->d_cml[1]); dfree(&c->d_cmk[0]); dfree(&c->d_cmk[1]); dfree(&c->d_done_at);
  dfree(&c->d_done_at0); dfree(&c->d_cmask0); dfree(&c->d_lostcnt); dfree(&c->d_alive);
  dfree(&c->d_tbits); dfree(&c->d_nbits); dfree(&c->d_touched); dfree(&c->d_active); dfree(&c->d_big);
  dfree(&c->d_midx); dfree(&c->d_cmask);
  bitcount_free(c);
  c->d_msg_fwd = nullptr;
  dfree(&c->d_inj_origin); dfree(&c->d_inj_bits); dfree(&c->d_inj_cnt);
  c->inject.clear();
  c->m = 0;
  c->words = 0;
}

// weakly connected components of the overlay into d_comp (Afforest, above)
static int components(Ctx* c) {
  hipStream_t s = c->stream;
  const int64_t n = c->n;
  const dim3 g(grid_for(n, 256));
  hipLaunchKernelGGL(k_cc_init, g, dim3(256), 0, s, c->d_comp, n);
  for (int32_t r = 0; r < CC_SAMPLE; ++r) {
    hipLaunchKernelGGL(k_cc_sample_link, g, dim3(256), 0, s, c->d_row_ptr, c->d_col, c->d_comp, n, r);
    hipLaunchKernelGGL(k_cc_compress, g, dim3(256), 0, s, c->d_comp, n);
  }
  int32_t skip = -1;
  if (!c->directed && n > 0) {   // the most frequent label among 1024 sampled vertices
    constexpr int K = 1024;
    int32_t* d_smp = nullptr;
    GP_TRY(dalloc(&d_smp, K));
    hipLaunchKernelGGL(k_cc_gather, dim3(K / 256), dim3(256), 0, s, c->d_comp, n, K, 0x5EEDull, d_smp);
    std::vector<int32_t> smp(K);
    const int rc = copy_sync(c, smp.data(), d_smp, K * 4, hipMemcpyDeviceToHost);
    dfree(&d_smp);
    GP_TRY(rc);
    std::sort(smp.begin(), smp.end());
    int best = 0;
    for (int i = 0, j; i < K; i = j) {
      for (j = i; j < K && smp[(size_t)j] == smp[(size_t)i]; ++j) {}
      if (j - i > best) {
        best = j - i;
        skip = smp[(size_t)i];
      }
    }
  }
  hipLaunchKernelGGL(k_cc_rest, g, dim3(256), 0, s, c->d_row_ptr, c->d_col, c->d_comp, n,
                     skip);
  hipLaunchKernelGGL(k_cc_final, g, dim3(256), 0, s, c->d_comp, n);
  GP_HIP(hipGetLastError());
  return 0;
}

int finish_graph(Ctx* c) {
  free_state(c);
  free_partition(c);   // a new overlay: partition again from the global CSR
  c->nnz_l = c->nnz;
  GP_TRY(dalloc(&c->d_deg_out, (size_t)c->n));
  const int64_t* rp = c->directed ? c->d_out_row_ptr : c->d_row_ptr;
  hipLaunchKernelGGL(k_degree, dim3(grid_for(c->n, 256)), dim3(256), 0, c->stream, rp, c->d_deg_out, c->n);
  GP_HIP(hipGetLastError());
  // weakly connected components (arcs in either direction)
  GP_TRY(dalloc(&c->d_comp, (size_t)c->n));
  GP_TRY(components(c));
  GP_TRY(build_gather_order(c));
  dfree(&c->d_prehi);   // (degree-split prefixes: rebuilt on first use for this overlay)
  c->prehi_deg = 0;
  c->h_deg_out.resize((size_t)c->n);
  GP_HIP(hipMemcpyAsync(c->h_deg_out.data(), c->d_deg_out, (size_t)c->n * 4, hipMemcpyDeviceToHost, c->stream));
  c->h_row_ptr.resize((size_t)c->n + 1);
  GP_HIP(hipMemcpyAsync(c->h_row_ptr.data(), c->d_row_ptr, ((size_t)c->n + 1) * sizeof(int64_t),
                        hipMemcpyDeviceToHost, c->stream));
  GP_HIP(hipStreamSynchronize(c->stream));
  c->m = 0;
  c->words = 0;
  const int32_t rank = c->rank, nranks = c->nranks;
  c->rank = 0;
  c->nranks = 1;
  return set_partition(c, rank, nranks);
}

// (re)allocate per-run state for the current graph/messages/config
static int alloc_state(Ctx* c) {
  if (c->n <= 0) return set_error(GP_ESTATE, "no graph loaded");
  if (c->words <= 0) return set_error(GP_ESTATE, "no messages set");
  const size_t W = (size_t)c->words, na = (size_t)c->n_alloc, nl = (size_t)std::max<int64_t>(c->nloc(), 1);
  // exact frontier rows only for per-message forwards (the pull reads whole
  // Message-Lists) and for the boundary exchange of a vertex
  // partition, which sends owned vertices' new bits: the owned rows only (a
  // ghost's slot row is its frontier)
  c->frx_rows = c->local ? c->nloc() : (c->cfg.track_msg_forwards ? c->n_alloc : 0);
  dfree(&c->d_slot[2]);   // (re)allocated at the first parking, for this W
  c->park_failed = false;
  // S[0] | S[1] | accumulator rows of the owned receivers, one allocation
  free_rows(c);
  GP_TRY(dalloc(&c->d_rows, (2 * na + nl) * W));
  c->d_slot[0] = c->d_rows;
  c->d_slot[1] = c->d_rows + na * W;
  c->d_acc = c->d_rows + 2 * na * W;
  for (int k = 0; k < 2; ++k) {
    GP_TRY(dalloc(&c->d_fpop[k], na));
    if (c->frx_rows > 0 || c->local) GP_TRY(dalloc(&c->d_frx[k], (size_t)std::max<int64_t>(c->frx_rows, 1) * W));
    else dfree(&c->d_frx[k]);
  }
  GP_TRY(dalloc(&c->d_sp, na));
  GP_TRY(dalloc(&c->d_ws, na));
  GP_TRY(dalloc(&c->d_seenpop, nl));
  if (c->cfg.track_first) GP_TRY(dalloc(&c->d_first, nl * W * 64));
  else dfree(&c->d_first);
  GP_TRY(dalloc(&c->d_digest, nl));
  GP_TRY(dalloc(&c->d_state, na));
  GP_TRY(dalloc(&c->d_miss, na));
  GP_TRY(dalloc(&c->d_deg_live, na));
  GP_TRY(dalloc(&c->d_cand, na));
  GP_TRY(dalloc(&c->d_det_big, (size_t)DET_CAP));
  GP_TRY(dalloc(&c->d_det_pre, (size_t)DET_CAP + 1));
  GP_TRY(dalloc(&c->d_det_live, (size_t)DET_CAP));
  GP_TRY(dalloc(&c->d_det_cur, (size_t)DET_CAP));
  GP_TRY(dalloc(&c->d_det_base, (size_t)DET_CAP));
  GP_TRY(dalloc(&c->d_abits, (na + 63) / 64));
  GP_TRY(dalloc(&c->d_dbits, (na + 63) / 64));
  dfree(&c->d_lm);
  if (c->words == 64) GP_TRY(dalloc(&c->d_lm, (na + 1) / 2 + 32));
  for (int k = 0; k < 2; ++k) {
    dfree(&c->d_lmw[k]);
    if (c->words == 64) GP_TRY(dalloc(&c->d_lmw[k], (na + 1) / 2 + 64));
  }
  GP_TRY(dalloc(&c->d_sbits, (na + 4095) / 4096));
  // compact Message-Lists: 2 x 128 B per vertex, single-rank W = 64 runs only
  if (c->cfg.compact_rows && W == 64 && c->nranks == 1) {
    GP_TRY(dalloc(&c->d_cml[0], na * CML_WORDS));
    GP_TRY(dalloc(&c->d_cml[1], na * CML_WORDS));
    GP_TRY(dalloc(&c->d_cmk[0], (na + 63) / 64));   // dense bitmaps
    GP_TRY(dalloc(&c->d_cmk[1], (na + 63) / 64));
  } else {
    dfree(&c->d_cml[0]);
    dfree(&c->d_cml[1]);
    dfree(&c->d_cmk[0]);
    dfree(&c->d_cmk[1]);
  }
  GP_TRY(dalloc(&c->d_amask, (size_t)((c->nnz_l + 63) / 64 + 2)));
  GP_HIP(hipMemsetAsync(c->d_amask, 0, (size_t)((c->nnz_l + 63) / 64 + 2) * 8, c->stream));
  GP_TRY(dalloc(&c->d_done_at, na));
  c->done_at_valid = false;
  GP_HIP(hipMemsetAsync(c->d_acc, 0, nl * W * 8, c->stream));   // (kept all-zero between uses)
  GP_TRY(dalloc(&c->d_tbits, (na + 63) / 64));
  GP_HIP(hipMemsetAsync(c->d_tbits, 0, (na + 63) / 64 * 8, c->stream));
  GP_TRY(dalloc(&c->d_nbits, (na + 63) / 64));
  GP_TRY(dalloc(&c->d_touched, na));
  GP_TRY(dalloc(&c->d_active, na));
  GP_TRY(dalloc(&c->d_big, na));
  GP_TRY(dalloc(&c->d_msg_cov, W * 64 * 4));
  GP_TRY(dalloc(&c->d_alive, 2 * W));   // [local cov | local fwd | global cov | global fwd]
  c->d_msg_fwd = c->d_msg_cov + W * 64;
  c->report_cap = std::max<int64_t>(c->cfg.report_capacity, 1);
  GP_TRY(dalloc(&c->d_reports, (size_t)c->report_cap));
  GP_TRY(dalloc(&c->d_hub_partial, std::max<size_t>(c->h_hub_items.size(), 1) * W));
  if (c->local) GP_TRY(alloc_exchange(c));
  GP_HIP(hipStreamSynchronize(c->stream));
  return 0;
}


__global__ void k_midx(const int32_t* __restrict__ comp, const int32_t* __restrict__ idx_of_root,
                       int32_t* __restrict__ midx, int64_t n) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) midx[v] = idx_of_root[comp[v]];
}

// done_at[v] = number of messages originating in v's weakly connected component;
// cmask[midx[v]] = those messages as a W-word row (the early-exit target)
static int compute_done_at(Ctx* c, int64_t groups) {
  uint32_t* cnt = nullptr;
  GP_TRY(dalloc(&cnt, (size_t)c->n));
  hipStream_t s = c->stream;
  GP_HIP(hipMemsetAsync(cnt, 0, (size_t)c->n * 4, s));
  GP_HIP(hipMemsetAsync(c->d_done_at, 0, (size_t)c->n_alloc * 4, s));
  // (labels are global vertex ids: cnt is indexed by label, the rest by local id)
  if (groups > 0)
    hipLaunchKernelGGL(k_count_origins, dim3(grid_for(groups, 256)), dim3(256), 0, s, c->d_inj_origin,
                       c->d_inj_cnt, groups, c->d_comp, cnt);
  hipLaunchKernelGGL(k_done_at, dim3(grid_for(c->n_alloc, 256)), dim3(256), 0, s, c->d_comp, cnt, c->d_done_at,
                     c->n_alloc);
  GP_HIP(hipGetLastError());
  GP_HIP(hipStreamSynchronize(s));
  dfree(&cnt);
  // component message masks (host: K <= #groups components carry messages)
  std::vector<int32_t> comp((size_t)c->n_alloc);
  GP_TRY(copy_sync(c, comp.data(), c->d_comp, (size_t)c->n_alloc * 4, hipMemcpyDeviceToHost));
  std::vector<int32_t> idx_of_root((size_t)c->n, -1);
  std::vector<u64> masks;
  const size_t W = (size_t)c->words;
  int32_t K = 0;
  for (int64_t g = 0; g < groups; ++g) {
    const int32_t root = comp[(size_t)c->h_inj_origin[(size_t)g]];
    if (idx_of_root[(size_t)root] < 0) {
      idx_of_root[(size_t)root] = K++;
      masks.resize((size_t)K * W, 0);
    }
    u64* row = masks.data() + (size_t)idx_of_root[(size_t)root] * W;
    for (size_t w = 0; w < W; ++w) row[w] |= c->h_inj_bits[(size_t)g * W + w];
  }
  if (masks.empty()) masks.assign(W, 0);
  GP_TRY(dalloc(&c->d_cmask, masks.size()));
  GP_TRY(copy_sync(c, c->d_cmask, masks.data(), masks.size() * 8, hipMemcpyHostToDevice));
  int32_t* ior = nullptr;
  GP_TRY(dalloc(&ior, (size_t)c->n));
  GP_TRY(copy_sync(c, ior, idx_of_root.data(), (size_t)c->n * 4, hipMemcpyHostToDevice));
  GP_TRY(dalloc(&c->d_midx, (size_t)c->n_alloc));
  // on the engine stream: the stream is non-blocking, so a null-stream memset
  // could land after k_midx
  GP_HIP(hipMemsetAsync(c->d_midx, 0xFF, (size_t)c->n_alloc * 4, s));
  hipLaunchKernelGGL(k_midx, dim3(grid_for(c->n_alloc, 256)), dim3(256), 0, s, c->d_comp, ior, c->d_midx,
                     c->n_alloc);
  GP_HIP(hipGetLastError());
  // pristine targets (a run drops its lost messages from the working ones)
  c->cmask_rows = (int32_t)(masks.size() / W);
  GP_TRY(dalloc(&c->d_cmask0, masks.size()));
  GP_TRY(dalloc(&c->d_done_at0, (size_t)c->n_alloc));
  GP_TRY(dalloc(&c->d_lostcnt, (size_t)c->cmask_rows));
  GP_HIP(hipMemcpyAsync(c->d_cmask0, c->d_cmask, masks.size() * 8, hipMemcpyDeviceToDevice, s));
  GP_HIP(hipMemcpyAsync(c->d_done_at0, c->d_done_at, (size_t)c->n_alloc * 4, hipMemcpyDeviceToDevice, s));
  c->done_dirty = false;
  GP_HIP(hipStreamSynchronize(s));
  dfree(&ior);
  return 0;
}


}  // namespace gp

using namespace gp;

// ===========================================================================
// C-ABI
extern "C" {


void gp_default_config(gp_config* cfg) {
  if (!cfg) return;
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->track_first = 0;
  cfg->track_digest = 1;
  cfg->track_msg_forwards = 0;
  cfg->churn = 0;
  cfg->p_fail = 0.0;
  cfg->churn_seed = 0;
  cfg->miss_threshold = 3;     // 2 missed heartbeats + 1 unanswered PING (Peer.py:299-311)
  cfg->hub_threshold = 4096;
  cfg->report_capacity = 1 << 20;
  cfg->push_ratio = 100.0;   // push when sender arcs <= nnz / 100
  cfg->early_exit = 1;
  cfg->arc_mask_permille = 0;   // per-arc mask off: its build costs what it saves
  cfg->prefilter_pct = 20;
  cfg->compact_rows = 0;   // off: the per-receiver loop is latency-bound in the rounds it would serve
  cfg->unfiltered_pct = 90;
  cfg->msg_word_base = 0;
  cfg->flat_max_words = 16;
  cfg->summary_min_n = 1ll << 25;   // activity bitmap > 4 MB: outgrows an XCD's L2
  cfg->partition_by_arcs = 0;       // vertex partitions: equal vertex counts (1: equal arc counts)
#ifndef GP_SPLIT_DEG_DEFAULT
#define GP_SPLIT_DEG_DEFAULT 128
#endif
#ifndef GP_SPLIT_MAX_PERMILLE
#define GP_SPLIT_MAX_PERMILLE 10
#endif
  cfg->split_deg = GP_SPLIT_DEG_DEFAULT;   // degree-split sparse rounds
  cfg->split_max_permille = GP_SPLIT_MAX_PERMILLE;   // ... while senders are a sliver
}

int gp_create(int device, gp_ctx** out) {
  if (!out) return set_error(GP_EINVAL, "null out");
  *out = nullptr;
  int ndev = 0;
  GP_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return set_error(GP_EINVAL, "device index out of range");
  GP_HIP(hipSetDevice(device));
  gp_ctx* c = new gp_ctx();
  c->device = device;
  gp_default_config(&c->cfg);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->cu_count = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return set_error(GP_EHIP, "hipStreamCreate failed");
  }
  for (auto& e : c->ev) (void)hipEventCreate(&e);
  if (dalloc(&c->d_stats, 64 + (size_t)NPART * NST) != 0) {
    gp_destroy(c);
    return GP_ENOMEM;
  }
  (void)hipMemsetAsync(c->d_stats, 0, (64 + (size_t)NPART * NST) * sizeof(u64), c->stream);
  (void)hipStreamSynchronize(c->stream);
  (void)hipHostMalloc((void**)&c->h_stats, 64 * sizeof(u64), hipHostMallocDefault);
  *out = c;
  return 0;
}

void gp_destroy(gp_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  shard_free(c);
  dfree(&c->d_row_ptr); dfree(&c->d_col); dfree(&c->d_out_row_ptr); dfree(&c->d_out_col);
  dfree(&c->d_deg_out); dfree(&c->d_comp); dfree(&c->d_abits); dfree(&c->d_dbits); dfree(&c->d_lm); dfree(&c->d_lmw[0]); dfree(&c->d_lmw[1]); dfree(&c->d_sbits); dfree(&c->d_amask); dfree(&c->d_cml[0]); dfree(&c->d_cml[1]); dfree(&c->d_cmk[0]); dfree(&c->d_cmk[1]); dfree(&c->d_done_at);
  dfree(&c->d_done_at0); dfree(&c->d_cmask0); dfree(&c->d_lostcnt); dfree(&c->d_alive);
  dfree(&c->d_gcol); dfree(&c->d_prehi); dfree(&c->d_midx); dfree(&c->d_cmask);
  dfree(&c->d_tbits); dfree(&c->d_nbits); dfree(&c->d_touched); dfree(&c->d_active); dfree(&c->d_big);
  dfree(&c->d_inj_origin); dfree(&c->d_inj_bits); dfree(&c->d_inj_cnt);
  dfree(&c->d_slot[2]);
  free_rows(c);
  for (int k = 0; k < 2; ++k) { dfree(&c->d_frx[k]); dfree(&c->d_fpop[k]); }
  dfree(&c->d_sp); dfree(&c->d_ws);
  dfree(&c->d_ulist[0]); dfree(&c->d_ulist[1]);
  dfree(&c->d_seenpop); dfree(&c->d_first); dfree(&c->d_digest);
  dfree(&c->d_state); dfree(&c->d_miss); dfree(&c->d_deg_live); dfree(&c->d_cand);
  dfree(&c->d_det_big); dfree(&c->d_det_pre); dfree(&c->d_det_live); dfree(&c->d_det_cur); dfree(&c->d_det_base);
  dfree(&c->d_msg_cov); dfree(&c->d_reports); dfree(&c->d_stats);
  dfree(&c->d_hub_items); dfree(&c->d_hubs); dfree(&c->d_hub_item_ptr);
  dfree(&c->d_hub_partial); dfree(&c->d_hub_pnz); dfree(&c->d_hub_done);
  bitcount_free(c);
  if (c->h_stats) (void)hipHostFree(c->h_stats);
  for (auto& e : c->ev) if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int gp_configure(gp_ctx* c, const gp_config* cfg) {
  if (!c || !cfg) return set_error(GP_EINVAL, "null argument");
  if (cfg->p_fail < 0.0 || !(cfg->p_fail <= 1.0)) return set_error(GP_EINVAL, "p_fail must be in [0,1]");
  if (cfg->miss_threshold < 1 || cfg->miss_threshold > 254) return set_error(GP_EINVAL, "miss_threshold in [1,254]");
  if (cfg->hub_threshold < 64) return set_error(GP_EINVAL, "hub_threshold must be >= 64");
  if (cfg->report_capacity < 0) return set_error(GP_EINVAL, "report_capacity < 0");
  if (cfg->msg_word_base < 0) return set_error(GP_EINVAL, "msg_word_base < 0");
  if (cfg->prefilter_pct < 0) return set_error(GP_EINVAL, "prefilter_pct < 0");
  if (cfg->summary_min_n < 0) return set_error(GP_EINVAL, "summary_min_n < 0");
  if (cfg->compact_rows != 0 && cfg->compact_rows != 1) return set_error(GP_EINVAL, "compact_rows must be 0 or 1");
  if (cfg->arc_mask_permille < 0) return set_error(GP_EINVAL, "arc_mask_permille < 0");
  if (cfg->partition_by_arcs != 0 && cfg->partition_by_arcs != 1)
    return set_error(GP_EINVAL, "partition_by_arcs must be 0 or 1");
  if (cfg->split_deg < 0) return set_error(GP_EINVAL, "split_deg must be >= 0");
  if (cfg->split_max_permille < 0) return set_error(GP_EINVAL, "split_max_permille must be >= 0");
  if (c->local && cfg->partition_by_arcs != c->cfg.partition_by_arcs)
    return set_error(GP_ESTATE, "a partitioned context keeps its partition: reload the overlay to change it");
  GP_HIP(hipSetDevice(c->device));
  const bool hub_changed = cfg->hub_threshold != c->cfg.hub_threshold;
  c->cfg = *cfg;
  if (c->n > 0 && hub_changed) GP_TRY(build_hubs(c));
  if (state_ready(c)) GP_TRY(alloc_state(c));
  return 0;
}

int gp_load_graph(gp_ctx* c, int64_t n, int64_t nnz, const int64_t* row_ptr, const int32_t* col,
                  int32_t directed, const int64_t* out_row_ptr, const int32_t* out_col) {
  if (!c || !row_ptr || (nnz > 0 && !col)) return set_error(GP_EINVAL, "null argument");
  if (n <= 0 || n >= (int64_t)0x7fffffff) return set_error(GP_EINVAL, "n out of range");
  if (nnz < 0 || row_ptr[0] != 0 || row_ptr[n] != nnz) return set_error(GP_EINVAL, "row_ptr inconsistent with nnz");
  for (int64_t v = 0; v < n; ++v)
    if (row_ptr[v + 1] < row_ptr[v]) return set_error(GP_EINVAL, "row_ptr not monotone");
  for (int64_t j = 0; j < nnz; ++j)
    if (col[j] < 0 || col[j] >= n) return set_error(GP_EINVAL, "col index out of range");
  GP_HIP(hipSetDevice(c->device));
  std::vector<int64_t> orp;
  std::vector<int32_t> ocol;
  if (directed) {
    if (out_row_ptr && out_col) {
      if (out_row_ptr[0] != 0 || out_row_ptr[n] != nnz) return set_error(GP_EINVAL, "out CSR inconsistent");
      orp.assign(out_row_ptr, out_row_ptr + n + 1);
      ocol.assign(out_col, out_col + nnz);
    } else {   // transpose the in-CSR: out(u) = {v : u in In(v)}
      orp.assign((size_t)n + 1, 0);
      for (int64_t j = 0; j < nnz; ++j) orp[(size_t)col[j] + 1]++;
      for (int64_t v = 0; v < n; ++v) orp[v + 1] += orp[v];
      ocol.resize((size_t)nnz);
      std::vector<int64_t> cur(orp.begin(), orp.end() - 1);
      for (int64_t v = 0; v < n; ++v)
        for (int64_t j = row_ptr[v]; j < row_ptr[v + 1]; ++j) ocol[cur[col[j]]++] = (int32_t)v;
    }
  }
  c->n = n;
  c->nnz = nnz;
  c->directed = directed ? 1 : 0;
  GP_TRY(dalloc(&c->d_row_ptr, (size_t)n + 1));
  GP_TRY(dalloc(&c->d_col, (size_t)nnz));
  GP_TRY(copy_sync(c, c->d_row_ptr, row_ptr, ((size_t)n + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (nnz) GP_TRY(copy_sync(c, c->d_col, col, (size_t)nnz * sizeof(int32_t), hipMemcpyHostToDevice));
  if (directed) {
    GP_TRY(dalloc(&c->d_out_row_ptr, (size_t)n + 1));
    GP_TRY(dalloc(&c->d_out_col, (size_t)nnz));
    GP_TRY(copy_sync(c, c->d_out_row_ptr, orp.data(), ((size_t)n + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
    if (nnz) GP_TRY(copy_sync(c, c->d_out_col, ocol.data(), (size_t)nnz * sizeof(int32_t), hipMemcpyHostToDevice));
  } else {
    dfree(&c->d_out_row_ptr);
    dfree(&c->d_out_col);
  }
  return finish_graph(c);
}

int gp_build_chung_lu(gp_ctx* c, int64_t n, double dbar, double gamma, uint64_t seed) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  if (n < 2 || n >= (int64_t)0x7fffffff) return set_error(GP_EINVAL, "n out of range");
  if (!(dbar > 0.0) || !(gamma > 2.0)) return set_error(GP_EINVAL, "need dbar > 0 and gamma > 2");
  GP_HIP(hipSetDevice(c->device));
  GP_TRY(build_chung_lu(c, n, dbar, gamma, seed));
  return finish_graph(c);
}

int gp_set_partition(gp_ctx* c, int32_t rank, int32_t nranks) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  if (c->n <= 0) return set_error(GP_ESTATE, "load a graph first");
  GP_HIP(hipSetDevice(c->device));
  GP_TRY(set_partition(c, rank, nranks));
  if (state_ready(c)) GP_TRY(alloc_state(c));
  return 0;
}

int gp_get_partition(gp_ctx* c, int64_t* vbegin, int64_t* vend) {
  if (!c || !vbegin || !vend) return set_error(GP_EINVAL, "null argument");
  *vbegin = c->vbegin;
  *vend = c->vend;
  return 0;
}

int gp_comm_unique_id(void* out128) {
  if (!out128) return set_error(GP_EINVAL, "null out");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  GP_RCCL(ncclGetUniqueId(&id));
  std::memcpy(out128, &id, sizeof(id));
  return 0;
}

int gp_comm_init(gp_ctx* c, const void* uid, int32_t nranks, int32_t rank) {
  if (!c || !uid) return set_error(GP_EINVAL, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return set_error(GP_EINVAL, "bad rank/nranks");
  GP_HIP(hipSetDevice(c->device));
  if (c->comm) {
    (void)ncclCommDestroy(c->comm);
    c->comm = nullptr;
  }
  if (nranks != c->nranks || rank != c->rank)
    return set_error(GP_EINVAL, "gp_comm_init: rank/nranks differ from the context's partition");
  // (one rank too: its exchange is the counters' all-reduce over a real
  // communicator, which is what a one-GPU box can test)
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  GP_RCCL(ncclCommInitRank(&c->comm, nranks, id, rank));
  return 0;
}

int gp_set_messages(gp_ctx* c, int32_t m, const int32_t* origin, const int32_t* inject_round) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  if (c->n <= 0) return set_error(GP_ESTATE, "load a graph first");
  if (m < 1 || m > 4096) return set_error(GP_EINVAL, "m must be in [1, 4096] per context");
  if (!origin) return set_error(GP_EINVAL, "null origin");
  GP_HIP(hipSetDevice(c->device));
  int words = 1;
  while (words * 64 < m) words <<= 1;
  // group by (round, origin)
  std::vector<std::pair<std::pair<int32_t, int32_t>, int32_t>> key((size_t)m);
  int32_t last = -1;
  for (int32_t k = 0; k < m; ++k) {
    const int32_t o = origin[k];
    const int32_t r = inject_round ? inject_round[k] : 0;
    if (o < 0 || o >= c->n) return set_error(GP_EINVAL, "origin out of range");
    if (r < 0 || r > 253) return set_error(GP_EINVAL, "inject_round must be in [0, 253]");
    key[(size_t)k] = {{r, o}, k};
    last = std::max(last, r);
  }
  std::sort(key.begin(), key.end());
  std::vector<int32_t> g_origin;
  std::vector<u64> g_bits;
  std::vector<uint32_t> g_cnt;
  c->inject.clear();
  for (size_t k = 0; k < key.size();) {
    const int32_t r = key[k].first.first, o = key[k].first.second;
    auto& span = c->inject[r];
    if (span.cnt == 0) span.off = (int64_t)g_origin.size();
    g_origin.push_back(o);
    g_bits.resize(g_bits.size() + (size_t)words, 0);
    u64* row = g_bits.data() + g_bits.size() - words;
    uint32_t cnt = 0;
    while (k < key.size() && key[k].first.first == r && key[k].first.second == o) {
      const int32_t msg = key[k].second;
      row[msg >> 6] |= 1ull << (msg & 63);
      ++cnt;
      ++k;
    }
    g_cnt.push_back(cnt);
    span.cnt++;
  }
  c->inj_arcs.assign((size_t)std::max(last + 1, 0), 0);
  for (auto& kv : c->inject)   // (global out-degrees: every rank takes the same direction)
    for (int64_t g = kv.second.off; g < kv.second.off + kv.second.cnt; ++g)
      c->inj_arcs[(size_t)kv.first] += c->h_deg_out[(size_t)g_origin[(size_t)g]];
  const int64_t nv_before = c->n_alloc;
  if (c->local) {   // every origin becomes a local vertex (partition.hip), then local ids
    GP_TRY(set_extras(c, g_origin));
    for (auto& o : g_origin) o = (int32_t)c->to_local(o);
  }
  c->m = m;
  c->last_inject_round = last;
  const bool realloc = words != c->words || c->n_alloc != nv_before;
  c->words = words;
  GP_TRY(dalloc(&c->d_inj_origin, g_origin.size()));
  GP_TRY(dalloc(&c->d_inj_bits, g_bits.size()));
  GP_TRY(dalloc(&c->d_inj_cnt, g_cnt.size()));
  GP_TRY(copy_sync(c, c->d_inj_origin, g_origin.data(), g_origin.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  GP_TRY(copy_sync(c, c->d_inj_bits, g_bits.data(), g_bits.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
  GP_TRY(copy_sync(c, c->d_inj_cnt, g_cnt.data(), g_cnt.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  if (realloc || !state_ready(c)) GP_TRY(alloc_state(c));
  c->n_groups = (int64_t)g_origin.size();
  c->h_inj_origin = g_origin;
  c->h_inj_bits = g_bits;
  c->done_at_valid = false;
  return 0;
}

int gp_spread_keys(gp_ctx* c, int32_t hops, int32_t m, const int32_t* origin, uint64_t* keys_out) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  if (c->n <= 0 || !c->d_row_ptr || !c->d_col || c->local)
    return set_error(GP_ESTATE, "gp_spread_keys needs the global overlay (before a vertex partition)");
  if (hops < 1 || hops > 3) return set_error(GP_EINVAL, "hops must be 1, 2 or 3");
  if (m < 0 || (m > 0 && (!origin || !keys_out))) return set_error(GP_EINVAL, "bad message table");
  if (m == 0) return 0;
  for (int32_t k = 0; k < m; ++k)
    if (origin[k] < 0 || origin[k] >= c->n) return set_error(GP_EINVAL, "origin out of range");
  GP_HIP(hipSetDevice(c->device));
  std::vector<u64> keys((size_t)m);
  if (hops == 1) {
    std::vector<int64_t> rp(2);
    for (int32_t k = 0; k < m; ++k) {
      GP_TRY(copy_sync(c, rp.data(), c->d_row_ptr + origin[k], 2 * sizeof(int64_t), hipMemcpyDeviceToHost));
      keys[(size_t)k] = (u64)(rp[1] - rp[0]);
    }
  } else {
    int32_t* d_o = nullptr;
    u64 *d_k = nullptr, *d_s2 = nullptr;
    // every allocation goes through rc, so the frees below always run
    int rc = 0;
    if (hipMalloc(&d_o, (size_t)m * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&d_k, (size_t)m * sizeof(u64)) != hipSuccess)
      rc = set_error(GP_ENOMEM, "gp_spread_keys: message scratch");
    if (rc == 0) rc = copy_sync(c, d_o, origin, (size_t)m * sizeof(int32_t), hipMemcpyHostToDevice);
    if (rc == 0 && hops == 3 && hipMalloc(&d_s2, (size_t)c->n * sizeof(u64)) != hipSuccess)
      rc = set_error(GP_ENOMEM, "gp_spread_keys: n u64 of scratch");
    if (rc == 0) {
      // grid-stride kernel: at most 64 K blocks (n / 4 blocks of 256 threads
      // would overflow the 2^32-thread grid at 2^26 vertices)
      if (hops == 3)   // hops-2 key of every vertex, then summed over the origins' neighbours
        hipLaunchKernelGGL(k_nbsum, dim3(std::min(grid_for(c->n, BLOCK / 64), 65536)), dim3(BLOCK), 0, c->stream,
                           c->d_row_ptr, c->d_col, (const u64*)nullptr, (const int32_t*)nullptr, c->n, d_s2);
      hipLaunchKernelGGL(k_nbsum, dim3(std::min(grid_for(m, BLOCK / 64), 65536)), dim3(BLOCK), 0, c->stream,
                         c->d_row_ptr, c->d_col, (const u64*)d_s2, (const int32_t*)d_o, (int64_t)m, d_k);
      if (hipGetLastError() != hipSuccess) rc = set_error(GP_EHIP, "gp_spread_keys: launch failed");
      if (rc == 0) rc = copy_sync(c, keys.data(), d_k, (size_t)m * sizeof(u64), hipMemcpyDeviceToHost);
    }
    if (d_o) (void)hipFree(d_o);
    if (d_k) (void)hipFree(d_k);
    if (d_s2) (void)hipFree(d_s2);
    if (rc) return rc;
  }
  std::memcpy(keys_out, keys.data(), (size_t)m * sizeof(u64));
  return 0;
}

int gp_reset(gp_ctx* c) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  if (!state_ready(c)) GP_TRY(alloc_state(c));
  GP_HIP(hipSetDevice(c->device));
  if (!c->done_at_valid) {
    GP_TRY(compute_done_at(c, c->n_groups));
    c->done_at_valid = true;
  } else if (c->done_dirty) {   // undo the previous run's lost-message drops
    GP_HIP(hipMemcpyAsync(c->d_cmask, c->d_cmask0, (size_t)c->cmask_rows * c->words * 8,
                          hipMemcpyDeviceToDevice, c->stream));
    GP_HIP(hipMemcpyAsync(c->d_done_at, c->d_done_at0, (size_t)c->n_alloc * 4, hipMemcpyDeviceToDevice,
                          c->stream));
    c->done_dirty = false;
  }
  const size_t W = (size_t)c->words, na = (size_t)c->n_alloc, nl = (size_t)std::max<int64_t>(c->nloc(), 1);
  hipStream_t s = c->stream;
  // the slot buffers are not cleared: sp = none marks every row as absent
  GP_HIP(hipMemsetAsync(c->d_sp, SLOT_NONE, na, s));
  GP_HIP(hipMemsetAsync(c->d_ws, 0, na, s));
  GP_HIP(hipMemsetAsync(c->d_seenpop, 0, nl * 4, s));
  GP_HIP(hipMemsetAsync(c->d_fpop[0], 0, na * 4, s));
  GP_HIP(hipMemsetAsync(c->d_fpop[1], 0, na * 4, s));
  if (c->d_first) GP_HIP(hipMemsetAsync(c->d_first, 0xFF, nl * W * 64, s));
  GP_HIP(hipMemsetAsync(c->d_digest, 0, nl * 8, s));
  GP_HIP(hipMemsetAsync(c->d_state, 0, na, s));
  GP_HIP(hipMemsetAsync(c->d_tbits, 0, (na + 63) / 64 * 8, s));
  c->prev_next_arcs = 0;
  c->prev_new_bits = 0;
  c->prev_receivers = 0;
  c->held_bits = 0;
  c->cml_written_prev = false;
  c->cml_read_now = c->cml_write_now = false;
  c->lm_written_prev = c->lm_write_now = false;
  c->sate_since = -1;
  GP_HIP(hipMemsetAsync(c->d_miss, 0, na, s));
  GP_HIP(hipMemsetAsync(c->d_deg_live, 0, na * 4, s));
  GP_HIP(hipMemcpyAsync(c->d_deg_live, c->d_deg_out, (size_t)c->n_alloc * 4, hipMemcpyDeviceToDevice, s));
  GP_HIP(hipMemsetAsync(c->d_msg_cov, 0, W * 64 * 4 * 8, s));
  GP_HIP(hipMemsetAsync(c->d_alive, 0, 2 * W * 8, s));
  GP_HIP(hipMemsetAsync(c->d_stats, 0, (64 + (size_t)NPART * NST) * 8, s));
  c->cur = 0;
  c->round = 0;
  c->liveness_active = c->cfg.churn != 0;
  c->alive_from = c->liveness_active ? 0 : -1;
  c->pending_crash = false;
  c->msg_forwards_valid = true;
  c->last_reports = 0;
  c->alias_active = c->alias_now = c->dprobe_now = false;
  c->ulist_valid = c->ulist_emit_now = c->ulist_read_now = false;
  c->ulist_valid = c->ulist_emit_now = c->ulist_read_now = false;
  shard_reset(c);
  GP_HIP(hipStreamSynchronize(s));
  return 0;
}

int gp_crash(gp_ctx* c, int32_t nverts, const int32_t* verts) {
  if (!c || (nverts > 0 && !verts)) return set_error(GP_EINVAL, "null argument");
  if (!state_ready(c)) return set_error(GP_ESTATE, "gp_reset first");
  GP_HIP(hipSetDevice(c->device));
  for (int32_t k = 0; k < nverts; ++k)
    if (verts[k] < 0 || verts[k] >= c->n) return set_error(GP_EINVAL, "vertex out of range");
  // global ids; a partitioned context applies the crashes of the vertices it
  // holds (owned, ghosts, origins) -- the others never touch its slice
  GP_TRY(unalias(c, false));   // (liveness turns on: the run's rounds can no longer keep aliases)
  std::vector<uint8_t> st((size_t)c->n_alloc);
  GP_HIP(hipStreamSynchronize(c->stream));
  GP_TRY(copy_sync(c, st.data(), c->d_state, (size_t)c->n_alloc, hipMemcpyDeviceToHost));
  for (int32_t k = 0; k < nverts; ++k) {
    const int64_t v = c->to_local(verts[k]);
    if (v >= 0 && !(st[(size_t)v] & ST_DOWN)) st[(size_t)v] |= ST_PENDING;
  }
  GP_TRY(copy_sync(c, c->d_state, st.data(), (size_t)c->n_alloc, hipMemcpyHostToDevice));
  if (nverts > 0) {
    if (!c->liveness_active) c->alive_from = c->round + 1;   // (this round builds F_{round + 1})
    c->liveness_active = true;
    c->pending_crash = true;
  }
  return 0;
}

}  // extern "C"
