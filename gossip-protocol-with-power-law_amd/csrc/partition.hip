// partition.hip -- 1D vertex partition of the overlay and the per-round
// boundary exchange.
//
// The reference sends gossip only over real links (Peer.py:402-404), so a rank
// needs from its peers exactly the rows of the vertices it has links to.  Rank
// p owns the contiguous slice [vbegin, vend) of the randomly relabelled ids and
// keeps, in local ids:
//   [0, nloc)              owned vertices: full in-lists, Message-List rows
//   [nloc, nloc + nghost)  ghosts: the non-owned in-neighbours of owned vertices,
//                          sorted by global id (so grouped by owner); their row
//                          in the slot a round reads is their frontier of that
//                          round, delivered by the exchange; their in-list in
//                          the local CSR holds their OWNED neighbours (the push
//                          direction and the liveness reporters this rank sees)
//   [nloc + nghost, ...)   extras: message origins that are neither, so that
//                          every rank sees every origin's crash state (lost
//                          messages) and applies every injection
// Every overlay is undirected here (Seed.py:131-149 symmetrises the topology),
// so "owned vertex v is a ghost on rank q" <=> "v has a neighbour owned by q":
// the send list B_pq that rank p computes and the ghosts of owner p that rank q
// computes are the same vertices in the same (global id) order.  Entries are
// addressed by their index in that list; no id lists cross the wire.
//
// Per round, after the expansion (X_r):
//   pack     every owned boundary vertex that received new bits this round (or
//            was removed by this rank's seed step) becomes one entry per peer
//            holding it: a head (index | flags | popcount) and the word mask
//            of its new bits followed by the nonzero words -- the frontier, not
//            the Message-List: summed over a run each bit crosses once
//   counts   every rank all-gathers the per-peer (heads, words) counts
//   send     ncclSend / ncclRecv per peer pair inside one group (xGMI is
//            point-to-point: each pair of GPUs has its own link)
//   unpack   ghost frontier rows written into the slot the next round reads,
//            their popcounts, removal flags (deg_live of owned neighbours)
// plus the counters' all-reduce and the alive sets' OR (all-gather + OR).
// gp_round_group runs the same pack / unpack with device-to-device copies.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <rocprim/device/device_scan.hpp>
#include <string>
#include <vector>

#include "gp_internal.h"
#include "xplan.h"

namespace gp {

constexpr int PBLOCK = 256;
constexpr int PWAVES = PBLOCK / 64;
constexpr int MAX_PARTS = 64;      // ranks of a vertex partition (kernel-argument tables)
constexpr u64 LOW40 = (1ull << 40) - 1ull;

// global -> local id (-1: this context does not hold the vertex)
int64_t Ctx::to_local(int64_t g) const {
  if (!local) return (g >= 0 && g < n) ? g : -1;
  if (g >= vbegin && g < vend) return g - vbegin;
  auto find = [&](int64_t lo, int64_t hi) -> int64_t {
    auto b = h_l2g.begin() + lo, e = h_l2g.begin() + hi;
    auto it = std::lower_bound(b, e, (int32_t)g);
    return (it != e && *it == (int32_t)g) ? (int64_t)(it - h_l2g.begin()) : -1;
  };
  const int64_t r = find(nloc(), base_nv);   // ghosts
  return r >= 0 ? r : find(base_nv, n_alloc);   // extras
}

void free_partition(Ctx* c) {
  dfree(&c->d_l2g);
  dfree(&c->d_bnd_e); dfree(&c->d_bnd_k); dfree(&c->d_bvx_v); dfree(&c->d_bvx_ptr); dfree(&c->d_bvx_t);
  dfree(&c->d_bnd_ptr);
  dfree(&c->d_bvx_info); dfree(&c->d_bvx_flag); dfree(&c->d_bnd_scan); dfree(&c->d_xsize);
  dfree(&c->d_sbuf_h); dfree(&c->d_sbuf_w); dfree(&c->d_rbuf_h); dfree(&c->d_rbuf_w); dfree(&c->d_rscan);
  dfree(&c->d_cnt); dfree(&c->d_cnt_all); dfree(&c->d_alive_all);
  if (c->d_scan_tmp) { (void)hipFree(c->d_scan_tmp); c->d_scan_tmp = nullptr; }
  c->scan_tmp_bytes = 0;
  if (c->h_cnt_all) { (void)hipHostFree(c->h_cnt_all); c->h_cnt_all = nullptr; }
  c->local = false;
  c->nghost = c->nextra = 0;
  c->n_bnd = c->n_bvx = 0;
  c->h_l2g.clear(); c->h_comp_g.clear(); c->h_bnd_ptr.clear(); c->h_gh_ptr.clear();
  c->h_ghosts_all.clear();
}

template <class T>
static int upload(Ctx* c, T** dst, const std::vector<T>& src) {
  GP_TRY(dalloc(dst, std::max<size_t>(src.size(), 1)));
  if (!src.empty()) GP_TRY(copy_sync(c, *dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

// per local vertex: global degree and component label (extras included)
static int upload_vertex_tables(Ctx* c) {
  const size_t nv = c->h_l2g.size();
  std::vector<int32_t> deg(nv), comp(nv);
  for (size_t x = 0; x < nv; ++x) {
    deg[x] = c->h_deg_out[(size_t)c->h_l2g[x]];   // global degree (finish_graph)
    comp[x] = c->h_comp_g[(size_t)c->h_l2g[x]];
  }
  GP_TRY(upload(c, &c->d_deg_out, deg));
  GP_TRY(upload(c, &c->d_comp, comp));
  GP_TRY(upload(c, &c->d_l2g, c->h_l2g));
  return upload(c, &c->d_row_ptr, c->h_row_ptr);
}

// global CSR (device + host row_ptr) -> this rank's local CSR and boundary lists
int localize(Ctx* c) {
  const int64_t n = c->n, P = c->nranks, p = c->rank;
  const int64_t vb = c->vbegin, ve = c->vend, nl = ve - vb;
  if (P > MAX_PARTS) return set_error(GP_EINVAL, "at most 64 ranks per vertex partition");
  const std::vector<int64_t>& rp = c->h_row_ptr;   // global row_ptr (finish_graph)
  const int64_t a0 = rp[(size_t)vb], a1 = rp[(size_t)ve];
  // only the owned rows of the global CSR are needed on the host
  std::vector<int32_t> col((size_t)(a1 - a0)), gcol((size_t)(a1 - a0));
  GP_TRY(copy_sync(c, col.data(), c->d_col + a0, col.size() * 4, hipMemcpyDeviceToHost));
  GP_TRY(copy_sync(c, gcol.data(), c->d_gcol + a0, gcol.size() * 4, hipMemcpyDeviceToHost));
  c->h_comp_g.resize((size_t)n);
  GP_TRY(copy_sync(c, c->h_comp_g.data(), c->d_comp, (size_t)n * 4, hipMemcpyDeviceToHost));
  auto owner = [&](int64_t u) { return owner_of(c->h_bounds, u); };

  // ghosts: non-owned in-neighbours of owned vertices, sorted
  std::vector<uint8_t> mark((size_t)n, 0);
  for (int32_t u : col)
    if (u < vb || u >= ve) mark[(size_t)u] = 1;
  std::vector<int32_t> ghosts;
  for (int64_t u = 0; u < n; ++u)
    if (mark[(size_t)u]) ghosts.push_back((int32_t)u);
  std::vector<uint8_t>().swap(mark);
  const int64_t ng = (int64_t)ghosts.size(), nv = nl + ng;
  c->h_gh_ptr.assign((size_t)P + 1, 0);
  for (int64_t q = 0; q <= P; ++q)
    c->h_gh_ptr[(size_t)q] =
        std::lower_bound(ghosts.begin(), ghosts.end(), (int32_t)c->h_bounds[(size_t)q]) - ghosts.begin();
  std::vector<int32_t> g2l((size_t)n, -1);
  for (int64_t i = 0; i < nl; ++i) g2l[(size_t)(vb + i)] = (int32_t)i;
  for (int64_t k = 0; k < ng; ++k) g2l[(size_t)ghosts[(size_t)k]] = (int32_t)(nl + k);

  // local CSR: owned rows (all neighbours, local ids; gather order kept), then
  // ghost rows (their owned neighbours)
  std::vector<int64_t> lrp((size_t)nv + 1, 0);
  for (int64_t i = 0; i < nl; ++i) lrp[(size_t)i + 1] = rp[(size_t)(vb + i) + 1] - rp[(size_t)(vb + i)];
  for (int32_t u : col)
    if (u < vb || u >= ve) lrp[(size_t)g2l[(size_t)u] + 1]++;
  for (int64_t x = 0; x < nv; ++x) lrp[(size_t)x + 1] += lrp[(size_t)x];
  const int64_t A = lrp[(size_t)nv];
  std::vector<int32_t> lcol((size_t)A), lgcol((size_t)A);
  {
    std::vector<int64_t> cur(lrp.begin() + nl, lrp.end() - 1);   // ghost row cursors
    for (int64_t i = 0; i < nl; ++i) {
      for (int64_t j = rp[(size_t)(vb + i)]; j < rp[(size_t)(vb + i) + 1]; ++j) {
        const int64_t jj = j - a0;
        const int32_t u = col[(size_t)jj];
        lcol[(size_t)(lrp[(size_t)i] + (j - rp[(size_t)(vb + i)]))] = g2l[(size_t)u];
        lgcol[(size_t)(lrp[(size_t)i] + (j - rp[(size_t)(vb + i)]))] = g2l[(size_t)gcol[(size_t)jj]];
        if (u < vb || u >= ve) {
          const int64_t g = g2l[(size_t)u] - nl;
          lcol[(size_t)cur[(size_t)g]] = (int32_t)i;
          lgcol[(size_t)cur[(size_t)g]] = (int32_t)i;
          cur[(size_t)g]++;
        }
      }
    }
  }
  std::vector<int32_t>().swap(g2l);

  // boundary lists: peer-major entries t, vertex-major owned boundary vertices k
  std::vector<int64_t> cnt((size_t)P, 0);
  std::vector<int64_t> stamp((size_t)P, -1);
  std::vector<int32_t> bvx_v, bvx_ptr(1, 0), peers_of;   // vertex-major: peers of vertex k
  for (int64_t i = 0; i < nl; ++i) {
    const size_t before = peers_of.size();
    for (int64_t j = rp[(size_t)(vb + i)]; j < rp[(size_t)(vb + i) + 1]; ++j) {
      const int32_t u = col[(size_t)(j - a0)];
      const int64_t q = owner(u);
      if (q == p || stamp[(size_t)q] == i) continue;
      stamp[(size_t)q] = i;
      peers_of.push_back((int32_t)q);
      cnt[(size_t)q]++;
    }
    if (peers_of.size() > before) {
      bvx_v.push_back((int32_t)i);
      bvx_ptr.push_back((int32_t)peers_of.size());
    }
  }
  c->h_bnd_ptr.assign((size_t)P + 1, 0);
  for (int64_t q = 0; q < P; ++q) c->h_bnd_ptr[(size_t)q + 1] = c->h_bnd_ptr[(size_t)q] + cnt[(size_t)q];
  const int64_t NB = c->h_bnd_ptr[(size_t)P], NK = (int64_t)bvx_v.size();
  std::vector<int32_t> bnd_e((size_t)NB), bnd_k((size_t)NB), bvx_t((size_t)NB);
  {
    std::vector<int64_t> cur(c->h_bnd_ptr.begin(), c->h_bnd_ptr.end() - 1);
    for (int64_t k = 0; k < NK; ++k) {   // vertices in increasing order: each B_pq comes out sorted
      for (int32_t x = bvx_ptr[(size_t)k]; x < bvx_ptr[(size_t)k + 1]; ++x) {
        const int32_t q = peers_of[(size_t)x];
        const int64_t t = cur[(size_t)q]++;
        bnd_e[(size_t)t] = (int32_t)(t - c->h_bnd_ptr[(size_t)q]);
        bnd_k[(size_t)t] = (int32_t)k;
        bvx_t[(size_t)x] = (int32_t)t;
      }
    }
  }
  // B_pq and rank q's ghosts of owner p must be the same list: their lengths
  // are compared across ranks before the first exchange (check_lists_*)

  // install: local CSR replaces the global one
  c->h_l2g.resize((size_t)nv);
  for (int64_t i = 0; i < nl; ++i) c->h_l2g[(size_t)i] = (int32_t)(vb + i);
  for (int64_t k = 0; k < ng; ++k) c->h_l2g[(size_t)(nl + k)] = ghosts[(size_t)k];
  c->h_row_ptr = std::move(lrp);
  c->nnz_l = A;
  c->nghost = ng;
  c->nextra = 0;
  c->base_nv = nv;
  c->n_alloc = nv;
  c->local = true;
  GP_TRY(upload_vertex_tables(c));
  GP_TRY(upload(c, &c->d_col, lcol));
  GP_TRY(upload(c, &c->d_gcol, lgcol));
  c->n_bnd = NB;
  c->n_bvx = NK;
  GP_TRY(upload(c, &c->d_bnd_e, bnd_e));
  GP_TRY(upload(c, &c->d_bnd_k, bnd_k));
  GP_TRY(upload(c, &c->d_bvx_v, bvx_v));
  GP_TRY(upload(c, &c->d_bvx_ptr, bvx_ptr));
  GP_TRY(upload(c, &c->d_bvx_t, bvx_t));
  GP_TRY(upload(c, &c->d_bnd_ptr, c->h_bnd_ptr));
  return 0;
}

int set_extras(Ctx* c, const std::vector<int32_t>& origins) {
  std::vector<int32_t> ex;
  for (int32_t o : origins) {
    if (o >= c->vbegin && o < c->vend) continue;
    auto b = c->h_l2g.begin() + c->nloc(), e = c->h_l2g.begin() + c->base_nv;
    if (std::binary_search(b, e, o)) continue;
    ex.push_back(o);
  }
  std::sort(ex.begin(), ex.end());
  ex.erase(std::unique(ex.begin(), ex.end()), ex.end());
  if ((int64_t)ex.size() == c->nextra &&
      std::equal(ex.begin(), ex.end(), c->h_l2g.begin() + c->base_nv))
    return 0;
  c->h_l2g.resize((size_t)c->base_nv);
  c->h_l2g.insert(c->h_l2g.end(), ex.begin(), ex.end());
  c->h_row_ptr.resize((size_t)c->base_nv + 1);
  c->h_row_ptr.insert(c->h_row_ptr.end(), ex.size(), c->h_row_ptr.back());   // no arcs
  c->nextra = (int64_t)ex.size();
  c->n_alloc = c->base_nv + c->nextra;
  return upload_vertex_tables(c);
}

static int scan_u64(Ctx* c, const u64* in, u64* out, size_t count) {
  size_t tb = c->scan_tmp_bytes;
  GP_HIP(rocprim::exclusive_scan(c->d_scan_tmp, tb, in, out, 0ull, count, rocprim::plus<u64>(), c->stream));
  return 0;
}

int alloc_exchange(Ctx* c) {
  const size_t W = (size_t)c->words, P = (size_t)c->nranks;
  const size_t NB = (size_t)c->n_bnd, NG = (size_t)c->nghost;
  GP_TRY(dalloc(&c->d_bvx_info, std::max<size_t>((size_t)c->n_bvx, 1)));
  GP_TRY(dalloc(&c->d_bvx_flag, std::max<size_t>((size_t)c->n_bvx, 1)));
  GP_TRY(dalloc(&c->d_bnd_scan, NB + 1));
  GP_TRY(dalloc(&c->d_xsize, std::max(NB, NG) + 1));   // scan inputs (sizes), out of place
  GP_TRY(dalloc(&c->d_sbuf_h, std::max<size_t>(NB, 1)));
  GP_TRY(dalloc(&c->d_sbuf_w, std::max<size_t>(NB * (W + 1), 1)));
  GP_TRY(dalloc(&c->d_rbuf_h, NG + 1));
  GP_TRY(dalloc(&c->d_rbuf_w, std::max<size_t>(NG * (W + 1), 1)));
  GP_TRY(dalloc(&c->d_rscan, NG + 1));
  GP_TRY(dalloc(&c->d_cnt, 4 * P));
  GP_TRY(dalloc(&c->d_cnt_all, 4 * P * P));
  GP_TRY(dalloc(&c->d_alive_all, std::max<size_t>(P * W, 1)));
  if (!c->h_cnt_all) GP_HIP(hipHostMalloc((void**)&c->h_cnt_all, 4 * P * P * sizeof(u64), hipHostMallocDefault));
  size_t t1 = 0, t2 = 0;
  GP_HIP(rocprim::exclusive_scan(nullptr, t1, c->d_xsize, c->d_bnd_scan, 0ull, NB + 1, rocprim::plus<u64>(),
                                 c->stream));
  GP_HIP(rocprim::exclusive_scan(nullptr, t2, c->d_xsize, c->d_rscan, 0ull, NG + 1, rocprim::plus<u64>(),
                                 c->stream));
  const size_t tb = std::max<size_t>(std::max(t1, t2), 16);
  if (tb > c->scan_tmp_bytes) {
    if (c->d_scan_tmp) (void)hipFree(c->d_scan_tmp);
    c->d_scan_tmp = nullptr;
    GP_HIP(hipMalloc(&c->d_scan_tmp, tb));
    c->scan_tmp_bytes = tb;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// pack: one wave per owned boundary vertex reads its new row once
__global__ __launch_bounds__(PBLOCK) void k_bnd_mark(const int32_t* __restrict__ bvx_v, int64_t nk,
                                                     const uint32_t* __restrict__ fpop_next,
                                                     const uint8_t* __restrict__ state,
                                                     const u64* __restrict__ frx_next, int32_t W,
                                                     u64* __restrict__ info, uint8_t* __restrict__ flag) {
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * PWAVES + (threadIdx.x >> 6);
  if (k >= nk) return;
  const int32_t v = bvx_v[k];
  const bool fresh = fpop_next[v] != 0u;
  u64 x = 0;
  if (fresh && lane < W) x = frx_next[(size_t)v * W + lane];
  const u64 mask = __ballot(x != 0ull);
  if (lane == 0) {
    info[k] = mask;
    flag[k] = (uint8_t)((fresh ? 1u : 0u) | ((state[v] & ST_RMNEW) ? 2u : 0u));
  }
}

// entry sizes, packed (heads << 40 | words): one head and 1 + popcount words
__global__ __launch_bounds__(PBLOCK) void k_bnd_size(const int32_t* __restrict__ bnd_k, int64_t nb,
                                                     const u64* __restrict__ info,
                                                     const uint8_t* __restrict__ flag, u64* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * PBLOCK + threadIdx.x;
  if (t > nb) return;
  u64 sz = 0;
  if (t < nb) {
    const int32_t k = bnd_k[t];
    if (flag[k]) sz = (1ull << 40) | (u64)(1 + __popcll(info[k]));
  }
  out[t] = sz;
}

__global__ __launch_bounds__(PBLOCK) void k_bnd_pack(const int32_t* __restrict__ bvx_v,
                                                     const int32_t* __restrict__ bvx_ptr,
                                                     const int32_t* __restrict__ bvx_t, int64_t nk,
                                                     const u64* __restrict__ info, const uint8_t* __restrict__ flag,
                                                     const u64* __restrict__ frx_next, int32_t W,
                                                     const int32_t* __restrict__ bnd_e, const u64* __restrict__ scan,
                                                     u64* __restrict__ sh, u64* __restrict__ sw) {
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * PWAVES + (threadIdx.x >> 6);
  if (k >= nk) return;
  const uint32_t f = flag[k];
  if (!f) return;
  const u64 mask = info[k];
  const int32_t v = bvx_v[k];
  u64 x = 0;
  if ((f & 1u) && lane < W) x = frx_next[(size_t)v * W + lane];
  const int idx = __popcll(mask & ((1ull << lane) - 1ull));
  const u64 head_hi = ((u64)f << 32) | ((u64)__popcll(mask) << 40);
  for (int32_t y = bvx_ptr[k]; y < bvx_ptr[k + 1]; ++y) {
    const int32_t t = bvx_t[y];
    const u64 off = scan[t];
    const u64 h = off >> 40, w = off & LOW40;
    if (lane == 0) {
      sh[h] = (u64)(uint32_t)bnd_e[t] | head_hi;
      sw[w] = mask;
    }
    if (x) sw[w + 1 + (u64)idx] = x;
  }
}

// per peer: head start, heads, word start, words; this rank's totals into the
// counter block (all-reduced with the others)
__global__ void k_bnd_counts(const u64* __restrict__ scan, const int64_t* __restrict__ bnd_ptr, int32_t P,
                             int32_t self, u64* __restrict__ cnt, u64* __restrict__ stats) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  u64 heads = 0, words = 0;
  for (int32_t q = 0; q < P; ++q) {
    const u64 a = scan[bnd_ptr[q]], b = scan[bnd_ptr[q + 1]];
    cnt[4 * q + 0] = a >> 40;
    cnt[4 * q + 1] = (b >> 40) - (a >> 40);
    cnt[4 * q + 2] = a & LOW40;
    cnt[4 * q + 3] = (b & LOW40) - (a & LOW40);
    if (q != self) {
      heads += cnt[4 * q + 1];
      words += cnt[4 * q + 3];
    }
  }
  stats[S_XROWS] = heads;
  stats[S_XBYTES] = 8 * (heads + words);
}

int pack_boundary(Ctx* c) {
  hipStream_t s = c->stream;
  const int nx = c->cur ^ 1;
  const int64_t NK = c->n_bvx, NB = c->n_bnd;
  if (NK > 0)
    hipLaunchKernelGGL(k_bnd_mark, dim3((unsigned)((NK + PWAVES - 1) / PWAVES)), dim3(PBLOCK), 0, s, c->d_bvx_v, NK,
                       c->d_fpop[nx], c->d_state, c->d_frx[nx], c->words, c->d_bvx_info, c->d_bvx_flag);
  hipLaunchKernelGGL(k_bnd_size, dim3((unsigned)((NB + 1 + PBLOCK - 1) / PBLOCK)), dim3(PBLOCK), 0, s, c->d_bnd_k,
                     NB, c->d_bvx_info, c->d_bvx_flag, c->d_xsize);
  GP_HIP(hipGetLastError());
  GP_TRY(scan_u64(c, c->d_xsize, c->d_bnd_scan, (size_t)NB + 1));
  if (NK > 0)
    hipLaunchKernelGGL(k_bnd_pack, dim3((unsigned)((NK + PWAVES - 1) / PWAVES)), dim3(PBLOCK), 0, s, c->d_bvx_v,
                       c->d_bvx_ptr, c->d_bvx_t, NK, c->d_bvx_info, c->d_bvx_flag, c->d_frx[nx], c->words,
                       c->d_bnd_e, c->d_bnd_scan, c->d_sbuf_h, c->d_sbuf_w);
  hipLaunchKernelGGL(k_bnd_counts, dim3(1), dim3(64), 0, s, c->d_bnd_scan, c->d_bnd_ptr, c->nranks, c->rank,
                     c->d_cnt, c->d_stats);
  GP_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// unpack
struct PeerTable {
  int32_t rk[MAX_PARTS + 1];   // received heads of sender q: [rk[q], rk[q + 1])
  int32_t gh[MAX_PARTS + 1];   // ghost index offsets per owner
};

__global__ __launch_bounds__(PBLOCK) void k_rx_size(const u64* __restrict__ rh, int64_t nh, u64* __restrict__ out) {
  const int64_t h = (int64_t)blockIdx.x * PBLOCK + threadIdx.x;
  if (h > nh) return;
  out[h] = h < nh ? 1ull + (rh[h] >> 40) : 0ull;
}

// Received entries are checked against the exchange plan before anything is
// written (a transfer that does not match it must fail loudly on every rank,
// not write out of bounds): the entry's ghost index lies within the ghosts of
// its sender, its flags are a new row and / or a removal, its word count is
// the popcount of its mask (which names only the row's W words), and the
// heads' word counts add up to the words the plan received.  Each bad entry
// adds 1 to stats[S_XERR], which the counters' all-reduce carries to every
// rank (round_collect turns it into GP_ERCCL).
__global__ __launch_bounds__(PBLOCK) void k_rx_unpack(const u64* __restrict__ rh, const u64* __restrict__ rw,
                                                      const u64* __restrict__ rscan, int64_t nh, PeerTable pt,
                                                      int32_t P, int64_t nloc, int32_t W, int32_t nx,
                                                      u64* __restrict__ slot, uint32_t* __restrict__ fpop_next,
                                                      uint8_t* __restrict__ sp, uint8_t* __restrict__ ws,
                                                      uint8_t* __restrict__ state, int32_t* __restrict__ deg_live,
                                                      const int64_t* __restrict__ row_ptr,
                                                      const int32_t* __restrict__ col, u64 words_expected,
                                                      u64* __restrict__ xerr) {
  const int lane = threadIdx.x & 63;
  const int64_t h = (int64_t)blockIdx.x * PWAVES + (threadIdx.x >> 6);
  if (h == 0 && lane == 0 && rscan[nh] != words_expected) atomicAdd(xerr, 1ull);
  if (h >= nh) return;
  const u64 head = rh[h];
  int q = 0;
  while (q + 1 < P && (int64_t)pt.rk[q + 1] <= h) ++q;
  const uint32_t idx = (uint32_t)head;
  const uint32_t f = (uint32_t)(head >> 32) & 0xFFu;
  const u64 woff = rscan[h];
  const u64 nwords = head >> 40;
  bool ok = idx < (uint32_t)(pt.gh[q + 1] - pt.gh[q]) && f >= 1u && f <= 3u && (u64)W <= 64 &&
            woff + 1 + nwords <= words_expected;
  const u64 mask = ok ? rw[woff] : 0ull;
  ok = ok && (u64)__popcll(mask) == nwords && (W == 64 || (mask >> W) == 0ull);
  if (!ok) {
    if (lane == 0) atomicAdd(xerr, 1ull);
    return;
  }
  const int64_t g = nloc + pt.gh[q] + (int64_t)idx;
  if (f & 1u) {
    u64 x = 0;
    if (lane < W && ((mask >> lane) & 1ull)) x = rw[woff + 1 + (u64)__popcll(mask & ((1ull << lane) - 1ull))];
    if (lane < W) slot[(size_t)g * W + lane] = x;
    uint32_t pc = (uint32_t)__popcll(x);
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) pc += (uint32_t)__shfl_xor((int)pc, s);
    if (lane == 0) {
      fpop_next[g] = pc;
      sp[g] = (uint8_t)nx;
      ws[g] |= (uint8_t)(1u << nx);
    }
  }
  if (f & 2u) {   // removed by its owner: its owned neighbours here lose a live link
    int first = 0;
    if (lane == 0) {
      first = !(state[g] & ST_REMOVED);
      if (first) state[g] |= ST_REMOVED;
    }
    first = __shfl(first, 0);
    if (first)
      for (int64_t j = row_ptr[g] + lane; j < row_ptr[g + 1]; j += 64) atomicSub(&deg_live[col[j]], 1);
  }
}

__global__ void k_or_alive(const u64* __restrict__ all, int32_t P, int32_t W, u64* __restrict__ alive) {
  const int w = threadIdx.x;
  if (w >= W) return;
  u64 x = 0;
  for (int q = 0; q < P; ++q) x |= all[(size_t)q * W + w];
  alive[w] = x;
}

// received heads / words are in place (by sender rank); rk = head prefix per sender
static int unpack_received(Ctx* c, const std::vector<int64_t>& rk, int64_t rw) {
  hipStream_t s = c->stream;
  const int nx = c->cur ^ 1;
  const int64_t nl = c->nloc(), P = c->nranks;
  // ghosts and extras receive nothing unless an entry says so
  if (c->n_alloc > nl)
    GP_HIP(hipMemsetAsync(c->d_fpop[nx] + nl, 0, (size_t)(c->n_alloc - nl) * 4, s));
  const int64_t nh = rk[(size_t)P];
  if (nh == 0) return 0;
  hipLaunchKernelGGL(k_rx_size, dim3((unsigned)((nh + 1 + PBLOCK - 1) / PBLOCK)), dim3(PBLOCK), 0, s, c->d_rbuf_h, nh,
                     c->d_xsize);
  GP_TRY(scan_u64(c, c->d_xsize, c->d_rscan, (size_t)nh + 1));
  PeerTable pt{};   // (P <= MAX_PARTS: checked by localize)
  for (int64_t q = 0; q <= P; ++q) {
    pt.rk[q] = (int32_t)rk[(size_t)q];
    pt.gh[q] = (int32_t)c->h_gh_ptr[(size_t)q];
  }
  hipLaunchKernelGGL(k_rx_unpack, dim3((unsigned)((nh + PWAVES - 1) / PWAVES)), dim3(PBLOCK), 0, s, c->d_rbuf_h,
                     c->d_rbuf_w, c->d_rscan, nh, pt, (int32_t)P, nl, c->words, nx, c->d_slot[nx], c->d_fpop[nx],
                     c->d_sp, c->d_ws, c->d_state, c->d_deg_live, c->d_row_ptr, c->d_col, (u64)rw,
                     c->d_stats + S_XERR);
  GP_HIP(hipGetLastError());
  return 0;
}

static bool alive_reduce_on(const Ctx* c) { return c->d_alive != nullptr && c->liveness_active; }

// this rank's send-list lengths |B_pq| and ghost counts per owner q
static void list_lengths(const Ctx* c, int64_t* bnd, int64_t* gh) {
  for (int64_t q = 0; q < c->nranks; ++q) {
    bnd[q] = q == c->rank ? 0 : c->h_bnd_ptr[(size_t)q + 1] - c->h_bnd_ptr[(size_t)q];
    gh[q] = q == c->rank ? 0 : c->h_gh_ptr[(size_t)q + 1] - c->h_gh_ptr[(size_t)q];
  }
}

// once per partition, on every rank: all-gather (|B_pq|, ghosts of q) and
// compare them pairwise (xplan_check_lists); every rank gets the same answer
static int check_lists_rccl(Ctx* c) {
  if (!c->h_ghosts_all.empty()) return 0;
  hipStream_t s = c->stream;
  const int64_t P = c->nranks;
  std::vector<u64> mine(2 * (size_t)P), all(2 * (size_t)(P * P));
  std::vector<int64_t> bnd((size_t)P), gh((size_t)P);
  list_lengths(c, bnd.data(), gh.data());
  for (int64_t q = 0; q < P; ++q) {
    mine[(size_t)q] = (u64)bnd[(size_t)q];
    mine[(size_t)(P + q)] = (u64)gh[(size_t)q];
  }
  GP_HIP(hipMemcpyAsync(c->d_cnt, mine.data(), mine.size() * 8, hipMemcpyHostToDevice, s));
  GP_RCCL(ncclAllGather(c->d_cnt, c->d_cnt_all, 2 * (size_t)P, ncclUint64, c->comm, s));
  GP_HIP(hipMemcpyAsync(all.data(), c->d_cnt_all, all.size() * 8, hipMemcpyDeviceToHost, s));
  GP_HIP(hipStreamSynchronize(s));
  std::vector<int64_t> bnd_all((size_t)(P * P)), gh_all((size_t)(P * P));
  for (int64_t r = 0; r < P; ++r)
    for (int64_t q = 0; q < P; ++q) {
      bnd_all[(size_t)(r * P + q)] = (int64_t)all[(size_t)(r * 2 * P + q)];
      gh_all[(size_t)(r * P + q)] = (int64_t)all[(size_t)(r * 2 * P + P + q)];
    }
  std::string err;
  if (!xplan_check_lists(bnd_all.data(), gh_all.data(), (int)P, &err)) return set_error(GP_EINVAL, err);
  c->h_ghosts_all = std::move(gh_all);
  return 0;
}

static int check_lists_group(Ctx** ctxs, int32_t P) {
  if (!ctxs[0]->h_ghosts_all.empty()) return 0;
  std::vector<int64_t> bnd_all((size_t)P * P), gh_all((size_t)P * P);
  for (int32_t k = 0; k < P; ++k) list_lengths(ctxs[k], &bnd_all[(size_t)k * P], &gh_all[(size_t)k * P]);
  std::string err;
  if (!xplan_check_lists(bnd_all.data(), gh_all.data(), P, &err)) return set_error(GP_EINVAL, err);
  for (int32_t k = 0; k < P; ++k) ctxs[k]->h_ghosts_all = gh_all;
  return 0;
}

int exchange_rccl(Ctx* c) {
  hipStream_t s = c->stream;
  const int64_t P = c->nranks, p = c->rank;
  const size_t W = (size_t)c->words;
  GP_TRY(check_lists_rccl(c));
  GP_TRY(pack_boundary(c));
  u64* alive_next = c->d_alive + (size_t)(c->cur ^ 1) * W;
  GP_RCCL(ncclGroupStart());
  GP_RCCL(ncclAllGather(c->d_cnt, c->d_cnt_all, 4 * (size_t)P, ncclUint64, c->comm, s));
  if (alive_reduce_on(c)) GP_RCCL(ncclAllGather(alive_next, c->d_alive_all, W, ncclUint64, c->comm, s));
  GP_RCCL(ncclGroupEnd());
  if (alive_reduce_on(c)) hipLaunchKernelGGL(k_or_alive, dim3(1), dim3(64), 0, s, c->d_alive_all, (int32_t)P,
                                             (int32_t)W, alive_next);
  GP_HIP(hipMemcpyAsync(c->h_cnt_all, c->d_cnt_all, 4 * (size_t)(P * P) * sizeof(u64), hipMemcpyDeviceToHost, s));
  GP_HIP(hipStreamSynchronize(s));
  // every rank checks every receiver's counts: all return, or none does
  std::string err;
  if (!xplan_check_all(c->h_cnt_all, (int)P, c->h_ghosts_all.data(), (int)W, &err))
    return set_error(GP_EINVAL, err);
  XPlan plan;
  (void)xplan_build(c->h_cnt_all, (int)P, (int)p, &c->h_ghosts_all[(size_t)(p * P)], (int)W, &plan, &err);
  GP_RCCL(ncclGroupStart());
  for (int64_t q = 0; q < P; ++q) {
    if (q == p) continue;
    const XSlice& out = plan.send[(size_t)q];
    if (out.nh) {
      GP_RCCL(ncclSend(c->d_sbuf_h + out.h0, (size_t)out.nh, ncclUint64, (int)q, c->comm, s));
      GP_RCCL(ncclSend(c->d_sbuf_w + out.w0, (size_t)out.nw, ncclUint64, (int)q, c->comm, s));
    }
    const XSlice& in = plan.recv[(size_t)q];
    if (in.nh) {
      GP_RCCL(ncclRecv(c->d_rbuf_h + in.h0, (size_t)in.nh, ncclUint64, (int)q, c->comm, s));
      GP_RCCL(ncclRecv(c->d_rbuf_w + in.w0, (size_t)in.nw, ncclUint64, (int)q, c->comm, s));
    }
  }
  GP_RCCL(ncclGroupEnd());
  GP_TRY(unpack_received(c, plan.rk, plan.rw.back()));
  // the counters' all-reduce after the unpack: it carries the unpack's entry
  // check (S_XERR) to every rank, so all ranks fail the round together
  GP_RCCL(ncclAllReduce(c->d_stats, c->d_stats, S_REPORT_CURSOR, ncclUint64, ncclSum, c->comm, s));
  return 0;
}

int exchange_group(Ctx** ctxs, int32_t P) {
  GP_TRY(check_lists_group(ctxs, P));
  for (int32_t k = 0; k < P; ++k) {
    GP_HIP(hipSetDevice(ctxs[k]->device));
    GP_TRY(pack_boundary(ctxs[k]));
  }
  // the count matrix as the RCCL path all-gathers it: [sender][4 * receiver]
  std::vector<u64> all(4 * (size_t)P * P);
  for (int32_t k = 0; k < P; ++k) {
    Ctx* c = ctxs[k];
    GP_HIP(hipSetDevice(c->device));
    GP_HIP(hipStreamSynchronize(c->stream));
    GP_TRY(copy_sync(c, all.data() + 4 * (size_t)P * k, c->d_cnt, 4 * (size_t)P * sizeof(u64),
                     hipMemcpyDeviceToHost));
  }
  // alive sets: OR of every context's partial set
  if (alive_reduce_on(ctxs[0])) {
    const size_t W = (size_t)ctxs[0]->words;
    std::vector<u64> acc(W, 0), part(W);
    for (int32_t k = 0; k < P; ++k) {
      Ctx* c = ctxs[k];
      GP_TRY(copy_sync(c, part.data(), c->d_alive + (size_t)(c->cur ^ 1) * W, W * 8, hipMemcpyDeviceToHost));
      for (size_t w = 0; w < W; ++w) acc[w] |= part[w];
    }
    for (int32_t k = 0; k < P; ++k) {
      Ctx* c = ctxs[k];
      GP_TRY(copy_sync(c, c->d_alive + (size_t)(c->cur ^ 1) * W, acc.data(), W * 8, hipMemcpyHostToDevice));
    }
  }
  std::string err;
  const int W = ctxs[0]->words;
  if (!xplan_check_all(all.data(), P, ctxs[0]->h_ghosts_all.data(), W, &err)) return set_error(GP_EINVAL, err);
  for (int32_t d = 0; d < P; ++d) {
    Ctx* dst = ctxs[d];
    GP_HIP(hipSetDevice(dst->device));
    XPlan plan;
    (void)xplan_build(all.data(), P, d, &dst->h_ghosts_all[(size_t)d * P], W, &plan, &err);
    for (int32_t q = 0; q < P; ++q) {
      if (q == d) continue;
      const XSlice& in = plan.recv[(size_t)q];
      if (!in.nh) continue;
      const XSlice& out = xplan_send_of(all.data(), P, q, d);
      GP_HIP(hipMemcpyAsync(dst->d_rbuf_h + in.h0, ctxs[q]->d_sbuf_h + out.h0, (size_t)in.nh * 8, hipMemcpyDefault,
                            dst->stream));
      GP_HIP(hipMemcpyAsync(dst->d_rbuf_w + in.w0, ctxs[q]->d_sbuf_w + out.w0, (size_t)in.nw * 8, hipMemcpyDefault,
                            dst->stream));
    }
    GP_TRY(unpack_received(dst, plan.rk, plan.rw.back()));
  }
  return 0;
}

}  // namespace gp
