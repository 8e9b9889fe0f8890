// push.hip -- the push direction of sparse rounds (DESIGN.md §3.3,
// direction-optimising BFS after Beamer et al. SC'12): senders OR their rows
// into their receivers' accumulator rows, then the same receiver side as the
// pull.  Also the push half of degree-split rounds (§3.2).
#include "gp_device.h"

namespace gp {

// ---------------------------------------------------------------------------
// push mode for sparse rounds (direction-optimising, Beamer et al. SC'12):
// every active sender ORs the NON-ZERO words of its row into the accumulator
// rows of its live out-neighbours (64-bit atomicOr, order-free so bit-exact)
// and sets the receiver's bit in `tbits` (fire-and-forget atomicOr on a 2 MB
// bitmap); k_touch_list compacts the bitmap and k_apply runs the same receiver
// side as the pull (finish_row) and re-zeroes acc.  The sender row is its
// whole Message-List S[r & 1][u] (a superset of its frontier whose extra bits
// every live out-neighbour already holds, see ExpandArgs), or the exact
// frontier row when track_msg_forwards keeps those.

// active senders from the bitmap: one thread per 64-vertex word, block-level
// compaction, one cursor add per block; big senders go to their own list
// (split_deg > 0: the push half of a degree-split round lists only senders of
// in-degree < split_deg; the others are pulled by the receivers' prefix probes)
__global__ __launch_bounds__(BLOCK) void k_active_list(const u64* __restrict__ abits, int64_t nwords,
                                                       const int64_t* __restrict__ orp, int32_t big_thr,
                                                       int32_t* __restrict__ active, int32_t* __restrict__ big,
                                                       u64* __restrict__ stats, const int64_t* __restrict__ rp_in,
                                                       int32_t split_deg) {
  __shared__ uint32_t s_cnt[BLOCK];
  __shared__ u64 s_base;
  const int64_t w = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const u64 bits = w < nwords ? abits[w] : 0ull;
  s_cnt[threadIdx.x] = (uint32_t)__popcll(bits);
  __syncthreads();
  for (int o = 1; o < BLOCK; o <<= 1) {   // inclusive scan
    const uint32_t x = threadIdx.x >= o ? s_cnt[threadIdx.x - o] : 0u;
    __syncthreads();
    s_cnt[threadIdx.x] += x;
    __syncthreads();
  }
  if (threadIdx.x == BLOCK - 1) s_base = atomicAdd(&stats[S_ACTIVE_CURSOR], (u64)s_cnt[BLOCK - 1]);
  __syncthreads();
  u64 pos = s_base + s_cnt[threadIdx.x] - (uint32_t)__popcll(bits);
  u64 m = bits;
  while (m) {
    const int b = __ffsll((long long)m) - 1;
    m &= m - 1;
    const int32_t u = (int32_t)(w * 64 + b);
    if (split_deg > 0 && rp_in[u + 1] - rp_in[u] >= split_deg) {
      active[pos++] = -1;   // pulled (placeholder: the block's slots stay dense)
    } else if (orp[u + 1] - orp[u] > big_thr) {
      const u64 k = atomicAdd(&stats[S_BIG_CURSOR], 1ull);
      big[k] = u;
      active[pos++] = -1;   // placeholder keeps the block's slots dense
    } else {
      active[pos++] = u;
    }
  }
}

// push arcs [jb, je) of sender u; the wave holds u's row and its non-zero
// word indices in LDS
template <int W>
__device__ __forceinline__ void push_arcs(const ExpandArgs& a, int64_t jb, int64_t je,
                                          const u64* __restrict__ srow, const int8_t* __restrict__ swords,
                                          int nnz, int lane) {
  const int64_t T = (je - jb) * nnz;
  for (int64_t t0 = 0; t0 < T; t0 += 64) {
    const int64_t t = t0 + lane;
    int32_t v = -1;
    if (t < T) {
      const int64_t j = t / nnz;
      const int q = (int)(t - j * nnz);
      v = a.ocol[jb + j];
      const bool recv = a.nbits ? ((a.nbits[v >> 6] >> (v & 63)) & 1ull) != 0ull
                                : (v >= a.vbegin && v < a.vbegin + a.nloc && !(a.state[v] & (ST_DOWN | ST_SATED)) &&
                                   a.seenpop[v - a.vbegin] < a.done_at[v]);
      if (recv) {
        const int w = swords[q];
        atomicOr(&a.acc[(size_t)v * W + w], srow[w]);
        if (q == 0) atomicOr(&a.tbits[v >> 6], 1ull << (v & 63));
      }
    }
  }
}

// touched receivers: compact the bitmap (one thread per word) and clear it
__global__ __launch_bounds__(BLOCK) void k_touch_list(u64* __restrict__ tbits, int64_t nwords,
                                                      int32_t* __restrict__ touched, u64* __restrict__ stats) {
  __shared__ uint32_t s_cnt[BLOCK];
  __shared__ u64 s_base;
  const int64_t w = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  u64 bits = 0;
  if (w < nwords) {
    bits = tbits[w];
    if (bits) tbits[w] = 0ull;
  }
  s_cnt[threadIdx.x] = (uint32_t)__popcll(bits);
  __syncthreads();
  for (int o = 1; o < BLOCK; o <<= 1) {   // inclusive scan
    const uint32_t x = threadIdx.x >= o ? s_cnt[threadIdx.x - o] : 0u;
    __syncthreads();
    s_cnt[threadIdx.x] += x;
    __syncthreads();
  }
  if (threadIdx.x == BLOCK - 1) s_base = atomicAdd(&stats[S_TOUCH_CURSOR], (u64)s_cnt[BLOCK - 1]);
  __syncthreads();
  u64 pos = s_base + s_cnt[threadIdx.x] - (uint32_t)__popcll(bits);
  while (bits) {
    const int b = __ffsll((long long)bits) - 1;
    bits &= bits - 1;
    touched[pos++] = (int32_t)(w * 64 + b);
  }
}

template <int W>
__device__ __forceinline__ int stage_row(const ExpandArgs& a, int32_t u, u64* __restrict__ srow,
                                         int8_t* __restrict__ swords, int lane) {
  u64 x = 0;
  if (lane < W) x = (a.frx && u < a.frx_rows) ? a.frx[(size_t)u * W + lane] : a.rows[(size_t)u * W + lane];
  const u64 nzm = __ballot(x != 0ull);
  if (lane < W) srow[lane] = x;
  if (x) swords[lane_rank(nzm)] = (int8_t)lane;
  wave_sync_lds();
  return __popcll(nzm);
}

__device__ __forceinline__ void push_sender_stats(const ExpandArgs& a, int32_t u, WaveStats& st) {
  if (a.split_push) return;   // (the pull half of a degree-split round counts every sender)
  if (u >= a.vbegin && u < a.vbegin + a.nloc) {
    st.add(S_SENDS, (u64)a.fpop[u] * (u64)(uint32_t)max(a.deg_live[u], 0));
    st.add(S_ACTIVE, 1);
  }
}

template <int W>
__global__ __launch_bounds__(BLOCK) void k_push(ExpandArgs a) {
  __shared__ u64 s_row[WAVES][64];
  __shared__ int8_t s_words[WAVES][64];
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  WaveStats st;
  ws_zero(st);
  const int64_t nact = (int64_t)a.stats[S_ACTIVE_CURSOR];
  const int64_t stride = (int64_t)gridDim.x * WAVES;
  for (int64_t k = (int64_t)blockIdx.x * WAVES + wib; k < nact; k += stride) {
    const int32_t u = a.active[k];
    if (u < 0) continue;   // big sender, pushed by k_push_big
    push_sender_stats(a, u, st);
    const int nnz = stage_row<W>(a, u, s_row[wib], s_words[wib], lane);
    const int64_t jb = a.orp[u], je = a.orp[u + 1];
    if (!a.split_push) {
      st.add(S_GATHERED, 1);
      st.add(S_ROW_BYTES, (u64)(8 * W));
      st.add(S_ARCS, (u64)(je - jb));
    }
    st.add(S_ATOMICS, (u64)(je - jb) * (u64)nnz);
    push_arcs<W>(a, jb, je, s_row[wib], s_words[wib], nnz, lane);
    __builtin_amdgcn_wave_barrier();
  }
  flush_stats(st, a.partial);
}

// big senders (out-degree > PUSH_CHUNK): chunk c of big sender k goes to wave
// (k * 7919 + c) mod #waves, which spreads every sender's chunks (and the
// senders) evenly over the grid without a prefix sum
constexpr int PUSH_CHUNK = 512;
template <int W>
__global__ __launch_bounds__(BLOCK) void k_push_big(ExpandArgs a) {
  __shared__ u64 s_row[WAVES][64];
  __shared__ int8_t s_words[WAVES][64];
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  WaveStats st;
  ws_zero(st);
  const int64_t nbig = (int64_t)a.stats[S_BIG_CURSOR];
  const int64_t gw = (int64_t)blockIdx.x * WAVES + wib, nw = (int64_t)gridDim.x * WAVES;
  for (int64_t k = 0; k < nbig; ++k) {
    const int32_t u = a.big[k];
    const int64_t jb = a.orp[u], je = a.orp[u + 1];
    const int64_t nch = (je - jb + PUSH_CHUNK - 1) / PUSH_CHUNK;
    const int64_t c0 = ((gw - (k * 7919) % nw) % nw + nw) % nw;   // first chunk of this wave
    if (c0 == 0 && gw == (k * 7919) % nw && !a.split_push) {
      push_sender_stats(a, u, st);
      st.add(S_GATHERED, 1);
      st.add(S_ROW_BYTES, (u64)(8 * W));
    }
    if (c0 >= nch) continue;
    const int nnz = stage_row<W>(a, u, s_row[wib], s_words[wib], lane);
    for (int64_t c = c0; c < nch; c += nw) {
      const int64_t cb = jb + c * PUSH_CHUNK, ce = min(je, cb + PUSH_CHUNK);
      if (!a.split_push) st.add(S_ARCS, (u64)(ce - cb));
      st.add(S_ATOMICS, (u64)(ce - cb) * (u64)nnz);
      push_arcs<W>(a, cb, ce, s_row[wib], s_words[wib], nnz, lane);
    }
    __builtin_amdgcn_wave_barrier();
  }
  flush_stats(st, a.partial);
}

// degree-split rounds, after the pull: zero the accumulator rows the push half
// wrote (every touched receiver's; the pull only read them) and the bitmap
template <int W>
__global__ __launch_bounds__(BLOCK) void k_acc_clear(u64* __restrict__ tbits, u64* __restrict__ acc, int64_t nwords) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * WAVES;
  for (int64_t w = (int64_t)blockIdx.x * WAVES + uniform(threadIdx.x >> 6); w < nwords; w += nw) {
    u64 bits = tbits[w];
    if (!bits) continue;
    while (bits) {
      const int b = __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      if (lane < W) acc[(size_t)(w * 64 + b) * W + lane] = 0ull;
    }
    if (lane == 0) tbits[w] = 0ull;
  }
}

// receiver side of the push: one wave per touched vertex
template <int W>
__global__ __launch_bounds__(BLOCK) void k_apply(ExpandArgs a) {
  constexpr int LPR = Geo<W>::LPR;
  __shared__ WaveLds s_w[WAVES];
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  const int g = lane / LPR, lw = lane % LPR;
  WaveStats st;
  ws_zero(st);
  const int64_t nt = (int64_t)a.stats[S_TOUCH_CURSOR];
  const int64_t stride = (int64_t)gridDim.x * WAVES;
  alive_zero<W>(a, s_w[wib].alive, lane);
  wave_sync_lds();
  for (int64_t k = (int64_t)blockIdx.x * WAVES + wib; k < nt; k += stride) {
    const int32_t v = a.touched[k];
    const int64_t i = v - a.vbegin;
    u64x2 acc = {0, 0};
    if (g == 0) {
      acc = load_piece<W>(a.acc, v, lw);
      store_piece<W>(a.acc, v, lw, u64x2{0, 0});
    }
    st.add(S_VISITED, 1);
    finish_row<W, false, false>(a, v, i, acc, lane, g, lw, st, s_w[wib], false, a.sp[v]);
  }
  alive_flush<W>(a, s_w[wib].alive, lane);
  flush_stats(st, a.partial);
}

// receivable bitmap of a narrow push round: bit v = v is owned, up and not
// done, i.e. the per-arc test of push_arcs done once per vertex (2 MB at 2^24,
// L2-resident, instead of three scattered loads per arc)
__global__ __launch_bounds__(BLOCK) void k_mkneed(const uint8_t* __restrict__ state,
                                                  const uint32_t* __restrict__ seenpop,
                                                  const uint32_t* __restrict__ done_at, int64_t vbegin,
                                                  int64_t nloc, int64_t n, u64* __restrict__ nbits) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t v0 = (int64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63); v0 < n; v0 += stride) {
    const int64_t v = v0 + lane;
    bool ok = false;
    if (v >= vbegin && v < vbegin + nloc)
      ok = !(state[v] & (ST_DOWN | ST_SATED)) && seenpop[v - vbegin] < done_at[v];
    const u64 m = __ballot(ok);
    if (lane == 0) nbits[v0 >> 6] = m;
  }
}

// receiver side of a narrow push round, lane-parallel: a wave takes 64
// touched receivers (the touched list is in vertex order within a block) and
// runs them RPI per wave-instruction with LPR lanes x 16 B per row, like the
// flat pull's receiver side; per-receiver words are committed one receiver
// per lane.  Same results as k_apply (finish_row), which spends a whole wave
// on each receiver: at W <= 32 most of its lanes idle.
template <int W>
__global__ __launch_bounds__(BLOCK) void k_apply_lanes(ExpandArgs a) {
  constexpr int LPR = Geo<W>::LPR;
  constexpr int RPI = Geo<W>::RPI;
  constexpr int WPL = Geo<W>::WPL;
  struct ApplyLds {
    uint32_t tot[64];
    u64 dig[64];
    int8_t rd[64];
    u64 alive[W];
  };
  __shared__ ApplyLds s_a[WAVES];
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  const int g = lane / LPR, lw = lane % LPR;
  ApplyLds& L = s_a[wib];
  WaveStats st;
  ws_zero(st);
  const int64_t nt = (int64_t)a.stats[S_TOUCH_CURSOR];
  alive_zero<W>(a, L.alive, lane);
  const int64_t stride = (int64_t)gridDim.x * WAVES * 64;
  for (int64_t base = ((int64_t)blockIdx.x * WAVES + wib) * 64; base < nt; base += stride) {
    const bool mine = base + lane < nt;
    const int v = mine ? a.touched[base + lane] : 0;
    const uint32_t slot_of = mine ? (uint32_t)a.sp[v] : SLOT_NONE;
    st.add(S_VISITED, (u64)__popcll(__ballot(mine)));
    wave_sync_lds();
    for (int r0 = 0; r0 < 64; r0 += RPI) {
      const int r = r0 + g;
      const int rv = __shfl(v, r);
      const uint32_t rslot = (uint32_t)__shfl((int)slot_of, r);
      const bool rn = base + r < nt;
      u64x2 acc = {0, 0};
      if (rn) {
        acc = load_piece<W>(a.acc, rv, lw);   // (indexed by v, as push_arcs and k_apply do)
        store_piece<W>(a.acc, rv, lw, u64x2{0, 0});   // the accumulator stays all-zero
      }
      const bool any = group_or<LPR>((acc.x | acc.y) != 0ull);
      u64x2 sv = {0, 0};
      if (any && rslot != SLOT_NONE) sv = load_piece<W>(a.slot[rslot], rv, lw);
      const u64x2 nw = acc & ~sv;
      const uint32_t tot = group_sum<LPR>((uint32_t)(__popcll(nw.x) + __popcll(nw.y)));
      u64 t = 0;
      if (tot) {
        alive_add<W>(a, L, lw, nw);
        store_piece<W>(a.slot[a.wslot], rv, lw, sv | nw);
        if (a.frx_next) store_piece<W>(a.frx_next, rv, lw, nw);
        if (a.first) {
          uint8_t* row = a.first + (size_t)(rv - a.vbegin) * (W * 64);
          if (nw.x) set_first_bytes(row, lw * WPL, nw.x, (uint32_t)a.rr);
          if (WPL == 2 && nw.y) set_first_bytes(row, lw * WPL + 1, nw.y, (uint32_t)a.rr);
        }
        if (a.digest) {
          if (nw.x) t ^= digest_term((uint32_t)a.rr, (uint32_t)(a.wbase + lw * WPL), nw.x);
          if (WPL == 2 && nw.y) t ^= digest_term((uint32_t)a.rr, (uint32_t)(a.wbase + lw * WPL + 1), nw.y);
        }
      }
      t = group_xor<LPR>(t);
      if (lw == 0) {
        L.tot[r] = tot;
        L.dig[r] = t;
        L.rd[r] = (int8_t)(any && rslot != SLOT_NONE);
      }
    }
    wave_sync_lds();
    u64 nbits = 0, nrecv = 0, narcs = 0, nseen = 0;
    if (mine) {
      const uint32_t tot = L.tot[lane];
      nseen = (u64)L.rd[lane];
      if (tot) {   // (fpop_next of the owned vertices was zeroed before the push)
        const int64_t i = v - a.vbegin;
        a.fpop_next[v] = tot;
        a.seenpop[i] += tot;
        a.sp[v] = (uint8_t)a.wslot;
        a.ws[v] |= (uint8_t)(1u << a.wslot);
        if (a.digest) a.digest[i] ^= L.dig[lane];
        nbits = tot;
        nrecv = 1;
        narcs = (u64)(uint32_t)max(a.deg_live[v], 0);
      }
    }
    st.add(S_NEW_BITS, wave_sum_u64(nbits));
    st.add(S_RECEIVERS, wave_sum_u64(nrecv));
    st.add(S_WRITTEN, wave_sum_u64(nrecv));
    st.add(S_NEXT_ARCS, wave_sum_u64(narcs));
    st.add(S_SEEN_READ, wave_sum_u64(nseen));
    wave_sync_lds();   // L.tot / L.dig are restaged by the next group
  }
  alive_flush<W>(a, L.alive, lane);
  flush_stats(st, a.partial);
}

// narrow rows (W <= GP_PUSH_LANES_MAXW): the receivable bitmap and the
// lane-parallel receiver side (k_mkneed, k_apply_lanes)
#ifndef GP_PUSH_LANES_MAXW
#define GP_PUSH_LANES_MAXW 32
#endif
template <int W>
void launch_push_w(Ctx* c, ExpandArgs a) {
  hipStream_t s = c->stream;
  const int64_t nwords = (c->n_alloc + 63) / 64;
  constexpr bool lanes = W <= GP_PUSH_LANES_MAXW;
  // the bitmap pays once the push has many arcs (a pass over n vertices
  // against three scattered loads per arc)
  if (lanes && c->push_est * 16.0 >= (double)c->n_alloc) {
    hipLaunchKernelGGL(k_mkneed, dim3(std::max(1, std::min(grid_for(c->n_alloc, BLOCK), c->cu_count * 8 * GS))),
                       dim3(BLOCK), 0, s, c->d_state, c->d_seenpop, c->d_done_at, a.vbegin, a.nloc, c->n_alloc,
                       c->d_nbits);
    a.nbits = c->d_nbits;
  }
  hipLaunchKernelGGL(k_active_list, dim3(grid_for(nwords, BLOCK)), dim3(BLOCK), 0, s, c->d_abits, nwords,
                     a.orp, PUSH_CHUNK, c->d_active, c->d_big, c->d_stats, (const int64_t*)nullptr, 0);
  hipLaunchKernelGGL(k_push<W>, dim3(c->cu_count * 8 * GS), dim3(BLOCK), 0, s, a);
  hipLaunchKernelGGL(k_push_big<W>, dim3(c->cu_count * 4 * GS), dim3(BLOCK), 0, s, a);
  hipLaunchKernelGGL(k_touch_list, dim3(grid_for(nwords, BLOCK)), dim3(BLOCK), 0, s, c->d_tbits, nwords,
                     c->d_touched, c->d_stats);
  if (lanes)   // a wave per 64 touched receivers at a time, grid-stride
    hipLaunchKernelGGL(k_apply_lanes<W>, dim3(std::max(1, std::min(grid_for(std::max<int64_t>(c->nloc(), 1),
                                                                             (int64_t)WAVES * 64),
                                                                    c->cu_count * 8 * GS))),
                       dim3(BLOCK), 0, s, a);
  else
    hipLaunchKernelGGL(k_apply<W>, dim3(c->cu_count * 8 * GS), dim3(BLOCK), 0, s, a);
}

template <int W>
void launch_split_push_w(Ctx* c, const ExpandArgs& a) {   // senders of in-degree < split_deg
  ExpandArgs p = a;
  p.split_push = 1;
  const int64_t nwords = (c->n_alloc + 63) / 64;
  hipLaunchKernelGGL(k_active_list, dim3(grid_for(nwords, BLOCK)), dim3(BLOCK), 0, c->stream, c->d_abits, nwords,
                     a.orp, PUSH_CHUNK, c->d_active, c->d_big, c->d_stats, (const int64_t*)c->d_row_ptr,
                     c->cfg.split_deg);
  hipLaunchKernelGGL(k_push<W>, dim3(c->cu_count * 8 * GS), dim3(BLOCK), 0, c->stream, p);
  hipLaunchKernelGGL(k_push_big<W>, dim3(c->cu_count * 4 * GS), dim3(BLOCK), 0, c->stream, p);
}

template <int W>
void launch_acc_clear_w(Ctx* c) {
  const int64_t nwords = (c->n_alloc + 63) / 64;
  hipLaunchKernelGGL(k_acc_clear<W>, dim3(std::max(1, std::min(grid_for(nwords, WAVES), c->cu_count * 8 * GS))),
                     dim3(BLOCK), 0, c->stream, c->d_tbits, c->d_acc, nwords);
}

template void launch_push_w<1>(Ctx*, ExpandArgs);
template void launch_push_w<2>(Ctx*, ExpandArgs);
template void launch_push_w<4>(Ctx*, ExpandArgs);
template void launch_push_w<8>(Ctx*, ExpandArgs);
template void launch_push_w<16>(Ctx*, ExpandArgs);
template void launch_push_w<32>(Ctx*, ExpandArgs);
template void launch_push_w<64>(Ctx*, ExpandArgs);
template void launch_split_push_w<1>(Ctx*, const ExpandArgs&);
template void launch_split_push_w<2>(Ctx*, const ExpandArgs&);
template void launch_split_push_w<4>(Ctx*, const ExpandArgs&);
template void launch_split_push_w<8>(Ctx*, const ExpandArgs&);
template void launch_split_push_w<16>(Ctx*, const ExpandArgs&);
template void launch_split_push_w<32>(Ctx*, const ExpandArgs&);
template void launch_split_push_w<64>(Ctx*, const ExpandArgs&);
template void launch_acc_clear_w<1>(Ctx*);
template void launch_acc_clear_w<2>(Ctx*);
template void launch_acc_clear_w<4>(Ctx*);
template void launch_acc_clear_w<8>(Ctx*);
template void launch_acc_clear_w<16>(Ctx*);
template void launch_acc_clear_w<32>(Ctx*);
template void launch_acc_clear_w<64>(Ctx*);

}  // namespace gp
