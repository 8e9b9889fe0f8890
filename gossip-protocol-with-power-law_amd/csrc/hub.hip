// hub.hip -- hub receivers of the pull (hub load balancing):
// vertices above hub_threshold in-arcs are split over waves, each wave ORs one
// chunk of the in-list into a partial row (k_hub_partial), k_hub_final combines
// a hub's partials and commits the row.  No atomics on rows, and the rows are
// deterministic: every chunk's OR is a subset of the hub's new bits, so the OR
// of the partials is exact whichever chunks stopped early.  The work counters
// are not: in early-exit rounds a chunk that covers the hub's target stamps
// hub_done and the hub's other chunks stop at their next 512 arcs, so
// arcs_scanned / rows_gathered / row_bytes of such rounds depend on wave
// timing ("Counters").
#include "gp_device.h"

namespace gp {

// hubs, pass 1: one wave per (hub, arc chunk) -> partial OR row
template <int W, int MODE>
__global__ __launch_bounds__(HBLOCK) void k_hub_partial(ExpandArgs a) {
  constexpr int LPR = Geo<W>::LPR;
  __shared__ WaveLds s_w[HWAVES];
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  const int g = lane / LPR, lw = lane % LPR;
  WaveStats st;
  ws_zero(st);
  const int64_t it = (int64_t)blockIdx.x * HWAVES + wib;
  if (it < a.n_items) {
    const HubItem h = a.hub_items[it];
    const int64_t i = h.v - a.vbegin;
    u64x2 acc = {0, 0};
    if (!(a.state[h.v] & (ST_DOWN | ST_SATED)) && a.seenpop[i] < a.done_at[h.v]) {
      const bool ee = a.early_exit != 0;
      u64x2 want = {0, 0};
      if (ee) want = early_exit_target<W>(a, h.v, s_w[wib], g, lw, a.sp[h.v], a.midx[h.v]);
      // degree-split rounds: the chunk's share of the gather-order prefix of
      // big senders (the push half ORed the others into the accumulator row)
      const int64_t hend = a.prehi ? min(h.end, a.row_ptr[h.v] + (int64_t)a.prehi[h.v]) : h.end;
      // early-exit rounds: a chunk that covers the hub's whole target says so
      // (hub_done = this launch's stamp), and the hub's other chunks stop at
      // their next 512 arcs -- the OR of all chunks is then exactly the target
      // whatever they gathered (every row is a subset of the component's
      // messages; under liveness nothing outside F_r is new, ExpandArgs)
      constexpr int64_t SUB = 512;
      for (int64_t s0 = h.beg; s0 < hend; s0 += SUB) {
        if (ee && a.hub_done) {
          uint32_t f = 0;
          if (lane == 0) f = __hip_atomic_load(a.hub_done + h.hub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((uint32_t)__builtin_amdgcn_readfirstlane((int)f) == a.hub_epoch) break;
        }
        gather_scan<W, MODE, W == 64 && (MODE == SCAN_FILTERED || MODE == SCAN_UNFILTERED)>(
            a, s0, min(hend, s0 + SUB), s_w[wib], lane, g, lw, acc, st, ee, want);
        if (ee) {
          u64x2 t = acc;
          reduce_slots<W>(t);
          const u64x2 miss = want & ~t;
          if (!__any((miss.x | miss.y) != 0ull)) {
            if (lane == 0 && a.hub_done)
              __hip_atomic_store(a.hub_done + h.hub, a.hub_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      reduce_slots<W>(acc);
    }
    const bool nz = __any((acc.x | acc.y) != 0);
    if (nz && g == 0) store_piece<W>(a.hub_partial, it, lw, acc);
    if (lane == 0) a.hub_pnz[it] = nz ? 1u : 0u;
  }
  flush_stats(st, a.partial);
}

// hubs, pass 2: one wave per hub -> OR the partials, then the receiver side
template <int W>
__global__ __launch_bounds__(HBLOCK) void k_hub_final(ExpandArgs a) {
  constexpr int LPR = Geo<W>::LPR;
  __shared__ WaveLds s_w[HWAVES];
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  const int g = lane / LPR, lw = lane % LPR;
  WaveStats st;
  ws_zero(st);
  const int64_t h = (int64_t)blockIdx.x * HWAVES + wib;
  alive_zero<W>(a, s_w[wib].alive, lane);
  wave_sync_lds();
  if (h < a.n_items) {
    const int v = a.hubs[h];
    const int64_t i = v - a.vbegin;
    if ((a.state[v] & (ST_DOWN | ST_SATED)) || a.seenpop[i] >= a.done_at[v]) {
      if (lane == 0) a.fpop_next[v] = 0;
    } else {
      st.add(S_VISITED, 1);
      u64x2 acc = {0, 0};
      const int p0 = a.hub_item_ptr[h], p1 = a.hub_item_ptr[h + 1];
      if (g == 0) {
        for (int p = p0; p < p1; ++p)
          if (a.hub_pnz[p]) acc |= load_piece<W>(a.hub_partial, p, lw);
        if (a.prehi) acc |= load_piece<W>(a.acc, v, lw);   // degree-split round: the push half's OR (k_acc_clear zeroes it)
      }
      // alive early-exit rounds with no injection left (liveness, DESIGN.md
      // §3.5): a hub whose chunks covered every alive message of its
      // component it lacked is sated, as k_expand marks its receivers.  Hubs
      // are the first in-neighbours of most gather orders, so their marks are
      // what the next round's done-neighbour probe finds
#ifndef GP_HUB_SATE
#define GP_HUB_SATE 1
#endif
      if (GP_HUB_SATE && a.sate && a.early_exit && a.alive) {
        u64x2 rem = {0, 0};
        if (g == 0) {
          const u64x2 sv = load_seen<W>(a, v, a.sp[v], lw);
          rem = load_piece<W>(a.cmask, a.midx[v], lw) & load_piece<W>(a.alive, 0, lw) & ~sv & ~acc;
        }
        if (!__any((rem.x | rem.y) != 0ull) && lane == 0) a.state[v] |= ST_SATED;
      }
      finish_row<W>(a, v, i, acc, lane, g, lw, st, s_w[wib], false, a.sp[v]);
    }
  }
  alive_flush<W>(a, s_w[wib].alive, lane);
  flush_stats(st, a.partial);
}


// (lines: the round's pull read its senders' line masks, SCAN_LINES -- the hub
// chunks probe the same masks and gather only the named 128-B lines: round 2
// C4 12.85 -> 12.70 ms, C5 42.35 -> 40.99 ms, profiles/r05_ab_hub_lines.txt)
template <int W>
void launch_hubs_w(Ctx* c, const ExpandArgs& a, bool unfiltered, bool lines) {
  ExpandArgs h = a;
  h.n_items = c->n_hub_items;
  const dim3 grid(grid_for(h.n_items, HWAVES));
  bool done = false;
  if constexpr (W == 64) {
    if (lines && !unfiltered) {
      hipLaunchKernelGGL((k_hub_partial<W, SCAN_FILTERED | SCAN_LINES>), grid, dim3(HBLOCK), 0, c->stream, h);
      done = true;
    }
  }
  if (done) {
  } else if (unfiltered)
    hipLaunchKernelGGL((k_hub_partial<W, SCAN_UNFILTERED>), grid, dim3(HBLOCK), 0, c->stream, h);
  else
    hipLaunchKernelGGL((k_hub_partial<W, SCAN_FILTERED>), grid, dim3(HBLOCK), 0, c->stream, h);
  h.n_items = c->n_hubs;
  hipLaunchKernelGGL(k_hub_final<W>, dim3(grid_for(h.n_items, HWAVES)), dim3(HBLOCK), 0, c->stream, h);
}
template void launch_hubs_w<1>(Ctx*, const ExpandArgs&, bool, bool);
template void launch_hubs_w<2>(Ctx*, const ExpandArgs&, bool, bool);
template void launch_hubs_w<4>(Ctx*, const ExpandArgs&, bool, bool);
template void launch_hubs_w<8>(Ctx*, const ExpandArgs&, bool, bool);
template void launch_hubs_w<16>(Ctx*, const ExpandArgs&, bool, bool);
template void launch_hubs_w<32>(Ctx*, const ExpandArgs&, bool, bool);
template void launch_hubs_w<64>(Ctx*, const ExpandArgs&, bool, bool);

}  // namespace gp
