// driver.hip -- host driver of one gossip round on MI355X (gfx950) and the
// run / output half of the C-ABI (include/gossip_capi.h; setup.hip has the
// configuration half).
//
// One gossip round r over all peers at once:
//   L_r  liveness: crash draws, heartbeat-miss counters, 3-miss detection,
//        dead-node reports, seed removal      (Peer.py:298-393, Seed.py:358-406;
//        liveness.hip)
//   I_r  injection of messages generated in round r     (Peer.py:395-400; k_inject)
//   E_r  expansion: next[v] = OR_{u in In(v)} frontier[u] & ~seen[v]; seen |= next
//        (forward-once with the Message-List slots; the send loop is
//        Peer.py:402-404, the receive side Peer.py:175-216).  launch_expand
//        picks the direction and scan mode; pull.hip / push.hip / hub.hip run it
//   X_r  (multi-GPU) counters' all-reduce, or the vertex partition's boundary
//        exchange over RCCL (partition.hip)
//
// Data layout in HBM: Message-List slots S[0], S[1]
// (u64[n_alloc][W], W words = 64*W messages per vertex), per-vertex fpop /
// seenpop / done_at / state, the in-CSR (row_ptr i64, col and gather-order
// gcol i32).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "gp_device.h"
#include "xplan.h"

namespace gp {

static thread_local std::string g_err;
int set_error(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int copy_sync(Ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
  if (bytes == 0) return 0;
  GP_HIP(hipMemcpyAsync(dst, src, bytes, kind, c->stream));
  GP_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

// partial layout [slot][NPART]: block k sums slot k with one coalesced sweep
__global__ void k_stats_reduce(u64* __restrict__ partial, u64* __restrict__ stats) {
  __shared__ u64 acc[BLOCK];
  const int k = blockIdx.x;
  u64 t = 0;
  for (int p = threadIdx.x; p < NPART; p += BLOCK) {
    t += partial[(size_t)k * NPART + p];
    partial[(size_t)k * NPART + p] = 0;
  }
  acc[threadIdx.x] = t;
  __syncthreads();
  for (int w = BLOCK / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) acc[threadIdx.x] += acc[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) stats[k] += acc[0];
}

// frontier activity bitmap: bit v = (fpop[v] != 0), one word per 64 vertices.
// With dbits (single context, early-exit round without liveness) also the done
// bitmap: bit v = v holds every message of its component (seenpop == done_at,
// components with messages only), as of the end of the last round.
// With liveness (sated: the state bytes) the done bitmap is bit v = v is up and
// sated: it holds every alive message of its component, and
// the alive sets only shrink once no injection is left.
// With deg_live (receiver-list rounds, DESIGN.md §3.5: the pull's waves visit
// only the listed receivers) also every sender's accounting: sends =
// fpop * deg_live and the active count, into the partial stat slots.
__global__ __launch_bounds__(BLOCK) void k_mkbits(const uint32_t* __restrict__ fpop, u64* __restrict__ abits,
                                                  int64_t n, const uint32_t* __restrict__ seenpop,
                                                  const uint32_t* __restrict__ done_at, u64* __restrict__ dbits,
                                                  const uint8_t* __restrict__ sated,
                                                  const int32_t* __restrict__ deg_live, u64* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  u64 sends = 0, active = 0;
  for (int64_t v0 = (int64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63); v0 < n; v0 += stride) {
    const int64_t v = v0 + lane;
    const uint32_t fp = v < n ? fpop[v] : 0u;
    const u64 m = __ballot(fp != 0u);
    if (deg_live && fp) {
      sends += (u64)fp * (u64)(uint32_t)max(deg_live[v], 0);
      ++active;
    }
    if (lane == 0) abits[v0 >> 6] = m;
    if (dbits) {
      bool d = false;
      if (v < n) {
        if (sated) {   // (a complete up vertex holds every alive message too: pulls never mark it)
          const uint8_t sv = sated[v];
          const uint32_t t = done_at[v];
          d = !(sv & ST_DOWN) && ((sv & ST_SATED) || (t != 0u && seenpop[v] == t));
        } else {
          const uint32_t t = done_at[v];
          d = t != 0u && seenpop[v] == t;
        }
      }
      const u64 dm = __ballot(d);
      if (lane == 0) dbits[v0 >> 6] = dm;
    }
  }
  if (deg_live) {
    sends = wave_sum_u64(sends);
    active = wave_sum_u64(active);
    if (lane == 0) {
      const size_t p = blockIdx.x % NPART;
      if (sends) atomicAdd(&partial[(size_t)S_SENDS * NPART + p], sends);
      if (active) atomicAdd(&partial[(size_t)S_ACTIVE * NPART + p], active);
    }
  }
}

// summary level of the activity bitmap: bit j of sbits[k] = (abits[64k + j] != 0)
__global__ __launch_bounds__(BLOCK) void k_mksum(const u64* __restrict__ abits, u64* __restrict__ sbits,
                                                 int64_t nwords) {
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  const int64_t w = k * 64 + lane;
  const u64 m = __ballot(w < nwords && abits[w] != 0ull);
  if (lane == 0 && k * 64 < nwords) sbits[k] = m;
}

// Lost messages (origin down at the inject round, S_LOST) never enter any
// Message-List: drop them from the component targets of this run, so that the
// early-exit and done-skip tests of E_r still fire for the component's
// vertices.  One thread per (group, word) of this round's injection span; the
// state test is k_inject's own (no kernel between them changes state).
__global__ void k_lost_clear(const int32_t* __restrict__ origin, const u64* __restrict__ bits,
                             const uint32_t* __restrict__ cnt, const uint8_t* __restrict__ state,
                             const int32_t* __restrict__ midx, u64* __restrict__ cmask,
                             uint32_t* __restrict__ lostcnt, int64_t off, int64_t groups, int32_t words) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= groups * words) return;
  const int64_t gi = off + t / words;
  const int32_t w = (int32_t)(t % words);
  const int32_t o = origin[gi];
  if (!(state[o] & ST_DOWN)) return;
  const int32_t k = midx[o];
  atomicAnd(cmask + (size_t)k * words + w, ~bits[gi * words + w]);
  if (w == 0) atomicAdd(lostcnt + k, cnt[gi]);
}
__global__ void k_done_fix(const int32_t* __restrict__ midx, const uint32_t* __restrict__ lostcnt,
                           uint32_t* __restrict__ done_at, int64_t n) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
    const int32_t k = midx[v];
    if (k >= 0) {
      const uint32_t l = lostcnt[k];
      if (l) done_at[v] -= l;
    }
  }
}

// ---------------------------------------------------------------------------
// injection (I_r): one wave per (round, origin) group.  The origin's seen row
// is copied into slot r & 1 with the new messages (so that it is read as a
// sender this round, see ExpandArgs) and its frontier count grows.  Slots and
// popcounts are replicated on every rank, so every rank applies every group;
// the owner of the origin also updates seenpop, first-receipt and counters.
struct InjectArgs {
  const int32_t* __restrict__ origin;
  const u64* __restrict__ bits;
  const uint32_t* __restrict__ cnt;
  u64* slot[2];
  int32_t rslot;                       // r & 1
  uint8_t* __restrict__ sp;
  uint8_t* __restrict__ ws;
  uint32_t* __restrict__ fpop;
  u64* __restrict__ frx;               // exact frontier rows (track_msg_forwards, partitioned)
  int64_t frx_rows;                    // ... of vertices [0, frx_rows)
  u64* __restrict__ cmk;               // dense bitmap of slot r & 1 (record rounds, or null)
  u64* __restrict__ alive;             // [W] alive messages of round r (or null)
  uint32_t* __restrict__ seenpop;
  uint8_t* __restrict__ first;
  u64* __restrict__ digest;
  const uint8_t* __restrict__ state;
  uint8_t* __restrict__ lm;            // written line masks of this round's senders (or null)
  u64* __restrict__ partial;
  int64_t off, groups;
  int64_t vbegin, vend;                // owned local ids [vbegin, vend); beyond: ghosts / extras
  int32_t words;
  int32_t wbase;                       // global word index of local word 0 (message shards)
  int32_t r;
};

__global__ __launch_bounds__(BLOCK) void k_inject(InjectArgs a) {
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  WaveStats st;
  ws_zero(st);
  const int64_t k = (int64_t)blockIdx.x * WAVES + wib;
  if (k < a.groups && a.origin[a.off + k] >= 0) {   // (partitioned: every origin is local, never < 0)
    const int64_t gi = a.off + k;
    const int o = a.origin[gi];
    const bool owned = o >= a.vbegin && o < a.vend;
    // partitioned contexts hold every origin; a ghost's row in
    // slot r & 1 is its frontier, valid while its fpop is nonzero
    const bool ghost = o >= a.vend;
    if (a.state[o] & ST_DOWN) {
      if (owned) st.add(S_LOST, a.cnt[gi]);
    } else {
      const uint32_t cur = a.sp[o];
      const uint32_t fp = a.fpop[o];
      const bool has_frx = a.frx && o < a.frx_rows;
      u64 b = 0, s = 0, f = 0;
      if (lane < a.words) {
        b = a.bits[gi * a.words + lane];
        if (ghost ? fp != 0u : cur != SLOT_NONE) s = a.slot[ghost ? a.rslot : cur][(size_t)o * a.words + lane];
        if (has_frx && fp) f = a.frx[(size_t)o * a.words + lane];
      }
      __builtin_amdgcn_wave_barrier();   // the old rows are read before they are rewritten
      if (lane < a.words) {
        a.slot[a.rslot][(size_t)o * a.words + lane] = s | b;
        if (has_frx) a.frx[(size_t)o * a.words + lane] = f | b;
      }
      if (a.cmk && lane == 0) set_dense(a.cmk, o);   // a sender this round: its record (if any) is stale
      if (a.lm) {   // written line masks (64 words): the origin's new row, a superset of its old one
        const u64 nzb = __ballot(lane < a.words && (s | b) != 0ull);
        uint32_t nib = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) nib |= ((nzb >> (16 * t)) & 0xFFFFull) ? (1u << t) : 0u;
        if (lane == 0 && nib) atomicOr(reinterpret_cast<uint32_t*>(a.lm) + (o >> 3), nib << ((o & 7) * 4));
      }
      if (a.alive && b) atomicOr(a.alive + lane, b);   // injected messages are forwarded this round
      const uint32_t nb = wave_sum_u32((uint32_t)__popcll(b));
      if (lane == 0) {
        a.fpop[o] = fp + nb;
        a.sp[o] = (uint8_t)a.rslot;
        a.ws[o] |= (uint8_t)(1u << a.rslot);
      }
      if (owned) {
        const int64_t i = o - a.vbegin;
        if (lane < a.words && a.first && b)
          set_first_bytes(a.first + (size_t)i * a.words * 64, lane, b, (uint32_t)a.r);
        if (a.digest) {
          u64 t = b ? digest_term((uint32_t)a.r, (uint32_t)(a.wbase + lane) | DIGEST_INJECT, b) : 0ull;
          t = wave_xor_u64(t);
          if (lane == 0) a.digest[i] ^= t;
        }
        if (lane == 0) a.seenpop[i] += nb;
        st.add(S_INJECTED, a.cnt[gi]);
      }
    }
  }
  flush_stats(st, a.partial);
}

// ---------------------------------------------------------------------------
// per-message bit sums: cnt[m] += bit_m(row(v)), wsum[m] += weight(v)*bit_m(row(v))
// over rows [0, count).  Lane l holds word l % W of vertex slot l / W; each lane
// keeps 64 register counters per output.
struct BitsumArgs {
  const u64* __restrict__ rows;       // [count][W]
  const uint32_t* __restrict__ guard; // optional: row valid iff guard[i] != 0
  const int32_t* __restrict__ weight; // [count]
  u64* __restrict__ cnt;              // [W*64] or null
  u64* __restrict__ wsum;             // [W*64] or null
  int64_t count;
};

template <int W, bool CNT, bool SUM>
__global__ __launch_bounds__(BLOCK) void k_bitsum(BitsumArgs a) {
  static_assert(W <= 64, "W <= 64");
  constexpr int VPS = 64 / W;   // vertices per wave step
  __shared__ uint32_t lc[CNT ? W * 64 : 1];
  __shared__ uint32_t lsum[SUM ? W * 64 : 1];
  for (int t = threadIdx.x; t < W * 64; t += BLOCK) {
    if (CNT) lc[t] = 0;
    if (SUM) lsum[t] = 0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int w = lane % W, q = lane / W;
  uint32_t c[64], s[64];
#pragma unroll
  for (int b = 0; b < 64; ++b) {
    c[b] = 0;
    s[b] = 0;
  }
  const int64_t step = (int64_t)gridDim.x * WAVES * VPS;
  for (int64_t i = ((int64_t)blockIdx.x * WAVES + wib) * VPS + q; i < a.count; i += step) {
    u64 x = 0;
    if (!a.guard || a.guard[i] != 0) {
      x = a.rows[i * W + w];
    }
    const uint32_t wt = SUM ? (uint32_t)max(a.weight[i], 0) : 0u;
#pragma unroll
    for (int b = 0; b < 64; ++b) {
      const uint32_t bit = (uint32_t)(x >> b) & 1u;
      if (CNT) c[b] += bit;
      if (SUM) s[b] += bit * wt;
    }
  }
#pragma unroll
  for (int b = 0; b < 64; ++b) {
#pragma unroll
    for (int st = W; st < 64; st <<= 1) {
      if (CNT) c[b] += __shfl_xor(c[b], st);
      if (SUM) s[b] += __shfl_xor(s[b], st);
    }
  }
  if (q == 0) {
#pragma unroll
    for (int b = 0; b < 64; ++b) {
      if (CNT && c[b]) atomicAdd(&lc[w * 64 + b], c[b]);
      if (SUM && s[b]) atomicAdd(&lsum[w * 64 + b], s[b]);
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < W * 64; t += BLOCK) {
    if (CNT && lc[t]) atomicAdd(&a.cnt[t], (u64)lc[t]);
    if (SUM && lsum[t]) atomicAdd(&a.wsum[t], (u64)lsum[t]);
  }
}

static void fill_expand(Ctx* c, ExpandArgs& a) {
  a.alive = alive_now(c) ? c->d_alive + (size_t)c->cur * c->words : nullptr;
  a.alive_next = alive_on(c) ? c->d_alive + (size_t)(c->cur ^ 1) * c->words : nullptr;
  a.row_ptr = c->d_row_ptr;
  a.col = c->d_col;
  a.rows = c->d_slot[c->cur];
  a.slot[0] = c->d_slot[0];
  a.slot[1] = c->d_slot[1];
  a.wslot = c->cur ^ 1;
  a.sp = c->d_sp;
  a.ws = c->d_ws;
  a.fpop = c->d_fpop[c->cur];
  a.abits = c->d_abits;
  a.sbits = c->sum_now ? c->d_sbits : nullptr;
  a.dbits = c->dnb_now ? c->d_dbits : nullptr;
  a.amask = c->d_amask;
  a.prehi = c->split_now ? c->d_prehi : nullptr;
  a.split_push = 0;
  a.acc_row = c->split_now ? c->acc_row : 0;
  a.lm = c->lines_now ? (c->lm_written_prev ? c->d_lmw[c->cur] : c->d_lm) : nullptr;
  a.lm_next = c->lm_write_now ? c->d_lmw[c->cur ^ 1] : nullptr;
  a.cmk = c->cml_read_now ? c->d_cmk[c->cur] : nullptr;
  a.cml = c->cml_read_now ? c->d_cml[c->cur] : nullptr;
  a.cmk_next = c->cml_write_now ? c->d_cmk[c->cur ^ 1] : nullptr;
  a.cml_next = c->cml_write_now ? c->d_cml[c->cur ^ 1] : nullptr;
  a.frx = c->d_frx[0] ? c->d_frx[c->cur] : nullptr;
  a.frx_next = c->d_frx[0] ? c->d_frx[c->cur ^ 1] : nullptr;
  a.frx_rows = c->frx_rows;
  a.done_at = c->d_done_at;
  a.gcol = c->d_gcol;
  a.midx = c->d_midx;
  a.cmask = c->d_cmask;
  a.early_exit = c->early_exit_now ? 1 : 0;
  a.dprobe = c->dprobe_now ? 1 : 0;
  a.alias = c->alias_now ? 1 : 0;
  a.ulist = c->ulist_read_now ? c->d_ulist[c->ul_cur] : nullptr;
  a.ulist_n = c->ulist_read_now ? c->ulist_n : 0;
  a.ulist_next = c->ulist_emit_now ? c->d_ulist[c->ul_cur ^ 1] : nullptr;
  a.fpop_next = c->d_fpop[c->cur ^ 1];
  a.seenpop = c->d_seenpop;
  a.first = c->cfg.track_first ? c->d_first : nullptr;
  a.digest = c->cfg.track_digest ? c->d_digest : nullptr;
  a.state = c->d_state;
  a.deg_live = c->d_deg_live;
  a.partial = c->d_stats + 64;   // partial slots live behind the stats block
  a.hub_items = c->d_hub_items;
  a.hubs = c->d_hubs;
  a.hub_item_ptr = c->d_hub_item_ptr;
  a.hub_partial = c->d_hub_partial;
  a.hub_pnz = c->d_hub_pnz;
  a.hub_done = c->d_hub_done;
  if (++c->hub_epoch == 0) c->hub_epoch = 1;   // (wraps after 2^32 launches: 0 is the never-set value)
  a.hub_epoch = c->hub_epoch;
  a.vbegin = 0;   // kernels address local ids: owned vertices are [0, nloc)
  a.nloc = c->nloc();
  a.m_total = c->m;
  a.wbase = c->cfg.msg_word_base;
  a.rr = c->round + 1;
  a.hub_thr = c->cfg.hub_threshold;
  a.orp = c->directed ? c->d_out_row_ptr : c->d_row_ptr;
  a.ocol = c->directed ? c->d_out_col : c->d_col;
  a.acc = c->d_acc;
  a.tbits = c->d_tbits;
  a.touched = c->d_touched;
  a.active = c->d_active;
  a.big = c->d_big;
  a.stats = c->d_stats;
}


#ifndef GP_EE_DIV
#define GP_EE_DIV 16.0
#endif
// rows of <= 8 words (the 512-message shards of an 8-GPU job) take the
// edge-parallel kernel, whose early-exit variant costs one 2-arc prefix pass
// when receivers cannot complete: it pays from m/64 new bits per vertex.  The
// shards of the slower messages cross m/16 a round late, and their dense
// round then gathered every active row (profiles/r05_ee_shards.txt: ranks 5-6
// of the N = 8 job 11.3-11.4 -> 8.7-9.0 ms; W = 16 and 64 keep m/16, the
// 1024-message shard's round 3 lost 0.7 ms at m/64)
#ifndef GP_EE_DIV_NARROW
#define GP_EE_DIV_NARROW 64.0
#endif
static int launch_expand(Ctx* c) {
  if (alive_on(c))   // F_{r+1} is built by this round's receivers
    GP_HIP(hipMemsetAsync(c->d_alive + (size_t)(c->cur ^ 1) * c->words, 0, (size_t)c->words * 8, c->stream));
  // direction: push when the senders' arcs are a small share of all arcs
  const int r = c->round;
  // early exit pays once frontier rows are dense: >= m/16 new bits per vertex last round
  // or once most messages are held: receivers then miss a few words at most, and
  // the word skip loads only those (under churn the component targets may be
  // out of reach -- a message cut off by crashes -- so the done-skip alone
  // leaves nearly every receiver scanning whole rows)
  const double ee_div = c->words <= 8 ? GP_EE_DIV_NARROW : GP_EE_DIV;
  c->early_exit_now = c->cfg.early_exit != 0 &&
                      ((double)c->prev_new_bits * ee_div >= (double)c->n * (double)c->m ||
                       (double)c->held_bits * 2.0 >= (double)c->n * (double)c->m);
  const u64 inj = (size_t)r < c->inj_arcs.size() ? (u64)c->inj_arcs[(size_t)r] : 0ull;
  const double est = (double)((r == 0 ? 0ull : c->prev_next_arcs) + inj);
  // narrow rows push at a lower ratio: the pull's per-arc scan does not
  // shrink with W, the push's row words do (k_apply_lanes, k_mkneed)
#ifndef GP_NARROW_PUSH_SCALE
#define GP_NARROW_PUSH_SCALE 0.25
#endif
  // (early rounds only: late rounds' pulls skip the done receivers, which the
  // estimate does not see -- the 512-message shard's round 6 pulls in 0.27 ms
  // and pushes in 0.72)
  const bool early = (double)c->held_bits * 2.0 < (double)c->n * (double)c->m;
#ifndef GP_NARROW_PUSH_MAXW
#define GP_NARROW_PUSH_MAXW 16
#endif
  const double ratio = c->cfg.push_ratio * (c->words <= GP_NARROW_PUSH_MAXW && early ? GP_NARROW_PUSH_SCALE : 1.0);
  c->mode_push = c->cfg.push_ratio > 0.0 && est * ratio <= (double)c->nnz;
  // last round's receivers + this round's injected origins send this round
  const double senders = (double)c->prev_receivers + (double)c->inj_groups_at(r);
  // narrow rows: a round that pushes only because of the narrow scale pulls
  // as a degree-split round instead (its prefix probes are a fraction of the
  // arcs, its push half only the low-degree senders' arcs) -- but only when
  // the pull would be one: the conditions of unfiltered_now, arc_mask_now,
  // prefilter_now and split_now below, for a pull (records: W = 64 only)
#ifndef GP_SPLIT_NARROW
#define GP_SPLIT_NARROW 1
#endif
  const bool pull_unfiltered = c->cfg.unfiltered_pct > 0 &&
                               senders * 100.0 >= (double)c->cfg.unfiltered_pct * (double)c->n;
  const bool pull_masked = !pull_unfiltered && c->cfg.arc_mask_permille > 0 &&
                           senders * 1000.0 >= (double)c->cfg.arc_mask_permille * (double)c->n;
  const bool pull_splits = c->cfg.split_deg > 0 && !c->early_exit_now && !c->local && c->nloc() == c->n_alloc &&
                           c->words < 64 && !pull_unfiltered && !pull_masked && c->cfg.prefilter_pct > 0 &&
                           senders * 100.0 < (double)c->cfg.prefilter_pct * (double)c->n &&
                           senders * 1000.0 < (double)c->cfg.split_max_permille * (double)c->n;
  const bool narrow_split = GP_SPLIT_NARROW && c->mode_push && pull_splits && est * c->cfg.push_ratio > (double)c->nnz;
  if (narrow_split) c->mode_push = false;
  c->push_est = est;
  if (c->mode_push && c->nloc() > 0)
    GP_HIP(hipMemsetAsync(c->d_fpop[c->cur ^ 1], 0, (size_t)c->nloc() * 4, c->stream));
  // unfiltered pull when (nearly) every vertex is a sender: last round's
  // receivers + this round's injected origins >= unfiltered_pct % of n.  With
  // liveness a crashed vertex's Message-List may hold bits it never sent, so
  // the down vertices' rows are parked first (k_park; one vertex set per
  // context, hence not in a vertex partition, whose ghosts' rows are frontiers)
  c->unfiltered_now = !c->mode_push && c->cfg.unfiltered_pct > 0 &&
                      senders * 100.0 >= (double)c->cfg.unfiltered_pct * (double)c->n;
  if (c->unfiltered_now && c->liveness_active) {
    if (c->local || c->park_failed) {
      c->unfiltered_now = false;
    } else if (!c->d_slot[2]) {
      if (dalloc(&c->d_slot[2], (size_t)c->n_alloc * c->words) != 0) {
        c->park_failed = true;   // (out of memory: stay filtered)
        c->unfiltered_now = false;
        (void)hipGetLastError();
      }
    }
  }
  // done in-neighbours: without liveness a receiver with an
  // in-neighbour that held its whole component at the end of the last round
  // receives exactly cmask & ~seen.  Pull rounds of the per-receiver kernel
  // once most messages are held (before that hardly any vertex is done, and
  // the probes only cost); the done bitmap comes with the activity bitmap (one
  // context: seenpop and done_at share the vertex index)
  // Narrow rows (W = 8 / 16: the message shards of 4- and 8-GPU jobs) take the
  // per-receiver kernel instead of the flat one in the thin late rounds (under
  // 1/GP_NARROW_ND_DIV of the n x m bits still missing): its receivers go
  // eight / sixteen per wave step (dnb_groups, gather_groups), while the flat
  // kernel keeps the dense rounds, the last of which leaves a shard ~1 % short
#ifndef GP_NARROW_ND
#define GP_NARROW_ND 1
#endif
#ifndef GP_NARROW_ND_DIV
#define GP_NARROW_ND_DIV 16
#endif
  const double nm = (double)c->n * (double)c->m;
  c->narrow_pr_now = GP_NARROW_ND && (c->words == 8 || c->words == 16) && c->words <= c->cfg.flat_max_words &&
                     c->early_exit_now && !c->mode_push && !c->liveness_active && !c->local &&
                     c->nloc() == c->n_alloc && (nm - (double)c->held_bits) * GP_NARROW_ND_DIV < nm;
  c->dnb_now = c->early_exit_now && !c->mode_push && !c->liveness_active && !c->local &&
               c->nloc() == c->n_alloc && (c->words > c->cfg.flat_max_words || c->narrow_pr_now) &&
               (double)c->held_bits * 2.0 >= (double)c->n * (double)c->m;
  // With liveness the done bitmap is the sated marks (up and sated: holds every
  // alive message of its component; k_mkbits): a receiver with such an
  // in-neighbour receives exactly cmask & F_r & ~seen, since every bit of it
  // lies in that neighbour's frontier (it sent everything older while both were
  // up, and crashes are final).  From the round after the first marking round.
  if (!c->dnb_now && c->liveness_active && alive_now(c) && c->early_exit_now && !c->mode_push &&
      !c->local && c->nloc() == c->n_alloc && c->words > c->cfg.flat_max_words && c->sate_since >= 0 &&
      c->round > c->sate_since)
    c->dnb_now = true;
  // aliased Message-Lists (W = 64, no liveness, one context,
  // no compact records): in done-neighbour rounds receivers that complete
  // commit SLOT_CMASK instead of a 512-B row.  Once a run holds aliases every
  // pull probes the done bitmap for each arc it scans (a receiver with any
  // done in-neighbour takes its target, so no aliased row slot is gathered);
  // held bits only grow, so early exit and the done bitmap stay on.  The
  // first aliasing round reads rows written before any alias and needs no
  // probe (C4 round 4: 74.6 M arcs whose probe would sit in each pass's
  // dependent chain).  A push round first writes its aliased senders' rows
  // (k_unalias)
#ifndef GP_ALIAS
#define GP_ALIAS 1
#endif
  const bool alias_ok = GP_ALIAS && c->words == 64 && !c->liveness_active && !c->local && c->nloc() == c->n_alloc &&
                        c->cfg.compact_rows == 0 && c->words > c->cfg.flat_max_words;
  c->alias_now = c->dnb_now && alias_ok;
  c->dprobe_now = c->alias_now && c->alias_active;
  // receiver lists (W = 64 early-exit pulls, one context):
  // once most messages are held, each pull appends the receivers that stay
  // neither done nor sated; a pull whose list is under a third of the
  // vertices launches waves for those alone, k_mkbits does every sender's
  // accounting and the receivers' fpop_next starts zeroed (C5 round 6: 1.26 M
  // receivers of 64 M vertices)
#ifndef GP_ULIST
#define GP_ULIST 1
#endif
  const bool list_ok = GP_ULIST && !c->mode_push && !c->local && c->nloc() == c->n_alloc && c->words == 64 &&
                       c->words > c->cfg.flat_max_words && c->cfg.compact_rows == 0 && c->early_exit_now;
#ifndef GP_ULIST_DIV
#define GP_ULIST_DIV 3
#endif
  c->ulist_read_now = list_ok && c->ulist_valid && c->ulist_n * GP_ULIST_DIV < c->n_alloc;
  if (c->ulist_read_now)
    GP_HIP(hipMemsetAsync(c->d_fpop[c->cur ^ 1], 0, (size_t)c->nloc() * 4, c->stream));
  hipLaunchKernelGGL(k_mkbits, dim3(std::max(1, std::min(grid_for(c->n_alloc, BLOCK), c->cu_count * 8 * GS))),
                     dim3(BLOCK), 0, c->stream, c->d_fpop[c->cur], c->d_abits, c->n_alloc,
                     c->d_seenpop, c->d_done_at, c->dnb_now ? c->d_dbits : nullptr,
                     c->dnb_now && c->liveness_active ? (const uint8_t*)c->d_state : nullptr,
                     c->ulist_read_now ? (const int32_t*)c->d_deg_live : nullptr, c->d_stats + 64);
  if (c->alias_active) {   // (after k_mkbits: a push round's senders are the activity bitmap's bits)
    if (c->mode_push) GP_TRY(unalias(c, true));
    else if (!c->dprobe_now) GP_TRY(unalias(c, false));   // (a pull that could gather a done sender's row)
  }
  // filtered pull: probe every arc inside the scan, or build the per-arc mask
  // first (pays once the probes are many: senders >= arc_mask_permille of n)
  c->arc_mask_now = !c->mode_push && !c->unfiltered_now && c->cfg.arc_mask_permille > 0 &&
                    senders * 1000.0 >= (double)c->cfg.arc_mask_permille * (double)c->n;
  // summary probes: filtered rounds of overlays whose activity bitmap outgrows
  // an XCD's L2, while few enough vertices send that most summary bits are 0
  c->sum_now = false;
  if (!c->mode_push && !c->unfiltered_now && !c->arc_mask_now && c->cfg.summary_min_n > 0 &&
      c->n_alloc >= c->cfg.summary_min_n &&
      senders * SUMMARY_RATIO <= (double)c->n) {
    const int64_t nwords = (c->n_alloc + 63) / 64;
    hipLaunchKernelGGL(k_mksum, dim3(grid_for((nwords + 63) / 64, WAVES)), dim3(BLOCK), 0, c->stream,
                       c->d_abits, c->d_sbits, nwords);
    c->sum_now = true;
  }
  // Message-List records (W = 64): written while the rows are sparse (last
  // round's receivers got <= CML_AVG_BITS new bits on average), read by a
  // filtered pull without early exit whose senders all wrote theirs (or their
  // dense bit) in the previous round.  Senders are exactly the vertices with
  // fpop != 0 under liveness too (a crash zeroes fpop), and a sender's record
  // mirrors its row, so records and full rows give the same OR.
  {
    constexpr double CML_AVG_BITS = 16.0;
    const bool ok = c->d_cml[0] != nullptr && c->words == 64 && !c->mode_push;
    const bool sparse = (double)c->prev_new_bits <= CML_AVG_BITS * (double)std::max<u64>(c->prev_receivers, 1);
    c->cml_read_now = ok && c->cml_written_prev && !c->unfiltered_now && !c->arc_mask_now && !c->early_exit_now;
    c->cml_write_now = ok && sparse && !c->unfiltered_now && !c->arc_mask_now;   // the kernels that write them
  }
  // line masks (W = 64): a filtered pull without early exit reads its
  // senders' rows while they are still sparse; their zero 128-B lines are
  // skipped.  The launch narrows this to the plain
  // per-receiver kernel (k_expand<64, SCAN_FILTERED | SCAN_LINES>)
  c->lines_now = c->words == 64 && c->d_lm != nullptr && !c->mode_push && !c->unfiltered_now &&
                 !c->arc_mask_now && !c->early_exit_now && c->n_alloc <= (int64_t(1) << 27);   // (u << 4) | lines
  // this round's 64-word pull commits write the next round's masks: one
  // context (ghosts' rows come from the exchange), per-receiver kernel, no
  // records; under liveness k_churn zeroes a crashing sender's nibble with
  // its fpop (round 4 of the build; k_mklm ran there until then)
  // (only sparse rounds: a line-mask round follows a round with few new bits,
  // and early-exit rounds would pay the commits' extra stores for nothing --
  // C4 rounds 3-4 +0.3 ms when every pull wrote them)
  c->lm_write_now = c->words == 64 && c->d_lmw[0] != nullptr && !c->mode_push &&
                    !c->early_exit_now && !c->local && !c->cml_read_now && !c->cml_write_now;
  // sparse filtered pull: the lane phase probes the in-lists of low-degree receivers
  c->prefilter_now = !c->mode_push && !c->unfiltered_now && !c->arc_mask_now && c->cfg.prefilter_pct > 0 &&
                     senders * 100.0 < (double)c->cfg.prefilter_pct * (double)c->n;
  // degree-split: a prefiltered per-receiver pull without
  // early exit (C4 / C5 round 1), one context, no compact Message-Lists:
  // senders of in-degree < split_deg push (few arcs: they are the
  // low-degree minority of a degree-biased sender set), receivers probe only
  // the gather-order prefix of bigger senders
  // Only while the senders are a sliver of the vertices (C4 / C5 round 1:
  // 0.1-0.4 %): the 512-message shards' round 2, prefiltered with 7-13 % of
  // the vertices sending, pushed 30-67 M low-degree arcs in 3.3-5.9 ms
  // against a 1.8-1.9 ms pull half (profiles/r04_split_cap.txt)
  c->split_now = c->cfg.split_deg > 0 && c->prefilter_now && !c->early_exit_now && !c->local &&
                 c->nloc() == c->n_alloc && !c->cml_read_now && !c->cml_write_now &&
                 senders * 1000.0 < (double)c->cfg.split_max_permille * (double)c->n;
  if (c->split_now) {   // accumulator rows as rows of this round's slot buffer: same allocation, same stride
    const int64_t row = (int64_t)(c->d_acc - c->d_slot[c->cur]) / c->words;   // (d_rows: S[0] | S[1] | acc)
    c->split_now = row > 0 && row + c->nloc() <= (int64_t)INT32_MAX;
    c->acc_row = (int32_t)row;
  }
  if (c->dprobe_now || c->ulist_read_now) {   // the scan modes of these variants: filtered and unfiltered
    c->arc_mask_now = c->prefilter_now = c->split_now = false;
    c->cml_read_now = c->cml_write_now = c->lines_now = c->lm_write_now = false;
  }
  // (only once the rounds thin out: last round's new bits under m/4 per
  // vertex -- C4 round 4's survivors, 7.6 M, would make no list worth reading,
  // and appending them cost the round 0.07 ms)
  c->ulist_emit_now = list_ok && (double)c->held_bits * 2.0 >= (double)c->n * (double)c->m &&
                      (double)c->prev_new_bits * 4.0 < (double)c->n * (double)c->m && !c->arc_mask_now &&
                      !c->prefilter_now && !c->split_now && !c->cml_read_now && !c->cml_write_now && !c->lines_now;
  if (c->ulist_emit_now && !c->d_ulist[0]) {
    if (dalloc(&c->d_ulist[0], (size_t)c->n_alloc) != 0 || dalloc(&c->d_ulist[1], (size_t)c->n_alloc) != 0) {
      dfree(&c->d_ulist[0]);   // (out of memory: no lists)
      dfree(&c->d_ulist[1]);
      c->ulist_emit_now = false;
      (void)hipGetLastError();
    }
  }
  if (narrow_split && !c->split_now)   // (the conditions above mirror these: a pull was promised a split)
    return set_error(GP_ESTATE, "internal: narrow-row split round not eligible");
  if (c->split_now) GP_TRY(build_prehi(c, c->cfg.split_deg));
  ExpandArgs a{};
  fill_expand(c, a);
  a.unfiltered = c->unfiltered_now ? 1 : 0;
  // (not with liveness: messages cut off by crashes keep the component targets
  // out of reach, receivers scan to the end and want every row in flight --
  // C5 rounds 5-6 56.8 -> 64.3 ms with the switch on)
  a.near_done = c->early_exit_now && !c->liveness_active &&
                (double)c->held_bits * 2.0 >= (double)c->n * (double)c->m ? 1 : 0;
  // sated vertices (churn): with no injection left, a receiver that ends the
  // round holding every alive message of its component never receives again
  a.sate = alive_now(c) && c->early_exit_now && c->round >= c->last_inject_round ? 1 : 0;
  if (a.sate && c->sate_since < 0) c->sate_since = c->round;
  c->lines_ran = c->lines_from_commits = false;
  return launch_round_kernels(c, a);
}

template <int W>
static void launch_bitsum_w(Ctx* c, BitsumArgs a, bool cnt, bool sum) {
  const int grid = std::max(1, std::min(grid_for(a.count, (int64_t)WAVES * (64 / W)), c->cu_count * 2 * GS));
  if (cnt && sum)
    hipLaunchKernelGGL((k_bitsum<W, true, true>), dim3(grid), dim3(BLOCK), 0, c->stream, a);
  else if (cnt)
    hipLaunchKernelGGL((k_bitsum<W, true, false>), dim3(grid), dim3(BLOCK), 0, c->stream, a);
  else if (sum)
    hipLaunchKernelGGL((k_bitsum<W, false, true>), dim3(grid), dim3(BLOCK), 0, c->stream, a);
}

static int launch_bitsum(Ctx* c, BitsumArgs a, bool cnt, bool sum) {
  if (a.count <= 0) return 0;
  switch (c->words) {
    case 1: launch_bitsum_w<1>(c, a, cnt, sum); break;
    case 2: launch_bitsum_w<2>(c, a, cnt, sum); break;
    case 4: launch_bitsum_w<4>(c, a, cnt, sum); break;
    case 8: launch_bitsum_w<8>(c, a, cnt, sum); break;
    case 16: launch_bitsum_w<16>(c, a, cnt, sum); break;
    case 32: launch_bitsum_w<32>(c, a, cnt, sum); break;
    case 64: launch_bitsum_w<64>(c, a, cnt, sum); break;
    default: return set_error(GP_EINVAL, "unsupported word count");
  }
  GP_HIP(hipGetLastError());
  return 0;
}

// phases L_r, I_r, E_r of one round on one context (no host sync)
static int round_launch(Ctx* c) {
  if (!state_ready(c) || c->words <= 0) return set_error(GP_ESTATE, "gp_set_messages + gp_reset first");
  if (c->round > 253) return set_error(GP_ESTATE, "round limit (254) reached");
  GP_HIP(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  u64* stats = c->d_stats;
  u64* partial = c->d_stats + 64;
  const int r = c->round;
  GP_HIP(hipMemsetAsync(stats, 0, 64 * sizeof(u64), s));
  GP_HIP(hipEventRecord(c->ev[0], s));
  if (c->liveness_active) {
    c->msg_forwards_valid = c->msg_forwards_valid && (c->cfg.track_msg_forwards != 0);
    GP_TRY(launch_liveness(c));
  }

  auto it = c->inject.find(r);
  if (it != c->inject.end() && it->second.cnt > 0) {
    GP_TRY(unalias(c, false));   // (k_inject reads the origins' rows; no vertex completes before the last injection)
    InjectArgs ia{};
    ia.origin = c->d_inj_origin;
    ia.bits = c->d_inj_bits;
    ia.cnt = c->d_inj_cnt;
    ia.slot[0] = c->d_slot[0];
    ia.slot[1] = c->d_slot[1];
    ia.rslot = c->cur;
    ia.sp = c->d_sp;
    ia.ws = c->d_ws;
    ia.fpop = c->d_fpop[c->cur];
    ia.frx = c->d_frx[0] ? c->d_frx[c->cur] : nullptr;
    ia.frx_rows = c->frx_rows;
    ia.cmk = c->d_cmk[0] ? c->d_cmk[c->cur] : nullptr;
    ia.alive = alive_on(c) ? c->d_alive + (size_t)c->cur * c->words : nullptr;
    ia.seenpop = c->d_seenpop;
    ia.first = c->cfg.track_first ? c->d_first : nullptr;
    ia.digest = c->cfg.track_digest ? c->d_digest : nullptr;
    ia.state = c->d_state;
    ia.lm = c->lm_written_prev ? c->d_lmw[c->cur] : nullptr;
    ia.partial = partial;
    ia.off = it->second.off;
    ia.groups = it->second.cnt;
    ia.vbegin = 0;
    ia.vend = c->nloc();
    ia.words = c->words;
    ia.wbase = c->cfg.msg_word_base;
    ia.r = r;
    hipLaunchKernelGGL(k_inject, dim3(grid_for(ia.groups, WAVES)), dim3(BLOCK), 0, s, ia);
    GP_HIP(hipGetLastError());
    if (c->liveness_active && c->cmask_rows > 0) {   // origins may be down: drop lost messages
      GP_HIP(hipMemsetAsync(c->d_lostcnt, 0, (size_t)c->cmask_rows * 4, s));
      hipLaunchKernelGGL(k_lost_clear, dim3(grid_for(ia.groups * c->words, 256)), dim3(256), 0, s,
                         c->d_inj_origin, c->d_inj_bits, c->d_inj_cnt, c->d_state, c->d_midx, c->d_cmask,
                         c->d_lostcnt, ia.off, ia.groups, c->words);
      hipLaunchKernelGGL(k_done_fix, dim3(std::min(grid_for(c->n_alloc, 256), c->cu_count * 8)), dim3(256), 0, s,
                         c->d_midx, c->d_lostcnt,
                         c->d_done_at, c->n_alloc);
      GP_HIP(hipGetLastError());
      c->done_dirty = true;
    }
  }

  if (c->cfg.track_msg_forwards) {   // sends of round r per message (owned senders)
    BitsumArgs b{};
    b.rows = c->d_frx[c->cur];   // exact frontier rows of the owned senders
    b.guard = c->d_fpop[c->cur];
    b.weight = c->d_deg_live;
    b.cnt = nullptr;
    b.wsum = c->d_msg_fwd;
    b.count = c->nloc();
    GP_TRY(launch_bitsum(c, b, false, true));
  }

  GP_HIP(hipEventRecord(c->ev[1], s));
  GP_TRY(launch_expand(c));
  hipLaunchKernelGGL(k_stats_reduce, dim3(NST), dim3(BLOCK), 0, s, partial, stats);
  GP_HIP(hipGetLastError());
  GP_HIP(hipEventRecord(c->ev[2], s));

  return 0;
}

// X_r over RCCL.  One rank: the counters' all-reduce is the whole exchange.
// Vertex partition: the boundary exchange of partition.hip (this round's new
// bits of the owned vertices other ranks hold as ghosts, removal flags, alive
// sets) and the counters' all-reduce, so that every rank takes the same
// decisions next round.
static int round_exchange_rccl(Ctx* c) {
  if (!c->comm) {
    if (c->local) return set_error(GP_ESTATE, "a partitioned context exchanges over RCCL (gp_comm_init) "
                                              "or in gp_round_group");
    return 0;
  }
  if (c->local) return exchange_rccl(c);
  // the report cursor (slot S_REPORT_CURSOR) stays rank-local
  GP_RCCL(ncclAllReduce(c->d_stats, c->d_stats, S_REPORT_CURSOR, ncclUint64, ncclSum, c->comm, c->stream));
  return 0;
}

static int round_collect(Ctx* c, gp_round_stats* out) {
  hipStream_t s = c->stream;
  const int r = c->round;
  GP_HIP(hipEventRecord(c->ev[3], s));
  GP_HIP(hipMemcpyAsync(c->h_stats, c->d_stats, 64 * sizeof(u64), hipMemcpyDeviceToHost, s));
  GP_HIP(hipStreamSynchronize(s));
  const u64* h = c->h_stats;
  if (h[S_XERR])   // (every rank of an RCCL partition sees the all-reduced count)
    return set_error(GP_ERCCL, "boundary exchange: " + std::to_string(h[S_XERR]) +
                                   " received entries do not match the exchange plan (round " + std::to_string(r) + ")");
  gp_round_stats own;
  {
    gp_round_stats* out = &own;   // (kept for the run: a shard job's combine reads it)
    std::memset(out, 0, sizeof(*out));
    out->round = r;
    out->injected = h[S_INJECTED];
    out->lost = h[S_LOST];
    out->new_bits = h[S_NEW_BITS];
    out->receivers = h[S_RECEIVERS];
    out->sends = h[S_SENDS];
    out->active = h[S_ACTIVE];
    out->crashed = h[S_CRASHED];
    out->reports = h[S_REPORTS];
    out->removals = h[S_REMOVALS];
    out->dup_reports = h[S_DUP];
    out->arcs_scanned = h[S_ARCS];
    out->rows_gathered = h[S_GATHERED];
    out->seen_rows_read = h[S_SEEN_READ];
    out->rows_written = h[S_WRITTEN];
    out->vertices_visited = h[S_VISITED];
    out->atomics = h[S_ATOMICS];
    out->next_arcs = h[S_NEXT_ARCS];
    out->row_bytes = h[S_ROW_BYTES];
    out->mode = c->mode_push ? 1 : 0;
    out->scan = c->mode_push ? 0 : (c->unfiltered_now ? 2 : c->arc_mask_now ? 1 : c->prefilter_now ? 3 : 0) |
                                       (c->cml_read_now ? 4 : 0) | (c->lines_ran ? 8 : 0) |
                                       (c->lines_from_commits ? 16 : 0) | (c->split_now ? 32 : 0) |
                                       (c->dprobe_now ? 64 : 0) | (c->ulist_read_now ? 128 : 0);
    out->kernel_ms = 0.0;
    if (!c->mode_push && c->nloc() > 0) {
      float kms = 0.f;
      (void)hipEventElapsedTime(&kms, c->ev[4], c->ev[5]);
      out->kernel_ms = kms;
    }
    out->overflow = (int64_t)h[S_REPORT_CURSOR] > c->report_cap ? 1 : 0;
    out->xchg_rows = h[S_XROWS];
    out->xchg_bytes = h[S_XBYTES];
    out->done_nb = h[S_DNB];
    out->lm_rows = h[S_LM_ROWS];
    out->aliased = h[S_ALIASED];
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, c->ev[1], c->ev[2]);
    out->expand_ms = ms;
    (void)hipEventElapsedTime(&ms, c->ev[2], c->ev[3]);
    out->exchange_ms = ms;
    (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[3]);
    out->round_ms = ms;
  }
  if (out) *out = own;
  c->run_stats.push_back(own);
  c->last_reports = (int64_t)h[S_REPORT_CURSOR];
  c->prev_next_arcs = h[S_NEXT_ARCS];
  c->prev_new_bits = h[S_NEW_BITS];
  c->prev_receivers = h[S_RECEIVERS];
  c->held_bits += h[S_INJECTED] + h[S_NEW_BITS];
  c->cml_written_prev = c->cml_write_now;
  c->lm_written_prev = c->lm_write_now;
  if (h[S_ALIASED]) c->alias_active = true;
  c->ulist_valid = c->ulist_emit_now;   // (a round that appends no list ends the last one)
  if (c->ulist_emit_now) {
    c->ulist_n = (int64_t)h[S_ULIST];
    c->ul_cur ^= 1;
  }
  c->ulist_emit_now = c->ulist_read_now = false;
  c->cur ^= 1;
  c->round = r + 1;
  return 0;
}

}  // namespace gp

using namespace gp;

// ===========================================================================
// C-ABI
extern "C" {

int gp_abi_version(void) { return GP_ABI_VERSION; }
const char* gp_last_error(void) { return g_err.c_str(); }

int gp_device_count(int* n_out) {
  if (!n_out) return set_error(GP_EINVAL, "null n_out");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *n_out = n;
  return 0;
}

}  // extern "C"

extern "C" {

int gp_round(gp_ctx* c, gp_round_stats* out) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  if (c->local && !c->comm)
    return set_error(GP_ESTATE, "a partitioned context exchanges over RCCL (gp_comm_init) or in gp_round_group");
  GP_TRY(round_launch(c));
  GP_TRY(round_exchange_rccl(c));
  if (c->jnranks > 0) GP_TRY(shard_record_round(c));   // (message-shard job: shard.hip)
  return round_collect(c, out);
}

int gp_round_group(gp_ctx** ctxs, int32_t nctx, gp_round_stats* out) {
  if (!ctxs || nctx < 1) return set_error(GP_EINVAL, "bad context list");
  for (int32_t k = 0; k < nctx; ++k) {
    Ctx* c = ctxs[k];
    if (!c) return set_error(GP_EINVAL, "null ctx in group");
    if (c->comm) return set_error(GP_EINVAL, "group rounds exchange without RCCL");
    if (c->nranks != nctx || c->rank != k) return set_error(GP_EINVAL, "ctxs[k] must own partition k of nctx");
    if (c->round != ctxs[0]->round || c->n != ctxs[0]->n || c->words != ctxs[0]->words)
      return set_error(GP_EINVAL, "contexts out of step");
  }
  for (int32_t k = 0; k < nctx; ++k) GP_TRY(round_launch(ctxs[k]));
  // X_r: the boundary exchange through device-to-device copies -- the same
  // pack / unpack as over RCCL (partition.hip)
  if (nctx > 1) {
    std::vector<Ctx*> cs(ctxs, ctxs + nctx);
    GP_TRY(exchange_group(cs.data(), nctx));
  }
  gp_round_stats sum;
  std::vector<u64> own_held((size_t)nctx, 0);
  std::memset(&sum, 0, sizeof(sum));
  for (int32_t k = 0; k < nctx; ++k) {
    gp_round_stats st;
    GP_TRY(round_collect(ctxs[k], &st));
    own_held[(size_t)k] = st.injected + st.new_bits;
    sum.round = st.round;
    sum.overflow |= st.overflow;
    sum.injected += st.injected; sum.lost += st.lost; sum.new_bits += st.new_bits;
    sum.receivers += st.receivers; sum.sends += st.sends; sum.active += st.active;
    sum.crashed += st.crashed; sum.reports += st.reports; sum.removals += st.removals;
    sum.dup_reports += st.dup_reports; sum.arcs_scanned += st.arcs_scanned;
    sum.rows_gathered += st.rows_gathered; sum.seen_rows_read += st.seen_rows_read;
    sum.rows_written += st.rows_written; sum.vertices_visited += st.vertices_visited;
    sum.atomics += st.atomics; sum.next_arcs += st.next_arcs; sum.mode = st.mode;
    sum.row_bytes += st.row_bytes; sum.scan = st.scan;
    sum.xchg_rows += st.xchg_rows; sum.xchg_bytes += st.xchg_bytes; sum.done_nb += st.done_nb;
    sum.lm_rows += st.lm_rows;
    sum.expand_ms = std::max(sum.expand_ms, st.expand_ms);
    sum.exchange_ms = std::max(sum.exchange_ms, st.exchange_ms);
    sum.round_ms = std::max(sum.round_ms, st.round_ms);
    sum.kernel_ms = std::max(sum.kernel_ms, st.kernel_ms);
  }
  for (int32_t k = 0; k < nctx; ++k) {   // every context takes the same decisions next round
    ctxs[k]->prev_next_arcs = sum.next_arcs;
    ctxs[k]->prev_new_bits = sum.new_bits;
    ctxs[k]->prev_receivers = sum.receivers;
    // round_collect added the context's own share; every context holds the sum
    ctxs[k]->held_bits += sum.injected + sum.new_bits - own_held[(size_t)k];
  }
  if (out) *out = sum;
  return 0;
}

int gp_run(gp_ctx* c, int32_t max_rounds, gp_round_stats* per_round, int32_t* rounds_out) {
  if (!c || max_rounds < 1) return set_error(GP_EINVAL, "bad argument");
  int32_t done = 0;
  for (int32_t k = 0; k < max_rounds; ++k) {
    gp_round_stats st;
    GP_TRY(gp_round(c, &st));
    if (per_round) per_round[k] = st;
    ++done;
    if (st.new_bits == 0 && st.round >= c->last_inject_round) break;
  }
  if (rounds_out) *rounds_out = done;
  return 0;
}

// finalize through the component targets (bitcount.hip); GP_FINALIZE_ROWS=1 in
// the environment counts every row instead (the tests compare the two)
static bool finalize_by_rows() {
  const char* e = getenv("GP_FINALIZE_ROWS");
  return e && e[0] == '1';
}
int gp_finalize_messages(gp_ctx* c) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  if (!state_ready(c)) return set_error(GP_ESTATE, "no run state");
  GP_HIP(hipSetDevice(c->device));
  const size_t M = (size_t)c->words * 64;
  hipStream_t s = c->stream;
  u64* cov = c->d_msg_cov;
  u64* fwd_local = c->d_msg_fwd;
  u64* gcov = c->d_msg_cov + 2 * M;
  u64* gfwd = c->d_msg_cov + 3 * M;
  const bool fwd_from_seen = !c->liveness_active && !c->cfg.track_msg_forwards;
  // seen row i = slot[sp[i]][i], owned local ids [0, nloc): bit-sliced counts
  // (bitcount.hip), forwards weighted by the static degree (= deg_live without liveness)
  if (c->done_at_valid && !finalize_by_rows()) GP_TRY(finalize_by_components(c, fwd_from_seen, cov, fwd_local));
  else GP_TRY(bitcount_messages(c, fwd_from_seen, cov, fwd_local));
  if (c->comm) {
    GP_RCCL(ncclGroupStart());
    GP_RCCL(ncclAllReduce(cov, gcov, M, ncclUint64, ncclSum, c->comm, s));
    GP_RCCL(ncclAllReduce(fwd_local, gfwd, M, ncclUint64, ncclSum, c->comm, s));
    GP_RCCL(ncclGroupEnd());
  } else {
    GP_HIP(hipMemcpyAsync(gcov, cov, M * 8, hipMemcpyDeviceToDevice, s));
    GP_HIP(hipMemcpyAsync(gfwd, fwd_local, M * 8, hipMemcpyDeviceToDevice, s));
  }
  GP_HIP(hipStreamSynchronize(s));
  c->fin_round = c->round;
  return 0;
}

int gp_read(gp_ctx* c, int32_t what, void* host, int64_t bytes) {
  if (!c || !host) return set_error(GP_EINVAL, "null argument");
  GP_HIP(hipSetDevice(c->device));
  GP_HIP(hipStreamSynchronize(c->stream));
  // partitioned contexts read their owned slice of the per-vertex arrays
  // (local ids [0, nloc) = global [vbegin, vend)) and their local CSR
  const int64_t W = c->words, nl = c->nloc(), M = c->m, n = c->local ? c->nloc() : c->n;
  auto need = [&](int64_t b) -> int {
    if (bytes != b) return set_error(GP_EINVAL, "bytes mismatch: expected " + std::to_string(b));
    return 0;
  };
  const bool run = state_ready(c);
  switch (what) {
    case GP_SEEN:
      if (!run) return set_error(GP_ESTATE, "no run state");
      GP_TRY(need(nl * W * 8));
      GP_TRY(unalias(c, false));   // (aliased Message-Lists become rows of S[cur])
      if (bytes) {   // owned rows of every slot, picked per vertex by its slot byte
        // blocks of rows: host scratch stays at 2 blocks whatever n (a 2^26 x
        // 4096 read would otherwise hold two more 32 GiB copies)
        const int64_t blk = std::max<int64_t>(1, (int64_t(64) << 20) / (W * 8));
        std::vector<uint64_t> s1((size_t)(std::min(nl, blk) * W)), s2(c->d_slot[2] ? s1.size() : 0);
        std::vector<uint8_t> sp((size_t)nl);
        GP_TRY(copy_sync(c, sp.data(), c->d_sp, (size_t)nl, hipMemcpyDeviceToHost));
        uint64_t* h = static_cast<uint64_t*>(host);
        for (int64_t v0 = 0; v0 < nl; v0 += blk) {
          const int64_t k = std::min(blk, nl - v0);
          const size_t kb = (size_t)(k * W * 8);
          GP_TRY(copy_sync(c, h + v0 * W, c->d_slot[0] + v0 * W, kb, hipMemcpyDeviceToHost));
          GP_TRY(copy_sync(c, s1.data(), c->d_slot[1] + v0 * W, kb, hipMemcpyDeviceToHost));
          if (c->d_slot[2]) GP_TRY(copy_sync(c, s2.data(), c->d_slot[2] + v0 * W, kb, hipMemcpyDeviceToHost));
          for (int64_t v = v0; v < v0 + k; ++v) {
            const uint8_t p = sp[(size_t)v];
            const int64_t o = (v - v0) * W;
            if (p == SLOT_NONE) std::memset(h + v * W, 0, (size_t)W * 8);
            else if (p == 1) std::memcpy(h + v * W, s1.data() + o, (size_t)W * 8);
            else if (p == SLOT_PARKED && !s2.empty()) std::memcpy(h + v * W, s2.data() + o, (size_t)W * 8);
          }
        }
      }
      return 0;
    case GP_FIRST:
      if (!run) return set_error(GP_ESTATE, "no run state");
      if (!c->d_first || !c->cfg.track_first) return set_error(GP_ENOTRACK, "track_first is off");
      GP_TRY(need(nl * M));
      if (bytes)
        GP_HIP(hipMemcpy2D(host, (size_t)M, c->d_first, (size_t)W * 64, (size_t)M, (size_t)nl,
                           hipMemcpyDeviceToHost));
      return 0;
    case GP_DIGEST:
      if (!run) return set_error(GP_ESTATE, "no run state");
      if (!c->cfg.track_digest) return set_error(GP_ENOTRACK, "track_digest is off");
      GP_TRY(need(nl * 8));
      if (bytes) GP_TRY(copy_sync(c, host, c->d_digest, (size_t)bytes, hipMemcpyDeviceToHost));
      return 0;
    case GP_COVERAGE:
    case GP_FORWARDS: {
      if (!run) return set_error(GP_ESTATE, "no run state");
      if (what == GP_FORWARDS && !c->msg_forwards_valid && c->liveness_active)
        return set_error(GP_ENOTRACK, "churn run without track_msg_forwards");
      GP_TRY(need(M * 8));
      const size_t MM = (size_t)W * 64;
      const u64* src = c->d_msg_cov + (what == GP_COVERAGE ? 2 * MM : 3 * MM);
      GP_TRY(copy_sync(c, host, src, (size_t)bytes, hipMemcpyDeviceToHost));
      return 0;
    }
    case GP_STATE:
    case GP_MISS:
      if (!run) return set_error(GP_ESTATE, "no run state");
      GP_TRY(need(n));
      GP_TRY(copy_sync(c, host, what == GP_STATE ? c->d_state : c->d_miss, (size_t)n, hipMemcpyDeviceToHost));
      if (what == GP_STATE)   // (the removal flag and the sated mark are engine bookkeeping)
        for (int64_t v = 0; v < n; ++v) static_cast<uint8_t*>(host)[v] &= (uint8_t)~(ST_RMNEW | ST_SATED);
      return 0;
    case GP_DEG_LIVE:
      if (!run) return set_error(GP_ESTATE, "no run state");
      GP_TRY(need(n * 4));
      GP_TRY(copy_sync(c, host, c->d_deg_live, (size_t)bytes, hipMemcpyDeviceToHost));
      return 0;
    case GP_ROW_PTR:   // partitioned: the local CSR over all local slots
      if (c->n <= 0) return set_error(GP_ESTATE, "no graph");
      GP_TRY(need((c->n_alloc + 1) * 8));
      GP_TRY(copy_sync(c, host, c->d_row_ptr, (size_t)bytes, hipMemcpyDeviceToHost));
      return 0;
    case GP_COL:
      if (c->n <= 0) return set_error(GP_ESTATE, "no graph");
      GP_TRY(need(c->nnz_l * 4));
      if (bytes) GP_TRY(copy_sync(c, host, c->d_col, (size_t)bytes, hipMemcpyDeviceToHost));
      return 0;
    case GP_L2G:   // global id of every local slot
      if (c->n <= 0) return set_error(GP_ESTATE, "no graph");
      GP_TRY(need(c->n_alloc * 4));
      if (c->local) {
        GP_TRY(copy_sync(c, host, c->d_l2g, (size_t)bytes, hipMemcpyDeviceToHost));
      } else {
        for (int64_t v = 0; v < c->n; ++v) static_cast<int32_t*>(host)[v] = (int32_t)v;
      }
      return 0;
    case GP_JOB_DIGEST:
    case GP_JOB_COVERAGE:
    case GP_JOB_FORWARDS: {   // the job record of gp_shard_combine (shard.hip)
      if (!c->j_ready) return set_error(GP_ESTATE, "gp_shard_combine first");
      if (what == GP_JOB_DIGEST) {
        if (!c->j_dig_valid) return set_error(GP_ENOTRACK, "track_digest is off");
        GP_TRY(need(c->n * 8));
        GP_TRY(copy_sync(c, host, c->d_jdig, (size_t)bytes, hipMemcpyDeviceToHost));
        return 0;
      }
      if (what == GP_JOB_FORWARDS && !c->j_fwd_valid)
        return set_error(GP_ENOTRACK, "churn run without track_msg_forwards (on some rank)");
      GP_TRY(need((int64_t)c->jm * 8));
      GP_TRY(copy_sync(c, host, c->d_jcf + (what == GP_JOB_COVERAGE ? 0 : (size_t)c->jm), (size_t)bytes,
                       hipMemcpyDeviceToHost));
      return 0;
    }
#ifdef GP_DBG_READ   // scripts/debug_mask2.py: arc mask, gather-order columns, activity bits
    case 100:
      GP_TRY(copy_sync(c, host, c->d_amask, (size_t)bytes, hipMemcpyDeviceToHost));
      return 0;
    case 101:
      GP_TRY(copy_sync(c, host, c->d_gcol, (size_t)bytes, hipMemcpyDeviceToHost));
      return 0;
    case 102:
      GP_TRY(copy_sync(c, host, c->d_abits, (size_t)bytes, hipMemcpyDeviceToHost));
      return 0;
#endif
    case GP_FPOP:
      if (!run) return set_error(GP_ESTATE, "no run state");
      GP_TRY(need(n * 4));
      GP_TRY(copy_sync(c, host, c->d_fpop[c->cur], (size_t)bytes, hipMemcpyDeviceToHost));
      return 0;
    case GP_FRONTIER: {
      if (!run) return set_error(GP_ESTATE, "no run state");
      // exact frontier rows exist only with track_msg_forwards: the pull reads
      // whole Message-Lists
      if (!c->cfg.track_msg_forwards) return set_error(GP_ENOTRACK, "frontier rows are kept only with track_msg_forwards");
      GP_TRY(need(n * W * 8));
      std::vector<uint32_t> fp((size_t)n);
      GP_TRY(copy_sync(c, fp.data(), c->d_fpop[c->cur], (size_t)n * 4, hipMemcpyDeviceToHost));
      GP_TRY(copy_sync(c, host, c->d_frx[c->cur], (size_t)bytes, hipMemcpyDeviceToHost));
      uint64_t* h = static_cast<uint64_t*>(host);
      for (int64_t v = 0; v < n; ++v)
        if (!fp[v]) std::memset(h + v * W, 0, (size_t)W * 8);
      return 0;
    }
    default:
      return set_error(GP_EINVAL, "unknown gp_what");
  }
}

int gp_reports(gp_ctx* c, gp_report* buf, int64_t cap, int64_t* n_out) {
  if (!c || !n_out || (cap > 0 && !buf)) return set_error(GP_EINVAL, "null argument");
  GP_HIP(hipSetDevice(c->device));
  const int64_t total = c->last_reports;
  *n_out = total;
  const int64_t k = std::min(std::min(total, cap), c->report_cap);
  if (k > 0) GP_TRY(copy_sync(c, buf, c->d_reports, (size_t)k * sizeof(gp_report), hipMemcpyDeviceToHost));
  return 0;
}

int gp_synchronize(gp_ctx* c) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  GP_HIP(hipSetDevice(c->device));
  GP_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

int gp_info(gp_ctx* c, int64_t* n, int64_t* nnz, int32_t* m, int32_t* words) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  if (n) *n = c->n;
  if (nnz) *nnz = c->nnz;
  if (m) *m = c->m;
  if (words) *words = c->words;
  return 0;
}

int gp_local_info(gp_ctx* c, int64_t* nloc, int64_t* nghost, int64_t* nextra, int64_t* nnz_local,
                  int64_t* n_boundary) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  if (nloc) *nloc = c->nloc();
  if (nghost) *nghost = c->nghost;
  if (nextra) *nextra = c->nextra;
  if (nnz_local) *nnz_local = c->nnz_l;
  if (n_boundary) *n_boundary = c->n_bnd;
  return 0;
}

}  // extern "C"
