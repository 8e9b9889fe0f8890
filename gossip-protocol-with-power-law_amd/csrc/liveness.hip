// liveness.hip -- L_r of DESIGN.md §2.2 / §3.5: crash draws, heartbeat-miss
// counters, 3-miss detection with one dead-node report per live link, and the
// seed's removal of a reported vertex (Peer.py:298-393, Seed.py:358-406).
#include <cmath>

#include "gp_device.h"

namespace gp {

// ---------------------------------------------------------------------------
// liveness (L_r).  Replicated on every rank (deterministic), counters and
// reports only for owned vertices.
struct LiveArgs {
  uint8_t* __restrict__ state;
  uint8_t* __restrict__ miss;
  uint32_t* __restrict__ fpop;       // frontier_r popcount: zeroed on crash
  int32_t* __restrict__ cand;
  int32_t* __restrict__ deg_live;
  const int64_t* __restrict__ row_ptr;
  const int32_t* __restrict__ col;
  const int64_t* __restrict__ out_row_ptr;   // directed only
  const int32_t* __restrict__ out_col;
  gp_report* __restrict__ reports;
  u64* __restrict__ stats;           // direct counters (cursor, cand)
  int32_t* __restrict__ det_big;     // [DET_CAP] deferred detection candidates (null: none deferred)
  int64_t* __restrict__ det_pre;     // [DET_CAP + 1] prefix of their link counts
  uint32_t* __restrict__ det_live;   // [DET_CAP] live reporters
  uint32_t* __restrict__ det_cur;    // [DET_CAP] reports written
  u64* __restrict__ det_base;        // [DET_CAP] first report slot (~0: none)
  u64* __restrict__ partial;
  const int32_t* __restrict__ l2g;   // global id of a local vertex (partitioned; null: identity)
  uint8_t* __restrict__ lm;          // line masks the last round's commits wrote for this round's
                                     //   pull (two vertices per byte; null: none): a crash zeroes the
                                     //   crashed vertex's nibble, as it zeroes its fpop
  int64_t n, vbegin, vend;           // local vertex slots, owned local range
  int64_t report_cap;
  u64 crash_key;
  u64 p_thresh;                      // crash iff draw < p_thresh
  int32_t p_always;                  // p_fail >= 1
  int32_t miss_thr;
  int32_t r;
};

// Four vertices per lane: state and miss bytes move as 32-bit words (a wave
// covers 256 vertices per instruction) and are stored only when they change.
// Detection candidates (~1 % of n every round under C5 churn) collect in an
// LDS list per block and reach the global list with one cursor add per block:
// a same-address add per candidate, or per wave, serialised k_churn at
// 4.7-5.9 ms per round on C5 (~0.5 M adds at ~12 ns).
constexpr int CHURN_CAND_LDS = 2048;
__global__ __launch_bounds__(BLOCK) void k_churn(LiveArgs a) {
  __shared__ int32_t s_cand[CHURN_CAND_LDS];
  __shared__ uint32_t s_ncand;
  __shared__ u64 s_base;
  WaveStats st;
  ws_zero(st);
  if (threadIdx.x == 0) s_ncand = 0u;
  __syncthreads();
  u64 ncrash = 0;
  const int64_t nw = (a.n + 3) >> 2;
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t w0 = (int64_t)blockIdx.x * BLOCK; w0 < nw; w0 += stride) {
    const int64_t w = w0 + threadIdx.x;
    const int64_t v0 = w << 2;
    const bool full = v0 + 4 <= a.n;
    uint32_t cand = 0;   // bit q: vertex v0 + q reached the miss threshold
    if (w < nw) {
      uint32_t sw = 0;
      if (full) {
        sw = reinterpret_cast<const uint32_t*>(a.state)[w];
      } else {
        for (int q = 0; q < 4; ++q)
          if (v0 + q < a.n) sw |= (uint32_t)a.state[v0 + q] << (8 * q);
      }
      uint32_t nsw = sw;
      bool anyc = false;
      uint32_t crashed_now = 0;   // bit q: vertex v0 + q crashes this round
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t v = v0 + q;
        uint8_t s = (uint8_t)(sw >> (8 * q)) & (uint8_t)~ST_RMNEW;   // last round's removal flag is sent
        if (v < a.n && !(s & ST_DOWN)) {
          bool crash = (s & ST_PENDING) != 0;
          // draws by global id: every rank holding v takes the same decision
          if (!crash && (a.p_always || a.p_thresh))
            crash = a.p_always || draw(a.crash_key, (u64)(a.l2g ? a.l2g[v] : (int32_t)v)) < a.p_thresh;
          if (crash) {
            s = (uint8_t)((s | ST_CRASHED) & ~ST_PENDING);
            a.fpop[v] = 0;   // crash-stop: its frontier is never sent
            crashed_now |= 1u << q;
            if (v >= a.vbegin && v < a.vend) ncrash += 1;
          }
        }
        anyc |= (s & ST_CRASHED) != 0;
        nsw = (nsw & ~(0xFFu << (8 * q))) | ((uint32_t)s << (8 * q));
      }
      if (anyc) {   // heartbeat misses of the crashed vertices
        uint32_t mw = 0;
        if (full) {
          mw = reinterpret_cast<const uint32_t*>(a.miss)[w];
        } else {
          for (int q = 0; q < 4; ++q)
            if (v0 + q < a.n) mw |= (uint32_t)a.miss[v0 + q] << (8 * q);
        }
        uint32_t nmw = mw;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint8_t s = (uint8_t)(nsw >> (8 * q));
          if (!(s & ST_CRASHED)) continue;
          uint32_t mi = (mw >> (8 * q)) & 0xFFu;
          if (mi < 255) ++mi;
          nmw = (nmw & ~(0xFFu << (8 * q))) | (mi << (8 * q));
          if ((int)mi == a.miss_thr && !(s & ST_REMOVED)) cand |= 1u << q;
        }
        if (nmw != mw) {
          if (full) {
            reinterpret_cast<uint32_t*>(a.miss)[w] = nmw;
          } else {
            for (int q = 0; q < 4; ++q)
              if (v0 + q < a.n) a.miss[v0 + q] = (uint8_t)(nmw >> (8 * q));
          }
        }
      }
      if (crashed_now && a.lm) {   // this lane's 4 vertices are the 2 bytes at v0 / 2 (v0 % 4 == 0)
        uint32_t keep = 0xFFFFu;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if ((crashed_now >> q) & 1u) keep &= ~(0xFu << (4 * q));
        if (full) {
          uint16_t* p = reinterpret_cast<uint16_t*>(a.lm) + (v0 >> 2);
          *p = (uint16_t)(*p & keep);
        } else {
          for (int q = 0; q < 4; ++q)
            if (v0 + q < a.n && ((crashed_now >> q) & 1u)) a.lm[(v0 + q) >> 1] &= (uint8_t)((q & 1) ? 0x0Fu : 0xF0u);
        }
      }
      if (nsw != sw) {
        if (full) {
          reinterpret_cast<uint32_t*>(a.state)[w] = nsw;
        } else {
          for (int q = 0; q < 4; ++q)
            if (v0 + q < a.n) a.state[v0 + q] = (uint8_t)(nsw >> (8 * q));
        }
      }
    }
    for (int q = 0; q < 4; ++q) {
      if (!((cand >> q) & 1u)) continue;
      const uint32_t k = atomicAdd(&s_ncand, 1u);
      if (k < (uint32_t)CHURN_CAND_LDS) {
        s_cand[k] = (int32_t)(v0 + q);
      } else {   // list full (p_fail near 1): straight to the global list
        const u64 slot = atomicAdd(&a.stats[S_CAND], 1ull);
        a.cand[slot] = (int32_t)(v0 + q);
      }
    }
  }
  __syncthreads();
  const uint32_t nl = min(s_ncand, (uint32_t)CHURN_CAND_LDS);
  if (threadIdx.x == 0 && nl) s_base = atomicAdd(&a.stats[S_CAND], (u64)nl);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < nl; k += BLOCK) a.cand[s_base + k] = s_cand[k];
  // crash counts differ per lane: wave-reduce, then one uniform add
  u64 c = ncrash;
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) c += __shfl_xor(c, s);
  st.add(S_CRASHED, c);
  flush_stats(st, a.partial);
}

// One wave per 64 detection candidates.  Pass 1 counts each candidate's live
// reporters (one per heartbeat link), kept by lane c for candidate c; one
// cursor add reserves the report slots of the wave's owned candidates (a
// same-address add per candidate serialised k_detect at 8.5 ms on C5, ~0.65 M
// candidates a round).  Pass 2 removes every reported candidate (replicated
// state) and writes the owned ones' reports.  Candidates are crashed, hence
// down, so removals in one wave never change another wave's counts.
// The wave's 64 candidates' heartbeat links (in-list then, directed,
// out-list of each candidate) are walked as one flat sequence (offsets f[c]
// from a wave scan of the degrees), DET_U chunks of 64 links in flight per
// lane.  Live reporters are counted with LDS adds per candidate; pass 2 takes
// report slots from a per-candidate LDS cursor (reports are a set per round:
// their order inside a candidate is not part of the result).  Candidates with
// more than DET_BIG links are deferred to the k_det_big_* kernels, which
// spread each one's links over the whole grid: walked inside one wave, a
// crashed hub (10^4-10^5 links at 2^26) kept k_detect at 2.2-2.4 ms a round
// (C5), 0.5 ms without them.
constexpr int DET_U = 4;
constexpr int64_t DET_BIG = 2048;   // links above which a candidate is deferred
struct DetectLds {
  int64_t f[65];      // flat offset of candidate c's first link; f[cnt] = total
  int64_t b[64];      // row_ptr[v]
  int64_t ob[64];     // out_row_ptr[v] (directed)
  int32_t din[64];    // in-degree
  int32_t v[64];      // the candidate
  uint32_t live[64];  // pass 1: live reporters; pass 2: same (0: not removed)
  uint32_t rk[64];    // pass 2: reports written so far
  uint64_t slot[64];  // pass 2: first report slot (owned, removed candidates; ~0: none)
};

// candidate owning flat link t: the largest c < cnt with f[c] <= t
__device__ __forceinline__ int det_owner(const DetectLds& L, int cnt, int64_t t) {
  int c = 0;
#pragma unroll
  for (int s = 32; s > 0; s >>= 1)
    if (c + s < cnt && L.f[c + s] <= t) c += s;
  return c;
}

__global__ __launch_bounds__(BLOCK) void k_detect(LiveArgs a) {
  __shared__ DetectLds s_det[WAVES];
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  DetectLds& L = s_det[wib];
  WaveStats st;
  ws_zero(st);
  const int64_t ncand = (int64_t)a.stats[S_CAND];
  const int64_t stride = (int64_t)gridDim.x * WAVES * 64;
  for (int64_t k0 = ((int64_t)blockIdx.x * WAVES + wib) * 64; k0 < ncand; k0 += stride) {
    const int cnt = (int)min((int64_t)64, ncand - k0);
    const int vme = lane < cnt ? a.cand[k0 + lane] : -1;
    int64_t deg = 0;
    bool vme_deferred = false;
    if (vme >= 0) {
      const int64_t b = a.row_ptr[vme], e = a.row_ptr[vme + 1];
      int64_t ob = 0, oe = 0;
      if (a.out_row_ptr) {
        ob = a.out_row_ptr[vme];
        oe = a.out_row_ptr[vme + 1];
      }
      L.b[lane] = b;
      L.ob[lane] = ob;
      L.v[lane] = vme;
      L.din[lane] = (int32_t)(e - b);
      deg = (e - b) + (oe - ob);
      if (deg > DET_BIG && a.det_big) {
        const u64 k = atomicAdd(&a.stats[S_DET_BIG], 1ull);
        if (k < (u64)DET_CAP) {   // deferred: no links here, no stats, no reports
          a.det_big[k] = vme;
          deg = 0;
          L.din[lane] = 0;
          vme_deferred = true;
        }
      }
    }
    L.live[lane] = 0u;
    // 64-bit exclusive scan of the degrees
    int64_t inc = deg;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    L.f[lane] = inc - deg;
    const int64_t T = __shfl(inc, 63);
    if (lane == 63) L.f[64] = T;
    wave_sync_lds();
    // pass 1: live reporters per candidate
    for (int64_t t0 = 0; t0 < T; t0 += 64 * DET_U) {
      int32_t u[DET_U];
      int cq[DET_U];
#pragma unroll
      for (int q = 0; q < DET_U; ++q) {
        const int64_t t = t0 + q * 64 + lane;
        u[q] = -1;
        cq[q] = 0;
        if (t < T) {
          const int c = det_owner(L, cnt, t);
          const int64_t j = t - L.f[c];
          cq[q] = c;
          u[q] = j < L.din[c] ? a.col[L.b[c] + j] : a.out_col[L.ob[c] + (j - L.din[c])];
        }
      }
      uint32_t sb[DET_U];
#pragma unroll
      for (int q = 0; q < DET_U; ++q) sb[q] = u[q] >= 0 ? a.state[u[q]] : (uint32_t)ST_DOWN;
#pragma unroll
      for (int q = 0; q < DET_U; ++q)
        if (!(sb[q] & ST_DOWN)) atomicAdd(&L.live[cq[q]], 1u);
    }
    wave_sync_lds();
    const uint32_t tot_me = lane < cnt && !vme_deferred ? L.live[lane] : 0u;
    const bool own = vme >= 0 && vme >= a.vbegin && vme < a.vend;
    const uint32_t emit = own ? tot_me : 0u;   // nobody holds a link to it (0): never reported
    const uint32_t excl = wave_excl_scan_u32(emit, lane);
    const uint32_t total = (uint32_t)__shfl((int)(excl + emit), 63);
    u64 base = 0;
    if (total) {
      if (lane == 0) base = atomicAdd(&a.stats[S_REPORT_CURSOR], (u64)total);
      base = __shfl(base, 0);
    }
    st.add(S_REPORTS, wave_sum_u64(emit));
    st.add(S_REMOVALS, (u64)__popcll(__ballot(emit != 0u)));
    st.add(S_DUP, wave_sum_u64(emit ? emit - 1u : 0u));
    // (partitioned: a ghost is removed here when an owned neighbour is live --
    // then its owner removes it too; otherwise the owner's flag comes with the
    // boundary exchange, partition.hip)
    if (tot_me) a.state[vme] |= (uint8_t)(ST_REMOVED | (own ? ST_RMNEW : 0));
    L.live[lane] = tot_me;
    L.rk[lane] = 0u;
    L.slot[lane] = emit ? base + excl : ~0ull;
    if (!__any(tot_me != 0u)) continue;
    wave_sync_lds();
    // pass 2: live-degree updates of removed candidates' in-neighbours, reports
    for (int64_t t0 = 0; t0 < T; t0 += 64 * DET_U) {
      int32_t u[DET_U];
      int cq[DET_U];
      bool in[DET_U];
#pragma unroll
      for (int q = 0; q < DET_U; ++q) {
        const int64_t t = t0 + q * 64 + lane;
        u[q] = -1;
        cq[q] = 0;
        in[q] = false;
        if (t < T) {
          const int c = det_owner(L, cnt, t);
          if (L.live[c]) {
            const int64_t j = t - L.f[c];
            cq[q] = c;
            in[q] = j < L.din[c];
            u[q] = in[q] ? a.col[L.b[c] + j] : a.out_col[L.ob[c] + (j - L.din[c])];
          }
        }
      }
      uint32_t sb[DET_U];
#pragma unroll
      for (int q = 0; q < DET_U; ++q) {
        sb[q] = (uint32_t)ST_DOWN;
        if (u[q] >= 0) {
          if (in[q]) atomicSub(&a.deg_live[u[q]], 1);
          if (L.slot[cq[q]] != ~0ull) sb[q] = a.state[u[q]];
        }
      }
#pragma unroll
      for (int q = 0; q < DET_U; ++q) {
        if (!(sb[q] & ST_DOWN)) {
          const int c = cq[q];
          const u64 slot = L.slot[c] + (u64)atomicAdd(&L.rk[c], 1u);
          if ((int64_t)slot < a.report_cap) {
            const int v = L.v[c];
            a.reports[slot] = a.l2g ? gp_report{a.l2g[v], a.l2g[u[q]], a.r} : gp_report{v, u[q], a.r};
          }
        }
      }
    }
  }
  flush_stats(st, a.partial);
}

// Deferred (big) candidates: their links form one flat sequence over the
// list, g in [0, pre[nb]), walked grid-stride by every thread of the grid.
// Per-candidate sums are combined per run of equal k inside a wave (one
// global add per run), so a hub's links do not serialise on one address.
__device__ __forceinline__ int det_big_n(const LiveArgs& a) {
  return (int)min(a.stats[S_DET_BIG], (u64)DET_CAP);
}
// the deferred candidate owning flat link g: the largest k < nb with pre[k] <= g
__device__ __forceinline__ int det_big_owner(const int64_t* __restrict__ pre, int nb, int64_t g) {
  int lo = 0, hi = nb;   // pre[lo] <= g < pre[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (pre[mid] <= g) lo = mid;
    else hi = mid;
  }
  return lo;
}
// link j of candidate v: in-list first, then (directed) out-list
__device__ __forceinline__ int32_t det_link(const LiveArgs& a, int v, int64_t j, bool& in) {
  const int64_t b = a.row_ptr[v], din = a.row_ptr[v + 1] - b;
  in = j < din;
  return in ? a.col[b + j] : a.out_col[a.out_row_ptr[v] + (j - din)];
}
// first lane of this lane's run of equal k, and the last
__device__ __forceinline__ void det_run(int k, int lane, int& first, int& last) {
  const int kp = __shfl_up(k, 1), kn = __shfl_down(k, 1);
  const u64 heads = __ballot(lane == 0 || kp != k), tails = __ballot(lane == 63 || kn != k);
  const u64 le = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1ull);
  first = 63 - __clzll((long long)(heads & le));
  last = __ffsll((long long)(tails & ~((1ull << lane) - 1ull))) - 1;
}

// one block: prefix of the deferred candidates' link counts, counters zeroed
__global__ __launch_bounds__(1024) void k_det_big_scan(LiveArgs a) {
  __shared__ int64_t s_part[1024];
  const int nb = det_big_n(a);
  const int t = threadIdx.x;
  const int per = (nb + 1023) / 1024;
  int64_t sum = 0;
  for (int q = 0; q < per; ++q) {
    const int k = t * per + q;
    if (k < nb) {
      const int v = a.det_big[k];
      int64_t d = a.row_ptr[v + 1] - a.row_ptr[v];
      if (a.out_row_ptr) d += a.out_row_ptr[v + 1] - a.out_row_ptr[v];
      sum += d;
      a.det_live[k] = 0u;
      a.det_cur[k] = 0u;
    }
  }
  s_part[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {   // inclusive scan of the per-thread sums
    const int64_t y = t >= o ? s_part[t - o] : 0;
    __syncthreads();
    s_part[t] += y;
    __syncthreads();
  }
  int64_t run = s_part[t] - sum;
  for (int q = 0; q < per; ++q) {
    const int k = t * per + q;
    if (k < nb) {
      a.det_pre[k] = run;
      const int v = a.det_big[k];
      int64_t d = a.row_ptr[v + 1] - a.row_ptr[v];
      if (a.out_row_ptr) d += a.out_row_ptr[v + 1] - a.out_row_ptr[v];
      run += d;
    }
  }
  if (t == 1023) a.det_pre[nb] = s_part[1023];
}

// pass 1: live reporters per deferred candidate
__global__ __launch_bounds__(BLOCK) void k_det_big_count(LiveArgs a) {
  const int nb = det_big_n(a);
  if (nb == 0) return;
  const int lane = threadIdx.x & 63;
  const int64_t total = a.det_pre[nb];
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t g0 = (int64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63); g0 < total; g0 += stride) {
    const int64_t g = g0 + lane;
    int k = nb;   // past the end: its own run, adds nothing
    bool live = false;
    if (g < total) {
      k = det_big_owner(a.det_pre, nb, g);
      bool in;
      const int32_t u = det_link(a, a.det_big[k], g - a.det_pre[k], in);
      live = !(a.state[u] & ST_DOWN);
    }
    const u64 m = __ballot(live);
    int first, last;
    det_run(k, lane, first, last);
    if (lane == last && k < nb) {
      const u64 run = (last == 63 ? ~0ull : ((1ull << (last + 1)) - 1ull)) & ~((1ull << first) - 1ull);
      const uint32_t c = (uint32_t)__popcll(m & run);
      if (c) atomicAdd(&a.det_live[k], c);
    }
  }
}

// removal flags, report slots and stats of the deferred candidates
__global__ __launch_bounds__(BLOCK) void k_det_big_reserve(LiveArgs a) {
  WaveStats st;
  ws_zero(st);
  const int nb = det_big_n(a);
  for (int k0 = (int)blockIdx.x * BLOCK + (threadIdx.x & ~63); k0 < nb; k0 += (int)gridDim.x * BLOCK) {
    const int k = k0 + (threadIdx.x & 63);
    uint32_t emit = 0;
    if (k < nb) {
      const int v = a.det_big[k];
      const uint32_t tot = a.det_live[k];
      const bool own = v >= a.vbegin && v < a.vend;
      if (tot) a.state[v] |= (uint8_t)(ST_REMOVED | (own ? ST_RMNEW : 0));
      emit = own ? tot : 0u;
      a.det_base[k] = emit ? atomicAdd(&a.stats[S_REPORT_CURSOR], (u64)emit) : ~0ull;
    }
    st.add(S_REPORTS, wave_sum_u64(emit));
    st.add(S_REMOVALS, (u64)__popcll(__ballot(emit != 0u)));
    st.add(S_DUP, wave_sum_u64(emit ? emit - 1u : 0u));
  }
  flush_stats(st, a.partial);
}

// pass 2: live-degree updates of removed deferred candidates' in-neighbours,
// reports of the owned ones
__global__ __launch_bounds__(BLOCK) void k_det_big_write(LiveArgs a) {
  const int nb = det_big_n(a);
  if (nb == 0) return;
  const int lane = threadIdx.x & 63;
  const int64_t total = a.det_pre[nb];
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t g0 = (int64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63); g0 < total; g0 += stride) {
    const int64_t g = g0 + lane;
    int k = nb;
    bool rep = false;
    int v = -1;
    int32_t u = -1;
    if (g < total) {
      k = det_big_owner(a.det_pre, nb, g);
      if (a.det_live[k]) {
        v = a.det_big[k];
        bool in;
        u = det_link(a, v, g - a.det_pre[k], in);
        if (in) atomicSub(&a.deg_live[u], 1);
        rep = a.det_base[k] != ~0ull && !(a.state[u] & ST_DOWN);
      }
    }
    const u64 m = __ballot(rep);
    int first, last;
    det_run(k, lane, first, last);
    const u64 run = (last == 63 ? ~0ull : ((1ull << (last + 1)) - 1ull)) & ~((1ull << first) - 1ull);
    u64 rb = 0;
    if (lane == last && k < nb && (m & run)) rb = (u64)atomicAdd(&a.det_cur[k], (uint32_t)__popcll(m & run));
    rb = (u64)__shfl((long long)rb, last);
    if (rep) {
      const u64 slot = a.det_base[k] + rb + (u64)__popcll(m & run & ((1ull << lane) - 1ull));
      if ((int64_t)slot < a.report_cap)
        a.reports[slot] = a.l2g ? gp_report{a.l2g[v], a.l2g[u], a.r} : gp_report{v, u, a.r};
    }
  }
}


int launch_liveness(Ctx* c) {
  hipStream_t s = c->stream;
  u64* stats = c->d_stats;
  u64* partial = c->d_stats + 64;
  const int r = c->round;
  LiveArgs la{};
  la.state = c->d_state;
  la.miss = c->d_miss;
  la.fpop = c->d_fpop[c->cur];
  la.cand = c->d_cand;
  la.deg_live = c->d_deg_live;
  la.row_ptr = c->d_row_ptr;
  la.col = c->d_col;
  la.out_row_ptr = c->directed ? c->d_out_row_ptr : nullptr;
  la.out_col = c->directed ? c->d_out_col : nullptr;
  la.reports = c->d_reports;
  la.stats = stats;
  la.partial = partial;
  la.l2g = c->local ? c->d_l2g : nullptr;
  la.lm = c->lm_written_prev ? c->d_lmw[c->cur] : nullptr;
  la.n = c->n_alloc;
  la.vbegin = 0;
  la.vend = c->nloc();
  la.report_cap = c->report_cap;
  la.crash_key = stream_key(c->cfg.churn_seed, STREAM_CRASH + (uint64_t)r);
  const double p = c->cfg.churn ? c->cfg.p_fail : 0.0;
  la.p_always = p >= 1.0;
  la.p_thresh = (p > 0.0 && p < 1.0) ? (uint64_t)std::ldexp(p, 64) : 0ull;
  la.miss_thr = c->cfg.miss_threshold;
  la.r = r;
  hipLaunchKernelGGL(k_churn, dim3(std::min(grid_for(c->n_alloc, BLOCK), c->cu_count * 8 * GS)), dim3(BLOCK), 0, s, la);
  la.det_big = c->d_det_big;
  la.det_pre = c->d_det_pre;
  la.det_live = c->d_det_live;
  la.det_cur = c->d_det_cur;
  la.det_base = c->d_det_base;
  hipLaunchKernelGGL(k_detect, dim3(c->cu_count * GP_DETECT_BLOCKS_PER_CU * GS), dim3(BLOCK), 0, s, la);
  if (la.det_big) {
    hipLaunchKernelGGL(k_det_big_scan, dim3(1), dim3(1024), 0, s, la);
    hipLaunchKernelGGL(k_det_big_count, dim3(c->cu_count * 4 * GS), dim3(BLOCK), 0, s, la);
    hipLaunchKernelGGL(k_det_big_reserve, dim3(DET_CAP / BLOCK), dim3(BLOCK), 0, s, la);
    hipLaunchKernelGGL(k_det_big_write, dim3(c->cu_count * 4 * GS), dim3(BLOCK), 0, s, la);
  }
  GP_HIP(hipGetLastError());
  c->pending_crash = false;
  return 0;
}

}  // namespace gp
