// pull.hip -- the pull expansion E_r of DESIGN.md §3.2-3.4: next[v] = OR over
// v's in-neighbours u of frontier[u] & ~seen[v] (the send loop of Peer.py:402-404,
// the receive side of Peer.py:175-216), with forward-once and Message-List
// dedup.  k_expand (a wave per 64 receivers, one receiver at a time, W >= 32),
// k_expand_flat (edge-parallel, narrow rows), k_expand_rec (compact
// Message-Lists), the per-round helpers of the pull (line masks, per-arc mask,
// row fix-up, parking) and the launch of a whole expansion round.
#include "gp_device.h"

namespace gp {

// Receivers two at a time, one per half-wave (W = 64).  A half-wave loads a
// whole 64-word row per instruction, so each receiver keeps its rows in flight
// on its own and the dependent chain (column ids -> probes -> rows -> commit)
// is walked for two receivers at once: the latency-bound rounds' lever, since
// 64 VGPRs already give the 8 waves per SIMD the hardware holds.  Same
// commits as finish_row (deferred per-vertex words in L.tot / L.dig / L.cd).
// rows in flight per half-wave in pre_pairs: 2 (70 VGPRs, 7 waves per SIMD)
// against 4 (78, 6 waves): C4 round 1 3.97 -> 3.78 ms same-box
#ifndef GP_PAIR_RIF
#define GP_PAIR_RIF 2
#endif

// receiver side of a pair: half h holds receiver ks (on: the half has one;
// kB < 0: half 1 idle) with its gathered OR acc and its seen row sv
// (alias: both receivers complete their component -- done in-neighbours in an
// a.alias round -- and commit SLOT_CMASK instead of a row, finish_row)
template <int W, class LDS>
__device__ __forceinline__ void pair_finish(const ExpandArgs& a, LDS& L, int h, int lw, bool on, int ks, int kB,
                                            int64_t i, int v, u64x2 acc, u64x2 sv, WaveStats& st,
                                            bool alias = false) {
  const u64x2 nw = acc & ~sv;
  uint32_t tot = (uint32_t)(__popcll(nw.x) + __popcll(nw.y));
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) tot += (uint32_t)__shfl_xor((int)tot, o);
  u64 t = 0;
  bool dense = true;   // record of the new Message-List (record-writing rounds)
  if constexpr (LDS::kCml) {
    if (a.cml_next) {
      const u64x2 row = sv | nw;
      const u64 bx = __ballot(row.x != 0ull), by = __ballot(row.y != 0ull);
      const u64 msk = spread32((bx >> (32 * h)) & 0xFFFFFFFFull) | (spread32((by >> (32 * h)) & 0xFFFFFFFFull) << 1);
      dense = __popcll(msk) > CML_MAXW;
      if (!dense && on && tot) {
        u64* rec = a.cml_next + (size_t)v * CML_WORDS;
        const int p = 1 + __popcll(msk & ((1ull << (2 * lw)) - 1ull));
        if (row.x) rec[p] = row.x;
        if (row.y) rec[p + (row.x ? 1 : 0)] = row.y;
        if (lw == 0) rec[0] = msk;
      }
    }
  }
  if (on && tot) {
    alive_add<W>(a, L, lw, nw);
    if (!alias) store_piece<W>(a.slot[a.wslot], v, lw, sv | nw);
    if (a.frx_next) store_piece<W>(a.frx_next, v, lw, nw);
    if (a.first) {
      uint8_t* row = a.first + (size_t)i * (W * 64);
      if (nw.x) set_first_bytes(row, 2 * lw, nw.x, (uint32_t)a.rr);
      if (nw.y) set_first_bytes(row, 2 * lw + 1, nw.y, (uint32_t)a.rr);
    }
    if (a.digest) {
      if (nw.x) t ^= digest_term((uint32_t)a.rr, (uint32_t)(a.wbase + 2 * lw), nw.x);
      if (nw.y) t ^= digest_term((uint32_t)a.rr, (uint32_t)(a.wbase + 2 * lw + 1), nw.y);
    }
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) t ^= __shfl_xor(t, o);
  uint32_t lmn = 0;   // lines of the new bits holding a nonzero word (lm_next; finish_row)
  if (a.lm_next) lmn = lines_of((uint32_t)(__ballot(on && (nw.x | nw.y) != 0ull) >> (32 * h)));
  if (lw == 0 && on && tot) {
    L.tot[ks] = tot;
    L.lmn[ks] = (uint8_t)lmn | (alias ? LMN_ALIAS : (uint8_t)0);
    L.dig[ks] = t;
    if constexpr (LDS::kCml) L.cd[ks] = dense ? 1 : 0;
  }
  const uint32_t tA = (uint32_t)__builtin_amdgcn_readlane((int)tot, 0);
  const uint32_t tB = kB >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)tot, 32) : 0u;
  st.add(S_NEW_BITS, (u64)tA + (u64)tB);
  st.add(S_RECEIVERS, (u64)((tA ? 1 : 0) + (tB ? 1 : 0)));
  // (alias is per half: gather_pairs' receivers complete or not each on its own)
  const bool aA = __builtin_amdgcn_readlane((int)alias, 0) != 0, aB = __builtin_amdgcn_readlane((int)alias, 32) != 0;
  st.add(S_ALIASED, (u64)((tA && aA ? 1 : 0) + (tB && aB ? 1 : 0)));
  st.add(S_WRITTEN, (u64)((tA && !aA ? 1 : 0) + (tB && !aB ? 1 : 0)));
}

// the seen row of a pair's receivers, loaded after a gather without early
// exit (only by a half that gathered something), and its S_SEEN_READ count
template <int W>
__device__ __forceinline__ u64x2 pair_seen(const ExpandArgs& a, int h, int lw, bool on, int kB, int v,
                                           uint32_t sv_slot, u64x2 acc, WaveStats& st) {
  const u64 bz = __ballot(on && (acc.x | acc.y) != 0ull);
  const bool any_h = ((bz >> (32 * h)) & 0xFFFFFFFFull) != 0ull;
  u64x2 sv = {0, 0};
  if (any_h && sv_slot != SLOT_NONE) sv = load_piece<W>(a.slot[sv_slot], v, lw);
  const uint32_t sA = (uint32_t)__builtin_amdgcn_readlane((int)sv_slot, 0);
  const uint32_t sB = (uint32_t)__builtin_amdgcn_readlane((int)sv_slot, 32);
  st.add(S_SEEN_READ, (u64)(((bz & 0xFFFFFFFFull) && sA != SLOT_NONE) ? 1 : 0) +
                          (u64)(((bz >> 32) && kB >= 0 && sB != SLOT_NONE) ? 1 : 0));
  return sv;
}

// SCAN_PRE rounds without early exit (round 1 of a C4 run: 7.9 M receivers,
// about 2 active in-neighbours each, already found by the lane phase)
template <int W, class LDS>
__device__ __forceinline__ void pre_pairs(const ExpandArgs& a, LDS& L, u64 mp, int64_t base, uint32_t slot_of,
                                          WaveStats& st) {
  static_assert(W == 64, "half-wave rows");
  const int lane = threadIdx.x & 63, h = lane >> 5, lw = lane & 31;
  while (mp) {
    const int kA = __ffsll((long long)mp) - 1;
    mp &= mp - 1;
    int kB = -1;
    if (mp) {
      kB = __ffsll((long long)mp) - 1;
      mp &= mp - 1;
    }
    const bool on = h == 0 || kB >= 0;
    const int ks = (h && kB >= 0) ? kB : kA;
    const uint32_t npA = L.np[kA], npB = kB >= 0 ? (uint32_t)L.np[kB] : 0u;
    const uint32_t np = on ? (h ? npB : npA) : 0u;
    const int64_t i = base + ks;
    const int v = (int)(a.vbegin + i);
    const uint32_t sv_slot = (uint32_t)__shfl((int)slot_of, ks);
    u64x2 acc = {0, 0};
    const uint32_t nmax = max(npA, npB);
    for (uint32_t q0 = 0; q0 < nmax; q0 += GP_PAIR_RIF) {
      u64x2 r[GP_PAIR_RIF];
#pragma unroll
      for (int q = 0; q < GP_PAIR_RIF; ++q) {
        r[q] = u64x2{0, 0};
        if (q0 + q < np) r[q] = load_piece<W>(a.rows, L.pre[ks][q0 + q], lw);
      }
#pragma unroll
      for (int q = 0; q < GP_PAIR_RIF; ++q) acc |= r[q];
    }
    st.add(S_GATHERED, (u64)(npA + npB));
    st.add(S_ROW_BYTES, (u64)(npA + npB) * (u64)(8 * W));
    const u64x2 sv = pair_seen<W>(a, h, lw, on, kB, v, sv_slot, acc, st);
    pair_finish<W>(a, L, h, lw, on, ks, kB, i, v, acc, sv, st);
  }
}

// The same four at a time (pre_quads; W = 64 without records): a
// quarter-wave per receiver holds a whole 512-B row at 32 B per lane (words
// 4ql .. 4ql + 3), and the receiver's seen row is loaded beside its staged
// rows, one round trip per step instead of two (a receiver whose rows are all
// zero has its seen row read for nothing: round 1's staged senders all send)
#ifndef GP_PRE_QUADS
#define GP_PRE_QUADS 1
#endif
#ifndef GP_PRE_QUADS_RIF
#define GP_PRE_QUADS_RIF 1   // rows in flight per quarter-wave (2: 80 VGPRs, a wave per SIMD less, no faster)
#endif
template <int NG>
__device__ __forceinline__ int take_group(u64& mq, int (&kq)[NG], int gq);
template <class LDS>
__device__ __forceinline__ void pre_quads(const ExpandArgs& a, LDS& L, u64 mq, int64_t base, uint32_t slot_of,
                                          WaveStats& st) {
  const int lane = threadIdx.x & 63, qd = lane >> 4, ql = lane & 15;
  while (mq) {
    int kq[4];
    const int ks = take_group<4>(mq, kq, qd);
    const bool on = ks >= 0;
    const int64_t i = base + (on ? ks : 0);
    const int v = (int)(a.vbegin + i);
    const uint32_t sv_slot = (uint32_t)__shfl((int)slot_of, on ? ks : 0);
    const int np = on ? (int)L.np[ks] : 0;
    int nmax = 0;
    uint32_t rows = 0, nsr = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int nq = __builtin_amdgcn_readlane(np, 16 * q);
      const uint32_t sq = (uint32_t)__builtin_amdgcn_readlane((int)sv_slot, 16 * q);
      nmax = max(nmax, nq);
      rows += (uint32_t)nq;
      nsr += (kq[q] >= 0 && sq != SLOT_NONE) ? 1u : 0u;
    }
    u64x2 s0 = {0, 0}, s1 = {0, 0}, c0 = {0, 0}, c1 = {0, 0};
    if (on && sv_slot != SLOT_NONE) {
      const u64* r = a.slot[sv_slot] + (size_t)v * 64 + 4 * ql;
      s0 = *reinterpret_cast<const u64x2*>(r);
      s1 = *reinterpret_cast<const u64x2*>(r + 2);
    }
    for (int q0 = 0; q0 < nmax; q0 += GP_PRE_QUADS_RIF) {
      if (q0 < np) {   // (one branch per batch; past the last row a lane reloads it: same line, in flight)
        u64x2 r0[GP_PRE_QUADS_RIF], r1[GP_PRE_QUADS_RIF];
#pragma unroll
        for (int q = 0; q < GP_PRE_QUADS_RIF; ++q) {
          const u64* p = a.rows + (size_t)L.pre[ks][min(q0 + q, np - 1)] * 64 + 4 * ql;
          r0[q] = *reinterpret_cast<const u64x2*>(p);
          r1[q] = *reinterpret_cast<const u64x2*>(p + 2);
        }
#pragma unroll
        for (int q = 0; q < GP_PRE_QUADS_RIF; ++q) {
          c0 |= r0[q];
          c1 |= r1[q];
        }
      }
    }
    st.add(S_GATHERED, (u64)rows);
    st.add(S_ROW_BYTES, (u64)rows * 512ull);
    st.add(S_SEEN_READ, nsr);
    const u64x2 n0 = c0 & ~s0, n1 = c1 & ~s1;
    uint32_t tot = (uint32_t)(__popcll(n0.x) + __popcll(n0.y) + __popcll(n1.x) + __popcll(n1.y));
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) tot += (uint32_t)__shfl_xor((int)tot, o);
    u64 t = 0;
    if (on && tot) {
      u64* out = a.slot[a.wslot] + (size_t)v * 64 + 4 * ql;
      *reinterpret_cast<u64x2*>(out) = s0 | n0;
      *reinterpret_cast<u64x2*>(out + 2) = s1 | n1;
      if (a.frx_next) {
        u64* f = a.frx_next + (size_t)v * 64 + 4 * ql;
        *reinterpret_cast<u64x2*>(f) = n0;
        *reinterpret_cast<u64x2*>(f + 2) = n1;
      }
      const u64 nw[4] = {n0.x, n0.y, n1.x, n1.y};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (!nw[j]) continue;
        if (a.alive_next) atomicOr(&L.alive[4 * ql + j], nw[j]);   // (alive_add's words)
        if (a.first) set_first_bytes(a.first + (size_t)i * (64 * 64), 4 * ql + j, nw[j], (uint32_t)a.rr);
        if (a.digest) t ^= digest_term((uint32_t)a.rr, (uint32_t)(a.wbase + 4 * ql + j), nw[j]);
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) t ^= __shfl_xor(t, o);
    uint32_t lmn = 0;   // lines of the new bits holding a nonzero word (lm_next; pair_finish)
    if (a.lm_next) {
      const uint32_t bq = (uint32_t)((__ballot(on && ((n0.x | n0.y | n1.x | n1.y) != 0ull)) >> (16 * qd)) & 0xFFFFull);
#pragma unroll
      for (int l = 0; l < 4; ++l) lmn |= ((bq >> (4 * l)) & 0xFu) ? (1u << l) : 0u;
    }
    if (ql == 0 && on && tot) {
      L.tot[ks] = tot;
      L.lmn[ks] = (uint8_t)lmn;
      L.dig[ks] = t;
    }
    uint32_t nb = 0, nr = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t tq = (uint32_t)__builtin_amdgcn_readlane((int)tot, 16 * q);
      nb += kq[q] >= 0 ? tq : 0u;
      nr += (kq[q] >= 0 && tq) ? 1u : 0u;
    }
    st.add(S_NEW_BITS, nb);
    st.add(S_RECEIVERS, nr);
    st.add(S_WRITTEN, nr);
  }
}

// Done in-neighbours (a.dbits rounds: early exit, no liveness,
// one context).  Without liveness a receiver's new bits are OR_u seen(u) &
// ~seen(v) over all its in-neighbours (ExpandArgs), and every Message-List is
// a subset of the component's messages cmask, so one in-neighbour that held
// all of them at the end of the last round makes the result exactly cmask &
// ~seen(v): the receiver takes the early-exit target and gathers no row.
// Probed for the first DNB_K arcs of the gather order (the biggest
// neighbours, the first to complete), all loads in flight together (1 or 4
// arcs measured no better).  (Not in
// the flat kernel: its 2-arc prefix pass already reads those rows, and the
// extra probe round trip made the 512-message shard's rounds slower.)
constexpr int DNB_K = 2;
__device__ __forceinline__ bool done_nb(const ExpandArgs& a, int64_t b, int64_t e) {
  int32_t c[DNB_K];
#pragma unroll
  for (int q = 0; q < DNB_K; ++q) c[q] = b + q < e ? a.gcol[b + q] : -1;
  u64 w[DNB_K];
#pragma unroll
  for (int q = 0; q < DNB_K; ++q) w[q] = c[q] >= 0 ? a.dbits[c[q] >> 6] : 0ull;
  bool d = false;
#pragma unroll
  for (int q = 0; q < DNB_K; ++q) d = d || (c[q] >= 0 && ((w[q] >> (c[q] & 63)) & 1ull));
  return d;
}

// Receivers with a done in-neighbour two at a time, one per half-wave (W =
// 64): nothing to gather, so each pair is one round trip (its seen rows and
// the component rows, the latter L2-resident) and the commit
template <int W, bool ALIVE, bool ALIAS, class LDS>
__device__ __forceinline__ void dnb_pairs(const ExpandArgs& a, LDS& L, u64 mp, int64_t base, uint32_t slot_of,
                                          WaveStats& st) {
  static_assert(W == 64, "half-wave rows");
  const int lane = threadIdx.x & 63, h = lane >> 5, lw = lane & 31;
  while (mp) {
    const int kA = __ffsll((long long)mp) - 1;
    mp &= mp - 1;
    int kB = -1;
    if (mp) {
      kB = __ffsll((long long)mp) - 1;
      mp &= mp - 1;
    }
    const bool on = h == 0 || kB >= 0;
    const int ks = (h && kB >= 0) ? kB : kA;
    int64_t i = base + ks;
    int v = (int)(a.vbegin + i);
    if constexpr (LDS::kList) {   // (list rounds: lane k's vertex)
      v = L.vid[ks];
      i = v - a.vbegin;
    }
    const uint32_t sv_slot = (uint32_t)__shfl((int)slot_of, ks);
    u64x2 sv = {0, 0}, cm = {0, 0};
    if (on) {
      if (sv_slot != SLOT_NONE) sv = load_piece<W>(a.slot[sv_slot], v, lw);
      cm = load_piece<W>(a.cmask, L.mi[ks], lw);
      if (ALIVE && a.alive) cm &= load_piece<W>(a.alive, 0, lw);   // liveness: the sated neighbour's alive set
    }
    const uint32_t sA = (uint32_t)__builtin_amdgcn_readlane((int)sv_slot, 0);
    const uint32_t sB = (uint32_t)__builtin_amdgcn_readlane((int)sv_slot, 32);
    st.add(S_SEEN_READ, (u64)((sA != SLOT_NONE ? 1 : 0) + (kB >= 0 && sB != SLOT_NONE ? 1 : 0)));
    pair_finish<W>(a, L, h, lw, on, ks, kB, i, v, cm, sv, st, ALIAS && a.alias != 0);
  }
}

// The same four at a time, one per quarter-wave (W = 64, the done-probe
// variants, i.e. the late rounds: C4 round 5's 7.5 M receivers are all done-
// neighbour ones): a quarter-wave holds a whole row at 32 B per lane (words
// 4ql .. 4ql + 3), so four receivers' seen and component rows are in flight
// per round trip instead of two.  No liveness (no alive sets, no records).
template <bool ALIAS, bool ALIVE, class LDS>
__device__ __forceinline__ void dnb_quads(const ExpandArgs& a, LDS& L, u64 mq, int64_t base, uint32_t slot_of,
                                          WaveStats& st) {
  const int lane = threadIdx.x & 63, qd = lane >> 4, ql = lane & 15;
  const bool alias = ALIAS && a.alias != 0;
  while (mq) {
    int kq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      kq[q] = -1;
      if (mq) {
        kq[q] = __ffsll((long long)mq) - 1;
        mq &= mq - 1;
      }
    }
    const int ks = qd == 0 ? kq[0] : qd == 1 ? kq[1] : qd == 2 ? kq[2] : kq[3];
    const bool on = ks >= 0;
    int64_t i = base + (on ? ks : 0);
    int v = (int)(a.vbegin + i);
    if constexpr (LDS::kList) {
      v = on ? L.vid[ks] : 0;
      i = v - a.vbegin;
    }
    const uint32_t sv_slot = (uint32_t)__shfl((int)slot_of, on ? ks : 0);
    u64x2 s0 = {0, 0}, s1 = {0, 0}, c0 = {0, 0}, c1 = {0, 0};
    if (on) {
      if (sv_slot != SLOT_NONE) {
        const u64* r = a.slot[sv_slot] + (size_t)v * 64 + 4 * ql;
        s0 = *reinterpret_cast<const u64x2*>(r);
        s1 = *reinterpret_cast<const u64x2*>(r + 2);
      }
      const u64* cr = a.cmask + (size_t)L.mi[ks] * 64 + 4 * ql;
      c0 = *reinterpret_cast<const u64x2*>(cr);
      c1 = *reinterpret_cast<const u64x2*>(cr + 2);
      if (ALIVE && a.alive) {   // liveness: the sated neighbour's alive set
        c0 &= *reinterpret_cast<const u64x2*>(a.alive + 4 * ql);
        c1 &= *reinterpret_cast<const u64x2*>(a.alive + 4 * ql + 2);
      }
    }
    const u64x2 n0 = c0 & ~s0, n1 = c1 & ~s1;
    uint32_t tot = (uint32_t)(__popcll(n0.x) + __popcll(n0.y) + __popcll(n1.x) + __popcll(n1.y));
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) tot += (uint32_t)__shfl_xor((int)tot, o);
    u64 t = 0;
    if (on && tot) {
      u64* out = a.slot[a.wslot] + (size_t)v * 64 + 4 * ql;
      if (!alias) {
        *reinterpret_cast<u64x2*>(out) = s0 | n0;
        *reinterpret_cast<u64x2*>(out + 2) = s1 | n1;
      }
      if (a.frx_next) {
        u64* f = a.frx_next + (size_t)v * 64 + 4 * ql;
        *reinterpret_cast<u64x2*>(f) = n0;
        *reinterpret_cast<u64x2*>(f + 2) = n1;
      }
      const u64 nw[4] = {n0.x, n0.y, n1.x, n1.y};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (!nw[j]) continue;
        if (ALIVE && a.alive_next) atomicOr(&L.alive[4 * ql + j], nw[j]);   // (alive_add's words)
        if (a.first) set_first_bytes(a.first + (size_t)i * (64 * 64), 4 * ql + j, nw[j], (uint32_t)a.rr);
        if (a.digest) t ^= digest_term((uint32_t)a.rr, (uint32_t)(a.wbase + 4 * ql + j), nw[j]);
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) t ^= __shfl_xor(t, o);
    if (ql == 0 && on && tot) {
      L.tot[ks] = tot;
      L.lmn[ks] = alias ? LMN_ALIAS : (uint8_t)0;   // (no line masks are written in early-exit rounds)
      L.dig[ks] = t;
    }
    uint32_t nb = 0, nr = 0, nsr = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t tq = (uint32_t)__builtin_amdgcn_readlane((int)tot, 16 * q);
      const uint32_t sq = (uint32_t)__builtin_amdgcn_readlane((int)sv_slot, 16 * q);
      nb += kq[q] >= 0 ? tq : 0u;
      nr += (kq[q] >= 0 && tq) ? 1u : 0u;
      nsr += (kq[q] >= 0 && sq != SLOT_NONE) ? 1u : 0u;
    }
    st.add(S_NEW_BITS, nb);
    st.add(S_RECEIVERS, nr);
    st.add(alias ? S_ALIASED : S_WRITTEN, nr);
    st.add(S_SEEN_READ, nsr);
  }
}

// W = 32 rows (two-rank message shards): receivers four per wave step, one
// per 16-lane group (a 256-B row at 16 B per lane, the load_piece layout of
// group g = lane / 16), where the serial loop took them one at a time -- the
// done-neighbour receivers (dnb_groups: the N = 2 job's slow rank ran 7.5 M
// of them in round 5 at 3.1 ms) and the prefiltered ones of sparse rounds
// (pre_groups).  group_finish commits like finish_row (deferred per-vertex
// words, L.tot / L.dig).
#ifndef GP_DNB_GROUPS
#define GP_DNB_GROUPS 1
#endif
#ifndef GP_PRE_GROUPS
#define GP_PRE_GROUPS 1
#endif
template <int W>
struct Groups {
  static constexpr int LG = Geo<W>::LPR;   // lanes per row
  static constexpr int NG = 64 / LG;       // receivers per step
  static_assert(Geo<W>::WPL == 2 && NG >= 2 && NG <= 16, "16-B pieces, two to sixteen rows per wave");
};

// the next NG receivers of mq (kq[q] = -1: none); returns group gq's
template <int NG>
__device__ __forceinline__ int take_group(u64& mq, int (&kq)[NG], int gq) {
  int ks = -1;
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    kq[q] = -1;
    if (mq) {
      kq[q] = __ffsll((long long)mq) - 1;
      mq &= mq - 1;
    }
    if (q == gq) ks = kq[q];
  }
  return ks;
}

template <int W, class LDS>
__device__ __forceinline__ void group_finish(const ExpandArgs& a, LDS& L, int lw, bool on, int ks,
                                             const int (&kq)[Groups<W>::NG], int64_t i, int v, u64x2 acc,
                                             u64x2 sv, WaveStats& st) {
  constexpr int LG = Groups<W>::LG, NG = Groups<W>::NG;
  const u64x2 nw = acc & ~sv;
  uint32_t tot = (uint32_t)(__popcll(nw.x) + __popcll(nw.y));
#pragma unroll
  for (int o = LG / 2; o > 0; o >>= 1) tot += (uint32_t)__shfl_xor((int)tot, o);
  u64 t = 0;
  if (on && tot) {
    alive_add<W>(a, L, lw, nw);
    store_piece<W>(a.slot[a.wslot], v, lw, sv | nw);
    if (a.frx_next) store_piece<W>(a.frx_next, v, lw, nw);
    if (a.first) {
      uint8_t* row = a.first + (size_t)i * (W * 64);
      if (nw.x) set_first_bytes(row, 2 * lw, nw.x, (uint32_t)a.rr);
      if (nw.y) set_first_bytes(row, 2 * lw + 1, nw.y, (uint32_t)a.rr);
    }
    if (a.digest) {
      if (nw.x) t ^= digest_term((uint32_t)a.rr, (uint32_t)(a.wbase + 2 * lw), nw.x);
      if (nw.y) t ^= digest_term((uint32_t)a.rr, (uint32_t)(a.wbase + 2 * lw + 1), nw.y);
    }
  }
#pragma unroll
  for (int o = LG / 2; o > 0; o >>= 1) t ^= __shfl_xor(t, o);
  if (lw == 0 && on && tot) {
    L.tot[ks] = tot;
    L.lmn[ks] = 0;   // (line masks: W = 64 only)
    L.dig[ks] = t;
  }
  uint32_t nb = 0, nr = 0;
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const uint32_t tq = (uint32_t)__builtin_amdgcn_readlane((int)tot, LG * q);
    nb += kq[q] >= 0 ? tq : 0u;
    nr += (kq[q] >= 0 && tq) ? 1u : 0u;
  }
  st.add(S_NEW_BITS, nb);
  st.add(S_RECEIVERS, nr);
  st.add(S_WRITTEN, nr);
}

// groups whose receiver's seen row was read (S_SEEN_READ): on[q] && slot[q] != SLOT_NONE
template <int W>
__device__ __forceinline__ uint32_t group_seen_reads(const int (&kq)[Groups<W>::NG], uint32_t sv_slot, u64 read) {
  constexpr int LG = Groups<W>::LG, NG = Groups<W>::NG;
  uint32_t n = 0;
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const uint32_t sq = (uint32_t)__builtin_amdgcn_readlane((int)sv_slot, LG * q);
    n += (kq[q] >= 0 && sq != SLOT_NONE && ((read >> (LG * q)) & 1ull)) ? 1u : 0u;
  }
  return n;
}

template <int W, bool ALIVE, class LDS>
__device__ __forceinline__ void dnb_groups(const ExpandArgs& a, LDS& L, u64 mq, int64_t base, uint32_t slot_of,
                                           WaveStats& st) {
  constexpr int LG = Groups<W>::LG, NG = Groups<W>::NG;
  const int lane = threadIdx.x & 63, gq = lane / LG, lw = lane % LG;
  while (mq) {
    int kq[NG];
    const int ks = take_group<NG>(mq, kq, gq);
    const bool on = ks >= 0;
    int64_t i = base + (on ? ks : 0);
    int v = (int)(a.vbegin + i);
    if constexpr (LDS::kList) {
      v = on ? L.vid[ks] : 0;
      i = v - a.vbegin;
    }
    const uint32_t sv_slot = (uint32_t)__shfl((int)slot_of, on ? ks : 0);
    u64x2 sv = {0, 0}, cm = {0, 0};
    if (on) {
      if (sv_slot != SLOT_NONE) sv = load_piece<W>(a.slot[sv_slot], v, lw);
      cm = load_piece<W>(a.cmask, L.mi[ks], lw);
      if (ALIVE && a.alive) cm &= load_piece<W>(a.alive, 0, lw);   // liveness: the sated neighbour's alive set
    }
    st.add(S_SEEN_READ, group_seen_reads<W>(kq, sv_slot, ~0ull));
    group_finish<W>(a, L, lw, on, ks, kq, i, v, cm & ~sv, sv, st);
  }
}

// SCAN_PRE rounds without early exit: the receivers whose active
// in-neighbours the lane phase staged (L.pre, at most PRE_IDS), four at a time
template <int W, class LDS>
__device__ __forceinline__ void pre_groups(const ExpandArgs& a, LDS& L, u64 mp, int64_t base, uint32_t slot_of,
                                           WaveStats& st) {
  constexpr int LG = Groups<W>::LG, NG = Groups<W>::NG;
  const int lane = threadIdx.x & 63, gq = lane / LG, lw = lane % LG;
  while (mp) {
    int kq[NG];
    const int ks = take_group<NG>(mp, kq, gq);
    const bool on = ks >= 0;
    const int64_t i = base + (on ? ks : 0);
    const int v = (int)(a.vbegin + i);
    const uint32_t sv_slot = (uint32_t)__shfl((int)slot_of, on ? ks : 0);
    const int np = on ? (int)L.np[ks] : 0;
    int nmax = 0;
    uint32_t rows = 0;
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      const int nq = __builtin_amdgcn_readlane(np, LG * q);
      nmax = max(nmax, nq);
      rows += (uint32_t)nq;
    }
    u64x2 acc = {0, 0};
    for (int q0 = 0; q0 < nmax; q0 += GP_PAIR_RIF) {
      if (q0 < np) {   // (one branch per batch; past the last row a lane reloads it: same line, in flight)
        u64x2 r[GP_PAIR_RIF];
#pragma unroll
        for (int q = 0; q < GP_PAIR_RIF; ++q) r[q] = load_piece<W>(a.rows, L.pre[ks][min(q0 + q, np - 1)], lw);
#pragma unroll
        for (int q = 0; q < GP_PAIR_RIF; ++q) acc |= r[q];
      }
    }
    st.add(S_GATHERED, (u64)rows);
    st.add(S_ROW_BYTES, (u64)rows * (u64)(8 * W));
    // the seen row only where the gather found something (pair_seen)
    const u64 bz = __ballot(on && (acc.x | acc.y) != 0ull);
    u64 gz = 0;   // bit LG * q: group q gathered a nonzero word
#pragma unroll
    for (int q = 0; q < NG; ++q)
      if ((bz >> (LG * q)) & ((1ull << LG) - 1ull)) gz |= 1ull << (LG * q);
    u64x2 sv = {0, 0};
    if (((gz >> (LG * gq)) & 1ull) && sv_slot != SLOT_NONE) sv = load_piece<W>(a.slot[sv_slot], v, lw);
    st.add(S_SEEN_READ, group_seen_reads<W>(kq, sv_slot, gz));
    group_finish<W>(a, L, lw, on, ks, kq, i, v, acc, sv, st);
  }
}

// rows in flight per receiver of gather_pairs (W = 64: 2, 72 VGPRs, 7 waves
// per SIMD; 3 took 76 and 6 waves: C4 round 4 6.70-6.74 -> 6.44-6.48 ms with
// 2) and of gather_groups (W = 32: 3; 2 was slower, profiles/r06_ab_grif.txt)
#ifndef GP_GPAIR_RIF
#define GP_GPAIR_RIF 2
#endif
#ifndef GP_GGROUP_RIF
#define GP_GGROUP_RIF 3
#endif

// W = 32 near-done unfiltered pulls: receivers of in-degree <= 16 four per
// wave step, one per 16-lane group (gather_pairs' scheme at a 256-B row per
// group-instruction): column ids, seen and component rows in one round trip,
// then GP_GGROUP_RIF rows per group in flight until the target is covered.
template <int W, class LDS>
__device__ __forceinline__ void gather_groups(const ExpandArgs& a, LDS& L, u64 mp, int64_t base, uint32_t slot_of,
                                              WaveStats& st) {
  constexpr int LG = Groups<W>::LG, NG = Groups<W>::NG;
  const int lane = threadIdx.x & 63, gq = lane / LG, lw = lane % LG;
  const bool ee = a.early_exit != 0;
  while (mp) {
    int kq[NG];
    const int ks = take_group<NG>(mp, kq, gq);
    const bool on = ks >= 0;
    const int64_t i = base + (on ? ks : 0);
    const int v = (int)(a.vbegin + i);
    const int64_t vb = L.rp[on ? ks : 0];
    const int deg = on ? (int)(L.rp[ks + 1] - vb) : 0;   // <= LG (the caller's mask)
    const uint32_t sv_slot = (uint32_t)__shfl((int)slot_of, on ? ks : 0);
    if (lw < deg) L.idx[LG * gq + lw] = a.gcol[vb + lw];
    u64x2 sv = {0, 0}, want = {0, 0};
    if (on) {
      if (sv_slot != SLOT_NONE) sv = load_piece<W>(a.slot[sv_slot], v, lw);
      if (ee) want = load_piece<W>(a.cmask, L.mi[ks], lw) & ~sv;
    }
    wave_sync_lds();
    int dq[NG], dmax = 0, arcs = 0;
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      dq[q] = __builtin_amdgcn_readlane(deg, LG * q);
      dmax = max(dmax, dq[q]);
      arcs += dq[q];
    }
    st.add(S_ARCS, (u64)arcs);
    st.add(S_SEEN_READ, group_seen_reads<W>(kq, sv_slot, ~0ull));
    bool live = on && (!ee || (want.x | want.y) != 0ull);
    u64x2 acc = {0, 0};
    u64 rows = 0, pieces = 0;
    for (int k0 = 0; k0 < dmax; k0 += GP_GGROUP_RIF) {
      const u64 lb = __ballot(live);
      if (lb == 0ull) break;
      if (live && k0 < deg) {   // (one branch per batch, gather_pairs)
        u64x2 r[GP_GGROUP_RIF];
#pragma unroll
        for (int q = 0; q < GP_GGROUP_RIF; ++q) r[q] = load_piece<W>(a.rows, L.idx[LG * gq + min(k0 + q, deg - 1)], lw);
#pragma unroll
        for (int q = 0; q < GP_GGROUP_RIF; ++q) acc |= r[q];
      }
#pragma unroll
      for (int q = 0; q < GP_GGROUP_RIF; ++q) pieces += line_pieces<W>(__ballot(live && k0 + q < deg));
#pragma unroll
      for (int q = 0; q < NG; ++q)
        if ((lb >> (LG * q)) & ((1ull << LG) - 1ull)) rows += (u64)min(GP_GGROUP_RIF, max(dq[q] - k0, 0));
      if (ee) {
        const u64x2 miss = want & ~acc;
        live = live && (miss.x | miss.y) != 0ull;
      }
    }
    st.add(S_GATHERED, rows);
    st.add(S_ROW_BYTES, pieces * 16ull);
    wave_sync_lds();   // (the next step's column ids overwrite L.idx)
    group_finish<W>(a, L, lw, on, ks, kq, i, v, acc, sv, st);
  }
}

// Receivers of in-degree <= 32 two at a time, one per half-wave (W = 64, the
// unfiltered SCAN_QUADS variants: near-done pulls, C4 round 4 / C5 rounds
// 4-5, where a receiver lacks a few words and gathers ~8 rows).  A half loads
// its receiver's column ids (one per lane), seen row and component row in one
// round trip, then gathers GP_GPAIR_RIF rows at a time (a whole 512-B row per
// half-wave instruction) until they cover its target (per-lane word skip as in
// gather_rows_n).  The serial loop walks target -> rows -> rows one receiver
// after the other; here two receivers' chains share each round trip.  Same
// rows, commits and sated marks as the serial loop (returned: the sated
// receivers, alive rounds).
template <bool ALIVE, bool ALIAS, class LDS>
__device__ __forceinline__ u64 gather_pairs(const ExpandArgs& a, LDS& L, u64 mp, int64_t base, uint32_t slot_of,
                                            WaveStats& st) {
  constexpr int W = 64;
  const int lane = threadIdx.x & 63, h = lane >> 5, lw = lane & 31;
  const bool ee = a.early_exit != 0;
  u64 sat = 0;
  while (mp) {
    const int kA = __ffsll((long long)mp) - 1;
    mp &= mp - 1;
    int kB = -1;
    if (mp) {
      kB = __ffsll((long long)mp) - 1;
      mp &= mp - 1;
    }
    const bool on = h == 0 || kB >= 0;
    const int ks = (h && kB >= 0) ? kB : kA;
    const int v = (int)(a.vbegin + base + ks);
    const int64_t vb = L.rp[ks];
    const int deg = on ? (int)(L.rp[ks + 1] - vb) : 0;   // <= 32 (the caller's mask)
    const uint32_t sv_slot = (uint32_t)__shfl((int)slot_of, ks);
    u64x2 want = {0, 0};
    if (lw < deg) L.idx[32 * h + lw] = a.gcol[vb + lw];   // (this pair's column ids: half h at 32h)
    wave_sync_lds();
    {
      u64x2 sv = {0, 0};
      if (on) {
        if (sv_slot != SLOT_NONE) sv = load_piece<W>(a.slot[sv_slot], v, lw);
        if (ee) {
          u64x2 cm = load_piece<W>(a.cmask, L.mi[ks], lw);
          if (ALIVE && a.alive) cm &= load_piece<W>(a.alive, 0, lw);
          want = cm & ~sv;
        }
      }
      L.seen[64 * h + 2 * lw] = sv.x;   // (parked for the commit: registers for the rows in flight)
      L.seen[64 * h + 2 * lw + 1] = sv.y;
    }
    const int dA = __builtin_amdgcn_readlane(deg, 0), dB = __builtin_amdgcn_readlane(deg, 32);
    const uint32_t sA = (uint32_t)__builtin_amdgcn_readlane((int)sv_slot, 0);
    const uint32_t sB = (uint32_t)__builtin_amdgcn_readlane((int)sv_slot, 32);
    st.add(S_ARCS, (u64)(dA + dB));
    st.add(S_SEEN_READ, (u64)((sA != SLOT_NONE ? 1 : 0) + (kB >= 0 && sB != SLOT_NONE ? 1 : 0)));
    bool live = on && (!ee || (want.x | want.y) != 0ull);   // this lane's words still miss messages
    u64x2 acc = {0, 0};
    u64 rows = 0, pieces = 0;
    for (int k0 = 0; k0 < max(dA, dB); k0 += GP_GPAIR_RIF) {
      const u64 lb = __ballot(live);
      if (lb == 0ull) break;
      // one branch for the batch: a lane past its receiver's last arc loads
      // that last row again (same line, already requested: no HBM bytes),
      // which keeps the RIF loads unconditional inside it
      if (live && k0 < deg) {
        u64x2 r[GP_GPAIR_RIF];
#pragma unroll
        for (int q = 0; q < GP_GPAIR_RIF; ++q) r[q] = load_piece<W>(a.rows, L.idx[32 * h + min(k0 + q, deg - 1)], lw);
#pragma unroll
        for (int q = 0; q < GP_GPAIR_RIF; ++q) acc |= r[q];
      }
#pragma unroll
      for (int q = 0; q < GP_GPAIR_RIF; ++q) pieces += line_pieces<W>(__ballot(live && k0 + q < deg));
      if (lb & 0xFFFFFFFFull) rows += (u64)min(GP_GPAIR_RIF, max(dA - k0, 0));
      if (lb >> 32) rows += (u64)min(GP_GPAIR_RIF, max(dB - k0, 0));
      if (ee) {
        const u64x2 miss = want & ~acc;
        live = live && (miss.x | miss.y) != 0ull;
      }
    }
    st.add(S_GATHERED, rows);
    st.add(S_ROW_BYTES, pieces * 16ull);
    // a half whose rows covered its whole target: the receiver completes its
    // component (alias rounds: it commits SLOT_CMASK) or, under liveness,
    // holds every alive message it lacked (sated)
    const u64x2 rem = want & ~acc;
    const u64 rb = __ballot(on && (rem.x | rem.y) != 0ull);
    const bool full = ((rb >> (32 * h)) & 0xFFFFFFFFull) == 0ull;
    if constexpr (ALIVE) {
      if (a.sate && ee && a.alive) {
        if (!(rb & 0xFFFFFFFFull)) sat |= 1ull << kA;
        if (kB >= 0 && !(rb >> 32)) sat |= 1ull << kB;
      }
    }
    wave_sync_lds();   // (the next pair's column ids overwrite L.idx)
    const u64x2 sv = {L.seen[64 * h + 2 * lw], L.seen[64 * h + 2 * lw + 1]};
    pair_finish<W>(a, L, h, lw, on, ks, kB, base + ks, v, acc, sv, st, ALIAS && a.alias != 0 && ee && full);
  }
  return sat;
}

// main pull kernel: a wave owns 64 consecutive vertices.  The per-vertex
// checks (sender accounting, down / done / hub / no in-arcs) run lane-parallel
// with coalesced loads; the wave then scans, one receiver at a time, only the
// vertices that can still receive something.  Kept lean on registers (7 waves
// per SIMD): the dense rounds are bound by the rows in flight.
// (occupancy is the compiler's choice: an 8-waves hint spilled and was slower
// for the alive variants, and for W < 64, r04_ab_waves.txt)
template <int W, int MODE>
__global__ EXPAND_BOUNDS __attribute__((amdgpu_waves_per_eu(1))) void k_expand(ExpandArgs a) {
  constexpr int LPR = Geo<W>::LPR;
  __shared__ LDS_OF(MODE) s_w[EWAVES];
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  const int g = lane / LPR, lw = lane % LPR;
  auto& L = s_w[wib];
  constexpr bool ALIVE = (MODE & SCAN_ALIVE) != 0;
  constexpr bool DPROBE = (MODE & SCAN_DPROBE) != 0;
  constexpr bool LIST = (MODE & SCAN_LIST) != 0;
  constexpr bool QUADS = (MODE & SCAN_QUADS) != 0;
  constexpr int SCAN = MODE & ~(SCAN_ALIVE | SCAN_DPROBE | SCAN_LIST | SCAN_QUADS);
  // the variants that can append this round's survivors to the next list
#ifndef GP_ULIST_EMIT
#define GP_ULIST_EMIT 1
#endif
  constexpr bool EMIT = GP_ULIST_EMIT && W == 64 && (SCAN == SCAN_FILTERED || SCAN == SCAN_UNFILTERED);
  // the variants done-neighbour rounds without liveness launch: their complete
  // receivers may alias (a.alias) and their scans probe the done bitmap
  // (a.dprobe); the other variants compile neither
  constexpr bool ALIASABLE = W == 64 && !ALIVE && (SCAN == SCAN_FILTERED || SCAN == SCAN_UNFILTERED);
  // the variants whose receivers of in-degree <= 32 go two at a time
  // (gather_pairs): the unfiltered near-done pulls without liveness
  // (SCAN_QUADS; C4 round 4 6.93-7.02 -> 6.61-6.65 ms, 80 VGPRs; in the alive
  // one C5 rounds 4-5 gained nothing: their receivers scan to the end,
  // profiles/r06_ab_gather_pairs.txt)
#ifndef GP_GATHER_PAIRS
#define GP_GATHER_PAIRS 1
#endif
#ifndef GP_GGROUPS_W8
#define GP_GGROUPS_W8 0   // gather_groups at W = 8 too (16 receivers per step: 96 VGPRs, slower)
#endif
  constexpr bool GPAIRS = GP_GATHER_PAIRS && W == 64 && QUADS && !ALIVE && SCAN == SCAN_UNFILTERED && !LIST;
  constexpr bool GGROUPS = GP_GATHER_PAIRS && (W == 32 || W == 16 || (W == 8 && GP_GGROUPS_W8)) && QUADS && !ALIVE && SCAN == SCAN_UNFILTERED && !LIST;
  WaveStats st;
  ws_zero<EWAVES>(st);
  const int64_t base = ((int64_t)blockIdx.x * EWAVES + wib) * 64;
  if (base < (LIST ? a.ulist_n : a.nloc)) {
    const int64_t li = base + lane;
    // lane's vertex (local index): base + lane, or the list's entry (list
    // rounds: every sender's accounting is k_mkbits', every non-receiver's
    // fpop_next was zeroed before the launch)
    const bool valid = LIST ? li < a.ulist_n : li < a.nloc;
    const int64_t vi = LIST ? (valid ? (int64_t)a.ulist[li] : 0) : li;
    bool need = false, act = false, dnb = false;
    // degree-split rounds: receivers the push half touched (bit k = vertex
    // base + k; one context: local = global ids).  A touched receiver's
    // accumulator row is one more entry of its staged list: row a.acc_row + v
    // of this round's slot buffer is row v of a.acc (same stride, host-checked
    // offset), so the gathers need no second base pointer.  k_acc_clear zeroes
    // the rows and the bitmap after the pull (no store here to the rows the
    // gathers read)
    u64 tw = 0;
    if constexpr ((MODE & 3) == SCAN_PRE) {
      if (a.prehi) tw = a.tbits[base >> 6];
    }
    u64 sends = 0;
    uint32_t slot_of = SLOT_NONE;
    uint32_t pre_arcs = 0;   // SCAN_PRE: arcs the lane phase scanned
    bool small = false;      // GPAIRS: in-degree <= 32
    if (valid) {
      const int v = (int)(a.vbegin + vi);
      if constexpr (!LIST) {
        const uint32_t fp = a.fpop[v];
        act = fp != 0u;
        if (act) sends = (u64)fp * (u64)(uint32_t)max(a.deg_live[v], 0);
      }
      const int64_t b = a.row_ptr[v], e = a.row_ptr[v + 1];
      L.rp[lane] = b;
      if constexpr (LIST) {
        L.re[lane] = e;
        L.vid[lane] = v;
      } else {
        if (lane == 63 || li + 1 == a.nloc) L.rp[lane + 1] = e;
      }
      const bool hub = e - b > a.hub_thr;   // split over waves by the hub kernels
      need = !(a.state[v] & (ST_DOWN | ST_SATED)) && a.seenpop[vi] < a.done_at[v] && !hub && e > b;
      if constexpr (GPAIRS) small = e - b <= 32;
      if constexpr (GGROUPS) small = e - b <= Geo<W>::LPR;
      if constexpr ((MODE & 3) == SCAN_MASKED) need = need && mask_any(a.amask, b, e);
      if constexpr ((MODE & 3) == SCAN_PRE) {
        // sparse filtered rounds: every lane probes the in-list of its own
        // vertex (up to PRE_MAX_DEG arcs, all loads in flight together), so the
        // wave's serial loop skips vertices with no active in-neighbour and
        // starts the others at their rows
        uint32_t np = 0xFFu;
        const bool tch = (tw >> lane) & 1ull;
        const int64_t se = a.prehi ? b + a.prehi[v] : e;   // end of the arcs this vertex scans
        L.len[lane] = (uint32_t)(se - b);
        if (need && se - b <= PRE_MAX_DEG) {
          const int deg = (int)(se - b);
          uint32_t cnt = 0;
#pragma unroll
          for (int h = 0; h < PRE_MAX_DEG / PRE_IDS; ++h) {
            if (h * PRE_IDS < deg) {
              int32_t c[PRE_IDS];
              u64 w[PRE_IDS];
#pragma unroll
              for (int q = 0; q < PRE_IDS; ++q) c[q] = h * PRE_IDS + q < deg ? a.gcol[b + h * PRE_IDS + q] : -1;
              if (a.sbits) {   // summary level first: L2-resident, most probes end there
                u64 sw[PRE_IDS];
#pragma unroll
                for (int q = 0; q < PRE_IDS; ++q) sw[q] = c[q] >= 0 ? a.sbits[c[q] >> 12] : 0ull;
#pragma unroll
                for (int q = 0; q < PRE_IDS; ++q)
                  w[q] = ((sw[q] >> ((c[q] >> 6) & 63)) & 1ull) ? a.abits[c[q] >> 6] : 0ull;
              } else
#pragma unroll
              for (int q = 0; q < PRE_IDS; ++q) w[q] = c[q] >= 0 ? a.abits[c[q] >> 6] : 0ull;
#pragma unroll
              for (int q = 0; q < PRE_IDS; ++q) {
                if (c[q] >= 0 && ((w[q] >> (c[q] & 63)) & 1ull)) {
                  if (cnt < (uint32_t)PRE_IDS) L.pre[lane][cnt] = c[q];
                  ++cnt;
                }
              }
            }
          }
          if (cnt + (tch ? 1u : 0u) <= (uint32_t)PRE_IDS) {
            if (tch) L.pre[lane][cnt++] = a.acc_row + v;   // the accumulator row: one more entry
            np = cnt;
            pre_arcs = (uint32_t)deg;
          }
          if (cnt == 0) need = false;
        }
        L.np[lane] = (uint8_t)np;
      }
      if (!need && !hub) a.fpop_next[v] = 0;
      slot_of = a.sp[v];
      if (a.early_exit && need) L.mi[lane] = a.midx[v];
      // (with alive sets -- liveness -- only the SCAN_ALIVE variants: the done
      // target is then cmask & F_r & ~seen, which the others cannot form)
      if (a.dbits && need && (ALIVE || !a.alive)) dnb = done_nb(a, b, e);
    }
    if constexpr ((MODE & 3) == SCAN_PRE) st.add(S_ARCS, (u64)wave_sum_u32(pre_arcs));
    st.add(S_SENDS, wave_sum_u64(sends));
    st.add(S_ACTIVE, (u64)__popcll(__ballot(act)));
    st.add(S_VISITED, (u64)__popcll(__ballot(need)));
    L.tot[lane] = 0u;
    L.dig[lane] = 0ull;
    alive_zero<W>(a, L.alive, lane);
    wave_sync_lds();
    const bool ee = a.early_exit != 0;
    u64 m = __ballot(need);
    const u64 mdn = __ballot(dnb);   // receivers with a done in-neighbour (a.dbits rounds)
    st.add(S_DNB, (u64)__popcll(mdn));
    if constexpr ((MODE & 3) == SCAN_PRE && GP_WAVE_PRE_MAX > PRE_MAX_DEG) {
      // receivers with PRE_MAX_DEG < deg <= GP_WAVE_PRE_MAX: the wave probes
      // their in-lists WAVE_PRE_N at a time (one coalesced pass each, all
      // loads in flight together) instead of one receiver's chain after the
      // other in the serial loop; those with at most PRE_IDS active
      // neighbours join the prefiltered receivers, those with none drop out
      u64 mw = __ballot(need && L.np[lane] == 0xFFu && L.len[lane] <= GP_WAVE_PRE_MAX);
      u64 zero = 0;   // no active in-neighbour: nothing to scan (commit writes fpop_next = 0)
      uint32_t arcs = 0;
      while (mw) {
        int kq[WAVE_PRE_N];
        int32_t c[WAVE_PRE_N];
#pragma unroll
        for (int q = 0; q < WAVE_PRE_N; ++q) {
          kq[q] = -1;
          if (mw) {
            kq[q] = __ffsll((long long)mw) - 1;
            mw &= mw - 1;
          }
          c[q] = -1;
          if (kq[q] >= 0) {
            const int64_t b = L.rp[kq[q]];
            if (lane < (int)L.len[kq[q]]) c[q] = a.gcol[b + lane];
          }
        }
        u64 w[WAVE_PRE_N];
        if (a.sbits) {
          u64 sw[WAVE_PRE_N];
#pragma unroll
          for (int q = 0; q < WAVE_PRE_N; ++q) sw[q] = c[q] >= 0 ? a.sbits[c[q] >> 12] : 0ull;
#pragma unroll
          for (int q = 0; q < WAVE_PRE_N; ++q)
            w[q] = ((sw[q] >> ((c[q] >> 6) & 63)) & 1ull) ? a.abits[c[q] >> 6] : 0ull;
        } else
#pragma unroll
        for (int q = 0; q < WAVE_PRE_N; ++q) w[q] = c[q] >= 0 ? a.abits[c[q] >> 6] : 0ull;
#pragma unroll
        for (int q = 0; q < WAVE_PRE_N; ++q) {
          if (kq[q] < 0) continue;
          const bool act = c[q] >= 0 && ((w[q] >> (c[q] & 63)) & 1ull);
          const u64 am = __ballot(act);
          const int tq = (int)((tw >> kq[q]) & 1ull);   // degree-split: + the accumulator row
          const int cnt = __popcll(am) + tq;
          if (cnt <= PRE_IDS) {   // (more: the serial loop scans it, and counts its arcs)
            if (act) L.pre[kq[q]][lane_rank(am)] = c[q];
            if (lane == 0) {
              if (tq) L.pre[kq[q]][cnt - 1] = a.acc_row + (int32_t)(base + kq[q]);
              L.np[kq[q]] = (uint8_t)cnt;
            }
            if (cnt == 0) zero |= 1ull << kq[q];
            arcs += L.len[kq[q]];
          }
        }
      }
      st.add(S_ARCS, (u64)arcs);
      wave_sync_lds();
      m &= ~zero;
    }
    if constexpr ((MODE & SCAN_CML) != 0) L.racc[lane] = 0ull;   // record rounds: first receiver's accumulator
    if constexpr (W == 64 && (MODE & 3) == SCAN_PRE) {
      if (!ee) {   // prefiltered receivers two at a time, the rest below
        const u64 mp = m & __ballot(need && L.np[lane] != 0xFFu);
        if constexpr (GP_PRE_QUADS && !LDS_OF(MODE)::kCml) pre_quads(a, L, mp, base, slot_of, st);
        else pre_pairs<W>(a, L, mp, base, slot_of, st);
        m &= ~mp;
      }
    } else if constexpr ((W == 32 || W == 16 || W == 8) && GP_PRE_GROUPS && (MODE & 3) == SCAN_PRE) {
      if (!ee) {   // four (eight) at a time (pre_groups)
        const u64 mp = m & __ballot(need && L.np[lane] != 0xFFu);
        pre_groups<W>(a, L, mp, base, slot_of, st);
        m &= ~mp;
      }
    }
    u64 sat = 0;   // receivers of this wave found sated (alive rounds)
    if constexpr (W == 64) {
      if (mdn) {   // done in-neighbours: two receivers at a time, the rest below
        const u64 md = m & mdn;
#ifndef GP_DNB_QUADS
#define GP_DNB_QUADS 1
#endif
        // (quads in the alive variants too: C5 round 5 11.95 -> 11.78 ms, but
        // round 3, the same kernel, 73.8 -> 78.7 ms, profiles/r06_ab_quads_c5.txt)
        // (in the alive SCAN_QUADS variant, which only the half-held rounds
        // launch, they pay: C5 round 5 12.2 -> 11.8 ms, r06_ab_gather_pairs.txt)
        if constexpr ((DPROBE || QUADS) && GP_DNB_QUADS) dnb_quads<ALIASABLE, ALIVE>(a, L, md, base, slot_of, st);
        else dnb_pairs<W, ALIVE, ALIASABLE>(a, L, md, base, slot_of, st);
        if constexpr (ALIVE) {   // they now hold every alive message of their component: sated too
          if (a.sate) sat |= md;
        }
        m &= ~md;
      }
    } else if constexpr ((W == 32 || W == 16 || W == 8) && GP_DNB_GROUPS) {
      if (mdn) {   // done in-neighbours, four (eight) at a time (dnb_groups)
        const u64 md = m & mdn;
        dnb_groups<W, ALIVE>(a, L, md, base, slot_of, st);
        if constexpr (ALIVE) {
          if (a.sate) sat |= md;
        }
        m &= ~md;
      }
    }
    if constexpr (GPAIRS) {   // low in-degree receivers two at a time, the rest below
      const u64 mg = m & __ballot(small);
      if (mg) {
        sat |= gather_pairs<ALIVE, ALIASABLE>(a, L, mg, base, slot_of, st);
        m &= ~mg;
      }
    }
    if constexpr (GGROUPS) {   // W = 32: low in-degree receivers four at a time
      const u64 mg = m & __ballot(small);
      if (mg) {
        gather_groups<W>(a, L, mg, base, slot_of, st);
        m &= ~mg;
      }
    }
    while (m) {
      const int k = __ffsll((long long)m) - 1;
      m &= m - 1;
      int64_t i = base + k;
      int v = uniform((int)(a.vbegin + i));
      const int64_t vb = L.rp[k];   // staged by the lane phase
      int64_t ve;
      if constexpr (LIST) {
        v = uniform(L.vid[k]);
        i = v - a.vbegin;
        ve = L.re[k];
      } else {
        ve = L.rp[k + 1];
      }
      const uint32_t sv_slot = (uint32_t)__builtin_amdgcn_readlane((int)slot_of, k);
      u64x2 acc = {0, 0}, want = {0, 0};
      // early-exit rounds: the first pass's column ids are loaded beside the
      // target's seen / component rows, one round trip instead of two
      int32_t col0 = INT32_MIN;
      if constexpr ((MODE & 3) != SCAN_MASKED && (MODE & SCAN_LINES) == 0 && (MODE & SCAN_CML) == 0) {
        if (ee && !((mdn >> k) & 1ull) && lane < (int)min((int64_t)64, ve - vb)) col0 = a.gcol[vb + lane];
      }
      // line-mask rounds (no early exit): the seen row comes up front too, beside
      // the first column ids, parked in LDS for the commit (one round trip less)
      constexpr bool SEEN_EARLY = W == 64 && (MODE & SCAN_LINES) != 0;
      if constexpr (SEEN_EARLY) {
        if (lane < (int)min((int64_t)64, ve - vb)) col0 = a.gcol[vb + lane];
        const u64x2 sv = load_seen<W>(a, v, sv_slot, lw);
        if (g == 0) {
          L.seen[2 * lw] = sv.x;
          L.seen[2 * lw + 1] = sv.y;
        }
        if (sv_slot != SLOT_NONE) st.add(S_SEEN_READ, 1);
      }
      if (ee) {
        if (sv_slot != SLOT_NONE) st.add(S_SEEN_READ, 1);
        want = early_exit_target<W, LDS_OF(MODE), ALIVE>(a, v, L, g, lw, sv_slot, L.mi[k]);
      }
      // (with alive sets a receiver may hold every alive message of its
      // component already: then there is nothing to scan)
      if (ALIVE && ee && a.alive && !__any((want.x | want.y) != 0ull)) {
        if (a.sate) sat |= 1ull << k;
      } else if ((mdn >> k) & 1ull) {   // a done in-neighbour: its Message-List is the whole target
        acc = want;
      } else if constexpr ((MODE & 3) == SCAN_PRE) {
        const uint32_t np = L.np[k];
        if (np != 0xFFu) {
          gather_rows<W>(a, L.pre[k], (int)np, g, lw, acc, st, ee, want);   // full rows
        } else {
          gather_scan<W, SCAN, false>(a, vb, vb + L.len[k], L, lane, g, lw, acc, st, ee, want, col0);
          if ((tw >> k) & 1ull) {   // degree-split: the accumulator row (not staged: a scanned receiver)
            if (g == 0) acc |= load_piece<W>(a.acc, v, lw);
            st.add(S_GATHERED, 1);
            st.add(S_ROW_BYTES, (u64)(8 * W));
          }
        }
      } else {
        gather_scan<W, SCAN, DPROBE>(a, vb, ve, L, lane, g, lw, acc, st, ee, want, col0);
      }
      reduce_slots<W>(acc);
      if constexpr (ALIVE) {   // the round's gather covered every alive message v lacked: sated
        if (a.sate && ee && a.alive) {
          const u64x2 rem = want & ~acc;
          if (!__any((rem.x | rem.y) != 0ull)) sat |= 1ull << k;
        }
      }
      if constexpr (W == 64 && (MODE & SCAN_CML) != 0) {
        if (a.cmk) {   // the gathered records (gather_scan ORs them into L.racc)
          wave_sync_lds();
          acc.x |= L.racc[2 * lw];
          acc.y |= L.racc[2 * lw + 1];
          wave_sync_lds();
          L.racc[lane] = 0ull;   // for the next receiver (read by every lane above first)
          wave_sync_lds();
        }
      }
      // alias rounds: a receiver whose gather covered its whole target now
      // holds its component's row (no liveness: want = cm & ~seen)
      bool full = false;
      if (ALIASABLE && a.alias && ee) {
        const u64x2 rem = want & ~acc;
        full = !__any((rem.x | rem.y) != 0ull);
      }
      finish_row<W, true, (MODE & SCAN_CML) != 0>(a, v, i, acc, lane, g, lw, st, L, ee || SEEN_EARLY, sv_slot, k,
                                                  full);
    }
    alive_flush<W>(a, L.alive, lane);
    commit_vertices(a, L, vi, need, st);
    if constexpr (ALIVE) {
      if (sat && ((sat >> lane) & 1ull)) a.state[a.vbegin + vi] |= ST_SATED;
    }
    // the next round's list: receivers still neither done
    // nor sated -- the set only shrinks (seenpop grows, done_at and the down /
    // sated marks only move one way), so it holds every later receiver
    if constexpr (EMIT) {
      if (a.ulist_next) {
        const bool surv = need && !((sat >> lane) & 1ull) &&
                          a.seenpop[vi] < a.done_at[a.vbegin + vi];   // (commit_vertices' sum: this lane's own write)
        const u64 sm = __ballot(surv);
        if (sm) {
          uint32_t p0 = 0;
          if (lane == 0) p0 = (uint32_t)atomicAdd(a.stats + S_ULIST, (u64)__popcll(sm));
          p0 = (uint32_t)__shfl((int)p0, 0);
          if (surv) a.ulist_next[p0 + lane_rank(sm)] = (int32_t)vi;
        }
      }
    }
  }
  flush_stats<EWAVES>(st, a.partial);
}

// ---------------------------------------------------------------------------
// edge-parallel pull for narrow rows (W <= 32: message shards, C2/C3 widths).
// The per-receiver loop of k_expand pays several dependent memory round trips
// per receiver, which narrow rows cannot amortise.  Here a wave streams the
// in-arcs of all its (non-hub) receivers as one flat sequence: QA chunks of 64
// arcs have their column ids and activity probes in flight together, the
// active rows are gathered RPI per wave-instruction whatever receiver they
// belong to, and OR-ed into per-receiver accumulators in LDS (ds_or_b64).  The
// receiver side then runs lane-parallel, one receiver per lane.  No early exit
// (narrow rows are cheap next to the arc scan).
constexpr int FLAT_CAP = 512;   // arc positions per owner window
// row wave-instructions in flight per lane (VGPRs vs occupancy).  Measured on
// the message shards (same box A/B): W = 8 (64-B rows, 16 per instruction)
// 15.6 -> 15.2 ms with 3 against 2 for a 512-message shard (round 3 of the
// build), and 5 against 3 at HEAD of round 5 (72 against 76 VGPRs; 4 takes 90):
// ranks 7 / 0 of the N = 8 job 12.12 -> 11.83 / 10.47 -> 10.16 ms
// (profiles/r05_ab_flat_w8.txt; forcing 8 waves per SIMD at 64 VGPRs was
// slower, 12.0-12.2 ms); W = 16 28.3 -> 24.4 ms with 4 and 22.9 ms with 6 for
// a 1024-message shard (8: 25.6).  W < 8: 3 (5 costs W = 1 16 VGPRs)
#ifndef GP_FLAT_RIF_NARROW
#define GP_FLAT_RIF_NARROW 5
#endif
#ifndef GP_FLAT_RIF_WIDE
#define GP_FLAT_RIF_WIDE 6
#endif
template <int W>
struct FlatRIF { static constexpr int value = W >= 16 ? GP_FLAT_RIF_WIDE : W == 8 ? GP_FLAT_RIF_NARROW : 3; };
// receivers per wave: 64, or 32 at W = 32 so that the LDS accumulators (8 KB
// per wave) leave room for 4 blocks per CU
template <int W>
struct FlatNR { static constexpr int value = W >= 32 ? 32 : 64; };
template <int W>
struct FlatLds {
  static constexpr int NR = FlatNR<W>::value;
  u64 acc[NR][W];               // OR accumulators of the wave's NR receivers
  // the passes' staging and the receiver side's words share their bytes (the
  // receiver side starts after the last pass): W = 8 takes 4,928 B + 176 B
  // of counters, so LDS no longer caps its waves (VGPRs do: 7 per SIMD)
  union {
    struct {
      int32_t idx[64];          // active neighbours of one chunk
      int8_t vtx[64];           // their receiver (lane) in the wave
      int8_t own[FLAT_CAP];     // receiver lane owning each arc position of the window
    };
    struct {
      uint16_t tot[NR];         // receiver side: new bits of receiver k (<= 64 W)
      u64 dig[NR];              // its digest terms
      int8_t rd[NR];            // between passes: still missing messages; receiver side: its seen row was read
      u64 alive[W];             // receiver side: OR of the new rows this wave wrote (alive_next)
    };
  };
};

// one flat pass: the arcs [start, start + sdeg) of every lane's receiver, as
// one sequence (owner windows of FLAT_CAP positions), OR-ed into F.acc.
// Returns the rows gathered.
template <int W, int MODE>
__device__ __forceinline__ u64 flat_pass(const ExpandArgs& a, FlatLds<W>& F, int lane, int g, int lw,
                                         uint32_t sdeg, int64_t start, WaveStats& st) {
  constexpr int RPI = Geo<W>::RPI;
  constexpr int WPL = Geo<W>::WPL;
  constexpr int QA = 4;
  constexpr int RIF = FlatRIF<W>::value;
  const uint32_t excl = wave_excl_scan_u32(sdeg, lane);
  const uint32_t incl = excl + sdeg;
  const uint32_t T = (uint32_t)__shfl((int)incl, 63);
  const uint32_t vb_lo = (uint32_t)start, vb_hi = (uint32_t)((u64)start >> 32);
  st.add(S_ARCS, T);
  u64 gathered = 0;
  for (uint32_t g0 = 0; g0 < T; g0 += FLAT_CAP) {
    const uint32_t wn = min((uint32_t)FLAT_CAP, T - g0);
    // owner table of positions [g0, g0 + wn): start markers, then a forward
    // fill seeded with the receiver that straddles g0
    {
      u64* own8 = reinterpret_cast<u64*>(F.own);
      own8[lane] = 0xFFFFFFFFFFFFFFFFull;
      wave_sync_lds();
      if (sdeg && excl >= g0 && excl < g0 + wn) F.own[excl - g0] = (int8_t)lane;
      const u64 before = __ballot(sdeg && excl < g0);
      const int carry_in = before ? 63 - __clzll((long long)before) : -1;
      wave_sync_lds();
      const u64 w8 = own8[lane];
      int run = -1;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int o = (int8_t)((w8 >> (8 * q)) & 0xFF);
        if (o >= 0) run = o;
      }
      int carry = run;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(carry, o);
        if (lane >= o) carry = max(carry, y);
      }
      int cur = __shfl_up(carry, 1);
      if (lane == 0) cur = carry_in;
      cur = max(cur, carry_in);
      u64 out = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int o = (int8_t)((w8 >> (8 * q)) & 0xFF);
        if (o >= 0) cur = o;
        out |= (u64)(uint8_t)(int8_t)cur << (8 * q);
      }
      own8[lane] = out;
      wave_sync_lds();
    }
    for (uint32_t c0 = 0; c0 < wn; c0 += 64 * QA) {
      int32_t col[QA];
      int8_t who[QA];
#pragma unroll
      for (int q = 0; q < QA; ++q) {
        const uint32_t p = c0 + (uint32_t)(q * 64 + lane);
        const int j = p < wn ? (int)F.own[p] : 0;
        // shuffles with the whole wave active (bpermute reads every lane)
        const int64_t b = (int64_t)(((u64)(uint32_t)__shfl((int)vb_hi, j) << 32) |
                                    (u64)(uint32_t)__shfl((int)vb_lo, j));
        const uint32_t s = (uint32_t)__shfl((int)excl, j);
        who[q] = (int8_t)j;
        col[q] = -1;
        if (p < wn) col[q] = a.gcol[b + (g0 + p - s)];
      }
      u64 raw[QA];   // activity words, all in flight before the first use
#pragma unroll
      for (int q = 0; q < QA; ++q) {
        raw[q] = ~0ull;
        if constexpr (MODE != SCAN_UNFILTERED)
          if (col[q] >= 0) raw[q] = a.abits[col[q] >> 6];
      }
      if constexpr (MODE != SCAN_UNFILTERED)
        if (a.sbits) {
          u64 sw[QA];
#pragma unroll
          for (int q = 0; q < QA; ++q) sw[q] = col[q] >= 0 ? a.sbits[col[q] >> 12] : 0ull;
#pragma unroll
          for (int q = 0; q < QA; ++q)
            raw[q] = ((sw[q] >> ((col[q] >> 6) & 63)) & 1ull) ? a.abits[col[q] >> 6] : 0ull;
        }
#pragma unroll
      for (int q = 0; q < QA; ++q) {
        const int32_t u = (col[q] >= 0 && ((raw[q] >> (col[q] & 63)) & 1ull)) ? col[q] : -1;
        const u64 am = __ballot(u >= 0);
        const int cnt = __popcll(am);
        if (cnt == 0) continue;
        if (u >= 0) {
          const int r = lane_rank(am);
          F.idx[r] = u;
          F.vtx[r] = who[q];
        }
        wave_sync_lds();
        gathered += (u64)cnt;
        for (int k0 = 0; k0 < cnt; k0 += RIF * RPI) {
          u64x2 r[RIF];
#pragma unroll
          for (int t = 0; t < RIF; ++t) {
            const int k = k0 + g + t * RPI;
            r[t] = u64x2{0, 0};
            if (k < cnt) r[t] = load_piece<W>(a.rows, F.idx[k], lw);
          }
#pragma unroll
          for (int t = 0; t < RIF; ++t) {
            const int k = k0 + g + t * RPI;
            if (k < cnt) {
              u64* dst = &F.acc[F.vtx[k]][lw * WPL];
              if (r[t].x) atomicOr(dst, r[t].x);
              if constexpr (WPL == 2) {
                if (r[t].y) atomicOr(dst + 1, r[t].y);
              }
            }
          }
        }
        wave_sync_lds();
      }
    }
  }
  return gathered;
}

// early-exit rounds: the first GP_FLAT_EE_PREFIX arcs of every
// receiver (its biggest neighbours: gather order) go in a first pass; only
// receivers still missing messages of their component after it scan further
// (a second prefix pass of 8 arcs measured no better, §3.7).
#ifndef GP_FLAT_EE_PREFIX
#define GP_FLAT_EE_PREFIX 2
#endif

template <int W, int MODE, bool EE>
__global__ __launch_bounds__(EBLOCK) void k_expand_flat(ExpandArgs a) {
  constexpr int LPR = Geo<W>::LPR;
  constexpr int RPI = Geo<W>::RPI;
  constexpr int WPL = Geo<W>::WPL;
  __shared__ FlatLds<W> s_f[EWAVES];
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  const int g = lane / LPR, lw = lane % LPR;
  FlatLds<W>& F = s_f[wib];
  constexpr int NR = FlatNR<W>::value;
  WaveStats st;
  ws_zero<EWAVES>(st);
  const int64_t base = ((int64_t)blockIdx.x * EWAVES + wib) * NR;
  if (base < a.nloc) {
    // per-lane state is reloaded (coalesced) where it is needed rather than
    // kept live across the passes: VGPRs are what bound this kernel's waves
    const int64_t li = base + lane;
    const bool mine = lane < NR && li < a.nloc;   // lane = receiver
    const int v = mine ? (int)(a.vbegin + li) : 0;
    u64 needm;
    {
      bool need = false, act = false;
      u64 sends = 0;
      if (mine) {
        const uint32_t fp = a.fpop[v];
        act = fp != 0u;
        if (act) sends = (u64)fp * (u64)(uint32_t)max(a.deg_live[v], 0);
        const int64_t b = a.row_ptr[v], e = a.row_ptr[v + 1];
        const bool hub = e - b > a.hub_thr;   // split over waves by the hub kernels
        need = !(a.state[v] & (ST_DOWN | ST_SATED)) && a.seenpop[li] < a.done_at[v] && !hub && e > b;
        if (!need && !hub) a.fpop_next[v] = 0;
      }
      st.add(S_SENDS, wave_sum_u64(sends));
      st.add(S_ACTIVE, (u64)__popcll(__ballot(act)));
      needm = __ballot(need);
      st.add(S_VISITED, (u64)__popcll(needm));
    }
    const bool need = (needm >> lane) & 1ull;
    // degree-split rounds: the receivers the push half touched (bit r =
    // receiver base + r; NR = 32 waves take their half of the 64-vertex word)
    u64 tw = 0;
    if (a.prehi) {
      tw = a.tbits[base >> 6] >> (base & 63);
      if constexpr (NR < 64) tw &= (1ull << NR) - 1ull;
    }
    // (a wave with no receiver to scan is done: late rounds leave most waves
    // with none, and the passes and the receiver side cost latency even empty)
    if (needm != 0ull) {
    if (lane < NR) {
#pragma unroll
      for (int w = 0; w < W; ++w) F.acc[lane][w] = 0ull;
    }
    // one pass, or (early-exit rounds) a prefix pass and a pass over the rest
    // of the in-lists of the receivers still missing messages
    constexpr uint32_t K1 = GP_FLAT_EE_PREFIX, K2 = 0;
    constexpr bool ee = EE && K1 > 0;   // compile-time: the lean kernel keeps its VGPRs
    constexpr int npass = !ee ? 1 : 2;
    u64 gathered = 0;
    u64 todo = needm;   // receivers of this pass
#pragma nounroll
    for (int pass = 0; pass < npass; ++pass) {
      // this pass covers in-list positions [lo, hi)
      const uint32_t lo = pass == 0 ? 0u : pass == 1 ? K1 : K2;
      const uint32_t hi = pass + 1 == npass ? 0xFFFFFFFFu : pass == 0 ? K1 : K2;
      uint32_t sdeg = 0;
      int64_t start = 0;
      if ((todo >> lane) & 1ull) {
        const int64_t b = a.row_ptr[v], e = a.row_ptr[v + 1];
        // (degree-split rounds, no early exit: the prefix of bigger senders)
        const uint32_t deg = a.prehi ? (uint32_t)a.prehi[v] : (uint32_t)(e - b);
        sdeg = deg > lo ? min(deg, hi) - lo : 0u;
        start = b + lo;
      }
      gathered += flat_pass<W, MODE>(a, F, lane, g, lw, sdeg, start, st);
      if (pass + 1 == npass) break;
      // which receivers with arcs left still miss messages of their component?
      bool longer = false;
      uint32_t slot_of = SLOT_NONE;
      int32_t mrow = -1;
      if ((todo >> lane) & 1ull) {
        longer = a.row_ptr[v + 1] - a.row_ptr[v] > (int64_t)hi;
        if (longer) {
          slot_of = a.sp[v];
          mrow = a.midx[v];
        }
      }
      const u64 longm = __ballot(longer);
      wave_sync_lds();
#pragma nounroll
      for (int r0 = 0; r0 < NR; r0 += RPI) {
        const int r = r0 + g;
        const uint32_t rslot = (uint32_t)__shfl((int)slot_of, r);
        const int rv = __shfl(v, r);
        const int32_t rm = __shfl(mrow, r);
        bool miss = false;
        if ((longm >> r) & 1ull) {
          u64x2 accp;
          accp.x = F.acc[r][lw * WPL];
          accp.y = 0;
          if constexpr (WPL == 2) accp.y = F.acc[r][lw * WPL + 1];
          const u64x2 sv = rslot != SLOT_NONE ? load_piece<W>(a.slot[rslot], rv, lw) : u64x2{0, 0};
          u64x2 cm = load_piece<W>(a.cmask, rm, lw);
          if (a.alive) cm &= load_piece<W>(a.alive, 0, lw);
          const u64x2 m = cm & ~(sv | accp);
          miss = (m.x | m.y) != 0ull;
        }
        miss = group_or<LPR>(miss);
        if (lw == 0) F.rd[r] = (int8_t)miss;
      }
      wave_sync_lds();
      todo = __ballot(((longm >> lane) & 1ull) && F.rd[lane]);
    }
    const u64 tn = (u64)__popcll(tw & needm);   // accumulator rows read by the receiver side
    st.add(S_GATHERED, gathered + tn);
    st.add(S_ROW_BYTES, (gathered + tn) * (u64)(8 * W));
    // receiver side: RPI receivers per wave-instruction, LPR lanes x 16 B per
    // row (coalesced, like the gather); a receiver with nothing new reads and
    // writes nothing.  Per-receiver words go to F.tot / F.dig, then one
    // coalesced commit with one receiver per lane.
    wave_sync_lds();
    alive_zero<W>(a, F.alive, lane);   // (shares its bytes with the passes' staging)
    wave_sync_lds();
    const uint32_t slot_of = need ? a.sp[v] : SLOT_NONE;
    for (int r0 = 0; r0 < NR; r0 += RPI) {
      const int r = r0 + g;
      const uint32_t rslot = (uint32_t)__shfl((int)slot_of, r);
      const int rv = __shfl(v, r);
      const bool rn = (needm >> r) & 1ull;
      u64x2 accp = {0, 0};
      if (rn) {
        accp.x = F.acc[r][lw * WPL];
        if constexpr (WPL == 2) accp.y = F.acc[r][lw * WPL + 1];
        if ((tw >> r) & 1ull) accp |= load_piece<W>(a.acc, rv, lw);   // degree-split: the pushed rows
      }
      const bool any = group_or<LPR>((accp.x | accp.y) != 0ull);
      u64x2 sv = {0, 0};
      if (any && rslot != SLOT_NONE) sv = load_piece<W>(a.slot[rslot], rv, lw);
      const u64x2 nw = accp & ~sv;
      const uint32_t tot = group_sum<LPR>((uint32_t)(__popcll(nw.x) + __popcll(nw.y)));
      u64 t = 0;
      if (tot) {
        alive_add<W>(a, F, lw, nw);
        store_piece<W>(a.slot[a.wslot], rv, lw, sv | nw);
        if (a.frx_next) store_piece<W>(a.frx_next, rv, lw, nw);
        if (a.first) {
          uint8_t* row = a.first + (size_t)(base + r) * (W * 64);
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
        F.tot[r] = tot;
        F.dig[r] = t;
        F.rd[r] = (int8_t)(any && rslot != SLOT_NONE);
      }
    }
    wave_sync_lds();
    u64 nbits = 0, nrecv = 0, nwritten = 0, narcs = 0, nseen = 0;
    if (need) {
      const uint32_t tot = F.tot[lane];
      nseen = (u64)F.rd[lane];
      a.fpop_next[v] = tot;
      if (tot) {
        a.seenpop[li] += tot;
        a.sp[v] = (uint8_t)a.wslot;
        a.ws[v] |= (uint8_t)(1u << a.wslot);
        if (a.digest) a.digest[li] ^= F.dig[lane];
        nbits = tot;
        nrecv = 1;
        nwritten = 1;
        narcs = (u64)(uint32_t)max(a.deg_live[v], 0);
      }
    }
    st.add(S_NEW_BITS, wave_sum_u64(nbits));
    st.add(S_RECEIVERS, wave_sum_u64(nrecv));
    st.add(S_WRITTEN, wave_sum_u64(nwritten));
    st.add(S_NEXT_ARCS, wave_sum_u64(narcs));
    st.add(S_SEEN_READ, wave_sum_u64(nseen));
    alive_flush<W>(a, F.alive, lane);
    }   // needm
  }
  flush_stats<EWAVES>(st, a.partial);
}

// ---------------------------------------------------------------------------
// Record pull (W = 64, compact Message-Lists read, no early exit: C4's round
// 2 with compact_rows).  The per-receiver loop of k_expand gathers records one
// receiver at a time, a chain of dependent round trips per receiver that the
// 128-B records cannot amortise (round 2: row bytes halve, time does not
// move).  Here a wave streams the in-arcs of REC_NR receivers as one flat
// sequence: column ids and probes of 64 arcs at a time, then the active
// sparse senders' records 8 per wave-instruction (8 lanes x 16 B, REC_RIF
// instructions in flight) and the dense senders' full rows 2 per
// instruction, every word OR-ed into its receiver's 512-B accumulator in LDS
// (ds_or_b64; a record's word p >= 1 goes to word select_bit(mask, p)).  The
// receiver side runs two receivers per instruction through pair_finish
// (rows, records of the next round, first bytes, digest).
constexpr int REC_NR = 8;
#ifndef GP_REC_RIF
#define GP_REC_RIF 4
#endif
struct RecLds {
  static constexpr bool kPre = false, kCml = true;
  u64 acc[REC_NR][64];   // OR accumulators of the wave's receivers
  int32_t sid[64];       // active sparse senders of one chunk (records)
  int32_t did[64];       // active dense senders of one chunk (full rows)
  int8_t sown[64];       // their receiver
  int8_t down[64];
  uint32_t tot[REC_NR];  // pair_finish: new bits of receiver k
  uint8_t lmn[REC_NR];   // pair_finish: its line mask (record rounds write none: lm_next is null)
  u64 dig[REC_NR];       // its digest terms
  uint8_t cd[REC_NR];    // its new row is dense (no record)
  u64 alive[64];         // alive_add (unused: record rounds run without liveness alive sets too)
};

__global__ __launch_bounds__(BLOCK) void k_expand_rec(ExpandArgs a) {
  constexpr int W = 64;
  __shared__ RecLds s_r[WAVES];
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  RecLds& L = s_r[wib];
  WaveStats st;
  ws_zero(st);
  const int64_t base = ((int64_t)blockIdx.x * WAVES + wib) * REC_NR;
  if (base < a.nloc) {
    const int64_t li = base + lane;
    const bool mine = lane < REC_NR && li < a.nloc;
    const int v = mine ? (int)(a.vbegin + li) : 0;
    bool need = false, act = false;
    u64 sends = 0;
    int64_t b = 0;
    uint32_t deg = 0;
    if (mine) {
      const uint32_t fp = a.fpop[v];
      act = fp != 0u;
      if (act) sends = (u64)fp * (u64)(uint32_t)max(a.deg_live[v], 0);
      b = a.row_ptr[v];
      const int64_t e = a.row_ptr[v + 1];
      const bool hub = e - b > a.hub_thr;   // split over waves by the hub kernels
      need = !(a.state[v] & (ST_DOWN | ST_SATED)) && a.seenpop[li] < a.done_at[v] && !hub && e > b;
      if (!need && !hub) a.fpop_next[v] = 0;
      if (need) deg = (uint32_t)(e - b);
    }
    st.add(S_SENDS, wave_sum_u64(sends));
    st.add(S_ACTIVE, (u64)__popcll(__ballot(act)));
    const u64 needm = __ballot(need);
    st.add(S_VISITED, (u64)__popcll(needm));
    if (lane < REC_NR) {
      L.tot[lane] = 0u;
      L.dig[lane] = 0ull;
      L.cd[lane] = 1;
    }
    alive_zero<W>(a, L.alive, lane);
    u64 gathered = 0, rbytes = 0;
    if (needm) {
#pragma unroll
      for (int q = 0; q < REC_NR; ++q) L.acc[q][lane] = 0ull;
      wave_sync_lds();
      const uint32_t excl = wave_excl_scan_u32(deg, lane);
      const uint32_t T = (uint32_t)__shfl((int)(excl + deg), 63);
      const uint32_t blo = (uint32_t)b, bhi = (uint32_t)((u64)b >> 32);
      st.add(S_ARCS, T);
      const int gq = lane >> 3, sl = lane & 7;     // record lanes: 8 records per instruction
      const int h = lane >> 5, lw = lane & 31;     // row lanes: 2 rows per instruction
      for (uint32_t c0 = 0; c0 < T; c0 += 64) {
        const uint32_t p = c0 + (uint32_t)lane;
        int own = -1;
#pragma unroll
        for (int r = 0; r < REC_NR; ++r) {
          const uint32_t er = (uint32_t)__shfl((int)excl, r), dr = (uint32_t)__shfl((int)deg, r);
          if (dr && p >= er && p < er + dr) own = r;
        }
        const int src = own >= 0 ? own : 0;
        const int64_t bo = (int64_t)(((u64)(uint32_t)__shfl((int)bhi, src) << 32) | (u64)(uint32_t)__shfl((int)blo, src));
        const uint32_t eo = (uint32_t)__shfl((int)excl, src);
        int32_t u = -1;
        bool dense = false;
        if (p < T && own >= 0) {
          u = a.gcol[bo + (int64_t)(p - eo)];
          if (((a.abits[u >> 6] >> (u & 63)) & 1ull) == 0ull) u = -1;
          else dense = ((a.cmk[u >> 6] >> (u & 63)) & 1ull) != 0ull;
        }
        const u64 ms = __ballot(u >= 0 && !dense), md = __ballot(u >= 0 && dense);
        if (u >= 0) {
          if (dense) {
            L.did[lane_rank(md)] = u;
            L.down[lane_rank(md)] = (int8_t)own;
          } else {
            L.sid[lane_rank(ms)] = u;
            L.sown[lane_rank(ms)] = (int8_t)own;
          }
        }
        wave_sync_lds();
        const int ns = __popcll(ms), nd = __popcll(md);
        gathered += (u64)(ns + nd);
        rbytes += (u64)ns * (8 * CML_WORDS) + (u64)nd * (8 * W);
        for (int k0 = 0; k0 < ns; k0 += 8 * GP_REC_RIF) {
          u64x2 rv[GP_REC_RIF];
#pragma unroll
          for (int t = 0; t < GP_REC_RIF; ++t) {
            const int k = k0 + t * 8 + gq;
            rv[t] = u64x2{0, 0};
            if (k < ns) rv[t] = *reinterpret_cast<const u64x2*>(a.cml + (size_t)L.sid[k] * CML_WORDS + 2 * sl);
          }
#pragma unroll
          for (int t = 0; t < GP_REC_RIF; ++t) {
            const int k = k0 + t * 8 + gq;
            const u64 mask = __shfl(rv[t].x, lane & ~7);   // word 0 of the record: its word mask
            if (k < ns) {
              const int c = __popcll(mask);
              u64* acc = L.acc[L.sown[k]];
              if (sl > 0 && 2 * sl <= c && rv[t].x) atomicOr(&acc[select_bit(mask, 2 * sl)], rv[t].x);
              if (2 * sl + 1 <= c && rv[t].y) atomicOr(&acc[select_bit(mask, 2 * sl + 1)], rv[t].y);
            }
          }
        }
        for (int k0 = 0; k0 < nd; k0 += 4) {
          u64x2 r0 = u64x2{0, 0}, r1 = u64x2{0, 0};
          const int ka = k0 + h, kb = k0 + 2 + h;
          if (ka < nd) r0 = load_piece<W>(a.rows, L.did[ka], lw);
          if (kb < nd) r1 = load_piece<W>(a.rows, L.did[kb], lw);
          if (ka < nd) {
            u64* acc = L.acc[L.down[ka]];
            if (r0.x) atomicOr(&acc[2 * lw], r0.x);
            if (r0.y) atomicOr(&acc[2 * lw + 1], r0.y);
          }
          if (kb < nd) {
            u64* acc = L.acc[L.down[kb]];
            if (r1.x) atomicOr(&acc[2 * lw], r1.x);
            if (r1.y) atomicOr(&acc[2 * lw + 1], r1.y);
          }
        }
        wave_sync_lds();
      }
    }
    st.add(S_GATHERED, gathered);
    st.add(S_ROW_BYTES, rbytes);
    // receiver side: two receivers per instruction, a half-wave per row
    const int h = lane >> 5, lw = lane & 31;
    const uint32_t slot_of = need ? (uint32_t)a.sp[v] : SLOT_NONE;
    wave_sync_lds();
    if (needm) {
      for (int k0 = 0; k0 < REC_NR; k0 += 2) {
        const int ks = k0 + h;
        const bool on = ((needm >> ks) & 1ull) != 0ull;
        const int vs = __shfl(v, ks);
        const uint32_t sslot = (uint32_t)__shfl((int)slot_of, ks);
        u64x2 acc = u64x2{0, 0};
        if (on) {
          acc.x = L.acc[ks][2 * lw];
          acc.y = L.acc[ks][2 * lw + 1];
        }
        const u64x2 sv = pair_seen<W>(a, h, lw, on, k0 + 1, vs, sslot, acc, st);
        pair_finish<W>(a, L, h, lw, on, ks, k0 + 1, base + ks, vs, acc, sv, st);
      }
    }
    wave_sync_lds();
    u64 next_arcs = 0;
    if (need) {
      const uint32_t tot = L.tot[lane];
      a.fpop_next[v] = tot;
      if (tot) {
        a.seenpop[li] += tot;
        a.sp[v] = (uint8_t)a.wslot;
        a.ws[v] |= (uint8_t)(1u << a.wslot);
        if (a.digest) a.digest[li] ^= L.dig[lane];
        next_arcs = (u64)(uint32_t)max(a.deg_live[v], 0);
      }
    }
    st.add(S_NEXT_ARCS, wave_sum_u64(next_arcs));
    if (a.cmk_next) {   // this wave's bits of the next round's dense bitmap (1: read the full row)
      const u64 dm = __ballot(mine && (!need || L.tot[lane] == 0u || L.cd[lane] != 0));
      const u64 mm = __ballot(mine);
      if (lane == 0) {
        const int sh = (int)(base & 63);
        u64* wd = a.cmk_next + (base >> 6);
        if (dm) atomicOr(wd, dm << sh);
        if (mm & ~dm) atomicAnd(wd, ~((mm & ~dm) << sh));
      }
    }
    alive_flush<W>(a, L.alive, lane);
  }
  flush_stats(st, a.partial);
}

// line masks of this round's senders (SCAN_LINES, W = 64): lm[v] = the 128-B
// lines of v's row in `rows` that hold a nonzero word, 0 for non-senders.  A
// wave takes 64 vertices; their senders' rows are read two per
// wave-instruction (a half-wave per row, 8 lanes per line), 4 instructions in
// flight; the 64 bytes are stored at once
__global__ __launch_bounds__(BLOCK) void k_mklm(const uint32_t* __restrict__ fpop, const u64* __restrict__ rows,
                                                int64_t n, uint8_t* __restrict__ lm, u64* __restrict__ partial) {
  const int lane = threadIdx.x & 63, h = lane >> 5, lw = lane & 31;
  __shared__ uint8_t s_lm[WAVES][64];
  uint8_t* out = s_lm[threadIdx.x >> 6];
  WaveStats st;
  ws_zero(st);
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t v0 = (int64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63); v0 < n; v0 += stride) {
    const int64_t v = v0 + lane;
    u64 m = __ballot(v < n && fpop[v] != 0u);
    st.add(S_LM_ROWS, (u64)__popcll(m));
    out[lane] = 0;
    wave_sync_lds();
    while (m) {
      int k[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {   // 4 pairs: rows k[2p] (half 0), k[2p + 1] (half 1)
        k[q] = -1;
        if (m) {
          k[q] = __ffsll((long long)m) - 1;
          m &= m - 1;
        }
      }
      u64x2 r[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int kk = h ? k[2 * p + 1] : k[2 * p];
        r[p] = kk >= 0 ? load_piece<64>(rows, (int)(v0 + kk), lw) : u64x2{0, 0};
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const u64 b = __ballot((r[p].x | r[p].y) != 0ull);
        const int kk = h ? k[2 * p + 1] : k[2 * p];
        if (lw == 0 && kk >= 0) {
          const uint32_t hb = (uint32_t)(b >> (32 * h));
          uint8_t l = 0;
#pragma unroll
          for (int t = 0; t < 4; ++t) l |= ((hb >> (8 * t)) & 0xFFu) ? (uint8_t)(1u << t) : (uint8_t)0;
          out[kk] = l ? l : (uint8_t)0x0F;   // (a sender whose row reads zero: load it whole)
        }
      }
    }
    wave_sync_lds();
    {   // (v0 is a multiple of 64: whole bytes per wave)
      if (lane < 32 && v0 + 2 * lane < n)
        lm[(v0 >> 1) + lane] = (uint8_t)(out[2 * lane] | (out[2 * lane + 1] << 4));
    }
    wave_sync_lds();
  }
  flush_stats(st, partial);
}

// per-arc activity mask of a filtered pull round: bit j of
// amask[k] says whether sender gcol[64k + j] is active.  Probing here, with
// no row stream evicting it, keeps the 2 MB activity bitmap L2-resident; the
// pull then skips inactive arcs, and vertices without an active in-arc,
// without loading their column ids.  AM_WORDS mask words per wave, over the
// mask words [kbeg, kbeg + grid) covering the owned vertices' arcs.
constexpr int AM_WORDS = 4;
__global__ __launch_bounds__(BLOCK) void k_arcmask(const int32_t* __restrict__ gcol, const u64* __restrict__ abits,
                                                   u64* __restrict__ amask, int64_t kbeg, int64_t nnz) {
  const int lane = threadIdx.x & 63;
  const int64_t k0 = kbeg + ((int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6)) * AM_WORDS;
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
  // one writer lane per word: selecting the four ballots into lanes 0-3 and
  // storing from there (one dwordx2 store per wave) produced wrong words for
  // the third ballot on gfx950, a few per 10^5 (found by scripts/debug_mask2.py)
#pragma unroll
  for (int q = 0; q < AM_WORDS; ++q) {
    const u64 m = __ballot(u[q] >= 0 && ((w[q] >> (u[q] & 63)) & 1ull));
    if (lane == 0 && (k0 + q) * 64 < nnz) amask[k0 + q] = m;
  }
}

// unfiltered rounds: every in-neighbour row of S[r & 1] is
// read, so each must be a subset of its vertex's Message-List -- true for
// every row written this run (seen rows only grow).  Rows of inactive vertices
// whose slot was not written this run hold data of an earlier run: zero them.
// One wave per 64-vertex bitmap word; fully active words cost two loads.
// (Only without liveness: a crashed vertex may hold bits it never sent.)
// Materialize aliased Message-Lists (SLOT_CMASK): write the
// component row of every aliased vertex (with abits: of this round's senders
// only, before a push round reads them -- the 2 MB activity bitmap first, the
// slot bytes of its set bits only) into S[cur] and point sp there.  One wave
// per 64 vertices, a row per aliased vertex in one coalesced store.
__global__ __launch_bounds__(BLOCK) void k_unalias(uint8_t* __restrict__ sp, uint8_t* __restrict__ ws,
                                                   const u64* __restrict__ abits, const int32_t* __restrict__ midx,
                                                   const u64* __restrict__ cmask, u64* __restrict__ rows,
                                                   int32_t cur, int64_t n, int32_t W) {
  const int lane = threadIdx.x & 63;
  for (int64_t w = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6); w * 64 < n; w += (int64_t)gridDim.x * WAVES) {
    const int64_t v = w * 64 + lane;
    const u64 sel = abits ? abits[w] : ~0ull;
    if (sel == 0ull) continue;
    const bool al = v < n && ((sel >> lane) & 1ull) && sp[v] == SLOT_CMASK;
    u64 todo = __ballot(al);
    if (al) {
      sp[v] = (uint8_t)cur;
      ws[v] |= (uint8_t)(1u << cur);
    }
    while (todo) {
      const int b = __ffsll((long long)todo) - 1;
      todo &= todo - 1;
      const int64_t u = w * 64 + b;
      const int32_t k = midx[u];
      if (lane < W) rows[(size_t)u * W + lane] = cmask[(size_t)k * W + lane];
    }
  }
}

int unalias(Ctx* c, bool senders_only) {
  if (!c->alias_active) return 0;
  hipLaunchKernelGGL(k_unalias, dim3(std::min(grid_for((c->n_alloc + 63) / 64, WAVES), c->cu_count * 8 * GS)),
                     dim3(BLOCK), 0, c->stream, c->d_sp, c->d_ws, senders_only ? c->d_abits : nullptr,
                     c->d_midx, c->d_cmask, c->d_slot[c->cur], c->cur, c->n_alloc, c->words);
  GP_HIP(hipGetLastError());
  if (!senders_only) c->alias_active = false;
  return 0;
}

template <int W>
__global__ __launch_bounds__(BLOCK) void k_fixup_rows(const u64* __restrict__ abits, uint8_t* __restrict__ ws,
                                                      u64* __restrict__ rows, int32_t rslot, int64_t n_alloc) {
  const int lane = threadIdx.x & 63;
  // grid-stride: one wave per 64 vertices as its own launch unit was wave-
  // dispatch-bound (0.39 ms at 2^26 for ~130 MB of bytes)
  for (int64_t w = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6); w * 64 < n_alloc;
       w += (int64_t)gridDim.x * WAVES) {
    const int64_t v0 = w * 64 + lane;
    const bool stale = v0 < n_alloc && !((abits[w] >> lane) & 1ull) && !((ws[v0] >> rslot) & 1u);
    u64 todo = __ballot(stale);
    if (stale) ws[v0] |= (uint8_t)(1u << rslot);
    while (todo) {
      const int b = __ffsll((long long)todo) - 1;
      todo &= todo - 1;
      if (lane < W) rows[(size_t)(w * 64 + b) * W + lane] = 0ull;
    }
  }
}

// Parking (before an unfiltered pull under liveness): a down vertex's row may
// hold bits it never sent (it crashed with them) and the unfiltered pull would
// forward them, so its row moves to slot 2 and both read-slot rows are zeroed.
// One wave per 64 vertices; rows stay parked for the rest of the run.
template <int W>
__global__ __launch_bounds__(BLOCK) void k_park(const uint8_t* __restrict__ state, uint8_t* __restrict__ sp,
                                                u64* __restrict__ s0, u64* __restrict__ s1, u64* __restrict__ s2,
                                                int64_t n_alloc) {
  const int lane = threadIdx.x & 63;
  for (int64_t w = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6); w * 64 < n_alloc;
       w += (int64_t)gridDim.x * WAVES) {
    const int64_t v0 = w * 64 + lane;
    uint32_t p = SLOT_NONE;
    if (v0 < n_alloc && (state[v0] & ST_DOWN)) p = sp[v0];
    const bool move = p < 2u;
    u64 todo = __ballot(move);
    if (move) sp[v0] = SLOT_PARKED;
    while (todo) {
      const int b = __ffsll((long long)todo) - 1;
      todo &= todo - 1;
      const uint32_t q = (uint32_t)__shfl((int)p, b);
      if (lane < W) {
        const size_t i = (size_t)(w * 64 + b) * W + lane;
        s2[i] = (q ? s1 : s0)[i];
        s0[i] = 0ull;
        s1[i] = 0ull;
      }
    }
  }
}

// the first aliasing round (alias without the done probe) runs the quads
// variant of the unfiltered pull (done-neighbour receivers four at a time,
// low in-degree ones two at a time), and so do the other unfiltered pulls
// once most messages are held: near-done rounds without liveness
// (GP_NEAR_QUADS) and, under liveness, the alive early-exit pulls from the
// round that starts with half the messages held (GP_ALIVE_QUADS: C5 rounds
// 4-5; round 3, the dense one, keeps the plain alive variant)
#ifndef GP_ALIAS_QUADS
#define GP_ALIAS_QUADS 1
#endif
#ifndef GP_NEAR_QUADS
#define GP_NEAR_QUADS 1
#endif
#ifndef GP_ALIVE_QUADS
#define GP_ALIVE_QUADS 1
#endif
template <int W>
static void launch_expand_w(Ctx* c, ExpandArgs a) {
  if (c->mode_push) {
    launch_push_w<W>(c, a);
    return;
  }
  const int64_t per_block = (int64_t)EWAVES * 64;   // k_expand
  if (a.unfiltered && c->liveness_active)
    hipLaunchKernelGGL(k_park<W>, dim3(std::min(grid_for((c->n_alloc + 63) / 64, WAVES), c->cu_count * 8 * GS)),
                       dim3(BLOCK), 0, c->stream,
                       c->d_state, c->d_sp, c->d_slot[0], c->d_slot[1], c->d_slot[2], c->n_alloc);
  if (a.unfiltered)
    hipLaunchKernelGGL(k_fixup_rows<W>, dim3(std::min(grid_for((c->n_alloc + 63) / 64, WAVES), c->cu_count * 8 * GS)),
                       dim3(BLOCK), 0, c->stream,
                       c->d_abits, c->d_ws, c->d_slot[c->cur], c->cur, c->n_alloc);
  // W = 32 rows take the per-receiver kernel.  GP_FLAT_ND = 1 sends dense
  // near-done rounds (most messages held, last round's new bits >= m/4 per
  // vertex) to the flat kernel, whose 2-arc prefix pass completes most
  // receivers from their hub rows: that won (2048-message shard round 4:
  // 10.2 -> 6.6 ms) until the per-receiver kernel took done-neighbour and low
  // in-degree receivers four per step (dnb_groups, gather_groups): N = 2
  // slow rank's round 4 7.1 -> 4.7 ms, the other rank's 3.78 -> 0.95 ms with
  // it off (profiles/r06_ab_w32_groups.txt)
#ifndef GP_FLAT_ND
#define GP_FLAT_ND 0
#endif
  const bool flat_nd = GP_FLAT_ND && W == 32 && c->cfg.flat_max_words > 0 && a.near_done &&
                       (double)c->prev_new_bits * 4.0 >= (double)c->n * (double)c->m;
  const bool flat = W <= 32 && (W <= c->cfg.flat_max_words || flat_nd) && !c->narrow_pr_now;
  const bool masked = !a.unfiltered && !flat && c->arc_mask_now;
  if (masked) {   // mask words of the owned vertices' in-arcs
    const int64_t kb = c->h_row_ptr[0] >> 6;
    const int64_t ke = (c->h_row_ptr[(size_t)c->nloc()] + 63) >> 6;
    if (ke > kb)
      hipLaunchKernelGGL(k_arcmask, dim3(grid_for(ke - kb, (int64_t)WAVES * AM_WORDS)), dim3(BLOCK), 0, c->stream,
                         c->d_gcol, c->d_abits, c->d_amask, kb, c->nnz_l);
  }
  const int mode = a.unfiltered ? SCAN_UNFILTERED : SCAN_FILTERED;
  // kernel_ms (ev[4] .. ev[5]) brackets every kernel of the round's pull: the
  // degree-split push half and accumulator clear too (their accumulator
  // updates are in the bench's algorithmic bytes, `atomics`)
  (void)hipEventRecord(c->ev[4], c->stream);
  if (a.prehi) {   // degree-split round, push half: senders of in-degree < split_deg
    launch_split_push_w<W>(c, a);
  }
  // line masks of the senders' rows (SCAN_LINES; inside the pull's events and bytes)
  const bool lines = W == 64 && a.lm != nullptr && !flat && !masked && mode == SCAN_FILTERED && !a.cmk &&
                     !a.cmk_next && !c->prefilter_now && !(a.alive && a.early_exit);

  const bool lm_from_commits = lines && a.lm != c->d_lm;
  if (lines && a.lm == c->d_lm)   // (the last round's commits did not write them)
    hipLaunchKernelGGL(k_mklm, dim3(std::max(1, std::min(grid_for(c->n_alloc, BLOCK), c->cu_count * 8 * GS))),
                       dim3(BLOCK), 0, c->stream, c->d_fpop[c->cur], a.rows, c->n_alloc, c->d_lm, a.partial);
  if (a.nloc > 0 && flat) {   // narrow rows: edge-parallel pull
    const dim3 grid(grid_for(a.nloc, (int64_t)EWAVES * FlatNR<W>::value));
    if constexpr (W <= 32) {
      const bool ee = a.early_exit != 0 && GP_FLAT_EE_PREFIX > 0;
      if (mode == SCAN_UNFILTERED) {
        if (ee) hipLaunchKernelGGL((k_expand_flat<W, SCAN_UNFILTERED, true>), grid, dim3(EBLOCK), 0, c->stream, a);
        else hipLaunchKernelGGL((k_expand_flat<W, SCAN_UNFILTERED, false>), grid, dim3(EBLOCK), 0, c->stream, a);
      } else {
        if (ee) hipLaunchKernelGGL((k_expand_flat<W, SCAN_FILTERED, true>), grid, dim3(EBLOCK), 0, c->stream, a);
        else hipLaunchKernelGGL((k_expand_flat<W, SCAN_FILTERED, false>), grid, dim3(EBLOCK), 0, c->stream, a);
      }
    }
  } else if (W == 64 && a.ulist) {   // receiver-list round (launch_expand): waves for the listed vertices
    if constexpr (W == 64) {
      const dim3 lgrid(grid_for(a.ulist_n, per_block));
      const bool unf = mode == SCAN_UNFILTERED;
      if (a.alive && a.early_exit) {
        if (unf) hipLaunchKernelGGL((k_expand<W, SCAN_UNFILTERED | SCAN_ALIVE | SCAN_LIST>), lgrid, dim3(EBLOCK), 0, c->stream, a);
        else hipLaunchKernelGGL((k_expand<W, SCAN_FILTERED | SCAN_ALIVE | SCAN_LIST>), lgrid, dim3(EBLOCK), 0, c->stream, a);
      } else if (a.dprobe) {
        if (unf) hipLaunchKernelGGL((k_expand<W, SCAN_UNFILTERED | SCAN_DPROBE | SCAN_LIST>), lgrid, dim3(EBLOCK), 0, c->stream, a);
        else hipLaunchKernelGGL((k_expand<W, SCAN_FILTERED | SCAN_DPROBE | SCAN_LIST>), lgrid, dim3(EBLOCK), 0, c->stream, a);
      } else {
        if (unf) hipLaunchKernelGGL((k_expand<W, SCAN_UNFILTERED | SCAN_LIST>), lgrid, dim3(EBLOCK), 0, c->stream, a);
        else hipLaunchKernelGGL((k_expand<W, SCAN_FILTERED | SCAN_LIST>), lgrid, dim3(EBLOCK), 0, c->stream, a);
      }
    }
  } else if (a.nloc > 0) {
    const dim3 grid(grid_for(a.nloc, per_block));
    bool alive_ee = false;   // unfiltered under liveness (parked rows) with early exit
    if constexpr (W >= 32) alive_ee = mode == SCAN_UNFILTERED && a.alive && a.early_exit;
    const bool half_held = (double)c->held_bits * 2.0 >= (double)c->n * (double)c->m;
    if (alive_ee) {
      if constexpr (W == 64) {
        if (GP_ALIVE_QUADS && half_held)
          hipLaunchKernelGGL((k_expand<W, SCAN_UNFILTERED | SCAN_ALIVE | SCAN_QUADS>), grid, dim3(EBLOCK), 0, c->stream, a);
        else
          hipLaunchKernelGGL((k_expand<W, SCAN_UNFILTERED | SCAN_ALIVE>), grid, dim3(EBLOCK), 0, c->stream, a);
      } else if constexpr (W >= 32) {
        hipLaunchKernelGGL((k_expand<W, SCAN_UNFILTERED | SCAN_ALIVE>), grid, dim3(EBLOCK), 0, c->stream, a);
      }
    } else if (W == 64 && a.dprobe) {   // (done-probe rounds: filtered or unfiltered, launch_expand)
      if constexpr (W == 64) {
        if (mode == SCAN_UNFILTERED)
          hipLaunchKernelGGL((k_expand<W, SCAN_UNFILTERED | SCAN_DPROBE>), grid, dim3(EBLOCK), 0, c->stream, a);
        else
          hipLaunchKernelGGL((k_expand<W, SCAN_FILTERED | SCAN_DPROBE>), grid, dim3(EBLOCK), 0, c->stream, a);
      }
    } else if (W >= 8 && mode == SCAN_UNFILTERED &&
               ((GP_ALIAS_QUADS && a.alias) || (GP_NEAR_QUADS && a.near_done))) {   // (the first aliasing round)
      if constexpr (W >= 8)
        hipLaunchKernelGGL((k_expand<W, SCAN_UNFILTERED | SCAN_QUADS>), grid, dim3(EBLOCK), 0, c->stream, a);
    } else if (mode == SCAN_UNFILTERED) {
      hipLaunchKernelGGL((k_expand<W, SCAN_UNFILTERED>), grid, dim3(EBLOCK), 0, c->stream, a);
    }
    else if (masked)
      hipLaunchKernelGGL((k_expand<W, SCAN_MASKED>), grid, dim3(EBLOCK), 0, c->stream, a);
    else if (W == 64 && (a.cmk || a.cmk_next)) {   // compact Message-Lists read and / or written
      if constexpr (W == 64) {
        if (a.cmk && !a.early_exit && !c->prefilter_now && !a.alive)
          hipLaunchKernelGGL(k_expand_rec, dim3(grid_for(a.nloc, (int64_t)WAVES * REC_NR)), dim3(BLOCK), 0,
                             c->stream, a);
        else if (c->prefilter_now)
          hipLaunchKernelGGL((k_expand<W, SCAN_PRE | SCAN_CML>), grid, dim3(EBLOCK), 0, c->stream, a);
        else
          hipLaunchKernelGGL((k_expand<W, SCAN_FILTERED | SCAN_CML>), grid, dim3(EBLOCK), 0, c->stream, a);
      }
    } else {
      // early-exit rounds with alive sets (liveness) take the SCAN_ALIVE
      // variants; instantiated for the widths the per-receiver kernel runs by
      // default (narrower rows take the flat kernel)
      bool done = false;
      if constexpr (W >= 32) {
        if (a.alive && a.early_exit) {
          if (c->prefilter_now)
            hipLaunchKernelGGL((k_expand<W, SCAN_PRE | SCAN_ALIVE>), grid, dim3(EBLOCK), 0, c->stream, a);
          else
            hipLaunchKernelGGL((k_expand<W, SCAN_FILTERED | SCAN_ALIVE>), grid, dim3(EBLOCK), 0, c->stream, a);
          done = true;
        }
      }
      if constexpr (W == 64) {
        if (!done && lines) {
          hipLaunchKernelGGL((k_expand<W, SCAN_FILTERED | SCAN_LINES>), grid, dim3(EBLOCK), 0, c->stream, a);
          c->lines_ran = true;
          c->lines_from_commits = lm_from_commits;
          done = true;
        }
      }
      if (done) {
      } else if (c->prefilter_now)
        hipLaunchKernelGGL((k_expand<W, SCAN_PRE>), grid, dim3(EBLOCK), 0, c->stream, a);
      else
        hipLaunchKernelGGL((k_expand<W, SCAN_FILTERED>), grid, dim3(EBLOCK), 0, c->stream, a);
    }
  }
  if (c->n_hub_items > 0) launch_hubs_w<W>(c, a, mode == SCAN_UNFILTERED, c->lines_ran);
  // kernel_ms brackets the pull kernel and the hub passes: the round's
  // counters (row bytes, arcs scanned, rows written) include the hubs' share
  if (a.prehi) launch_acc_clear_w<W>(c);   // degree-split round: the accumulator back to all-zero
  (void)hipEventRecord(c->ev[5], c->stream);
}

int launch_round_kernels(Ctx* c, const ExpandArgs& a) {
  switch (c->words) {
    case 1: launch_expand_w<1>(c, a); break;
    case 2: launch_expand_w<2>(c, a); break;
    case 4: launch_expand_w<4>(c, a); break;
    case 8: launch_expand_w<8>(c, a); break;
    case 16: launch_expand_w<16>(c, a); break;
    case 32: launch_expand_w<32>(c, a); break;
    case 64: launch_expand_w<64>(c, a); break;
    default: return set_error(GP_EINVAL, "unsupported word count");
  }
  GP_HIP(hipGetLastError());
  return 0;
}

}  // namespace gp
