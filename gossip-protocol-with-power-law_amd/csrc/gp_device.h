// gp_device.h -- device-side definitions shared by the kernel translation
// units of libgossip_hip.so (pull.hip, hub.hip, push.hip, driver.hip): row
// geometry, per-wave counters, the pull's argument block, the gather and
// commit helpers every receiver side uses (k_expand, k_expand_flat, the hub
// passes, k_apply), and the host launch entry points each unit defines.
// DESIGN.md §3 describes the layout and the kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "gp_internal.h"

namespace gp {

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

constexpr int BLOCK = 256;         // 4 waves
constexpr int WAVES = BLOCK / 64;
constexpr int GS = 256 / BLOCK;     // grid-stride kernels' blocks per CU scale: same threads per CU at every BLOCK
// the per-receiver and edge-parallel pull kernels run in blocks of their own
// size: one wave per block, so that a CU slot frees as soon as its wave ends
// instead of waiting for the block's slowest wave (C4 47.4-47.6 -> 44.5-45.4
// ms, C5 222-225 -> 210-216 ms; profiles/r04_ab_block.txt)
#ifndef GP_EXPAND_BLOCK
#define GP_EXPAND_BLOCK 64
#endif
constexpr int EBLOCK = GP_EXPAND_BLOCK;
constexpr int EWAVES = EBLOCK / 64;
// the hub passes keep 4-wave blocks (64 threads measured equal, r04_ab_hub_block.txt)
constexpr int HBLOCK = 256;
constexpr int HWAVES = HBLOCK / 64;
constexpr int NPART = 2048;        // partial stat slots (spread the atomics)

// ---------------------------------------------------------------------------
// geometry: a wave loads 16 B per lane -> W/2 lanes per row, 128/W rows per
// wave-instruction (W == 1: 8 B per lane, 64 rows per instruction)
template <int W>
struct Geo {
  static constexpr int WPL = W >= 2 ? 2 : 1;   // words per lane
  static constexpr int LPR = W / WPL;          // lanes per row
  static constexpr int RPI = 64 / LPR;         // rows per wave-instruction
};

template <int W>
__device__ __forceinline__ u64x2 load_piece(const u64* __restrict__ base, int64_t row, int lw) {
  if constexpr (W >= 2) {
    return *reinterpret_cast<const u64x2*>(base + row * W + lw * 2);
  } else {
    u64x2 r;
    r.x = base[row];
    r.y = 0;
    return r;
  }
}
template <int W>
__device__ __forceinline__ void store_piece(u64* __restrict__ base, int64_t row, int lw, u64x2 x) {
  if constexpr (W >= 2) {
    *reinterpret_cast<u64x2*>(base + row * W + lw * 2) = x;
  } else {
    base[row] = x.x;
  }
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) x += __shfl_xor(x, s);
  return x;
}
__device__ __forceinline__ u64 wave_xor_u64(u64 x) {
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) x ^= __shfl_xor(x, s);
  return x;
}
__device__ __forceinline__ int lane_rank(u64 mask) {  // set bits of mask below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}
__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

// ---------------------------------------------------------------------------
// per-wave counters, flushed once per block into one of NPART slots
// Per-wave counters live in LDS (one row per wave, written by lane 0 only):
// every update is wave-uniform, and keeping NST u64 counters out of the VGPR
// file is worth several waves per SIMD of occupancy in the gather kernels.
// (NW: waves per block of the kernel -- the one-wave pull kernels keep one row)
template <int NW = WAVES>
__device__ __forceinline__ u64* stats_lds() {
  __shared__ u64 rows[NW][NST];
  return &rows[0][0];
}
struct WaveStats {
  u64* row;
  bool lead;
  __device__ __forceinline__ void add(int k, u64 x) {
    if (lead) row[k] += x;
  }
};
template <int NW = WAVES>
__device__ __forceinline__ void ws_zero(WaveStats& s) {
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  s.row = stats_lds<NW>() + wib * NST;
  s.lead = lane == 0;
  if (lane < NST) s.row[lane] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int NW = WAVES>
__device__ inline void flush_stats(const WaveStats& s, u64* __restrict__ partial) {
  (void)s;
  u64* red = stats_lds<NW>();
  __syncthreads();
  if (threadIdx.x < NST) {
    u64 t = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w)
      if (w < (int)(blockDim.x >> 6)) t += red[w * NST + threadIdx.x];
    if (t) atomicAdd(&partial[(size_t)threadIdx.x * NPART + (blockIdx.x % NPART)], t);
  }
}

// ---------------------------------------------------------------------------
// expansion
//
// Message-List slots: vertex v's seen row lives in one of two
// slot buffers S[0], S[1]; sp[v] says which (0xFF: none yet, reads as zero).
// In round r the neighbours' rows are read from S[r & 1] and every receiver
// writes its new seen row to S[(r + 1) & 1].  A sender u of round r received
// in round r - 1 (or was injected in round r), so S[r & 1][u] is exactly
// seen_r(u).  Reading u's whole Message-List instead of its frontier is exact:
// every older bit of seen_r(u) was sent to all of u's live out-neighbours when
// u first received it (forward-once), so a live receiver already holds it and
// OR(...) & ~seen(v) is unchanged.  This drops the separate frontier rows: a
// receiver writes one row per round instead of two.
struct ExpandArgs {
  const int64_t* __restrict__ row_ptr;
  const int32_t* __restrict__ col;
  const u64* __restrict__ rows;        // S[r & 1]: seen rows of the round's senders
  u64* slot[2];                        // S[0], S[1] (the receiver's own rows)
  int32_t wslot;                       // (r + 1) & 1: the slot receivers write
  uint8_t* __restrict__ sp;            // [n_alloc] slot of v's current seen row (0xFF: none)
  uint8_t* __restrict__ ws;            // [n_alloc] bit p: slot p written this run
  const uint32_t* __restrict__ fpop;   // |frontier_r|: bits received in round r - 1 (+ injected)
  const u64* __restrict__ abits;       // bit v: fpop(v) != 0 (2 MB at 2^24)
  const u64* __restrict__ sbits;       // bit k: abits[k] != 0 (sparse probe rounds of big overlays; else null)
  const u64* __restrict__ dbits;       // early-exit rounds without liveness: bit u = u held every message
                                       //   of its component at the end of the last round (else null)
  const int32_t* __restrict__ gcol;    // in-CSR columns in gather order (neighbour degree desc)
  const int32_t* __restrict__ midx;    // [n] row of v's component in cmask (-1: no messages)
  const u64* __restrict__ cmask;       // [K][W] messages originating in each component
  int32_t early_exit;                  // this round scans with the coverage check
  int32_t dprobe;                      // early exit + dbits (W = 64 pulls): every scanned arc probes the done
                                       //   bitmap first; a done in-neighbour anywhere makes the receiver's
                                       //   new bits its target (done_nb's rule) -- no aliased row is gathered
  int32_t alias;                       // done-neighbour rounds (W = 64, no liveness): receivers that complete
                                       //   commit SLOT_CMASK, no row (every later pull is a dprobe round)
  const int32_t* __restrict__ ulist;   // SCAN_LIST rounds: the vertices that could still receive
  int64_t ulist_n;
  int32_t* __restrict__ ulist_next;    // (or null) the same after this round: each wave appends its
                                       //   receivers that are still neither done nor sated (late rounds)
  int32_t unfiltered;                  // read every in-neighbour row (k_fixup_rows ran)
  int32_t near_done;                   // early-exit round with most messages held: fewer rows in flight
  const u64* __restrict__ alive;       // [W] messages some sender forwards this round (or null)
  int32_t sate;                        // alive early-exit round, no injection left: mark sated receivers
  u64* __restrict__ alive_next;        // [W] the same for round r + 1: OR of the new rows (or null)
  const u64* __restrict__ amask;       // SCAN_MASKED: bit j of word k = sender gcol[64k + j] active
  const int32_t* __restrict__ prehi;   // degree-split rounds (SCAN_PRE): probe only the first prehi[v]
                                       //   arcs of v's in-list (senders of in-degree >= split_deg); the
                                       //   others pushed into acc / tbits before the pull (else null)
  int32_t split_push;                  // the push half of a degree-split round: no sender / scan counters
  int32_t acc_row;                     // degree-split rounds: row of `rows` that is row 0 of `acc`
  const uint8_t* __restrict__ lm;      // SCAN_LINES: line mask of each sender's row (0: inactive)
  uint8_t* __restrict__ lm_next;       // W = 64 pulls: the same for round r + 1, written by the commits
                                       //   (nibbles; or null)
  const u64* __restrict__ cmk;         // record rounds: dense bitmap of this round's senders (bit v:
                                       //   read v's full row) (or null)
  const u64* __restrict__ cml;         // their records (word 0 mask, then the nonzero words)
  u64* __restrict__ cmk_next;          // dense bitmap / records the receivers write (or null)
  u64* __restrict__ cml_next;
  const uint32_t* __restrict__ done_at;// |messages of v's component|: seenpop == done_at -> done
  uint32_t* __restrict__ fpop_next;
  u64* __restrict__ frx;               // exact frontier rows of round r (track_msg_forwards, partitioned)
  u64* __restrict__ frx_next;          // exact frontier rows of round r + 1 (idem)
  int64_t frx_rows;                    // frx covers vertices [0, frx_rows) (partitioned: the owned
                                       // ones; a ghost's slot row IS its frontier)
  uint32_t* __restrict__ seenpop;
  uint8_t* __restrict__ first;         // may be null
  u64* __restrict__ digest;            // may be null
  uint8_t* __restrict__ state;         // read by every pull kernel; k_expand's alive variants set ST_SATED
  const int32_t* __restrict__ deg_live;
  u64* __restrict__ partial;
  const HubItem* __restrict__ hub_items;
  const int32_t* __restrict__ hubs;
  const int32_t* __restrict__ hub_item_ptr;
  u64* __restrict__ hub_partial;
  uint32_t* __restrict__ hub_pnz;
  uint32_t* __restrict__ hub_done;     // [n_hubs] early-exit rounds: = hub_epoch once a chunk covered its hub's target
  uint32_t hub_epoch;                  // this pull launch's stamp (never 0, never repeats within a context)
  // push mode
  const int64_t* __restrict__ orp;     // out-CSR (undirected: == row_ptr/col)
  const int32_t* __restrict__ ocol;
  u64* __restrict__ acc;               // [n_alloc][W] OR accumulator (all-zero between uses)
  u64* __restrict__ tbits;             // [n_alloc/64] receivers pushed to this round
  const u64* __restrict__ nbits;       // push rounds of narrow rows: bit v = v can still receive
                                       //   (owned, up, not done); null: checked per arc
  int32_t* __restrict__ touched;       // receivers touched this round
  const int32_t* __restrict__ active;  // senders with deg <= hub_thr
  const int32_t* __restrict__ big;     // senders with deg > hub_thr
  u64* __restrict__ stats;             // device counters (cursors)
  int64_t vbegin, nloc;
  int64_t n_items;                     // hub items / hubs for the hub kernels
  int32_t m_total;
  int32_t wbase;                       // global word index of local word 0 (message shards)
  int32_t rr;                          // receipt round of this expansion (r + 1)
  int32_t hub_thr;
};

constexpr uint8_t SLOT_NONE = 0xFF;
constexpr uint8_t SLOT_PARKED = 2;   // row in d_slot[2] (a down vertex, before an unfiltered pull)
// aliased Message-List: v completed its component in a dprobe
// round without liveness, so its Message-List is cmask[midx[v]] and no row was
// written.  Only dprobe pulls run while a context holds aliases (they never
// gather a done sender's row); every other reader materializes them first
// (k_unalias)
constexpr uint8_t SLOT_CMASK = 3;
// commit flag beside the 4-bit line mask in the deferred per-vertex words
constexpr uint8_t LMN_ALIAS = 0x10;

// Message-List records (W = 64): a round whose receivers end
// up with sparse Message-Lists also writes, per receiver, a 128-B record --
// word 0 the mask of its nonzero words (bit w = word w), then those words in
// order (at most CML_MAXW) -- or sets its bit in a dense bitmap (more nonzero
// words: read the full row).  The next round, a filtered pull, probes the
// dense bitmap beside the activity bitmap (both 2 MB at 2^24, L2-resident) and
// gathers one 128-B line per sparse sender instead of four, four senders per
// wave-instruction.
constexpr int CML_WORDS = 16;             // u64 per record
constexpr int CML_MAXW = CML_WORDS - 1;   // nonzero words a record holds

// k_detect grid: blocks per CU
#ifndef GP_DETECT_BLOCKS_PER_CU
#define GP_DETECT_BLOCKS_PER_CU 16   // 4 -> 16: C5 304.1-304.5 -> 302.2-302.4 ms per run same-box
#endif
// summary probes only while at most n / SUMMARY_RATIO vertices send
constexpr double SUMMARY_RATIO = 256.0;
#define EXPAND_BOUNDS __launch_bounds__(EBLOCK)
// rows each lane keeps in flight per gather step (MLP vs VGPRs)
#ifndef GP_ROWS_IN_FLIGHT
#define GP_ROWS_IN_FLIGHT 4
#endif
// 64-word rows (C4 / C5: a wave-instruction moves 1 KB): 3 rows per lane in
// flight -- fewer rows loaded past an early exit, and the alive variant at 65
// VGPRs: C4 48.2 -> 46.1 ms, C5 245.7-253.5 -> 238.2-241.4 ms same-box
// (profiles/r03_ab_rif3.txt); 32-word rows keep 4 (the 2048-message shard ran
// 37.6 -> 38.2 ms with 3)
#ifndef GP_ROWS_IN_FLIGHT_64
#define GP_ROWS_IN_FLIGHT_64 3
#endif
// W = 8: the per-receiver kernel runs the 8-GPU job's thin late rounds
// (narrow_pr_now); 2 rows in flight keep it at ~59 VGPRs against ~103 with 4
// (N = 8 slowest rank 11.8 -> 11.3 ms, profiles/r06_ab_w8.txt)
#ifndef GP_ROWS_IN_FLIGHT_NARROW
#define GP_ROWS_IN_FLIGHT_NARROW 2
#endif
template <int W>
struct RowsInFlight {
  static constexpr int value = W >= 64 ? GP_ROWS_IN_FLIGHT_64 : W == 8 ? GP_ROWS_IN_FLIGHT_NARROW : GP_ROWS_IN_FLIGHT;
};

// per-wave LDS of the pull kernels; the mode-specific arrays take one element
// when their mode is compiled out (LDS is what bounds the waves per CU)
constexpr int PRE_IDS = 8;       // active neighbours kept per prefiltered vertex
constexpr int PRE_MAX_DEG = 16;  // in-degree up to which the lane phase probes
// in-degree up to which the wave probes receivers' in-lists together (SCAN_PRE
// rounds), and how many receivers per step
#ifndef GP_WAVE_PRE_MAX
#define GP_WAVE_PRE_MAX 64
#endif
constexpr int WAVE_PRE_N = 4;   // (2 and 8 measured equal)
template <bool PRE, bool CML, bool LIST = false, bool PAIRS = false>
struct WaveLdsT {
  static constexpr bool kPre = PRE, kCml = CML, kList = LIST;
  u64 seen[PAIRS ? 128 : 64];   // early exit: the receiver's seen row (read once, reused by finish_row; gather_pairs: two)
  int32_t idx[64];      // active neighbours of one pass
  uint32_t tot[64];     // k_expand: new bits of the wave's vertex k (committed after the loop)
  uint8_t lmn[64];      // k_expand: line mask of vertex k's new row (committed with tot)
  u64 dig[64];          // k_expand: digest terms of vertex k
  int64_t rp[65];       // k_expand: row_ptr of the wave's vertices (rp[k], rp[k + 1])
  int32_t mi[64];       // k_expand: component-mask row of vertex k (early-exit rounds)
  u64 racc[CML ? 64 : 1];         // record rounds: OR of the gathered records, word w
  int32_t sid[CML ? 64 : 1];      // record rounds: sparse senders of one pass
  uint8_t cd[CML ? 64 : 1];       // record-writing rounds: vertex k's row is dense (no record)
  int32_t pre[PRE ? 64 : 1][PRE_IDS];   // SCAN_PRE: active neighbours of vertex k found by the lane phase
  uint8_t np[PRE ? 64 : 1];       // SCAN_PRE: how many (0xFF: not prefiltered, scan as usual)
  uint32_t len[PRE ? 64 : 1];     // SCAN_PRE: in-arcs vertex k scans (its prefix in degree-split rounds)
  u64 alive[64];                  // OR of the new rows this wave wrote (alive_next)
  int32_t vid[LIST ? 64 : 1];     // SCAN_LIST: vertex of lane k (the list is not consecutive ids)
  int64_t re[LIST ? 64 : 1];      // SCAN_LIST: end of vertex k's in-list
};
using WaveLds = WaveLdsT<false, false>;
#define LDS_OF(MODE) \
  WaveLdsT<((MODE) & 3) == SCAN_PRE, ((MODE) & SCAN_CML) != 0, ((MODE) & SCAN_LIST) != 0, ((MODE) & SCAN_QUADS) != 0>

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Alive messages: F_r, the messages some sender forwards in
// round r, is the OR of the rows received for the first time in round r - 1
// plus the messages injected in round r.  A live receiver already holds every
// bit of a sender's row outside its frontier (ExpandArgs), so nothing outside
// F_r can be new to it and the early-exit target is cm & F_r & ~seen.  Under
// churn this is what lets receivers stop when crashes cut a message off (the
// component target cm then stays out of reach).  Each wave ORs its new rows
// into LDS and flushes them once, skipping words the global row already has.
template <int W, class LDS>
__device__ __forceinline__ void alive_add(const ExpandArgs& a, LDS& L, int lw, u64x2 nw) {
  constexpr int WPL = Geo<W>::WPL;
  if (!a.alive_next) return;
  if (nw.x) atomicOr(&L.alive[lw * WPL], nw.x);
  if (WPL == 2 && nw.y) atomicOr(&L.alive[lw * WPL + 1], nw.y);
}
template <int W>
__device__ __forceinline__ void alive_zero(const ExpandArgs& a, u64* alive, int lane) {
  if (a.alive_next && lane < W) alive[lane] = 0ull;
}
template <int W>
__device__ __forceinline__ void alive_flush(const ExpandArgs& a, const u64* alive, int lane) {
  if (!a.alive_next) return;
  wave_sync_lds();
  if (lane < W) {
    const u64 x = alive[lane];
    if (x) {
      const u64 cur = __hip_atomic_load(a.alive_next + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (x & ~cur) atomicOr(a.alive_next + lane, x);
    }
  }
}

__device__ __forceinline__ uint32_t wave_excl_scan_u32(uint32_t x, int lane) {
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  return inc - x;
}

// reductions over the LPR lanes of one row slot (lanes g*LPR .. g*LPR + LPR - 1)
template <int LPR>
__device__ __forceinline__ bool group_or(bool x) {
  uint32_t y = x ? 1u : 0u;
#pragma unroll
  for (int s = 1; s < LPR; s <<= 1) y |= (uint32_t)__shfl_xor((int)y, s);
  return y != 0u;
}
template <int LPR>
__device__ __forceinline__ uint32_t group_sum(uint32_t x) {
#pragma unroll
  for (int s = 1; s < LPR; s <<= 1) x += (uint32_t)__shfl_xor((int)x, s);
  return x;
}
template <int LPR>
__device__ __forceinline__ u64 group_xor(u64 x) {
#pragma unroll
  for (int s = 1; s < LPR; s <<= 1) x ^= __shfl_xor(x, s);
  return x;
}

__device__ __forceinline__ u64 wave_sum_u64(u64 x) {
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) x += __shfl_xor(x, s);
  return x;
}

// OR-reduce the row slots of the wave: afterwards every lane holds the full
// result for its lw column.
template <int W>
__device__ __forceinline__ void reduce_slots(u64x2& acc) {
  constexpr int LPR = Geo<W>::LPR;
#pragma unroll
  for (int s = LPR; s < 64; s <<= 1) {
    acc.x |= __shfl_xor(acc.x, s);
    if constexpr (W >= 2) acc.y |= __shfl_xor(acc.y, s);
  }
}

// scan modes of a pull round (compile-time): the per-arc activity probe, the
// per-arc activity mask built by k_arcmask before the round, or no check at all
// (unfiltered dense rounds)
enum ScanMode { SCAN_FILTERED = 0, SCAN_MASKED = 1, SCAN_UNFILTERED = 2, SCAN_PRE = 3,
                SCAN_CML = 4 /* flag: read / write compact Message-Lists (W = 64) */,
                SCAN_ALIVE = 8 /* flag: early-exit targets narrowed to the alive messages (k_expand);
                                  a variant of its own: +2-3 VGPRs cost a wave per SIMD */,
                SCAN_LINES = 32 /* flag (W = 64, filtered): the probe reads the sender's line mask
                                   (k_mklm) and the gather loads only its nonzero 128-B lines */,
                SCAN_DPROBE = 64 /* flag (k_expand, W = 64, filtered / unfiltered): every scanned arc
                                    probes the done bitmap (a.dprobe rounds, aliased Message-Lists);
                                    a variant of its own: +4 VGPRs cost the unfiltered pull a wave */,
                SCAN_LIST = 128 /* flag (k_expand, W >= 32, filtered / unfiltered): the waves take
                                   their receivers from a.ulist, the vertices that could still
                                   receive (late rounds), not 64 consecutive ids */,
                SCAN_QUADS = 256 /* flag (k_expand, unfiltered): W = 64: done-neighbour receivers
                                    four per wave step (dnb_quads) without the done probe, and (no
                                    liveness) receivers of in-degree <= 32 two per step
                                    (gather_pairs): the first aliasing round, near-done pulls,
                                    alive pulls from the half-held round; W = 32 / 16 / 8
                                    near-done pulls: low in-degree receivers 4 / 8 / 16 per step
                                    (gather_groups) */ };

// activity bits of arcs [j0, j0 + n) (n <= 64) from the per-arc mask, bit t =
// arc j0 + t; j0 wave-uniform, so both words come in through scalar loads
__device__ __forceinline__ u64 mask_window(const u64* __restrict__ amask, int64_t j0, int n) {
  const int64_t k = j0 >> 6;
  const int sh = (int)(j0 & 63);
  u64 win = amask[k] >> sh;
  if (sh) win |= amask[k + 1] << (64 - sh);
  if (n < 64) win &= (1ull << n) - 1ull;
  return win;
}

// any active arc in [b, e) (e > b)?  In-lists spanning more than two mask
// words are taken as active (the scan finds out).
__device__ __forceinline__ bool mask_any(const u64* __restrict__ amask, int64_t b, int64_t e) {
  const int64_t k0 = b >> 6, k1 = (e - 1) >> 6;
  if (k1 - k0 > 1) return true;
  const u64 lo = ~0ull << (b & 63);
  const int hi = (int)((e - 1) & 63);
  const u64 him = hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1ull);
  if (k0 == k1) return (amask[k0] & lo & him) != 0ull;
  return ((amask[k0] & lo) | (amask[k1] & him)) != 0ull;
}

// line masks (SCAN_LINES): two vertices per byte (v even: low nibble), 8 MB
// at 2^24 (a byte per vertex measured the same, r03_ab_nibble.txt)
__device__ __forceinline__ uint8_t lm_of(const uint8_t* __restrict__ lm, int32_t u) {
  return (uint8_t)((lm[u >> 1] >> ((u & 1) * 4)) & 0xF);
}
// 4-bit line mask from a ballot over 32 lanes of 16 B (8 lanes per 128-B line)
__device__ __forceinline__ uint32_t lines_of(uint32_t b) {
  uint32_t l = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) l |= ((b >> (8 * t)) & 0xFFu) ? (1u << t) : 0u;
  return l;
}
// neighbour u if its row is read this round, else -1
template <int MODE>
__device__ __forceinline__ int32_t probe(const ExpandArgs& a, int32_t u) {
  if constexpr ((MODE & 3) == SCAN_UNFILTERED) {
    return u;
  } else {
    return ((a.abits[u >> 6] >> (u & 63)) & 1ull) ? u : -1;
  }
}

// OR the staged rows of one pass (L.idx[0, cnt)) into acc, GP_ROWS_IN_FLIGHT
// wave-instructions of 16 B per lane in flight.  Early exit (bottom-up,
// Beamer et al. SC'12): with `ee` the wave stops once acc | seen covers every
// message of the vertex's component (want = cm & ~seen); OR is idempotent, so
// acc & ~seen is exactly what the full scan would give.  Per word, the same
// rule skips the loads of a lane whose words are already complete (`miss`,
// carried across passes): a 128-B line of a row is not fetched once its 16
// words are.  Returns true on early exit.
// Row bytes are counted per 128-B line a row load touches: HBM delivers whole
// lines, so a lane that skips its 16 B while others of its line load theirs
// saves no traffic (measured: skipping whole lines only, GP_LINE_SKIP in round
// 2's notes, fetched exactly the same bytes and ran 1 ms slower).  Rows of
// W >= 16 span whole lines (8 lanes x 16 B each); narrower rows count pieces.
// ballot b of a row-load instruction -> 16-B pieces of the lines it touches
template <int W>
__device__ __forceinline__ u64 line_pieces(u64 b) {
  if constexpr (Geo<W>::LPR >= 8) {
    u64 t = b | (b >> 4);
    t |= t >> 2;
    t |= t >> 1;
    return 8ull * (u64)__popcll(t & 0x0101010101010101ull);
  } else {
    return (u64)__popcll(b);
  }
}
template <int W, int RIF>
__device__ __forceinline__ bool gather_rows_n(const ExpandArgs& a, const int32_t* idx, int cnt, int g, int lw,
                                              u64x2& acc, WaveStats& st, bool ee, u64x2 want) {
  constexpr int RPI = Geo<W>::RPI;
  bool live = true;   // this lane's words still miss messages
  if (ee) {
    u64x2 t = acc;
    reduce_slots<W>(t);
    const u64x2 miss = want & ~t;
    live = (miss.x | miss.y) != 0ull;
  }
  for (int k0 = 0; k0 < cnt; k0 += RIF * RPI) {
    u64x2 r[RIF];
#pragma unroll
    for (int q = 0; q < RIF; ++q) {
      const int k = k0 + g + q * RPI;
      r[q] = u64x2{0, 0};
      if (k < cnt && live) r[q] = load_piece<W>(a.rows, idx[k], lw);
    }
#pragma unroll
    for (int q = 0; q < RIF; ++q) acc |= r[q];
    st.add(S_GATHERED, (u64)min(RIF * RPI, cnt - k0));
    u64 pieces = 0;   // 8 * WPL-byte pieces of the lines the loads touched (word skip)
#pragma unroll
    for (int q = 0; q < RIF; ++q) pieces += line_pieces<W>(__ballot(k0 + g + q * RPI < cnt && live));
    st.add(S_ROW_BYTES, pieces * (u64)(8 * Geo<W>::WPL));
    if (ee) {
      u64x2 t = acc;
      reduce_slots<W>(t);
      const u64x2 miss = want & ~t;
      live = (miss.x | miss.y) != 0ull;
      if (!__any(live)) return true;
    }
  }
  return false;
}
// near the end of a run (early exit, most messages held) receivers complete
// after a few rows, and rows already in flight past that point are wasted:
// gather 2 rows per lane at a time there (C4 round 4: 12.8 -> 10.4 ms, 67.2 ->
// 64.6 ms per run same-box), the full GP_ROWS_IN_FLIGHT elsewhere
template <int W>
__device__ __forceinline__ bool gather_rows(const ExpandArgs& a, const int32_t* idx, int cnt, int g, int lw,
                                            u64x2& acc, WaveStats& st, bool ee, u64x2 want) {
#ifndef GP_NEAR_DONE_RIF
#define GP_NEAR_DONE_RIF 2
#endif
// (64-word rows already keep 3 in flight; 2 there cost round 4 0.2 ms, r03_ab_nd_lr.txt)
#ifndef GP_NEAR_DONE_RIF_64
#define GP_NEAR_DONE_RIF_64 3
#endif
  constexpr int ND = W >= 64 ? GP_NEAR_DONE_RIF_64 : GP_NEAR_DONE_RIF;
  if (RowsInFlight<W>::value > ND && a.near_done)
    return gather_rows_n<W, ND>(a, idx, cnt, g, lw, acc, st, ee, want);
  return gather_rows_n<W, RowsInFlight<W>::value>(a, idx, cnt, g, lw, acc, st, ee, want);
}

// SCAN_LINES rounds (W = 64, filtered, no early exit): staged entries carry the
// sender's line mask in their low 4 bits ((u << 4) | lines, n <= 2^27), and
// each lane loads its 16-B piece of a row only when its 128-B line is named.
// No early-exit state: 64 VGPRs less pressure than gather_rows_n with masks.
#ifndef GP_LINES_RIF
#define GP_LINES_RIF 3   // 62 VGPRs, 8 waves per SIMD (4: 66, 7 waves): C4 round 2 14.5 -> 14.1 ms
#endif
template <int RIF>
__device__ __forceinline__ void gather_lines(const ExpandArgs& a, const int32_t* ent, int cnt, int g, int lw,
                                             u64x2& acc, WaveStats& st) {
  constexpr int RPI = Geo<64>::RPI;
  const int32_t lbit = 1 << (lw >> 3);
  for (int k0 = 0; k0 < cnt; k0 += RIF * RPI) {
    u64x2 r[RIF];
    u64 pieces = 0;
#pragma unroll
    for (int q = 0; q < RIF; ++q) {
      const int k = k0 + g + q * RPI;
      r[q] = u64x2{0, 0};
      const int32_t e = k < cnt ? ent[k] : 0;
      const bool on = (e & lbit) != 0;
      if (on) r[q] = load_piece<64>(a.rows, e >> 4, lw);
      pieces += line_pieces<64>(__ballot(on));
    }
#pragma unroll
    for (int q = 0; q < RIF; ++q) acc |= r[q];
    st.add(S_GATHERED, (u64)min(RIF * RPI, cnt - k0));
    st.add(S_ROW_BYTES, pieces * 16ull);
  }
}

// position of the k-th (1-based) set bit of m
__device__ __forceinline__ int select_bit(u64 m, int k) {
  int pos = 0;
#pragma unroll
  for (int sh = 32; sh > 0; sh >>= 1) {
    const int c = __popcll(m & ((1ull << sh) - 1ull));
    if (c < k) {
      k -= c;
      m >>= sh;
      pos += sh;
    }
  }
  return pos;
}

// records of the staged sparse senders idx[0, cnt): a 16-lane group loads one
// 128-B record (lane 0 of the group its mask), GP_ROWS_IN_FLIGHT records per
// group in flight; each word is OR-ed into L.racc at its word index.
template <class LDS>
__device__ __forceinline__ void gather_recs(const ExpandArgs& a, LDS& L, const int32_t* idx, int cnt,
                                            WaveStats& st) {
  const int lane = threadIdx.x & 63, gq = lane >> 4, sl = lane & 15;
  for (int k0 = 0; k0 < cnt; k0 += 4 * GP_ROWS_IN_FLIGHT) {
    u64 val[GP_ROWS_IN_FLIGHT];
#pragma unroll
    for (int q = 0; q < GP_ROWS_IN_FLIGHT; ++q) {
      const int k = k0 + 4 * q + gq;
      val[q] = k < cnt ? a.cml[(size_t)idx[k] * CML_WORDS + sl] : 0ull;
    }
#pragma unroll
    for (int q = 0; q < GP_ROWS_IN_FLIGHT; ++q) {
      const u64 m = __shfl(val[q], lane & ~15);
      if (sl >= 1 && sl <= __popcll(m) && val[q]) atomicOr(&L.racc[select_bit(m, sl)], val[q]);
    }
  }
  st.add(S_GATHERED, (u64)cnt);
  st.add(S_ROW_BYTES, (u64)cnt * (u64)(8 * CML_WORDS));
}

// stage one pass of probed neighbours (e: this lane's entry, -1 = none) in
// LDS; returns their count
template <class LDS>
__device__ __forceinline__ int stage_pass(LDS& L, int32_t e) {
  const u64 m = __ballot(e >= 0);
  if (e >= 0) L.idx[lane_rank(m)] = e;
  wave_sync_lds();
  return __popcll(m);
}

// the receiver's current seen row, piece lw (slot sv_slot; SLOT_NONE: empty)
template <int W>
__device__ __forceinline__ u64x2 load_seen(const ExpandArgs& a, int v, uint32_t sv_slot, int lw) {
  return sv_slot != SLOT_NONE ? load_piece<W>(a.slot[sv_slot], v, lw) : u64x2{0, 0};
}

// early exit: park the receiver's seen row in LDS (finish_row reuses it) and
// return, in group-0 lanes, the messages of its component it still lacks
template <int W, class LDS, bool ALIVE = true>
__device__ __forceinline__ u64x2 early_exit_target(const ExpandArgs& a, int v, LDS& L, int g, int lw,
                                                   uint32_t sv_slot, int32_t mrow) {
  constexpr int WPL = Geo<W>::WPL;
  // every row slot group loads the same pieces (one fetch per line): each lane
  // needs its words' target to skip the loads of words already complete
  const u64x2 sv = load_seen<W>(a, v, sv_slot, lw);
  u64x2 cm = load_piece<W>(a.cmask, mrow, lw);
  if (ALIVE && a.alive) cm &= load_piece<W>(a.alive, 0, lw);
  if (g == 0) {
    L.seen[lw * WPL] = sv.x;
    if constexpr (WPL == 2) L.seen[lw * WPL + 1] = sv.y;
  }
  return cm & ~sv;
}

// per-receiver scan of arcs [b, e): 64 arcs per pass -- column ids, activity
// probes, staging, gather.  DP: the variant can run in a done-probe round
// (a.dprobe; W = 64 filtered / unfiltered pulls without liveness): compiled
// out elsewhere, so the other variants keep their registers
template <int W, int MODE, bool DP, class LDS>
__device__ __forceinline__ void gather_scan(const ExpandArgs& a, int64_t b, int64_t e, LDS& L, int lane,
                                            int g, int lw, u64x2& acc, WaveStats& st, bool ee, u64x2 want,
                                            int32_t col0 = INT32_MIN) {
  // col0: this lane's column id of the first pass, when the caller loaded it
  // early (beside the early-exit target's loads; INT32_MIN: not loaded)
  for (int64_t j0 = b; j0 < e; j0 += 64) {
    const int n = (int)min((int64_t)64, e - j0);
    st.add(S_ARCS, n);
    int cnt;
    if constexpr (W == 64 && (MODE & SCAN_CML) != 0) {
      if (a.cmk) {   // record round (no early exit): sparse senders' records, dense senders' rows
        int32_t u = -1;
        bool act = false, dense = false;
        if (lane < n) {
          u = a.gcol[j0 + lane];
          act = probe<MODE>(a, u) >= 0;
          if (act) dense = ((a.cmk[u >> 6] >> (u & 63)) & 1ull) != 0ull;
        }
        const u64 md = __ballot(act && dense), ms = __ballot(act && !dense);
        if (act) {
          if (dense) L.idx[lane_rank(md)] = u;
          else L.sid[lane_rank(ms)] = u;
        }
        wave_sync_lds();
        if (md) gather_rows<W>(a, L.idx, __popcll(md), g, lw, acc, st, false, want);
        if (ms) gather_recs(a, L, L.sid, __popcll(ms), st);
        wave_sync_lds();
        continue;
      }
    }
    if constexpr (W == 64 && (MODE & SCAN_LINES) != 0) {
      // line masks: the probe reads the sender's byte (0: inactive), the
      // gather loads only the lines it names
      uint8_t lv = 0;
      int32_t u = -1;
      if (lane < n) {
        u = (col0 != INT32_MIN && j0 == b) ? col0 : a.gcol[j0 + lane];
        lv = lm_of(a.lm, u);
      }
      const u64 ml = __ballot(lv != 0);
      if (lv) L.idx[lane_rank(ml)] = (u << 4) | (int32_t)lv;
      wave_sync_lds();
      if (ml == 0ull) continue;
      gather_lines<GP_LINES_RIF>(a, L.idx, __popcll(ml), g, lw, acc, st);
      wave_sync_lds();
      continue;
    }
    if constexpr ((MODE & 3) == SCAN_MASKED) {
      // the mask names the active arcs: column ids of the others are not loaded
      const u64 win = mask_window(a.amask, j0, n);
      if (win == 0ull) continue;
      if ((win >> lane) & 1ull) L.idx[lane_rank(win)] = a.gcol[j0 + lane];
      wave_sync_lds();
      cnt = __popcll(win);
    } else {
      int32_t ent = -1, u = -1;
      u64 dw = 0;
      if (lane < n) {
        u = (col0 != INT32_MIN && j0 == b) ? col0 : a.gcol[j0 + lane];
        if (DP && a.dprobe) dw = a.dbits[u >> 6];   // (beside the activity probe: one round trip)
        ent = probe<MODE>(a, u);
      }
      // a done in-neighbour in this pass: the receiver's new bits are its
      // whole target (done_nb's rule, any arc), and none of the pass's rows
      // is gathered -- an aliased sender's row slot holds no Message-List
      if (DP && a.dprobe && __any(u >= 0 && ((dw >> (u & 63)) & 1ull))) {
        acc = want;
        break;
      }
      cnt = stage_pass(L, ent);
      if (cnt == 0) continue;
    }
    const bool stop = gather_rows<W>(a, L.idx, cnt, g, lw, acc, st, ee, want);
    wave_sync_lds();
    if (stop) break;
  }
}

__device__ __forceinline__ void set_first_bytes(uint8_t* __restrict__ row, int word, u64 bits,
                                                uint32_t rr) {
  // row: first-receipt bytes of one vertex (stride W*64); 8-byte RMW per byte group
  u64* p = reinterpret_cast<u64*>(row + (size_t)word * 64);
  while (bits) {
    const int grp = (__ffsll((long long)bits) - 1) >> 3;   // byte group of lowest set bit
    const u64 gbits = (bits >> (grp * 8)) & 0xFFull;
    u64 f = p[grp];
    u64 m = gbits;
    while (m) {
      const int b = __ffsll((long long)m) - 1;
      f = (f & ~(0xFFull << (8 * b))) | ((u64)rr << (8 * b));
      m &= m - 1;
    }
    p[grp] = f;
    bits &= ~(0xFFull << (grp * 8));
  }
}

// bit i of x -> bit 2i
__device__ __forceinline__ u64 spread32(u64 x) {
  x &= 0xFFFFFFFFull;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}
// the record of a 64-word Message-List held as (g, lw) pieces by the group-0
// lanes (W = 64: lanes 0..31, words 2lw and 2lw + 1); returns true (uniform)
// when the row is dense and no record is written
__device__ __forceinline__ bool write_rec(u64* __restrict__ cml, int v, int g, int lw, u64x2 row) {
  const u64 bx = __ballot(g == 0 && row.x != 0ull), by = __ballot(g == 0 && row.y != 0ull);
  const u64 m = spread32(bx) | (spread32(by) << 1);
  if (__popcll(m) > CML_MAXW) return true;
  u64* rec = cml + (size_t)v * CML_WORDS;
  if (g == 0) {
    const int p = 1 + __popcll(m & ((1ull << (2 * lw)) - 1ull));
    if (row.x) rec[p] = row.x;
    if (row.y) rec[p + (row.x ? 1 : 0)] = row.y;
    if (lw == 0) rec[0] = m;
  }
  return false;
}

// dense bit of vertex v in a record-writing round (one atomic: hubs, push)
__device__ __forceinline__ void set_dense(u64* __restrict__ bm, int v) {
  atomicOr(bm + (v >> 6), 1ull << (v & 63));
}

// receiver side of vertex v (local index i): new = acc & ~seen; write the new
// seen row to slot wslot, counters.  have_sv: the seen row is parked in L.seen
// (early exit), else it is loaded here from slot sv_slot.
// DEFER (k_expand): the per-vertex words (fpop, seenpop, slot bytes, digest)
// go to L.tot/L.dig[k] and the wave commits them for its 64 vertices at once,
// coalesced, after its loop -- one scattered read-modify-write chain less per
// receiver, and whole cache lines instead of 1-8 byte pieces.
// alias (DEFER, a.alias rounds): the receiver completes its component this
// round (acc covers its early-exit target), so its new Message-List is its
// component row: no row is written, the commit sets SLOT_CMASK
template <int W, bool DEFER = false, bool CMLW = true, class LDS = WaveLds>
__device__ __forceinline__ void finish_row(const ExpandArgs& a, int v, int64_t i, u64x2 acc, int lane,
                                           int g, int lw, WaveStats& st, LDS& L, bool have_sv,
                                           uint32_t sv_slot, int k = 0, bool alias = false) {
  constexpr int WPL = Geo<W>::WPL;
  const bool nz = (acc.x | acc.y) != 0;
  if (!__any(nz)) {
    if (!DEFER && lane == 0) a.fpop_next[v] = 0;
    return;
  }
  if (!have_sv && sv_slot != SLOT_NONE) st.add(S_SEEN_READ, 1);
  u64x2 sv = {0, 0}, nw = {0, 0};
  if (g == 0) {
    if (have_sv) {
      sv.x = L.seen[lw * WPL];
      if constexpr (WPL == 2) sv.y = L.seen[lw * WPL + 1];
    } else {
      sv = load_seen<W>(a, v, sv_slot, lw);
    }
    nw = acc & ~sv;
  }
  const uint32_t pc = (uint32_t)(__popcll(nw.x) + __popcll(nw.y));
  const uint32_t tot = wave_sum_u32(pc);
  if (tot == 0) {
    if (!DEFER && lane == 0) a.fpop_next[v] = 0;
    return;
  }
  bool dense = true;
  if constexpr (W == 64 && CMLW) {
    if (a.cml_next) dense = write_rec(a.cml_next, v, g, lw, sv | nw);
  }
  // W = 64: the lines of the new bits -- the frontier the next round sends --
  // holding a nonzero word (lm_next).  Gathering only those lines of a
  // sender's Message-List is exact: the rest of the row was sent before (a
  // superset such as k_mklm's whole-row lines is exact too)
  uint32_t lmn = 0;
  if constexpr (W == 64) {
    if (a.lm_next) lmn = lines_of((uint32_t)__ballot(g == 0 && (nw.x | nw.y) != 0ull));
  }
  if (g == 0) {
    alive_add<W>(a, L, lw, nw);
    if (!alias) store_piece<W>(a.slot[a.wslot], v, lw, sv | nw);   // the whole row: the slot may hold an older one
    if (a.frx_next) store_piece<W>(a.frx_next, v, lw, nw);
    if (a.first) {
      uint8_t* row = a.first + (size_t)i * (W * 64);
      if (nw.x) set_first_bytes(row, lw * WPL, nw.x, (uint32_t)a.rr);
      if (WPL == 2 && nw.y) set_first_bytes(row, lw * WPL + 1, nw.y, (uint32_t)a.rr);
    }
  }
  if (a.digest) {
    u64 t = 0;
    if (g == 0) {
      if (nw.x) t ^= digest_term((uint32_t)a.rr, (uint32_t)(a.wbase + lw * WPL), nw.x);
      if (WPL == 2 && nw.y) t ^= digest_term((uint32_t)a.rr, (uint32_t)(a.wbase + lw * WPL + 1), nw.y);
    }
    t = wave_xor_u64(t);
    if constexpr (DEFER) {
      if (lane == 0) L.dig[k] = t;
    } else if (lane == 0) {
      a.digest[i] ^= t;
    }
  }
  if constexpr (DEFER) {
    if (lane == 0) {
      L.tot[k] = tot;
      L.lmn[k] = (uint8_t)lmn | (alias ? LMN_ALIAS : (uint8_t)0);
      if constexpr (CMLW && LDS::kCml) L.cd[k] = dense ? 1 : 0;
    }
  } else {
    if (lane == 0) {
      if (a.cmk_next) set_dense(a.cmk_next, v);
      // (hub passes: the pull's commit left this vertex's nibble 0)
      if (W == 64 && a.lm_next && lmn) atomicOr(reinterpret_cast<uint32_t*>(a.lm_next) + (v >> 3), lmn << ((v & 7) * 4));
      a.fpop_next[v] = tot;
      a.seenpop[i] += tot;
      a.sp[v] = (uint8_t)a.wslot;
      a.ws[v] |= (uint8_t)(1u << a.wslot);
    }
    st.add(S_NEXT_ARCS, (u64)(uint32_t)max(a.deg_live[v], 0));
  }
  st.add(S_NEW_BITS, tot);
  st.add(S_RECEIVERS, 1);
  st.add(alias ? S_ALIASED : S_WRITTEN, 1);
}

// k_expand's commit of the deferred per-vertex words: lane k holds vertex
// li = base + k, or in SCAN_LIST rounds the list's vertex (need: it was scanned)
template <class LDS>
__device__ __forceinline__ void commit_vertices(const ExpandArgs& a, LDS& L, int64_t li, bool need,
                                                WaveStats& st) {
  wave_sync_lds();
  const int lane = threadIdx.x & 63;
  u64 next_arcs = 0;
  if (need) {
    const int v = (int)(a.vbegin + li);
    const uint32_t tot = L.tot[lane];
    a.fpop_next[v] = tot;
    if (tot) {
      a.seenpop[li] += tot;
      if (L.lmn[lane] & LMN_ALIAS) {
        a.sp[v] = SLOT_CMASK;
      } else {
        a.sp[v] = (uint8_t)a.wslot;
        a.ws[v] |= (uint8_t)(1u << a.wslot);
      }
      if (a.digest) a.digest[li] ^= L.dig[lane];
      next_arcs = (u64)(uint32_t)max(a.deg_live[v], 0);
    }
  }
  st.add(S_NEXT_ARCS, wave_sum_u64(next_arcs));
  if (a.lm_next) {   // line masks of the next round's senders, two vertices per byte (hubs: 0 here)
    const uint32_t nib = (need && L.tot[lane]) ? (uint32_t)(L.lmn[lane] & 0xF) : 0u;
    const uint32_t hi = (uint32_t)__shfl_xor((int)nib, 1);
    if (!(lane & 1) && li < a.nloc) a.lm_next[li >> 1] = (uint8_t)(nib | (hi << 4));
  }
  if constexpr (LDS::kCml) {   // the wave's 64 vertices are one word of the dense bitmap
    if (a.cmk_next) {
      const u64 dm = __ballot(!need || L.tot[lane] == 0u || L.cd[lane] != 0);
      if (lane == 0 && li < a.nloc) a.cmk_next[li >> 6] = dm;
    }
  }
}


// ---------------------------------------------------------------------------
// host side: grid sizing, run-state tests and the launch entry points of the
// kernel units (explicitly instantiated there for W in {1, 2, 4, 8, 16, 32, 64})

inline int grid_for(int64_t work, int64_t per_block) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > (int64_t)0x7fffffff) g = 0x7fffffff;
  return (int)g;
}
// alive sets: F_{r+1} is the OR of every receiver's new row, so partitioned
// contexts OR-reduce their partial sets in the boundary exchange
// (partition.hip).  Only with liveness: without crashes a message stops only
// once its whole component holds it, so F_r never narrows cm & ~seen and the
// bookkeeping is pure cost
inline bool alive_on(const Ctx* c) { return c->d_alive != nullptr && c->liveness_active; }
// the alive set of this round is complete and may narrow targets (alive_on
// alone says the round builds the next one)
inline bool alive_now(const Ctx* c) { return alive_on(c) && c->alive_from >= 0 && c->round >= c->alive_from; }
inline bool state_ready(const Ctx* c) { return c->d_sp != nullptr && c->d_slot[0] != nullptr; }

// pull.hip: every kernel of one expansion round (push or pull, hub passes,
// the degree-split push half) for the context's row width
int launch_round_kernels(Ctx* c, const ExpandArgs& a);
// push.hip
template <int W> void launch_push_w(Ctx* c, ExpandArgs a);            // a push round
template <int W> void launch_split_push_w(Ctx* c, const ExpandArgs& a);   // degree-split round: the push half
template <int W> void launch_acc_clear_w(Ctx* c);                     // ... and its accumulator back to zero
// hub.hip: the hub receivers of a pull round (partials, then the final rows)
template <int W> void launch_hubs_w(Ctx* c, const ExpandArgs& a, bool unfiltered, bool lines);
// liveness.hip: L_r (crash draws, miss counters, detection, seed removal)
int launch_liveness(Ctx* c);
constexpr int DET_CAP = 16384;   // deferred (big) detection candidates per round (more: walked in-wave)

}  // namespace gp
