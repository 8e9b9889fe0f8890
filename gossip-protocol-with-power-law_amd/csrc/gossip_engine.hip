// gossip_engine.hip -- MI355X (gfx950) gossip-propagation engine: round kernels
// and the C-ABI of include/gossip_capi.h.
//
// One gossip round r over all peers at once:
//   L_r  liveness: crash draws, heartbeat-miss counters, 3-miss detection,
//        dead-node reports, seed removal      (Peer.py:298-393, Seed.py:358-406)
//   I_r  injection of messages generated in round r     (Peer.py:395-400)
//   E_r  pull expansion: next[v] = OR_{u in In(v)} frontier[u] & ~seen[v];
//        seen |= next  (forward-once with the Message-List bitmap `seen`;
//        the send loop is Peer.py:402-404, the receive side Peer.py:175-216)
//   X_r  (multi-GPU) RCCL all-gather of the owned next rows + popcounts.
//
// Data layout in HBM (row = W uint64 words = 64*W messages of one vertex):
//   frontier/next  u64[n_alloc][W]   rows whose fpop == 0 are never read
//   fpop           u32[n_alloc]      |frontier(v)|, doubles as the row-valid flag
//   seen           u64[nloc][W]      Message-List of the owned vertices
//   seenpop        u32[nloc]         |seen(v)| -> vertices holding all m skip E_r
//   in-CSR         i64 row_ptr[n+1], i32 col[nnz]
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "gp_internal.h"
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

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

#ifndef GP_BLOCK
#define GP_BLOCK 256
#endif
constexpr int BLOCK = GP_BLOCK;    // 4 waves (GP_BLOCK: experiment builds)
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
// the hub passes the same way (GP_HUB_BLOCK; experiment: 256 = before)
#ifndef GP_HUB_BLOCK
#define GP_HUB_BLOCK 256
#endif
constexpr int HBLOCK = GP_HUB_BLOCK;
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
__device__ __forceinline__ u64* stats_lds() {
  __shared__ u64 rows[WAVES][NST];
  return &rows[0][0];
}
struct WaveStats {
  u64* row;
  bool lead;
  __device__ __forceinline__ void add(int k, u64 x) {
    if (lead) row[k] += x;
  }
};
__device__ __forceinline__ void ws_zero(WaveStats& s) {
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  s.row = stats_lds() + wib * NST;
  s.lead = lane == 0;
  if (lane < NST) s.row[lane] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ void flush_stats(const WaveStats& s, u64* __restrict__ partial) {
  (void)s;
  u64* red = stats_lds();
  __syncthreads();
  if (threadIdx.x < NST) {
    u64 t = 0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w)
      if (w < (int)(blockDim.x >> 6)) t += red[w * NST + threadIdx.x];   // (pull kernels: EWAVES)
    if (t) atomicAdd(&partial[(size_t)threadIdx.x * NPART + (blockIdx.x % NPART)], t);
  }
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

// occupancy target of k_expand (waves per SIMD; 0 = compiler's choice)
#ifndef GP_DETECT_BLOCKS_PER_CU
#define GP_DETECT_BLOCKS_PER_CU 16   // 4 -> 16: C5 304.1-304.5 -> 302.2-302.4 ms per run same-box
#endif
#ifndef GP_SUMMARY_PROBE
#define GP_SUMMARY_PROBE 1
#endif
#ifndef GP_SUMMARY_RATIO
#define GP_SUMMARY_RATIO 256.0
#endif
#ifndef GP_EXPAND_WAVES
#define GP_EXPAND_WAVES 0
#endif
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
template <int W>
struct RowsInFlight { static constexpr int value = W >= 64 ? GP_ROWS_IN_FLIGHT_64 : GP_ROWS_IN_FLIGHT; };

// per-wave LDS of the pull kernels; the mode-specific arrays take one element
// when their mode is compiled out (LDS is what bounds the waves per CU)
constexpr int PRE_IDS = 8;       // active neighbours kept per prefiltered vertex
constexpr int PRE_MAX_DEG = 16;  // in-degree up to which the lane phase probes
// in-degree up to which the wave probes receivers' in-lists together (SCAN_PRE
// rounds), and how many receivers per step
#ifndef GP_WAVE_PRE_MAX
#define GP_WAVE_PRE_MAX 64
#endif
#ifndef GP_WAVE_PRE_N
#define GP_WAVE_PRE_N 4
#endif
template <bool PRE, bool CML>
struct WaveLdsT {
  static constexpr bool kPre = PRE, kCml = CML;
  u64 seen[64];         // early exit: the receiver's seen row (read once, reused by finish_row)
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
};
using WaveLds = WaveLdsT<false, false>;
#define LDS_OF(MODE) WaveLdsT<((MODE) & 3) == SCAN_PRE, ((MODE) & SCAN_CML) != 0>

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
                                   (k_mklm) and the gather loads only its nonzero 128-B lines */ };

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

// line masks (SCAN_LINES): GP_LM_NIBBLE packs two vertices per byte (v even:
// low nibble), halving the array the per-arc probe reads (8 MB at 2^24: a
// byte array's 16 MB missed L2 on most probes, C4 round 2 HBM / alg 1.37)
#ifndef GP_LM_NIBBLE
#define GP_LM_NIBBLE 1
#endif
__device__ __forceinline__ uint8_t lm_of(const uint8_t* __restrict__ lm, int32_t u) {
  if constexpr (GP_LM_NIBBLE) return (uint8_t)((lm[u >> 1] >> ((u & 1) * 4)) & 0xF);
  else return lm[u];
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
#ifndef GP_WORD_SKIP
#define GP_WORD_SKIP 1
#endif
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
  if (GP_WORD_SKIP && ee) {
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
// probes, staging, gather
template <int W, int MODE, class LDS>
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
      int32_t ent = -1;
      if (lane < n) ent = probe<MODE>(a, (col0 != INT32_MIN && j0 == b) ? col0 : a.gcol[j0 + lane]);
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
template <int W, bool DEFER = false, bool CMLW = true, class LDS = WaveLds>
__device__ __forceinline__ void finish_row(const ExpandArgs& a, int v, int64_t i, u64x2 acc, int lane,
                                           int g, int lw, WaveStats& st, LDS& L, bool have_sv,
                                           uint32_t sv_slot, int k = 0) {
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
    store_piece<W>(a.slot[a.wslot], v, lw, sv | nw);   // the whole row: the slot may hold an older one
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
      L.lmn[k] = (uint8_t)lmn;
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
  st.add(S_WRITTEN, 1);
}

// Receivers two at a time, one per half-wave (W = 64).  A half-wave loads a
// whole 64-word row per instruction, so each receiver keeps its rows in flight
// on its own and the dependent chain (column ids -> probes -> rows -> commit)
// is walked for two receivers at once: the latency-bound rounds' lever, since
// 64 VGPRs already give the 8 waves per SIMD the hardware holds.  Same
// commits as finish_row (deferred per-vertex words in L.tot / L.dig / L.cd).
#ifndef GP_PRE_PAIRS
#define GP_PRE_PAIRS 1
#endif
// rows in flight per half-wave in pre_pairs: 2 (70 VGPRs, 7 waves per SIMD)
// against 4 (78, 6 waves): C4 round 1 3.97 -> 3.78 ms same-box
#ifndef GP_PAIR_RIF
#define GP_PAIR_RIF 2
#endif

// receiver side of a pair: half h holds receiver ks (on: the half has one;
// kB < 0: half 1 idle) with its gathered OR acc and its seen row sv
template <int W, class LDS>
__device__ __forceinline__ void pair_finish(const ExpandArgs& a, LDS& L, int h, int lw, bool on, int ks, int kB,
                                            int64_t i, int v, u64x2 acc, u64x2 sv, WaveStats& st) {
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
  for (int o = 16; o > 0; o >>= 1) t ^= __shfl_xor(t, o);
  uint32_t lmn = 0;   // lines of the new bits holding a nonzero word (lm_next; finish_row)
  if (a.lm_next) lmn = lines_of((uint32_t)(__ballot(on && (nw.x | nw.y) != 0ull) >> (32 * h)));
  if (lw == 0 && on && tot) {
    L.tot[ks] = tot;
    L.lmn[ks] = (uint8_t)lmn;
    L.dig[ks] = t;
    if constexpr (LDS::kCml) L.cd[ks] = dense ? 1 : 0;
  }
  const uint32_t tA = (uint32_t)__builtin_amdgcn_readlane((int)tot, 0);
  const uint32_t tB = kB >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)tot, 32) : 0u;
  st.add(S_NEW_BITS, (u64)tA + (u64)tB);
  st.add(S_RECEIVERS, (u64)((tA ? 1 : 0) + (tB ? 1 : 0)));
  st.add(S_WRITTEN, (u64)((tA ? 1 : 0) + (tB ? 1 : 0)));
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

// Done in-neighbours (a.dbits rounds: early exit, no liveness,
// one context).  Without liveness a receiver's new bits are OR_u seen(u) &
// ~seen(v) over all its in-neighbours (ExpandArgs), and every Message-List is
// a subset of the component's messages cmask, so one in-neighbour that held
// all of them at the end of the last round makes the result exactly cmask &
// ~seen(v): the receiver takes the early-exit target and gathers no row.
// Probed for the first GP_DNB_K arcs of the gather order (the biggest
// neighbours, the first to complete), all loads in flight together.  (Not in
// the flat kernel: its 2-arc prefix pass already reads those rows, and the
// extra probe round trip made the 512-message shard's rounds slower.)
#ifndef GP_DNB_K
#define GP_DNB_K 2
#endif
__device__ __forceinline__ bool done_nb(const ExpandArgs& a, int64_t b, int64_t e) {
  int32_t c[GP_DNB_K];
#pragma unroll
  for (int q = 0; q < GP_DNB_K; ++q) c[q] = b + q < e ? a.gcol[b + q] : -1;
  u64 w[GP_DNB_K];
#pragma unroll
  for (int q = 0; q < GP_DNB_K; ++q) w[q] = c[q] >= 0 ? a.dbits[c[q] >> 6] : 0ull;
  bool d = false;
#pragma unroll
  for (int q = 0; q < GP_DNB_K; ++q) d = d || (c[q] >= 0 && ((w[q] >> (c[q] & 63)) & 1ull));
  return d;
}

// Receivers with a done in-neighbour two at a time, one per half-wave (W =
// 64): nothing to gather, so each pair is one round trip (its seen rows and
// the component rows, the latter L2-resident) and the commit
#ifndef GP_DNB_PAIRS
#define GP_DNB_PAIRS 1
#endif
template <int W, bool ALIVE, class LDS>
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
    const int64_t i = base + ks;
    const int v = (int)(a.vbegin + i);
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
    pair_finish<W>(a, L, h, lw, on, ks, kB, i, v, cm, sv, st);
  }
}

// k_expand's commit of the deferred per-vertex words: lane k holds vertex
// base + k (need: it was scanned)
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
      a.sp[v] = (uint8_t)a.wslot;
      a.ws[v] |= (uint8_t)(1u << a.wslot);
      if (a.digest) a.digest[li] ^= L.dig[lane];
      next_arcs = (u64)(uint32_t)max(a.deg_live[v], 0);
    }
  }
  st.add(S_NEXT_ARCS, wave_sum_u64(next_arcs));
  if (a.lm_next) {   // line masks of the next round's senders, two vertices per byte (hubs: 0 here)
    const uint32_t nib = (need && L.tot[lane]) ? (uint32_t)L.lmn[lane] : 0u;
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

// main pull kernel: a wave owns 64 consecutive vertices.  The per-vertex
// checks (sender accounting, down / done / hub / no in-arcs) run lane-parallel
// with coalesced loads; the wave then scans, one receiver at a time, only the
// vertices that can still receive something.  Kept lean on registers (7 waves
// per SIMD): the dense rounds are bound by the rows in flight.
// waves per SIMD asked of the compiler for the alive early-exit variants (C5's
// rounds 3-5; 0: the compiler's choice)
#ifndef GP_ALIVE_WAVES
#define GP_ALIVE_WAVES 0
#endif
// the same for W < 64 (message shards, C3 widths; 0: the compiler's choice):
// 8 on the 2048-message shard (W = 32) 37.6 -> 41.1 ms (r04_ab_waves.txt)
#ifndef GP_NARROW_WAVES
#define GP_NARROW_WAVES 0
#endif
template <int W, int MODE>
struct ExpandWaves {
  static constexpr int value = (MODE & SCAN_ALIVE) != 0 && GP_ALIVE_WAVES > 0 ? GP_ALIVE_WAVES
                               : W < 64 && GP_NARROW_WAVES > 0                ? GP_NARROW_WAVES
                               : GP_EXPAND_WAVES > 0                          ? GP_EXPAND_WAVES
                                                                              : 1;
};
template <int W, int MODE>
__global__ EXPAND_BOUNDS __attribute__((amdgpu_waves_per_eu(ExpandWaves<W, MODE>::value))) void k_expand(ExpandArgs a) {
  constexpr int LPR = Geo<W>::LPR;
  __shared__ LDS_OF(MODE) s_w[EWAVES];
  const int lane = threadIdx.x & 63;
  const int wib = uniform(threadIdx.x >> 6);
  const int g = lane / LPR, lw = lane % LPR;
  auto& L = s_w[wib];
  constexpr bool ALIVE = (MODE & SCAN_ALIVE) != 0;
  constexpr int SCAN = MODE & ~SCAN_ALIVE;
  WaveStats st;
  ws_zero(st);
  const int64_t base = ((int64_t)blockIdx.x * EWAVES + wib) * 64;
  if (base < a.nloc) {
    const int64_t li = base + lane;
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
    if (li < a.nloc) {
      const int v = (int)(a.vbegin + li);
      const uint32_t fp = a.fpop[v];
      act = fp != 0u;
      if (act) sends = (u64)fp * (u64)(uint32_t)max(a.deg_live[v], 0);
      const int64_t b = a.row_ptr[v], e = a.row_ptr[v + 1];
      L.rp[lane] = b;
      if (lane == 63 || li + 1 == a.nloc) L.rp[lane + 1] = e;
      const bool hub = e - b > a.hub_thr;   // split over waves by the hub kernels
      need = !(a.state[v] & (ST_DOWN | ST_SATED)) && a.seenpop[li] < a.done_at[v] && !hub && e > b;
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
#if GP_SUMMARY_PROBE
              if (a.sbits) {   // summary level first: L2-resident, most probes end there
                u64 sw[PRE_IDS];
#pragma unroll
                for (int q = 0; q < PRE_IDS; ++q) sw[q] = c[q] >= 0 ? a.sbits[c[q] >> 12] : 0ull;
#pragma unroll
                for (int q = 0; q < PRE_IDS; ++q)
                  w[q] = ((sw[q] >> ((c[q] >> 6) & 63)) & 1ull) ? a.abits[c[q] >> 6] : 0ull;
              } else
#endif
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
      // their in-lists GP_WAVE_PRE_N at a time (one coalesced pass each, all
      // loads in flight together) instead of one receiver's chain after the
      // other in the serial loop; those with at most PRE_IDS active
      // neighbours join the prefiltered receivers, those with none drop out
      u64 mw = __ballot(need && L.np[lane] == 0xFFu && L.len[lane] <= GP_WAVE_PRE_MAX);
      u64 zero = 0;   // no active in-neighbour: nothing to scan (commit writes fpop_next = 0)
      uint32_t arcs = 0;
      while (mw) {
        int kq[GP_WAVE_PRE_N];
        int32_t c[GP_WAVE_PRE_N];
#pragma unroll
        for (int q = 0; q < GP_WAVE_PRE_N; ++q) {
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
        u64 w[GP_WAVE_PRE_N];
#if GP_SUMMARY_PROBE
        if (a.sbits) {
          u64 sw[GP_WAVE_PRE_N];
#pragma unroll
          for (int q = 0; q < GP_WAVE_PRE_N; ++q) sw[q] = c[q] >= 0 ? a.sbits[c[q] >> 12] : 0ull;
#pragma unroll
          for (int q = 0; q < GP_WAVE_PRE_N; ++q)
            w[q] = ((sw[q] >> ((c[q] >> 6) & 63)) & 1ull) ? a.abits[c[q] >> 6] : 0ull;
        } else
#endif
#pragma unroll
        for (int q = 0; q < GP_WAVE_PRE_N; ++q) w[q] = c[q] >= 0 ? a.abits[c[q] >> 6] : 0ull;
#pragma unroll
        for (int q = 0; q < GP_WAVE_PRE_N; ++q) {
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
    if constexpr (GP_PRE_PAIRS && W == 64 && (MODE & 3) == SCAN_PRE) {
      if (!ee) {   // prefiltered receivers two at a time, the rest below
        const u64 mp = m & __ballot(need && L.np[lane] != 0xFFu);
        pre_pairs<W>(a, L, mp, base, slot_of, st);
        m &= ~mp;
      }
    }
    u64 sat = 0;   // receivers of this wave found sated (alive rounds)
    if constexpr (W == 64 && GP_DNB_PAIRS) {
      if (mdn) {   // done in-neighbours: two receivers at a time, the rest below
        const u64 md = m & mdn;
        dnb_pairs<W, ALIVE>(a, L, md, base, slot_of, st);
        if constexpr (ALIVE) {   // they now hold every alive message of their component: sated too
          if (a.sate) sat |= md;
        }
        m &= ~md;
      }
    }
    while (m) {
      const int k = __ffsll((long long)m) - 1;
      m &= m - 1;
      const int64_t i = base + k;
      const int v = uniform((int)(a.vbegin + i));
      const int64_t vb = L.rp[k], ve = L.rp[k + 1];   // staged by the lane phase
      const uint32_t sv_slot = (uint32_t)__builtin_amdgcn_readlane((int)slot_of, k);
      u64x2 acc = {0, 0}, want = {0, 0};
      // early-exit rounds: the first pass's column ids are loaded beside the
      // target's seen / component rows, one round trip instead of two
#ifndef GP_COL_EARLY
#define GP_COL_EARLY 1
#endif
      int32_t col0 = INT32_MIN;
      if constexpr (GP_COL_EARLY && (MODE & 3) != SCAN_MASKED && (MODE & SCAN_LINES) == 0 && (MODE & SCAN_CML) == 0) {
        if (ee && !((mdn >> k) & 1ull) && lane < (int)min((int64_t)64, ve - vb)) col0 = a.gcol[vb + lane];
      }
      // line-mask rounds (no early exit): the seen row comes up front too, beside
      // the first column ids, parked in LDS for the commit (one round trip less)
#ifndef GP_LINES_SEEN_EARLY
#define GP_LINES_SEEN_EARLY 1
#endif
      constexpr bool SEEN_EARLY = GP_LINES_SEEN_EARLY && W == 64 && (MODE & SCAN_LINES) != 0;
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
          gather_scan<W, SCAN>(a, vb, vb + L.len[k], L, lane, g, lw, acc, st, ee, want, col0);
          if ((tw >> k) & 1ull) {   // degree-split: the accumulator row (not staged: a scanned receiver)
            if (g == 0) acc |= load_piece<W>(a.acc, v, lw);
            st.add(S_GATHERED, 1);
            st.add(S_ROW_BYTES, (u64)(8 * W));
          }
        }
      } else {
        gather_scan<W, SCAN>(a, vb, ve, L, lane, g, lw, acc, st, ee, want, col0);
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
      finish_row<W, true, (MODE & SCAN_CML) != 0>(a, v, i, acc, lane, g, lw, st, L, ee || SEEN_EARLY, sv_slot, k);
    }
    alive_flush<W>(a, L.alive, lane);
    commit_vertices(a, L, li, need, st);
    if constexpr (ALIVE) {
      if (sat && ((sat >> lane) & 1ull)) a.state[a.vbegin + li] |= ST_SATED;
    }
  }
  flush_stats(st, a.partial);
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
// row wave-instructions in flight per lane (VGPRs vs occupancy: 2 -> 66 VGPRs
// at W = 8).  Measured on the message shards (same box A/B): W = 8 (64-B rows,
// 16 per instruction) 15.6 -> 15.2 ms with 3 for a 512-message shard; W = 16
// 28.3 -> 24.4 ms with 4 and 22.9 ms with 6 for a 1024-message shard (8: 25.6)
#ifndef GP_FLAT_RIF_NARROW
#define GP_FLAT_RIF_NARROW 3
#endif
#ifndef GP_FLAT_RIF_WIDE
#define GP_FLAT_RIF_WIDE 6
#endif
template <int W>
struct FlatRIF { static constexpr int value = W >= 16 ? GP_FLAT_RIF_WIDE : GP_FLAT_RIF_NARROW; };
// receivers per wave: 64, or 32 at W = 32 so that the LDS accumulators (8 KB
// per wave) leave room for 4 blocks per CU
template <int W>
struct FlatNR { static constexpr int value = W >= 32 ? 32 : 64; };
template <int W>
struct FlatLds {
  static constexpr int NR = FlatNR<W>::value;
  u64 acc[NR][W];               // OR accumulators of the wave's NR receivers
  int32_t idx[64];              // active neighbours of one chunk
  int8_t vtx[64];               // their receiver (lane) in the wave
  int8_t own[FLAT_CAP];         // receiver lane owning each arc position of the window
  uint32_t tot[NR];             // receiver side: new bits of receiver k
  u64 dig[NR];                  // its digest terms
  int8_t rd[NR];                // its seen row was read
  u64 alive[W];                 // OR of the new rows this wave wrote (alive_next); W words, so
                                // that W = 16 keeps 4 blocks per CU
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
#if GP_SUMMARY_PROBE
      if constexpr (MODE != SCAN_UNFILTERED)
        if (a.sbits) {
          u64 sw[QA];
#pragma unroll
          for (int q = 0; q < QA; ++q) sw[q] = col[q] >= 0 ? a.sbits[col[q] >> 12] : 0ull;
#pragma unroll
          for (int q = 0; q < QA; ++q)
            raw[q] = ((sw[q] >> ((col[q] >> 6) & 63)) & 1ull) ? a.abits[col[q] >> 6] : 0ull;
        }
#endif
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
// receiver (its biggest neighbours: gather order) go in a first pass, arcs up to
// GP_FLAT_EE_PREFIX2 in a second; only receivers still missing messages of
// their component after a pass scan further.
#ifndef GP_FLAT_EE_PREFIX
#define GP_FLAT_EE_PREFIX 2
#endif
#ifndef GP_FLAT_EE_PREFIX2
#define GP_FLAT_EE_PREFIX2 0
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
  ws_zero(st);
  const int64_t base = ((int64_t)blockIdx.x * EWAVES + wib) * NR;
  if (base < a.nloc) {
    alive_zero<W>(a, F.alive, lane);
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
    constexpr uint32_t K1 = GP_FLAT_EE_PREFIX, K2 = GP_FLAT_EE_PREFIX2;
    constexpr bool ee = EE && K1 > 0;   // compile-time: the lean kernel keeps its VGPRs
    constexpr int npass = !ee ? 1 : (K2 > K1 ? 3 : 2);
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
  flush_stats(st, a.partial);
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
#ifndef GP_REC_FLAT
#define GP_REC_FLAT 1
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
      gather_scan<W, MODE>(a, h.beg, h.end, s_w[wib], lane, g, lw, acc, st, ee, want);
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
      finish_row<W>(a, v, i, acc, lane, g, lw, st, s_w[wib], false, a.sp[v]);
    }
  }
  alive_flush<W>(a, s_w[wib].alive, lane);
  flush_stats(st, a.partial);
}

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

// frontier activity bitmap: bit v = (fpop[v] != 0), one word per 64 vertices.
// With dbits (single context, early-exit round without liveness) also the done
// bitmap: bit v = v holds every message of its component (seenpop == done_at,
// components with messages only), as of the end of the last round.
// With liveness (sated: the state bytes) the done bitmap is bit v = v is up and
// sated: it holds every alive message of its component, and
// the alive sets only shrink once no injection is left.
__global__ __launch_bounds__(BLOCK) void k_mkbits(const uint32_t* __restrict__ fpop, u64* __restrict__ abits,
                                                  int64_t n, const uint32_t* __restrict__ seenpop,
                                                  const uint32_t* __restrict__ done_at, u64* __restrict__ dbits,
                                                  const uint8_t* __restrict__ sated) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  for (int64_t v0 = (int64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63); v0 < n; v0 += stride) {
    const int64_t v = v0 + lane;
    const u64 m = __ballot(v < n && fpop[v] != 0u);
    if (lane == 0) abits[v0 >> 6] = m;
    if (dbits) {
      bool d = false;
      if (v < n) {
        if (sated) {
          d = (sated[v] & (ST_SATED | ST_DOWN)) == ST_SATED;
        } else {
          const uint32_t t = done_at[v];
          d = t != 0u && seenpop[v] == t;
        }
      }
      const u64 dm = __ballot(d);
      if (lane == 0) dbits[v0 >> 6] = dm;
    }
  }
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
    if constexpr (GP_LM_NIBBLE) {   // (v0 is a multiple of 64: whole bytes per wave)
      if (lane < 32 && v0 + 2 * lane < n)
        lm[(v0 >> 1) + lane] = (uint8_t)(out[2 * lane] | (out[2 * lane + 1] << 4));
    } else if (v < n) {
      lm[v] = out[lane];
    }
    wave_sync_lds();
  }
  flush_stats(st, partial);
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
constexpr int DET_CAP = 16384;      // deferred candidates per round (more: walked in-wave)
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

// ---------------------------------------------------------------------------
// host side

static int grid_for(int64_t work, int64_t per_block) {
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
static bool alive_on(const Ctx* c) { return c->d_alive != nullptr && c->liveness_active; }

static void fill_expand(Ctx* c, ExpandArgs& a) {
  a.alive = alive_on(c) ? c->d_alive + (size_t)c->cur * c->words : nullptr;
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

// narrow rows (W <= GP_PUSH_LANES_MAXW): the receivable bitmap and the
// lane-parallel receiver side (k_mkneed, k_apply_lanes)
#ifndef GP_PUSH_LANES_MAXW
#define GP_PUSH_LANES_MAXW 32
#endif
template <int W>
static void launch_push_w(Ctx* c, ExpandArgs a) {
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
  // W = 32 rows take the per-receiver kernel, except in dense near-done rounds
  // (most messages held, last round's new bits >= m/4 per vertex): there the
  // flat kernel's 2-arc prefix pass completes most receivers from their hub
  // rows (2048-message shard round 4: 10.2 -> 6.6 ms; round 5, with m/16,
  // went 3.2 -> 4.2 ms, hence m/4)
#ifndef GP_FLAT_NEAR_DONE
#define GP_FLAT_NEAR_DONE 1
#endif
  const bool flat_nd = GP_FLAT_NEAR_DONE && W == 32 && c->cfg.flat_max_words > 0 && a.near_done &&
                       (double)c->prev_new_bits * 4.0 >= (double)c->n * (double)c->m;
  // W = 32 in a dense filtered round without early exit (a shard's round 2):
  // the flat kernel's arc stream beats the per-receiver loop there (10.3 ->
  // 9.8 ms on the 2048-message shard)
#ifndef GP_FLAT_DENSE32
#define GP_FLAT_DENSE32 0
#endif
  const bool flat_d32 = GP_FLAT_DENSE32 && W == 32 && c->cfg.flat_max_words > 0 && !a.unfiltered &&
                        !a.early_exit && !c->prefilter_now && !c->arc_mask_now;
  const bool flat = W <= 32 && (W <= c->cfg.flat_max_words || flat_nd || flat_d32);
  const bool masked = !a.unfiltered && !flat && c->arc_mask_now;
  if (masked) {   // mask words of the owned vertices' in-arcs
    const int64_t kb = c->h_row_ptr[0] >> 6;
    const int64_t ke = (c->h_row_ptr[(size_t)c->nloc()] + 63) >> 6;
    if (ke > kb)
      hipLaunchKernelGGL(k_arcmask, dim3(grid_for(ke - kb, (int64_t)WAVES * AM_WORDS)), dim3(BLOCK), 0, c->stream,
                         c->d_gcol, c->d_abits, c->d_amask, kb, c->nnz_l);
  }
  const int mode = a.unfiltered ? SCAN_UNFILTERED : SCAN_FILTERED;
  if (a.prehi) {   // degree-split round, push half: senders of in-degree < split_deg
    ExpandArgs p = a;
    p.split_push = 1;
    const int64_t nwords = (c->n_alloc + 63) / 64;
    hipLaunchKernelGGL(k_active_list, dim3(grid_for(nwords, BLOCK)), dim3(BLOCK), 0, c->stream, c->d_abits, nwords,
                       a.orp, PUSH_CHUNK, c->d_active, c->d_big, c->d_stats, (const int64_t*)c->d_row_ptr,
                       c->cfg.split_deg);
    hipLaunchKernelGGL(k_push<W>, dim3(c->cu_count * 8 * GS), dim3(BLOCK), 0, c->stream, p);
    hipLaunchKernelGGL(k_push_big<W>, dim3(c->cu_count * 4 * GS), dim3(BLOCK), 0, c->stream, p);
  }
  (void)hipEventRecord(c->ev[4], c->stream);
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
  } else if (a.nloc > 0) {
    const dim3 grid(grid_for(a.nloc, per_block));
    bool alive_ee = false;   // unfiltered under liveness (parked rows) with early exit
    if constexpr (W >= 32) alive_ee = mode == SCAN_UNFILTERED && a.alive && a.early_exit;
    if (alive_ee) {
      if constexpr (W >= 32)
        hipLaunchKernelGGL((k_expand<W, SCAN_UNFILTERED | SCAN_ALIVE>), grid, dim3(EBLOCK), 0, c->stream, a);
    } else if (mode == SCAN_UNFILTERED) {
      hipLaunchKernelGGL((k_expand<W, SCAN_UNFILTERED>), grid, dim3(EBLOCK), 0, c->stream, a);
    }
    else if (masked)
      hipLaunchKernelGGL((k_expand<W, SCAN_MASKED>), grid, dim3(EBLOCK), 0, c->stream, a);
    else if (W == 64 && (a.cmk || a.cmk_next)) {   // compact Message-Lists read and / or written
      if constexpr (W == 64) {
        if (GP_REC_FLAT && a.cmk && !a.early_exit && !c->prefilter_now && !a.alive)
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
  if (c->n_hub_items > 0) {
    ExpandArgs h = a;
    h.n_items = c->n_hub_items;
    const dim3 grid(grid_for(h.n_items, HWAVES));
    if (mode == SCAN_UNFILTERED)
      hipLaunchKernelGGL((k_hub_partial<W, SCAN_UNFILTERED>), grid, dim3(HBLOCK), 0, c->stream, h);
    else
      hipLaunchKernelGGL((k_hub_partial<W, SCAN_FILTERED>), grid, dim3(HBLOCK), 0, c->stream, h);
    h.n_items = c->n_hubs;
    hipLaunchKernelGGL(k_hub_final<W>, dim3(grid_for(h.n_items, HWAVES)), dim3(HBLOCK), 0, c->stream, h);
  }
  // kernel_ms brackets the pull kernel and the hub passes: the round's
  // counters (row bytes, arcs scanned, rows written) include the hubs' share
  (void)hipEventRecord(c->ev[5], c->stream);
  if (a.prehi) {   // degree-split round: the accumulator back to all-zero
    const int64_t nwords = (c->n_alloc + 63) / 64;
    hipLaunchKernelGGL(k_acc_clear<W>, dim3(std::max(1, std::min(grid_for(nwords, WAVES), c->cu_count * 8 * GS))),
                       dim3(BLOCK), 0, c->stream, c->d_tbits, c->d_acc, nwords);
  }
}

#ifndef GP_PARK
#define GP_PARK 1
#endif
#ifndef GP_EE_DIV
#define GP_EE_DIV 16.0
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
  c->early_exit_now = c->cfg.early_exit != 0 &&
                      ((double)c->prev_new_bits * GP_EE_DIV >= (double)c->n * (double)c->m ||
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
  // narrow rows: a round that pushes only because of the narrow scale pulls
  // as a degree-split round instead when that is on (its prefix probes are a
  // fraction of the arcs, its push half only the low-degree senders' arcs)
#ifndef GP_SPLIT_NARROW
#define GP_SPLIT_NARROW 1
#endif
  if (GP_SPLIT_NARROW && c->mode_push && c->cfg.split_deg > 0 && !c->local && c->nloc() == c->n_alloc &&
      est * c->cfg.push_ratio > (double)c->nnz)
    c->mode_push = false;
  c->push_est = est;
  if (c->mode_push && c->nloc() > 0)
    GP_HIP(hipMemsetAsync(c->d_fpop[c->cur ^ 1], 0, (size_t)c->nloc() * 4, c->stream));
  // unfiltered pull when (nearly) every vertex is a sender: last round's
  // receivers + this round's injected origins >= unfiltered_pct % of n.  With
  // liveness a crashed vertex's Message-List may hold bits it never sent, so
  // the down vertices' rows are parked first (k_park; one vertex set per
  // context, hence not in a vertex partition, whose ghosts' rows are frontiers)
  const double senders = (double)c->prev_receivers + (double)c->inj_groups_at(r);
  c->unfiltered_now = !c->mode_push && c->cfg.unfiltered_pct > 0 &&
                      senders * 100.0 >= (double)c->cfg.unfiltered_pct * (double)c->n;
  if (c->unfiltered_now && c->liveness_active) {
    if (c->local || c->park_failed || !GP_PARK) {
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
#ifndef GP_DONE_NB
#define GP_DONE_NB 1
#endif
  c->dnb_now = GP_DONE_NB && c->early_exit_now && !c->mode_push && !c->liveness_active && !c->local &&
               c->nloc() == c->n_alloc && c->words > c->cfg.flat_max_words &&
               (double)c->held_bits * 2.0 >= (double)c->n * (double)c->m;
  // With liveness the done bitmap is the sated marks (up and sated: holds every
  // alive message of its component; k_mkbits): a receiver with such an
  // in-neighbour receives exactly cmask & F_r & ~seen, since every bit of it
  // lies in that neighbour's frontier (it sent everything older while both were
  // up, and crashes are final).  From the round after the first marking round.
#ifndef GP_DONE_NB_LIVE
#define GP_DONE_NB_LIVE 1
#endif
  if (GP_DONE_NB_LIVE && !c->dnb_now && c->liveness_active && alive_on(c) && c->early_exit_now && !c->mode_push &&
      !c->local && c->nloc() == c->n_alloc && c->words > c->cfg.flat_max_words && c->sate_since >= 0 &&
      c->round > c->sate_since)
    c->dnb_now = true;
  hipLaunchKernelGGL(k_mkbits, dim3(std::max(1, std::min(grid_for(c->n_alloc, BLOCK), c->cu_count * 8 * GS))),
                     dim3(BLOCK), 0, c->stream, c->d_fpop[c->cur], c->d_abits, c->n_alloc,
                     c->d_seenpop, c->d_done_at, c->dnb_now ? c->d_dbits : nullptr,
                     c->dnb_now && c->liveness_active ? (const uint8_t*)c->d_state : nullptr);
  // filtered pull: probe every arc inside the scan, or build the per-arc mask
  // first (pays once the probes are many: senders >= arc_mask_permille of n)
  c->arc_mask_now = !c->mode_push && !c->unfiltered_now && c->cfg.arc_mask_permille > 0 &&
                    senders * 1000.0 >= (double)c->cfg.arc_mask_permille * (double)c->n;
  // summary probes: filtered rounds of overlays whose activity bitmap outgrows
  // an XCD's L2, while few enough vertices send that most summary bits are 0
  c->sum_now = false;
#if GP_SUMMARY_PROBE
  if (!c->mode_push && !c->unfiltered_now && !c->arc_mask_now && c->cfg.summary_min_n > 0 &&
      c->n_alloc >= c->cfg.summary_min_n &&
      senders * GP_SUMMARY_RATIO <= (double)c->n) {
    const int64_t nwords = (c->n_alloc + 63) / 64;
    hipLaunchKernelGGL(k_mksum, dim3(grid_for((nwords + 63) / 64, WAVES)), dim3(BLOCK), 0, c->stream,
                       c->d_abits, c->d_sbits, nwords);
    c->sum_now = true;
  }
#endif
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
#ifndef GP_LINE_MASKS
#define GP_LINE_MASKS 1
#endif
  c->lines_now = GP_LINE_MASKS && c->words == 64 && c->d_lm != nullptr && !c->mode_push && !c->unfiltered_now &&
                 !c->arc_mask_now && !c->early_exit_now && c->n_alloc <= (int64_t(1) << 27);   // (u << 4) | lines
  // this round's 64-word pull commits write the next round's masks: one
  // context (ghosts' rows come from the exchange), per-receiver kernel, no
  // records; under liveness k_churn zeroes a crashing sender's nibble with
  // its fpop (round 4 of the build; k_mklm ran there until then)
#ifndef GP_LM_WRITE
#define GP_LM_WRITE 1
#endif
  // (only sparse rounds: a line-mask round follows a round with few new bits,
  // and early-exit rounds would pay the commits' extra stores for nothing --
  // C4 rounds 3-4 +0.3 ms when every pull wrote them)
#ifndef GP_LM_WRITE_LIVE
#define GP_LM_WRITE_LIVE 1
#endif
  c->lm_write_now = GP_LM_WRITE && c->words == 64 && c->d_lmw[0] != nullptr && !c->mode_push &&
                    !c->early_exit_now && !c->local && !c->cml_read_now &&
                    (GP_LM_WRITE_LIVE || !c->liveness_active) &&
                    !c->cml_write_now;
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
  if (c->split_now) {   // accumulator rows as rows of this round's slot buffer (same stride)
    const ptrdiff_t d = reinterpret_cast<const char*>(c->d_acc) - reinterpret_cast<const char*>(c->d_slot[c->cur]);
    const ptrdiff_t rb = (ptrdiff_t)c->words * 8;
    const int64_t row = d / rb;
    c->split_now = d % rb == 0 && row >= (int64_t)INT32_MIN && row + c->n_alloc <= (int64_t)INT32_MAX;
    c->acc_row = (int32_t)row;
  }
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
#ifndef GP_SATE
#define GP_SATE 1
#endif
  a.sate = GP_SATE && alive_on(c) && c->early_exit_now && c->round >= c->last_inject_round ? 1 : 0;
  if (a.sate && c->sate_since < 0) c->sate_since = c->round;
  c->lines_ran = c->lines_from_commits = false;
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

static void free_state(Ctx* c) {
  dfree(&c->d_slot[2]);
  c->park_failed = false;
  for (int k = 0; k < 2; ++k) {
    dfree(&c->d_slot[k]);
    dfree(&c->d_frx[k]);
    dfree(&c->d_fpop[k]);
  }
  dfree(&c->d_sp); dfree(&c->d_ws);
  dfree(&c->d_seenpop); dfree(&c->d_first); dfree(&c->d_digest);
  dfree(&c->d_state); dfree(&c->d_miss); dfree(&c->d_deg_live); dfree(&c->d_cand);
  dfree(&c->d_det_big); dfree(&c->d_det_pre); dfree(&c->d_det_live); dfree(&c->d_det_cur); dfree(&c->d_det_base);
  dfree(&c->d_msg_cov); dfree(&c->d_reports); dfree(&c->d_abits); dfree(&c->d_dbits); dfree(&c->d_lm); dfree(&c->d_lmw[0]); dfree(&c->d_lmw[1]); dfree(&c->d_sbits); dfree(&c->d_amask); dfree(&c->d_cml[0]); dfree(&c->d_cml[1]); dfree(&c->d_cmk[0]); dfree(&c->d_cmk[1]); dfree(&c->d_done_at);
  dfree(&c->d_done_at0); dfree(&c->d_cmask0); dfree(&c->d_lostcnt); dfree(&c->d_alive);
  dfree(&c->d_acc); dfree(&c->d_tbits); dfree(&c->d_nbits); dfree(&c->d_touched); dfree(&c->d_active); dfree(&c->d_big);
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
  for (int k = 0; k < 2; ++k) {
    GP_TRY(dalloc(&c->d_slot[k], na * W));
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
  if (c->words == 64) GP_TRY(dalloc(&c->d_lm, GP_LM_NIBBLE ? (na + 1) / 2 + 32 : na));
  for (int k = 0; k < 2; ++k) {
    dfree(&c->d_lmw[k]);
    if (c->words == 64 && GP_LM_NIBBLE) GP_TRY(dalloc(&c->d_lmw[k], (na + 1) / 2 + 64));
  }
#if GP_SUMMARY_PROBE
  GP_TRY(dalloc(&c->d_sbits, (na + 4095) / 4096));
#endif
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
  GP_TRY(dalloc(&c->d_acc, nl * W));   // push accumulators of the owned receivers
  GP_HIP(hipMemsetAsync(c->d_acc, 0, nl * W * 8, c->stream));
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

static bool state_ready(const Ctx* c) { return c->d_sp != nullptr && c->d_slot[0] != nullptr; }

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
  dfree(&c->d_row_ptr); dfree(&c->d_col); dfree(&c->d_out_row_ptr); dfree(&c->d_out_col);
  dfree(&c->d_deg_out); dfree(&c->d_comp); dfree(&c->d_abits); dfree(&c->d_dbits); dfree(&c->d_lm); dfree(&c->d_lmw[0]); dfree(&c->d_lmw[1]); dfree(&c->d_sbits); dfree(&c->d_amask); dfree(&c->d_cml[0]); dfree(&c->d_cml[1]); dfree(&c->d_cmk[0]); dfree(&c->d_cmk[1]); dfree(&c->d_done_at);
  dfree(&c->d_done_at0); dfree(&c->d_cmask0); dfree(&c->d_lostcnt); dfree(&c->d_alive);
  dfree(&c->d_gcol); dfree(&c->d_prehi); dfree(&c->d_midx); dfree(&c->d_cmask);
  dfree(&c->d_acc); dfree(&c->d_tbits); dfree(&c->d_nbits); dfree(&c->d_touched); dfree(&c->d_active); dfree(&c->d_big);
  dfree(&c->d_inj_origin); dfree(&c->d_inj_bits); dfree(&c->d_inj_cnt);
  dfree(&c->d_slot[2]);
  for (int k = 0; k < 2; ++k) { dfree(&c->d_slot[k]); dfree(&c->d_frx[k]); dfree(&c->d_fpop[k]); }
  dfree(&c->d_sp); dfree(&c->d_ws);
  dfree(&c->d_seenpop); dfree(&c->d_first); dfree(&c->d_digest);
  dfree(&c->d_state); dfree(&c->d_miss); dfree(&c->d_deg_live); dfree(&c->d_cand);
  dfree(&c->d_det_big); dfree(&c->d_det_pre); dfree(&c->d_det_live); dfree(&c->d_det_cur); dfree(&c->d_det_base);
  dfree(&c->d_msg_cov); dfree(&c->d_reports); dfree(&c->d_stats);
  dfree(&c->d_hub_items); dfree(&c->d_hubs); dfree(&c->d_hub_item_ptr);
  dfree(&c->d_hub_partial); dfree(&c->d_hub_pnz);
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
  c->pending_crash = false;
  c->msg_forwards_valid = true;
  c->last_reports = 0;
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
  std::vector<uint8_t> st((size_t)c->n_alloc);
  GP_HIP(hipStreamSynchronize(c->stream));
  GP_TRY(copy_sync(c, st.data(), c->d_state, (size_t)c->n_alloc, hipMemcpyDeviceToHost));
  for (int32_t k = 0; k < nverts; ++k) {
    const int64_t v = c->to_local(verts[k]);
    if (v >= 0 && !(st[(size_t)v] & ST_DOWN)) st[(size_t)v] |= ST_PENDING;
  }
  GP_TRY(copy_sync(c, c->d_state, st.data(), (size_t)c->n_alloc, hipMemcpyHostToDevice));
  if (nverts > 0) {
    c->liveness_active = true;
    c->pending_crash = true;
  }
  return 0;
}

}  // extern "C"

namespace gp {

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
  }

  auto it = c->inject.find(r);
  if (it != c->inject.end() && it->second.cnt > 0) {
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
  if (out) {
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
                                       (c->lines_from_commits ? 16 : 0) | (c->split_now ? 32 : 0);
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
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, c->ev[1], c->ev[2]);
    out->expand_ms = ms;
    (void)hipEventElapsedTime(&ms, c->ev[2], c->ev[3]);
    out->exchange_ms = ms;
    (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[3]);
    out->round_ms = ms;
  }
  c->last_reports = (int64_t)h[S_REPORT_CURSOR];
  c->prev_next_arcs = h[S_NEXT_ARCS];
  c->prev_new_bits = h[S_NEW_BITS];
  c->prev_receivers = h[S_RECEIVERS];
  c->held_bits += h[S_INJECTED] + h[S_NEW_BITS];
  c->cml_written_prev = c->cml_write_now;
  c->lm_written_prev = c->lm_write_now;
  c->cur ^= 1;
  c->round = r + 1;
  return 0;
}

}  // namespace gp

extern "C" {

int gp_round(gp_ctx* c, gp_round_stats* out) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  if (c->local && !c->comm)
    return set_error(GP_ESTATE, "a partitioned context exchanges over RCCL (gp_comm_init) or in gp_round_group");
  GP_TRY(round_launch(c));
  GP_TRY(round_exchange_rccl(c));
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
