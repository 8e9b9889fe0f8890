// gp_internal.h -- context layout and helpers shared by the translation units of
// libgossip_hip.so.  Not part of the ABI (include/gossip_capi.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "../../include/gossip_capi.h"
#include "gp_common.h"

namespace gp {

typedef unsigned long long u64;

// stats slots in the device counter block (u64 each)
// slots [0, NST) are per-block partial sums (all-reduced across ranks);
// the cursors above are rank-local device counters
enum StatSlot {
  S_INJECTED = 0, S_LOST, S_NEW_BITS, S_RECEIVERS, S_SENDS, S_ACTIVE, S_CRASHED,
  S_REPORTS, S_REMOVALS, S_DUP, S_ARCS, S_GATHERED, S_SEEN_READ, S_WRITTEN,
  S_VISITED, S_NEXT_ARCS, S_ATOMICS, S_ROW_BYTES,
  S_XROWS, S_XBYTES,   // boundary entries / bytes sent (vertex partition, written by the pack step)
  S_DNB,               // receivers completed from a done in-neighbour (k_expand)
  S_LM_ROWS,           // senders' rows read by k_mklm to build line masks
  S_ALIASED,           // receivers committed as an alias of their component row (no row write, §3.2)
  NST,
  // boundary entries the unpack found inconsistent with the exchange plan
  // (partition.hip k_rx_unpack); all-reduced with the counters, fails the round
  S_XERR = NST + 1,
  S_REPORT_CURSOR = 26, S_CAND, S_ACTIVE_CURSOR, S_BIG_CURSOR, S_TOUCH_CURSOR, S_DET_BIG,
  S_ULIST   // entries of the next round's receiver list (k_expand survivors)
};
static_assert(S_XERR < S_REPORT_CURSOR, "S_XERR must be inside the all-reduced counter slots");

struct HubItem {       // one wave's share of a hub's in-list
  int32_t v;           // hub vertex
  int32_t hub;         // index into the hub table
  int64_t beg, end;    // arc range
};

struct InjectSpan { int64_t off; int64_t cnt; };

struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[6] = {};
  gp_config cfg{};

  // graph (full, replicated on every rank)
  int64_t n = 0, nnz = 0;
  int directed = 0;
  int64_t* d_row_ptr = nullptr;
  int32_t* d_col = nullptr;
  int64_t* d_out_row_ptr = nullptr;   // directed only
  int32_t* d_out_col = nullptr;
  int32_t* d_deg_out = nullptr;
  int32_t* d_comp = nullptr;          // weakly connected component label (min vertex id)
  std::vector<int64_t> h_row_ptr;     // host copy (hub table, partition)

  // partition.  Kernels address vertices by LOCAL id: one rank (nranks == 1)
  // holds the whole overlay and local == global; a vertex-partitioned context
  // (nranks > 1, partition.hip) holds its owned slice as local ids [0, nloc),
  // then its ghosts -- the non-owned in-neighbours of owned vertices, sorted by
  // global id, hence grouped by owner -- then the message origins that are
  // neither ("extras", so that every rank sees every origin's liveness).
  int32_t rank = 0, nranks = 1;
  std::vector<int64_t> h_bounds;      // [nranks + 1] owned slices (xplan.h partition_bounds)
  int64_t vbegin = 0, vend = 0;       // owned vertices, GLOBAL ids
  int64_t n_alloc = 0;                // local vertex slots: nloc + nghost + nextra
  bool local = false;                 // vertex-partitioned (local ids != global ids)
  int64_t nghost = 0, nextra = 0;
  int64_t nnz_l = 0;                  // arcs of the device CSR (local CSR when partitioned)
  int32_t* d_l2g = nullptr;           // [n_alloc] global id of each local vertex (partitioned only)
  std::vector<int32_t> h_l2g;         // host copy
  std::vector<int32_t> h_comp_g;      // global component labels (extras need theirs)
  std::vector<int32_t> h_deg_g;       // global degrees (partitioned: extras, inj_arcs)
  int64_t base_nv = 0;                // nloc + nghost (local slots before the extras)
  // boundary exchange (partitioned): the owned vertices that are
  // ghosts on rank q, peer-major (flat entry t, [bnd_ptr[q], bnd_ptr[q+1])) and
  // vertex-major (owned boundary vertex k -> its entries).  Rank q's ghosts of
  // owner p are, in the same order, exactly B_pq: no id lists are exchanged.
  std::vector<int64_t> h_bnd_ptr;     // [nranks + 1]
  std::vector<int64_t> h_gh_ptr;      // [nranks + 1] ghost index offsets per owner
  int64_t n_bnd = 0, n_bvx = 0;       // flat entries, owned boundary vertices
  int32_t* d_bnd_e = nullptr;         // [n_bnd] index of entry t within its peer list
  int32_t* d_bnd_k = nullptr;         // [n_bnd] vertex-major index of entry t
  int32_t* d_bvx_v = nullptr;         // [n_bvx] owned local vertex
  int32_t* d_bvx_ptr = nullptr;       // [n_bvx + 1] -> d_bvx_t
  int32_t* d_bvx_t = nullptr;         // [n_bnd] entries of vertex k
  int64_t* d_bnd_ptr = nullptr;       // [nranks + 1]
  u64* d_bvx_info = nullptr;          // [n_bvx] word mask of this round's new row (0: none)
  uint8_t* d_bvx_flag = nullptr;      // [n_bvx] bit 0: new row, bit 1: removed this round
  u64* d_bnd_scan = nullptr;          // [n_bnd + 1] exclusive scan of (heads << 40 | words)
  u64* d_xsize = nullptr;             // [max(n_bnd, nghost) + 1] entry sizes (scan input)
  u64* d_sbuf_h = nullptr;            // send heads (e | flags << 32 | popc << 40)
  u64* d_sbuf_w = nullptr;            // send words (mask word, then the nonzero words)
  u64* d_rbuf_h = nullptr;            // received heads, by sender rank
  u64* d_rbuf_w = nullptr;            // received words, by sender rank
  u64* d_rscan = nullptr;             // [nghost + 1] word offsets of the received entries
  u64* d_cnt = nullptr;               // [4 * nranks] per peer: head start, heads, word start, words
  u64* d_cnt_all = nullptr;           // [nranks][4 * nranks]
  u64* h_cnt_all = nullptr;           // pinned copy
  std::vector<int64_t> h_ghosts_all;  // [nranks][nranks] ghosts rank d holds of owner q (checked once)
  u64* d_alive_all = nullptr;         // [nranks][W]
  void* d_scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;

  // messages
  int32_t m = 0, words = 0;
  std::map<int32_t, InjectSpan> inject;   // round -> groups
  int32_t last_inject_round = -1;
  int64_t n_groups = 0;               // (round, origin) injection groups
  bool done_at_valid = false;
  int32_t* d_inj_origin = nullptr;
  u64* d_inj_bits = nullptr;
  uint32_t* d_inj_cnt = nullptr;

  // per-run state
  // Message-List slots: v's seen row lives in d_slot[d_sp[v]];
  // round r reads S[r & 1] and writes S[(r + 1) & 1]; cur == r & 1
  u64* d_slot[3] = {nullptr, nullptr, nullptr};    // [n_alloc][W]; slot 2: parked rows (below)
  u64* d_rows = nullptr;            // the allocation of d_slot[0], d_slot[1] and d_acc (in that order)
  // parking: an unfiltered pull under liveness reads every in-neighbour's row
  // of slot r & 1, so before it the rows of down vertices move to slot 2
  // (sp = 2) and both read-slot rows are zeroed; slot 2 is allocated lazily
  bool park_failed = false;         // slot 2 could not be allocated: no unfiltered pull under liveness
  uint8_t* d_sp = nullptr;          // [n_alloc] slot of v's seen row (0xFF: none)
  uint8_t* d_ws = nullptr;          // [n_alloc] bit p: slot p written this run
  u64* d_frx[2] = {nullptr, nullptr};     // exact frontier rows (track_msg_forwards; partitioned)
  int64_t frx_rows = 0;                   // rows d_frx covers (partitioned: the owned ones)
  uint32_t* d_fpop[2] = {nullptr, nullptr};    // [n_alloc]
  int cur = 0;
  uint32_t* d_seenpop = nullptr;    // [nloc]
  uint8_t* d_first = nullptr;       // [nloc][W*64]
  u64* d_digest = nullptr;     // [nloc]
  uint8_t* d_state = nullptr;       // [n_alloc]
  uint8_t* d_miss = nullptr;        // [n_alloc]
  int32_t* d_deg_live = nullptr;    // [n_alloc]
  int32_t* d_cand = nullptr;        // [n] detection candidates of a round
  int32_t* d_det_big = nullptr;     // deferred (big) detection candidates and their counters (k_det_big_*)
  int64_t* d_det_pre = nullptr;
  uint32_t* d_det_live = nullptr;
  uint32_t* d_det_cur = nullptr;
  u64* d_det_base = nullptr;
  // [n_alloc/64] frontier_r activity bitmap (fpop != 0): 2 MB at 2^24
  double push_est = 0.0;            // sender arcs the direction estimate saw this round
  u64* d_nbits = nullptr;           // [n_alloc/64] narrow push rounds: receivable vertices (k_mkneed)
  u64* d_abits = nullptr;
  u64* d_sbits = nullptr;   // summary level of d_abits (summary probes)
  // [n_alloc/64] done bitmap of early-exit rounds without liveness (single
  // context): bit v = v held every message of its component at the end of the
  // last round (done in-neighbours)
  u64* d_dbits = nullptr;
  bool dnb_now = false;             // this round's pull reads d_dbits
  bool narrow_pr_now = false;       // W = 8 / 16 near-done pull on the per-receiver kernel (launch_expand)
  int32_t sate_since = -1;          // first round that marked sated vertices (-1: none yet this run)
  // [n_alloc] line masks (W = 64): bit l = 128-B line l of v's
  // row in this round's slot holds a nonzero word; 0 = not a sender.  Built by
  // k_mklm from the very rows the round's filtered pull reads (SCAN_LINES)
  uint8_t* d_lm = nullptr;
  bool lines_now = false;
  // [2][n_alloc / 2] the same masks written by the commits of a 64-word pull
  // for the next round's senders (nibbles, by round parity like d_fpop): a
  // line-mask round after such a round (no liveness, one context) probes them
  // without k_mklm's pass over the senders' rows
  uint8_t* d_lmw[2] = {nullptr, nullptr};
  bool lm_write_now = false, lm_written_prev = false;
  // what this round's pull actually ran (round stats' scan bits 8 / 16): the
  // line-mask variant, and with masks the previous round's commits wrote
  bool lines_ran = false, lines_from_commits = false;
  bool split_now = false;   // degree-split round: low-degree senders push, receivers probe a prefix
  // aliased Message-Lists: a receiver that completes its
  // component in a W = 64 early-exit pull writes no row; sp = SLOT_CMASK says
  // its Message-List is cmask[midx[v]].  dprobe_now: the pull probes the done
  // bitmap for every arc it scans (a receiver with any done in-neighbour takes
  // its target and gathers nothing, so an aliased row is never gathered);
  // alias_now: its complete receivers alias; alias_active: the run holds
  // aliases (readers of rows outside such pulls materialize them, k_unalias)
  bool dprobe_now = false, alias_now = false, alias_active = false;
  // receiver lists: late early-exit pulls append the
  // receivers that are still neither done nor sated to d_ulist[ul_cur ^ 1];
  // the next pull, when the list is short, launches waves for those alone
  // (SCAN_LIST) and leaves the senders' accounting to k_mkbits
  int32_t* d_ulist[2] = {nullptr, nullptr};
  int ul_cur = 0;
  bool ulist_valid = false, ulist_emit_now = false, ulist_read_now = false;
  int64_t ulist_n = 0;
  int32_t acc_row = 0;      // its accumulator rows addressed as rows of the round's slot buffer
  // [nnz/64 + 2] per-arc activity mask of filtered pull rounds (gcol order): 33.5 MB at C4
  u64* d_amask = nullptr;
  // push (sparse-round) mode
  u64* d_acc = nullptr;             // [nloc][W] OR accumulator, kept all-zero between uses (inside d_rows)
  u64* d_tbits = nullptr;           // [n_alloc/64] receivers pushed to this round
  int32_t* d_touched = nullptr;     // [n_alloc] receivers touched this round
  int32_t* d_active = nullptr;      // [n_alloc] senders (deg <= hub threshold)
  int32_t* d_big = nullptr;         // [n_alloc] senders above the hub threshold
  std::vector<int64_t> inj_arcs;    // per inject round: sum of origin out-degrees
  u64 prev_next_arcs = 0;           // out-degree sum of the last round's receivers
  bool mode_push = false;           // direction of the current round
  bool early_exit_now = false;      // coverage-checked scan this round
  u64 prev_new_bits = 0;            // new bits of the last round (global)
  u64 prev_receivers = 0;           // receivers of the last round (global)
  u64 held_bits = 0;                // messages held so far, summed over vertices (global)
  bool unfiltered_now = false;      // this round's pull skips the activity check
  bool arc_mask_now = false;        // this round's filtered pull reads the per-arc mask
  bool sum_now = false;             // this round's probes read the summary level first
  bool prefilter_now = false;       // this round's filtered pull probes low-degree in-lists lane-parallel
  // compact Message-Lists: 128-B records per vertex, per slot
  u64* d_cml[2] = {nullptr, nullptr};   // [n_alloc][16] records
  u64* d_cmk[2] = {nullptr, nullptr};   // [n_alloc / 64] dense bitmaps (bit v: no record, read the row)
  bool cml_read_now = false, cml_write_now = false, cml_written_prev = false;
  int64_t inj_groups_at(int32_t r) const {
    auto it = inject.find(r);
    return it == inject.end() ? 0 : it->second.cnt;
  }
  int32_t* d_gcol = nullptr;        // [nnz] in-CSR columns, rows sorted by neighbour degree desc
  uint32_t* d_hub_done = nullptr;   // [n_hubs] early-exit rounds: a chunk covered its hub's target (hub.hip)
  uint32_t hub_epoch = 0;           // stamp of the last pull launch (k_hub_partial's hub_done)
  int32_t* d_prehi = nullptr;       // [n] degree-split rounds: gather-order prefix of senders with
                                    //   in-degree >= prehi_deg (build_prehi, built on first use)
  int32_t prehi_deg = 0;
  int32_t* d_midx = nullptr;        // [n_alloc] component mask row of v (-1: none)
  u64* d_cmask = nullptr;           // [K][W] messages per component
  std::vector<int32_t> h_inj_origin;   // host copies of the injection groups
  std::vector<u64> h_inj_bits;
  std::vector<int32_t> h_deg_out;
  uint32_t* d_done_at = nullptr;    // [n_alloc] messages of the vertex's component (this run)
  // pristine copies of done_at / cmask: a message whose origin is down at its
  // inject round never exists, so the run drops it from its component's target
  // (k_lost_clear, k_done_fix); gp_reset restores the pristine targets
  uint32_t* d_done_at0 = nullptr;   // [n_alloc]
  u64* d_cmask0 = nullptr;          // [K][W]
  uint32_t* d_lostcnt = nullptr;    // [K] messages lost per component this round
  int32_t cmask_rows = 0;           // K
  bool done_dirty = false;          // the working targets differ from the pristine ones
  u64* d_msg_cov = nullptr;    // [W*64]
  u64* d_msg_fwd = nullptr;    // [W*64]
  u64* d_alive = nullptr;      // [2][W] alive messages per round parity
  u64* d_bc_keys = nullptr;    // [nloc] (degree << 32 | v) sorted: weighted bitcount order (bitcount.hip)
  uint32_t* d_bc_part = nullptr;   // per-block bitcount partials
  size_t bc_part_words = 0;
  int64_t bc_split = 0;        // owned vertices of degree <= the bitcount tail threshold
  u64* d_fin_comp = nullptr;   // finalize by components: [K] counts, [K] degree sums, list cursor
  u64* d_fin_list = nullptr;   // [nloc] incomplete rows (degree << 32 | v)
  int32_t fin_comp_rows = 0;
  gp_report* d_reports = nullptr;
  int64_t report_cap = 0;
  u64* d_stats = nullptr;      // [NSTAT]
  u64* h_stats = nullptr;      // pinned [NSTAT]
  int32_t round = 0;
  bool liveness_active = false;
  // first round whose alive set F_r is complete in d_alive (-1: none yet).
  // The sets are built only while liveness is active, so when an explicit
  // crash turns it on at round r, F_r was never built: r's pull must not
  // narrow its early-exit target with it (F_{r+1} is built by round r)
  int32_t alive_from = -1;
  bool pending_crash = false;
  bool msg_forwards_valid = true;
  int64_t last_reports = 0;

  // hub split
  std::vector<HubItem> h_hub_items;
  HubItem* d_hub_items = nullptr;
  int32_t* d_hubs = nullptr;          // hub vertex per hub
  int32_t* d_hub_item_ptr = nullptr;  // [n_hubs+1]
  u64* d_hub_partial = nullptr;  // [items][W]
  uint32_t* d_hub_pnz = nullptr;      // [items]
  int64_t n_hubs = 0, n_hub_items = 0;

  // rccl
  ncclComm_t comm = nullptr;

  // message-shard job (shard.hip): jnranks > 0 once a transport
  // is set; the rounds then record the receiver / sender bitmaps of the run
  ncclComm_t jcomm = nullptr;           // gp_shard_comm_init
  gp_allgather_fn jhost = nullptr;      // gp_shard_host_init
  void* jhost_user = nullptr;
  int32_t jrank = 0, jnranks = 0;
  u64* d_hist = nullptr;                // [hist_cap][2][nwords]: round r's receivers, then senders
  int32_t hist_cap = 0, hist_rounds = 0;
  std::vector<gp_round_stats> run_stats;   // this run's rounds, as gp_round returned them
  int32_t fin_round = -1;               // round count at the last gp_finalize_messages of this run
  u64* d_jscr = nullptr;                // combine scratch (send / receive chunks)
  size_t jscr_words = 0;
  u64* d_jdig = nullptr;                // [P * ceil(n / P)] the job's digest (first n valid)
  size_t jdig_words = 0;
  u64* d_jcf = nullptr;                 // [2][jm] the job's coverage, forwards
  int32_t jm = 0;                       // messages of the job
  bool j_ready = false, j_fwd_valid = false, j_dig_valid = false;

  // kernel geometry
  int cu_count = 256;

  int64_t nloc() const { return vend - vbegin; }
  // lookup of a global vertex id among the local ids (-1: not local)
  int64_t to_local(int64_t g) const;

};

// error helpers (thread-local message, negative status)
int set_error(int code, const std::string& msg);
#define GP_HIP(call)                                                              \
  do {                                                                            \
    hipError_t _e = (call);                                                       \
    if (_e != hipSuccess)                                                         \
      return ::gp::set_error(GP_EHIP, std::string(#call) + ": " + hipGetErrorString(_e)); \
  } while (0)
#define GP_RCCL(call)                                                             \
  do {                                                                            \
    ncclResult_t _r = (call);                                                     \
    if (_r != ncclSuccess)                                                        \
      return ::gp::set_error(GP_ERCCL, std::string(#call) + ": " + ncclGetErrorString(_r)); \
  } while (0)
#define GP_TRY(expr)                                                              \
  do { int _rc = (expr); if (_rc != 0) return _rc; } while (0)

template <class T>
int dalloc(T** p, size_t count) {
  if (*p) { (void)hipFree(*p); *p = nullptr; }
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void**)p, count * sizeof(T));
  if (e != hipSuccess) {
    *p = nullptr;
    return set_error(GP_ENOMEM, std::string("hipMalloc ") + std::to_string(count * sizeof(T)) +
                                    " bytes: " + hipGetErrorString(e));
  }
  return 0;
}
template <class T>
void dfree(T** p) {
  if (*p) { (void)hipFree(*p); *p = nullptr; }
}

// blocking copy ordered on the engine stream.  A plain hipMemcpy runs on the
// null stream, which a non-blocking stream does not wait for (and a pageable
// host-to-device hipMemcpy may return before its DMA lands), so kernels on
// c->stream could read stale data or race with the copy.
int copy_sync(Ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind);
// graph_build.hip
int build_chung_lu(Ctx* c, int64_t n, double dbar, double gamma, uint64_t seed);
int build_gather_order(Ctx* c);
int build_prehi(Ctx* c, int32_t T);
// setup.hip
int finish_graph(Ctx* c);
int build_hubs(Ctx* c);
// bitcount.hip
int bitcount_messages(Ctx* c, bool weighted, u64* cov, u64* fwd);   // coverage / forwards of the owned rows
int finalize_by_components(Ctx* c, bool weighted, u64* cov, u64* fwd);   // the same via cmask rows
void bitcount_free(Ctx* c);
// partition.hip
int localize(Ctx* c);                          // global overlay -> owned + ghost local CSR, boundary lists
int set_extras(Ctx* c, const std::vector<int32_t>& origins_global);   // origins neither owned nor ghosts
void free_partition(Ctx* c);
int alloc_exchange(Ctx* c);                    // exchange buffers for the current row width
int pack_boundary(Ctx* c);                     // after E_r: this round's boundary entries -> send buffers
int exchange_rccl(Ctx* c);                     // counts, rows, alive sets over RCCL, then unpack
int exchange_group(Ctx** ctxs, int32_t nctx);  // the same through device-to-device copies
// pull.hip: write the component rows of aliased vertices (all, or this
// round's senders only) into S[cur]; with all, the run holds no alias after
int unalias(Ctx* c, bool senders_only);
// shard.hip
int shard_record_round(Ctx* c);                // after E_r of a shard job: round r's bitmaps
void shard_free(Ctx* c);
void shard_reset(Ctx* c);                      // new run (gp_reset, checkpoint load)
// state bit: removed by this rank's seed step in the current round (sent to the
// ranks holding the vertex as a ghost; cleared by the next round's k_churn)
constexpr uint8_t ST_RMNEW = 8;
// sated (churn runs): no injection left and v holds every
// message of its component that anyone still forwards; the alive sets only
// shrink from round to round, so v never receives again and the pull skips it
constexpr uint8_t ST_SATED = 16;

}  // namespace gp

// the ABI handle is the context itself
struct gp_ctx : public gp::Ctx {};
