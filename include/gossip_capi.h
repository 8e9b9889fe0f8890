/*
 * gossip_capi.h -- C-ABI of the MI355X gossip-propagation engine (libgossip_hip.so).
 *
 * The reference (Sidharthshanu/Gossip-protocol-with-power-law) has no FFI: its
 * hot path is one OS thread per TCP socket.  This ABI replaces, for ALL peers at
 * once, one round of
 *   - gossip generation + fan-out         Peer.py:395-408  (gossip_sender)
 *   - receive dispatch                    Peer.py:175-216, 258-296
 *   - forward-once / Message-List dedup   (spec-level: absent from the reference,
 *                                          SURVEY.md §0 finding 1)
 *   - heartbeat liveness + dead report    Peer.py:298-393, 128-151
 *   - seed dead-node removal              Seed.py:358-406
 * over an overlay built by the seed registry (Seed.py:127-149) or by the
 * degree-weighted selector (demonstrate_powerlaw.py:7-39).
 *
 * Conventions
 *   - Every function returns 0 on success and a negative gp_status on failure;
 *     gp_last_error() gives a thread-local message.  Nothing aborts or exits.
 *   - The caller owns host arrays; they are copied in.  The context owns all
 *     device memory.  One context = one device + one HIP stream; not thread-safe.
 *   - Vertex ids are 0..n-1 int32; arc offsets int64.  Messages are 0..m-1 and
 *     are packed 64 per uint64 word, W = ceil(m/64) rounded up to a power of two
 *     (1..64 words per vertex row, i.e. m <= 4096 per context; larger message
 *     sets are run as independent batches by the host -- messages never interact).
 *   - Multi-GPU: one process per GPU.  Either message shards (each context
 *     runs the whole overlay for a word-aligned block of messages,
 *     gp_config.msg_word_base; no collective), or a vertex partition
 *     (gp_set_partition, nranks > 1, undirected overlays): each context keeps
 *     its owned slice [vbegin, vend) plus ghost rows for the non-owned
 *     in-neighbours of owned vertices, and after every round sends each peer
 *     only the new bits of the boundary vertices that received something
 *     (ncclSend / ncclRecv over xGMI, gp_comm_init; or device-to-device copies
 *     in gp_round_group).  Per-vertex reads of a partitioned context return its
 *     owned slice; its CSR reads return the local CSR (GP_L2G maps local ids).
 */
#ifndef GOSSIP_CAPI_H
#define GOSSIP_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GP_ABI_VERSION 18

typedef struct gp_ctx gp_ctx;

typedef enum gp_status {
  GP_OK = 0,
  GP_EINVAL = -1,     /* bad argument / shape                              */
  GP_EHIP = -2,       /* HIP runtime error                                 */
  GP_ENOMEM = -3,     /* device allocation failed                          */
  GP_ESTATE = -4,     /* call out of order (e.g. round before load_graph)  */
  GP_ERCCL = -5,      /* RCCL error                                        */
  GP_ENOTRACK = -6    /* requested output was not tracked (see gp_config)  */
} gp_status;

/* Per-round counters (all exact integers, summed over ranks). */
typedef struct gp_round_stats {
  int32_t round;            /* r                                                      */
  int32_t overflow;         /* 1 if the report buffer overflowed this round          */
  uint64_t injected;        /* messages injected at live origins in round r          */
  uint64_t lost;            /* messages whose origin was down at their inject round  */
  uint64_t new_bits;        /* first receipts produced by round r (receipt round r+1)*/
  uint64_t receivers;       /* vertices with >= 1 first receipt in round r           */
  uint64_t sends;           /* edge-deliveries attempted in round r:
                               sum_u deg_live(u) * |frontier_r(u)|                   */
  uint64_t active;          /* senders with a non-empty frontier in round r          */
  uint64_t crashed;         /* vertices that crashed in round r                      */
  uint64_t reports;         /* "Dead Node" reports emitted in round r (Peer.py:311)  */
  uint64_t removals;        /* vertices removed by the seed (Seed.py:387-391)        */
  uint64_t dup_reports;     /* reports hitting "not found" (Seed.py:373-375)         */
  uint64_t arcs_scanned;    /* in-arcs visited by the pull (byte accounting)         */
  uint64_t rows_gathered;   /* neighbour Message-List rows loaded (8*W bytes each)   */
  uint64_t seen_rows_read;  /* receiver seen rows read (8*W bytes each)              */
  uint64_t rows_written;    /* receiver seen rows written to the next slot (8*W B)   */
  uint64_t vertices_visited;/* receivers whose in-list was scanned                   */
  uint64_t atomics;         /* push mode: 64-bit atomicOr issued                      */
  uint64_t next_arcs;       /* out-degree sum of this round's receivers (direction)   */
  uint64_t row_bytes;       /* bytes of neighbour rows actually loaded (the pull skips
                               the words a receiver already completed, §3.4)         */
  int32_t mode;             /* 0 = pull expansion, 1 = push expansion                 */
  int32_t scan;             /* pull arc check (bits 0-1 as a number): 0 = activity-
                               bitmap probe per arc, 1 = per-arc activity mask built
                               first, 2 = none, every in-neighbour row read (§3.4),
                               3 = probe, low-degree in-lists prefiltered (§3.2);
                               + 4: senders gathered from compact Message-Lists;
                               + 8: 64-word line masks read (only named 128-B lines
                               gathered, §3.2); + 16: those masks were written by
                               the previous round's commits (no k_mklm pass);
                               + 32: degree-split round (senders of in-degree <
                               split_deg pushed, receivers probe the gather-order
                               prefix of the others, §3.2); + 64: every scanned
                               arc probed the done bitmap (complete receivers
                               alias their component row, `aliased`, §3.2);
                               + 128: the waves took their receivers from the
                               list the previous round left (§3.5)                */
  double expand_ms;         /* device time of the expansion kernels (HIP events)     */
  double exchange_ms;       /* device time of the RCCL exchange (0 on 1 GPU)         */
  double round_ms;          /* device time of the whole round                        */
  double kernel_ms;         /* device time of the pull kernel + its hub passes (and
                               of a degree-split round's push half and clear)    */
  uint64_t xchg_rows;       /* vertex partition: boundary entries sent (all peers)   */
  uint64_t xchg_bytes;      /* vertex partition: bytes sent (entry heads + words)    */
  uint64_t done_nb;         /* receivers that took every message of their component
                               from an in-neighbour holding all of them (§3.4)      */
  uint64_t lm_rows;         /* senders' rows read to build line masks before a
                               filtered 64-word pull (8*W bytes each, §3.2)         */
  uint64_t aliased;         /* receivers that completed their component and took it
                               as their Message-List without writing a row (their
                               slot byte names the component row, §3.2; ABI 18)    */
} gp_round_stats;

/* One dead-node report: reporter saw `dead` miss 3 heartbeats in `round`. */
typedef struct gp_report {
  int32_t dead;
  int32_t reporter;
  int32_t round;
} gp_report;

typedef struct gp_config {
  int32_t track_first;         /* keep the u8 first-receipt matrix [n][m] (255 = never) */
  int32_t track_digest;        /* keep per-vertex first-receipt digest u64[n]          */
  int32_t track_msg_forwards;  /* accumulate per-message forwards every round          */
  int32_t churn;               /* run the liveness phase every round                   */
  double p_fail;               /* per-round crash probability of a live vertex         */
  uint64_t churn_seed;         /* crash draws: splitmix stream        */
  int32_t miss_threshold;      /* heartbeat misses before report (reference: 3)        */
  int32_t hub_threshold;       /* in-degree above which a vertex is split over waves   */
  int64_t report_capacity;     /* reports kept per round (counts stay exact)           */
  double push_ratio;           /* push a round when its sender arcs * push_ratio <= nnz;
                                  0 = always pull                      */
  int32_t early_exit;          /* coverage-checked pull scans in dense rounds (§3.4)   */
  int32_t arc_mask_permille;   /* filtered pull rounds with >= this many senders per 1000
                                  vertices build the per-arc activity mask first
                                  (0 = always probe per arc)           */
  int32_t prefilter_pct;       /* filtered pull rounds with < this % of vertices sending
                                  probe the in-lists of receivers of in-degree <= 16
                                  lane-parallel first (0 = never)       */
  int32_t compact_rows;        /* 1: 64-word runs keep 128-B compact Message-Lists while
                                  rows are sparse and gather them instead of full rows
                                  (single-rank contexts only)           */
  int32_t unfiltered_pct;      /* pull without the per-arc activity check when >= this %
                                  of vertices are senders (0 = never)   */
  int32_t msg_word_base;       /* message shards: this context's message k
                                  is global message 64*msg_word_base + k; the digest uses
                                  global word indices, so shard digests XOR together     */
  int32_t flat_max_words;      /* rows of at most this many words (<= 32) take the
                                  edge-parallel pull kernel (0 = never)  */
  int64_t summary_min_n;       /* filtered probe rounds of overlays with >= this many
                                  vertices, with at most n/256 senders, probe a summary
                                  level (1 bit per 64 vertices) before the activity
                                  bitmap (0 = never)                    */
  int32_t partition_by_arcs;   /* vertex partitions (gp_set_partition): 0 = slices of equal
                                  vertex count, 1 = slices of equal in-arc count
                                  (set before the partition is made)     */
  int32_t split_deg;           /* degree-split sparse rounds: in a
                                  prefiltered pull without early exit, senders of
                                  in-degree < split_deg push their rows (atomicOr into
                                  the accumulator) and receivers probe only the prefix of
                                  their gather-ordered in-list whose senders have
                                  in-degree >= split_deg (0 = off; single-rank contexts) */
  int32_t split_max_permille;  /* ... only while fewer than this many vertices per 1000
                                  send (default 10: the push half grows with the low-
                                  degree senders; 1000 = whenever prefiltered; ABI 17)   */
} gp_config;

/* what for gp_read */
typedef enum gp_what {
  GP_SEEN = 0,        /* u64 [vend-vbegin][W]  owned rows of the Message-List bitmap */
  GP_FIRST = 1,       /* u8  [vend-vbegin][m]  first-receipt round, 255 = never      */
  GP_DIGEST = 2,      /* u64 [vend-vbegin]                                           */
  GP_COVERAGE = 3,    /* u64 [m]  vertices holding message m (this rank's slice)     */
  GP_FORWARDS = 4,    /* u64 [m]  sends of message m (this rank's senders)           */
  GP_STATE = 5,       /* u8  [n]  bit0 crashed, bit1 removed                         */
  GP_MISS = 6,        /* u8  [n]  heartbeat miss counter                             */
  GP_DEG_LIVE = 7,    /* i32 [n]  neighbours not removed                             */
  GP_ROW_PTR = 8,     /* i64 [n+1] in-CSR offsets (as loaded / built)                */
  GP_COL = 9,         /* i32 [nnz] in-CSR columns                                    */
  GP_FRONTIER = 10,   /* u64 [n][W] current frontier (rows with FPOP==0 read as 0);
                         kept only with track_msg_forwards (else GP_ENOTRACK)      */
  GP_FPOP = 11,       /* u32 [n] |frontier(v)|                                       */
  GP_L2G = 12,        /* i32 [local slots] global id of each local vertex (identity
                         unless partitioned: owned, then ghosts, then origin extras) */
  /* the whole job of a message-shard run, after gp_shard_combine (else GP_ESTATE) */
  GP_JOB_DIGEST = 13,   /* u64 [n]        per-vertex digest of every shard's messages    */
  GP_JOB_COVERAGE = 14, /* u64 [m_total]  vertices holding message k of the job table    */
  GP_JOB_FORWARDS = 15  /* u64 [m_total]  sends of message k (GP_ENOTRACK as GP_FORWARDS) */
} gp_what;

int gp_abi_version(void);
const char* gp_last_error(void);
int gp_device_count(int* n_out);

int gp_create(int device, gp_ctx** out);
void gp_destroy(gp_ctx* ctx);
void gp_default_config(gp_config* cfg);
int gp_configure(gp_ctx* ctx, const gp_config* cfg);

/* Overlay.  In-CSR: row_ptr[v]..row_ptr[v+1] lists u with an arc u->v (the peers
 * whose gossip v receives; Peer.py:402 sends on outgoing links).  out_degree may
 * be NULL for undirected graphs (= in-degree).  For directed graphs the out-CSR
 * (out_row_ptr/out_col, may be NULL when directed == 0) gives the other side of
 * every heartbeat link for liveness reports (Peer.py:369-392 covers outgoing and
 * incoming connections). */
int gp_load_graph(gp_ctx* ctx, int64_t n, int64_t nnz, const int64_t* row_ptr,
                  const int32_t* col, int32_t directed, const int64_t* out_row_ptr,
                  const int32_t* out_col);

/* Build an undirected Chung-Lu power-law overlay on the device:
 * ~dbar*n/2 candidate edges, endpoints drawn ∝ (i+1)^(-1/(gamma-1)) with an
 * integer alias table, self-loops dropped, de-duplicated, ids randomly relabelled. */
int gp_build_chung_lu(gp_ctx* ctx, int64_t n, double dbar, double gamma, uint64_t seed);

/* Vertex slice owned by this context (default: all). */
int gp_set_partition(gp_ctx* ctx, int32_t rank, int32_t nranks);
int gp_get_partition(gp_ctx* ctx, int64_t* vbegin, int64_t* vend);

/* RCCL: rank 0 calls gp_comm_unique_id, the host distributes the 128 bytes. */
int gp_comm_unique_id(void* out128);
int gp_comm_init(gp_ctx* ctx, const void* unique_id128, int32_t nranks, int32_t rank);

/* Messages: origin vertex and inject round of each message (Peer.py:397-399:
 * message #n of a peer is its n-th generated gossip). */
int gp_set_messages(gp_ctx* ctx, int32_t m, const int32_t* origin, const int32_t* inject_round);

/* Spread keys of candidate origins, for ordering a message table before
 * gp_set_messages (DESIGN.md §3.4 "message order"; no reference counterpart:
 * the reference's Message-List is an unordered set of strings, Peer.py:175-216,
 * so the bit position of a message is the engine's choice).  keys_out[k] is the
 * number of arc endpoints within `hops` (1..3) of origin[k]: hops 1 = degree,
 * 2 = the sum of its neighbours' degrees, 3 = the sum over its neighbours of
 * their hops-2 key.  Messages whose keys are close spread at similar speed, so
 * placing them in adjacent bits lets the late early-exit rounds skip whole
 * 128-B lines of Message-List rows.  Needs the global overlay (before
 * gp_set_partition with nranks > 1). */
int gp_spread_keys(gp_ctx* ctx, int32_t hops, int32_t m, const int32_t* origin, uint64_t* keys_out);

/* Explicit crash injection (the reference's silent mode, Peer.py:437-439),
 * applied at the start of the next round in addition to random churn. */
int gp_crash(gp_ctx* ctx, int32_t nverts, const int32_t* verts);

int gp_reset(gp_ctx* ctx);                       /* new run: clear all per-run state */
int gp_round(gp_ctx* ctx, gp_round_stats* out);  /* liveness + injection + expansion */
int gp_run(gp_ctx* ctx, int32_t max_rounds, gp_round_stats* per_round, int32_t* rounds_out);
/* Single-process multi-context round: ctxs[k] owns partition k of nctx (same or
 * different devices, no RCCL); the exchange is device-to-device copies and the
 * counters are summed into *out.  Used for partition-invariance checks on one GPU. */
int gp_round_group(gp_ctx** ctxs, int32_t nctx, gp_round_stats* out);
int gp_finalize_messages(gp_ctx* ctx);           /* per-message coverage/forwards    */
int gp_read(gp_ctx* ctx, int32_t what, void* host, int64_t bytes);
int gp_reports(gp_ctx* ctx, gp_report* buf, int64_t cap, int64_t* n_out);
int gp_synchronize(gp_ctx* ctx);
int gp_info(gp_ctx* ctx, int64_t* n, int64_t* nnz, int32_t* m, int32_t* words);
/* Local shape of a (partitioned) context: owned vertices, ghosts, origin
 * extras, arcs of the local CSR, boundary entries it sends to (all peers). */
int gp_local_info(gp_ctx* ctx, int64_t* nloc, int64_t* nghost, int64_t* nextra, int64_t* nnz_local,
                  int64_t* n_boundary);

/* Message-shard jobs.  Messages never interact, so an N-GPU
 * job runs one context per GPU on the whole overlay, rank p holding the
 * word-aligned block of the message table that starts at global word
 * gp_config.msg_word_base.  The reference keeps each peer's whole receive
 * record (Peer.py:175-216); gp_shard_combine makes the job's record out of the
 * ranks' after gp_run: the per-vertex digests XOR-reduced (reduce-scatter by
 * ncclSend/ncclRecv of 1/N vertex slices + an XOR kernel, then ncclAllGather),
 * the per-message coverage / forwards all-gathered into the job's message
 * order, and the per-round counters: additive ones summed, `receivers` and
 * `active` as the popcount of the OR of the ranks' per-round vertex bitmaps
 * (reduce-scattered like the digests: a vertex receiving in two shards counts
 * once), liveness counters checked equal across ranks.  Every rank gets the
 * same job record.
 *
 * The transport is a communicator of the shard ranks (gp_shard_comm_init: one
 * GPU per rank), or the host's own all-gather (gp_shard_host_init: ranks
 * sharing a GPU, which RCCL refuses -- the rehearsal of a one-GPU box; the
 * reductions still run on the device).  Rounds of a shard job take no
 * collective: each rank decides its own direction / scan modes.  A shard job
 * records two n-bit bitmaps per round (exchange_ms of gp_round_stats). */
typedef int (*gp_allgather_fn)(void* user, const void* send, int64_t bytes, void* recv);   /* recv: [nranks][bytes] */
int gp_shard_comm_init(gp_ctx* ctx, const void* unique_id128, int32_t nranks, int32_t rank);
int gp_shard_host_init(gp_ctx* ctx, gp_allgather_fn fn, void* user, int32_t nranks, int32_t rank);
/* the communicator's own count and rank (ncclCommCount / ncclCommUserRank), or
 * those given to gp_shard_host_init; transport_out: 1 = RCCL, 2 = host */
int gp_shard_info(gp_ctx* ctx, int32_t* nranks_out, int32_t* rank_out, int32_t* transport_out);
/* after gp_run (uninterrupted since gp_reset) on every rank; finalizes first if
 * needed.  job[0..*rounds_out) = the job's per-round counters (cap >= rounds);
 * *ms_out (may be NULL) = device time of the combine on the engine stream. */
int gp_shard_combine(gp_ctx* ctx, gp_round_stats* job, int32_t cap, int32_t* rounds_out, double* ms_out);

/* Checkpoints (no reference counterpart -- the
 * reference's peers keep no state across restarts).  Taken between rounds:
 * the blob holds the whole per-run state of this context (Message-List rows in
 * canonical form, popcounts, liveness state, counters, tracked outputs, round
 * number and direction history).  Loading it into a context with the same
 * overlay, messages, partition and tracked outputs continues the run exactly
 * as if it had never stopped.  The blob is opaque; gp_checkpoint_size gives
 * its length (8*W bytes per vertex plus ~30 B of vertex state). */
int gp_checkpoint_size(gp_ctx* ctx, int64_t* bytes);
int gp_checkpoint_save(gp_ctx* ctx, void* host, int64_t bytes);
int gp_checkpoint_load(gp_ctx* ctx, const void* host, int64_t bytes);

#ifdef __cplusplus
}
#endif

#endif /* GOSSIP_CAPI_H */
