// shard.hip -- the whole-job record of a message-shard run.
//
// Messages never interact: the run of a message table A u B is the run of A
// beside the run of B.  An N-GPU job therefore runs one context per GPU on the
// whole overlay, rank p holding a word-aligned block of the table
// (gp_config.msg_word_base), with no collective inside the rounds.  What the
// reference keeps per peer -- its whole receive record (Peer.py:175-216, the
// log at :206, the forward loop at :402-404) -- is then spread over the ranks,
// and gp_shard_combine assembles the job's:
//   - per-vertex digest D[v] = XOR over ranks (the digest uses global word
//     indices, so shard digests XOR into the whole run's): a reduce-scatter
//     (grouped ncclSend / ncclRecv of 1/N vertex slices, k_shard_xor) and an
//     ncclAllGather of the reduced slices;
//   - per-message coverage / forwards: an all-gather of each rank's columns,
//     placed at the rank's block of the job table;
//   - per-round counters: additive ones summed; `receivers` (vertices with a
//     first receipt in round r) and `active` (vertices sending in round r) are
//     not additive -- a vertex receiving in two shards is one receiver -- so
//     every round of a shard job records two n-bit bitmaps (k_shard_hist), and
//     the combine ORs them across ranks (reduce-scatter again) and counts the
//     bits (k_shard_union); liveness counters (crashes, reports, removals) do
//     not depend on the messages and are checked equal on every rank.
// Every rank ends with the same job record.
//
// Transports: a communicator of the shard ranks (one GPU per rank), or the
// host's own all-gather of byte strings (ranks sharing a GPU, which RCCL
// refuses: the rehearsal on a one-GPU box).  Both move the same chunks; the
// reductions run on the device either way.
#include <hip/hip_runtime.h>

#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "gp_device.h"

namespace gp {

// ---------------------------------------------------------------------------
// kernels

// round r of a shard job: rx word k = receivers of the round (fpop_next != 0:
// the vertices with first receipts, which send next round), act word k = the
// round's senders (the activity bitmap k_mkbits built from fpop)
__global__ __launch_bounds__(BLOCK) void k_shard_hist(const uint32_t* __restrict__ fpop_next,
                                                      const u64* __restrict__ abits, u64* __restrict__ rx,
                                                      u64* __restrict__ act, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (n + 63) >> 6;
  const int64_t stride = (int64_t)gridDim.x * WAVES;
  for (int64_t k = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6); k < nw; k += stride) {
    const int64_t v = k * 64 + lane;
    const u64 m = __ballot(v < n && fpop_next[v] != 0u);
    if (lane == 0) {
      rx[k] = m;
      act[k] = abits[k];
    }
  }
}

// send chunk q = words [q*L, q*L + L) of each of the 2R bitmaps (zero past the
// rank's own rounds and past nw): out[q][b][j]
__global__ void k_shard_pack(const u64* __restrict__ hist, int32_t own_bitmaps, int64_t nw, int32_t P,
                             int32_t nbitmaps, int64_t L, u64* __restrict__ out) {
  const int64_t total = (int64_t)P * nbitmaps * L;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = t % L;
    const int64_t b = (t / L) % nbitmaps;
    const int64_t q = t / (L * nbitmaps);
    const int64_t w = q * L + j;
    out[t] = (b < own_bitmaps && w < nw) ? hist[b * nw + w] : 0ull;
  }
}

// cnt[b] = popcount of the OR over ranks of bitmap b's words in this rank's
// slice; in[q][b][j], j < len
__global__ __launch_bounds__(BLOCK) void k_shard_union(const u64* __restrict__ in, int32_t P, int32_t nbitmaps,
                                                       int64_t L, int64_t len, u64* __restrict__ cnt) {
  const int b = blockIdx.y;
  u64 s = 0;
  for (int64_t j = (int64_t)blockIdx.x * BLOCK + threadIdx.x; j < len; j += (int64_t)gridDim.x * BLOCK) {
    u64 x = 0;
    for (int q = 0; q < P; ++q) x |= in[((int64_t)q * nbitmaps + b) * L + j];
    s += (u64)__popcll(x);
  }
  s = wave_sum_u64(s);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd(cnt + b, s);
}

// out[j] = XOR over ranks of in[q][j] (this rank's vertex slice), 0 past len
__global__ void k_shard_xor(const u64* __restrict__ in, int32_t P, int64_t L, int64_t len, u64* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < L; j += (int64_t)gridDim.x * blockDim.x) {
    u64 x = 0;
    if (j < len)
      for (int q = 0; q < P; ++q) x ^= in[(int64_t)q * L + j];
    out[j] = x;
  }
}

// ---------------------------------------------------------------------------
// history

static int64_t hist_words(const Ctx* c) { return (c->n_alloc + 63) / 64; }

int shard_record_round(Ctx* c) {
  const int r = c->round;
  const int64_t nw = hist_words(c);
  if (r >= c->hist_cap) {   // grow (doubling): the rounds of a run are not known in advance
    const int32_t cap = std::max(16, 2 * c->hist_cap);
    u64* d = nullptr;
    GP_TRY(dalloc(&d, (size_t)cap * 2 * nw));
    if (c->d_hist && c->hist_rounds > 0)
      GP_HIP(hipMemcpyAsync(d, c->d_hist, (size_t)c->hist_rounds * 2 * nw * 8, hipMemcpyDeviceToDevice, c->stream));
    GP_HIP(hipStreamSynchronize(c->stream));
    dfree(&c->d_hist);
    c->d_hist = d;
    c->hist_cap = cap;
  }
  if (r != c->hist_rounds) return set_error(GP_ESTATE, "shard history out of step with the rounds");
  u64* rx = c->d_hist + (size_t)r * 2 * nw;
  hipLaunchKernelGGL(k_shard_hist, dim3(std::max(1, std::min(grid_for(nw, WAVES), c->cu_count * 8))), dim3(BLOCK),
                     0, c->stream, c->d_fpop[c->cur ^ 1], c->d_abits, rx, rx + nw, c->n_alloc);
  GP_HIP(hipGetLastError());
  c->hist_rounds = r + 1;
  return 0;
}

void shard_reset(Ctx* c) {
  c->hist_rounds = 0;
  c->run_stats.clear();
  c->fin_round = -1;
  c->j_ready = false;
}

void shard_free(Ctx* c) {
  if (c->jcomm) (void)ncclCommDestroy(c->jcomm);
  c->jcomm = nullptr;
  c->jhost = nullptr;
  c->jnranks = 0;
  dfree(&c->d_hist);
  c->hist_cap = 0;
  dfree(&c->d_jscr);
  c->jscr_words = 0;
  dfree(&c->d_jdig);
  c->jdig_words = 0;
  dfree(&c->d_jcf);
  shard_reset(c);
}

// ---------------------------------------------------------------------------
// transport: all-gather of equal chunks, and all-to-all of chunks (chunk q of
// the send region to rank q, chunk q of the receive region from rank q)

namespace {

struct Xport {
  Ctx* c;
  int P, me;

  int allgather(const u64* send, u64* recv, size_t words) {
    hipStream_t s = c->stream;
    if (c->jcomm) {
      GP_RCCL(ncclAllGather(send, recv, words, ncclUint64, c->jcomm, s));
      return 0;
    }
    std::vector<u64> hs(words), hr((size_t)P * words);
    GP_TRY(copy_sync(c, hs.data(), send, words * 8, hipMemcpyDeviceToHost));
    if (c->jhost(c->jhost_user, hs.data(), (int64_t)(words * 8), hr.data()) != 0)
      return set_error(GP_ERCCL, "shard combine: the host all-gather failed");
    GP_TRY(copy_sync(c, recv, hr.data(), hr.size() * 8, hipMemcpyHostToDevice));
    return 0;
  }

  // send chunk q: sbase + soff[q], sw[q] words; receive chunk q: rbase +
  // roff[q], rw[q] words (rw[q] on this rank == sw[me] on rank q); cap >= every
  // chunk on every rank (the host path pads to it)
  int alltoall(const u64* sbase, const std::vector<size_t>& soff, const std::vector<size_t>& sw, u64* rbase,
               const std::vector<size_t>& roff, const std::vector<size_t>& rw, size_t cap) {
    hipStream_t s = c->stream;
    if (rw[(size_t)me] != sw[(size_t)me]) return set_error(GP_ESTATE, "shard combine: self chunk sizes differ");
    if (sw[(size_t)me])
      GP_HIP(hipMemcpyAsync(rbase + roff[(size_t)me], sbase + soff[(size_t)me], sw[(size_t)me] * 8,
                            hipMemcpyDeviceToDevice, s));
    if (c->jcomm) {
      // xGMI is point to point: one send and one receive per peer, all in one group
      GP_RCCL(ncclGroupStart());
      for (int q = 0; q < P; ++q) {
        if (q == me) continue;
        if (sw[(size_t)q]) GP_RCCL(ncclSend(sbase + soff[(size_t)q], sw[(size_t)q], ncclUint64, q, c->jcomm, s));
        if (rw[(size_t)q]) GP_RCCL(ncclRecv(rbase + roff[(size_t)q], rw[(size_t)q], ncclUint64, q, c->jcomm, s));
      }
      GP_RCCL(ncclGroupEnd());
      return 0;
    }
    std::vector<u64> hs((size_t)P * cap, 0ull), hr((size_t)P * P * cap);
    for (int q = 0; q < P; ++q) {
      if (sw[(size_t)q] > cap) return set_error(GP_ESTATE, "shard combine: chunk over its cap");
      if (q != me && sw[(size_t)q])
        GP_TRY(copy_sync(c, hs.data() + (size_t)q * cap, sbase + soff[(size_t)q], sw[(size_t)q] * 8,
                         hipMemcpyDeviceToHost));
    }
    if (c->jhost(c->jhost_user, hs.data(), (int64_t)(hs.size() * 8), hr.data()) != 0)
      return set_error(GP_ERCCL, "shard combine: the host all-gather failed");
    for (int q = 0; q < P; ++q)   // rank q's chunk for this rank
      if (q != me && rw[(size_t)q])
        GP_TRY(copy_sync(c, rbase + roff[(size_t)q], hr.data() + ((size_t)q * P + me) * cap, rw[(size_t)q] * 8,
                         hipMemcpyHostToDevice));
    return 0;
  }
};

// the per-round counters of a rank as u64 words (doubles by bit pattern)
constexpr int NF = 32;
enum {
  F_INJECTED, F_LOST, F_NEW_BITS, F_RECEIVERS, F_SENDS, F_ACTIVE, F_CRASHED, F_REPORTS, F_REMOVALS, F_DUP,
  F_ARCS, F_GATHERED, F_SEEN_READ, F_WRITTEN, F_VISITED, F_ATOMICS, F_NEXT_ARCS, F_ROW_BYTES, F_XROWS, F_XBYTES,
  F_DNB, F_LM_ROWS, F_OVERFLOW, F_MODE, F_SCAN, F_EXPAND_MS, F_EXCHANGE_MS, F_ROUND_MS, F_KERNEL_MS, F_RAN
};
static_assert(F_RAN < NF, "counter words");

u64 dbits(double x) {
  u64 b;
  std::memcpy(&b, &x, 8);
  return b;
}
double dval(u64 b) {
  double x;
  std::memcpy(&x, &b, 8);
  return x;
}

void pack_stats(const gp_round_stats& s, u64* f) {
  std::memset(f, 0, NF * 8);
  f[F_INJECTED] = s.injected; f[F_LOST] = s.lost; f[F_NEW_BITS] = s.new_bits; f[F_RECEIVERS] = s.receivers;
  f[F_SENDS] = s.sends; f[F_ACTIVE] = s.active; f[F_CRASHED] = s.crashed; f[F_REPORTS] = s.reports;
  f[F_REMOVALS] = s.removals; f[F_DUP] = s.dup_reports; f[F_ARCS] = s.arcs_scanned;
  f[F_GATHERED] = s.rows_gathered; f[F_SEEN_READ] = s.seen_rows_read; f[F_WRITTEN] = s.rows_written;
  f[F_VISITED] = s.vertices_visited; f[F_ATOMICS] = s.atomics; f[F_NEXT_ARCS] = s.next_arcs;
  f[F_ROW_BYTES] = s.row_bytes; f[F_XROWS] = s.xchg_rows; f[F_XBYTES] = s.xchg_bytes; f[F_DNB] = s.done_nb;
  f[F_LM_ROWS] = s.lm_rows; f[F_OVERFLOW] = (u64)s.overflow; f[F_MODE] = (u64)s.mode; f[F_SCAN] = (u64)s.scan;
  f[F_EXPAND_MS] = dbits(s.expand_ms); f[F_EXCHANGE_MS] = dbits(s.exchange_ms); f[F_ROUND_MS] = dbits(s.round_ms);
  f[F_KERNEL_MS] = dbits(s.kernel_ms); f[F_RAN] = 1;
}

// header words all-gathered first: every rank validates every rank's shape
enum { H_N, H_NNZ, H_M, H_WORDS, H_WBASE, H_ROUNDS, H_DIGEST, H_FWD, H_CHURN, H_SEED, H_PFAIL, H_DIRECTED, H_OK,
       NH = 16 };

int ensure_scratch(Ctx* c, size_t words) {
  if (c->jscr_words >= words) return 0;
  dfree(&c->d_jscr);
  c->jscr_words = 0;
  GP_TRY(dalloc(&c->d_jscr, words));
  c->jscr_words = words;
  return 0;
}

int combine(Ctx* c, gp_round_stats* job, int32_t cap, int32_t* rounds_out, double* ms_out) {
  const int P = c->jnranks, me = c->jrank;
  hipStream_t s = c->stream;
  Xport x{c, P, me};
  const int32_t own = c->round;
  // a rank that cannot take part still joins the header all-gather, so that
  // every rank returns the same status instead of its peers waiting in a
  // collective it never enters
  std::string why;
  if (own < 1 || (int32_t)c->run_stats.size() != own || c->hist_rounds != own)
    why = "gp_shard_combine needs a run of gp_round / gp_run since gp_reset on this context (a run restored "
          "from a checkpoint has no per-round history)";
  else if (c->fin_round != c->round && gp_finalize_messages(static_cast<gp_ctx*>(c)) != 0)
    why = std::string("finalize: ") + gp_last_error();
  GP_HIP(hipEventRecord(c->ev[0], s));

  // 1. headers: shapes, the shards' message blocks, the rounds each ran
  GP_TRY(ensure_scratch(c, (size_t)NH * (P + 1)));
  std::vector<u64> hdr(NH, 0ull), all((size_t)NH * P);
  hdr[H_N] = (u64)c->n; hdr[H_NNZ] = (u64)c->nnz; hdr[H_M] = (u64)c->m; hdr[H_WORDS] = (u64)c->words;
  hdr[H_WBASE] = (u64)c->cfg.msg_word_base; hdr[H_ROUNDS] = (u64)own;
  hdr[H_DIGEST] = c->cfg.track_digest ? 1 : 0;
  hdr[H_FWD] = (!c->msg_forwards_valid && c->liveness_active) ? 0 : 1;
  hdr[H_CHURN] = (u64)c->cfg.churn; hdr[H_SEED] = c->cfg.churn_seed; hdr[H_PFAIL] = dbits(c->cfg.p_fail);
  hdr[H_DIRECTED] = (u64)c->directed;
  hdr[H_OK] = why.empty() ? 1 : 0;
  GP_TRY(copy_sync(c, c->d_jscr, hdr.data(), NH * 8, hipMemcpyHostToDevice));
  GP_TRY(x.allgather(c->d_jscr, c->d_jscr + NH, NH));
  GP_TRY(copy_sync(c, all.data(), c->d_jscr + NH, all.size() * 8, hipMemcpyDeviceToHost));
  auto H = [&](int q, int k) { return all[(size_t)q * NH + k]; };
  // every rank checks the same words, so every rank returns the same status
  std::vector<int> order((size_t)P);
  int32_t R = 0, wmax = 0;
  int64_t mt = 0;
  if (!why.empty()) return set_error(GP_ESTATE, why);
  for (int q = 0; q < P; ++q)
    if (!H(q, H_OK)) return set_error(GP_ESTATE, "gp_shard_combine: rank " + std::to_string(q) + " has no run to combine");
  for (int q = 0; q < P; ++q) {
    for (int k : {H_N, H_NNZ, H_DIGEST, H_CHURN, H_SEED, H_PFAIL, H_DIRECTED})
      if (H(q, k) != H(0, k))
        return set_error(GP_EINVAL, "gp_shard_combine: rank " + std::to_string(q) +
                                        " ran another overlay or configuration (header word " + std::to_string(k) + ")");
    order[(size_t)q] = q;
    R = std::max(R, (int32_t)H(q, H_ROUNDS));
    wmax = std::max(wmax, (int32_t)H(q, H_WORDS));
    mt += (int64_t)H(q, H_M);
  }
  std::sort(order.begin(), order.end(), [&](int a, int b) { return H(a, H_WBASE) < H(b, H_WBASE); });
  {   // the blocks tile the job table: word-aligned, in word order, no gaps
    int64_t next = 0;
    for (int i = 0; i < P; ++i) {
      const int q = order[(size_t)i];
      if ((int64_t)H(q, H_WBASE) * 64 != next || (i + 1 < P && H(q, H_M) % 64 != 0))
        return set_error(GP_EINVAL, "gp_shard_combine: the ranks' message blocks do not tile one table "
                                    "(msg_word_base / message counts)");
      next += (int64_t)H(q, H_M);
    }
  }
  if (cap < R) return set_error(GP_EINVAL, "gp_shard_combine: cap < the job's rounds (" + std::to_string(R) + ")");
  const int64_t n = c->n, nw = hist_words(c);
  const int32_t NB = 2 * R;   // bitmaps: per round receivers, senders
  const int64_t L = (nw + P - 1) / P;
  const int64_t len = std::max<int64_t>(0, std::min<int64_t>(L, nw - (int64_t)me * L));
  const int64_t Ld = (n + P - 1) / P;
  const int64_t lend = std::max<int64_t>(0, std::min<int64_t>(Ld, n - (int64_t)me * Ld));
  const size_t MS = (size_t)wmax * 64;   // per-rank message columns, padded
  // scratch: [stats: R*NF + P*R*NF][counts: NB + P*NB][bitmaps: 2*P*NB*L][digest: P*Ld + Ld][cov/fwd: 2*MS + P*2*MS]
  const size_t o_st = 0, o_sta = o_st + (size_t)R * NF, o_cnt = o_sta + (size_t)P * R * NF,
               o_cnta = o_cnt + NB, o_bs = o_cnta + (size_t)P * NB, o_br = o_bs + (size_t)P * NB * L,
               o_dr = o_br + (size_t)P * NB * L, o_ds = o_dr + (size_t)P * Ld, o_cf = o_ds + Ld,
               o_cfa = o_cf + 2 * MS, total = o_cfa + (size_t)P * 2 * MS;
  GP_TRY(ensure_scratch(c, total));
  u64* S = c->d_jscr;

  // 2. per-round counters of every rank
  std::vector<u64> st((size_t)R * NF, 0ull), sta((size_t)P * R * NF);
  for (int32_t r = 0; r < own; ++r) pack_stats(c->run_stats[(size_t)r], &st[(size_t)r * NF]);
  GP_HIP(hipMemcpyAsync(S + o_st, st.data(), st.size() * 8, hipMemcpyHostToDevice, s));
  GP_TRY(x.allgather(S + o_st, S + o_sta, (size_t)R * NF));

  // 3. receiver / sender bitmaps: OR reduce-scatter over vertex-word slices, popcount
  hipLaunchKernelGGL(k_shard_pack, dim3(std::max(1, std::min(grid_for((int64_t)P * NB * L, 256), c->cu_count * 8))),
                     dim3(256), 0, s, c->d_hist, 2 * own, nw, P, NB, L, S + o_bs);
  GP_HIP(hipGetLastError());
  {
    const size_t ch = (size_t)NB * L;
    std::vector<size_t> off((size_t)P), w((size_t)P, ch);
    for (int q = 0; q < P; ++q) off[(size_t)q] = (size_t)q * ch;
    GP_TRY(x.alltoall(S + o_bs, off, w, S + o_br, off, w, ch));
  }
  GP_HIP(hipMemsetAsync(S + o_cnt, 0, (size_t)NB * 8, s));
  if (len > 0)
    hipLaunchKernelGGL(k_shard_union, dim3(std::max(1, std::min(grid_for(len, BLOCK), 64)), NB), dim3(BLOCK), 0, s,
                       S + o_br, P, NB, L, len, S + o_cnt);
  GP_HIP(hipGetLastError());
  GP_TRY(x.allgather(S + o_cnt, S + o_cnta, (size_t)NB));

  // 4. digests: XOR reduce-scatter over vertex slices, then all-gather the slices
  const bool dig = H(0, H_DIGEST) != 0;
  if (dig) {
    if (c->jdig_words != (size_t)P * Ld) {
      dfree(&c->d_jdig);
      c->jdig_words = 0;
      GP_TRY(dalloc(&c->d_jdig, (size_t)P * Ld));
      c->jdig_words = (size_t)P * Ld;
    }
    std::vector<size_t> soff((size_t)P), sw((size_t)P), roff((size_t)P), rw((size_t)P, (size_t)lend);
    for (int q = 0; q < P; ++q) {
      soff[(size_t)q] = (size_t)q * Ld;
      sw[(size_t)q] = (size_t)std::max<int64_t>(0, std::min<int64_t>(Ld, n - (int64_t)q * Ld));
      roff[(size_t)q] = (size_t)q * Ld;
    }
    GP_TRY(x.alltoall(c->d_digest, soff, sw, S + o_dr, roff, rw, (size_t)Ld));
    hipLaunchKernelGGL(k_shard_xor, dim3(std::max(1, std::min(grid_for(Ld, 256), c->cu_count * 8))), dim3(256), 0, s,
                       S + o_dr, P, Ld, lend, S + o_ds);
    GP_HIP(hipGetLastError());
    GP_TRY(x.allgather(S + o_ds, c->d_jdig, (size_t)Ld));
  }

  // 5. coverage / forwards columns, placed at each rank's block of the job table
  {
    const size_t MM = (size_t)c->words * 64;
    GP_HIP(hipMemsetAsync(S + o_cf, 0, 2 * MS * 8, s));
    GP_HIP(hipMemcpyAsync(S + o_cf, c->d_msg_cov + 2 * MM, (size_t)c->m * 8, hipMemcpyDeviceToDevice, s));
    GP_HIP(hipMemcpyAsync(S + o_cf + MS, c->d_msg_cov + 3 * MM, (size_t)c->m * 8, hipMemcpyDeviceToDevice, s));
    GP_TRY(x.allgather(S + o_cf, S + o_cfa, 2 * MS));
    if (c->jm != (int32_t)mt || !c->d_jcf) {
      dfree(&c->d_jcf);
      GP_TRY(dalloc(&c->d_jcf, 2 * (size_t)std::max<int64_t>(mt, 1)));
    }
    for (int q = 0; q < P; ++q) {
      const size_t at = (size_t)H(q, H_WBASE) * 64, mq = (size_t)H(q, H_M);
      for (int k = 0; k < 2; ++k)
        GP_HIP(hipMemcpyAsync(c->d_jcf + (size_t)k * mt + at, S + o_cfa + ((size_t)q * 2 + k) * MS, mq * 8,
                              hipMemcpyDeviceToDevice, s));
    }
  }
  GP_HIP(hipEventRecord(c->ev[5], s));
  std::vector<u64> cnta((size_t)P * NB);
  GP_HIP(hipMemcpyAsync(sta.data(), S + o_sta, sta.size() * 8, hipMemcpyDeviceToHost, s));
  GP_HIP(hipMemcpyAsync(cnta.data(), S + o_cnta, cnta.size() * 8, hipMemcpyDeviceToHost, s));
  GP_HIP(hipStreamSynchronize(s));

  // the job's rounds
  for (int32_t r = 0; r < R; ++r) {
    gp_round_stats& o = job[r];
    std::memset(&o, 0, sizeof(o));
    o.round = r;
    o.mode = -1;
    bool first = true;
    for (int q = 0; q < P; ++q) {
      const u64* f = &sta[((size_t)q * R + r) * NF];
      if (!f[F_RAN]) continue;
      if (first) {
        o.crashed = f[F_CRASHED]; o.reports = f[F_REPORTS]; o.removals = f[F_REMOVALS]; o.dup_reports = f[F_DUP];
        o.mode = (int32_t)f[F_MODE];
        o.scan = (int32_t)f[F_SCAN];
        first = false;
      } else if (o.crashed != f[F_CRASHED] || o.reports != f[F_REPORTS] || o.removals != f[F_REMOVALS] ||
                 o.dup_reports != f[F_DUP]) {
        return set_error(GP_ESTATE, "gp_shard_combine: the ranks' liveness rounds differ (round " +
                                        std::to_string(r) + "): not one job");
      }
      o.injected += f[F_INJECTED]; o.lost += f[F_LOST]; o.new_bits += f[F_NEW_BITS]; o.sends += f[F_SENDS];
      o.arcs_scanned += f[F_ARCS]; o.rows_gathered += f[F_GATHERED]; o.seen_rows_read += f[F_SEEN_READ];
      o.rows_written += f[F_WRITTEN]; o.vertices_visited += f[F_VISITED]; o.atomics += f[F_ATOMICS];
      o.next_arcs += f[F_NEXT_ARCS]; o.row_bytes += f[F_ROW_BYTES]; o.xchg_rows += f[F_XROWS];
      o.xchg_bytes += f[F_XBYTES]; o.done_nb += f[F_DNB]; o.lm_rows += f[F_LM_ROWS];
      o.overflow |= (int32_t)f[F_OVERFLOW];
      o.expand_ms = std::max(o.expand_ms, dval(f[F_EXPAND_MS]));
      o.exchange_ms = std::max(o.exchange_ms, dval(f[F_EXCHANGE_MS]));
      o.round_ms = std::max(o.round_ms, dval(f[F_ROUND_MS]));
      o.kernel_ms = std::max(o.kernel_ms, dval(f[F_KERNEL_MS]));
    }
    for (int q = 0; q < P; ++q) {
      o.receivers += cnta[(size_t)q * NB + 2 * r];
      o.active += cnta[(size_t)q * NB + 2 * r + 1];
    }
  }
  bool fwd = true;
  for (int q = 0; q < P; ++q) fwd = fwd && H(q, H_FWD) != 0;
  c->jm = (int32_t)mt;
  c->j_fwd_valid = fwd;
  c->j_dig_valid = dig;
  c->j_ready = true;
  if (rounds_out) *rounds_out = R;
  if (ms_out) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[5]);
    *ms_out = ms;
  }
  return 0;
}

}  // namespace

}  // namespace gp

using namespace gp;

extern "C" {

int gp_shard_comm_init(gp_ctx* c, const void* uid, int32_t nranks, int32_t rank) {
  if (!c || !uid) return set_error(GP_EINVAL, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return set_error(GP_EINVAL, "bad rank/nranks");
  if (c->local || c->comm) return set_error(GP_ESTATE, "a shard job runs unpartitioned contexts without a partition communicator");
  GP_HIP(hipSetDevice(c->device));
  if (c->jcomm) (void)ncclCommDestroy(c->jcomm);
  c->jcomm = nullptr;
  c->jhost = nullptr;
  c->jnranks = 0;
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  GP_RCCL(ncclCommInitRank(&c->jcomm, nranks, id, rank));
  c->jnranks = nranks;
  c->jrank = rank;
  shard_reset(c);
  return 0;
}

int gp_shard_host_init(gp_ctx* c, gp_allgather_fn fn, void* user, int32_t nranks, int32_t rank) {
  if (!c || !fn) return set_error(GP_EINVAL, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return set_error(GP_EINVAL, "bad rank/nranks");
  if (c->local || c->comm) return set_error(GP_ESTATE, "a shard job runs unpartitioned contexts without a partition communicator");
  GP_HIP(hipSetDevice(c->device));
  if (c->jcomm) (void)ncclCommDestroy(c->jcomm);
  c->jcomm = nullptr;
  c->jhost = fn;
  c->jhost_user = user;
  c->jnranks = nranks;
  c->jrank = rank;
  shard_reset(c);
  return 0;
}

int gp_shard_info(gp_ctx* c, int32_t* nranks_out, int32_t* rank_out, int32_t* transport_out) {
  if (!c) return set_error(GP_EINVAL, "null ctx");
  int32_t n = 0, r = 0, t = 0;
  if (c->jcomm) {
    int cn = 0, cr = 0;
    GP_RCCL(ncclCommCount(c->jcomm, &cn));
    GP_RCCL(ncclCommUserRank(c->jcomm, &cr));
    n = cn;
    r = cr;
    t = 1;
  } else if (c->jhost) {
    n = c->jnranks;
    r = c->jrank;
    t = 2;
  }
  if (nranks_out) *nranks_out = n;
  if (rank_out) *rank_out = r;
  if (transport_out) *transport_out = t;
  return 0;
}

int gp_shard_combine(gp_ctx* c, gp_round_stats* job, int32_t cap, int32_t* rounds_out, double* ms_out) {
  if (!c || !job || cap < 1) return set_error(GP_EINVAL, "bad argument");
  if (c->jnranks < 1) return set_error(GP_ESTATE, "gp_shard_comm_init or gp_shard_host_init first");
  if (!state_ready(c)) return set_error(GP_ESTATE, "no run state");
  GP_HIP(hipSetDevice(c->device));
  c->j_ready = false;
  return combine(c, job, cap, rounds_out, ms_out);
}

}  // extern "C"
