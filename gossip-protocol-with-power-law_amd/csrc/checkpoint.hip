// checkpoint.hip -- snapshot / restore of a context's per-run state between
// rounds (checkpointed long runs, e.g. 2^26-node churn
// sweeps).  The reference keeps no state worth saving (its peers log and
// exit), so this has no reference counterpart; parity is "restore + continue
// == uninterrupted run", tested bit for bit in tests/test_gpu_parity.py.
//
// The blob is opaque to the caller (engine.py writes it into an .npz).  It
// holds each vertex's Message-List row in canonical form -- one row per
// vertex, wherever its slot byte put it -- rather than both slot buffers, so a
// 2^24 x 4096 checkpoint is 8 GiB of rows instead of 16.  Restoring places
// every row in the slot that round r reads (S[r & 1]); the other slot is
// marked unwritten, as after gp_reset.  That state is equivalent for every
// later round: senders are read from S[r & 1], receivers read their own row
// through the slot byte and write whole rows into S[(r + 1) & 1], and the
// unfiltered pull zeroes unwritten rows before it reads them (k_fixup_rows).
#include <cstring>

#include "gp_internal.h"

namespace gp {

constexpr uint64_t CKPT_MAGIC = 0x3130545048434b47ull;   // "GKCHPT01"
constexpr uint8_t CK_SLOT_NONE = 0xFF;                   // gp_device.h SLOT_NONE
constexpr int64_t CK_CHUNK_WORDS = (int64_t)8 << 20;     // 64 MB of rows per staging pass

struct CkptHeader {
  uint64_t magic;
  int32_t abi, words;
  int64_t n, nnz, n_alloc, vbegin, vend;
  int32_t m, msg_word_base;
  int32_t round, cur;
  int32_t liveness_active, pending_crash, msg_forwards_valid, done_dirty;
  int32_t has_first, has_frx, cmask_rows, alive_from1;   // alive_from + 1 (0: no complete alive set)
  uint64_t prev_next_arcs, prev_new_bits, prev_receivers, held_bits;
  int64_t last_reports;     // reports of the round just taken (exact count)
  int64_t saved_reports;    // how many of them the blob holds (<= the report buffer)
};

static int64_t align8(int64_t b) { return (b + 7) & ~(int64_t)7; }

// one section of the blob: a device array copied whole
struct Section {
  void* dev;
  int64_t bytes;
};

static std::vector<Section> plain_sections(Ctx* c) {
  const int64_t na = c->n_alloc, nl = std::max<int64_t>(c->nloc(), 1), W = c->words;
  std::vector<Section> s = {
      {c->d_sp, na},
      {c->d_fpop[0], na * 4},
      {c->d_fpop[1], na * 4},
      {c->d_seenpop, nl * 4},
      {c->d_digest, nl * 8},
      {c->d_state, na},
      {c->d_miss, na},
      {c->d_deg_live, na * 4},
      {c->d_tbits, (na + 63) / 64 * 8},
      {c->d_msg_cov, W * 64 * 4 * 8},
      {c->d_alive, 2 * W * 8},
      {c->d_done_at, na * 4},
      {c->d_cmask, (int64_t)c->cmask_rows * W * 8},
  };
  if (c->d_first && c->cfg.track_first) s.push_back({c->d_first, nl * W * 64});
  if (c->d_frx[0]) s.push_back({c->d_frx[c->cur], c->frx_rows * W * 8});
  return s;
}

// reports of the last round held in the device buffer (gp_reports reads them
// after a restore exactly as after the round itself)
static int64_t saved_reports(const Ctx* c) { return std::min(c->last_reports, c->report_cap); }

static int64_t blob_bytes(Ctx* c, int64_t nrep) {
  int64_t b = align8((int64_t)sizeof(CkptHeader)) + c->n_alloc * c->words * 8;   // canonical rows
  for (const Section& s : plain_sections(c)) b += align8(s.bytes);
  return b + align8(nrep * (int64_t)sizeof(gp_report));
}

// rows[t] = word t % W of vertex v0 + t / W's Message-List row (zero if none)
__global__ void k_ckpt_gather(const u64* __restrict__ s0, const u64* __restrict__ s1, const u64* __restrict__ s2,
                              const uint8_t* __restrict__ sp, u64* __restrict__ out, int64_t v0,
                              int64_t words_total, int32_t W) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= words_total) return;
  const int64_t v = v0 + t / W;
  const uint8_t p = sp[v];
  const size_t i = (size_t)v * W + (size_t)(t % W);
  out[t] = p == CK_SLOT_NONE ? 0ull : (p == 0 ? s0[i] : p == 1 ? s1[i] : s2[i]);   // 2: parked
}
__global__ void k_ckpt_scatter(u64* __restrict__ slot, const u64* __restrict__ in, int64_t v0,
                               int64_t words_total, int32_t W) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < words_total) slot[(size_t)v0 * W + (size_t)t] = in[t];
}

static bool run_state(const Ctx* c) { return c->d_sp != nullptr && c->d_slot[0] != nullptr && c->words > 0; }

}  // namespace gp

using namespace gp;

extern "C" {

int gp_checkpoint_size(gp_ctx* c, int64_t* bytes) {
  if (!c || !bytes) return set_error(GP_EINVAL, "null argument");
  if (!run_state(c)) return set_error(GP_ESTATE, "no run state (gp_reset first)");
  *bytes = blob_bytes(c, saved_reports(c));
  return 0;
}

int gp_checkpoint_save(gp_ctx* c, void* host, int64_t bytes) {
  if (!c || !host) return set_error(GP_EINVAL, "null argument");
  if (!run_state(c)) return set_error(GP_ESTATE, "no run state (gp_reset first)");
  const int64_t nrep = saved_reports(c);
  if (bytes != blob_bytes(c, nrep))
    return set_error(GP_EINVAL, "bytes mismatch: expected " + std::to_string(blob_bytes(c, nrep)));
  GP_HIP(hipSetDevice(c->device));
  GP_TRY(unalias(c, false));   // aliased Message-Lists are saved as the rows they stand for
  GP_HIP(hipStreamSynchronize(c->stream));
  uint8_t* out = static_cast<uint8_t*>(host);
  CkptHeader h{};
  h.magic = CKPT_MAGIC;
  h.abi = GP_ABI_VERSION;
  h.words = c->words;
  h.n = c->n; h.nnz = c->nnz; h.n_alloc = c->n_alloc; h.vbegin = c->vbegin; h.vend = c->vend;
  h.m = c->m; h.msg_word_base = c->cfg.msg_word_base;
  h.round = c->round; h.cur = c->cur;
  h.liveness_active = c->liveness_active; h.pending_crash = c->pending_crash;
  h.msg_forwards_valid = c->msg_forwards_valid; h.done_dirty = c->done_dirty;
  h.has_first = c->d_first && c->cfg.track_first ? 1 : 0;
  h.has_frx = c->d_frx[0] ? 1 : 0;
  h.cmask_rows = c->cmask_rows;
  h.alive_from1 = c->alive_from + 1;
  h.prev_next_arcs = c->prev_next_arcs; h.prev_new_bits = c->prev_new_bits;
  h.prev_receivers = c->prev_receivers; h.held_bits = c->held_bits;
  h.last_reports = c->last_reports;
  h.saved_reports = nrep;
  std::memcpy(out, &h, sizeof(h));
  int64_t off = align8((int64_t)sizeof(CkptHeader));
  // canonical rows, staged through a device buffer
  const int64_t W = c->words, total = c->n_alloc * W;
  const int64_t chunk = std::max<int64_t>(CK_CHUNK_WORDS / W, 1) * W;
  u64* stage = nullptr;
  GP_TRY(dalloc(&stage, (size_t)std::min(chunk, std::max<int64_t>(total, 1))));
  for (int64_t t0 = 0; t0 < total; t0 += chunk) {
    const int64_t cnt = std::min(chunk, total - t0);
    hipLaunchKernelGGL(k_ckpt_gather, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, c->stream, c->d_slot[0],
                       c->d_slot[1], c->d_slot[2], c->d_sp, stage, t0 / W, cnt, (int32_t)W);
    hipError_t e = hipGetLastError();
    int rc = e == hipSuccess ? copy_sync(c, out + off + t0 * 8, stage, (size_t)cnt * 8, hipMemcpyDeviceToHost)
                             : set_error(GP_EHIP, std::string("k_ckpt_gather: ") + hipGetErrorString(e));
    if (rc) { dfree(&stage); return rc; }
  }
  dfree(&stage);
  off += total * 8;
  for (const Section& s : plain_sections(c)) {
    GP_TRY(copy_sync(c, out + off, s.dev, (size_t)s.bytes, hipMemcpyDeviceToHost));
    off += align8(s.bytes);
  }
  GP_TRY(copy_sync(c, out + off, c->d_reports, (size_t)nrep * sizeof(gp_report), hipMemcpyDeviceToHost));
  return 0;
}

int gp_checkpoint_load(gp_ctx* c, const void* host, int64_t bytes) {
  if (!c || !host) return set_error(GP_EINVAL, "null argument");
  if (bytes < (int64_t)sizeof(CkptHeader)) return set_error(GP_EINVAL, "checkpoint too short");
  CkptHeader h;
  std::memcpy(&h, host, sizeof(h));
  if (h.magic != CKPT_MAGIC) return set_error(GP_EINVAL, "not a gossip checkpoint");
  if (h.abi != GP_ABI_VERSION) return set_error(GP_EINVAL, "checkpoint of ABI " + std::to_string(h.abi));
  // Everything is checked against what the context knows BEFORE gp_reset, so
  // a rejected blob leaves the run in progress untouched: same overlay,
  // messages, partition, tracked outputs, component targets and size.
  if (h.n != c->n || h.nnz != c->nnz || h.m != c->m || h.words != c->words || h.msg_word_base != c->cfg.msg_word_base)
    return set_error(GP_EINVAL, "checkpoint of another overlay or message set");
  if (h.n_alloc != c->n_alloc || h.vbegin != c->vbegin || h.vend != c->vend)
    return set_error(GP_EINVAL, "checkpoint of another partition");
  if (h.has_first != (c->cfg.track_first ? 1 : 0) || h.has_frx != (c->cfg.track_msg_forwards || c->local ? 1 : 0))
    return set_error(GP_EINVAL, "checkpoint tracks other outputs (track_first / track_msg_forwards)");
  GP_HIP(hipSetDevice(c->device));
  // the component targets (cmask rows) of this message set; computing them
  // touches no run state that could be in progress (set_messages invalidated it)
  if (!c->d_sp || !c->d_slot[0] || !c->done_at_valid) GP_TRY(gp_reset(c));
  if (h.cmask_rows != c->cmask_rows) return set_error(GP_EINVAL, "checkpoint of another message set (targets)");
  if (h.saved_reports < 0 || h.saved_reports > h.last_reports || h.saved_reports > c->report_cap)
    return set_error(GP_EINVAL, "checkpoint holds more reports than report_capacity");
  if (bytes != blob_bytes(c, h.saved_reports))
    return set_error(GP_EINVAL, "bytes mismatch: expected " + std::to_string(blob_bytes(c, h.saved_reports)));
  GP_TRY(gp_reset(c));   // accepted: clear the run state, then fill it from the blob
  GP_HIP(hipSetDevice(c->device));
  const uint8_t* in = static_cast<const uint8_t*>(host);
  c->round = h.round;
  c->cur = h.cur & 1;
  int64_t off = align8((int64_t)sizeof(CkptHeader));
  const int64_t W = c->words, total = c->n_alloc * W;
  const int64_t chunk = std::max<int64_t>(CK_CHUNK_WORDS / W, 1) * W;
  u64* stage = nullptr;
  GP_TRY(dalloc(&stage, (size_t)std::min(chunk, std::max<int64_t>(total, 1))));
  for (int64_t t0 = 0; t0 < total; t0 += chunk) {   // every row into the slot round r reads
    const int64_t cnt = std::min(chunk, total - t0);
    int rc = copy_sync(c, stage, in + off + t0 * 8, (size_t)cnt * 8, hipMemcpyHostToDevice);
    if (rc) { dfree(&stage); return rc; }
    hipLaunchKernelGGL(k_ckpt_scatter, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, c->stream,
                       c->d_slot[c->cur], stage, t0 / W, cnt, (int32_t)W);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) { dfree(&stage); return set_error(GP_EHIP, std::string("k_ckpt_scatter: ") + hipGetErrorString(e)); }
  }
  dfree(&stage);
  off += total * 8;
  for (const Section& s : plain_sections(c)) {
    GP_TRY(copy_sync(c, s.dev, in + off, (size_t)s.bytes, hipMemcpyHostToDevice));
    off += align8(s.bytes);
  }
  GP_TRY(copy_sync(c, c->d_reports, in + off, (size_t)h.saved_reports * sizeof(gp_report), hipMemcpyHostToDevice));
  // slot bytes: saved rows now live in S[cur]; the other slot reads as unwritten
  {
    const size_t na = (size_t)c->n_alloc;
    std::vector<uint8_t> sp(na), ws(na);
    GP_TRY(copy_sync(c, sp.data(), c->d_sp, na, hipMemcpyDeviceToHost));
    for (size_t v = 0; v < na; ++v) {
      const bool none = sp[v] == CK_SLOT_NONE;
      sp[v] = none ? CK_SLOT_NONE : (uint8_t)c->cur;
      ws[v] = none ? 0 : (uint8_t)(1u << c->cur);
    }
    GP_TRY(copy_sync(c, c->d_sp, sp.data(), na, hipMemcpyHostToDevice));
    GP_TRY(copy_sync(c, c->d_ws, ws.data(), na, hipMemcpyHostToDevice));
  }
  c->liveness_active = h.liveness_active != 0;
  c->alive_from = h.alive_from1 - 1;
  // a blob written before the field was alive_from + 1 holds 0 there; current
  // code never saves an active liveness phase without a complete alive set
  // from some round, so 0 with liveness on means "unknown": the alive set the
  // next round builds is complete from the round after it (as after gp_crash)
  if (h.alive_from1 == 0 && c->liveness_active) c->alive_from = c->round + 1;
  c->pending_crash = h.pending_crash != 0;
  c->msg_forwards_valid = h.msg_forwards_valid != 0;
  c->done_dirty = true;   // the working targets came from the blob; the next reset restores the pristine ones
  c->prev_next_arcs = h.prev_next_arcs;
  c->prev_new_bits = h.prev_new_bits;
  c->prev_receivers = h.prev_receivers;
  c->held_bits = h.held_bits;
  c->cml_written_prev = false;   // compact lists are rebuilt by the next sparse round
  c->cml_read_now = c->cml_write_now = false;
  c->last_reports = h.last_reports;
  return 0;
}

}  // extern "C"
