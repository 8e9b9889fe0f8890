// xplan.h -- host-side bookkeeping of the vertex partition's boundary exchange
// (partition.hip).  Plain C++, no HIP: the RCCL path
// (exchange_rccl) and the device-copy path (exchange_group) both turn the
// per-round count matrix into buffer offsets through these functions, and
// tests/test_xplan.py drives them on synthetic count matrices on the CPU.
//
// The reference sends gossip only over real links (Peer.py:402-404); here a
// rank sends each peer one entry per owned boundary vertex the peer holds as a
// ghost, and the receiver addresses it by its index in that peer's ghost list.
#pragma once
#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

namespace gp {

// One peer's part of a send or receive buffer: heads [h0, h0 + nh), words
// [w0, w0 + nw) (u64 units).
struct XSlice {
  int64_t h0 = 0, nh = 0, w0 = 0, nw = 0;
};

// Rank d's view of one round's exchange.
struct XPlan {
  std::vector<int64_t> rk, rw;   // [P + 1] receive offsets by sender (heads, words); self gets 0
  std::vector<XSlice> send;      // [P] what d sends to q (offsets into d's send buffers)
  std::vector<XSlice> recv;      // [P] what d receives from q (offsets into d's receive buffers)
};

// What sender q sends to receiver d, as offsets into q's send buffers.
inline XSlice xplan_send_of(const unsigned long long* cnt_all, int P, int q, int d) {
  const unsigned long long* x = cnt_all + ((size_t)q * P + (size_t)d) * 4;
  return XSlice{(int64_t)x[0], (int64_t)x[1], (int64_t)x[2], (int64_t)x[3]};
}

// cnt_all: P rows of 4P u64, row q = sender q, entry 4d + {0,1,2,3} = (head
// offset, heads, word offset, words) of what q sends to d, as k_bnd_counts
// wrote them.  ghosts[q]: ghosts of owner q that rank d holds (h_gh_ptr
// differences).  W: words per Message-List row.  An entry is one head plus a
// mask word and at most W row words, and entry e of sender q lands on ghost
// gh_ptr[q] + e: a sender with more entries than d holds ghosts of it would
// write into another owner's ghosts, so that is an error, not a clamp.
inline bool xplan_build(const unsigned long long* cnt_all, int P, int d, const int64_t* ghosts, int W, XPlan* out,
                        std::string* err) {
  out->rk.assign((size_t)P + 1, 0);
  out->rw.assign((size_t)P + 1, 0);
  out->send.assign((size_t)P, XSlice{});
  out->recv.assign((size_t)P, XSlice{});
  for (int q = 0; q < P; ++q) {
    int64_t nh = 0, nw = 0;
    if (q != d) {
      const XSlice in = xplan_send_of(cnt_all, P, q, d);
      nh = in.nh;
      nw = in.nw;
      if (nh > ghosts[q]) {
        if (err) *err = "exchange: rank " + std::to_string(q) + " sends " + std::to_string(nh) +
                        " entries to rank " + std::to_string(d) + ", which holds " + std::to_string(ghosts[q]) +
                        " of its vertices as ghosts";
        return false;
      }
      if (nw < nh || nw > nh * (int64_t)(W + 1)) {
        if (err) *err = "exchange: rank " + std::to_string(q) + " sends " + std::to_string(nw) + " words in " +
                        std::to_string(nh) + " entries to rank " + std::to_string(d);
        return false;
      }
      out->send[(size_t)q] = xplan_send_of(cnt_all, P, d, q);
    }
    out->rk[(size_t)q + 1] = out->rk[(size_t)q] + nh;
    out->rw[(size_t)q + 1] = out->rw[(size_t)q] + nw;
    out->recv[(size_t)q] = XSlice{out->rk[(size_t)q], nh, out->rw[(size_t)q], nw};
  }
  return true;
}

// Every receiver's plan from the same count matrix: the RCCL path checks all
// of them before any send, so every rank takes the same decision (one rank
// returning early while its peers enter ncclSend / ncclRecv would hang them).
// ghosts_all: P rows of P, row d = ghosts rank d holds of each owner.
inline bool xplan_check_all(const unsigned long long* cnt_all, int P, const int64_t* ghosts_all, int W, std::string* err) {
  XPlan tmp;
  for (int d = 0; d < P; ++d)
    if (!xplan_build(cnt_all, P, d, ghosts_all + (size_t)d * P, W, &tmp, err)) return false;
  return true;
}

// Once per partition: the send list B_qd of every rank q must be as long as
// rank d's ghost list of owner q (the two are the same vertices in the same
// order on a symmetric overlay, Seed.py:131-149).  bnd_all: P rows of P, row q
// = |B_qd| for each d; ghosts_all as above.  A mismatch means the overlay is
// not symmetric (or the ranks disagree on the partition).
inline bool xplan_check_lists(const int64_t* bnd_all, const int64_t* ghosts_all, int P, std::string* err) {
  for (int q = 0; q < P; ++q)
    for (int d = 0; d < P; ++d) {
      if (q == d) continue;
      const int64_t b = bnd_all[(size_t)q * P + d], g = ghosts_all[(size_t)d * P + q];
      if (b != g) {
        if (err) *err = "partition: rank " + std::to_string(q) + " sends " + std::to_string(b) +
                        " boundary vertices to rank " + std::to_string(d) + ", which holds " + std::to_string(g) +
                        " ghosts of it (overlay not symmetric?)";
        return false;
      }
    }
  return true;
}

// Owned slices of a vertex partition: bounds[p] .. bounds[p + 1] for rank p.
// by_arcs == 0: equal vertex counts (ceil(n / P) each); by_arcs == 1: equal
// in-arc counts (the power-law skew is in the degrees,
// demonstrate_powerlaw.py:24-27), bounds[p] = the first vertex whose arcs
// start at or after ceil(p * nnz / P).  row_ptr: the global in-CSR offsets.
inline std::vector<int64_t> partition_bounds(int64_t n, int P, int by_arcs, const int64_t* row_ptr) {
  std::vector<int64_t> b((size_t)P + 1, n);
  b[0] = 0;
  const int64_t nnz = row_ptr ? row_ptr[n] : 0;
  for (int p = 1; p < P; ++p) {
    if (by_arcs && row_ptr && nnz > 0) {
      const int64_t target = (p * nnz + P - 1) / P;
      int64_t lo = 0, hi = n;   // first v in [0, n] with row_ptr[v] >= target
      while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (row_ptr[mid] < target) lo = mid + 1;
        else hi = mid;
      }
      b[(size_t)p] = lo;
    } else {
      const int64_t S = (n + P - 1) / P;
      b[(size_t)p] = std::min<int64_t>(n, (int64_t)p * S);
    }
    if (b[(size_t)p] < b[(size_t)p - 1]) b[(size_t)p] = b[(size_t)p - 1];
  }
  return b;
}

// Owner of global vertex u under `bounds` (the last p with bounds[p] <= u).
inline int64_t owner_of(const std::vector<int64_t>& bounds, int64_t u) {
  int64_t lo = 0, hi = (int64_t)bounds.size() - 2;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) / 2;
    if (bounds[(size_t)mid] <= u) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

}  // namespace gp
