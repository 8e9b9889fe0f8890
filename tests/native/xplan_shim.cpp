// xplan_shim.cpp -- test-only C wrapper around csrc/xplan.h (host code, no HIP),
// compiled with g++ by tests/test_xplan.py so the exchange bookkeeping of the
// vertex partition is exercised on the CPU with synthetic count matrices.
#include <cstring>

#include "xplan.h"

extern "C" {

// rk, rw: [P + 1]; send, recv: [P][4] (h0, nh, w0, nw).  Returns 1 / 0; err: 256 bytes.
int xs_build(const unsigned long long* cnt_all, int P, int d, const long long* ghosts, int W, long long* rk,
             long long* rw, long long* send, long long* recv, char* err) {
  gp::XPlan plan;
  std::string e;
  const bool ok = gp::xplan_build(cnt_all, P, d, reinterpret_cast<const int64_t*>(ghosts), W, &plan, &e);
  std::strncpy(err, e.c_str(), 255);
  if (!ok) return 0;
  for (int q = 0; q <= P; ++q) {
    rk[q] = plan.rk[(size_t)q];
    rw[q] = plan.rw[(size_t)q];
  }
  for (int q = 0; q < P; ++q) {
    const gp::XSlice* s[2] = {&plan.send[(size_t)q], &plan.recv[(size_t)q]};
    long long* o[2] = {send + 4 * q, recv + 4 * q};
    for (int k = 0; k < 2; ++k) {
      o[k][0] = s[k]->h0; o[k][1] = s[k]->nh; o[k][2] = s[k]->w0; o[k][3] = s[k]->nw;
    }
  }
  return 1;
}

int xs_check_all(const unsigned long long* cnt_all, int P, const long long* ghosts_all, int W, char* err) {
  std::string e;
  const bool ok = gp::xplan_check_all(cnt_all, P, reinterpret_cast<const int64_t*>(ghosts_all), W, &e);
  std::strncpy(err, e.c_str(), 255);
  return ok ? 1 : 0;
}

int xs_check_lists(const long long* bnd_all, const long long* ghosts_all, int P, char* err) {
  std::string e;
  const bool ok = gp::xplan_check_lists(reinterpret_cast<const int64_t*>(bnd_all),
                                        reinterpret_cast<const int64_t*>(ghosts_all), P, &e);
  std::strncpy(err, e.c_str(), 255);
  return ok ? 1 : 0;
}

void xs_bounds(long long n, int P, int by_arcs, const long long* row_ptr, long long* out) {
  const std::vector<int64_t> b = gp::partition_bounds(n, P, by_arcs, reinterpret_cast<const int64_t*>(row_ptr));
  for (int p = 0; p <= P; ++p) out[p] = b[(size_t)p];
}

long long xs_owner(const long long* bounds, int P, long long u) {
  const std::vector<int64_t> b(bounds, bounds + P + 1);
  return gp::owner_of(b, u);
}

}  // extern "C"
