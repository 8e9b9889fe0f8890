// gp_common.h -- constants and integer mixing functions shared by the device
// kernels and the host side of libgossip_hip.so.  The CPU oracle restates these
// independently (oracle/gossip_oracle.c); DESIGN.md §2 is the normative text.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GP_HD __host__ __device__ __forceinline__
#else
#define GP_HD static inline
#endif

namespace gp {

// vertex state bits (u8 per vertex)
constexpr uint8_t ST_CRASHED = 1;   // crash-stop: neither receives nor sends
constexpr uint8_t ST_REMOVED = 2;   // removed by the seed registry (Seed.py:387-391)
constexpr uint8_t ST_PENDING = 4;   // explicit crash requested for the next round
constexpr uint8_t ST_DOWN = ST_CRASHED | ST_REMOVED;

// splitmix64 output function (Steele/Lea/Flood), DESIGN.md §2.6
GP_HD uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
// per-(seed, stream) key and counter-based draw
GP_HD uint64_t stream_key(uint64_t seed, uint64_t stream) {
  return splitmix64(seed ^ splitmix64(stream));
}
GP_HD uint64_t draw(uint64_t key, uint64_t idx) {
  return splitmix64(key + idx * 0x9E3779B97F4A7C15ULL);
}
// uniform integer in [0, n) from 64 random bits (multiply-high, exact)
GP_HD uint64_t below(uint64_t r, uint64_t n) {
  return (uint64_t)(((unsigned __int128)r * (unsigned __int128)n) >> 64);
}
// MurmurHash3 fmix64: the per-vertex first-receipt digest term
GP_HD uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
// digest term of the first receipts `bits` of word `w` at receipt round `rr`
GP_HD uint64_t digest_term(uint32_t rr, uint32_t w, uint64_t bits) {
  return fmix64(bits ^ fmix64(((uint64_t)(rr + 1) << 32) | (uint64_t)w));
}

// injection receipts are salted so that the digest is a function of the
// first-receipt matrix (own-origin messages are known from the message table)
constexpr uint32_t DIGEST_INJECT = 0x80000000u;

// RNG streams
constexpr uint64_t STREAM_EDGE = 1;
constexpr uint64_t STREAM_RELABEL = 2;
constexpr uint64_t STREAM_CRASH = 0x100;   // + round

}  // namespace gp
