// trace_rng.hpp — host copy of the engine's trace definition (counter RNG),
// so a host-driven loop can feed the handlers exactly the client values the
// fused tick generates on the device (raft_device.hpp: sm64/group_key/rng_k).
#pragma once
#include <cstdint>

namespace raft {
inline uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
// rand.Int() of main.go:92 for client entry e of (group, leader replica, tick)
inline int64_t client_value(uint64_t seed, uint64_t gid, uint32_t replica, uint64_t tick, uint32_t e) {
  const uint64_t k = sm64(seed ^ sm64(gid));
  const uint64_t h = sm64(sm64(k ^ ((uint64_t(1) << 32) | replica)) ^ tick);
  return int64_t(sm64(h ^ e) >> 1);
}
}  // namespace raft
