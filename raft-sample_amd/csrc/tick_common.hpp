// tick_common.hpp — device code shared by the kernel translation units:
// EXT isolation windows, wave/block statistic reductions, the general tick
// (run_tick) and the R-dispatch macro of the host launchers.
#pragma once
#include "kernels.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <mutex>
#include <vector>

namespace raftstep {

// EXT isolation windows (same definition as the oracle's iso_window()): per
// 32-tick epoch e, with probability iso_p/65536, one replica is cut off for
// [start, start+len). Bit (e&1) of *active: epoch e's window covers T.tick;
// of *starting: T.tick is its first tick. Returns the hashed victims.
template <int R>
__device__ __forceinline__ uint32_t iso_windows(uint64_t key, const Trace& T, uint32_t* active, uint32_t* starting) {
  uint32_t mask = 0;
  *active = *starting = 0;
  const int64_t ep = T.tick >> 5;
  // rng_k(key, 0, ST_ISOLATE, e) = sm64(inner ^ e): the inner hash is shared by both epochs
  const uint64_t inner = sm64(key ^ (uint64_t(ST_ISOLATE) << 32));
  for (int64_t e = ep; e >= ep - 1 && e >= 0; --e) {
    const uint64_t h = sm64(inner ^ uint64_t(e));
    if ((h & 0xFFFF) >= T.iso_p) continue;
    const uint32_t victim = uint32_t((h >> 16) & 0xFF) % uint32_t(R);
    const int64_t start = e * 32 + int64_t((h >> 24) & 31);
    const uint32_t x = uint32_t(h >> 32);   // len = iso_min + x mod iso_span
    const int64_t len = int64_t(T.iso_min) + int64_t(x - udiv_magic(x, T.iso_m, T.iso_l) * T.iso_span);
    if (T.tick >= start && T.tick < start + len) {
      mask |= 1u << victim;
      *active |= 1u << (e & 1);
      *starting |= (T.tick == start ? 1u : 0u) << (e & 1);
    }
  }
  return mask;
}
// Hashed-victim mode: the replicas cut off this tick.
template <int R>
__device__ __forceinline__ uint32_t isolation_mask(uint64_t key, const Trace& T) {
  uint32_t a, s;
  return iso_windows<R>(key, T, &a, &s);
}
// Leader mode (isolate_leader, oracle group_iso_mask): a window's victim is
// the lowest-id Leader when its first tick begins (`leaders`: bit r = replica
// r is a Leader), recorded in giso (nibble per epoch parity); no leader then,
// nobody. decide = false (message-level handlers, the steady-state kernel)
// only reads what was recorded.
__device__ __forceinline__ uint32_t leader_iso_mask(uint32_t active, uint32_t starting, uint32_t& giso, uint32_t leaders,
                                                    bool decide) {
  uint32_t mask = 0;
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    if (!((active >> par) & 1u)) continue;
    const int sh = 4 * par;
    if (decide && ((starting >> par) & 1u))
      giso = (giso & ~(0xFu << sh)) | ((leaders ? (8u | uint32_t(__builtin_ctz(leaders))) : 0u) << sh);
    const uint32_t nib = (giso >> sh) & 0xFu;
    if (nib & 8u) mask |= 1u << (nib & 7u);
  }
  return mask;
}
// The replicas cut off this tick, either mode (Group / general kernels).
template <int R>
__device__ __forceinline__ uint32_t tick_iso_mask(uint64_t key, const Trace& T, uint32_t& giso, uint32_t leaders,
                                                  bool decide) {
  uint32_t a, s;
  const uint32_t hashed = iso_windows<R>(key, T, &a, &s);
  return T.iso_leader ? leader_iso_mask(a, s, giso, leaders, decide) : hashed;
}

// Sum of one small per-lane counter over the wave. Counters are almost
// always in [0,15]: four ballots + scalar popcounts; otherwise a shuffle tree.
__device__ __forceinline__ long long wave_sum(int v) {
  if (__all((unsigned)v < 16u)) {
    long long s = __popcll(__ballot(v & 1));
    s += 2ll * __popcll(__ballot(v & 2));
    s += 4ll * __popcll(__ballot(v & 4));
    s += 8ll * __popcll(__ballot(v & 8));
    return s;
  }
  long long x = v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// Leaders of a Group as a replica bit mask (roles: 2 bits per replica).
__device__ __forceinline__ uint32_t leader_bits(uint32_t roles, int R) {
  uint32_t m = 0;
  for (int r = 0; r < R; ++r) m |= (((roles >> (2 * r)) & 3u) == uint32_t(ROLE_L) ? 1u : 0u) << r;
  return m;
}

template <int R, int SEM>
__device__ __forceinline__ void run_tick(Group<R, SEM>& G, const DevPlanes& P, const Trace& T, uint32_t E) {
  if (T.iso_p) G.iso = tick_iso_mask<R>(G.key, T, G.giso, leader_bits(G.roles, R), true);

  // 1. client: every Leader receives E NewLogRequests (main.go:87-93 -> 327-329).
  if (E) {
    static_for<R>([&](auto RI) {
      constexpr int r = decltype(RI)::value;
      if (G.role(r) != ROLE_L || !G.alive()) return;
      const uint64_t vb = P.cv ? cv_base(P, 0, r, G.tick, G.g) : rng_k_call(G.key, r, ST_VALUE, uint64_t(G.tick));
      const int l = G.last[r];
      if (l == 0) G.align_ring(P, T);   // first entry of an empty group: choose the ring phase
      const int room = I32MAX - l;
      const int n_ok = int(E) <= room ? int(E) : room;
      if (G.cache_leader < 0) {
        G.cache_leader = r; G.cache_from = l + 1; G.cache_term = G.term[r]; G.cache_vbase = vb;
      }
      const int e0 = n_ok > int(P.K) ? n_ok - int(P.K) : 0;   // only the last K stay in the ring
      for (int e = e0; e < n_ok; ++e) {
        const int64_t v = entry_value(vb, uint32_t(e), cv_stride(P));
        G.ring_term(P, r, l + 1 + e) = G.term[r];
        G.ring_value(P, r, l + 1 + e) = v;
        if (P.crc_on) G.ring_crc(P, r, l + 1 + e) = crc_entry(P.crc_tab, G.term[r], v);
      }
      if (n_ok) {
        G.last[r] = l + n_ok;
        G.d_last |= 1u << r;
        G.set_lterm(r, G.term[r]);
        if constexpr (SEM == SEM_RAFT) G.template r_grew<r>(l + n_ok);
      }
      if (n_ok < int(E)) G.raise(F_OVERFLOW);
    });
  }

  // 2. rounds in ascending replica id, against the roles as they are now.
  const TickSrc base{P.log_term, P.log_value, P.log_crc, P.crc_tab, P.crc_on, uint32_t(R), G.g, P.KP, P.kmask, G.rot, G.rota, G.rotb, G.sb, G.sb2, 0, 1,
                     G.cache_leader, G.cache_from, G.cache_term, G.cache_vbase, cv_stride(P)};
  auto make_src = [base](int c) {
    TickSrc s = base;
    s.leader = c;
    return s;
  };
  int c = -1;
  while (G.alive()) {
    const uint32_t active = (G.roles | (G.roles >> 1)) & 0x5555u;  // bit 2r: role(r) != Follower
    const uint32_t rest = active & ~((1u << (2 * c + 2)) - 1u);    // replicas after c (c=-1: all)
    if (!rest) break;
    c = int(__builtin_ctz(rest)) >> 1;
    if constexpr (SEM == SEM_RAFT) {
      if (G.role(c) == ROLE_L) G.r_leader_round(P, T, c, make_src);
      else G.r_candidate_round(P, T, c);
    } else {
      if (G.role(c) == ROLE_L) G.leader_round(P, T, c, make_src);  // main.go:332-391
      else G.candidate_round(P, T, c);                             // main.go:253-284
    }
  }

  // 3. expired election timers in (deadline, id) order; each new candidate
  //    runs its vote round at once (main.go:171-177, 248-251 -> 253-284).
#pragma unroll 1
  for (int it = 0; it < R && G.alive(); ++it) {
    int best = -1, bdl = 0;
    static_for<R>([&](auto RI) {
      constexpr int r = decltype(RI)::value;
      if (G.role(r) == ROLE_L) return;
      const int d = G.template deadline_of<r>(P);
      if (d <= G.now && (best < 0 || d < bdl)) { best = r; bdl = d; }
    });
    if (best < 0) break;
    if constexpr (SEM == SEM_RAFT) G.r_timeout_fire(T, best);
    else G.timeout_fire(T, best);
    if (!G.alive()) break;
    if constexpr (SEM == SEM_RAFT) G.r_candidate_round(P, T, best);
    else G.candidate_round(P, T, best);
  }

  if (!G.alive()) {
    ++G.st[S_FAULTS];
  } else if ((G.roles >> 1) & ~G.roles & 0x5555u) {
    ++G.st[S_LEADER_GROUPS];
  }
}

// Block-level sum of per-lane counters into the tick's stats slot (one
// device-scope atomic per non-zero counter per block, spread over
// STAT_SLOTS slots).
template <int N>
__device__ __forceinline__ void block_stats(const int (&v)[N], const int (&idx)[N], unsigned long long* stats) {
  __shared__ long long red[N][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int s = 0; s < N; ++s) {
    const long long w = wave_sum(v[s]);
    if (lane == 0) red[s][wave] = w;
  }
  __syncthreads();
  if (threadIdx.x < N) {
    const int s = threadIdx.x;
    long long x = red[s][0];   // (blocks of 64..256 lanes)
    for (int w = 1; w < int(blockDim.x >> 6); ++w) x += red[s][w];
    int which = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) which = (s == k) ? idx[k] : which;
    if (x) atomicAdd(&stats[(blockIdx.x % STAT_SLOTS) * NSTAT + which], (unsigned long long)x);
  }
}

// The lean / fused kernels' statistics of one tick, as exceptions (round 5).
// The reduce kernel adds, for every tick of a two-pass call, the statistics
// of every live group taking a normal tick with `lean_base_committed` entries
// committed (k_init.hip stats_reduce_kernel: R-1 accepted AppendEntries and
// one leader group each); a lane reports only how it differs from that — a
// committed count other than the base, a tick that is not normal (passed on,
// skipped, held by the list kernel), an LXS or an SXS tick (k_fast.hip: an
// LXS tick has R-1 AppendEntries dropped, an SXS tick R-2 accepted and R
// dropped). A wave whose lanes are all the base does nothing; one that is not
// adds its sums to one of STAT_PKS slots (64-B lines: committed difference,
// not-normal | LXS << 21 | SXS << 42). Measured (round 5, tools/stats_cost.py): the
// per-block sums with a barrier cost the C2-shape kernel 8% per tick with
// statistics, atomics or not; in steady state this costs one ballot. Under
// isolation churn (most waves hold an exception) the lean kernel keeps the
// per-block absolute counters (block_stats; 2% faster on C4) and the call
// has no base (engine.cpp call_lean).
__host__ __device__ __forceinline__ int lean_base_committed(int sem_raft, int R, uint32_t n) {
  return (sem_raft || 2 * (R - 1) > R) ? int(n) : 0;   // (k_fast.hip: the commit rule of a normal tick)
}
template <bool RAFT>
__device__ __forceinline__ void lean_stats(bool live, int dcommitted, bool normal, bool lxs, bool sxs,
                                           unsigned long long* stats) {
  if (!__ballot(live && (dcommitted != 0 || !normal))) return;   // (wave-uniform)
  const unsigned long long c = (unsigned long long)wave_sum(live ? dcommitted : 0);
  // not-normal | LXS << 21 | SXS << 42 (per slot and tick at most 64 * ceil(G / 64 / STAT_PKS) lanes each,
  // < 2^21: engine.cpp limits G to Gp * recw * 4 < 2^32, i.e. G < 2^27)
  const unsigned long long k = (unsigned long long)__popcll(__ballot(live && !normal)) |
                               (RAFT ? ((unsigned long long)__popcll(__ballot(live && lxs)) << 21) |
                                           ((unsigned long long)__popcll(__ballot(live && sxs)) << 42)
                                     : 0ull);
  if ((threadIdx.x & 63u) == 0) {
    unsigned long long* pk = stats + STAT_PK + ((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % STAT_PKS) * 8;
    if (c) atomicAdd(&pk[0], c);
    if (k) atomicAdd(&pk[1], k);
  }
}

template <int R, typename F>
__device__ __forceinline__ void with_replica(int x, F&& f) {
  static_for<R>([&](auto PI) {
    if (x == decltype(PI)::value) f(PI);
  });
}

#define RAFT_DISPATCH_R(R_, CALL)                                              \
  switch (R_) {                                                                \
    case 1: { constexpr int RR = 1; CALL; } break;                             \
    case 2: { constexpr int RR = 2; CALL; } break;                             \
    case 3: { constexpr int RR = 3; CALL; } break;                             \
    case 4: { constexpr int RR = 4; CALL; } break;                             \
    case 5: { constexpr int RR = 5; CALL; } break;                             \
    case 6: { constexpr int RR = 6; CALL; } break;                             \
    case 7: { constexpr int RR = 7; CALL; } break;                             \
    case 8: { constexpr int RR = 8; CALL; } break;                             \
    default: return hipErrorInvalidValue;                                      \
  }

static inline dim3 grid_for(uint64_t n) { return dim3(unsigned((n + 255) / 256)); }

// Resident blocks of kernel `k` at `block` threads per block on the current
// device (CUs x blocks per CU at its register / LDS occupancy), cached per
// (device, kernel, block size): kernels of one signature (e.g. every R's
// general kernel) must not share an entry, and engines on different GPUs of
// one process may see different CU counts.
template <typename Kern>
static unsigned resident_blocks(Kern k, int block = 256) {
  struct Ent { int dev; const void* fn; int block; unsigned n; };
  static std::mutex mu;
  static std::vector<Ent> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  const void* fn = reinterpret_cast<const void*>(k);
  std::lock_guard<std::mutex> lock(mu);
  for (const Ent& x : cache)
    if (x.dev == dev && x.fn == fn && x.block == block) return x.n;
  int cus = 0, per = 0;
  unsigned n = 2048;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, block, 0) == hipSuccess && cus > 0 && per > 0)
    n = unsigned(cus) * unsigned(per);
  cache.push_back(Ent{dev, fn, block, n});
  return n;
}

}  // namespace raftstep
