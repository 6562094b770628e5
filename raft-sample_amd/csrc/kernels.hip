// kernels.hip — gfx950 kernels of the batched Raft step engine.
//
//  tick_kernel<R>  : the fused per-tick step (client append, leader
//                    replication round + commit / candidate vote round,
//                    election timers) for every group, one lane per group.
//                    HBM-bound: ~233 B per group-step at R=5, E=1.
//  ops_kernel<R>   : the message-level handler API (AppendEntries /
//                    RequestVote receivers, node steps) over distinct groups.
//  init_*_kernel<R>: NewNode state / post-election state.
#include "kernels.h"

namespace raftstep {

// EXT isolation windows (same definition as oracle_isolated()).
template <int R>
__device__ __forceinline__ uint32_t isolation_mask(uint64_t key, const Trace& T) {
  uint32_t mask = 0;
  const int64_t ep = T.tick >> 5;
  for (int64_t e = ep; e >= ep - 1 && e >= 0; --e) {
    const uint64_t h = rng_k(key, 0, ST_ISOLATE, uint64_t(e));
    if ((h & 0xFFFF) >= T.iso_p) continue;
    const uint32_t victim = uint32_t((h >> 16) & 0xFF) % uint32_t(R);
    const int64_t start = e * 32 + int64_t((h >> 24) & 31);
    const int64_t len = int64_t(T.iso_min) + int64_t(uint32_t(h >> 32) % T.iso_span);
    if (T.tick >= start && T.tick < start + len) mask |= 1u << victim;
  }
  return mask;
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

template <int R>
__device__ __forceinline__ void run_tick(Group<R>& G, const DevPlanes& P, const Trace& T, uint32_t E) {
  if (T.iso_p) G.iso = isolation_mask<R>(G.key, T);

  // 1. client: every Leader receives E NewLogRequests (main.go:87-93 -> 327-329).
  if (E) {
    static_for<R>([&](auto RI) {
      constexpr int r = decltype(RI)::value;
      if (G.role(r) != ROLE_L || !G.alive()) return;
      const uint64_t vb = rng_k(G.key, r, ST_VALUE, uint64_t(G.tick));
      const int l = G.last[r];
      const int room = I32MAX - l;
      const int n_ok = int(E) <= room ? int(E) : room;
      if (G.cache_leader < 0) {
        G.cache_leader = r; G.cache_from = l + 1; G.cache_term = G.term[r]; G.cache_vbase = vb;
      }
      const int e0 = n_ok > int(P.K) ? n_ok - int(P.K) : 0;   // only the last K stay in the ring
      for (int e = e0; e < n_ok; ++e) {
        const uint64_t o = G.ring(P, r, l + 1 + e);
        P.log_term[o] = G.term[r];
        P.log_value[o] = int64_t(sm64(vb ^ uint64_t(uint32_t(e))) >> 1);
      }
      if (n_ok) { G.last[r] = l + n_ok; G.d_last |= 1u << r; }
      if (n_ok < int(E)) G.raise(F_OVERFLOW);
    });
  }

  // 2. rounds in ascending replica id, against the roles as they are now.
  const TickSrc base{P.log_term, P.log_value, P.Gp, G.g, P.K, P.kmask, 0, 1,
                     G.cache_leader, G.cache_from, G.cache_term, G.cache_vbase};
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
    if (G.role(c) == ROLE_L) G.leader_round(P, T, c, make_src);    // main.go:332-391
    else G.candidate_round(P, T, c);                               // main.go:253-284
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
    G.timeout_fire(T, best);
    if (!G.alive()) break;
    G.candidate_round(P, T, best);
  }

  if (!G.alive()) {
    ++G.st[S_FAULTS];
  } else if ((G.roles >> 1) & ~G.roles & 0x5555u) {
    ++G.st[S_LEADER_GROUPS];
  }
}

template <int R>
__global__ __launch_bounds__(256) void tick_kernel(DevPlanes P, Trace T, uint32_t E,
                                                   unsigned long long* stats) {
  const uint64_t g = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  int st[NSTAT];
#pragma unroll
  for (int s = 0; s < NSTAT; ++s) st[s] = 0;
  if (g < P.G) {
    Group<R> G;
    G.begin(P, T, g);
    if (G.fault == 0) {
      G.load(P, false);
      run_tick<R>(G, P, T, E);
      G.store(P);
#pragma unroll
      for (int s = 0; s < NSTAT; ++s) st[s] = G.st[s];
    }
  }
  if (!stats) return;
  __shared__ long long red[NSTAT][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int s = 0; s < NSTAT; ++s) {
    const long long w = wave_sum(st[s]);
    if (lane == 0) red[s][wave] = w;
  }
  __syncthreads();
  if (threadIdx.x < NSTAT) {
    const int s = threadIdx.x;
    const long long v = red[s][0] + red[s][1] + red[s][2] + red[s][3];
    if (v) atomicAdd(&stats[(blockIdx.x % STAT_SLOTS) * NSTAT + s], (unsigned long long)v);
  }
}

template <int R, typename F>
__device__ __forceinline__ void with_replica(int x, F&& f) {
  static_for<R>([&](auto PI) {
    if (x == decltype(PI)::value) f(PI);
  });
}

template <int R>
__global__ __launch_bounds__(256) void ops_kernel(DevPlanes P, Trace T, const DevOp* ops, uint32_t n,
                                                  const int32_t* et, const int64_t* ev, DevRes* out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const DevOp op = ops[i];
  DevRes res{0, 0, 0, 0, 0};
  Group<R> G;
  G.begin(P, T, op.group);
  if (G.fault) {
    res.fault = G.fault;
    out[i] = res;
    return;
  }
  G.load(P, true);
  const int x = int(op.replica);
  const int ro = G.role(x);
  const TickSrc ring_only{P.log_term, P.log_value, P.Gp, G.g, P.K, P.kmask, 0, 1, -1, 0, 0, 0};
  auto make_src = [ring_only](int c) {
    TickSrc s = ring_only;
    s.leader = c;
    return s;
  };
  switch (op.kind) {
    case OP_AE: {
      AEReq q{op.term, op.prev_idx, op.prev_term, op.lc, int(op.n)};
      HostSrc src{et, ev, op.off, 0};
      with_replica<R>(x, [&](auto PI) {
        constexpr int p = decltype(PI)::value;
        const AEResp a = G.template deliver_ae<p>(P, T, q, src);
        res.term = a.term; res.ok = a.ok; res.value = a.match;
      });
      break;
    }
    case OP_VR: {
      with_replica<R>(x, [&](auto PI) {
        constexpr int p = decltype(PI)::value;
        int rt;
        const int gr = G.template deliver_vr<p>(T, op.term, &rt);
        res.term = rt; res.ok = gr; res.value = gr;
      });
      break;
    }
    case OP_CLIENT_APPEND:
      if (ro != ROLE_L) { res.status = -22; break; }
      G.client_append_value(P, x, op.arg);
      res.value = sel(G.last, x);
      break;
    case OP_LEADER_ROUND:
      if (ro != ROLE_L) { res.status = -22; break; }
      G.leader_round(P, T, x, make_src);
      res.value = sel(G.commit, x);
      break;
    case OP_CANDIDATE_ROUND:
      if (ro != ROLE_C) { res.status = -22; break; }
      res.value = G.candidate_round(P, T, x);
      break;
    case OP_TIMEOUT:
      if (ro == ROLE_L) { res.status = -22; break; }
      G.timeout_fire(T, x);
      res.value = sel(G.term, x);
      break;
    case OP_LEADER_COMMIT: {
      if (ro != ROLE_L) { res.status = -22; break; }
      const int32_t* row = G.match_row(P, x);
      int m[R];
#pragma unroll
      for (int p = 0; p < R; ++p) m[p] = (p != x) ? row[uint64_t(p) * P.Gp + G.g] : 0;
      const int lc = sel(G.commit, x);
      const int nc = G.commit_rule(m, x, lc);
      if (nc != lc) { put(G.commit, x, nc); G.d_commit |= 1u << x; }
      res.value = nc;
      break;
    }
    default:
      res.status = -22;
  }
  G.store(P);
  res.fault = G.fault;
  if (G.fault) res.ok = 0;
  out[i] = res;
}

// NewNode (main.go:59-76) + FollowerRun entry (main.go:113-115).
template <int R>
__global__ __launch_bounds__(256) void init_new_kernel(DevPlanes P, Trace T) {
  const uint64_t g = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (g >= P.G) return;
  const uint64_t key = group_key(T.seed, P.gbase + g);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t i = uint64_t(r) * P.Gp + g;
    const int d = T.f_min + int(uint32_t(rng_k(key, r, ST_TIMER_F, uint64_t(T.tick)) >> 32) % uint32_t(T.f_span));
    P.term[i] = 0; P.last[i] = 0; P.commit[i] = 0;
    P.deadline[i] = T.now + d;
    P.rs[i] = uint16_t(ROLE_F | (uint32_t(d) << 3));
  }
  P.gmeta[g] = uint8_t(NO_PRIMARY);
}

// Post-election state (KAT-1 generalised).
template <int R>
__global__ __launch_bounds__(256) void init_steady_kernel(DevPlanes P, Trace T, int32_t leader) {
  const uint64_t g = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (g >= P.G) return;
  const uint64_t gid = P.gbase + g;
  const uint64_t key = group_key(T.seed, gid);
  const int L = leader >= 0 ? leader % R : int(uint32_t(sm64(T.seed ^ 0x1EADE5ULL ^ sm64(gid)) >> 33) % uint32_t(R));
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t i = uint64_t(r) * P.Gp + g;
    const bool isL = r == L;
    const uint64_t h = rng_k(key, r, isL ? ST_TIMER_C : ST_TIMER_F, uint64_t(T.tick));
    const int d = isL ? T.c_min + int(uint32_t(h >> 32) % uint32_t(T.c_span))
                      : T.f_min + int(uint32_t(h >> 32) % uint32_t(T.f_span));
    P.term[i] = 1; P.last[i] = 0; P.commit[i] = 0;
    P.deadline[i] = T.now + d;
    P.rs[i] = uint16_t((isL ? ROLE_L : ROLE_F) | (1u << 2) | (uint32_t(d) << 3));
    P.lmatch[i] = 0;
  }
  P.gmeta[g] = uint8_t(L);
}

// ------------------------------------------------------ host launchers ---
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

hipError_t launch_tick(int R, const DevPlanes& P, const Trace& T, uint32_t E, unsigned long long* stats,
                       hipStream_t s) {
  RAFT_DISPATCH_R(R, hipLaunchKernelGGL(tick_kernel<RR>, grid_for(P.G), dim3(256), 0, s, P, T, E, stats));
  return hipGetLastError();
}
hipError_t launch_ops(int R, const DevPlanes& P, const Trace& T, const DevOp* ops, uint32_t n,
                      const int32_t* et, const int64_t* ev, DevRes* out, hipStream_t s) {
  RAFT_DISPATCH_R(R, hipLaunchKernelGGL(ops_kernel<RR>, grid_for(n), dim3(256), 0, s, P, T, ops, n, et, ev, out));
  return hipGetLastError();
}
hipError_t launch_init_new(int R, const DevPlanes& P, const Trace& T, hipStream_t s) {
  RAFT_DISPATCH_R(R, hipLaunchKernelGGL(init_new_kernel<RR>, grid_for(P.G), dim3(256), 0, s, P, T));
  return hipGetLastError();
}
hipError_t launch_init_steady(int R, const DevPlanes& P, const Trace& T, int32_t leader, hipStream_t s) {
  RAFT_DISPATCH_R(R, hipLaunchKernelGGL(init_steady_kernel<RR>, grid_for(P.G), dim3(256), 0, s, P, T, leader));
  return hipGetLastError();
}

}  // namespace raftstep
