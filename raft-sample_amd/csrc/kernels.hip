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

#include <hip/hip_ext.h>

#include <algorithm>

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

template <int R, int SEM>
__device__ __forceinline__ void run_tick(Group<R, SEM>& G, const DevPlanes& P, const Trace& T, uint32_t E) {
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
        const int64_t v = int64_t(sm64(vb ^ uint64_t(uint32_t(e))) >> 1);
        G.ring_term(P, r, l + 1 + e) = G.term[r];
        G.ring_value(P, r, l + 1 + e) = v;
        if (P.crc_on) G.ring_crc(P, r, l + 1 + e) = crc_entry(P.crc_tab, G.term[r], v);
      }
      if (n_ok) {
        G.last[r] = l + n_ok;
        G.d_last |= 1u << r;
        at(prow(P.lterm, r, P.Gp), G.g) = G.term[r];
        if constexpr (SEM == SEM_RAFT) G.template r_grew<r>(l + n_ok);
      }
      if (n_ok < int(E)) G.raise(F_OVERFLOW);
    });
  }

  // 2. rounds in ascending replica id, against the roles as they are now.
  const TickSrc base{P.log_term, P.log_value, P.log_crc, P.crc_tab, P.crc_on, P.Gp, G.g, P.K, P.kmask, 0, 1,
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
    const long long x = red[s][0] + red[s][1] + red[s][2] + red[s][3];
    int which = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) which = (s == k) ? idx[k] : which;
    if (x) atomicAdd(&stats[(blockIdx.x % STAT_SLOTS) * NSTAT + which], (unsigned long long)x);
  }
}

// ---------------------------------------------------------------------------
// Steady-state tick (the metric path). A group qualifies when it is STEADY
// (not frozen, its only leader is its primary, every other replica a
// follower), no EXT isolation touches it this tick, and every peer's
// MatchIndex equals the leader's LastApplied (NextIndex = LastApplied+1).
// For such a group the tick is exactly: client append (main.go:327-329),
// one AppendEntries per follower carrying just this tick's entries
// (main.go:341-372 -> 121-156), the responses (main.go:375-378) and the
// commit rule (main.go:381-391). Every follower's timer is reset by its
// AppendEntries (main.go:124-127) — recorded once per group as hb = now —
// so no timer can expire. Anything else, or any condition on the way that
// would fault or need a ring read, defers the group to the general kernel
// (worklist + DEFER flag) before a single store; a DEFERred group is left
// alone until the general kernel has caught it up.
// MSYNC: after a fast tick every follower's MatchIndex equals its
// LastApplied (main.go:156 -> 376), so the row is kept implicit.
// Store policy of the fast kernel: plain (write-back L2) or write-through
// (agent-scope relaxed atomic store = global_store ... sc1, which drops the
// line from L2 so that less dirty data is left for the end-of-kernel flush).
template <bool WT, typename T>
__device__ __forceinline__ void st(T* base, uint32_t idx, T v) {
  if constexpr (WT) __hip_atomic_store(&at(base, idx), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else at(base, idx) = v;
}

template <int R, bool WT, bool CRC>
__global__ __launch_bounds__(256) void tick_fast_kernel(DevPlanes P, Trace T, unsigned long long* stats,
                                                        uint32_t* work, int32_t* work_tick, uint32_t* work_count,
                                                        int force_slow) {
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  // EXT CRC32C tables (8 KiB) staged in LDS for the stamp/verify lookups
  __shared__ uint32_t tab[CRC ? 2048 : 1];
  if constexpr (CRC) {
    const uint4* src = reinterpret_cast<const uint4*>(P.crc_tab);
    uint4* dst = reinterpret_cast<uint4*>(tab);
    dst[threadIdx.x] = src[threadIdx.x];
    dst[threadIdx.x + 256] = src[threadIdx.x + 256];
    __syncthreads();
  }
  int sv[4] = {0, 0, 0, 0};   // committed, ae_ok, ae_fail, leader_groups
  bool bail = false;
  if (g < P.G) {
    const int meta = at(P.gmeta, g);
    const int c = meta & 0xF;
    const bool skip = (meta & M_DEFER) || ((meta >> 4) & 0xF);   // pending catch-up / frozen group
    bail = !skip && (force_slow || !(meta & M_STEADY));
    int term[R], last[R], commit[R], lt[R], m[R];
    const bool go = !skip && !bail;
    if (go) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        term[r] = at(prow(P.term, r, P.Gp), g);
        last[r] = at(prow(P.last, r, P.Gp), g);
        commit[r] = at(prow(P.commit, r, P.Gp), g);
        lt[r] = at(prow(P.lterm, r, P.Gp), g);
      }
      if (meta & M_MSYNC) {
#pragma unroll
        for (int r = 0; r < R; ++r) m[r] = (r != c) ? last[r] : 0;
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) m[r] = (r != c) ? at(prow(P.lmatch, r, P.Gp), g) : 0;
      }
    }
    const int n = int(T.client_entries());
    uint64_t key = 0;
    if (go && (T.iso_p || n)) key = group_key(T.seed, P.gbase + g);
    if (go && T.iso_p) bail = isolation_mask<R>(key, T) != 0;
    // leader view
    const int Lt = sel(term, c), Ll = sel(last, c), Lc = sel(commit, c), Llt = sel(lt, c);
    if (go && !bail) bail = int64_t(Ll) + n > I32MAX || n >= int(P.K);
    if (go) {
#pragma unroll
      for (int p = 0; p < R; ++p) bail |= (p != c) && m[p] != Ll;
    }
    // one AppendEntries shape for every peer (NextIndex == Ll+1)
    int prev_idx, prev_term;
    if (n == 0 || Ll == 0) { prev_idx = Ll; prev_term = Lt; }   // heartbeat / whole-log (PrevLogIndex 0)
    else { prev_idx = Ll; prev_term = Llt; }                      // GetLog(MatchIndex).Term
    // EXT: every follower verifies the CRC32C stamp of each entry it received
    // (the term's CRC state is shared, the term bytes are never corrupted)
    uint32_t crcbad = 0;
    if constexpr (CRC) {
      if (go && !bail && n) {
        uint32_t cm = 0;   // followers whose message is corrupted this tick
#pragma unroll
        for (int p = 0; p < R; ++p)
          if (p != c && P.corrupt_p && (rng_k(key, uint32_t(p), ST_CORRUPT, uint64_t(T.tick)) & 0xFFFF) < P.corrupt_p)
            cm |= 1u << p;
        const uint64_t vb = rng_k(key, uint32_t(c), ST_VALUE, uint64_t(T.tick));
        const uint32_t cs = crc_term_state(tab, Lt);
        for (int e = 0; e < n; ++e) {
          const int64_t v = int64_t(sm64(vb ^ uint64_t(uint32_t(e))) >> 1);
          const uint32_t stamp = crc_value_final(tab, cs, v);               // leader's stamp
#pragma unroll
          for (int p = 0; p < R; ++p) {
            if (p == c) continue;
            const int64_t rv = v ^ ((((cm >> p) & 1u) && e == n - 1) ? 1 : 0);  // what p received
            if (crc_value_final(tab, cs, rv) != stamp) crcbad |= 1u << p;
          }
        }
      }
    }
    uint32_t okm = 0, cch = 0, mch = 0, ltch = 0;
    if (go && !bail) {
#pragma unroll
      for (int p = 0; p < R; ++p) {
        if (p == c) continue;
        bool ok = Lt >= term[p];                                  // main.go:129-133
        const int l = last[p];
        if (ok && l > 0) {                                        // main.go:135
          if (int64_t(l) + n < prev_idx) ok = false;              // 137-140
          else if (prev_idx < 1 || prev_idx > l || prev_idx <= l - int(P.K) || prev_idx != l) bail = true;
          else ok = lt[p] == prev_term;                           // 142-145 (GetLog(l) == last entry)
        }
        if (ok && int64_t(l) + n > I32MAX) bail = true;
        if (ok && ((crcbad >> p) & 1u)) ok = false;               // EXT: payload rejected
        if (ok) {
          const int nl = l + n;                                   // 148-149
          last[p] = nl;
          if (n && lt[p] != Lt) ltch |= 1u << p;
          if (Lc > commit[p]) {                                   // 151-152
            const int nc = Lc < nl + 1 ? Lc : nl + 1;
            if (nc != commit[p]) { commit[p] = nc; cch |= 1u << p; }
          }
          if (nl != m[p]) { m[p] = nl; mch |= 1u << p; }          // 156 -> 375-377
          okm |= 1u << p;
        }
      }
    }
    if (go && !bail) {
      // commit rule (main.go:381-391)
      int cm = Lc;
      bool sync = true;
#pragma unroll
      for (int p = 0; p < R; ++p) {
        int cnt = 0;
#pragma unroll
        for (int q = 0; q < R; ++q) cnt += (q != c && m[q] == m[p]) ? 1 : 0;
        if (p != c && 2 * cnt > R && m[p] > cm) cm = m[p];
        sync &= (p == c) || m[p] == last[p];
      }
      sv[0] = cm - Lc;
      sv[1] = __builtin_popcount(okm);
      sv[2] = (R - 1) - sv[1];
      sv[3] = 1;
      // ---- stores (no bail past this point) ----
      if (n) {
        st<WT>(P.last + uint64_t(c) * P.Gp, g, Ll + n);
        if (Llt != Lt) st<WT>(P.lterm + uint64_t(c) * P.Gp, g, Lt);
      }
      if (cm != Lc) st<WT>(P.commit + uint64_t(c) * P.Gp, g, cm);
      st<WT>(P.hb, g, T.now);                                     // timer.Reset(d) of every follower
#pragma unroll
      for (int p = 0; p < R; ++p) {
        if (p == c || !((okm >> p) & 1u)) continue;
        if (n) st<WT>(prow(P.last, p, P.Gp), g, last[p]);
        if (!sync && ((mch >> p) & 1u)) st<WT>(prow(P.lmatch, p, P.Gp), g, m[p]);
        if ((cch >> p) & 1u) st<WT>(prow(P.commit, p, P.Gp), g, commit[p]);
        if ((ltch >> p) & 1u) st<WT>(prow(P.lterm, p, P.Gp), g, Lt);
        if (term[p] != Lt) st<WT>(prow(P.term, p, P.Gp), g, Lt);  // main.go:155
      }
      const int nm = sync ? (meta | M_MSYNC) : (meta & ~M_MSYNC);
      if (nm != meta) at(P.gmeta, g) = uint16_t(nm);
      // this tick's entries: leader log + every follower that accepted
      if (n) {
        const uint64_t vb = rng_k(key, uint32_t(c), ST_VALUE, uint64_t(T.tick));
        const uint64_t cb = uint64_t(c) * P.K * P.Gp;
        uint32_t cs = 0;
        if constexpr (CRC) cs = crc_term_state(tab, Lt);
        for (int e = 0; e < n; ++e) {
          const int64_t v = int64_t(sm64(vb ^ uint64_t(uint32_t(e))) >> 1);
          const uint32_t o = uint32_t((Ll + e) & int(P.kmask)) * uint32_t(P.Gp) + g;
          uint32_t stamp = 0;
          if constexpr (CRC) stamp = crc_value_final(tab, cs, v);
          st<WT>(P.log_term + cb, o, Lt);
          st<WT>(P.log_value + cb, o, v);
          if constexpr (CRC) st<WT>(P.log_crc + cb, o, stamp);
#pragma unroll
          for (int p = 0; p < R; ++p) {
            if (p == c || !((okm >> p) & 1u)) continue;
            const uint32_t op = uint32_t((last[p] - n + e) & int(P.kmask)) * uint32_t(P.Gp) + g;
            const uint64_t pb = uint64_t(p) * P.K * P.Gp;
            st<WT>(P.log_term + pb, op, Lt);
            st<WT>(P.log_value + pb, op, v);
            if constexpr (CRC) st<WT>(P.log_crc + pb, op, stamp);
          }
        }
      }
    }
    if (bail) at(P.gmeta, g) = uint16_t(meta | M_DEFER);
  }
  // groups that need the general path go to the worklist (one atomic per wave)
  const uint64_t bm = __ballot(bail);
  if (bm) {
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == __builtin_ctzll(bm)) base = atomicAdd(work_count, uint32_t(__popcll(bm)));
    base = __shfl(base, __builtin_ctzll(bm));
    if (bail) {
      const uint32_t slot = base + uint32_t(__popcll(bm & ((1ull << lane) - 1ull)));
      work[slot] = g;
      work_tick[slot] = int32_t(T.tick);
    }
  }
  if (stats) {
    const int idx[4] = {S_COMMITTED, S_AE_OK, S_AE_FAIL, S_LEADER_GROUPS};
    block_stats<4>(sv, idx, stats);
  }
}

// General tick over the worklist: every deferred group is caught up, tick
// by tick in order, from the tick it was deferred at to `last_tick`, with
// the full REF semantics of run_tick() (elections, candidates, step-downs,
// faults, EXT drops); stats go to each tick's own record.
template <int R, int SEM>
__global__ __launch_bounds__(256) void tick_slow_kernel(DevPlanes P, Trace T0, int64_t first_tick, int64_t last_tick,
                                                        unsigned long long* stats, const uint32_t* work,
                                                        const int32_t* work_tick, const uint32_t* work_count,
                                                        uint32_t* next_count) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *next_count = 0;
  const uint32_t n = *work_count;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    const uint32_t g = work[i];
    for (int64_t t = work_tick[i]; t <= last_tick; ++t) {
      const Trace T = T0.at_tick(t);
      Group<R, SEM> G;
      G.begin(P, T, g);
      if (G.fault) {            // frozen earlier in this catch-up
        if (G.meta0 & M_DEFER) at(P.gmeta, g) = uint16_t(G.meta0 & ~M_DEFER);
        break;
      }
      G.load(P, false);
      run_tick<R, SEM>(G, P, T, T.client_entries());
      G.store(P);
      if (stats) {
        unsigned long long* rec = stats + size_t(t - first_tick) * STAT_SLOTS * NSTAT + (g % STAT_SLOTS) * NSTAT;
#pragma unroll
        for (int s = 0; s < NSTAT; ++s)
          if (G.st[s]) atomicAdd(&rec[s], (unsigned long long)G.st[s]);
      }
    }
  }
}

template <int R, typename F>
__device__ __forceinline__ void with_replica(int x, F&& f) {
  static_for<R>([&](auto PI) {
    if (x == decltype(PI)::value) f(PI);
  });
}

template <int R, int SEM>
__global__ __launch_bounds__(256) void ops_kernel(DevPlanes P, Trace T, const DevOp* ops, uint32_t n,
                                                  const int32_t* et, const int64_t* ev, const uint32_t* ec,
                                                  DevRes* out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const DevOp op = ops[i];
  DevRes res{0, 0, 0, 0, 0};
  Group<R, SEM> G;
  G.begin(P, T, uint32_t(op.group));
  if (G.fault) {
    res.fault = G.fault;
    out[i] = res;
    return;
  }
  G.load(P, true);
  const int x = int(op.replica);
  const int ro = G.role(x);
  const TickSrc ring_only{P.log_term, P.log_value, P.log_crc, P.crc_tab, P.crc_on, P.Gp, G.g, P.K, P.kmask, 0, 1,
                          -1, 0, 0, 0};
  auto make_src = [ring_only](int c) {
    TickSrc s = ring_only;
    s.leader = c;
    return s;
  };
  switch (op.kind) {
    case OP_AE: {
      AEReq q{op.term, op.prev_idx, op.prev_term, op.lc, int(op.n), 0};
      HostSrc src{et, ev, ec, op.off, 0};
      with_replica<R>(x, [&](auto PI) {
        constexpr int p = decltype(PI)::value;
        AEResp a;
        if constexpr (SEM == SEM_RAFT) a = G.template r_deliver_ae<p>(P, T, q, src);
        else a = G.template deliver_ae<p>(P, T, q, src);
        res.term = a.term; res.ok = a.ok; res.value = a.match;
      });
      break;
    }
    case OP_VR: {
      with_replica<R>(x, [&](auto PI) {
        constexpr int p = decltype(PI)::value;
        int rt;
        int gr;
        // RAFT: CandidateId = arg, LastLogIndex = prev_idx, LastLogTerm = prev_term
        if constexpr (SEM == SEM_RAFT) gr = G.template r_deliver_vr<p>(P, T, op.term, int(op.arg), op.prev_idx, op.prev_term, &rt);
        else gr = G.template deliver_vr<p>(T, op.term, &rt);
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
      if constexpr (SEM == SEM_RAFT) G.r_leader_round(P, T, x, make_src);
      else G.leader_round(P, T, x, make_src);
      res.value = sel(G.commit, x);
      break;
    case OP_CANDIDATE_ROUND:
      if (ro != ROLE_C) { res.status = -22; break; }
      if constexpr (SEM == SEM_RAFT) res.value = G.r_candidate_round(P, T, x);
      else res.value = G.candidate_round(P, T, x);
      break;
    case OP_TIMEOUT:
      if (ro == ROLE_L) { res.status = -22; break; }
      if constexpr (SEM == SEM_RAFT) G.r_timeout_fire(T, x);
      else G.timeout_fire(T, x);
      res.value = sel(G.term, x);
      break;
    case OP_LEADER_COMMIT: {
      if (ro != ROLE_L) { res.status = -22; break; }
      int m[R];
      G.load_match(P, x, m);
      const int lc = sel(G.commit, x);
      int nc;
      if constexpr (SEM == SEM_RAFT) nc = G.r_commit_rule(P, m, x, lc);
      else nc = G.commit_rule(m, x, lc);
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
    P.tstart[i] = T.now;
    P.rs[i] = uint16_t(ROLE_F | (uint32_t(d) << 6));   // vote 0 (REF: not voted; RAFT: votedFor none)
    P.lterm[i] = 0;
    if (P.hwm) P.hwm[i] = 0;
  }
  P.hb[g] = HB_NONE;
  P.gmeta[g] = uint16_t(NO_PRIMARY);
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
    // REF: Voted = true; RAFT: everyone voted for L (votedFor + 1)
    const uint32_t vote = P.hwm ? uint32_t(L + 1) : 1u;
    P.term[i] = 1; P.last[i] = 0; P.commit[i] = 0;
    P.tstart[i] = T.now;
    P.rs[i] = uint16_t((isL ? ROLE_L : ROLE_F) | (vote << 2) | (uint32_t(d) << 6));
    P.lmatch[i] = 0;
    P.lterm[i] = 0;
    if (P.hwm) {                       // RAFT mode: NextIndex = last + 1 = 1, high-water 0
      P.lnext[i] = 1;
      P.hwm[i] = 0;
    }
  }
  P.hb[g] = HB_NONE;
  P.gmeta[g] = uint16_t(L | (P.hwm ? 0 : M_MSYNC) | M_STEADY);
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

template <int R, bool WT, bool CRC>
static void launch_fast_t(const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* work,
                          int32_t* work_tick, uint32_t* work_count, int force_slow, hipStream_t s, hipEvent_t a,
                          hipEvent_t b) {
  hipExtLaunchKernelGGL(tick_fast_kernel<R, WT, CRC>, grid_for(P.G), dim3(256), 0, s, a, b, 0, P, T, stats, work,
                        work_tick, work_count, force_slow);
}
hipError_t launch_tick_fast(int R, const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* work,
                            int32_t* work_tick, uint32_t* work_count, int force_slow, int write_through, hipStream_t s,
                            hipEvent_t ev_start, hipEvent_t ev_stop) {
  const bool crc = P.crc_on != 0;
#define RAFT_FAST(WT_, CRC_) \
  RAFT_DISPATCH_R(R, (launch_fast_t<RR, WT_, CRC_>(P, T, stats, work, work_tick, work_count, force_slow, s, ev_start, ev_stop)))
  if (write_through) {
    if (crc) { RAFT_FAST(true, true); } else { RAFT_FAST(true, false); }
  } else {
    if (crc) { RAFT_FAST(false, true); } else { RAFT_FAST(false, false); }
  }
#undef RAFT_FAST
  return hipGetLastError();
}
hipError_t launch_tick_slow(int R, int sem, const DevPlanes& P, const Trace& T0, int64_t first_tick, int64_t last_tick,
                            unsigned long long* stats, const uint32_t* work, const int32_t* work_tick,
                            const uint32_t* work_count, uint32_t* next_count, hipStream_t s) {
  const unsigned blocks = unsigned(std::min<uint64_t>((P.G + 255) / 256, 1024));
  if (sem == SEM_RAFT) {
    RAFT_DISPATCH_R(R, hipLaunchKernelGGL((tick_slow_kernel<RR, SEM_RAFT>), dim3(blocks), dim3(256), 0, s, P, T0,
                                          first_tick, last_tick, stats, work, work_tick, work_count, next_count));
  } else {
    RAFT_DISPATCH_R(R, hipLaunchKernelGGL((tick_slow_kernel<RR, SEM_REF>), dim3(blocks), dim3(256), 0, s, P, T0,
                                          first_tick, last_tick, stats, work, work_tick, work_count, next_count));
  }
  return hipGetLastError();
}
hipError_t launch_ops(int R, int sem, const DevPlanes& P, const Trace& T, const DevOp* ops, uint32_t n,
                      const int32_t* et, const int64_t* ev, const uint32_t* ec, DevRes* out, hipStream_t s) {
  if (sem == SEM_RAFT) {
    RAFT_DISPATCH_R(R, hipLaunchKernelGGL((ops_kernel<RR, SEM_RAFT>), grid_for(n), dim3(256), 0, s, P, T, ops, n, et,
                                          ev, ec, out));
  } else {
    RAFT_DISPATCH_R(R, hipLaunchKernelGGL((ops_kernel<RR, SEM_REF>), grid_for(n), dim3(256), 0, s, P, T, ops, n, et,
                                          ev, ec, out));
  }
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
