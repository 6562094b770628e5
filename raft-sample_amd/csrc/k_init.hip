// k_init.hip — NewNode / post-election initialisation kernels and the
// semantics dispatch of the general and handler launchers.
#include "tick_common.hpp"

namespace raftstep {

// NewNode (main.go:59-76) + FollowerRun entry (main.go:113-115).
template <int R>
__global__ __launch_bounds__(256) void init_new_kernel(DevPlanes P, Trace T) {
  const uint64_t g = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  if (g >= P.G) return;
  const uint64_t key = group_key(T.seed, P.gbase + g);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t i = rix<R>(uint32_t(g), r);   // group record (rix)
    const int d = T.f_min + int(uint32_t(rng_k(key, r, ST_TIMER_F, uint64_t(T.tick)) >> 32) % uint32_t(T.f_span));
    P.term[i] = 0; P.last[i] = 0; P.commit[i] = 0;
    P.tstart[i] = T.now;
    P.rs[i] = int32_t(ROLE_F | (uint32_t(d) << 6));   // vote 0 (REF: not voted; RAFT: votedFor none)
    P.lterm[i] = 0;
    P.lmatch[i] = 0;
    if (P.hwm) P.hwm[i] = 0;
  }
  P.hb[g] = HB_NONE;
  P.gmeta[g] = uint16_t(NO_PRIMARY);
  P.giso[g] = 0;
  P.grot[g] = 0;   // empty logs: the phase is chosen at the first append
  P.grota[g] = 0;
  P.gsb[g] = 0;
  P.grotb[g] = 0;
  P.gsb2[g] = 0;
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
    const uint32_t i = rix<R>(uint32_t(g), r);   // group record (rix)
    const bool isL = r == L;
    const uint64_t h = rng_k(key, r, isL ? ST_TIMER_C : ST_TIMER_F, uint64_t(T.tick));
    const int d = isL ? T.c_min + int(uint32_t(h >> 32) % uint32_t(T.c_span))
                      : T.f_min + int(uint32_t(h >> 32) % uint32_t(T.f_span));
    // REF: Voted = true; RAFT: everyone voted for L (votedFor + 1)
    const uint32_t vote = P.hwm ? uint32_t(L + 1) : 1u;
    P.term[i] = 1; P.last[i] = 0; P.commit[i] = 0;
    P.tstart[i] = T.now;
    P.rs[i] = int32_t((isL ? ROLE_L : ROLE_F) | (vote << 2) | (uint32_t(d) << 6));
    P.lmatch[i] = 0;
    P.lterm[i] = 0;
    if (P.hwm) {                       // RAFT mode: NextIndex = last + 1 = 1, high-water 0
      P.lnext[i] = 1;
      P.hwm[i] = 0;
    }
  }
  P.hb[g] = HB_NONE;
  P.giso[g] = 0;
  P.gmeta[g] = uint16_t(L | (P.hwm ? 0 : M_MSYNC) | M_STEADY);
  P.grot[g] = uint16_t(T.entries_before(T.tick + 1) & P.kmask);   // entry 1 lands in the global phase
  P.grota[g] = 0;
  P.gsb[g] = 0;
  P.grotb[g] = 0;
  P.gsb2[g] = 0;
}

// State digest (raft_state_digest): one lane per group derives the canonical
// host view exactly as raft_store_state does (implicit MSYNC rows, heartbeat
// timer starts, REF NextIndex = MatchIndex+1) and chains it through
// splitmix64; the per-group digests are summed with one atomic per wave.
// Same definition as oracle_state_digest().
__device__ __forceinline__ uint64_t dg_mix(uint64_t h, uint64_t w) { return sm64(h ^ w); }
__device__ __forceinline__ uint64_t lo32(int v) { return uint64_t(uint32_t(v)); }

template <int R>
__global__ __launch_bounds__(256) void digest_kernel(DevPlanes P, int raft, uint64_t* per_group,
                                                     unsigned long long* total) {
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  uint64_t h = 0;
  if (g < P.G) {
    const int meta = at(P.gmeta, g);
    const int primary = meta & 0xF, fault = (meta >> 4) & 7;
    const bool msync = (meta & M_MSYNC) && primary < R;
    const bool ssync = (meta & M_SSYNC) && primary < R;   // compressed state: the gss record
    const SsRec ss = ssync ? P.gss[g] : SsRec{0, 0, 0, 0};
    const LxRec lx = (ssync && uses_glx(meta)) ? P.glx[g] : LxRec{0, 0};
    const int hb = (P.sh && (at(P.grot, g) & ROT_SH)) ? P.sh_hb : at(P.hb, g);   // (SH: implied)
    int last[R];
#pragma unroll
    for (int r = 0; r < R; ++r) last[r] = ssync ? ss_last(ss, r, primary, meta, lx) : at(P.last, rix<R>(g, r));
    h = sm64(0x5241465444494721ULL ^ (P.gbase + g));
#pragma unroll 1
    for (int r = 0; r < R; ++r) {
      const uint32_t x = at(P.rs, rix<R>(g, r));
      const int role = int(x & 3u), dur = int(x >> 6);
      const int l = sel(last, r);
      const int ts = at(P.tstart, rix<R>(g, r));
      const int dl = (role == ROLE_L ? ts : max(ts, hb)) + dur;
      // MSYNC: max(plane, LastApplied) (HWX; the plane is at most LastApplied without it)
      const int hwm = raft ? (msync ? max(at(P.hwm, rix<R>(g, r)), l) : at(P.hwm, rix<R>(g, r))) : l;
      h = dg_mix(h, uint64_t(role) | (uint64_t((x >> 2) & 15u) << 8) | (uint64_t(r) << 16));
      const int tm = ssync ? ss_term(ss, r, meta, lx) : at(P.term, rix<R>(g, r));
      const int cm = ssync ? ss_commit(ss, r, primary, meta, lx, at(P.commit, rix<R>(g, r))) : at(P.commit, rix<R>(g, r));
      h = dg_mix(h, lo32(tm) | (lo32(l) << 32));
      h = dg_mix(h, lo32(cm) | (lo32(dl) << 32));
      h = dg_mix(h, lo32(dur) | (lo32(hwm) << 32));
#pragma unroll 1
      for (int p = 0; p < R; ++p) {
        int m = 0, nx = 0;
        if (role == ROLE_L && p != r) {
          const int lp = sel(last, p);
          const bool mp = msync && msync_peer(meta, lx, p);   // (SXS: the stale leader's row is explicit)
          if (r == primary) m = mp ? lp : at(P.lmatch, rix<R>(g, p));
          else m = at(prow(P.xmatch, r * R + p, P.Gp), g);
          if (!raft) nx = m + 1;
          else if (r == primary) nx = mp ? lp + 1 : at(P.lnext, rix<R>(g, p));
          else nx = at(prow(P.xnext, r * R + p, P.Gp), g);
        }
        h = dg_mix(h, lo32(m) | (lo32(nx) << 32));
      }
      const uint64_t rb = ring_tile(g, P.KP, R);
      const uint32_t rot = at(P.grot, g), rota = at(P.grota, g), rotb = at(P.grotb, g);
      const int sb = at(P.gsb, g), sb2 = at(P.gsb2, g);
      // SH (ROT_SH): entries from shf on are read from the shared ring (the
      // digest of the materialised state, without materialising it)
      const int shf = (P.sh && (rot & ROT_SH)) ? at(P.gshf, g) : 2147483647;
      const uint64_t shb = sh_tile(g, P.KP);
#pragma unroll 1
      for (int idx = hwm > int(P.K) ? hwm - int(P.K) + 1 : 1; idx <= l; ++idx) {
        const uint32_t slot = ring_slot(idx, rot, rota, rotb, sb, sb2, P.kmask);
        int32_t lt;
        int64_t lv;
        uint32_t lc = 0;
        if (idx >= shf) {
          const uint32_t so = sh_in_tile(g, slot, P.sh_cs);
          lt = at(P.sh_term + shb, so);
          lv = at(P.sh_value + shb, so);
          if (P.crc_on) lc = at(P.sh_crc + shb, so);
        } else {
          const uint32_t o = ring_in_tile(g, R, slot, uint32_t(r));
          lt = at(P.log_term + rb, o);
          lv = at(P.log_value + rb, o);
          if (P.crc_on) lc = at(P.log_crc + rb, o);
        }
        h = dg_mix(h, lo32(lt) | (lo32(idx) << 32));
        h = dg_mix(h, uint64_t(lv));
        h = dg_mix(h, P.crc_on ? uint64_t(lc) : 0ull);
      }
    }
    h = dg_mix(h, uint64_t(fault));
    const uint32_t gi = at(P.giso, g);
    if (gi) h = dg_mix(h, 0x1500u | gi);   // EXT leader-isolation victims (absent: digest unchanged)
    per_group[g] = h;
  }
  // wrapping 64-bit sum: two 32-bit halves through the shuffle tree
  unsigned long long x = h;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  if ((threadIdx.x & 63) == 0 && x) atomicAdd(total, x);
}

// Per-tick statistics: the STAT_SLOTS x NSTAT atomic slots of each tick in
// [0, nt) are summed into out[t][NSTAT] (the 64-B record the multi-GPU
// all-reduce carries) and zeroed for the next raft_tick call, so the atomic
// targets never need a memset on the critical path. One 64-lane block per
// tick; lane = slot.
// With a CallCheck, one more block (the last) writes the end-of-call check
// record: the groups the lean kernel passed to the list at the call's last
// tick (every list's counters), the groups the last general window took, and —
// in a list-skipping call, where no list kernel consumed or zeroed them — the
// list counters are zeroed so a later list kernel never reads stale entries.
__device__ __forceinline__ void call_check_block(const CallCheck& c) {
  uint64_t listed = 0, deferred = 0, last = 0;
  if (threadIdx.x < uint32_t(NSHARD)) {
    const uint32_t k = threadIdx.x * SHARD_STRIDE;
    for (int q = 0; q < NLISTS; ++q) {
      const uint64_t n = c.wcount[(NWORK + q) * SHARD_WORDS + k];
      listed += n;
      if (q == c.llast) last = n;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    listed += __shfl_xor(listed, o);
    last += __shfl_xor(last, o);
  }
  // what the last window tail took (its counters are zeroed by then); a
  // list-skipping call defers nothing and runs no tail
  deferred = c.zero_lists ? 0u : c.wcount[WC_TAKEN + c.wlast];
  __syncthreads();   // every lane has read the counters before any is zeroed
  if (c.zero_lists && threadIdx.x < uint32_t(NSHARD))
    for (int q = 0; q < NLISTS; ++q) c.wcount[(NWORK + q) * SHARD_WORDS + threadIdx.x * SHARD_STRIDE] = 0u;
  if (threadIdx.x < NSTAT) {
    const unsigned long long v = threadIdx.x == CHK_LISTED ? listed : threadIdx.x == CHK_DEFERRED ? deferred
                                 : threadIdx.x == CHK_LAST_LIST ? last
                                 : threadIdx.x == CHK_MAGIC ? 0x5241465443484Bull : 0ull;
    c.out[threadIdx.x] = v;
    if (c.hout) c.hout[size_t(blockIdx.x) * NSTAT + threadIdx.x] = v;   // (the check block is the launch's last index)
  }
}

// Host mirror completion (CallCheck::hdone): every block's writes are made
// visible system-wide, then the last block to finish publishes the call's
// sequence number.
__device__ __forceinline__ void host_mirror_done(const CallCheck& c) {
  if (!c.hout) return;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(c.ctr, 1u) == gridDim.x - 1) {
    *c.ctr = 0u;
    __threadfence_system();
    __hip_atomic_store(c.hdone, c.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Window tail: after the general kernel has caught the window's deferred
// groups up, their DEFER flags are cleared here (the general kernel keeps
// them, so that it can run beside the next tick's fast kernels, which leave
// DEFER groups alone), the total is kept for the check record, and the last
// block to finish zeroes the window's worklist counters for the window after
// next (its parity's next use).
__global__ __launch_bounds__(256) void window_tail_kernel(uint16_t* gmeta, const uint32_t* work, uint32_t scap,
                                                          uint32_t* wcount, int parity) {
  __shared__ uint32_t pre[NSHARD + 1];
  __shared__ bool last;
  uint32_t* cnt = wcount + parity * SHARD_WORDS;
  const uint32_t n = shard_prefix(cnt, pre);
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    const uint32_t g = work[shard_locate(pre, scap, i)];
    const uint16_t m = at(gmeta, g);
    if (m & M_DEFER) at(gmeta, g) = uint16_t(m & ~M_DEFER);
  }
  __syncthreads();   // every thread of the block has read the counters
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(&wcount[WC_DONE], 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last) {
    if (threadIdx.x < uint32_t(NSHARD)) cnt[threadIdx.x * SHARD_STRIDE] = 0u;
    if (threadIdx.x == 0) {
      wcount[WC_TAKEN + parity] = n;
      wcount[WC_DONE] = 0u;
    }
  }
}
hipError_t launch_window_tail(const DevPlanes& P, const uint32_t* work, uint32_t* wcount, int parity, hipStream_t s) {
  hipLaunchKernelGGL(window_tail_kernel, dim3(64), dim3(256), 0, s, P.gmeta, work, P.scap, wcount, parity);
  return hipGetLastError();
}

__global__ __launch_bounds__(64) void stats_reduce_kernel(unsigned long long* hist, unsigned long long* out,
                                                          uint32_t nticks, LeanBase lb, CallCheck chk) {
  static_assert(STAT_SLOTS == 64, "one lane per slot");
  if (blockIdx.x == nticks) {
    call_check_block(chk);
    host_mirror_done(chk);
    return;
  }
  unsigned long long* h = hist + size_t(blockIdx.x) * STAT_TICK + threadIdx.x * NSTAT;
  unsigned long long v[NSTAT];
#pragma unroll
  for (int s = 0; s < NSTAT; ++s) {
    v[s] = h[s];
    h[s] = 0ull;
  }
  // the lean / fused kernels' exception sums (tick_common.hpp lean_stats):
  // this lane's STAT_PKS / 64 slots
  // (none without a base: the lean kernel then counts absolutely)
  unsigned long long dc = 0, nn = 0, nl = 0, ns = 0;
#pragma unroll 4
  for (int j = 0; j < (lb.G ? STAT_PKS / 64 : 0); ++j) {
    unsigned long long* pk = hist + size_t(blockIdx.x) * STAT_TICK + STAT_PK + (threadIdx.x + 64u * j) * 8;
    const unsigned long long w0 = pk[0], w1 = pk[1];
    if (w0 | w1) {
      pk[0] = 0ull;
      pk[1] = 0ull;
    }
    dc += w0;   // (two's complement: the sum of signed differences)
    nn += w1 & 0x1FFFFFull;
    nl += (w1 >> 21) & 0x1FFFFFull;
    ns += w1 >> 42;
  }
  {   // the base (lane 0, once per tick): every live group a normal tick with the tick's base commits;
      // the differences wrap in unsigned arithmetic and the tick's totals are exact
    const int64_t t = lb.t0 + int64_t(blockIdx.x);
    const uint32_t n = (lb.period && t % int64_t(lb.period) == 0) ? lb.E : 0u;
    const unsigned long long R = lb.R, base = threadIdx.x == 0 ? lb.G : 0ull;
    v[S_COMMITTED] += base * (unsigned long long)lean_base_committed(int(lb.raft), int(lb.R), n) + dc;
    v[S_AE_OK] += (base - nn) * (R - 1u) + (R >= 2u ? ns * (R - 2u) : 0ull);
    v[S_AE_FAIL] += nl * (R - 1u) + ns * R;
    v[S_LEADER_GROUPS] += base - nn + nl + ns;
  }
#pragma unroll
  for (int s = 0; s < NSTAT; ++s)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[s] += __shfl_xor(v[s], o);
  if (threadIdx.x < NSTAT) {
    unsigned long long x = 0;
#pragma unroll
    for (int s = 0; s < NSTAT; ++s) x = (int(threadIdx.x) == s) ? v[s] : x;
    out[size_t(blockIdx.x) * NSTAT + threadIdx.x] = x;
    if (chk.hout) chk.hout[size_t(blockIdx.x) * NSTAT + threadIdx.x] = x;
  }
  host_mirror_done(chk);
}
hipError_t launch_stats_reduce(unsigned long long* hist, unsigned long long* out, uint32_t nticks, const LeanBase& lb,
                               hipStream_t s, const CallCheck* chk) {
  const uint32_t blocks = nticks + (chk ? 1u : 0u);
  if (!blocks) return hipSuccess;
  hipLaunchKernelGGL(stats_reduce_kernel, dim3(blocks), dim3(64), 0, s, hist, out, chk ? nticks : 0xFFFFFFFFu, lb,
                     chk ? *chk : CallCheck{});
  return hipGetLastError();
}

hipError_t launch_tick_slow_ref(int R, const DevPlanes& P, const Trace& T0, int64_t first_tick, int64_t win_first, int64_t last_tick,
                                unsigned long long* stats, const uint32_t* work, const int32_t* work_tick,
                                const uint32_t* work_count, uint32_t* next_count, int lane_per_group, hipStream_t s);
hipError_t launch_tick_slow_raft(int R, const DevPlanes& P, const Trace& T0, int64_t first_tick, int64_t win_first, int64_t last_tick,
                                 unsigned long long* stats, const uint32_t* work, const int32_t* work_tick,
                                 const uint32_t* work_count, uint32_t* next_count, int lane_per_group, hipStream_t s);
hipError_t launch_ops_ref(int R, const DevPlanes& P, const Trace& T, const DevOp* ops, uint32_t n, const int32_t* et,
                          const int64_t* ev, const uint32_t* ec, DevRes* out, hipStream_t s);
hipError_t launch_ops_raft(int R, const DevPlanes& P, const Trace& T, const DevOp* ops, uint32_t n, const int32_t* et,
                           const int64_t* ev, const uint32_t* ec, DevRes* out, hipStream_t s);

hipError_t launch_tick_slow(int R, int sem, const DevPlanes& P, const Trace& T0, int64_t first_tick, int64_t win_first, int64_t last_tick,
                            unsigned long long* stats, const uint32_t* work, const int32_t* work_tick,
                            const uint32_t* work_count, uint32_t* next_count, int lane_per_group, hipStream_t s) {
  return sem == SEM_RAFT
             ? launch_tick_slow_raft(R, P, T0, first_tick, win_first, last_tick, stats, work, work_tick, work_count, next_count,
                                     lane_per_group, s)
             : launch_tick_slow_ref(R, P, T0, first_tick, win_first, last_tick, stats, work, work_tick, work_count, next_count,
                                    lane_per_group, s);
}
hipError_t launch_ops(int R, int sem, const DevPlanes& P, const Trace& T, const DevOp* ops, uint32_t n,
                      const int32_t* et, const int64_t* ev, const uint32_t* ec, DevRes* out, hipStream_t s) {
  return sem == SEM_RAFT ? launch_ops_raft(R, P, T, ops, n, et, ev, ec, out, s)
                         : launch_ops_ref(R, P, T, ops, n, et, ev, ec, out, s);
}
hipError_t launch_init_new(int R, const DevPlanes& P, const Trace& T, hipStream_t s) {
  RAFT_DISPATCH_R(R, hipLaunchKernelGGL(init_new_kernel<RR>, grid_for(P.G), dim3(256), 0, s, P, T));
  return hipGetLastError();
}
hipError_t launch_init_steady(int R, const DevPlanes& P, const Trace& T, int32_t leader, hipStream_t s) {
  RAFT_DISPATCH_R(R, hipLaunchKernelGGL(init_steady_kernel<RR>, grid_for(P.G), dim3(256), 0, s, P, T, leader));
  return hipGetLastError();
}
hipError_t launch_digest(int R, const DevPlanes& P, int raft, uint64_t* per_group, unsigned long long* total,
                         hipStream_t s) {
  RAFT_DISPATCH_R(R, hipLaunchKernelGGL(digest_kernel<RR>, grid_for(P.G), dim3(256), 0, s, P, raft, per_group, total));
  return hipGetLastError();
}

// Stream probe (measurement only; no Raft state): the steady lean kernel's
// byte mix and access shape on fresh buffers of n elements. Per element it
// reads 2 + 16 + 2 B (gmeta, the 16-B record, the ring rotation) in one round
// trip and writes the record 16 B, the heartbeat 4 B and R entries of 12 B as
// whole ring rows (a wave's 64 elements x R contiguous per plane, streaming
// stores to the slot `slot` of `kslots`) — 20 + 20 + 12 R B, 100 B at R = 5.
// bench.py times it on the same GPU as the lean kernel, so the lean kernel's
// rate can be read against what this device sustains for that pattern.
template <int R>
__global__ __launch_bounds__(256) void stream_probe_kernel(const uint16_t* a, SsRec* b, const uint16_t* c, int32_t* d,
                                                           int32_t* rt, int64_t* rv, uint32_t n, uint32_t slot,
                                                           uint32_t kslots, uint32_t mode) {
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  SsRec s{0, 0, 0, 0};
  uint32_t x = 0;
  if (g < n) {
    x = uint32_t(a[g]) ^ (uint32_t(c[g]) << 16);
    s = b[g];
  }
  const int lane = int(threadIdx.x & 63u);
  const uint64_t tb = (uint64_t(g >> 6) * kslots + slot) * 64u * R;
  const int32_t v32 = s.term ^ int32_t(x);
  const int64_t v64 = (int64_t(s.last) << 32) ^ int64_t(uint32_t(s.cl) + x);
  const int vlo = int(uint32_t(uint64_t(v64))), vhi = int(uint32_t(uint64_t(v64) >> 32));
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int src = (k * 64 + lane) / R;
    const int t = __shfl(v32, src), lo = __shfl(vlo, src), hi = __shfl(vhi, src);
    const int64_t val = int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo));
    if (mode & 1u) {   // (mode bit 0: plain ring stores)
      rt[tb + uint64_t(k * 64 + lane)] = t;
      rv[tb + uint64_t(k * 64 + lane)] = val;
    } else {
      __builtin_nontemporal_store(t, &rt[tb + uint64_t(k * 64 + lane)]);
      __builtin_nontemporal_store(val, &rv[tb + uint64_t(k * 64 + lane)]);
    }
  }
  if (g < n) {
    if (mode & 2u) {   // (mode bit 1: non-temporal record / heartbeat stores)
      typedef int32_t i4 __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(i4{s.last + 1, s.term, s.cl + 1, s.cf + 1}, reinterpret_cast<i4*>(&b[g]));
      if (!(mode & 4u)) __builtin_nontemporal_store(int32_t(s.term + int32_t(slot)), &d[g]);
    } else {
      b[g] = SsRec{s.last + 1, s.term, s.cl + 1, s.cf + 1};
      if (!(mode & 4u)) d[g] = s.term + int32_t(slot);   // (bit 2: no heartbeat store, as in shared form)
    }
  }
}

// VX (raft_device.hpp M_VX): every group's virtual suffix into the ring (the
// engine runs this before host reads of the state and handler batches)
template <int R>
__global__ __launch_bounds__(256) void vx_flush_kernel(DevPlanes P, uint64_t Qb, uint32_t E, uint32_t period,
                                                       uint64_t seed) {
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  if (g < P.G) vx_materialize<R>(P, g, Qb, E, period, seed);
}
hipError_t launch_vx_flush(int R, const DevPlanes& P, uint64_t Qb, uint32_t E, uint32_t period, uint64_t seed,
                           hipStream_t s) {
  RAFT_DISPATCH_R(R, hipLaunchKernelGGL(vx_flush_kernel<RR>, grid_for(P.G), dim3(256), 0, s, P, Qb, E, period, seed));
  return hipGetLastError();
}

template <int R>
__global__ __launch_bounds__(256) void sh_flush_kernel(DevPlanes P) {
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  if (g < P.G) sh_materialize<R>(P, g, P.sh_hb);
}
hipError_t launch_sh_flush(int R, const DevPlanes& P, hipStream_t s) {
  RAFT_DISPATCH_R(R, hipLaunchKernelGGL(sh_flush_kernel<RR>, grid_for(P.G), dim3(256), 0, s, P));
  return hipGetLastError();
}

hipError_t launch_stream_probe(int R, const uint16_t* a, SsRec* b, const uint16_t* c, int32_t* d, int32_t* rt,
                               int64_t* rv, uint32_t n, uint32_t slot, uint32_t kslots, hipStream_t s, uint32_t mode) {
  RAFT_DISPATCH_R(R, hipLaunchKernelGGL(stream_probe_kernel<RR>, grid_for(n), dim3(256), 0, s, a, b, c, d, rt, rv, n,
                                        slot, kslots, mode));
  return hipGetLastError();
}

}  // namespace raftstep
