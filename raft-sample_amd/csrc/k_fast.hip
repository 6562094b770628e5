// k_fast.hip — the steady-state tick kernel (the metric path).
#include <cstdlib>
#include "tick_common.hpp"

namespace raftstep {

// Diagnostics build only (make DIAG=1 / -DRAFTSTEP_WAVE_PROF): lane 0 of
// every list-kernel wave adds the cycles (s_memtime) it spent in each phase
// to the device counters (P.dbg, raft_diag_read) instead of the class
// counts: [0] staging, [1] step 1, [2] step 2, [3] write-back, [4] waves,
// [5] max wave cycles, [6..21] log2 histogram of a wave's cycles; inside
// fast_group (list steps): [32] per-group code, [33] copy gathers, [34] own
// ring writes, [35] copy scatters, [36] worklist + stats, [37] steps.
#ifdef RAFTSTEP_WAVE_PROF
#define WPROF(...) __VA_ARGS__
__device__ __forceinline__ void wprof_add(unsigned long long* d, int k, uint64_t v) {
  if (d && (threadIdx.x & 63) == 0) atomicAdd(&d[k], (unsigned long long)v);
}
#else
#define WPROF(...)
#endif

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
template <typename T>
__device__ __forceinline__ void st(T* base, uint32_t idx, T v) {
  at(base, idx) = v;
}

// Log ring entries are written once and read, if ever, K or fewer ticks
// later by the same group: every ring store is non-temporal (global_store
// ... nt), so the rings stream past the caches and the 256 MiB Infinity
// Cache keeps the per-group words and records that every tick re-reads
// (measured: C2 at 2^22 groups, lean kernel 87 -> 62 us; C4 list kernel
// 111 -> 95 us).
// (A/B, round 4, C2 one tick per launch: write-through sc1 ring stores 2%
// slower on C2 and 12% on C4; non-temporal / sc1 record and heartbeat stores
// 3% / 20% slower than plain ones)
template <typename T>
__device__ __forceinline__ void ring_st(T* base, uint32_t idx, T v) {
  __builtin_nontemporal_store(v, &base[idx]);
}
// Ring loads of the list / one-pass kernels: the entries may have been
// written earlier in the same kernel (a carried group's first step, another
// lane's copy) with non-temporal stores, which do not refresh the CU's L1,
// so the loads bypass L1 (agent-scope relaxed: global_load ... sc1, served
// by the XCD's L2, which holds those stores).
template <typename T>
__device__ __forceinline__ T ring_ld(const T* base, uint32_t idx) {
  return __hip_atomic_load(&base[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// R copies of one value into R consecutive ring elements (4-B aligned) with
// the widest non-temporal stores: 16-B pieces, then the remainder (a drifted
// lane's ring segment: 2 store instructions for R=7 terms instead of 7).
template <int N, typename T>
__device__ __forceinline__ void fill_seg(T* p, T v) {
  constexpr int per = int(16 / sizeof(T));   // elements per 16-B piece
  typedef T V16 __attribute__((ext_vector_type(per), aligned(4)));
  V16 w;
#pragma unroll
  for (int i = 0; i < per; ++i) w[i] = v;
#pragma unroll
  for (int i = 0; i + per <= N; i += per) __builtin_nontemporal_store(w, reinterpret_cast<V16*>(p + i));
  constexpr int rem = N % per;
  if constexpr (rem == 1) {
    __builtin_nontemporal_store(v, p + (N - 1));
  } else if constexpr (rem > 1) {
    typedef T VR __attribute__((ext_vector_type(rem), aligned(4)));
    VR r;
#pragma unroll
    for (int i = 0; i < rem; ++i) r[i] = v;
    __builtin_nontemporal_store(r, reinterpret_cast<VR*>(p + (N - rem)));
  }
}

// The list kernel's ring stores (scattered groups: each lane writes its own
// R-contiguous segment, i.e. partial lines). Its own-segment writes are plain
// (write-back) stores, so that the partial lines merge in L2 before they go
// to HBM; its entry copies stay non-temporal. Measured (round 4, interleaved
// A/B, profiles/r04/README.md): C4R 0.98e10 -> 1.07-1.08e10 (the lean kernel
// beside it 275-283 -> 236 us), C4 1.82 -> 1.85e10; every list-kernel ring
// store plain: the same on C4R, C4 within noise; copies alone plain: C4R
// 1.01-1.06e10. (A/B builds: RAFTSTEP_LIST_PLAIN 0 = all non-temporal, 1 =
// all plain, 3 = copies plain.)
#ifndef RAFTSTEP_LIST_PLAIN
#define RAFTSTEP_LIST_PLAIN 2
#endif
// (1: every list-kernel ring store; 2: its own-segment writes only; 3: its
// entry copies only)
template <bool LIST, typename T, int KIND = 2>
__device__ __forceinline__ void ring_stx(T* base, uint32_t idx, T v) {
  if constexpr (LIST && (RAFTSTEP_LIST_PLAIN == 1 || RAFTSTEP_LIST_PLAIN == KIND)) base[idx] = v;
  else ring_st(base, idx, v);
}
template <bool LIST, int N, typename T>
__device__ __forceinline__ void fill_segx(T* p, T v) {
  if constexpr (LIST && (RAFTSTEP_LIST_PLAIN == 1 || RAFTSTEP_LIST_PLAIN == 2)) {
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = v;
  } else {
    fill_seg<N>(p, v);
  }
}

// A group's R values of one per-replica plane are contiguous ([Gp][R], rix):
// a lane moves them with R/4 dwordx4 accesses plus one for the remainder
// (4-B aligned wide accesses are legal on gfx950) instead of R dword ones,
// which keeps the wave's requests at ~2 per 128-B line instead of R.
typedef int32_t row2 __attribute__((ext_vector_type(2), aligned(4)));
typedef int32_t row3 __attribute__((ext_vector_type(3), aligned(4)));
typedef int32_t row4 __attribute__((ext_vector_type(4), aligned(4)));
template <int R>
__device__ __forceinline__ void load_row_p(const int32_t* q, int (&o)[R]) {
#pragma unroll
  for (int i = 0; i + 4 <= R; i += 4) {
    const row4 a = *reinterpret_cast<const row4*>(q + i);
    o[i] = a.x; o[i + 1] = a.y; o[i + 2] = a.z; o[i + 3] = a.w;
  }
  constexpr int b = R & ~3, rem = R & 3;
  if constexpr (rem == 3) { const row3 a = *reinterpret_cast<const row3*>(q + b); o[b] = a.x; o[b + 1] = a.y; o[b + 2] = a.z; }
  if constexpr (rem == 2) { const row2 a = *reinterpret_cast<const row2*>(q + b); o[b] = a.x; o[b + 1] = a.y; }
  if constexpr (rem == 1) o[b] = q[b];
}
template <int R>
__device__ __forceinline__ void store_row_p(int32_t* q, const int (&v)[R]) {
#pragma unroll
  for (int i = 0; i + 4 <= R; i += 4) *reinterpret_cast<row4*>(q + i) = row4{v[i], v[i + 1], v[i + 2], v[i + 3]};
  constexpr int b = R & ~3, rem = R & 3;
  if constexpr (rem == 3) *reinterpret_cast<row3*>(q + b) = row3{v[b], v[b + 1], v[b + 2]};
  if constexpr (rem == 2) *reinterpret_cast<row2*>(q + b) = row2{v[b], v[b + 1]};
  if constexpr (rem == 1) q[b] = v[b];
}

// Row and per-group word access of one group inside fast_group: in the
// dense launches its record in HBM (the SGPR plane base and a 32-bit lane
// offset) and the per-group planes at g; in the list kernel the lane's LDS
// copies (pointers derived from the __shared__ arrays, so the accesses are
// ds_ instructions: a flat access would wait on every outstanding global
// store, vmcnt counting stores on gfx950).
template <int R, bool LDS>
struct RowAcc {
  int32_t* base;   // global: P.rec; LDS: the lane's record copy
  uint32_t o;      // global: g * recw (element offset); LDS: 0
  uint32_t* dm;    // LDS: the lane's dirty-row mask (the list kernel writes back only those rows' pieces)
  __device__ __forceinline__ int32_t& at(int k, int r) const {
    if constexpr (LDS) return base[k * R + r];
    else return raftstep::at(base, o + uint32_t(k * R + r));
  }
  __device__ __forceinline__ void st(int k, int r, int32_t v) const {
    if constexpr (LDS) { base[k * R + r] = v; *dm |= 1u << k; }
    else raftstep::st(base, o + uint32_t(k * R + r), v);
  }
  __device__ __forceinline__ void load(int k, int (&a)[R]) const {
    if constexpr (LDS) {
#pragma unroll
      for (int r = 0; r < R; ++r) a[r] = base[k * R + r];
    } else {
      load_row_p<R>(&raftstep::at(base, o + uint32_t(k * R)), a);
    }
  }
  __device__ __forceinline__ void store(int k, const int (&a)[R]) const {
    if constexpr (LDS) {
#pragma unroll
      for (int r = 0; r < R; ++r) base[k * R + r] = a[r];
      *dm |= 1u << k;
    } else {
      store_row_p<R>(&raftstep::at(base, o + uint32_t(k * R)), a);
    }
  }
};
template <bool LDS>
struct WordAcc {
  // global: the plane bases and g; LDS: the lane's slots (g unused). The
  // packed cold words (GSeg) are strided views in global memory.
  template <typename T>
  using Cold = std::conditional_t<LDS, T*, Strided<T, 16>>;
  uint16_t* meta_;
  uint16_t* rot_;
  Cold<uint16_t> rota_;
  std::conditional_t<LDS, uint8_t*, Strided<uint8_t, 1>> iso_;
  int32_t* hb_;
  int32_t* sb_;
  SsRec* ss_;
  Cold<uint16_t> rotb_;
  Cold<int32_t> sb2_;
  LxRec* lx_;
  uint32_t g;
  __device__ __forceinline__ uint16_t& meta() const { if constexpr (LDS) return *meta_; else return raftstep::at(meta_, g); }
  __device__ __forceinline__ uint16_t& rot() const { if constexpr (LDS) return *rot_; else return raftstep::at(rot_, g); }
  __device__ __forceinline__ uint16_t& rota() const { if constexpr (LDS) return *rota_; else return raftstep::at(rota_, g); }
  __device__ __forceinline__ uint8_t& iso() const { if constexpr (LDS) return *iso_; else return raftstep::at(iso_, g); }
  __device__ __forceinline__ int32_t& hb() const { if constexpr (LDS) return *hb_; else return raftstep::at(hb_, g); }
  __device__ __forceinline__ int32_t& sb() const { if constexpr (LDS) return *sb_; else return raftstep::at(sb_, g); }
  __device__ __forceinline__ uint16_t& rotb() const { if constexpr (LDS) return *rotb_; else return raftstep::at(rotb_, g); }
  __device__ __forceinline__ int32_t& sb2() const { if constexpr (LDS) return *sb2_; else return raftstep::at(sb2_, g); }
  __device__ __forceinline__ LxRec& lx() const { if constexpr (LDS) return *lx_; else return lx_[g]; }
  __device__ __forceinline__ SsRec& ss() const { if constexpr (LDS) return *ss_; else return ss_[g]; }
  __device__ __forceinline__ void st_hb(int32_t v) const {
    if constexpr (LDS) *hb_ = v;
    else raftstep::st(hb_, g, v);
  }
};
template <int R>
__device__ __forceinline__ RowAcc<R, false> rows_global(const DevPlanes& P, uint32_t g) {
  return RowAcc<R, false>{P.rec, rix<R>(g, 0), nullptr};
}
__device__ __forceinline__ WordAcc<false> words_global(const DevPlanes& P, uint32_t g) {
  return WordAcc<false>{P.gmeta, P.grot, P.grota, P.giso, P.hb, P.gsb, P.gss, P.grotb, P.gsb2, P.glx, g};
}

// A ONECAND group is taken only when a replica is isolated this tick (its
// role, which must be the candidate, is checked once the rs row is read).
template <bool RAFT>
__device__ __forceinline__ bool xi_ok(int meta, int xi) {
  return (meta & M_STEADY) || (RAFT && (meta & (M_ONECAND | M_ONESTALE)) && xi >= 0);
}

// A group without a leader whose tick changes nothing: no timer expires
// and the one candidate's vote round (if any) is refused by every peer it
// reaches without a state change — the run_tick steps of such a tick are
// client (no leader: nothing, main.go:327), rounds (CandidateRun's default
// branch, main.go:253-284 -> 157-170 / RAFT r_deliver_vr) and timers
// (main.go:171-177, 248-251), none of which fires. This is the common state
// of a group between a disruption and its next election, so the tick is
// taken here instead of deferring the group. Conservative: anything else
// (a second candidate, a grant, a term to adopt, a timer due) defers.
template <int R, bool RAFT, class Rows, class Words>
__device__ __forceinline__ bool quiet_leaderless(const DevPlanes& P, const Trace& T, const Rows& RW, const Words& GW,
                                                 uint64_t key) {
  if (R < 2) return false;   // a lone candidate would win its round
  int term[R], last[R], lt[R], ts[R];
  RW.load(PL_TERM, term);
  RW.load(PL_LAST, last);
  RW.load(PL_LTERM, lt);
  RW.load(PL_TSTART, ts);
  const int hb = GW.hb();
  int rs[R];   // role:2 | vote:4 | d:10
#pragma unroll
  for (int r = 0; r < R; ++r) rs[r] = RW.at(PL_RS, r);
  int c = -1;
  bool quiet = true;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int role = rs[r] & 3;
    quiet &= role != ROLE_L;
    if (role == ROLE_C) { quiet &= c < 0; c = r; }
    // non-leaders' effective timer start counts the last heartbeat (Group::eff_start)
    quiet &= max(ts[r], hb) + (rs[r] >> 6) > T.now;
  }
  if (!quiet || c < 0) return quiet;
  uint32_t im = 0;
  if (T.iso_p) {
    uint32_t act = 0, starting = 0;
    im = iso_windows<R>(key, T, &act, &starting);
    if (T.iso_leader) {   // a window starting now is decided (and recorded) by the general kernel
      if (starting) return false;
      uint32_t gi = act ? uint32_t(GW.iso()) : 0u;
      im = leader_iso_mask(act, 0u, gi, 0u, false);
    }
  }
  const int ct = sel(term, c), cl = sel(last, c);
  const int clt = cl > 0 ? sel(lt, c) : 0;
  const uint32_t cvote = (uint32_t(sel(rs, c)) >> 2) & 15u;
  if (!RAFT && cvote == 0u) return false;   // REF: the round would set the candidate's Voted
#pragma unroll
  for (int p = 0; p < R; ++p) {
    if (p == c || (((im >> p) | (im >> c)) & 1u)) continue;   // dropped: never delivered
    const int vote = (rs[p] >> 2) & 15;
    if constexpr (RAFT) {
      // r_deliver_vr: the peer already holds the candidate's term (nothing to
      // adopt, no stop) and refuses: voted for another, or log more up to date
      const int mt = last[p] > 0 ? lt[p] : 0;
      const bool uptodate = clt > mt || (clt == mt && cl >= last[p]);
      quiet &= term[p] == ct && !((vote == 0 || vote == c + 1) && uptodate);
    } else {
      // deliver_vr (main.go:160-162): a follower refuses without a change
      quiet &= ct < term[p] || vote != 0;
    }
  }
  return quiet;
}

// The tick of one group (lane) — the body of both launch forms: the dense
// one over all groups (tick_fast_kernel, `g` = the lane's group) and the one
// over the list of groups the lean kernel passed on (tick_list_kernel, LIST:
// the lanes of a wave hold scattered groups, so every ring write is the
// lane's own). Block-uniform control flow (it reduces over the block).
template <int R, bool CRC, int SEM, bool LIST, class Rows, class Words>
__device__ __forceinline__ bool fast_group(const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* work,
                                           int32_t* work_tick, uint32_t* work_count, int force_slow, const uint32_t g,
                                           const uint32_t* tab, const Rows& RW, const Words& GW, const int shf = -1) {
  constexpr bool RAFT = SEM == SEM_RAFT;
  WPROF(uint64_t wp0 = __builtin_amdgcn_s_memtime(); uint64_t wp1 = wp0, wp2 = wp0, wp3 = wp0;)
  int sv[7] = {0, 0, 0, 0, 0, 0, 0};   // committed, ae_ok, ae_fail, leader_groups, term bumps, votes, won
  bool bail = false;
  const int n = int(T.client_entries());   // entries per leader this tick (wave-uniform)
  // this lane's ring writes, issued after the per-group code (wave-converged)
  uint32_t wr = 0;      // replicas that append this tick's entries (leader + accepting followers)
  int w_term = 0, w_ph = 0;    // their term and the ring slot of the first entry
  uint64_t w_vb = 0;    // value stream base of this tick's entries
  // RAFT entry job of this lane (written by the whole wave below): a
  // returning stale leader's catch-up (the primary's entries L0+1..Ll into
  // its column) or a stale leader's entries above a ring segment switch (to
  // the new segment's slots). Either is one leader's own client appends, one
  // batch per client tick up to the present (a leader appends at every client
  // tick, main.go:327-329, and a cut-off one too), so entry jb_from+j is its
  // appender's global client entry jb_q0+j: the entries are regenerated from
  // the trace RNG (value stream jb_kv, term jb_term) instead of read back.
  int jb_n = 0, jb_from = 0, jb_term = 0, jb_sb = 0, jb_sb2 = 0;
  uint32_t jb_col = 0, jb_rot = 0, jb_rotb = 0;   // destination column; ring words (rot | rota << 16, rotb)
  uint64_t jb_q0 = 0, jb_kv = 0;
  int jb_scol = -1;     // >= 0: the entries are read from this column instead (staged values), jb_sd slots back
  int jb_sd = 0;
  uint32_t df = 0;      // diagnostics: lane class bits (P.dbg)
  uint32_t vxf = 0;     // diagnostics: 1 = a return with a virtual suffix (no copy), 2 = LXS entered with one
  bool stored = false;  // the group's rows may have been written (returned)
  // deferral-reason bits 11-15 only in a diagnostics build (make DIAG=1),
  // so the product kernel carries no extra instructions for them
#ifdef RAFTSTEP_DIAG_REASONS
#define DIAG_REASON(x) x
#else
#define DIAG_REASON(x)
#endif
  if (g < P.G) {
    int meta = GW.meta();
    const int meta_st = meta;   // as stored (meta may drop the compressed-form flags below)
    const int c = meta & 0xF;
    const bool skip = (meta & M_DEFER) || ((meta >> 4) & 7);   // pending catch-up / frozen group
    // RAFT also takes ONECAND groups (their candidate must be isolated this tick, checked below)
    bail = !skip && (force_slow || !(meta & (RAFT ? (M_STEADY | M_ONECAND | M_ONESTALE) : M_STEADY)));
    if (bail && !force_slow && c == NO_PRIMARY) {   // leaderless: a quiet tick needs no general kernel
      const bool q = quiet_leaderless<R, RAFT>(P, T, RW, GW, T.iso_p ? group_key(T.seed, P.gbase + g) : 0ull);
      bail = !q;
      df |= q ? 65536u : 0u;
    }
    int term[R], last[R], commit[R], lt[R], m[R];
    uint32_t rowbad = 0;   // RAFT explicit rows out of step (replica bits)
    uint32_t fresh = 0;    // RAFT: a new leader's rows (MatchIndex 0, NextIndex = its length + 1)
    uint32_t hwup = 0;     // RAFT: replicas whose high-water mark is above their log length (truncated)
    bool empty = true;   // every log of the group empty before this tick
    const bool go = !skip && !bail && c != NO_PRIMARY;
    // SSYNC: the group's term / last / commit / lterm rows are one 16-B record
    // (every replica at the same length and term, the followers at one
    // CommitIndex; implies MSYNC). The rows are rebuilt in registers here and
    // either written back as the record or, when the tick breaks the form,
    // spilled as whole rows.
    bool ss = go && (meta & M_SSYNC);
    df |= skip ? 1u : 0u;
    DIAG_REASON(df |= bail ? 2048u : 0u;);   // diagnostics: deferral reason "group not steady"
    if (go) {
      if (ss) {
        const SsRec ss_rec = GW.ss();
        const LxRec lxr = (RAFT && uses_glx(meta)) ? GW.lx() : LxRec{0, 0};   // LXS: the leader is k ahead
#pragma unroll
        for (int r = 0; r < R; ++r) {
          term[r] = ss_term(ss_rec, r, meta, lxr); last[r] = ss_last(ss_rec, r, c, meta, lxr);
          commit[r] = r == c ? ss_rec.cl : ss_rec.cf;
          lt[r] = term[r];
        }
        if (RAFT && is_sxs(meta)) {
          // SXS: the tick runs on the explicit ONESTALE form, so materialise it
          // in the rows (Group::load's rule): every row but the stale leader's
          // as the record says, its CommitIndex and the primary's MatchIndex /
          // NextIndex for it as they stand, high-water marks max(plane, last)
          const int xs = lxr.dl;
          put(commit, xs, RW.at(PL_COMMIT, xs));
          RW.store(PL_TERM, term);
          RW.store(PL_LAST, last);
          RW.store(PL_COMMIT, commit);
          RW.store(PL_LTERM, lt);
#pragma unroll
          for (int p = 0; p < R; ++p) {
            if (p != c && p != xs) {
              RW.st(PL_LMATCH, p, last[p]);
              RW.st(PL_LNEXT, p, last[p] + 1);
            }
            if (RW.at(PL_HWM, p) < last[p]) RW.st(PL_HWM, p, last[p]);
          }
          meta &= ~(M_SSYNC | M_MSYNC);
          ss = false;
          df |= 1u << 29;   // class: an SXS group taken by the full body (materialised)
        }
      } else {
        RW.load(PL_TERM, term);
        RW.load(PL_LAST, last);
        RW.load(PL_COMMIT, commit);
        RW.load(PL_LTERM, lt);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) empty &= last[r] == 0;
      if (meta & M_MSYNC) {
#pragma unroll
        for (int r = 0; r < R; ++r) m[r] = (r != c) ? last[r] : 0;
        if constexpr (RAFT) {
          if (meta & M_HWX) {   // high-water marks max(plane, LastApplied): truncated logs in step
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const int hwd = RW.at(PL_HWM, r) - last[r];
              if (hwd >= int(P.K)) rowbad |= 1u << r;
              if (hwd > 0) hwup |= 1u << r;
            }
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) m[r] = (r != c) ? RW.at(PL_LMATCH, r) : 0;
        if constexpr (RAFT) {
          // RAFT rows kept explicitly: NextIndex must be MatchIndex+1 and no
          // log may be shorter than its high-water mark (no pending truncation)
          const int lc1 = sel(last, c) + 1;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int nxr = RW.at(PL_LNEXT, r);
            if (r != c && nxr != m[r] + 1) {
              // the rows a leader starts its term with (r_candidate_round):
              // in step for a follower holding the leader's log (checked below)
              if (m[r] == 0 && nxr == lc1) fresh |= 1u << r;
              else rowbad |= 1u << r;
            }
            // a log truncated below its high-water mark stays in step as long as
            // the entry this tick's AppendEntries checks (its last) is still
            // inside the ring window (hwm-K, last] (Group::r_deliver_ae's evicted rule)
            const int hwd = RW.at(PL_HWM, r) - last[r];
            if (hwd < 0 || hwd >= int(P.K)) rowbad |= 1u << r;
            if (hwd > 0) hwup |= 1u << r;
          }
        }
      }
    }
    // ONESTALE: the stale leader's row is its own (checked below, once it is known)
    if (!RAFT || !(meta & M_ONESTALE)) bail |= rowbad != 0u;
    DIAG_REASON(if (bail && !(df & 2048u)) df |= 16384u;);   // reason: explicit RAFT rows out of step
    uint64_t key = 0;
    if (go && (T.iso_p || n)) key = group_key(T.seed, P.gbase + g);
    // RAFT: one isolated replica xi (not the leader) is handled here: it
    // receives nothing and sends nothing (its AppendEntries is dropped, its
    // vote requests too), so the rest of the group ticks as usual and xi only
    // runs its own election timer. Its lagging MatchIndex stays implicit
    // (MSYNC: MatchIndex[xi] == LastApplied[xi], both unchanged).
    int xi = -1;
    int giso_w = -1;   // giso to store (a window decided this tick), -1: unchanged
    bool lx = false;   // RAFT: the primary leader is the one isolated replica (see below)
    uint32_t im = 0;   // replicas cut off this tick
    if (go && T.iso_p) {
      uint32_t act = 0, starting = 0;
      im = iso_windows<R>(key, T, &act, &starting);
      if (T.iso_leader) {
        // leader mode: a window starting now takes the lowest-id Leader as the
        // tick begins (tick_iso_mask, decide); in a STEADY group that is the
        // primary, recorded in giso with the tick's stores. Other groups with
        // a window starting go to the general kernel.
        uint32_t gi = act ? uint32_t(GW.iso()) : 0u;
        if (starting && (meta & M_STEADY)) {
          const uint32_t g0 = gi;
          im = leader_iso_mask(act, starting, gi, 1u << c, true);
          if (gi != g0) giso_w = int(gi);
        } else {
          if (starting) bail = true;
          im = leader_iso_mask(act, 0u, gi, 0u, false);
        }
      }
      if (RAFT && R >= 3 && im && (im & (im - 1u)) == 0u && int(__builtin_ctz(im)) != c) xi = int(__builtin_ctz(im));
      else if (RAFT && R >= 3 && im == (1u << c) && (meta & M_STEADY)) lx = true;
      else bail |= im != 0u;
      if (im) df |= 4u;
    }
    DIAG_REASON(if (bail && !(df & (2048u | 16384u))) df |= 4096u;);   // reason: leader or >1 replica isolated
    // RAFT ONESTALE with nobody cut off this tick: the stale leader is
    // reachable again (its window ended) — the return tick, taken below when
    // it is a plain catch-up (sr: the returning stale leader)
    int sr = -1;
    if (RAFT && go && !bail && (meta & M_ONESTALE) && im == 0u && !P.crc_on) {
#pragma unroll
      for (int p = 0; p < R; ++p)
        if (p != c && (RW.at(PL_RS, p) & 3) == ROLE_L) sr = p;
    }
    if (go && !xi_ok<RAFT>(meta, xi) && sr < 0) bail = true;   // ONECAND needs its candidate isolated (role checked below)
    // RAFT ONESTALE: the one non-follower besides the primary is a leader of a
    // lower term, cut off this tick (xi). It appends this tick's client entries
    // to its own log and every AppendEntries it sends is dropped; its commit
    // rule cannot move (its MatchIndex row has not changed since it was cut
    // off and its own log only grows past it). Its row in the primary's
    // planes stays explicit, so the group keeps explicit rows (no MSYNC).
    const bool stale = RAFT && (meta & M_ONESTALE) && xi >= 0;
    if (RAFT && (meta & M_ONESTALE))
      bail |= (rowbad & ~(stale ? 1u << xi : 0u) & ~(sr >= 0 ? 1u << sr : 0u)) != 0u;
    // leader view
    const int Lt = sel(term, c), Ll = sel(last, c), Lc = sel(commit, c), Llt = sel(lt, c);
    // RAFT: the leader itself cut off (leader isolation), every other replica
    // a follower waiting for it. The tick is: the leader appends this tick's
    // entries to its own log (client, main.go:327-329), every AppendEntries
    // it sends is dropped (EXT: the sender sees a failure), the commit rule
    // runs over unchanged MatchIndex values, and nobody's timer is reset; it
    // is taken here while no follower's timer is due (that would start an
    // election). MatchIndex must equal LastApplied for every follower (RAFT
    // rows were checked against NextIndex / high-water marks above); both
    // stand still, so the rows become implicit (MSYNC).
    if (go && !bail && lx) {
      // (a truncated log, high-water mark above its length, would break MSYNC's hwm == last)
      // (fresh rows are in step only for a follower that accepts this tick; here nobody does)
      bail = int64_t(Ll) + n > I32MAX || n >= int(P.K) || Ll == 0 || hwup != 0u || fresh != 0u;
#pragma unroll
      for (int p = 0; p < R; ++p) bail |= p != c && m[p] != last[p];
      int ts[R], rsv[R];
      RW.load(PL_TSTART, ts);
      const int hbt = GW.hb();
      int w = -1, wdl = 0;   // the first follower, in (deadline, id) order, whose election timeout is due
#pragma unroll
      for (int p = 0; p < R; ++p) {
        rsv[p] = RW.at(PL_RS, p);
        const int dl = max(ts[p], hbt) + (rsv[p] >> 6);
        if (p != c && dl <= T.now && (w < 0 || dl < wdl)) { w = p; wdl = dl; }
      }
      // Election (step 3 of the tick, after the cut-off leader's round):
      // w times out (r_timeout_fire: Term+1, votes for itself, candidate
      // timer) and runs its vote round at once (r_candidate_round,
      // main.go:253-284 -> 157-170 with Raft's up-to-date check). Every other
      // follower holds w's log and term, so each adopts Term+1 and grants
      // (its timer reset), the cut-off leader is never reached: w wins with
      // R-1 > R/2 votes; no other timer is still due. Taken when every
      // follower's log and term equal w's; anything else: general path.
      if (w >= 0) {
        const int fl = sel(last, w), flt = sel(lt, w);
        bail |= Lt >= I32MAX;
#pragma unroll
        for (int p = 0; p < R; ++p)
          if (p != c) bail |= term[p] != Lt || last[p] != fl || (fl > 0 && lt[p] != flt);
      }
      // commitIndex: the largest N held by a majority (leader included), if
      // log[N].term == currentTerm (Group::r_commit_rule); MatchIndex = LastApplied (MSYNC)
      int N = -1;
#pragma unroll
      for (int p = 0; p < R; ++p) {
        const int vp = p == c ? Ll + n : last[p];
        int cnt = 0;
#pragma unroll
        for (int q = 0; q < R; ++q) cnt += (q == c ? Ll + n : last[q]) >= vp ? 1 : 0;
        if (cnt >= R / 2 + 1 && vp > N) N = vp;
      }
      int cm = Lc;
      if (N > Lc) {
        if (N == Ll + n && n > 0) cm = N;                 // this tick's entries: current term
        else if (N == Ll) cm = Llt == Lt ? N : Lc;        // the cached last-entry term
        else bail = true;                                 // would need a ring read: general path
      }
      // VX (M_VX): a virtual suffix is kept only in LXS and through the
      // election into ONESTALE; a cut-off leader leaving the compressed form
      // without an election goes to the general kernel (which materialises it)
      if (RAFT && (meta & M_VX) && w < 0 && !(ss && T.iso_leader && Llt == Lt)) bail = true;
      if (!bail) {
        df |= 131072u;
        // a compressed group stays compressed (LXS: the record holds the
        // followers, glx the leader's lead and the earliest follower deadline,
        // and the lean kernel takes the following ticks of the window)
        const bool to_lxs = ss && w < 0 && T.iso_leader && Llt == Lt;
        if (ss && !to_lxs) {   // the record's rows become explicit (the leader's elements change below)
          int trow[R], lrow[R], crow[R];
#pragma unroll
          for (int p = 0; p < R; ++p) { trow[p] = term[p]; lrow[p] = last[p]; crow[p] = commit[p]; }
          RW.store(PL_TERM, trow);
          RW.store(PL_LAST, lrow);
          RW.store(PL_COMMIT, crow);
          RW.store(PL_LTERM, trow);
        }
        sv[0] = cm - Lc;
        sv[1] = 0;
        sv[2] = R - 1;                                    // every AppendEntries dropped
        sv[3] = 1;
        sv[4] = 0;
        if (n) {
          if (!to_lxs) {
            RW.st(PL_LAST, c, Ll + n);
            if (Llt != Lt) RW.st(PL_LTERM, c, Lt);
          }
          wr = 1u << c;                                   // only the leader's log grows
          w_term = Lt;
          w_ph = int((uint32_t(Ll) + uint32_t(GW.rot())) & P.kmask);
          w_vb = cv_base(P, key, uint32_t(c), T.tick, g);
        }
        if (cm != Lc && !to_lxs) RW.st(PL_COMMIT, c, cm);
        int nm = (meta | M_MSYNC) & ~(M_SSYNC | M_HWX | M_LXS);   // (no truncated log here: hwup == 0)
        if (to_lxs) {
          const int f = c == 0 ? 1 : 0;   // any follower (SSYNC: one length, term, CommitIndex)
          int dmin = I32MAX;
#pragma unroll
          for (int p = 0; p < R; ++p)
            if (p != c) dmin = min(dmin, max(ts[p], hbt) + (rsv[p] >> 6));
          GW.ss() = SsRec{sel(last, f), Lt, cm, sel(commit, f)};
          GW.lx() = LxRec{Ll + n - sel(last, f), dmin};
          nm |= M_SSYNC | M_LXS;
          // entering LXS from the steady form (the leader's log was the
          // followers'): its entries from this tick on are its own client
          // appends, one batch per client tick — a virtual suffix (M_VX)
          if (P.vx && !(meta & M_LXS) && Ll == sel(last, f)) {
            nm |= M_VX;
            vxf |= 2u;
          }
        }
        if (w >= 0) {   // the election (see above)
          const int nt = Lt + 1, fl = sel(last, w);
          const int dc = T.c_min + int(uint32_t(rng_k(key, uint32_t(w), ST_TIMER_C, uint64_t(T.tick)) >> 32) %
                                       uint32_t(T.c_span));
          int hwr[R], mz[R], nx[R];
#pragma unroll
          for (int p = 0; p < R; ++p) {
            hwr[p] = p == c ? Ll + n : last[p];   // high-water marks become explicit (MSYNC ends)
            mz[p] = 0;                            // w's rows: MatchIndex 0, NextIndex = its length + 1
            nx[p] = fl + 1;
            if (p == c) continue;
            RW.st(PL_TERM, p, nt);
            RW.st(PL_TSTART, p, T.now);   // candidate timer start / vote granted: timer reset
            RW.st(PL_RS, p, p == w ? int32_t(ROLE_L | (uint32_t(w + 1) << 2) | (uint32_t(dc) << 6))
                                                : int32_t((rsv[p] & ~0x3F) | ROLE_F | ((w + 1) << 2)));
            // the cut-off leader's rows (implicit: MatchIndex = LastApplied) move to its xmatch / xnext rows
            st(prow(P.xmatch, c * R + p, P.Gp), g, last[p]);
            st(prow(P.xnext, c * R + p, P.Gp), g, last[p] + 1);
          }
          RW.store(PL_HWM, hwr);
          RW.store(PL_LMATCH, mz);
          RW.store(PL_LNEXT, nx);
          // w (the highest term) becomes the primary; the cut-off leader is a stale one
          nm = (meta & ~(0xF | M_MSYNC | M_SSYNC | M_HWX | M_LXS | M_STEADY | M_ONECAND)) | w | M_ONESTALE;
          sv[4] = 1;       // term bumps: w's timeout
          sv[5] = R - 2;   // votes granted
          sv[6] = 1;       // elections won
          df |= 1u << 19;  // class: the election tick of a cut-off leader's group
        }
        if (nm != meta_st) GW.meta() = uint16_t(nm);
      }
    }
    const bool gom = go && !lx;   // the main steady-state path
    if (gom && !bail) bail = int64_t(Ll) + n > I32MAX || n >= int(P.K);
    // REF with payload CRC (round 6): one follower whose last AppendEntries
    // was rejected (a corrupted copy, EXT) lags — its log ends at its
    // MatchIndex m < Ll (REF keeps MatchIndex on a failure, main.go:375-378).
    // Its AppendEntries this tick is case (ii) of main.go:353-360: entries
    // m+1 .. Ll+n with prevLogIndex m and prevLogTerm GetLog(m).Term (one ring
    // read); accepted, the leader's entries m+1..Ll are copied into its
    // column by the wave (GetLogsFrom, main.go:357) and the group is in step
    // again. Taken while m > 0, the batch fits the ring (Ll+n-m < K) and this
    // tick has entries; anything else takes the general path as before.
    // Several followers may lag at once (round 6: two rejections in one tick
    // were C5V's deferrals, ~130 groups a tick): any number whose catch-up
    // copies nothing — a group kept in shared form (shf >= 0) whose follower
    // holds every entry below shf — and at most one whose catch-up is copied (lg).
    int lg = -1;
    uint32_t lgm = 0;   // the lagging followers
    if (gom) {
#pragma unroll
      for (int p = 0; p < R; ++p) {
        if (p == sr) continue;   // the returning stale leader: checked with its AppendEntries below
        if (p == xi) {   // MSYNC stays exact for an isolated follower / candidate (not a fresh row: unchanged, explicit)
          if (!stale) bail |= m[p] != last[p] || m[p] > Ll || ((fresh >> p) & 1u);
          continue;
        }
        if (!RAFT && CRC && p != c && n > 0 && m[p] > 0 && m[p] < Ll && m[p] == last[p] &&
            Ll + n - m[p] < int(P.K)) {
          const bool nocopy = shf >= 0 && m[p] + 1 >= shf;
          if (nocopy || lg < 0) {
            lgm |= 1u << p;
            if (!nocopy) lg = p;
            continue;
          }
        }
        bail |= (p != c) && m[p] != Ll && !((fresh >> p) & 1u);
        // RAFT: a follower with extra entries or another term takes the general path
        if constexpr (RAFT) bail |= (p != c) && (last[p] != Ll || term[p] != Lt);
      }
    }
    DIAG_REASON(if (bail && !(df & (2048u | 4096u | 16384u))) df |= 8192u;);   // reason: a follower's log or term not in step
    // the isolated replica's own state: role, vote, timer (eff. start = max(tstart, hb))
    int x_rs = 0, x_term = 0, x_fire = 0, x_dur = 0;
    if constexpr (RAFT) {
      if (gom && !bail && xi >= 0) {
        x_rs = RW.at(PL_RS, xi);
        x_term = sel(term, xi);
        const int role = x_rs & 3;
        // STEADY: xi is a follower; ONECAND: the group's one candidate; ONESTALE: the stale leader
        if (role != ((meta & M_STEADY) ? ROLE_F : stale ? ROLE_L : ROLE_C)) bail = true;
        // (the stale leader appends at its own log's end with the ring rotation as it stands:
        // an empty group would pick a new phase, see below)
        if (stale && (x_term >= Lt || int64_t(sel(last, xi)) + n > I32MAX || empty)) bail = true;
        const int dl = max(RW.at(PL_TSTART, xi), GW.hb()) + (x_rs >> 6);
        if (!stale && dl <= T.now) {   // timer.C: Term++, vote for itself, new candidate timer (Raft §5.2)
          if (x_term >= I32MAX) bail = true;
          x_fire = 1;
          x_dur = T.c_min + int(uint32_t(rng_k(key, uint32_t(xi), ST_TIMER_C, uint64_t(T.tick)) >> 32) %
                                uint32_t(T.c_span));
        }
      }
    }
    // one AppendEntries shape for every peer (NextIndex == Ll+1)
    int prev_idx, prev_term;
    if constexpr (RAFT) { prev_idx = Ll; prev_term = Ll > 0 ? Llt : 0; }   // log[nextIndex-1].term
    else if (n == 0 || Ll == 0) { prev_idx = Ll; prev_term = Lt; }          // REF heartbeat / whole-log
    else { prev_idx = Ll; prev_term = Llt; }                                 // GetLog(MatchIndex).Term
    // EXT: every follower verifies the CRC32C stamp of each entry it received
    // (the term's CRC state is shared, the term bytes are never corrupted)
    uint32_t crcbad = 0;
    if constexpr (CRC) {
      if (gom && !bail && n) {
        uint32_t cm = 0;   // followers whose message is corrupted this tick
#pragma unroll
        for (int p = 0; p < R; ++p)
          if (p != c && p != xi && P.corrupt_p &&
              (rng_k(key, uint32_t(p), ST_CORRUPT, uint64_t(T.tick)) & 0xFFFF) < P.corrupt_p)
            cm |= 1u << p;
        // (an unaltered copy carries the leader's stamp: CRCs only for cm)
        if (cm) crcbad = crc_reject_mask(tab, crc_term_state(tab, Lt), cv_base(P, key, uint32_t(c), T.tick, g),
                                         cv_stride(P), n, cm);
      }
    }
    int lg_pt[R];   // each lagging follower's prevLogTerm: the leader's entry at its MatchIndex (one ring read each)
#pragma unroll
    for (int p = 0; p < R; ++p) {
      lg_pt[p] = 0;
      if (!RAFT && CRC && gom && !bail && ((lgm >> p) & 1u)) {
        const int ml = m[p];
        const uint32_t so = ring_slot(ml, GW.rot(), GW.rota(), GW.rotb(), GW.sb(), GW.sb2(), P.kmask);
        // (a group kept in shared form, shf >= 0: entries from shf on are in the shared ring)
        lg_pt[p] = (shf >= 0 && ml >= shf) ? ring_ld(P.sh_term + sh_tile(g, P.KP), sh_in_tile(g, so, P.sh_cs))
                                           : ring_ld(P.log_term + ring_tile(g, P.KP, R), ring_in_tile(g, R, so, uint32_t(c)));
      }
    }
    uint32_t okm = 0, cch = 0, mch = 0, ltch = 0;
    if (gom && !bail) {
#pragma unroll
      for (int p = 0; p < R; ++p) {
        if (p == c || p == xi || p == sr) continue;   // xi: dropped (sender sees false, receiver unchanged)
        const int l = last[p];
        const bool lgp = !RAFT && CRC && ((lgm >> p) & 1u);
        const int np = lgp ? Ll + n - l : n;          // len(Logs) of p's AppendEntries
        bool ok;
        if constexpr (RAFT) {
          // same term (checked), log exactly as long as the leader's before this tick
          if (l > 0 && lt[p] != prev_term) bail = true;           // conflict: hint + backoff path
          if ((crcbad >> p) & 1u) bail = true;                    // rejected payload: backoff path
          ok = true;
        } else {
          const int pi = lgp ? l : prev_idx, pt = lgp ? lg_pt[p] : prev_term;
          ok = Lt >= term[p];                                     // main.go:129-133
          if (ok && l > 0) {                                      // main.go:135
            if (int64_t(l) + np < pi) ok = false;                 // 137-140
            else if (pi < 1 || pi > l || pi <= l - int(P.K) || pi != l) bail = true;
            else ok = lt[p] == pt;                                // 142-145 (GetLog(l) == last entry)
          }
          if (ok && int64_t(l) + np > I32MAX) bail = true;
          if (ok && ((crcbad >> p) & 1u)) ok = false;             // EXT: payload rejected
        }
        if (ok) {
          const int nl = l + np;                                  // 148-149
          last[p] = nl;
          if (n && lt[p] != Lt) ltch |= 1u << p;
          if (Lc > commit[p]) {                                   // 151-152
            // REF: min(LC, len(Log)+1); RAFT: min(leaderCommit, index of last new entry)
            const int cap = RAFT ? nl : nl + 1;
            const int nc = Lc < cap ? Lc : cap;
            if (nc != commit[p]) { commit[p] = nc; cch |= 1u << p; }
          }
          if (nl != m[p]) { m[p] = nl; mch |= 1u << p; }          // 156 -> 375-377
          okm |= 1u << p;
          if (lgp && p != lg && P.dbg) atomicAdd(&P.dbg[6], 1ull);   // (a catch-up that copies nothing)
          if (lgp && p == lg) {   // its catch-up: the leader's entries l+1..Ll, copied from the leader's column below
            // (kept in shared form: only those below shf; the rest are the shared ones it now holds too)
            jb_n = max(0, (shf >= 0 ? min(Ll, shf - 1) : Ll) - l);
            jb_from = l + 1;
            jb_col = uint32_t(p);
            jb_term = Lt;
            jb_scol = c;
            jb_sd = 0;
            jb_rot = GW.rot() | (uint32_t(GW.rota()) << 16);
            jb_rotb = GW.rotb();
            jb_sb = GW.sb();
            jb_sb2 = GW.sb2();
            if (P.dbg) atomicAdd(&P.dbg[6], 1ull);   // diagnostics: a lagging follower caught up
          }
        }
      }
    }
    // The return tick (sr >= 0, see above). sr is still a Leader at step 1 and
    // appends its own client entries; at step 2 it learns the primary's higher
    // term — from the first peer its own round reaches when its id is lower
    // (one failed AppendEntries), else from the primary's AppendEntries — and
    // steps down (r_observe_term: Term, votedFor none, a new follower timer).
    // The primary's AppendEntries carries prevLogIndex NextIndex[sr]-1 = L0,
    // its length when it was elected (sr's row never moved while sr's
    // messages were dropped), so the entries it holds after L0 are of its own
    // term, above every term in sr's log. Taken when sr's entry L0 has the
    // primary's term (accepted) and the two logs differ at L0+1 (checked, one
    // ring read each): r_deliver_ae then truncates sr's log at L0 and appends
    // everything, so sr's log becomes the primary's — entries L0+1..Ll copied
    // from the primary's ring, this tick's written with everyone's.
    int sr_hw = 0, sr_dur = 0;
    if (RAFT && sr >= 0 && gom && !bail) {
      const int L0 = RW.at(PL_LNEXT, sr) - 1;
      const int ls = sel(last, sr), hws = RW.at(PL_HWM, sr), hwc = RW.at(PL_HWM, c);
      sr_hw = max(hws, ls + n);   // its high-water mark after its own client append
      const int Kd = int(P.K);
      // (n == 0 would leave sr's LastApplied out of the row stores below: general path)
      bail |= n == 0 || sel(term, sr) >= Lt || L0 < 0 || L0 > ls || L0 > Ll || int64_t(ls) + n > I32MAX ||
              hwc < Ll || (L0 >= 1 ? L0 : 1) <= max(hwc, Ll + n) - Kd ||   // NextIndex / prevLogTerm in the ring
              (L0 >= 1 ? L0 : 1) <= sr_hw - Kd;   // sr's entries L0 (prevLogTerm) and L0+1 (conflict) are read
      // every read this needs is issued at once (one round trip for the lane,
      // whose wave waits on it): sr's NextIndex for p0 and the terms of both
      // logs at L0 and L0+1 (the ring addresses are valid whatever the values)
      const uint64_t tb = ring_tile(g, P.KP, R);
      const uint32_t rot = GW.rot(), rota = GW.rota(), rotb = GW.rotb();
      const int sbo = GW.sb(), sb2 = GW.sb2();
      const int p0 = sr == 0 ? 1 : 0;   // the lowest-id peer: where sr's own round goes first
      const uint32_t o0 = ring_in_tile(g, R, ring_slot(L0, rot, rota, rotb, sbo, sb2, P.kmask), 0u);
      const uint32_t o1 = ring_in_tile(g, R, ring_slot(L0 + 1, rot, rota, rotb, sbo, sb2, P.kmask), 0u);
      const int32_t* const rt = P.log_term + tb;
      const int nx0 = at(prow(P.xnext, sr * R + p0, P.Gp), g);
      const int tc0 = ring_ld(rt, o0 + uint32_t(c)), ts0 = ring_ld(rt, o0 + uint32_t(sr));
      const int tc1 = ring_ld(rt, o1 + uint32_t(c)), ts1 = ring_ld(rt, o1 + uint32_t(sr));
      // sr's own round (sr < c) reaches p0 before it learns the higher term:
      // r_leader_round's NextIndex / prevLogTerm checks on sr's row must not fault
      if (sr < c) bail |= nx0 < 1 || nx0 > ls + n + 1 || (nx0 >= 2 ? nx0 - 1 : 1) <= sr_hw - Kd;
      // prevLogTerm: the primary's entry L0 against sr's (cached last-entry terms where they apply)
      if (L0 >= 1) bail |= (L0 == Ll ? Llt : tc0) != (L0 == ls ? sel(lt, sr) : ts0);
      // the first conflict must be at L0+1 (else r_deliver_ae skips the entries present);
      // sr's entry L0+1 is from its ring or the one its own client append adds this tick
      // (VX: sr's entries above L0 = xlo are virtual, of its own term)
      bail |= (L0 + 1 <= Ll ? tc1 : Lt) == ((L0 + 1 <= ls && !(meta & M_VX)) ? ts1 : sel(term, sr));
      // (the catch-up regenerates the primary's entries L0+1..Ll: they must
      // all be from the current run of consecutive calls, T.contig_q; with
      // staged client values nothing is regenerable and the catch-up reads
      // them from the primary's column instead — GetLogsFrom, main.go:357)
      if (!(meta & M_VX) && !P.cv) bail |= T.entries_before(T.tick) - uint64_t(Ll - L0) < T.contig_q;
      if (!bail) {
        df |= (1u << 21) | (ls > L0 ? 1u << 22 : 0u);   // class: stale leader's return (its log truncated at L0)
        // the primary's entries after L0 (at most K): copied below by the whole wave
        // (entries L0+1..Ll: the primary's own appends since its election, the
        // last one at the client tick before this one)
        // (VX: sr's column already holds them — every write of the primary's
        // entries since the election included it — so there is nothing to copy)
        jb_n = (meta & M_VX) ? 0 : Ll - L0;
        vxf |= (meta & M_VX) ? 1u : 0u;
        jb_from = L0 + 1;
        jb_col = uint32_t(sr);
        jb_term = Lt;
        jb_q0 = T.entries_before(T.tick) - uint64_t(jb_n);
        jb_kv = sm64(key ^ ((uint64_t(ST_VALUE) << 32) | uint32_t(c)));
        jb_scol = P.cv ? c : -1;   // (staged values: read from the primary's column, same slots)
        jb_rot = rot | (rota << 16);
        jb_rotb = rotb;
        jb_sb = sbo;
        jb_sb2 = sb2;
        sr_dur = T.f_min + int(uint32_t(rng_k(key, uint32_t(sr), ST_TIMER_F, uint64_t(T.tick)) >> 32) %
                               uint32_t(T.f_span));
        const int nl = Ll + n;
        put(last, sr, nl);
        const int cs = sel(commit, sr);
        if (Lc > cs) {   // min(leaderCommit, index of the last new entry)
          const int nc = Lc < nl ? Lc : nl;
          if (nc != cs) { put(commit, sr, nc); cch |= 1u << sr; }
        }
        ltch |= 1u << sr;   // its last entry is now one of the primary's term
        put(m, sr, nl);
        mch |= 1u << sr;
        okm |= 1u << sr;
      }
    }
    if (gom && !bail) {
      int cm = Lc;
      // (ONESTALE: the stale leader's row is explicit. A returning one is in
      // step after this tick — MatchIndex = its new length — and its
      // high-water mark, above its truncated log, goes in the plane: HWX)
      bool sync = !stale;
      bool hwx = false;               // RAFT: MSYNC with a high-water mark above its log's length (M_HWX)
      if constexpr (RAFT) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (!((hwup >> r) & 1u) || r == sr) continue;
          const int la = r == c ? Ll + n : last[r];   // (accepting followers' last already moved)
          if (RW.at(PL_HWM, r) > la) hwx = true;      // the plane holds it (exact: rows were explicit or HWX)
        }
        if (sr >= 0 && sr_hw > Ll + n) hwx = true;    // the returning stale leader's truncated log
      }
      if constexpr (RAFT) {
        // every log now ends at Ll+n (all but at most one lagging isolated
        // replica, and R >= 3): the majority index is Ll+n, committed only if
        // that entry is of the current term (this tick's entries are)
        const int N = Ll + n;
        if (N > Lc && (n > 0 || Llt == Lt)) cm = N;
      } else {
        // commit rule (main.go:381-391)
#pragma unroll
        for (int p = 0; p < R; ++p) {
          int cnt = 0;
#pragma unroll
          for (int q = 0; q < R; ++q) cnt += (q != c && m[q] == m[p]) ? 1 : 0;
          if (p != c && 2 * cnt > R && m[p] > cm) cm = m[p];
          sync &= (p == c) || m[p] == last[p];
        }
      }
      df |= (fresh ? 1u << 20 : 0u) | (stale ? 1u << 23 : 0u) | (xi >= 0 && !stale ? 1u << 26 : 0u) |
            (x_fire ? 1u << 27 : 0u) | (hwx || hwup ? 1u << 24 : 0u);   // classes taken this tick
      sv[0] = cm - Lc;
      sv[1] = __builtin_popcount(okm);
      sv[2] = (R - 1) - sv[1] + (stale ? R - 1 : 0) + (sr >= 0 && sr < c ? 1 : 0);   // + every AppendEntries of the
      // cut-off stale leader; a returning one with a lower id sends one (rejected) before stepping down
      sv[3] = 1;
      sv[4] = x_fire;
      // ---- stores (no bail past this point) ----
      // LastApplied / CommitIndex rows: one wide row store when every replica
      // changes (the steady state), else the changed elements
      const uint32_t all = (1u << R) - 1u;
      const uint32_t peers = all & ~(1u << c);
      // SSYNC after this tick: every follower accepted and every log ends at
      // Ll+n with an entry of term Lt (REF: an accepting follower takes Lt,
      // main.go:155; RAFT: terms were checked equal), the followers share one
      // CommitIndex, and the rows stay implicit (MSYNC)
      const int cf = sel(commit, c == 0 ? 1 : 0);
      bool keep_ss = R >= 2 && sync && !stale && xi < 0 && okm == peers && Ll + n > 0 && (n > 0 || Llt == Lt);
#pragma unroll
      for (int p = 0; p < R; ++p)
        if (p != c) keep_ss &= commit[p] == cf && last[p] == Ll + n && (n > 0 || lt[p] == Lt);
      if (keep_ss) {
        df |= 262144u;
        GW.ss() = SsRec{Ll + n, Lt, cm, cf};
        GW.st_hb(T.now);                                   // timer.Reset(d) of every follower
        if (RAFT && sr >= 0) {   // the returning stale leader stepped down: a follower (term, length: the record)
          RW.st(PL_RS, sr, int32_t(ROLE_F | (uint32_t(sr_dur) << 6)));   // votedFor none, new timer
          RW.st(PL_HWM, sr, sr_hw);   // (its timer starts now: hb)
        }
      } else {
      if (ss) {   // leaving the compressed form: the rows as they stood, then the element stores below
        const SsRec ss_rec = GW.ss();   // (re-read: rare, keeps it out of the live registers)
        const LxRec lxr = (RAFT && (meta & M_LXS)) ? GW.lx() : LxRec{0, 0};
        int trow[R], lrow[R], crow[R];
#pragma unroll
        for (int p = 0; p < R; ++p) {
          trow[p] = ss_rec.term; lrow[p] = ss_last(ss_rec, p, c, meta, lxr); crow[p] = p == c ? ss_rec.cl : ss_rec.cf;
        }
        RW.store(PL_TERM, trow);
        RW.store(PL_LAST, lrow);
        RW.store(PL_COMMIT, crow);
        RW.store(PL_LTERM, trow);
      }
      const bool last_row = n && okm == peers;
      const bool commit_row = cm != Lc && cch == peers;
      if (last_row || commit_row) {
        int lrow[R], crow[R];
#pragma unroll
        for (int p = 0; p < R; ++p) {
          lrow[p] = p == c ? Ll + n : last[p];
          crow[p] = p == c ? cm : commit[p];
        }
        if (last_row) RW.store(PL_LAST, lrow);
        if (commit_row) RW.store(PL_COMMIT, crow);
      }
      if (n) {
        if (!last_row) RW.st(PL_LAST, c, Ll + n);
        if (Llt != Lt) RW.st(PL_LTERM, c, Lt);
      }
      if (cm != Lc && !commit_row) RW.st(PL_COMMIT, c, cm);
      if (xi < 0) GW.st_hb(T.now);                         // timer.Reset(d) of every follower
#pragma unroll
      for (int p = 0; p < R; ++p) {
        if (p == c || !((okm >> p) & 1u)) continue;
        if (xi >= 0) RW.st(PL_TSTART, p, T.now);   // xi isolated: reset each receiver, not hb
        if (n && !last_row) RW.st(PL_LAST, p, last[p]);
        if (!sync && ((mch >> p) & 1u)) RW.st(PL_LMATCH, p, m[p]);
        if (((cch >> p) & 1u) && !commit_row) RW.st(PL_COMMIT, p, commit[p]);
        if ((ltch >> p) & 1u) RW.st(PL_LTERM, p, Lt);
        if (!RAFT && term[p] != Lt) RW.st(PL_TERM, p, Lt);  // main.go:155
        if (RAFT && !sync && ((mch >> p) & 1u)) RW.st(PL_LNEXT, p, m[p] + 1);   // NextIndex explicit too
        if (RAFT && !sync && n) {   // high-water mark = max(itself, new length)
          const int h = ((hwup >> p) & 1u) ? RW.at(PL_HWM, p) : 0;
          if (h < last[p]) RW.st(PL_HWM, p, last[p]);
        }
      }
      if constexpr (RAFT) {
        if (!sync && n) {   // the leader's high-water mark
          const int h = ((hwup >> c) & 1u) ? RW.at(PL_HWM, c) : 0;
          if (h < Ll + n) RW.st(PL_HWM, c, Ll + n);
        }
        if (stale) {
          // the stale leader's own client append (main.go:327-329) at its own log's end
          const int xl = sel(last, xi);
          if (n) {
            const uint64_t xvb = cv_base(P, key, uint32_t(xi), T.tick, g);
            const uint64_t tb = ring_tile(g, P.KP, R);
            const uint32_t xrot = GW.rot(), xrota = GW.rota(), xrotb = GW.rotb();
            const int xsb = GW.sb(), xsb2 = GW.sb2();
            uint32_t cs = 0;
            if constexpr (CRC) cs = crc_term_state(tab, x_term);
            // (VX: its entries are virtual — its column mirrors the primary's)
            for (int e = 0; e < ((meta & M_VX) ? 0 : n); ++e) {
              const int64_t v = cv_value(xvb, uint32_t(e), cv_stride(P));
              const uint32_t o = ring_in_tile(g, R, ring_slot(xl + 1 + e, xrot, xrota, xrotb, xsb, xsb2, P.kmask), uint32_t(xi));
              ring_stx<LIST>(P.log_term + tb, o, x_term);
              ring_stx<LIST>(P.log_value + tb, o, v);
              if constexpr (CRC) ring_stx<LIST>(P.log_crc + tb, o, crc_value_final(tab, cs, v));
            }
            RW.st(PL_LAST, xi, xl + n);
            if (sel(lt, xi) != x_term) RW.st(PL_LTERM, xi, x_term);
            if (RW.at(PL_HWM, xi) < xl + n) RW.st(PL_HWM, xi, xl + n);
          }
        }
        if (x_fire) {   // the isolated replica became / stays a candidate: Term+1, votedFor itself
          RW.st(PL_TERM, xi, x_term + 1);
          RW.st(PL_RS, xi, int32_t(ROLE_C | (uint32_t(xi + 1) << 2) | (uint32_t(x_dur) << 6)));
          RW.st(PL_TSTART, xi, T.now);
        }
        if (sr >= 0) {   // the returning stale leader stepped down: a follower of the primary's term
          RW.st(PL_TERM, sr, Lt);
          RW.st(PL_RS, sr, int32_t(ROLE_F | (uint32_t(sr_dur) << 6)));   // votedFor none
          RW.st(PL_TSTART, sr, T.now);
          RW.st(PL_HWM, sr, sr_hw);
        }
      }
      }   // !keep_ss
      // RAFT: MSYNC also makes NextIndex (= match+1) and the high-water marks (= last) implicit
      int nm = sync ? (meta | M_MSYNC) : (meta & ~M_MSYNC);
      nm = (sync && hwx) ? (nm | M_HWX) : (nm & ~M_HWX);
      if (RAFT && sync && hwx) {
        // HWX: the highest high-water mark, for the lean kernel, in glx (unused
        // by an HWX group, which is never LXS / SXS): it reads 8 B with the
        // group's other words instead of the R-wide hwm row after them
        int mx = RW.at(PL_HWM, 0);
#pragma unroll
        for (int r = 1; r < R; ++r) mx = max(mx, int(RW.at(PL_HWM, r)));
        GW.lx() = LxRec{mx, 0};
      }
      nm &= ~M_LXS;   // (a fresh record when compressed: every log at Ll+n)
      nm = keep_ss ? (nm | M_SSYNC) : (nm & ~M_SSYNC);
      if (x_fire) nm = (nm & ~M_STEADY) | M_ONECAND;
      if (sr >= 0) nm = (nm & ~M_ONESTALE) | M_STEADY;   // one leader, every other replica a follower
      // (a virtual suffix lives only with a cut-off leader: LXS / ONESTALE;
      // the return truncates it away, and any other way out of those forms
      // bailed above while the suffix was non-empty)
      if (!(nm & (M_LXS | M_ONESTALE))) nm &= ~M_VX;
      // SXS after this tick (RAFT; the rows were stored explicitly above and are
      // now stale but for the stale leader's): every follower of the primary
      // accepted, every log but the stale leader's ends at Ll+n with an entry
      // of term Lt, the followers share one CommitIndex; the stale leader
      // (term Lt-1, its last entry of that term) only appended to its own log
      if constexpr (RAFT && !CRC) {
        if (stale && !hwx && R >= 3 && okm == (peers & ~(1u << xi)) && Ll + n > 0 && (n > 0 || Llt == Lt) &&
            x_term == Lt - 1 && (n > 0 || sel(lt, xi) == x_term)) {
          const int f = (c != 0 && xi != 0) ? 0 : ((c != 1 && xi != 1) ? 1 : 2);   // any follower of the primary
          const int cf = sel(commit, f);
          bool sx = true;
#pragma unroll
          for (int p = 0; p < R; ++p)
            if (p != c && p != xi) sx &= commit[p] == cf && last[p] == Ll + n && (n > 0 || lt[p] == Lt);
          if (sx) {
            GW.ss() = SsRec{Ll + n, Lt, cm, cf};
            GW.lx() = LxRec{sel(last, xi) + n - (Ll + n), xi};
            GW.st_hb(T.now);   // (the stale leader's timer ignores hb: a leader's start is its own)
            nm |= M_SSYNC | M_MSYNC;
            df |= 1u << 30;   // class: entered SXS
          }
        }
      }
      if (nm != meta_st) GW.meta() = uint16_t(nm);
      // this tick's entries go to the leader log + every follower that accepted
      if (n) {
        bool same = true;   // every writer appends at Ll+1 (REF: a follower's log may run past its MatchIndex)
#pragma unroll
        for (int p = 0; p < R; ++p)
          if (((okm >> p) & 1u) && last[p] - n != Ll) same = false;
        const uint64_t vb = cv_base(P, key, uint32_t(c), T.tick, g);
        // ring rotation: index i at slot (i-1+rot) mod K; an empty group's first
        // entry goes to the global phase (its logs hold nothing to move)
        int rot = GW.rot();
        if (empty) {
          const int r0 = int(T.entries_before(T.tick) & P.kmask);
          if (r0 != rot) { rot = r0; GW.rot() = uint16_t(rot); }
        }
        if (same) {
          wr = okm | (1u << c);
          if (stale && (meta & M_VX)) wr |= 1u << xi;   // VX: the stale leader's column mirrors the primary's
          w_term = Lt;
          w_ph = (Ll + rot) & int(P.kmask);
          w_vb = vb;
          // out of the global phase (logs stood still while leaderless):
          // switch the ring segment in place when that is safe (ring_slot)
          const int ph = int(T.entries_before(T.tick) & P.kmask);
          const uint32_t d = uint32_t(ph - w_ph) & P.kmask;
          if (d != 0u) df |= d <= P.K ? 8u : 16u;
          // A stale leader cut off this tick (RAFT, typically the new leader's
          // first round: the followers' logs stood still while the old leader
          // appended alone in the global phase) holds entries above Ll: they
          // are moved to the new segment's slots (placement only) by the wave
          // below, so that the primary and its followers append in the global
          // phase from now on (whole ring rows) and the stale leader alone
          // writes out of phase.
          if (P.KP > P.K && d != 0u && d <= P.K && Ll > 0 && sr < 0) {
            int lo = Ll, hi = Ll;   // log lengths before this tick (== high-water marks on this path)
#pragma unroll
            for (int p = 0; p < R; ++p) {
              const int pre = (p != c && ((okm >> p) & 1u)) ? last[p] - n : last[p];
              lo = min(lo, pre);
              if (!(stale && p == xi)) hi = max(hi, pre);
            }
            const int xtop = stale ? sel(last, xi) + n : 0;   // the stale leader's length after this tick
            const int sbo = GW.sb();
            const uint32_t rota = GW.rota();
            // (a stale leader's entries above Ll are moved by regenerating them:
            // only when they are all from the current run of calls, T.contig_q;
            // with staged values by reading them from their old slots, all in
            // the current segment (sb <= Ll+1); else no switch — placement
            // only, the entries stay where they are)
            const bool mv_ok = P.cv ? sbo <= Ll + 1
                                    : T.entries_before(T.tick + 1) - uint64_t(xtop - Ll) >= T.contig_q;
            const bool ok = ring_switch_ok(d, uint32_t(rot), rota, sbo, GW.sb2(), lo, P.K, P.kmask) &&
                            xtop - Ll <= int(P.K) && !(stale && xtop > Ll && !(meta & M_VX) && !mv_ok);
            df |= hi > Ll ? 64u : 0u;
            df |= ok ? 0u : 128u;
            if (hi <= Ll && ok) {
              df |= 32u | ((sbo <= 1 || sbo <= lo - int(P.K) + 1) ? 0u : 1u << 25);   // (+ the previous segment stays live)
              // (VX: the stale leader's entries are virtual: nothing to move)
              if (stale && xtop > Ll && !(meta & M_VX)) {   // its entries Ll+1..xtop: slot (i-1+rot) -> (i-1+rot+d)
                // (its entries above Ll: its own appends since it was cut off,
                // the last ones this tick; every index uses the new rotation)
                jb_n = xtop - Ll;
                jb_from = Ll + 1;
                jb_col = uint32_t(xi);
                jb_term = x_term;
                jb_q0 = T.entries_before(T.tick + 1) - uint64_t(jb_n);
                jb_kv = sm64(key ^ ((uint64_t(ST_VALUE) << 32) | uint32_t(xi)));
                jb_scol = P.cv ? xi : -1;   // (staged values: read from its old slot, d back)
                jb_sd = int(d);
                jb_rot = uint32_t((rot + int(d)) & int(P.kmask));
                jb_rotb = 0;
                jb_sb = -2147483647 - 1;
                jb_sb2 = -2147483647 - 1;
                df |= 1u << 31;
              }
              GW.rotb() = uint16_t(rota);   // the three segments shift
              GW.sb2() = sbo;
              GW.rota() = uint16_t(rot);
              GW.sb() = Ll + 1;
              rot = (rot + int(d)) & int(P.kmask);
              GW.rot() = uint16_t(rot);
              w_ph = ph;
            }
          }
        } else {   // rare: write here, each replica at its own LastApplied+1+e
          const uint64_t tb = ring_tile(g, P.KP, R);
          const uint32_t rota = GW.rota(), rotb = GW.rotb();
          const int sb = GW.sb(), sb2 = GW.sb2();
          uint32_t cs = 0;
          if constexpr (CRC) cs = crc_term_state(tab, Lt);
          for (int e = 0; e < n; ++e) {
            const int64_t v = cv_value(vb, uint32_t(e), cv_stride(P));
            uint32_t stamp = 0;
            if constexpr (CRC) stamp = crc_value_final(tab, cs, v);
            // (VX: the stale leader's column mirrors the primary's entries)
            const uint32_t mir = (stale && (meta & M_VX)) ? 1u << xi : 0u;
#pragma unroll
            for (int p = 0; p < R; ++p) {
              if (p != c && !((okm >> p) & 1u) && !((mir >> p) & 1u)) continue;
              const int i0 = (p == c || ((mir >> p) & 1u)) ? Ll : last[p] - n;
              const uint32_t o = ring_in_tile(g, R, ring_slot(i0 + e + 1, uint32_t(rot), rota, rotb, sb, sb2, P.kmask), uint32_t(p));
              ring_stx<LIST>(P.log_term + tb, o, Lt);
              ring_stx<LIST>(P.log_value + tb, o, v);
              if constexpr (CRC) ring_stx<LIST>(P.log_crc + tb, o, stamp);
            }
          }
        }
      }
    }
    if (bail) GW.meta() = uint16_t(meta_st | M_DEFER);
    else if (giso_w >= 0) GW.iso() = uint8_t(giso_w);   // a leader-isolation window decided this tick
    df |= (!bail && giso_w >= 0) ? 1u << 28 : 0u;
    stored = !skip && !bail;
  }
  if (LIST && (P.diag & 128u)) {   // timing only (results wrong): the per-group code alone
    wr = 0; jb_n = 0;
  }
  if (LIST && (P.diag & 512u)) {   // timing only (results wrong): no entry copies or moves
    jb_n = 0;
  }
  // ---- this tick's log entries into the rings (all lanes of the wave) ----
  // Ring row of one slot = 64 lanes x R replicas, contiguous. The lanes of
  // the wave that append at the wave's common slot s0 (logs in step: the
  // steady state; groups that drifted apart under churn do not) write whole
  // rows cooperatively: store k covers row elements k*64 + lane, i.e. (group
  // lane (k*64+lane)/R, replica (k*64+lane)%R), whose term/value/stamp come
  // from that group's lane by shuffle — R contiguous stores per plane and
  // entry. Every other writing lane stores its own R-contiguous segment.
  // s0: the global phase entries_before(tick) (groups rotated at their first
  // entry, init_steady) or the first writer's slot, whichever more lanes share.
  // Entry jobs (RAFT, see jb_*): every entry of all the wave's jobs is
  // spread over its lanes (CPS per lane and pass), regenerated from the trace
  // RNG and stored after this tick's own entries — no ring reads (round 5:
  // reading them back cost two scattered line fetches per entry, a quarter of
  // C4's tick in a diagnostic run). A move's new slots never hold a live entry
  // of its column (ring_switch_ok), and copy and move never meet in one group
  // (a switch needs sr < 0).
  constexpr int CPS = 4;   // entries per lane and pass
  WPROF(wp1 = __builtin_amdgcn_s_memtime(); uint64_t wg = 0, wo = 0, wsc = 0;)
  constexpr bool JOBS = RAFT || CRC;   // (entry jobs: RAFT returns / moves, REF + CRC lagging followers)
  int jn = 0, jpre = 0, jtot = 0;   // this lane's job size, exclusive wave prefix, wave total
  if constexpr (JOBS) {
    jn = jb_n;
    jpre = jn;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {   // inclusive scan
      const int y = __shfl_up(jpre, o);
      if (int(threadIdx.x & 63) >= o) jpre += y;
    }
    jtot = __shfl(jpre, 63);
    jpre -= jn;
  }
  const int passes = JOBS ? (jtot + 64 * CPS - 1) / (64 * CPS) : 0;   // (wave-uniform)
  // jobs that read entries (staged values; a lagging follower's catch-up)
  // may read what this wave wrote in its previous step (pipelined list
  // kernel) from other lanes: those stores complete before the job's loads
  // (which bypass L1)
  if (JOBS && passes > 0 && __ballot(jb_scol >= 0)) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  for (int pass_i = 0; pass_i < (passes > 0 ? passes : 1); ++pass_i) {
    int32_t ct[CPS];
    int64_t cv[CPS];
    uint32_t cdst[CPS];      // destination element offset inside the ring (64-bit tile base below)
    uint64_t ctb[CPS];
    bool con[CPS];
    if constexpr (JOBS) {
      const int lane = threadIdx.x & 63;
#pragma unroll
      for (int k = 0; k < CPS; ++k) {
        const int e = pass_i * 64 * CPS + k * 64 + lane;
        con[k] = e < jtot;
        ct[k] = 0; cv[k] = 0; cdst[k] = 0; ctb[k] = 0;
        // owner: the last lane whose prefix is <= e (its job holds entry e)
        int o = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)
          if (__shfl(jpre, o + step) <= e) o += step;
        const int j0 = e - __shfl(jpre, o);
        // (every shuffle unconditional: a shuffle reading a lane that is off
        // in a divergent branch returns 0)
        const int from = __shfl(jb_from, o), term = __shfl(jb_term, o);
        const uint32_t col = uint32_t(__shfl(int(jb_col), o));
        const uint32_t gg = uint32_t(__shfl(int(g), o));
        const uint32_t rr = uint32_t(__shfl(int(jb_rot), o)), rb = uint32_t(__shfl(int(jb_rotb), o));
        const int sb_ = __shfl(jb_sb, o), sb2_ = __shfl(jb_sb2, o);
        const uint64_t q0 = (uint64_t(uint32_t(__shfl(int(uint32_t(jb_q0 >> 32)), o))) << 32) |
                            uint32_t(__shfl(int(uint32_t(jb_q0)), o));
        const uint64_t kv = (uint64_t(uint32_t(__shfl(int(uint32_t(jb_kv >> 32)), o))) << 32) |
                            uint32_t(__shfl(int(uint32_t(jb_kv)), o));
        const int scol = __shfl(jb_scol, o), sd = __shfl(jb_sd, o), jnn = __shfl(jn, o);
        // a move read from its old slots goes from the top down: entry i's new
        // slot is entry i+d's old one, so every entry is read (this pass, or
        // an earlier one) before a lower one overwrites its old slot
        const int j = (scol >= 0 && sd != 0) ? jnn - 1 - j0 : j0;
        if (con[k]) {
          ct[k] = term;
          ctb[k] = ring_tile(gg, P.KP, R);
          const uint32_t ds = ring_slot(from + j, rr & 0xFFFFu, rr >> 16, rb, sb_, sb2_, P.kmask);
          cdst[k] = ring_in_tile(gg, R, ds, col);
          if (scol >= 0) {   // the entry read from column scol, sd slots back (a return or a lagging
                             // follower: the leader's column, same slot; a move: its own column, its old slot)
            const uint32_t so = ring_in_tile(gg, R, (ds - uint32_t(sd)) & P.kmask, uint32_t(scol));
            ct[k] = ring_ld(P.log_term + ctb[k], so);
            cv[k] = ring_ld(P.log_value + ctb[k], so);
          } else {
            // global client entry q: tick (q / E) * period, entry q mod E of that tick
            const uint64_t q = q0 + uint64_t(j);
            const uint64_t qt = T.entries == 1u ? q : q / T.entries;
            const uint32_t qe = T.entries == 1u ? 0u : uint32_t(q - qt * T.entries);
            cv[k] = int64_t(sm64(sm64(kv ^ (qt * T.period)) ^ uint64_t(qe)) >> 1);
          }
        }
      }
    }
    WPROF(uint64_t wq0 = __builtin_amdgcn_s_memtime(); if constexpr (JOBS) { int z = 0; for (int k = 0; k < CPS; ++k) z += ct[k]; if (__ballot(z == 0x7FFFFFFF)) wg += 1; } uint64_t wq1 = __builtin_amdgcn_s_memtime(); wg += wq1 - wq0;)
    // Batches of at least LIST_COOP entries (C5: 64) are written by the whole
    // wave, one group at a time, one entry per lane: the lane-per-group loop
    // had each store instruction touch 64 groups' ring tiles (256-512 KB
    // apart) — 64 address translations per instruction; C5V's list kernel
    // spent 615K of a step's 650K cycles in those stores (tools/list_prof.py,
    // profiles/r06/t/). One group's batch spans a few KB of one tile.
    constexpr int LIST_COOP = 8;
    const bool coop_w = LIST && pass_i == 0 && n >= LIST_COOP;   // (wave-uniform)
    const bool kept = !RAFT && CRC && wr != 0 && shf >= 0;
    if (coop_w) {
      const int lane = int(threadIdx.x & 63);
      for (uint64_t bm = __ballot(wr != 0); bm; bm &= bm - 1) {
        const int src = int(__builtin_ctzll(bm));
        const uint32_t gs = uint32_t(__shfl(int(g), src));
        const int ts = __shfl(w_term, src), phs = __shfl(w_ph, src);
        const uint32_t ws = uint32_t(__shfl(int(wr), src));
        const bool ks = __shfl(int(kept), src) != 0;
        const uint64_t vbs = (uint64_t(uint32_t(__shfl(int(uint32_t(w_vb >> 32)), src))) << 32) |
                             uint32_t(__shfl(int(uint32_t(w_vb)), src));
        uint32_t cs = 0;
        if constexpr (CRC) cs = crc_term_state(tab, ts);
        if (ks) {   // a group kept in shared form: one shared copy (see below)
          const uint64_t shb = sh_tile(gs, P.KP);
          for (int e = lane; e < n; e += 64) {
            const int64_t v = cv_value(vbs, uint32_t(e), cv_stride(P));
            const uint32_t so = sh_in_tile(gs, uint32_t((phs + e) & int(P.kmask)), P.sh_cs);
            P.sh_term[shb + so] = ts;
            P.sh_value[shb + so] = v;
            if constexpr (CRC) P.sh_crc[shb + so] = crc_value_final(tab, cs, v);
          }
        } else {    // its own R-contiguous segment per entry
          const uint64_t tb = ring_tile(gs, P.KP, R);
          int32_t* const rt = P.log_term + tb;
          int64_t* const rv = P.log_value + tb;
          uint32_t* const rc = CRC ? P.log_crc + tb : nullptr;
          for (int e = lane; e < n; e += 64) {
            const int64_t v = cv_value(vbs, uint32_t(e), cv_stride(P));
            uint32_t stamp = 0;
            if constexpr (CRC) stamp = crc_value_final(tab, cs, v);
            const uint32_t o = ring_in_tile(gs, R, uint32_t((phs + e) & int(P.kmask)), 0u);
            if (ws == (1u << R) - 1u) {
              fill_segx<LIST, R>(rt + o, ts);
              fill_segx<LIST, R>(rv + o, v);
              if constexpr (CRC) fill_segx<LIST, R>(rc + o, stamp);
            } else {
#pragma unroll
              for (int p = 0; p < R; ++p) {
                if (!((ws >> p) & 1u)) continue;
                ring_stx<LIST>(rt, o + p, ts);
                ring_stx<LIST>(rv, o + p, v);
                if constexpr (CRC) ring_stx<LIST>(rc, o + p, stamp);
              }
            }
          }
        }
      }
      if (wr != 0) df |= 512u;
    } else if (LIST && pass_i == 0 && n && kept) {
      // a group kept in shared form (DevPlanes::sh_keep): this tick's entries
      // are the leader's, held by every replica that accepted them (and, once
      // it catches up, by a follower that rejected its copy): one shared copy
      const uint64_t shb = sh_tile(g, P.KP);
      const uint32_t cs = crc_term_state(tab, w_term);
      for (int e = 0; e < n; ++e) {
        const int64_t v = cv_value(w_vb, uint32_t(e), cv_stride(P));
        const uint32_t so = sh_in_tile(g, uint32_t((w_ph + e) & int(P.kmask)), P.sh_cs);
        P.sh_term[shb + so] = w_term;
        P.sh_value[shb + so] = v;
        P.sh_crc[shb + so] = crc_value_final(tab, cs, v);
      }
    } else if (LIST && pass_i == 0 && n && wr != 0) {   // this tick's entries: scattered groups, each lane its own R-contiguous segment
      const uint64_t tb = ring_tile(g, P.KP, R);
      int32_t* const rt = P.log_term + tb;
      int64_t* const rv = P.log_value + tb;
      uint32_t* const rc = CRC ? P.log_crc + tb : nullptr;
      df |= 512u;
      uint32_t cs = 0;
      if constexpr (CRC) cs = crc_term_state(tab, w_term);
      for (int e = 0; e < n; ++e) {
        const int64_t v = cv_value(w_vb, uint32_t(e), cv_stride(P));
        uint32_t stamp = 0;
        if constexpr (CRC) stamp = crc_value_final(tab, cs, v);
        const uint32_t o = ring_in_tile(g, R, uint32_t((w_ph + e) & int(P.kmask)), 0u);
        if (wr == (1u << R) - 1u) {   // every replica appends: R-wide vector stores
          fill_segx<LIST, R>(rt + o, w_term);
          fill_segx<LIST, R>(rv + o, v);
          if constexpr (CRC) fill_segx<LIST, R>(rc + o, stamp);
        } else {
#pragma unroll
          for (int p = 0; p < R; ++p) {
            if (!((wr >> p) & 1u)) continue;
            ring_stx<LIST>(rt, o + p, w_term);
            ring_stx<LIST>(rv, o + p, v);
            if constexpr (CRC) ring_stx<LIST>(rc, o + p, stamp);
          }
        }
      }
    }
    WPROF(uint64_t wq2 = __builtin_amdgcn_s_memtime(); wo += wq2 - wq1;)
    if constexpr (JOBS) {
#pragma unroll
      for (int k = 0; k < CPS; ++k) {
        if (!con[k]) continue;
        ring_stx<LIST, int32_t, 3>(P.log_term + ctb[k], cdst[k], ct[k]);
        ring_stx<LIST, int64_t, 3>(P.log_value + ctb[k], cdst[k], cv[k]);
        if constexpr (CRC)
          ring_stx<LIST, uint32_t, 3>(P.log_crc + ctb[k], cdst[k], crc_value_final(tab, crc_term_state(tab, ct[k]), cv[k]));
      }
    }
    WPROF(wsc += __builtin_amdgcn_s_memtime() - wq2;)
  }
  WPROF(wp2 = __builtin_amdgcn_s_memtime();)
  if (!LIST && n) {
    const uint64_t wball = __ballot(wr != 0);
    if (wball) {
      const int lane = threadIdx.x & 63;
      // the tile base is wave-uniform (blocks are whole waves of consecutive groups)
      const uint64_t tb = ring_tile(__builtin_amdgcn_readfirstlane(g), P.KP, R);
      int32_t* const rt = P.log_term + tb;
      int64_t* const rv = P.log_value + tb;
      uint32_t* const rc = CRC ? P.log_crc + tb : nullptr;
      const int sa = __shfl(w_ph, int(__builtin_ctzll(wball)));
      const int sb = int(T.entries_before(T.tick) & P.kmask);
      const int na = __popcll(__ballot(wr != 0 && w_ph == sa)), nb = __popcll(__ballot(wr != 0 && w_ph == sb));
      const int s0 = nb >= na ? sb : sa;
      const bool coop = wr != 0 && w_ph == s0;
      df |= coop ? 256u : (wr != 0 ? 512u : 0u);
      uint32_t cs = 0;
      if constexpr (CRC) cs = crc_term_state(tab, w_term);
      {
        int k_term[R];
        uint32_t k_on[R];
        int k_src[R];
        const int cwr = coop ? int(wr) : 0;
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int j = k * 64 + lane;
          const int src = j / R, rr = j - src * R;
          k_src[k] = src;
          k_term[k] = __shfl(w_term, src);
          k_on[k] = (uint32_t(__shfl(cwr, src)) >> rr) & 1u;
        }
        for (int e = 0; e < n; ++e) {
          const int64_t v = cv_value(w_vb, uint32_t(e), cv_stride(P));
          uint32_t stamp = 0;
          if constexpr (CRC) stamp = crc_value_final(tab, cs, v);
          const uint32_t row = uint32_t((s0 + e) & int(P.kmask)) * 64u * R;
          const int vlo = int(uint32_t(uint64_t(v))), vhi = int(uint32_t(uint64_t(v) >> 32));
#pragma unroll
          for (int k = 0; k < R; ++k) {
            const int lo = __shfl(vlo, k_src[k]), hi = __shfl(vhi, k_src[k]);
            uint32_t sk = 0;
            if constexpr (CRC) sk = uint32_t(__shfl(int(stamp), k_src[k]));
            if (k_on[k]) {
              const uint32_t o = row + uint32_t(k * 64 + lane);
              ring_stx<LIST>(rt, o, k_term[k]);
              ring_stx<LIST>(rv, o, int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo)));
              if constexpr (CRC) ring_stx<LIST>(rc, o, sk);
            }
          }
          if (wr != 0 && !coop) {   // drifted lane: its own segment
            const uint32_t o = ring_in_tile(g, R, uint32_t((w_ph + e) & int(P.kmask)), 0u);
            if (wr == (1u << R) - 1u) {   // every replica appends: R-wide vector stores
              fill_segx<LIST, R>(rt + o, w_term);
              fill_segx<LIST, R>(rv + o, v);
              if constexpr (CRC) fill_segx<LIST, R>(rc + o, stamp);
            } else {
#pragma unroll
              for (int p = 0; p < R; ++p) {
                if (!((wr >> p) & 1u)) continue;
                ring_stx<LIST>(rt, o + p, w_term);
                ring_stx<LIST>(rv, o + p, v);
                if constexpr (CRC) ring_stx<LIST>(rc, o + p, stamp);
              }
            }
          }
        }
      }
    }
  }
#ifndef RAFTSTEP_WAVE_PROF
  if (P.dbg) {   // diagnostics: lanes per class, one atomic per wave and class
    df |= bail ? 2u : 0u;
    df |= (g < P.G) ? 1024u : 0u;
    DIAG_REASON(if (bail && !(df & (2048u | 4096u | 8192u | 16384u))) df |= 32768u;);   // reason: anything later
    DIAG_REASON(if (!bail) df &= ~(2048u | 4096u | 8192u | 16384u););
    if (bail) df &= ~0x7FF80000u;   // the class bits 19-30 count taken ticks only
    if (bail) vxf = 0u;
#pragma unroll 1
    for (int k = 0; k < 32; ++k) {
      const uint64_t b = __ballot((df >> k) & 1u);
      if ((threadIdx.x & 63) == 0 && b) atomicAdd(&P.dbg[32 + k], (unsigned long long)__popcll(b));
    }
#pragma unroll 1
    for (int k = 0; k < 2; ++k) {   // (the VX classes: lean-range slots 28, 29)
      const uint64_t b = __ballot((vxf >> k) & 1u);
      if ((threadIdx.x & 63) == 0 && b) atomicAdd(&P.dbg[28 + k], (unsigned long long)__popcll(b));
    }
  }
#endif
  // groups that need the general path go to the sharded worklist: dense
  // launch, block-local prefix over the wave ballots and one atomic on the
  // block's shard; list launch (scattered groups), one atomic per deferred
  // lane on its group's shard
  if constexpr (LIST) {
    if (bail) {
      const uint32_t k = shard_home(g, P.shard_sb);
      const uint32_t off = k * P.scap + atomicAdd(&work_count[k * SHARD_STRIDE], 1u);
      work[off] = g;
      work_tick[off] = int32_t(T.tick);
    }
  } else {
    __shared__ uint32_t wn[4], wbase;
    const uint64_t bm = __ballot(bail);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t k = shard_of_block(blockIdx.x, P.shard_sb);   // == shard_home(g)
    if (lane == 0) wn[wave] = uint32_t(__popcll(bm));
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t tot = wn[0] + wn[1] + wn[2] + wn[3];
      wbase = tot ? atomicAdd(&work_count[k * SHARD_STRIDE], tot) : 0u;
    }
    __syncthreads();
    if (bail) {
      uint32_t off = k * P.scap + wbase + uint32_t(__popcll(bm & ((1ull << lane) - 1ull)));
      for (int w = 0; w < wave; ++w) off += wn[w];
      work[off] = g;
      work_tick[off] = int32_t(T.tick);
    }
  }
  if (stats) {
    if constexpr (RAFT) {
      const int idx[7] = {S_COMMITTED, S_AE_OK, S_AE_FAIL, S_LEADER_GROUPS, S_BUMPS, S_VOTES, S_WON};
      block_stats<7>(sv, idx, stats);
    } else {
      const int idx[4] = {S_COMMITTED, S_AE_OK, S_AE_FAIL, S_LEADER_GROUPS};
      const int v4[4] = {sv[0], sv[1], sv[2], sv[3]};
      block_stats<4>(v4, idx, stats);
    }
  }
  WPROF(if (LIST && P.dbg) {
    wp3 = __builtin_amdgcn_s_memtime();
    wprof_add(P.dbg, 32, wp1 - wp0); wprof_add(P.dbg, 33, wg); wprof_add(P.dbg, 34, wo); wprof_add(P.dbg, 35, wsc);
    wprof_add(P.dbg, 36, wp3 - wp2); wprof_add(P.dbg, 37, 1);
  })
  return stored;
}

// EXT CRC32C tables (8 KiB) staged in LDS for the stamp/verify lookups
template <bool CRC>
__device__ __forceinline__ void stage_crc_tab(const DevPlanes& P, uint32_t* tab) {
  if constexpr (CRC) {
    const uint4* src = reinterpret_cast<const uint4*>(P.crc_tab);
    uint4* dst = reinterpret_cast<uint4*>(tab);
    for (uint32_t i = threadIdx.x; i < 512u; i += blockDim.x) dst[i] = src[i];   // (blocks of 64..256 lanes)
    __syncthreads();
  }
}

// Every group, one lane each (the single-pass plan).
template <int R, bool CRC, int SEM>
__global__ __launch_bounds__(256) void tick_fast_kernel(DevPlanes P, Trace T, unsigned long long* stats,
                                                        uint32_t* work, int32_t* work_tick, uint32_t* work_count,
                                                        int force_slow) {
  __shared__ uint32_t tab[CRC ? 2048 : 1];
  stage_crc_tab<CRC>(P, tab);
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  if (g < P.G) sh_materialize<R>(P, g, T.at_tick(T.tick - 1).now);   // (ROT_SH: a group the lean kernel left in shared form)
  fast_group<R, CRC, SEM, false>(P, T, stats, work, work_tick, work_count, force_slow, g, tab,
                                     rows_global<R>(P, g), words_global(P, g));
}

// The groups the lean kernel passed on (list[0 .. *count)), grid-striding
// with a resident grid; zeroes the other parity's list counter (the next
// tick's lean kernel appends there). Listed groups are scattered, so a lane
// reading its group's rows and per-group words from HBM would issue ~25
// dependent, uncoalesced requests. Instead each block stages the records of
// its 256 groups into LDS with coalesced loads (consecutive lanes read
// consecutive 16-B pieces of one record: recw*4 contiguous bytes per group) plus
// each lane's per-group words (meta, heartbeat, isolation victims, ring
// rotation/segment, compressed record), runs fast_group on the LDS copies
// (RowAcc / WordAcc over the __shared__ arrays: ds_ instructions), and
// writes back the records
// it may have changed (coalesced) and the per-group words that did change.
// Active lanes per wave of the list kernel: the listed groups of a tick are
// few (C4: ~50K of 4M) and the kernel is latency-bound (a chain of dependent
// loads per group), so spreading them over more waves, each with fewer
// groups, puts more of those chains in flight at once.
#ifndef RAFTSTEP_LIST_LANES
#define RAFTSTEP_LIST_LANES 64
#endif
constexpr uint32_t LIST_LANES = RAFTSTEP_LIST_LANES;
static_assert(LIST_LANES >= 1 && LIST_LANES <= 64, "active lanes per wave");

template <int R, bool CRC, int SEM, int LB>
__global__ __launch_bounds__(LB) void tick_list_kernel(DevPlanes P, Trace T, unsigned long long* stats,
                                                        uint32_t* work, int32_t* work_tick, uint32_t* work_count,
                                                        const uint32_t* list, const uint32_t* count,
                                                        uint32_t* next_count, int steps, ListNext nx) {
  constexpr uint32_t RW = recw<R>();   // words per group record (16-B multiple)
  constexpr uint32_t RQ = RW / 4;      // 16-B pieces per record
  __shared__ uint32_t tab[CRC ? 2048 : 1];
  __shared__ uint32_t pre[NSHARD + 1];
  __shared__ int4 srec4[LB * RQ];
  int32_t* const srec = reinterpret_cast<int32_t*>(srec4);
  __shared__ uint32_t sg[LB];
  __shared__ SsRec sgss[LB];
  __shared__ int32_t shb[LB];
  __shared__ uint16_t smeta[LB], sgrot[LB];
  __shared__ LxRec sglx[LB];
  __shared__ uint8_t sgiso[LB];
  __shared__ uint16_t sgrota[LB], sgrotb[LB];
  __shared__ int32_t sgsb[LB], sgsb2[LB];
  __shared__ uint32_t sdm[LB];   // dirty rows, then dirty 16-B pieces, of each lane's record
  __shared__ uint32_t skey[LB];  // (form key, slot), sorted (P.list_sort)
  __shared__ int32_t sshk[LB];   // fast_group's `shf` of each slot
  constexpr uint32_t GPB = uint32_t(LB) / 64u * LIST_LANES;   // groups per block and round
  shard_zero(next_count);
  const uint32_t n = shard_prefix(count, pre);
  if (blockIdx.x * GPB >= n || (P.diag & 256u)) return;   // (diag 256, timing only: no list work at all)
  stage_crc_tab<CRC>(P, tab);
  const uint32_t t = threadIdx.x;
  const uint32_t lane = t & 63u;
  WPROF(const uint64_t wk0 = __builtin_amdgcn_s_memtime(); uint64_t wk1 = 0, wk2 = 0, wk3 = 0, wk4 = 0;)
  for (uint32_t base = blockIdx.x * GPB; base < n; base += gridDim.x * GPB) {
    WPROF(const uint64_t wi0 = __builtin_amdgcn_s_memtime();)
    const uint32_t i = base + (t >> 6) * LIST_LANES + lane;
    const bool in = lane < LIST_LANES && i < n;
    const uint32_t slot = in ? shard_locate(pre, P.scap, i) : 0u;
    const uint32_t g = in ? list[slot] : 0xFFFFFFFFu;
    const bool valid = g < P.G;
    sg[t] = g;
    // (each is a separate scattered line per group, all loaded in the same
    // round trip; the ring segment words too: a return or a segment switch
    // is in most waves of a churn tick, and reading them from HBM there put
    // one more dependent round trip on every such wave's critical path)
    uint16_t m0 = 0, r0 = 0, ra0 = 0, rb0 = 0;
    int32_t sb0 = 0, sc0 = 0;
    uint8_t gi0 = 0;
    int32_t hb0 = 0;
    SsRec ss0{0, 0, 0, 0};
    // glx is staged only when the group's form uses it; otherwise a sentinel
    // no real record equals, so that any record the tick writes (LXS / SXS
    // entry, whatever its value) is written back
    LxRec lx0{-2147483647 - 1, -2147483647 - 1};
    int shf0 = 0;   // SH: the group's first shared index (ROT_SH)
    if (valid) {
      // gmeta, grot, gsb and gss from the list entry (the lean kernel's reads,
      // LIST_WORDS: coalesced by slot), the other words from their planes
      const uint64_t cap = uint64_t(NSHARD) * P.scap;
      uint32_t* const lst = const_cast<uint32_t*>(list);
      const uint32_t mr = list_mr(lst, cap)[slot];
      m0 = uint16_t(mr); r0 = uint16_t(mr >> 16); ss0 = list_ss(lst, cap)[slot];
      sb0 = P.KP > P.K ? list_sb(lst, cap)[slot] : at(P.gsb, g);
      hb0 = at(P.hb, g);
      const GSeg cw = P.gseg[g];   // the cold words, one 16-B load (GSeg)
      ra0 = cw.rota; rb0 = cw.rotb; sc0 = cw.sb2;
      // giso only where fast_group reads it: leader-isolation mode, a window
      // of the group active at this tick or (two steps) the next one
      if (T.iso_p && T.iso_leader) {
        const uint64_t key = group_key(T.seed, P.gbase + g);
        uint32_t a0 = 0, a1 = 0, s0 = 0;
        iso_windows<R>(key, T, &a0, &s0);
        if (steps > 1) iso_windows<R>(key, T.at_tick(T.tick + 1), &a1, &s0);
        if (a0 | a1) gi0 = at(P.giso, g);
      }
      if (uses_glx(m0)) lx0 = P.glx[g];
      shf0 = cw.shf;
    }
    // a group the lean kernel left in shared form (ROT_SH): its shared entries
    // back into the R columns first (the bit is cleared in the staged rotation
    // and written back with it). Wave-cooperative (round 6): the wave's lanes
    // take such groups one at a time and copy each one's live entries
    // together, one entry per lane and pass — up to K entries x R columns per
    // group, which one lane copying its own group took K dependent passes for
    // (C5 with corrupted copies, K = 512: every rejection copies a group back).
    // The block barrier below orders these stores before the tick's own.
    // (REF with corrupted copies, DevPlanes::sh_keep: the group keeps its
    // shared form through the tick — fast_group's `shf` — and nothing is copied)
    const bool keep = SEM != SEM_RAFT && CRC && P.sh_keep;
    for (uint64_t shm = __ballot(valid && (r0 & ROT_SH) && !keep); shm; shm &= shm - 1) {
      const int src = int(__builtin_ctzll(shm));
      const uint32_t gs = uint32_t(__shfl(int(g), src));
      const int L = __shfl(ss0.last, src), lo = max(__shfl(shf0, src), L - int(P.K) + 1);
      const uint32_t rs = uint32_t(__shfl(int(r0), src)), ras = uint32_t(__shfl(int(ra0), src)),
                     rbs = uint32_t(__shfl(int(rb0), src));
      const int sbs = __shfl(sb0, src), scs = __shfl(sc0, src);
      const uint64_t tb = ring_tile(gs, P.KP, R), shb = sh_tile(gs, P.KP);
      for (int idx = lo + int(lane); idx <= L; idx += 64) {
        const uint32_t slot = ring_slot(idx, rs, ras, rbs, sbs, scs, P.kmask);
        const uint32_t so = sh_in_tile(gs, slot, P.sh_cs), o = ring_in_tile(gs, R, slot, 0u);
        const int32_t tt = at(P.sh_term + shb, so);
        const int64_t vv = at(P.sh_value + shb, so);
        fill_seg<R>(P.log_term + tb + o, tt);
        fill_seg<R>(P.log_value + tb + o, vv);
        if constexpr (CRC) fill_seg<R>(P.log_crc + tb + o, at(P.sh_crc + shb, so));
      }
      if (P.dbg && lane == 0) {
        atomicAdd(&P.dbg[31], 1ull);
        if (L >= lo) atomicAdd(&P.dbg[1], (unsigned long long)(L - lo + 1));
      }
    }
    // (a group in shared form was taken by the lean kernel at the tick before
    // this one: its heartbeat time is implied, and written back from here)
    const int32_t hbs = (r0 & ROT_SH) ? T.at_tick(T.tick - 1).now : hb0;
    smeta[t] = m0; sgrot[t] = uint16_t(keep ? r0 : (r0 & ~ROT_SH)); sgiso[t] = gi0; shb[t] = hbs; sgss[t] = ss0;
    sglx[t] = lx0;
    const int shk = (keep && (r0 & ROT_SH)) ? shf0 : -1;   // (kept in shared form from this index on)
    if (P.dbg && shk >= 0) atomicAdd(&P.dbg[7], 1ull);
    sgrota[t] = ra0; sgrotb[t] = rb0; sgsb[t] = sb0; sgsb2[t] = sc0;
    sshk[t] = shk;
    // the tick runs on slot p of the block's staged groups: with P.list_sort
    // the slots ordered by the groups' form bits (gmeta above the leader and
    // fault fields, and whether an isolation record is live), a bitonic sort
    // of (key, slot) in LDS, so that a wave's lanes take fewer distinct paths
    // through fast_group; staging and write-back stay by slot (coalesced)
    uint32_t p = t;
    if (P.list_sort) {
      skey[t] = (valid ? ((uint32_t(m0) >> 7) << 1 | (gi0 ? 1u : 0u)) : 0x3FFu) << 8 | t;
      __syncthreads();
#pragma unroll 1
      for (uint32_t k = 2; k <= uint32_t(LB); k <<= 1)
#pragma unroll 1
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
          const uint32_t x = t ^ j;
          if (x > t) {
            const uint32_t a = skey[t], b = skey[x];
            if ((a > b) == ((t & k) == 0)) { skey[t] = b; skey[x] = a; }
          }
          __syncthreads();
        }
      p = skey[t] & 0xFFu;
    }
    __syncthreads();
    {   // coalesced record staging, 16 B per lane and load, RQ loads in flight per lane
      const int4* grec = reinterpret_cast<const int4*>(P.rec);
      int4 v[RQ];
#pragma unroll
      for (uint32_t k = 0; k < RQ; ++k) {
        const uint32_t w = t + uint32_t(LB) * k, j = w / RQ, gj = sg[j];
        v[k] = gj < P.G ? grec[uint64_t(gj) * RQ + (w - j * RQ)] : int4{0, 0, 0, 0};
      }
#pragma unroll
      for (uint32_t k = 0; k < RQ; ++k) srec4[t + uint32_t(LB) * k] = v[k];
    }
    __syncthreads();
    WPROF(const uint64_t wi1 = __builtin_amdgcn_s_memtime(); wk1 += wi1 - wi0;)
    sdm[t] = 0u;
    __syncthreads();
    const uint32_t gp = sg[p];
    const bool vp = gp < P.G;
    const int shp = sshk[p];
    const RowAcc<R, true> rw{&srec[p * RW], 0u, &sdm[p]};
    const WordAcc<true> gw{&smeta[p], &sgrot[p], &sgrota[p], &sgiso[p], &shb[p], &sgsb[p], &sgss[p], &sgrotb[p],
                           &sgsb2[p], &sglx[p], gp};
    // (P.diag, timing only, results wrong: 32 = staging alone, 64 = staging and write-back, no tick)
    if (P.diag & 32u) { __syncthreads(); continue; }
    bool wrote = (P.diag & 64u) ? vp
                                : fast_group<R, CRC, SEM, true>(P, T, stats, work, work_tick, work_count, 0, gp, tab,
                                                                    rw, gw, shp);
    WPROF(const uint64_t wi2 = __builtin_amdgcn_s_memtime(); wk2 += wi2 - wi1;)
    if (steps > 1) {   // the following tick too, on the staged state (pipelined tick)
      __threadfence_block();   // this step's ring stores, seen by the next step's gathers
      wrote |= fast_group<R, CRC, SEM, true>(P, T.at_tick(T.tick + 1), nx.stats, nx.work, nx.work_tick,
                                                 nx.work_count, 0, gp, tab, rw, gw, shp);
    }
    WPROF(const uint64_t wi3 = __builtin_amdgcn_s_memtime(); wk3 += wi3 - wi2;)
    {   // dirty rows -> the 16-B pieces of the record they touch
      const uint32_t rows = (vp && wrote) ? sdm[p] : 0u;
      uint32_t pm = 0;
#pragma unroll
      for (int k = 0; k < NPL; ++k)
        if ((rows >> k) & 1u) {
          const uint32_t q0 = uint32_t(k * R) / 4u, q1 = uint32_t(k * R + R - 1) / 4u;
          pm |= ((2u << q1) - 1u) & ~((1u << q0) - 1u);
        }
      sdm[p] = pm;
    }
    __syncthreads();
    {   // coalesced write-back of the records that may have changed
      int4* grec = reinterpret_cast<int4*>(P.rec);
#pragma unroll
      for (uint32_t k = 0; k < RQ; ++k) {
        const uint32_t w = t + uint32_t(LB) * k, j = w / RQ;
        if ((sdm[j] >> (w - j * RQ)) & 1u) grec[uint64_t(sg[j]) * RQ + (w - j * RQ)] = srec4[w];
      }
    }
    if (valid) {   // per-group words that changed
      if (smeta[t] != m0) at(P.gmeta, g) = smeta[t];
      if (sgrot[t] != r0) at(P.grot, g) = sgrot[t];
      if (sgrota[t] != ra0) at(P.grota, g) = sgrota[t];
      if (sgrotb[t] != rb0) at(P.grotb, g) = sgrotb[t];
      if (sgsb[t] != sb0) at(P.gsb, g) = sgsb[t];
      if (sgsb2[t] != sc0) at(P.gsb2, g) = sgsb2[t];
      if (sgiso[t] != gi0) at(P.giso, g) = sgiso[t];
      if (shb[t] != hb0) at(P.hb, g) = shb[t];
      const LxRec x1 = sglx[t];
      if (x1.k != lx0.k || x1.dl != lx0.dl) P.glx[g] = x1;
      const SsRec s1 = sgss[t];
      if (s1.last != ss0.last || s1.term != ss0.term || s1.cl != ss0.cl || s1.cf != ss0.cf) P.gss[g] = s1;
    }
    __syncthreads();   // the LDS copies and the body's block reductions are reused next round
    WPROF(wk4 += __builtin_amdgcn_s_memtime() - wi3;)
  }
  WPROF(if (P.dbg) {
    const uint64_t tot = __builtin_amdgcn_s_memtime() - wk0;
    wprof_add(P.dbg, 0, wk1); wprof_add(P.dbg, 1, wk2); wprof_add(P.dbg, 2, wk3); wprof_add(P.dbg, 3, wk4);
    wprof_add(P.dbg, 4, 1);
    if ((threadIdx.x & 63) == 0) atomicMax(&P.dbg[5], (unsigned long long)tot);
    wprof_add(P.dbg, 6 + min(15, 63 - __builtin_clzll(tot | 1ull) - 10), 1);
  })
}

// ---------------------------------------------------------------------------
// Lean steady-state kernel (the two-pass plan's first pass): one lane per
// group, takes exactly the groups that are in the compressed steady state
// (SSYNC: one 16-B record for term / LastApplied / CommitIndex rows), that
// no EXT isolation window touches this tick (drifted ring phases included);
// every other live group goes to the list that
// tick_list_kernel (the full fast_group) runs right after. For a taken
// group the tick of fast_group reduces to closed form (all R logs end at
// L = LastApplied with an entry of the leader's term T, the followers share
// one CommitIndex cf, leader's CommitIndex cl):
//   client append of n entries (main.go:327-329) -> LastApplied L+n;
//   one AppendEntries per follower with prevLogIndex L, prevLogTerm T and the
//   n entries (main.go:341-372): each accepts (main.go:121-156: same term,
//   prevIdx = its length, log[L].term = T), appends, takes CommitIndex
//   max(cf, cl) (min(LeaderCommit, len+1) / min(LeaderCommit, last new)),
//   MatchIndex = L+n (main.go:375-377), timer reset (hb = now);
//   commit rule (main.go:381-391): all R-1 peers at L+n -> cl' = L+n if
//   2(R-1) > R and L+n > cl; RAFT (majority order statistic incl. the
//   leader, entry of the current term): cl' = max(cl, L+n).
// Per group it reads gmeta 2 B + gss 16 B + grot 2 B and writes gss 16 B,
// hb 4 B and the entries (12·n·R B, +4·n·R with CRC32C) as whole ring rows
// (a drifted group: its own R-contiguous segment, or a ring segment switch).
// A/B hooks (round 5, interleaved A/Bs in profiles/r05/ab/): LEAN_HOIST_LX=1 (default)
// reads glx (and giso while a window is active) for every lane with gmeta
// instead of after it for the lanes that use them; with HWX's highest mark
// kept in glx too (fast_group) every lane of a C4 tick then needs one round
// trip: C4 2.62 -> 2.71e10 (r5ab9.txt; alone, without the HWX mark in glx,
// it was neutral: 85% of waves still waited for an HWX row). Hoisting HWX's
// 28-B high-water-mark row instead was 35% slower (C4's per-group words then
// no longer stay in the Infinity Cache).
#ifndef RAFTSTEP_LEAN_HOIST_LX
#define RAFTSTEP_LEAN_HOIST_LX 1
#endif
template <int R, bool CRC, int SEM>
__global__ __launch_bounds__(256) void tick_lean_kernel(DevPlanes P, Trace T, unsigned long long* stats, uint32_t* list,
                                                        uint32_t* count, int lflags, uint32_t gofs, uint32_t* zc) {
  constexpr bool RAFT = SEM == SEM_RAFT;
  shard_zero(zc);   // (ping-pong pipelined tick: the counter of the next tick's list, read by no running kernel)
  // (gofs: the first group of this launch, a multiple of 256 — the steady
  // tick may run as two launches over the two halves of the groups)
  const uint32_t gblk = (gofs >> 8) + blockIdx.x;   // this block's 256 groups
  const uint32_t g = gblk * 256u + threadIdx.x;
  __shared__ uint32_t tab[CRC ? 2048 : 1];
  stage_crc_tab<CRC>(P, tab);
  const int n = int(T.client_entries());
  const int ph = int(T.entries_before(T.tick) & P.kmask);   // global ring phase of this tick's first entry
  bool take = false, pass = false, lxs = false;   // lxs: an LXS tick (the cut-off leader appends alone)
  bool sxs = false;                             // an SXS tick (the stale leader appends alone, the primary replicates)
  int committed = 0, w_term = 0, w_slot = -1;   // w_slot >= 0: drifted lane, its own segment from that slot
  uint32_t wmask = 0;                           // replicas whose ring column gets this tick's entries
  uint64_t w_vb = 0;
  int x_slot = -1, x_r = 0;                     // SXS: the stale leader's first slot and its replica
  uint64_t x_vb = 0;
  uint32_t df = 0;
  // The group's key and its isolation windows this tick need no memory: they
  // are computed before the loads, so that everything a lane reads after
  // gmeta goes out in one round trip (the record, glx, giso, the ring
  // rotation and segment boundary, HWX's high-water marks).
  const uint64_t key = group_key(T.seed, P.gbase + g);
  uint32_t act = 0, starting = 0, im = 0;
  if (T.iso_p) im = iso_windows<R>(key, T, &act, &starting);
  bool held = false;
  bool shw = false;             // SH: this tick's entries go to the shared ring (ROT_SH)
  uint32_t p_mr = 0;            // a passed group's words as read here, for its list entry
  int32_t p_sb = 0;
  SsRec p_ss{0, 0, 0, 0};
  int64_t cv0 = 0;              // RAFT_CLIENT_STAGED: the group's entry 0 of this tick
  if (g < P.G) {
    // gmeta and, speculatively, the record, the ring rotation and the segment
    // boundary go out together: one round trip instead of two for the groups
    // the lean pass takes (nearly all of them; round 5, C2 at 2^24 groups,
    // where these reads miss the Infinity Cache)
    const int meta = at(P.gmeta, g);
    const SsRec s = P.gss[g];
    const int rot = at(P.grot, g);
    const int sb0 = P.KP > P.K ? at(P.gsb, g) : 0;
    // staged client values: this tick's entry 0 in the same round trip
    if (P.cv && n) cv0 = __builtin_nontemporal_load(P.cv + uint64_t(T.tick - P.cv_t0) * P.cv_tstride + g);
    p_mr = uint32_t(meta) | (uint32_t(rot) << 16);
    p_sb = sb0;
    p_ss = s;
    // RAFT under isolation churn, glx (and giso while a window is active) in
    // the same round trip: an LXS or SXS lane is in most waves of such a tick,
    // and each such wave waited a second round trip for them
    const bool hl = RAFT && RAFTSTEP_LEAN_HOIST_LX && T.iso_p;
    LxRec gx_h{0, 0};
    uint32_t gi_h = 0;
    if (hl) {
      gx_h = P.glx[g];
      if (act) gi_h = at(P.giso, g);
    }
    // pipelined tick: a group the last list kernel carries through this tick
    // too is left alone (its state is being written beside this kernel); the
    // mark is cleared with the kernel's other stores at the end (a store here
    // made every later load of the lane wait for it: vmcnt counts stores)
    held = (lflags & 1) && at(P.glst, g) != 0;
    const int c = meta & 0xF;
    const bool skip = held || (meta & M_DEFER) || ((meta >> 4) & 7);   // carried / pending catch-up / frozen group
    // (a group in shared form is in the plain normal class: anything else,
    // which only the list / general kernels could have set, goes to the list)
    const bool shm = (uint32_t(rot) & ROT_SH) != 0u;
    take = !skip && (meta & M_SSYNC) && c < R && g != P.dbg_pass &&   // (test knob: pass one group on)
           !(shm && (uses_glx(meta) || (RAFT && (meta & M_HWX))));
    pass = !skip && !take;
    df |= (!skip && g == P.dbg_pass) ? 1u << 24 : 0u;
    df |= skip ? 1u : 0u;
    if (take) {
      const LxRec gx = (RAFT && uses_glx(meta)) ? (hl ? gx_h : P.glx[g]) : LxRec{0, 0};
      uint32_t gi = (RAFT && T.iso_p && act && uses_glx(meta)) ? (hl ? gi_h : uint32_t(at(P.giso, g))) : 0u;
      int hwmx = 0;   // RAFT HWX: the highest high-water mark (the hwm plane)
      if (RAFT && (meta & M_HWX) && hl) {
        hwmx = gx_h.k;   // (its copy in glx, kept by the list kernel while HWX holds)
      } else if (RAFT && (meta & M_HWX)) {
        int hw[R];
        load_row_p<R>(&at(P.hwm, rix<R>(g, 0)), hw);
        hwmx = hw[0];
#pragma unroll
        for (int r = 1; r < R; ++r) hwmx = max(hwmx, hw[r]);
      }
      if (T.iso_p) {   // any window over this group this tick (either mode): the list kernel ...
        if (RAFT && (meta & M_LXS)) {
          // ... except an LXS group whose window still cuts off exactly its primary
          lxs = T.iso_leader && !starting && leader_iso_mask(act, 0u, gi, 0u, false) == (1u << c);
          take = lxs;
        } else if (RAFT && !CRC && is_sxs(meta)) {
          // ... and an SXS group whose windows cut off exactly its stale leader
          // (leader mode: no window deciding a victim this tick)
          const uint32_t cut = T.iso_leader ? (starting ? 0u : leader_iso_mask(act, 0u, gi, 0u, false)) : im;
          sxs = cut == (1u << gx.dl);
          take = sxs;
        } else if (T.iso_leader ? act != 0u : im != 0u) {
          take = false;
        }
      } else if (uses_glx(meta)) {
        take = false;
      }
      // The three classes below differ only in their conditions and in the
      // record they store; the value stream of the writing leader, the record
      // and timer stores and the ring writes are shared (one copy of each per
      // wave, whatever mix of classes its lanes hold).
      const int L = s.last;
      // (the value stream of this tick's entries: the primary's, the only
      // appending leader but SXS's stale one, whose stream follows below)
      const uint64_t vb = cv_base(P, key, uint32_t(c), T.tick, g);
      int nl = L, cl2 = s.cl, cf2 = s.cf;   // the record after this tick
      bool hbw = false;                     // every follower's timer reset (hb = now)
      int hwx_clear = 0;                    // RAFT HWX: a truncated log in step (high-water marks in the hwm plane)
      int sbo = 0, sw_d = 0, sw_rota = -1;  // a ring segment switch (normal class)
      if (RAFT && lxs) {
        // LXS tick (fast_group's isolated-leader tick in closed form): the
        // leader appends its client entries alone (main.go:327-329), every
        // AppendEntries it sends is dropped (EXT), nobody's timer is reset;
        // taken while no follower's election deadline is due (an election is
        // the list kernel's) and the leader's log is in the global ring
        // phase. Commit (r_leader_commit): the majority order statistic is the
        // followers' length L, an entry of the current term (SSYNC).
        const int Lc = L + gx.k;
        take = gx.dl > T.now && n < int(P.K) && int64_t(Lc) + n <= I32MAX && (n == 0 || ((Lc + rot) & int(P.kmask)) == ph);
        cl2 = L > s.cl ? L : s.cl;
        // The whole row, not only the leader's column, when every
        // follower's slot there is dead: with KP = 2K slots, all of a
        // follower's live entries (L-K, L] in the current segment (gsb at
        // most L-K+1, no segment gap) and the lead k+n at most K, the slot
        // of leader index L+k+e last held follower index L+k+e-2K <= L-K;
        // the follower rewrites it before its log reaches it. No partial
        // lines then; otherwise the leader's column alone.
        const bool whole = take && P.KP >= 2u * P.K && gx.k + n <= int(P.K) && sb0 <= L - int(P.K) + 1;
        wmask = whole ? (1u << R) - 1u : (1u << c);
        df |= take ? (131072u | 256u | (1u << 19) | (whole ? 1u << 21 : 0u)) : 0u;
      } else if (RAFT && !CRC && sxs) {
        // SXS tick (fast_group's stale-leader tick in closed form): the
        // primary appends its client entries (main.go:327-329) and replicates
        // them to its R-2 followers, which all accept (same term, prevLogIndex
        // = their length, log[L].term = T: main.go:121-156 with Raft's rules),
        // take CommitIndex max(cf, cl) and reset their timers (hb); the
        // AppendEntries to the stale leader xs is dropped (EXT), and xs — cut
        // off, still a leader of term T-1 — appends its own client entries to
        // its own log and every AppendEntries it sends is dropped; its commit
        // rule cannot move (its MatchIndex row is frozen). Commit
        // (r_leader_commit): R-1 of R logs at L+n, an entry of the current
        // term. The followers' entries go in the whole-row stores without
        // xs's column, or as the lane's own segment without it when they
        // append out of the global phase (no segment switch here: xs's
        // entries above L live in the current segment); xs's own entries
        // (index L+k+1+e, current segment: k >= 0) go in its column, inside
        // the common row when xs is in the global phase, else at its own slots.
        const int xs = gx.dl, k = gx.k;
        take = L > 0 && k >= 0 && int64_t(L) + k + n <= I32MAX && n < int(P.K) && s.cl <= L + n && !(meta & M_HWX);
        nl = L + n;
        cl2 = nl > s.cl ? nl : s.cl;
        cf2 = s.cl > s.cf ? s.cl : s.cf;
        hbw = true;
        const int wph = (L + rot) & int(P.kmask);
        if (take && n && wph != ph) w_slot = wph;
        // VX (M_VX): xs's entries are virtual and its column mirrors the
        // primary's: whole rows, nothing of its own to write
        const bool vx = (meta & M_VX) != 0;
        wmask = vx ? (1u << R) - 1u : ((1u << R) - 1u) & ~(1u << xs);
        x_slot = (take && !vx) ? (L + k + rot) & int(P.kmask) : -1;
        x_r = xs;
        df |= take ? ((w_slot < 0 ? 256u : 512u) | (1u << 25) | (x_slot == ph ? 1u << 26 : 0u) | (vx ? 1u << 27 : 0u))
                   : 0u;
      } else {
        // (the followers' CommitIndex min(LeaderCommit, last new entry) is the
        // leader's only while that is at most L+n: a leader's CommitIndex above
        // its log, left by a truncation, goes to the list kernel)
        take &= L > 0 && int64_t(L) + n <= I32MAX && n < int(P.K) && s.cl <= L + n;
        if (RAFT && take && (meta & M_HWX)) {
          // every AppendEntries' prevLogIndex (L) and NextIndex (L+1) must stay
          // inside the ring window of every log: max hwm < L+K (r_deliver_ae /
          // r_leader_round's evicted rules); the flag clears once every log has
          // grown to its mark (the marks are then LastApplied again)
          take &= hwmx - L < int(P.K);
          hwx_clear = hwmx <= L + n ? 1 : 0;
        }
        // ring phase: a group whose logs stood still under churn appends out of
        // the global phase (drifted); it switches its ring segment in place
        // when that is safe (ring_slot; as fast_group), else writes its own
        // R-contiguous segment at its own slot
        sbo = sb0;
        const int wph = (L + rot) & int(P.kmask);
        if (take && n && wph != ph) {
          const uint32_t d = uint32_t(ph - wph) & P.kmask;
          df |= d <= P.K ? 8u : 16u;
          bool sw = false;
          if (P.KP > P.K && d <= P.K) {
            sw = sbo <= 1 || sbo <= L - int(P.K) + 1;   // the previous segment holds no readable entry
            if (!sw) {   // it does: the segments shift when the oldest is dead and both jumps fit (ring_switch_ok)
              const uint32_t rota = at(P.grota, g);
              sw = ring_switch_ok(d, uint32_t(rot), rota, sbo, at(P.gsb2, g), L, P.K, P.kmask);
              sw_rota = int(rota);
              df |= sw ? 1u << 20 : 0u;   // class: a switch while the previous segment stays live (three segments)
            }
          }
          if (sw) sw_d = int(d);
          else w_slot = wph;
        }
        // SH: a group in step at the global phase writes one shared copy; one
        // already in shared form that would not (a drift after a tick gap) is
        // the list kernel's (which copies its shared entries back first)
        if (shm && (sw_d || w_slot >= 0)) take = false;
        if constexpr (CRC) {   // EXT: every follower verifies the stamp of each entry it received
          if (take && n) {
            uint32_t cm = 0;   // followers whose message is corrupted this tick: the list kernel (rejection)
#pragma unroll
            for (int p = 0; p < R; ++p)
              if (p != c && P.corrupt_p && (rng_k(key, uint32_t(p), ST_CORRUPT, uint64_t(T.tick)) & 0xFFFF) < P.corrupt_p)
                cm |= 1u << p;
            // (as fast_group: each follower checks the copy it received; an
            // unaltered copy carries the leader's stamp, so only cm's need a
            // CRC — the stamps themselves are computed once, in the row stores)
            if (cm) take &= crc_reject_mask(tab, crc_term_state(tab, s.term), vb, cv_stride(P), n, cm) == 0u;
          }
        }
        shw = P.sh && take && n > 0 && w_slot < 0 && !sw_d && !(RAFT && (meta & M_HWX));   // (in phase only)
        nl = L + n;
        if (RAFT ? nl > s.cl : (2 * (R - 1) > R && nl > s.cl)) cl2 = nl;
        cf2 = s.cl > s.cf ? s.cl : s.cf;
        hbw = true;
        wmask = (1u << R) - 1u;
        df |= take ? (262144u | (w_slot < 0 ? 256u : 512u) | ((RAFT && (meta & M_HWX)) ? 1u << 22 : 0u) |
                      (sw_d ? 32u : 0u))
                   : 0u;
      }
      if (take) {
        // (SH: the heartbeat time of a group in shared form is implied, P.sh_hb)
        if (shw || shm) hbw = false;
        if (P.rec_nt) {   // (per-group words beyond the Infinity Cache: streamed, DevPlanes::rec_nt)
          typedef int32_t i4 __attribute__((ext_vector_type(4)));
          if (nl != L || cl2 != s.cl || cf2 != s.cf)
            __builtin_nontemporal_store(i4{nl, s.term, cl2, cf2}, reinterpret_cast<i4*>(&P.gss[g]));
          if (hbw) __builtin_nontemporal_store(int32_t(T.now), &P.hb[g]);   // timer.Reset(d) of every follower
        } else {
          if (nl != L || cl2 != s.cl || cf2 != s.cf) P.gss[g] = SsRec{nl, s.term, cl2, cf2};
          if (hbw) at(P.hb, g) = T.now;                   // timer.Reset(d) of every follower
        }
        if (RAFT && lxs) P.glx[g] = LxRec{gx.k + n, gx.dl};   // (SXS: unchanged, both logs grow by n)
        if (shw && !shm) {   // SH from this tick's first entry on
          at(P.grot, g) = uint16_t(uint32_t(rot) | ROT_SH);
          at(P.gshf, g) = L + 1;
        }
        if (hwx_clear) at(P.gmeta, g) = uint16_t(meta & ~M_HWX);
        if (sw_d) {   // the new segment starts at this tick's first entry
          if (sw_rota >= 0) at(P.grotb, g) = uint16_t(sw_rota);   // (else the older segments are dead)
          at(P.gsb2, g) = sbo;
          at(P.grota, g) = uint16_t(rot);
          at(P.gsb, g) = L + 1;
          at(P.grot, g) = uint16_t((rot + sw_d) & int(P.kmask));
        }
        committed = cl2 - s.cl;
        w_term = s.term;
        w_vb = vb;
        if (RAFT && !CRC && sxs && x_slot >= 0) x_vb = cv_base(P, key, uint32_t(x_r), T.tick, g);
      } else {
        pass = true;
        w_slot = -1;
        x_slot = -1;
        shw = false;
      }
    }
  }
  // this tick's entries: the taken lanes at the global phase as whole ring
  // rows, all R replicas (the cooperative row stores of fast_group); a
  // drifted lane its own R-contiguous segment. SXS: the stale leader's
  // column carries its own entry (term T-1, its value stream) — in the common
  // row when it is in the global phase (xrow), else at its own slot (wx).
  bool wr = take && n && w_slot < 0;
  const bool wsh = wr && shw;   // SH: the shared ring's row instead (ROT_SH)
  wr = wr && !shw;
  bool wd = take && n && w_slot >= 0;
  const bool xrow = RAFT && !CRC && take && n && x_slot == ph;
  bool wx = RAFT && !CRC && take && n && x_slot >= 0 && !xrow;
  bool holes = true;   // rows keep the columns of lanes that do not write them (diag 4: no holes)
  if (P.diag) {   // timing-only diagnostics (wrong results): drifted lanes skip / write the common row,
                  // 4: whole rows written (no holes left by passed lanes), 8: no stale-column writes
    if (P.diag & 2u) wr |= wd;
    if (P.diag & 3u) wd = false;
    if (P.diag & 4u) holes = false;
    if (P.diag & 8u) wx = false;
  }
  if (__ballot(wr || wd || xrow || wx || wsh)) {
    const int lane = threadIdx.x & 63;
    const uint32_t g0 = __builtin_amdgcn_readfirstlane(g);
    const uint64_t tb = ring_tile(g0, P.KP, R);
    int32_t* const rt = P.log_term + tb;
    int64_t* const rv = P.log_value + tb;
    uint32_t* const rc = CRC ? P.log_crc + tb : nullptr;
    const bool anyrow = __ballot(wr || xrow || !holes) != 0ull;   // (wave-uniform: a whole-row lane in the wave)
    const bool anysh = __ballot(wsh) != 0ull;
    const uint64_t shb = anysh ? sh_tile(g0, P.KP) : 0u;
    uint32_t cs = 0;
    if constexpr (CRC) cs = crc_term_state(tab, w_term);
    const bool anyx = RAFT && !CRC && __ballot(xrow) != 0ull;   // (wave-uniform)
    int k_term[R], k_src[R];
    bool k_on[R], k_x[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int src = (k * 64 + lane) / R, rr = (k * 64 + lane) - src * R;
      k_src[k] = src;
      k_term[k] = __shfl(w_term, src);
      k_on[k] = ((uint32_t(__shfl(int(wr ? wmask : 0u), src)) >> rr) & 1u) != 0u || !holes;   // (LXS: the leader's column)
      k_x[k] = anyx && ((uint32_t(__shfl(xrow ? int(1u << x_r) : 0, src)) >> rr) & 1u) != 0u;
    }
    const uint64_t cvs = cv_stride(P);
    // Shared ring in slot chunks (P.sh_cs > 0, C5V): a chunk of 16 slots x 64
    // groups is contiguous, group-major inside, so the wave writes it
    // transposed — element k*64 + lane of the chunk is group (k*64+lane) >> 4's
    // slot (k*64+lane) & 15 — with that group's term, value stream and CRC
    // state by shuffle: whole lines, as the row form does for cs = 0. (The
    // row loop below would write 4 B of a different line per lane and entry.)
    const bool shx = anysh && P.sh_cs != 0u;   // (wave-uniform)
    if (shx) {
      const uint32_t csz = 1u << P.sh_cs;
      const uint32_t vb_lo = uint32_t(w_vb), vb_hi = uint32_t(w_vb >> 32);
      for (uint32_t cb = uint32_t(ph) & ~(csz - 1u); cb < uint32_t(ph + n); cb += csz) {
        for (uint32_t k = 0; k < csz; ++k) {
          const uint32_t idx = k * 64u + uint32_t(lane);
          const int gl = int(idx >> P.sh_cs);
          const uint32_t sl = cb + (idx & (csz - 1u));
          const int e = int(sl) - ph;
          const bool on = __shfl(int(wsh), gl) != 0 && e >= 0 && e < n;
          const int ts = __shfl(w_term, gl);
          const uint64_t vbg = (uint64_t(uint32_t(__shfl(int(vb_hi), gl))) << 32) | uint32_t(__shfl(int(vb_lo), gl));
          uint32_t csg = 0;
          if constexpr (CRC) csg = uint32_t(__shfl(int(cs), gl));
          const int64_t c0 = int64_t((uint64_t(uint32_t(__shfl(int(uint32_t(uint64_t(cv0) >> 32)), gl))) << 32) |
                                     uint32_t(__shfl(int(uint32_t(uint64_t(cv0))), gl)));
          if (on) {
            const int64_t v = (cvs && e == 0) ? c0 : cv_value(vbg, uint32_t(e), cvs);
            const uint32_t so = sh_in_tile(uint32_t(gl), sl & P.kmask, P.sh_cs);
            ring_st(P.sh_term + shb, so, ts);
            ring_st(P.sh_value + shb, so, v);
            if constexpr (CRC) ring_st(P.sh_crc + shb, so, crc_value_final(tab, csg, v));
          }
        }
      }
    }
    const bool rowloop = anyrow || __ballot(wd || wx) != 0ull || (anysh && !shx);   // (wave-uniform)
    for (int e = 0; rowloop && e < n; ++e) {
      // (staged values: every leader of the group appends the same request,
      // entry 0 already loaded with the group's words)
      const int64_t v = (cvs && e == 0) ? cv0 : cv_value(w_vb, uint32_t(e), cvs);
      uint32_t stamp = 0;
      if constexpr (CRC) stamp = crc_value_final(tab, cs, v);
      const uint32_t row = uint32_t((ph + e) & int(P.kmask)) * 64u * R;
      const int vlo = int(uint32_t(uint64_t(v))), vhi = int(uint32_t(uint64_t(v) >> 32));
      int64_t xv = 0;
      if (RAFT && !CRC && x_slot >= 0) xv = cvs ? v : cv_value(x_vb, uint32_t(e), 0u);
      const int xlo = int(uint32_t(uint64_t(xv))), xhi = int(uint32_t(uint64_t(xv) >> 32));
      if (wsh && !shx) {   // SH: one copy, 64 consecutive groups' entries per wave row
        const uint32_t so = sh_in_tile(uint32_t(lane), uint32_t((ph + e) & int(P.kmask)), P.sh_cs);
        ring_st(P.sh_term + shb, so, w_term);
        ring_st(P.sh_value + shb, so, v);
        if constexpr (CRC) ring_st(P.sh_crc + shb, so, stamp);
      }
#pragma unroll
      for (int k = 0; k < R; ++k) {
        if (!anyrow) break;
        const int lo = __shfl(vlo, k_src[k]), hi = __shfl(vhi, k_src[k]);
        uint32_t sk = 0;
        if constexpr (CRC) sk = uint32_t(__shfl(int(stamp), k_src[k]));
        int xl = 0, xh = 0;
        if (anyx) { xl = __shfl(xlo, k_src[k]); xh = __shfl(xhi, k_src[k]); }
        if (k_on[k] || k_x[k]) {
          const uint32_t o = row + uint32_t(k * 64 + lane);
          ring_st(rt, o, k_x[k] ? k_term[k] - 1 : k_term[k]);
          ring_st(rv, o, k_x[k] ? int64_t((uint64_t(uint32_t(xh)) << 32) | uint32_t(xl))
                                : int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo)));
          if constexpr (CRC) ring_st(rc, o, sk);
        }
      }
      if (wd) {
        const uint32_t o = ring_in_tile(g, R, uint32_t((w_slot + e) & int(P.kmask)), 0u);
        if (wmask == (1u << R) - 1u) {   // every replica appends: R-wide vector stores
          fill_seg<R>(rt + o, w_term);
          fill_seg<R>(rv + o, v);
          if constexpr (CRC) fill_seg<R>(rc + o, stamp);
        } else {                         // SXS: every replica but the stale leader
#pragma unroll
          for (int p = 0; p < R; ++p) {
            if (!((wmask >> p) & 1u)) continue;
            ring_st(rt, o + uint32_t(p), w_term);
            ring_st(rv, o + uint32_t(p), v);
          }
        }
      }
      if (wx) {   // SXS: the stale leader out of the global phase: its own entry in its column
        const uint32_t o = ring_in_tile(g, R, uint32_t((x_slot + e) & int(P.kmask)), uint32_t(x_r));
        ring_st(rt, o, w_term - 1);
        ring_st(rv, o, xv);
      }
    }
  }
#ifdef RAFTSTEP_WAVE_PROF
  if (false) {
#else
  if (P.dbg) {   // diagnostics (same class bits as fast_group): lanes, skipped, taken by the lean pass
#endif
    df |= (g < P.G) ? 1024u : 0u;
    df |= pass ? 1u << 23 : 0u;
    if (!take) df &= ~0xE780000u;   // the class bits 19-22, 25-27 count taken ticks only
#pragma unroll 1
    for (int k = 0; k < 28; ++k) {
      const uint64_t b = __ballot((df >> k) & 1u);
      if ((threadIdx.x & 63) == 0 && b) atomicAdd(&P.dbg[k], (unsigned long long)__popcll(b));
    }
    const uint64_t bsh = __ballot(wsh);   // SH: ticks written to the shared ring
    if ((threadIdx.x & 63) == 0 && bsh) atomicAdd(&P.dbg[30], (unsigned long long)__popcll(bsh));
  }
  if (held) at(P.glst, g) = uint8_t(0);   // (the mark read above)
  // the rest go to the list kernel: block-local prefix, one atomic per block
  // on the block's shard of the list
  __shared__ uint32_t wn[4], wbase;
  const uint64_t bm = __ballot(pass);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t k = shard_of_block(gblk, P.shard_sb);   // == shard_home(g)
  if (lane == 0) wn[wave] = uint32_t(__popcll(bm));
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tot = wn[0] + wn[1] + wn[2] + wn[3];
    wbase = tot ? atomicAdd(&count[k * SHARD_STRIDE], tot) : 0u;
  }
  __syncthreads();
  if (pass) {
    uint32_t off = k * P.scap + wbase + uint32_t(__popcll(bm & ((1ull << lane) - 1ull)));
    for (int w = 0; w < wave; ++w) off += wn[w];
    list[off] = g;
    // the words read above, for the list kernel's coalesced staging (LIST_WORDS)
    const uint64_t cap = uint64_t(NSHARD) * P.scap;
    list_mr(list, cap)[off] = p_mr;
    list_sb(list, cap)[off] = p_sb;
    list_ss(list, cap)[off] = p_ss;
    if (lflags & 2) at(P.glst, g) = uint8_t(1);   // the list kernel carries it through the next tick too
  }
  // (packed, tick_common.hpp lean_stats: a normal tick R-1 accepted
  // AppendEntries; an LXS tick every AppendEntries of the cut-off leader
  // dropped; an SXS tick the one to the stale leader and every one it sends)
  if (stats && !T.iso_p) {
    lean_stats<RAFT>(g < P.G, committed - lean_base_committed(RAFT, R, uint32_t(n)), take && !lxs && !sxs,
                     take && lxs, take && sxs, stats);
  } else if (stats) {   // (isolation churn: absolute per-block counters, no base — engine.cpp call_lean)
    const int t = take ? 1 : 0;
    if constexpr (RAFT) {
      // (an LXS tick: every AppendEntries of the cut-off leader dropped; an SXS
      // tick: the one to the stale leader and every one it sends)
      const int v[5] = {committed, (take && !lxs) ? (sxs ? R - 2 : R - 1) : 0,
                        (take && lxs) ? R - 1 : ((take && sxs) ? R : 0), t, 0};
      const int idx[5] = {S_COMMITTED, S_AE_OK, S_AE_FAIL, S_LEADER_GROUPS, S_BUMPS};
      block_stats<5>(v, idx, stats);
    } else {
      const int v[4] = {committed, t * (R - 1), 0, t};
      const int idx[4] = {S_COMMITTED, S_AE_OK, S_AE_FAIL, S_LEADER_GROUPS};
      block_stats<4>(v, idx, stats);
    }
  }
}

// Fused steady ticks (the steady-state list skip, engine.cpp): every live
// group is proven compressed and takeable and no isolation or corruption is
// configured, so the lean kernel's normal class is the whole tick of every
// group, and `nt` consecutive ticks run in one launch: the record, ring
// rotation and meta are read once, each tick's closed form (client append,
// AppendEntries to every follower, responses, commit rule, heartbeat — see
// tick_lean_kernel) is applied in registers and its entries are written as
// whole ring rows, the tick's statistics go to its own record, and the
// record and heartbeat are stored once after the last tick. Per group and
// tick this moves the ring bytes (12·E·R) plus 1/nt of the record / meta /
// rotation / heartbeat bytes. A group that stops being takeable at tick j
// (which the skip's proof excludes) is stored as of tick j-1 and passed to
// the list, which the end-of-call check turns into RAFT_EINTERNAL.
template <int R, bool CRC, int SEM>
__global__ __launch_bounds__(256) void tick_fused_kernel(DevPlanes P, Trace T, int nt, unsigned long long* stats,
                                                         uint32_t* list, uint32_t* count) {
  constexpr bool RAFT = SEM == SEM_RAFT;
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  __shared__ uint32_t tab[CRC ? 2048 : 1];
  stage_crc_tab<CRC>(P, tab);
  const uint64_t key = group_key(T.seed, P.gbase + g);
  bool live = false, pass = false;
  int c = 0, rot = 0, L = 0, term = 0, cl = 0, cf = 0, done = 0;
  int sh_from = -1;   // SH: the first entry this launch wrote, for a group entering shared form
  SsRec s0{0, 0, 0, 0};
  if (g < P.G) {
    const int meta = at(P.gmeta, g);
    c = meta & 0xF;
    const bool skip = (meta & M_DEFER) || ((meta >> 4) & 7);
    live = !skip && (meta & M_SSYNC) && c < R && !uses_glx(meta) && !(RAFT && (meta & M_HWX)) &&
           g != P.dbg_pass;
    pass = !skip && !live;
    if (live) {
      s0 = P.gss[g];
      rot = at(P.grot, g);
      L = s0.last; term = s0.term; cl = s0.cl; cf = s0.cf;
    }
  }
  const int lane = threadIdx.x & 63;
  const uint32_t g0 = __builtin_amdgcn_readfirstlane(g);
  const uint64_t tb = ring_tile(g0, P.KP, R);
  int32_t* const rt = P.log_term + tb;
  int64_t* const rv = P.log_value + tb;
  uint32_t* const rc = CRC ? P.log_crc + tb : nullptr;
  const uint64_t shb = P.sh ? sh_tile(g0, P.KP) : 0u;   // SH: every live group writes the shared ring (ROT_SH)
  int k_src[R];
#pragma unroll
  for (int k = 0; k < R; ++k) k_src[k] = (k * 64 + lane) / R;
  for (int j = 0; j < nt; ++j) {   // (wave-uniform)
    const Trace Tj = T.at_tick(T.tick + j);
    const int n = int(Tj.client_entries());
    const int ph = int(Tj.entries_before(Tj.tick) & P.kmask);
    // the lean kernel's normal class, in phase (init_steady puts every group there)
    bool take = live && L > 0 && int64_t(L) + n <= I32MAX && n < int(P.K) && cl <= L + n &&
                (n == 0 || ((L + rot) & int(P.kmask)) == ph);
    if (live && !take) { pass = true; live = false; }
    int committed = 0;
    if (take) {
      const int nl = L + n;
      if (P.sh && n && sh_from < 0 && !(uint32_t(rot) & ROT_SH)) sh_from = L + 1;
      const int cl2 = (RAFT ? nl > cl : (2 * (R - 1) > R && nl > cl)) ? nl : cl;
      cf = cl > cf ? cl : cf;
      committed = cl2 - cl;
      L = nl;
      cl = cl2;
      done = j + 1;
    }
    if (n && __ballot(take)) {   // this tick's entries as whole ring rows (holes for the other lanes)
      const uint64_t vb = take ? cv_base(P, key, uint32_t(c), Tj.tick, g) : 0ull;
      uint32_t cs = 0;
      if constexpr (CRC) cs = crc_term_state(tab, term);
      int k_term[R];
      bool k_on[R];
#pragma unroll
      for (int k = 0; k < R; ++k) {
        k_term[k] = __shfl(term, k_src[k]);
        k_on[k] = __shfl(take ? 1 : 0, k_src[k]) != 0;
      }
      for (int e = 0; e < n; ++e) {
        const int64_t v = cv_value(vb, uint32_t(e), cv_stride(P));
        uint32_t stamp = 0;
        if constexpr (CRC) stamp = crc_value_final(tab, cs, v);
        if (P.sh) {   // (wave-uniform)
          if (take) {
            const uint32_t so = sh_in_tile(uint32_t(lane), uint32_t((ph + e) & int(P.kmask)), P.sh_cs);
            ring_st(P.sh_term + shb, so, term);
            ring_st(P.sh_value + shb, so, v);
            if constexpr (CRC) ring_st(P.sh_crc + shb, so, stamp);
          }
          continue;
        }
        const uint32_t row = uint32_t((ph + e) & int(P.kmask)) * 64u * R;
        const int vlo = int(uint32_t(uint64_t(v))), vhi = int(uint32_t(uint64_t(v) >> 32));
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int lo = __shfl(vlo, k_src[k]), hi = __shfl(vhi, k_src[k]);
          uint32_t sk = 0;
          if constexpr (CRC) sk = uint32_t(__shfl(int(stamp), k_src[k]));
          if (k_on[k]) {
            const uint32_t o = row + uint32_t(k * 64 + lane);
            ring_st(rt, o, k_term[k]);
            ring_st(rv, o, int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo)));
            if constexpr (CRC) ring_st(rc, o, sk);
          }
        }
      }
    }
    if (stats)   // tick j's record (exceptions: normal ticks only)
      lean_stats<RAFT>(g < P.G, committed - lean_base_committed(RAFT, R, uint32_t(n)), take, false, false,
                       stats + size_t(j) * STAT_TICK);
  }
  if (done) {   // the record and every follower's timer as of the last tick taken (SH: implied)
    if (L != s0.last || cl != s0.cl || cf != s0.cf) P.gss[g] = SsRec{L, term, cl, cf};
    if (!(sh_from >= 0 || (uint32_t(rot) & ROT_SH))) at(P.hb, g) = T.at_tick(T.tick + done - 1).now;
  }
  if (sh_from >= 0) {   // SH from that entry on
    at(P.grot, g) = uint16_t(uint32_t(rot) | ROT_SH);
    at(P.gshf, g) = sh_from;
  }
  if (P.dbg) {   // diagnostics (lean kernel counters): lanes x ticks, compressed ticks taken, passed on
    const uint64_t b0 = __ballot(g < P.G), b1 = __ballot(pass);
    const long long tk = wave_sum(done);
    if (lane == 0) {
      atomicAdd(&P.dbg[10], (unsigned long long)(__popcll(b0) * uint64_t(nt)));
      if (tk) atomicAdd(&P.dbg[18], (unsigned long long)tk);
      if (b1) atomicAdd(&P.dbg[23], (unsigned long long)__popcll(b1));
    }
  }
  // passed on (the skip's proof violated): one atomic per passing lane (the
  // id only: no list kernel runs in a list-skipping call, and the end-of-call
  // check turns any such entry into RAFT_EINTERNAL before one could)
  if (pass) {
    const uint32_t k = shard_of_block(blockIdx.x, P.shard_sb);
    list[k * P.scap + atomicAdd(&count[k * SHARD_STRIDE], 1u)] = g;
  }
}

template <int R, bool CRC, int SEM>
static void launch_fused_t(const DevPlanes& P, const Trace& T, int nt, unsigned long long* stats, uint32_t* list,
                           uint32_t* count, hipStream_t s, hipEvent_t a, hipEvent_t b) {
  hipExtLaunchKernelGGL(tick_fused_kernel<R, CRC, SEM>, grid_for(P.G), dim3(256), 0, s, a, b, 0, P, T, nt, stats,
                        list, count);
}
hipError_t launch_tick_fused(int R, int sem, const DevPlanes& P, const Trace& T, int nticks, unsigned long long* stats,
                             uint32_t* list, uint32_t* count, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
  const bool crc = P.crc_on != 0;
#define RAFT_FUSED(CRC_)                                                                                        \
  if (sem == SEM_RAFT) {                                                                                         \
    RAFT_DISPATCH_R(R, (launch_fused_t<RR, CRC_, SEM_RAFT>(P, T, nticks, stats, list, count, s, ev_start, ev_stop))) \
  } else {                                                                                                       \
    RAFT_DISPATCH_R(R, (launch_fused_t<RR, CRC_, SEM_REF>(P, T, nticks, stats, list, count, s, ev_start, ev_stop)))  \
  }
  if (crc) { RAFT_FUSED(true); } else { RAFT_FUSED(false); }
#undef RAFT_FUSED
  return hipGetLastError();
}

template <int R, bool CRC, int SEM>
static void launch_fast_t(const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* work,
                          int32_t* work_tick, uint32_t* work_count, int force_slow, hipStream_t s, hipEvent_t a,
                          hipEvent_t b) {
  hipExtLaunchKernelGGL(tick_fast_kernel<R, CRC, SEM>, grid_for(P.G), dim3(256), 0, s, a, b, 0, P, T, stats, work,
                        work_tick, work_count, force_slow);
}
hipError_t launch_tick_fast(int R, int sem, const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* work,
                            int32_t* work_tick, uint32_t* work_count, int force_slow, hipStream_t s,
                            hipEvent_t ev_start, hipEvent_t ev_stop) {
  const bool crc = P.crc_on != 0;
#define RAFT_FAST(CRC_)                                                                                            \
  if (sem == SEM_RAFT) {                                                                                           \
    RAFT_DISPATCH_R(R, (launch_fast_t<RR, CRC_, SEM_RAFT>(P, T, stats, work, work_tick, work_count, force_slow, s, \
                                                          ev_start, ev_stop)))                                     \
  } else {                                                                                                         \
    RAFT_DISPATCH_R(R, (launch_fast_t<RR, CRC_, SEM_REF>(P, T, stats, work, work_tick, work_count, force_slow, s,  \
                                                         ev_start, ev_stop)))                                      \
  }
  if (crc) { RAFT_FAST(true); } else { RAFT_FAST(false); }
#undef RAFT_FAST
  return hipGetLastError();
}

template <int R, bool CRC, int SEM>
static void launch_lean_t(const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* list,
                          uint32_t* count, int lflags, hipStream_t s, hipEvent_t a, hipEvent_t b, uint64_t g0 = 0,
                          uint64_t ng = ~0ull, uint32_t* zc = nullptr) {
  const uint64_t n = std::min<uint64_t>(ng, P.G - g0);
  hipExtLaunchKernelGGL(tick_lean_kernel<R, CRC, SEM>, grid_for(n), dim3(256), 0, s, a, b, 0, P, T, stats, list,
                        count, lflags, uint32_t(g0), zc);
}

template <int R, bool CRC, int SEM>
static void launch_list_t(const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* work,
                          int32_t* work_tick, uint32_t* work_count, uint32_t* list, uint32_t* count,
                          uint32_t* next_count, const ListNext* next, hipStream_t s, hipEvent_t c, hipEvent_t d) {
  const int steps = next ? 2 : 1;
  const ListNext nx = next ? *next : ListNext{nullptr, nullptr, nullptr, nullptr};
  // blocks of four waves, a resident grid striding over the list (one-wave
  // blocks measured the same list kernel time on C4 and a 15% slower lean
  // kernel beside it, round 2)
  constexpr uint64_t GPB = 256 / 64 * LIST_LANES;
  static const unsigned cap = [] {
    const char* v = std::getenv("RAFTSTEP_LIST_BLOCKS");   // experiment knob: cap the resident grid
    return v ? unsigned(std::strtoul(v, nullptr, 10)) : 0u;
  }();
  uint64_t lim = resident_blocks(tick_list_kernel<R, CRC, SEM, 256>, 256);
  if (cap) lim = std::min<uint64_t>(lim, cap);
  const unsigned blocks = unsigned(std::min<uint64_t>((P.G + GPB - 1) / GPB, lim));
  hipExtLaunchKernelGGL(tick_list_kernel<R, CRC, SEM, 256>, dim3(blocks), dim3(256), 0, s, c, d, 0, P, T, stats, work,
                        work_tick, work_count, list, count, next_count, steps, nx);
}

template <int R, bool CRC, int SEM>
static void launch_two_pass_t(const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* work,
                              int32_t* work_tick, uint32_t* work_count, uint32_t* list, uint32_t* count,
                              uint32_t* next_count, hipStream_t s, hipEvent_t a, hipEvent_t b, hipEvent_t c,
                              hipEvent_t d, bool skip_list) {
  launch_lean_t<R, CRC, SEM>(P, T, stats, list, count, 0, s, a, b);
  if (skip_list) return;   // the engine proved the list empty (engine.cpp, steady-state list skip)
  launch_list_t<R, CRC, SEM>(P, T, stats, work, work_tick, work_count, list, count, next_count, nullptr, s, c, d);
}
hipError_t launch_tick_two_pass(int R, int sem, const DevPlanes& P, const Trace& T, unsigned long long* stats,
                                uint32_t* work, int32_t* work_tick, uint32_t* work_count, uint32_t* list,
                                uint32_t* count, uint32_t* next_count, hipStream_t s, hipEvent_t lean_start,
                                hipEvent_t lean_stop, hipEvent_t list_start, hipEvent_t list_stop, bool skip_list) {
  const bool crc = P.crc_on != 0;
#define RAFT_TWO(CRC_)                                                                                            \
  if (sem == SEM_RAFT) {                                                                                           \
    RAFT_DISPATCH_R(R, (launch_two_pass_t<RR, CRC_, SEM_RAFT>(P, T, stats, work, work_tick, work_count, list, count, \
                                                              next_count, s, lean_start, lean_stop, list_start,      \
                                                              list_stop, skip_list)))                                \
  } else {                                                                                                         \
    RAFT_DISPATCH_R(R, (launch_two_pass_t<RR, CRC_, SEM_REF>(P, T, stats, work, work_tick, work_count, list, count,  \
                                                             next_count, s, lean_start, lean_stop, list_start,       \
                                                             list_stop, skip_list)))                                 \
  }
  if (crc) { RAFT_TWO(true); } else { RAFT_TWO(false); }
#undef RAFT_TWO
  return hipGetLastError();
}
hipError_t launch_tick_lean(int R, int sem, const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* list,
                            uint32_t* count, int lflags, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop,
                            uint64_t g0, uint64_t ng, uint32_t* zero_count) {
  const bool crc = P.crc_on != 0;
#define RAFT_LEAN(CRC_)                                                                                          \
  if (sem == SEM_RAFT) {                                                                                          \
    RAFT_DISPATCH_R(R, (launch_lean_t<RR, CRC_, SEM_RAFT>(P, T, stats, list, count, lflags, s, ev_start, ev_stop,   \
                                                          g0, ng, zero_count)))                                   \
  } else {                                                                                                        \
    RAFT_DISPATCH_R(R, (launch_lean_t<RR, CRC_, SEM_REF>(P, T, stats, list, count, lflags, s, ev_start, ev_stop,    \
                                                         g0, ng, zero_count)))                                    \
  }
  if (crc) { RAFT_LEAN(true); } else { RAFT_LEAN(false); }
#undef RAFT_LEAN
  return hipGetLastError();
}
hipError_t launch_tick_list(int R, int sem, const DevPlanes& P, const Trace& T, unsigned long long* stats, uint32_t* work,
                            int32_t* work_tick, uint32_t* work_count, uint32_t* list, uint32_t* count,
                            uint32_t* next_count, const ListNext* next, hipStream_t s, hipEvent_t ev_start,
                            hipEvent_t ev_stop) {
  const bool crc = P.crc_on != 0;
#define RAFT_LIST(CRC_)                                                                                          \
  if (sem == SEM_RAFT) {                                                                                          \
    RAFT_DISPATCH_R(R, (launch_list_t<RR, CRC_, SEM_RAFT>(P, T, stats, work, work_tick, work_count, list, count,   \
                                                          next_count, next, s, ev_start, ev_stop)))                \
  } else {                                                                                                        \
    RAFT_DISPATCH_R(R, (launch_list_t<RR, CRC_, SEM_REF>(P, T, stats, work, work_tick, work_count, list, count,    \
                                                         next_count, next, s, ev_start, ev_stop)))                 \
  }
  if (crc) { RAFT_LIST(true); } else { RAFT_LIST(false); }
#undef RAFT_LIST
  return hipGetLastError();
}

}  // namespace raftstep
