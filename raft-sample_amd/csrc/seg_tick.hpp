// seg_tick.hpp — the general tick, replica-parallel: one 8-lane segment of
// a wave per Raft group, one lane per replica (R <= 8; lanes r >= R idle).
//
// The reference delivers a round's messages one peer after the other
// (LeaderRun main.go:334-379, CandidateRun main.go:259-269), but each peer's
// handler reads only the sender's request and its own state, so the R-1
// deliveries of a round run side by side, each in its peer's lane. What the
// sequential order still decides is WHERE a round stops: at the first peer
// whose handler faults (a Go panic or block, main.go:142, 242, 308) or, in
// RAFT mode, whose answer carries a higher term. Every lane therefore saves
// its registers before a round, handles its message, and after a segment
// ballot locates that first peer p*, lanes above p* restore what they saved
// (their message was never delivered). Handlers write the ring only after
// p* is known. Commit rules and timer order are segment reductions.
//
// Compared with the one-lane-per-group form of Group (raft_device.hpp, still
// used by the message-level handler batches): one copy of each handler
// instead of R unrolled ones, ~1/R of the registers per lane, no LDS slab,
// and the group's loads issued by R lanes at once. Semantics are identical,
// handler by handler: every function cites the Group method it mirrors,
// which in turn cites main.go.
#pragma once
#include "tick_common.hpp"

namespace raftstep {

constexpr int SEGW = 8;   // lanes per group

enum : uint32_t {   // per-lane dirty bits (fields written back by store)
  SD_TERM = 1, SD_LAST = 2, SD_COMMIT = 4, SD_DL = 8, SD_RS = 16, SD_HW = 32, SD_LT = 64, SD_PM = 128, SD_PN = 256
};

__device__ __forceinline__ int seg_lane() { return int(threadIdx.x & 63u); }

template <int R, int SEM>
struct Seg {
  // ---- lane identity
  int me;          // replica id of this lane
  bool act;        // me < R
  int sb0l;        // first lane of this segment in the wave
  uint32_t ri;     // element index of this replica's slot in the [Gp][R] planes: g*R + r
                   // (r = 0 on idle lanes); the R slots of a group are contiguous
  // ---- this replica's state (registers)
  int term, last, commit, dl, dur, hw, ltm, role, vote;
  int pm, pn;      // primary leader's MatchIndex / NextIndex for this replica (as its peer)
  uint32_t dirty;
  // ---- group state (the same value in every lane of the segment)
  uint32_t g;
  uint64_t key;
  int64_t tick;
  int32_t now;
  int primary, fault, meta0;
  uint32_t rot, rota, rotb;
  int sbd, sb2;    // ring segment boundaries (gsb, gsb2)
  bool rot_dirty;  // rot / sbd changed (align_ring)
  uint32_t iso;
  uint32_t giso;   // EXT leader-isolation victims (giso plane)
  bool giso_dirty;
  int ecur;        // client entries appended to every leader this tick
  // per-tick statistics: S_COMMITTED in full, the others (each < 256 per
  // group and tick) packed 8 bits apiece, to keep the lane's registers down
  int st_commit;
  uint32_t st_pack0, st_pack1;
  __device__ __forceinline__ void stat_add(int s, int v) {
    if (s == S_COMMITTED) { st_commit += v; return; }
    const int k = s - 1;   // S_WON .. S_LEADER_GROUPS -> 0..6
    if (k < 4) st_pack0 += uint32_t(v) << (8 * k);
    else st_pack1 += uint32_t(v) << (8 * (k - 4));
  }
  __device__ __forceinline__ int stat(int s) const {
    if (s == S_COMMITTED) return st_commit;
    const int k = s - 1;
    return int(((k < 4 ? st_pack0 >> (8 * k) : st_pack1 >> (8 * (k - 4)))) & 255u);
  }
  __device__ __forceinline__ void stat_reset() { st_commit = 0; st_pack0 = st_pack1 = 0; }

  // ------------------------------------------------ segment primitives --
  __device__ __forceinline__ int bc(int v, int src) const { return __shfl(v, sb0l + src); }
  __device__ __forceinline__ uint64_t bc64(uint64_t v, int src) const {
    return (uint64_t(uint32_t(__shfl(int(v >> 32), sb0l + src))) << 32) | uint32_t(__shfl(int(uint32_t(v)), sb0l + src));
  }
  __device__ __forceinline__ uint32_t mask(bool p) const { return uint32_t(__ballot(p) >> sb0l) & 0xFFu; }
  __device__ __forceinline__ int first_of(uint32_t m) const { return m ? int(__builtin_ctz(m)) : SEGW; }
  __device__ __forceinline__ uint64_t seg_min64(uint64_t v) const {
#pragma unroll
    for (int o = 1; o < SEGW; o <<= 1) {
      const uint64_t w = uint64_t(uint32_t(__shfl_xor(int(uint32_t(v)), o))) |
                         (uint64_t(uint32_t(__shfl_xor(int(v >> 32), o))) << 32);
      v = w < v ? w : v;
    }
    return v;
  }
  __device__ __forceinline__ int seg_max(int v) const {
#pragma unroll
    for (int o = 1; o < SEGW; o <<= 1) v = max(v, __shfl_xor(v, o));
    return v;
  }
  __device__ __forceinline__ void raise(int f) {   // uniform
    if (!fault) fault = f;
  }
  __device__ __forceinline__ bool alive() const { return fault == 0; }
  __device__ __forceinline__ bool dropped(int a, int b) const { return ((iso >> a) | (iso >> b)) & 1u; }

  // ---------------------------------------------------------- load/store --
  // Group::begin + Group::load, every replica in its own lane, deadlines eager.
  __device__ __forceinline__ void begin(const DevPlanes& P, const Trace& T, uint32_t g_) {
    const int lane = seg_lane();
    sb0l = lane & ~(SEGW - 1);
    me = lane & (SEGW - 1);
    act = me < R;
    g = g_;
    ri = rix<R>(g, act ? me : 0);
    key = group_key(T.seed, P.gbase + g);
    tick = T.tick;
    now = T.now;
    iso = 0;
    ecur = 0;
    stat_reset();
    const int m = at(P.gmeta, g);
    meta0 = m;
    primary = m & 0xF;
    fault = (m >> 4) & 7;
    rot = at(P.grot, g);
    rota = at(P.grota, g);
    sbd = at(P.gsb, g);
    rotb = at(P.grotb, g);
    sb2 = at(P.gsb2, g);
    rot_dirty = false;
    giso = at(P.giso, g);
    giso_dirty = false;
    dirty = 0;
  }
  __device__ __forceinline__ void load(const DevPlanes& P) {
    const int hbt = at(P.hb, g);
    term = at(P.term, ri);
    last = at(P.last, ri);
    commit = at(P.commit, ri);
    const uint32_t x = at(P.rs, ri);
    role = int(x & 3u);
    vote = int((x >> 2) & 15u);
    dur = int(x >> 6);
    hw = (SEM == SEM_RAFT) ? at(P.hwm, ri) : 0;
    ltm = at(P.lterm, ri);
    const int ts = at(P.tstart, ri);
    pm = 0; pn = 0;
    const bool peer_of_pri = primary < R && me != primary;
    const LxRec gx = (uses_glx(meta0) && primary < R) ? P.glx[g] : LxRec{0, 0};
    const bool mrow = msync_peer(meta0, gx, me);   // this lane's MatchIndex row implicit (MSYNC)
    if (peer_of_pri && !mrow) {
      pm = at(P.lmatch, ri);
      if constexpr (SEM == SEM_RAFT) pn = at(P.lnext, ri);
    }
    dl = (role == ROLE_L ? ts : max(ts, hbt)) + dur;   // effective timer start counts the heartbeat
    if ((meta0 & M_SSYNC) && primary < R && act) {     // compressed state (Group::load)
      const SsRec s = P.gss[g];
      term = ss_term(s, me, meta0, gx); last = ss_last(s, me, primary, meta0, gx);
      commit = ss_commit(s, me, primary, meta0, gx, commit); ltm = ss_term(s, me, meta0, gx);
      dirty |= SD_TERM | SD_LAST | SD_COMMIT | SD_LT;
    }
    if (!act) { role = ROLE_F; dl = I32MAX; last = 0; hw = 0; }
    // rows the fast kernel kept implicit (MSYNC): MatchIndex = LastApplied
    // (RAFT also NextIndex = LastApplied+1, high-water mark = LastApplied)
    if ((meta0 & M_MSYNC) && primary < R && act) {
      if (me != primary && mrow) {
        pm = last;
        dirty |= SD_PM;
        if constexpr (SEM == SEM_RAFT) { pn = last + 1; dirty |= SD_PN; }
      }
      if constexpr (SEM == SEM_RAFT) {
        if (hw < last) { hw = last; dirty |= SD_HW; }   // max(plane, LastApplied) (HWX)
      }
    }
  }
  // Group::store: this lane's dirty fields, then group placement (ring phase
  // of empty logs, primary rows, gmeta).
  __device__ __forceinline__ void store(const DevPlanes& P, uint32_t next_phase) {
    if (act) {
      if (dirty & SD_TERM) at(P.term, ri) = term;
      if (dirty & SD_LAST) at(P.last, ri) = last;
      if (dirty & SD_COMMIT) at(P.commit, ri) = commit;
      if (dirty & SD_DL) at(P.tstart, ri) = dl - dur;
      if (dirty & SD_RS) at(P.rs, ri) = int32_t(uint32_t(role) | (uint32_t(vote) << 2) | (uint32_t(dur) << 6));
      if (SEM == SEM_RAFT && (dirty & SD_HW)) at(P.hwm, ri) = hw;
      if (dirty & SD_LT) at(P.lterm, ri) = ltm;
      if (dirty & SD_PM) at(P.lmatch, ri) = pm;
      if (SEM == SEM_RAFT && (dirty & SD_PN)) at(P.lnext, ri) = pn;
    }
    // logs still empty: the next tick's first entry goes to the global phase
    const bool empty = mask(act && (last != 0 || (SEM == SEM_RAFT && hw != 0))) == 0u;
    uint32_t rt = rot;
    int sbn = sbd;
    bool rd = rot_dirty;
    if (empty && !fault) { rt = next_phase & P.kmask; sbn = 0; rd = true; }
    // primary placement: the leader of the highest term (Group::store)
    const uint32_t leaders = mask(act && role == ROLE_L);
    int pri = primary;
    if (!fault && leaders) {
      // highest term, ties to the lowest id; the current primary keeps the planes on a tie
      const uint64_t kv = (act && role == ROLE_L)
                              ? ((uint64_t(uint32_t(~term) ^ 0x80000000u) << 3) | uint64_t(me)) : ~0ull;
      int best = int(seg_min64(kv) & 7u);
      if (pri < R && ((leaders >> pri) & 1u) && bc(term, pri) == bc(term, best)) best = pri;
      if (best != pri) {
        if (act) {
          const int a = at(P.lmatch, ri);
          at(P.lmatch, ri) = at(prow(P.xmatch, best * R + me, P.Gp), g);
          if (pri < R) at(prow(P.xmatch, pri * R + me, P.Gp), g) = a;
          if constexpr (SEM == SEM_RAFT) {
            const int b = at(P.lnext, ri);
            at(P.lnext, ri) = at(prow(P.xnext, best * R + me, P.Gp), g);
            if (pri < R) at(prow(P.xnext, pri * R + me, P.Gp), g) = b;
          }
        }
        pri = best;
      }
    }
    const uint32_t nonf = mask(act && role != ROLE_F);
    const uint32_t cands = mask(act && role == ROLE_C);
    const bool led = pri < R && ((leaders >> pri) & 1u);
    const uint32_t others = nonf & ~(1u << (pri & 15));
    const bool steady = led && others == 0u;
    const bool one = led && others != 0u && (others & (others - 1u)) == 0u;
    const bool onecand = one && (others & cands) != 0u;
    const int sx = one ? first_of(others) : 0;
    const bool onestale = SEM == SEM_RAFT && one && (others & leaders) != 0u && bc(term, sx) < bc(term, pri & 7);
    // (DEFER stays until the window tail: the general kernel may run beside the
    // next tick's fast kernels, which must keep leaving this group alone)
    const int m = pri | (fault << 4) | (steady ? M_STEADY : 0) | (onecand ? M_ONECAND : 0) |
                  (onestale ? M_ONESTALE : 0) | (meta0 & M_DEFER);
    if (me == 0) {
      if (rd) {   // (grota never changes here)
        at(P.grot, g) = uint16_t(rt);
        at(P.gsb, g) = sbn;
      }
      if (m != meta0) at(P.gmeta, g) = uint16_t(m);
      if (giso_dirty) at(P.giso, g) = uint8_t(giso);
    }
  }

  // ---------------------------------------------------------------- ring --
  __device__ __forceinline__ uint32_t ring_off(const DevPlanes& P, int r, int idx) const {
    return ring_in_tile(g, R, ring_slot(idx, rot, rota, rotb, sbd, sb2, P.kmask), uint32_t(r));
  }
  __device__ __forceinline__ int32_t& ring_term(const DevPlanes& P, int r, int idx) const {
    return at(P.log_term + ring_tile(g, P.KP, R), ring_off(P, r, idx));
  }
  __device__ __forceinline__ int64_t& ring_value(const DevPlanes& P, int r, int idx) const {
    return at(P.log_value + ring_tile(g, P.KP, R), ring_off(P, r, idx));
  }
  __device__ __forceinline__ uint32_t& ring_crc(const DevPlanes& P, int r, int idx) const {
    return at(P.log_crc + ring_tile(g, P.KP, R), ring_off(P, r, idx));
  }
  // Group::term_at for this lane's own log
  __device__ __forceinline__ int own_term_at(const DevPlanes& P, int idx) const {
    return idx == last ? ltm : ring_term(P, me, idx);
  }
  __device__ __forceinline__ void set_lterm(int t) {
    if (ltm != t) { ltm = t; dirty |= SD_LT; }
  }
  __device__ __forceinline__ void set_term(int t) {
    if (term != t) { term = t; dirty |= SD_TERM; }
  }
  __device__ __forceinline__ void set_role(int r_) { role = r_; dirty |= SD_RS; }
  __device__ __forceinline__ void set_vote(int v) { vote = v; dirty |= SD_RS; }
  __device__ __forceinline__ void reset_timer() { dl = now + dur; dirty |= SD_DL; }
  __device__ __forceinline__ int draw(const Trace& T, bool cand) const {
    // rand.Intn (main.go:114, 194); inline here: the segment form has one copy per call site
    const uint64_t h = rng_k(key, uint32_t(me), cand ? ST_TIMER_C : ST_TIMER_F, uint64_t(tick));
    return cand ? T.c_min + int(uint32_t(h >> 32) % uint32_t(T.c_span)) : T.f_min + int(uint32_t(h >> 32) % uint32_t(T.f_span));
  }
  __device__ __forceinline__ void enter_follower(const Trace& T) {   // FollowerRun entry (main.go:113-115)
    set_role(ROLE_F);
    dur = draw(T, false);
    dl = now + dur;
    dirty |= SD_DL;
  }
  __device__ __forceinline__ void enter_candidate(const Trace& T) {  // CandidateRun entry (main.go:194-195)
    set_role(ROLE_C);
    dur = draw(T, true);
    dl = now + dur;
    dirty |= SD_DL;
  }

  // Register snapshot of a peer lane for the round-stop rule (see the
  // header): only what a handler changes before the stop point is known
  // (LastApplied / CommitIndex / ring change after it).
  struct Saved {
    int term, dl;
    uint32_t rs, dirty;
    __device__ __forceinline__ int role() const { return int(rs & 3u); }
  };
  __device__ __forceinline__ Saved save() const {
    return Saved{term, dl, uint32_t(role) | (uint32_t(vote) << 2) | (uint32_t(dur) << 6), dirty};
  }
  __device__ __forceinline__ void restore(const Saved& s) {
    term = s.term; dl = s.dl; dirty = s.dirty;
    role = int(s.rs & 3u); vote = int((s.rs >> 2) & 15u); dur = int(s.rs >> 6);
  }

  // Entry j of the AppendEntries leader c sends (Logs[j] = c's entry
  // from+j): entries c appended this tick are regenerated from the trace
  // RNG, older ones read from c's ring (written by c's lane; the round
  // starts with a workgroup fence, see leader rounds). A leader that has a
  // leader round was a leader when the tick began, so it appended ecur
  // entries of its term at [last-ecur+1, last].
  struct Src {
    int leader, from, a_n, a_from, a_term;
    uint64_t a_vb;   // value base of c's appends this tick (cv_base)
  };
  __device__ __forceinline__ Src leader_src(const DevPlanes& P, int c, int lt, int ll) const {
    return Src{c, 1, ecur, ll - ecur + 1, lt, ecur ? cv_base(P, key, uint32_t(c), tick, g) : 0ull};
  }
  __device__ __forceinline__ void fetch(const DevPlanes& P, const Src& s, int j, int& t, int64_t& v, uint32_t& c) const {
    const int idx = s.from + j;
    c = 0;
    if (s.a_n && idx >= s.a_from) {
      t = s.a_term;
      v = cv_value(s.a_vb, uint32_t(idx - s.a_from), cv_stride(P));   // entry_value
      if (P.crc_on) c = crc_entry(P.crc_tab, t, v);
    } else {
      const uint64_t tb = ring_tile(g, P.KP, R);
      const uint32_t o = ring_off(P, s.leader, idx);
      t = at(P.log_term + tb, o);
      v = at(P.log_value + tb, o);
      if (P.crc_on) c = at(P.log_crc + tb, o);
    }
  }
  // Group::copy_entries into this lane's ring (loads of a batch of 4 issued before its stores)
  __device__ __forceinline__ int copy_entries(const DevPlanes& P, const Src& s, int base, int j0, int n) {
    int tl = 0;
    for (int j = j0; j < n; j += 4) {
      int t[4];
      int64_t v[4];
      uint32_t c[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (j + u < n) fetch(P, s, j + u, t[u], v[u], c[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (j + u >= n) break;
        ring_term(P, me, base + 1 + j + u) = t[u];
        ring_value(P, me, base + 1 + j + u) = v[u];
        if (P.crc_on) ring_crc(P, me, base + 1 + j + u) = c[u];
        tl = t[u];
      }
    }
    return tl;
  }
  // Leader c's log term at idx (Group::term_at(c, idx)), read by any lane of the segment.
  __device__ __forceinline__ int leader_term_at(const DevPlanes& P, int c, int c_last, int c_ltm, int idx) const {
    return idx == c_last ? c_ltm : ring_term(P, c, idx);
  }
  __device__ __forceinline__ int corrupted(const DevPlanes& P) const {
    if (!P.crc_on || !P.corrupt_p) return 0;
    return (rng_k(key, uint32_t(me), ST_CORRUPT, uint64_t(tick)) & 0xFFFF) < P.corrupt_p;
  }

  // ------------------------------------------------------- client (step 1)
  // run_tick step 1: every Leader appends E entries (main.go:327-329).
  __device__ __forceinline__ void client_append(const DevPlanes& P, const Trace& T, uint32_t E) {
    const bool ld = act && role == ROLE_L && alive();
    const uint32_t lm = mask(ld);
    if (!lm || !alive()) return;
    // align_ring runs for the first leader iff every log is empty
    if (mask(act && (last != 0 || (SEM == SEM_RAFT && hw != 0))) == 0u) {
      rot = uint32_t(T.entries_before(T.tick)) & P.kmask;
      sbd = 0;
      rot_dirty = true;
    }
    int n_ok = 0;
    if (ld) {
      const int room = I32MAX - last;
      n_ok = int(E) <= room ? int(E) : room;
    }
    // a leader that overflows raises F_OVERFLOW after its appends; later leaders skip theirs
    const uint32_t ov = mask(ld && n_ok < int(E));
    const int first_ov = first_of(ov);
    if (ld && me <= first_ov) {
      const uint64_t vb = cv_base(P, key, uint32_t(me), tick, g);
      const int l = last;
      const int e0 = n_ok > int(P.K) ? n_ok - int(P.K) : 0;
      for (int e = e0; e < n_ok; ++e) {
        const int64_t v = cv_value(vb, uint32_t(e), cv_stride(P));   // entry_value
        ring_term(P, me, l + 1 + e) = term;
        ring_value(P, me, l + 1 + e) = v;
        if (P.crc_on) ring_crc(P, me, l + 1 + e) = crc_entry(P.crc_tab, term, v);
      }
      if (n_ok) {
        last = l + n_ok;
        dirty |= SD_LAST;
        set_lterm(term);
        if (SEM == SEM_RAFT && last > hw) { hw = last; dirty |= SD_HW; }
      }
    }
    if (ov) raise(F_OVERFLOW);
  }

  // MatchIndex (and RAFT NextIndex) of leader c for this lane: the primary's
  // rows are resident (pm/pn), a further leader's live in xmatch / xnext.
  __device__ __forceinline__ void load_rows(const DevPlanes& P, int c, bool peer, int& m, int& nx) const {
    m = 0; nx = 0;
    if (!peer) return;
    if (primary == c) { m = pm; nx = pn; }
    else {
      m = at(prow(P.xmatch, c * R + me, P.Gp), g);
      if constexpr (SEM == SEM_RAFT) nx = at(prow(P.xnext, c * R + me, P.Gp), g);
    }
  }
  // Group::store_match / store_next for one peer lane (rows are written where they were read: pri)
  __device__ __forceinline__ void store_rows(const DevPlanes& P, int c, int pri, bool peer, bool dm, int m, bool dn,
                                             int nx) {
    if (!peer) return;
    if (pri == c) {
      if (dm) { pm = m; dirty |= SD_PM; }
      if (SEM == SEM_RAFT && dn) { pn = nx; dirty |= SD_PN; }
    } else {
      if (dm) at(prow(P.xmatch, c * R + me, P.Gp), g) = m;
      if (SEM == SEM_RAFT && dn) at(prow(P.xnext, c * R + me, P.Gp), g) = nx;
    }
  }

  // ============================================================ REF rounds
  // LeaderRun default branch (main.go:332-391), Group::leader_round.
  __device__ __forceinline__ void leader_round(const DevPlanes& P, const Trace& T, int c) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // c's ring stores before the peers read them
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const int lt = bc(term, c), ll = bc(last, c), lc = bc(commit, c), lltm = bc(ltm, c);
    Src src = leader_src(P, c, lt, ll);
    const bool peer = act && me != c;
    int m, nx_unused;
    load_rows(P, c, peer, m, nx_unused);
    const bool drop = peer && dropped(c, me);
    const bool part = peer && !drop;
    const Saved sv = save();
    int f = 0, ok = 0, match = 0;
    bool copy = false;
    int q_n = 0, q_prev = 0, j0 = 0;
    if (part) {
      // AppendEntries for this peer (main.go:341-372), NextIndex = MatchIndex+1
      const int nxt = m + 1;
      int prev_term = lt;
      if (nxt <= ll) {
        if (nxt == 1) { q_n = ll; q_prev = 0; prev_term = lt; src.from = 1; }              // 343-351
        else if (nxt < 1 || m > ll) f = F_PANIC_GETLOG;
        else if (m <= ll - int(P.K)) f = F_RING_EVICTED;
        else { prev_term = leader_term_at(P, c, ll, lltm, m); q_prev = m; q_n = ll - nxt + 1; src.from = nxt; }  // 353-360
      } else { q_n = 0; q_prev = m; prev_term = lt; }                                       // 364-371
      if (!f) {
        // Run (main.go:98-109) -> the receiver's handler
        if (role == ROLE_F) {                               // FollowerRun case AEReq (main.go:121-156)
          match = last;
          reset_timer();                                    // 124-127
          bool rej = lt < term;                             // 129-133
          const int l = last;
          if (!rej && l > 0) {                              // 135
            if (int64_t(l) + q_n < q_prev) rej = true;      // 137-140
            else if (q_prev < 1 || q_prev > l) f = F_PANIC_GETLOG;   // 142 -> 404
            else if (q_prev <= l - int(P.K)) f = F_RING_EVICTED;
            else if (own_term_at(P, q_prev) != prev_term) rej = true;  // 142-145
          }
          if (!rej && !f && int64_t(l) + q_n > I32MAX) f = F_OVERFLOW;
          j0 = q_n > int(P.K) ? q_n - int(P.K) : 0;
          if (!rej && !f && P.crc_on) {                     // EXT: verify what will be stored
            const int cor = corrupted(P);
            for (int j = j0; j < q_n; ++j) {
              int t; int64_t v; uint32_t cc;
              fetch(P, src, j, t, v, cc);
              if (cor && j == q_n - 1) v ^= 1;
              if (crc_entry(P.crc_tab, t, v) != cc) { rej = true; break; }
            }
          }
          if (!rej && !f) { ok = 1; copy = q_n > 0; match = l + q_n; }
        } else if (role == ROLE_C) {                        // CandidateRun case AEReq (main.go:200-223)
          match = last;
          if (lt >= term) { ok = 1; set_vote(1); set_term(lt); enter_follower(T); }
        } else {                                            // LeaderRun case AEReq (main.go:309-326)
          match = 0;
          if (lt > term) { ok = 1; set_vote(0); set_term(lt); enter_follower(T); }
        }
      }
    }
    // the round stops at the first peer that faults
    const uint32_t fm = mask(part && f != 0);
    const int ps = first_of(fm);
    if (me > ps) restore(sv);
    const bool done = part && me < ps;   // message delivered and answered
    if (done && copy) {                  // 148-149: append all Logs at the end, the last K kept in the ring
      const int l = last;
      const int tl = copy_entries(P, src, l, j0, q_n);
      last = l + q_n;
      dirty |= SD_LAST;
      set_lterm(tl);
    }
    if (done && ok && sv.role() == ROLE_F) {  // follower success path: commit min(LC, len+1), Term (151-156)
      if (lc > commit) {
        const int64_t cap = int64_t(last) + 1;
        const int nc = int64_t(lc) < cap ? lc : int(cap);
        if (nc != commit) { commit = nc; dirty |= SD_COMMIT; }
      }
      set_term(lt);
    }
    // the primary leader stepped down (LeaderRun case AEReq, main.go:317)
    if (mask(done && ok && sv.role() == ROLE_L && me == primary)) primary = NO_PRIMARY;
    if (fm) raise(bc(f, ps));
    stat_add(S_AE_OK, __builtin_popcount(mask(done && ok)));
    stat_add(S_AE_FAIL, __builtin_popcount(mask((done && !ok) || (drop && me < ps))));
    bool dm = false;
    if (done && ok && match != m) { m = match; dm = true; }  // 375-378
    if (alive()) {   // commit rule (main.go:381-391): exact-value histogram over the peers
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const int mq = bc(m, q);
        cnt += (q != c && mq == m) ? 1 : 0;
      }
      const uint32_t qual = mask(peer && 2 * cnt > R && m > lc);
      if (qual) {
        const int nc = bc(m, first_of(qual));
        stat_add(S_COMMITTED, nc - lc);
        if (me == c) { commit = nc; dirty |= SD_COMMIT; }
      }
    }
    store_rows(P, c, primary, peer, dm, m, false, 0);   // c never changes role in its own REF round
  }

  // CandidateRun default branch (main.go:253-284), Group::candidate_round.
  __device__ __forceinline__ int candidate_round(const DevPlanes& P, const Trace& T, int c) {
    if (me == c) set_vote(1);                                // 256
    const int ct = bc(term, c);
    const bool peer = act && me != c;
    const bool part = peer && !dropped(c, me);
    const Saved sv = save();
    int f = 0, gr = 0;
    if (part) {                                              // 259-269 -> the receiver's VReq case
      if (role == ROLE_F) {                                  // main.go:157-170
        if (!(ct < term || vote != 0)) { reset_timer(); set_term(ct); set_vote(1); gr = 1; }
      } else if (role == ROLE_C) {                           // main.go:224-246
        if (ct > term) { set_vote(1); set_term(ct); enter_follower(T); gr = 1; }
        else { reset_timer(); f = F_DEADLOCK_VRES; }         // 242: reply into its own VRes
      } else {
        f = F_DEADLOCK_LEADER_VREQ;                          // main.go:308: no VReq case
      }
    }
    const uint32_t fm = mask(part && f != 0);
    const int ps = first_of(fm);
    if (me > ps) restore(sv);
    if (fm) raise(bc(f, ps));
    const uint32_t gm = mask(part && me < ps && gr);
    const int count = 1 + __builtin_popcount(gm);
    stat_add(S_VOTES, __builtin_popcount(gm));
    if (alive() && 2 * count > R) {                          // 273
      if (me == c) set_role(ROLE_L);                         // 274
      if (primary == NO_PRIMARY) {                           // 275-282: MatchIndex 0 / NextIndex 1
        if (peer) { pm = 0; dirty |= SD_PM; }
        primary = c;
      } else if (peer) {
        at(prow(P.xmatch, c * R + me, P.Gp), g) = 0;
      }
      stat_add(S_WON, 1);
      return 1;
    }
    return 0;
  }

  // timer.C (main.go:171-177, 248-251), Group::timeout_fire, for lane b
  __device__ __forceinline__ void timeout_fire(const Trace& T, int b) {
    const int t = bc(term, b);
    if (t >= I32MAX) { raise(F_OVERFLOW); return; }
    if (me == b) {
      term = t + 1;
      dirty |= SD_TERM;
      if constexpr (SEM == SEM_RAFT) set_vote(b + 1);   // votes for itself
      enter_candidate(T);
    }
    stat_add(S_BUMPS, 1);
  }

  // =========================================================== RAFT rounds
  // A higher term in any RPC: adopt it, forget the vote, become a follower
  // (Group::r_observe). Returns 1 if this lane was a non-follower that stepped down.
  __device__ __forceinline__ int r_observe(const Trace& T, int t) {
    if (t <= term) return 0;
    set_term(t);
    set_vote(0);
    if (role != ROLE_F) { enter_follower(T); return 1; }
    return 0;
  }

  // Group::r_leader_round
  __device__ __forceinline__ void r_leader_round(const DevPlanes& P, const Trace& T, int c) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const int lt = bc(term, c), ll = bc(last, c), lc = bc(commit, c), lh = bc(hw, c), lltm = bc(ltm, c);
    const int K = int(P.K);
    Src src = leader_src(P, c, lt, ll);
    const bool peer = act && me != c;
    const int pri = primary;   // rows are written back where they were read
    int m, nx;
    load_rows(P, c, peer, m, nx);
    const bool drop = peer && dropped(c, me);
    const bool part = peer && !drop;
    const Saved sv = save();
    int f = 0, ok = 0, match = 0, rterm = 0, stepped = 0;
    bool copy = false;
    int q_n = 0, q_prev = 0, jc = 0;
    if (part) {
      const int nxt = nx;
      int prev_term = 0;
      if (nxt < 1 || nxt > ll + 1) f = F_PANIC_GETLOG;
      else if (nxt <= lh - K) f = F_RING_EVICTED;
      else {
        q_prev = nxt - 1;
        if (q_prev > 0) {
          if (q_prev <= lh - K) f = F_RING_EVICTED;
          else prev_term = leader_term_at(P, c, ll, lltm, q_prev);
        }
        q_n = ll - q_prev;
        src.from = nxt;
      }
      if (!f) {   // Group::r_deliver_ae
        stepped = r_observe(T, lt);
        rterm = term;
        match = last;
        if (lt < term) {
        } else if (role == ROLE_L) {                  // same-term second leader: cannot happen
        } else {
          if (role == ROLE_C) enter_follower(T);
          reset_timer();
          const int l = last;
          bool rej = false;
          if (q_prev > l) rej = true;                 // log too short: hint = last
          else if (q_prev > 0) {
            if (q_prev <= hw - K) f = F_RING_EVICTED;
            else if (own_term_at(P, q_prev) != prev_term) {   // conflict: back off to the committed prefix
              match = q_prev - 1 < commit ? q_prev - 1 : commit;
              rej = true;
            }
          }
          if (!rej && !f && P.crc_on) {               // EXT: verify what will be stored
            const int cor = corrupted(P);
            const int j0 = q_n > K ? q_n - K : 0;
            for (int j = j0; j < q_n; ++j) {
              int t; int64_t v; uint32_t cc;
              fetch(P, src, j, t, v, cc);
              if (cor && j == q_n - 1) v ^= 1;
              if (crc_entry(P.crc_tab, t, v) != cc) { match = q_prev; rej = true; break; }
            }
          }
          if (!rej && !f && int64_t(q_prev) + q_n > I32MAX) f = F_OVERFLOW;
          if (!rej && !f) {
            // skip entries already present, truncate at the first conflict
            int j = 0;
            for (; j < q_n; ++j) {
              const int idx = q_prev + 1 + j;
              if (idx > l) break;
              if (idx <= hw - K) { f = F_RING_EVICTED; break; }
              int t; int64_t v; uint32_t cc;
              fetch(P, src, j, t, v, cc);
              if (own_term_at(P, idx) != t) break;
            }
            if (!f) {
              jc = j;
              copy = j < q_n;
              ok = 1;
              match = q_prev + q_n;
            }
          }
        }
      }
    }
    // the round stops at the first peer that faults or answers a higher term
    const bool stop_me = part && (f != 0 || (rterm > lt));
    const uint32_t fm = mask(stop_me);
    const int ps = first_of(fm);
    if (me > ps) restore(sv);
    const bool done = part && me < ps;
    if (done && ok) {
      if (copy) {
        const int tl = copy_entries(P, src, q_prev, jc, q_n);
        const int nl = q_prev + q_n;
        if (nl != last) { last = nl; dirty |= SD_LAST; }
        set_lterm(tl);
        if (nl > hw) { hw = nl; dirty |= SD_HW; }
      }
      const int last_new = q_prev + q_n;
      if (lc > commit) {
        const int nc = lc < last_new ? lc : last_new;
        if (nc != commit) { commit = nc; dirty |= SD_COMMIT; }
      }
    }
    if (mask(part && me <= ps && stepped && me == primary)) primary = NO_PRIMARY;
    const bool faulted = fm && bc(f, ps) != 0;
    if (faulted) raise(bc(f, ps));
    bool stop = false;
    if (fm && !faulted) {                               // the leader observes the higher term
      const int t2 = bc(rterm, ps);
      stop = true;
      if (me == c) r_observe(T, t2);
      if (primary == c) primary = NO_PRIMARY;           // c stepped down (it was a leader)
      stat_add(S_AE_FAIL, 1);
    }
    stat_add(S_AE_OK, __builtin_popcount(mask(done && ok)));
    stat_add(S_AE_FAIL, __builtin_popcount(mask((done && !ok) || (drop && me < ps))));
    bool dm = false, dn = false;
    if (done) {
      if (ok) { m = match; nx = match + 1; dm = dn = true; }
      else {
        int nn = nx - 1 < match + 1 ? nx - 1 : match + 1;
        nn = nn < 1 ? 1 : nn;
        if (nn != nx) { nx = nn; dm = dn = true; }
      }
    }
    if (alive() && !stop) {   // majority order statistic, current-term rule (Group::r_commit_rule)
      const int v = me == c ? ll : m;
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < R; ++q) cnt += bc(v, q) >= v ? 1 : 0;
      const int N = seg_max(act && cnt >= R / 2 + 1 ? v : -1);
      if (N > lc) {
        int fc = 0, tn = 0;
        if (N < 1 || N > ll) fc = F_PANIC_GETLOG;
        else if (N <= lh - K) fc = F_RING_EVICTED;
        else if (me == c) tn = own_term_at(P, N);
        tn = bc(tn, c);
        if (fc) raise(fc);
        else if (tn == lt) {
          stat_add(S_COMMITTED, N - lc);
          if (me == c) { commit = N; dirty |= SD_COMMIT; }
        }
      }
    }
    store_rows(P, c, pri, peer, dm, m, dn, nx);
  }

  // Group::r_candidate_round
  __device__ __forceinline__ int r_candidate_round(const DevPlanes& P, const Trace& T, int c) {
    const int ct = bc(term, c), cl = bc(last, c);
    const int clt = cl > 0 ? bc(ltm, c) : 0;
    const bool peer = act && me != c;
    const bool part = peer && !dropped(c, me);
    const Saved sv = save();
    int gr = 0, rt = 0, stepped = 0;
    if (part) {   // Group::r_deliver_vr
      stepped = r_observe(T, ct);
      rt = term;
      if (!(ct < term)) {
        const int mt = last > 0 ? ltm : 0;
        const bool uptodate = clt > mt || (clt == mt && cl >= last);
        if ((vote == 0 || vote == c + 1) && uptodate) { set_vote(c + 1); reset_timer(); gr = 1; }
      }
    }
    const uint32_t sm = mask(part && rt > ct);
    const int ps = first_of(sm);
    if (me > ps) restore(sv);
    if (mask(part && me <= ps && stepped && me == primary)) primary = NO_PRIMARY;
    bool stop = false;
    if (sm) {                                             // the candidate observes the higher term
      const int t2 = bc(rt, ps);
      stop = true;
      if (me == c) r_observe(T, t2);
      if (primary == c) primary = NO_PRIMARY;
    }
    const uint32_t gm = mask(part && me < ps && gr);
    const int count = 1 + __builtin_popcount(gm);
    stat_add(S_VOTES, __builtin_popcount(gm));
    if (alive() && !stop && bc(role, c) == ROLE_C && 2 * count > R) {
      if (me == c) set_role(ROLE_L);
      if (primary == NO_PRIMARY) primary = c;
      if (peer) {   // MatchIndex 0, NextIndex = last + 1 for every peer
        if (primary == c) { pm = 0; pn = cl + 1; dirty |= SD_PM | SD_PN; }
        else {
          at(prow(P.xmatch, c * R + me, P.Gp), g) = 0;
          at(prow(P.xnext, c * R + me, P.Gp), g) = cl + 1;
        }
      }
      stat_add(S_WON, 1);
      return 1;
    }
    return 0;
  }

  // ================================================================ tick
  // run_tick (tick_common.hpp), segment-parallel.
  __device__ __forceinline__ void run(const DevPlanes& P, const Trace& T, uint32_t E) {
    if (T.iso_p) {
      const uint32_t g0 = giso;
      iso = tick_iso_mask<R>(key, T, giso, mask(act && role == ROLE_L), true);
      giso_dirty |= giso != g0;
    }
    ecur = int(E);
    if (E) client_append(P, T, E);
    // 2. rounds in ascending replica id, against the roles as they are now
    int c = -1;
    while (alive()) {
      const uint32_t rest = mask(act && role != ROLE_F && me > c);
      if (!rest) break;
      c = first_of(rest);
      const bool isl = bc(role, c) == ROLE_L;
      if constexpr (SEM == SEM_RAFT) {
        if (isl) r_leader_round(P, T, c);
        else r_candidate_round(P, T, c);
      } else {
        if (isl) leader_round(P, T, c);                  // main.go:332-391
        else candidate_round(P, T, c);                   // main.go:253-284
      }
    }
    // 3. expired election timers in (deadline, id) order; each new candidate
    //    runs its vote round at once (main.go:171-177, 248-251 -> 253-284)
#pragma unroll 1
    for (int it = 0; it < R && alive(); ++it) {
      const bool cand = act && role != ROLE_L && dl <= now;
      const uint64_t kv = cand ? ((uint64_t(uint32_t(dl) ^ 0x80000000u) << 3) | uint64_t(me)) : ~0ull;
      const uint64_t best = seg_min64(kv);
      if (best == ~0ull) break;
      const int b = int(best & 7u);
      timeout_fire(T, b);
      if (!alive()) break;
      if constexpr (SEM == SEM_RAFT) r_candidate_round(P, T, b);
      else candidate_round(P, T, b);
    }
    if (!alive()) stat_add(S_FAULTS, 1);
    else if (mask(act && role == ROLE_L)) stat_add(S_LEADER_GROUPS, 1);
  }
  __device__ __forceinline__ void next_tick(const Trace& T) {
    tick = T.tick;
    now = T.now;
    iso = 0;
    ecur = 0;
    stat_reset();
  }
};

}  // namespace raftstep
