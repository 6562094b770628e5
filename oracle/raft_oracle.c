/*
 * raft_oracle.c — TEST INFRASTRUCTURE ONLY (see raft_oracle.h).
 *
 * Plain-C restatement of eastwd/raft-sample main.go, one group at a time,
 * array-of-structs, Go-slice logs. Every handler cites the main.go lines it
 * restates. The only additions are the ones the tick model needs and the
 * engine shares by definition:
 *   - a virtual clock (1 tick = cfg.tick_seconds, main.go:394) replacing
 *     time.Timer / time.Sleep;
 *   - a counter RNG keyed by (seed, group, replica, stream, tick) replacing
 *     math/rand (main.go:92, 114, 194);
 *   - fault codes where Go would panic (main.go:142 -> 404) or block forever
 *     (main.go:242, 265, 308), freezing the group;
 *   - EXT: ring-depth visibility (RAFT_F_RING_EVICTED), int32 range
 *     (RAFT_F_OVERFLOW), seeded isolation windows (dropped messages).
 */
#include "raft_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define I32MAX 2147483647LL

enum { ST_VALUE = 1, ST_TIMER_F = 2, ST_TIMER_C = 3, ST_ISOLATE = 4, ST_CORRUPT = 5 };

/* ---------------------------------------------------------------- RNG ---- */
static uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
uint64_t oracle_rng(uint64_t seed, uint64_t gid, uint32_t replica, uint32_t stream, uint64_t tick) {
  uint64_t k = sm64(seed ^ sm64(gid));
  uint64_t h = sm64(k ^ (((uint64_t)stream << 32) | replica));
  return sm64(h ^ tick);
}
/* rand.Int() (main.go:92): uniform in [0, 2^63). */
uint64_t oracle_client_value(uint64_t seed, uint64_t gid, uint32_t replica, uint64_t tick, uint32_t e) {
  return sm64(oracle_rng(seed, gid, replica, ST_VALUE, tick) ^ (uint64_t)e) >> 1;
}
/* rand.Intn(20)+10 (main.go:114) / rand.Intn(4)+10 (main.go:194). */
int32_t oracle_timer_draw(const raft_config* c, uint64_t gid, uint32_t replica, int role, uint64_t tick) {
  int cand = role == RAFT_CANDIDATE;
  uint64_t h = oracle_rng(c->seed, gid, replica, cand ? ST_TIMER_C : ST_TIMER_F, tick);
  uint32_t span = (uint32_t)(cand ? c->candidate_timeout_span : c->follower_timeout_span);
  int32_t mn = cand ? c->candidate_timeout_min : c->follower_timeout_min;
  return mn + (int32_t)((uint32_t)(h >> 32) % span);
}
/* EXT isolation windows: per 32-tick epoch e, with probability p/65536 one
 * replica is cut off for [start, start+len) ticks (len <= 32). Returns 1 if
 * epoch e has a window covering `tick`; *start and the hashed victim out. */
static int iso_window(const raft_config* c, uint64_t gid, int64_t e, int64_t tick, int64_t* start,
                      uint32_t* victim) {
  uint64_t h = oracle_rng(c->seed, gid, 0, ST_ISOLATE, (uint64_t)e);
  if ((h & 0xFFFF) >= c->isolate_per_65536) return 0;
  *victim = (uint32_t)((h >> 16) & 0xFF) % c->replicas;
  *start = e * 32 + (int64_t)((h >> 24) & 31);
  uint32_t span = c->isolate_max_ticks - c->isolate_min_ticks + 1;
  int64_t len = c->isolate_min_ticks + (int64_t)((uint32_t)(h >> 32) % span);
  return tick >= *start && tick < *start + len;
}
/* Hashed-victim mode (isolate_leader = 0): is `replica` cut off at `tick`? */
int oracle_isolated(const raft_config* c, uint64_t gid, uint32_t replica, int64_t tick) {
  if (c->isolate_per_65536 == 0 || tick < 0) return 0;
  int64_t ep = tick >> 5;
  for (int64_t e = ep; e >= ep - 1 && e >= 0; --e) {
    int64_t start;
    uint32_t victim;
    if (iso_window(c, gid, e, tick, &start, &victim) && victim == replica) return 1;
  }
  return 0;
}

/* EXT (config C5): CRC32C (Castagnoli, reflected poly 0x82F63B78, init and
 * final xor 0xFFFFFFFF) of an entry's 12 payload bytes: Term as 4 bytes
 * little-endian, then Value as 8 bytes little-endian. Bitwise reference
 * implementation; check value CRC32C("123456789") = 0xE3069283. */
uint32_t oracle_crc32c(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
  }
  return c ^ 0xFFFFFFFFu;
}
uint32_t oracle_entry_crc(int64_t term, int64_t value) {
  uint8_t b[12];
  uint32_t t = (uint32_t)term;
  uint64_t v = (uint64_t)value;
  for (int i = 0; i < 4; ++i) b[i] = (uint8_t)(t >> (8 * i));
  for (int i = 0; i < 8; ++i) b[4 + i] = (uint8_t)(v >> (8 * i));
  return oracle_crc32c(b, 12);
}
/* EXT: does the AppendEntries delivered to `replica` at `tick` arrive with its
 * last entry's Value bit 0 flipped? */
int oracle_corrupted(const raft_config* c, uint64_t gid, uint32_t replica, int64_t tick) {
  if (!c->payload_crc || !c->corrupt_per_65536) return 0;
  return (oracle_rng(c->seed, gid, replica, ST_CORRUPT, (uint64_t)tick) & 0xFFFF) < c->corrupt_per_65536;
}

/* ------------------------------------------------------------ state ---- */
typedef struct { int64_t term, value; uint32_t crc; } o_ent;   /* Log (main.go:46-49) + EXT crc */

typedef struct {                                 /* Node (main.go:14-39) */
  int role;                                      /* State */
  int voted;                                     /* Voted */
  int64_t term;                                  /* Term */
  int64_t last;                                  /* LastApplied == len(Log) */
  int64_t commit;                                /* CommitIndex */
  int64_t deadline, timeout;                     /* timer (virtual seconds) */
  int64_t match[RAFT_MAX_REPLICAS];              /* MatchIndex; REF: NextIndex = match+1 */
  int64_t next[RAFT_MAX_REPLICAS];               /* NextIndex (RAFT mode only; REF derives it) */
  int64_t hwm;                                   /* highest LastApplied ever (ring window; == last in REF) */
  o_ent* log;
  int64_t cap;
} o_node;

typedef struct {
  o_node n[RAFT_MAX_REPLICAS];
  int fault;
  uint8_t iso;   /* EXT leader-isolation mode: victim per epoch parity, nibble e&1 = 8|replica (0 = none) */
} o_group;

/* Replicas cut off at `tick` (bit r). Leader mode (isolate_leader): a
 * window's victim is the lowest-id Leader when the window's first tick
 * begins (decided then, with decide = 1, and recorded in G->iso); no leader
 * then, nobody. */
static uint32_t group_iso_mask(const raft_config* c, uint64_t gid, o_group* G, int64_t tick, int decide) {
  if (c->isolate_per_65536 == 0 || tick < 0) return 0;
  uint32_t mask = 0;
  int64_t ep = tick >> 5;
  for (int64_t e = ep; e >= ep - 1 && e >= 0; --e) {
    int64_t start;
    uint32_t victim;
    if (!iso_window(c, gid, e, tick, &start, &victim)) continue;
    if (!c->isolate_leader) { mask |= 1u << victim; continue; }
    int sh = 4 * (int)(e & 1);
    if (decide && tick == start) {
      int v = -1;
      for (uint32_t r = 0; r < c->replicas && v < 0; ++r)
        if (G->n[r].role == RAFT_LEADER) v = (int)r;
      G->iso = (uint8_t)((G->iso & ~(0xF << sh)) | ((v >= 0 ? 8 | v : 0) << sh));
    }
    int nib = (G->iso >> sh) & 0xF;
    if (nib & 8) mask |= 1u << (nib & 7);
  }
  return mask;
}

struct oracle {
  raft_config cfg;
  o_group* g;
  /* RAFT_CLIENT_STAGED: the caller's client values [cv_n][E][G] for ticks
   * [cv_t0, cv_t0 + cv_n) (oracle_stage_values; raftstep.h raft_stage_values) */
  int64_t* cv;
  int64_t cv_t0;
  uint32_t cv_n;
};

typedef struct {                                 /* one handler invocation's context */
  const raft_config* cfg;
  uint64_t gid;
  const int64_t* cv;                             /* staged values of this group and tick (entry e at cv[e*G]), or NULL */
  uint64_t cv_stride;
  int64_t tick, now;
  int64_t st[RAFT_NSTATS];
  uint32_t iso;                                  /* EXT: replicas cut off this tick (bit r) */
} o_ctx;

typedef struct {                                 /* AppendEntriesRequest (main.go:289-296) */
  int64_t term, prev_idx, prev_term, lc;
  const o_ent* ents;
  int64_t n;
  int corrupt;                                   /* EXT: last entry arrives with a flipped bit */
} o_ae;
typedef struct { int64_t term, match; int ok; } o_aer;  /* AppendEntriesResponse (main.go:298-302) */

static void set_fault(o_group* G, int f) {
  if (!G->fault) G->fault = f;
}

/* append(n.Log, ...) (main.go:148, 328): Go slices grow by doubling. */
static void log_append(o_node* n, const o_ent* src, int64_t cnt) {
  if (cnt <= 0) return;
  if (n->last + cnt > n->cap) {
    int64_t nc = n->cap ? n->cap : 8;
    while (nc < n->last + cnt) nc *= 2;
    n->log = (o_ent*)realloc(n->log, (size_t)nc * sizeof(o_ent));
    n->cap = nc;
  }
  memmove(n->log + n->last, src, (size_t)cnt * sizeof(o_ent));
  n->last += cnt;
  if (n->last > n->hwm) n->hwm = n->last;
}

/* GetLog(i) = Log[i-1] (main.go:403-405): panics outside [1, len]; the
 * EXT ring-depth rule makes entries at or below hwm-K unreadable (hwm is
 * the highest length the log ever had; == last without truncation). */
static int get_log_term(const o_ctx* c, o_group* G, const o_node* n, int64_t i, int64_t* out) {
  if (i < 1 || i > n->last) { set_fault(G, RAFT_F_PANIC_GETLOG); return 0; }
  if (i <= n->hwm - (int64_t)c->cfg->ring_depth) { set_fault(G, RAFT_F_RING_EVICTED); return 0; }
  *out = n->log[i - 1].term;
  return 1;
}

/* FollowerRun entry (main.go:111-115): draw d, start the timer. */
static void enter_follower(const o_ctx* c, o_node* n, int x) {
  n->role = RAFT_FOLLOWER;
  n->timeout = oracle_timer_draw(c->cfg, c->gid, (uint32_t)x, RAFT_FOLLOWER, (uint64_t)c->tick);
  n->deadline = c->now + n->timeout;
}
/* CandidateRun entry (main.go:193-195). */
static void enter_candidate(const o_ctx* c, o_node* n, int x) {
  n->role = RAFT_CANDIDATE;
  n->timeout = oracle_timer_draw(c->cfg, c->gid, (uint32_t)x, RAFT_CANDIDATE, (uint64_t)c->tick);
  n->deadline = c->now + n->timeout;
}

/* ------------------------------------------------ AppendEntries handlers */
/* FollowerRun case r := <-n.AEReq (main.go:121-156). */
static o_aer follower_ae(const o_ctx* c, o_group* G, int x, const o_ae* r) {
  o_node* n = &G->n[x];
  o_aer res = {n->term, n->last, 0};
  n->deadline = c->now + n->timeout;                     /* 124-127: timer.Reset(d) */
  if (r->term < n->term) return res;                     /* 129-133 */
  if (n->last > 0) {                                     /* 135 */
    if (n->last + r->n < r->prev_idx) return res;        /* 137-140 */
    int64_t t;
    if (!get_log_term(c, G, n, r->prev_idx, &t)) return res; /* 142: GetLog may panic */
    if (t != r->prev_term) return res;                   /* 142-145 */
  }
  if (n->last + r->n > I32MAX) { set_fault(G, RAFT_F_OVERFLOW); return res; }
  if (c->cfg->payload_crc) {                             /* EXT: verify what will be stored (last K) */
    int64_t j0 = r->n > (int64_t)c->cfg->ring_depth ? r->n - (int64_t)c->cfg->ring_depth : 0;
    for (int64_t j = j0; j < r->n; ++j) {
      int64_t v = r->ents[j].value ^ ((r->corrupt && j == r->n - 1) ? 1 : 0);
      if (oracle_entry_crc(r->ents[j].term, v) != r->ents[j].crc) return res;
    }
  }
  log_append(n, r->ents, r->n);                          /* 148-149 */
  if (r->lc > n->commit)                                 /* 151-152: min(LC, len(Log)+1) */
    n->commit = r->lc < n->last + 1 ? r->lc : n->last + 1;
  n->term = r->term;                                     /* 155 */
  res.term = n->term; res.match = n->last; res.ok = 1;   /* 156 */
  return res;
}
/* CandidateRun case r := <-n.AEReq (main.go:200-223). */
static o_aer candidate_ae(const o_ctx* c, o_group* G, int x, const o_ae* r) {
  o_node* n = &G->n[x];
  o_aer res = {n->term, n->last, 0};
  if (r->term >= n->term) {                              /* 204 */
    res.ok = 1;                                          /* 205-209: MatchIndex = LastApplied, nothing appended */
    n->voted = 1;                                        /* 211 */
    n->term = r->term;                                   /* 212 */
    enter_follower(c, n, x);                             /* 210, 213-216 -> Run -> FollowerRun */
  }
  return res;                                            /* 219-223 */
}
/* LeaderRun case r := <-n.AEReq (main.go:309-326). */
static o_aer leader_ae(const o_ctx* c, o_group* G, int x, const o_ae* r) {
  o_node* n = &G->n[x];
  o_aer res = {n->term, 0, 0};                           /* MatchIndex unset -> 0 */
  if (r->term > n->term) {                               /* 312 */
    res.ok = 1;                                          /* 313-316 */
    n->voted = 0;                                        /* 318 */
    n->term = r->term;                                   /* 319 */
    enter_follower(c, n, x);                             /* 317, 320 */
    memset(n->match, 0, sizeof n->match);
  }
  return res;
}
/* Run (main.go:98-109) dispatches the message to the receiver's role loop. */
static o_aer deliver_ae(const o_ctx* c, o_group* G, int x, const o_ae* r) {
  switch (G->n[x].role) {
    case RAFT_FOLLOWER: return follower_ae(c, G, x, r);
    case RAFT_CANDIDATE: return candidate_ae(c, G, x, r);
    default: return leader_ae(c, G, x, r);
  }
}

/* -------------------------------------------------- RequestVote handlers */
/* Returns 1 if granted; sets a fault where the requester would block. */
static int deliver_vr(const o_ctx* c, o_group* G, int x, int64_t rterm, int64_t* resp_term) {
  o_node* n = &G->n[x];
  *resp_term = n->term;
  switch (n->role) {
    case RAFT_FOLLOWER:                                  /* main.go:157-170 */
      if (rterm < n->term || n->voted) return 0;         /* 160-162 (no timer reset) */
      n->deadline = c->now + n->timeout;                 /* 164-167 */
      n->term = rterm;                                   /* 168 */
      n->voted = 1;                                      /* 169 */
      *resp_term = n->term;
      return 1;                                          /* 170 */
    case RAFT_CANDIDATE:                                 /* main.go:224-246 */
      if (rterm > n->term) {                             /* 227-238 */
        n->voted = 1;
        n->term = rterm;
        enter_follower(c, n, x);
        return 1;
      }
      /* 242: the rejection goes into the candidate's OWN VRes, the requester
       * blocks at main.go:265 forever; 243-246 reset this candidate's timer. */
      n->deadline = c->now + n->timeout;
      set_fault(G, RAFT_F_DEADLOCK_VRES);
      return 0;
    default:                                             /* LeaderRun has no VReq case (main.go:308) */
      set_fault(G, RAFT_F_DEADLOCK_LEADER_VREQ);
      return 0;
  }
}

/* ------------------------------------------------------- node steps ----- */
static int dropped(const o_ctx* c, int a, int b) { return (int)(((c->iso >> a) | (c->iso >> b)) & 1u); }

/* CandidateRun default branch (main.go:253-284). Returns 1 if elected. */
static int candidate_round(o_ctx* c, o_group* G, int cand) {
  const int R = (int)c->cfg->replicas;
  o_node* n = &G->n[cand];
  int count = 1;                                         /* 255 */
  n->voted = 1;                                          /* 256 */
  for (int p = 0; p < R; ++p) {                          /* 259-269 */
    if (p == cand) continue;
    if (dropped(c, cand, p)) continue;                   /* EXT */
    int64_t rt;
    int grant = deliver_vr(c, G, p, n->term, &rt);       /* 264-265 */
    if (G->fault) return 0;
    if (grant) { count++; c->st[RAFT_STAT_VOTES_GRANTED]++; } /* 266-268 */
  }
  if (2 * count > R) {                                   /* 273: float64(count) > float64(N)/2 */
    n->role = RAFT_LEADER;                               /* 274 */
    memset(n->match, 0, sizeof n->match);                /* 275-282: MatchIndex 0, NextIndex 1 */
    c->st[RAFT_STAT_ELECTIONS_WON]++;
    return 1;
  }
  return 0;
}

/* Commit rule (main.go:381-391): exact-value histogram of the peers'
 * MatchIndex, leader excluded, no current-term rule. */
static void leader_commit(o_ctx* c, o_group* G, int L) {
  const int R = (int)c->cfg->replicas;
  o_node* n = &G->n[L];
  for (int p = 0; p < R; ++p) {                          /* 386: at most one value can qualify */
    if (p == L) continue;
    int cnt = 0;
    for (int q = 0; q < R; ++q)                          /* 382-385 */
      if (q != L && n->match[q] == n->match[p]) cnt++;
    if (2 * cnt > R && n->match[p] > n->commit) {        /* 387 */
      c->st[RAFT_STAT_COMMITTED] += n->match[p] - n->commit;
      n->commit = n->match[p];                           /* 389 */
    }
  }
}

/* LeaderRun default branch (main.go:332-391). */
static void leader_round(o_ctx* c, o_group* G, int L) {
  const int R = (int)c->cfg->replicas;
  o_node* n = &G->n[L];
  for (int p = 0; p < R; ++p) {                          /* 334-379 */
    if (p == L) continue;
    if (dropped(c, L, p)) { c->st[RAFT_STAT_AE_FAIL]++; continue; }  /* EXT */
    o_ae r;
    r.term = n->term; r.lc = n->commit;
    r.corrupt = oracle_corrupted(c->cfg, c->gid, (uint32_t)p, c->tick);
    int64_t nxt = n->match[p] + 1;                       /* NextIndex == MatchIndex + 1 */
    if (nxt <= n->last) {                                /* 341 */
      if (nxt == 1) {                                    /* 343-351: whole log, PrevLogIndex 0 */
        r.ents = n->log; r.n = n->last;
        r.prev_term = n->term; r.prev_idx = 0;
      } else {                                           /* 353-360 */
        if (nxt < 1) { set_fault(G, RAFT_F_PANIC_GETLOG); return; }  /* GetLogsFrom(<1) panics */
        int64_t pt;
        if (!get_log_term(c, G, n, n->match[p], &pt)) return;       /* GetLog(MatchIndex) */
        r.ents = n->log + (nxt - 1); r.n = n->last - nxt + 1;
        r.prev_term = pt; r.prev_idx = n->match[p];
      }
    } else {                                             /* 364-371: heartbeat, PrevLogTerm = Term */
      r.ents = NULL; r.n = 0;
      r.prev_term = n->term; r.prev_idx = n->match[p];
    }
    o_aer res = deliver_ae(c, G, p, &r);                 /* 344/353/364 -> 373 */
    if (G->fault) return;
    if (res.ok) {                                        /* 375-378; response Term ignored */
      n->match[p] = res.match;
      c->st[RAFT_STAT_AE_OK]++;
    } else {
      c->st[RAFT_STAT_AE_FAIL]++;
    }
  }
  leader_commit(c, G, L);
}

/* timer.C fires (main.go:171-177 follower, 248-251 candidate). */
static void timeout_fire(o_ctx* c, o_group* G, int x) {
  o_node* n = &G->n[x];
  if (n->term >= I32MAX) { set_fault(G, RAFT_F_OVERFLOW); return; }
  n->term++;                                             /* 176 / 250 */
  c->st[RAFT_STAT_TERM_BUMPS]++;
  enter_candidate(c, n, x);                              /* 175 / 251 -> CandidateRun */
}

/* LeaderRun case LogReq (main.go:327-329). */
static void client_append(const o_ctx* c, o_group* G, int L, int64_t value) {
  o_node* n = &G->n[L];
  if (n->last >= I32MAX) { set_fault(G, RAFT_F_OVERFLOW); return; }
  o_ent e = {n->term, value, c->cfg->payload_crc ? oracle_entry_crc(n->term, value) : 0u};
  log_append(n, &e, 1);
}


/* ======================================================================
 * RAFT-paper semantics (EXT mode RAFT_SEM_RAFT; Ongaro & Ousterhout,
 * "In Search of an Understandable Consensus Algorithm", Figure 2) on the
 * same tick model, for churn workloads where the
 * reference's own semantics fault. Divergences from main.go, by line:
 * votedFor instead of the sticky bool (20, 160); up-to-date check (185-186,
 * 264); consistency check + truncate-on-conflict (135-149); nextIndex
 * backoff (376-377); majority order statistic with the current-term rule
 * (382-391); commit = min(LC, last new entry) (152); any higher term steps
 * down (265-268, 373-378). voted holds votedFor (-1 = none).
 * ==================================================================== */
static int64_t last_term_of(const o_node* n) { return n->last ? n->log[n->last - 1].term : 0; }

/* Figure 2, all servers: a higher term in any RPC -> adopt it, forget the
 * vote, and (if not already) become a follower. */
static void r_observe_term(const o_ctx* c, o_group* G, int x, int64_t t) {
  o_node* n = &G->n[x];
  if (t <= n->term) return;
  n->term = t;
  n->voted = -1;
  if (n->role != RAFT_FOLLOWER) {
    enter_follower(c, n, x);
    memset(n->match, 0, sizeof n->match);
    memset(n->next, 0, sizeof n->next);
  }
}

static int r_deliver_vr(const o_ctx* c, o_group* G, int x, int64_t term, int cand, int64_t llast,
                        int64_t llterm, int64_t* resp_term) {
  o_node* n = &G->n[x];
  r_observe_term(c, G, x, term);
  *resp_term = n->term;
  if (term < n->term) return 0;
  int64_t mt = last_term_of(n);
  int uptodate = llterm > mt || (llterm == mt && llast >= n->last);
  if ((n->voted < 0 || n->voted == cand) && uptodate) {
    n->voted = cand;
    n->deadline = c->now + n->timeout;     /* granting a vote resets the election timer */
    return 1;
  }
  return 0;
}

/* On failure res.match is the hint H: the leader retries from min(next-1, H+1).
 * H = last (log too short), min(prevLogIndex-1, commitIndex) (term conflict),
 * prevLogIndex (EXT payload CRC mismatch). */
static o_aer r_deliver_ae(const o_ctx* c, o_group* G, int x, const o_ae* r) {
  o_node* n = &G->n[x];
  r_observe_term(c, G, x, r->term);
  o_aer res = {n->term, n->last, 0};
  if (r->term < n->term) return res;
  if (n->role == RAFT_LEADER) return res;          /* same-term second leader: cannot happen (election safety) */
  if (n->role == RAFT_CANDIDATE) {                 /* a current leader exists: step down */
    enter_follower(c, n, x);
    memset(n->match, 0, sizeof n->match);
    memset(n->next, 0, sizeof n->next);
  }
  n->deadline = c->now + n->timeout;               /* AppendEntries from the current leader resets the timer */
  if (r->prev_idx > n->last) return res;           /* log too short: hint = last */
  if (r->prev_idx > 0) {
    int64_t t;
    if (!get_log_term(c, G, n, r->prev_idx, &t)) return res;
    /* conflict: hint = min(prevLogIndex-1, commitIndex) -- the committed prefix
       matches every later leader's log (Leader Completeness), so the leader
       can jump back there in one step instead of one entry per round */
    if (t != r->prev_term) { res.match = r->prev_idx - 1 < n->commit ? r->prev_idx - 1 : n->commit; return res; }
  }
  if (c->cfg->payload_crc) {                       /* EXT: verify what will be stored */
    int64_t j0 = r->n > (int64_t)c->cfg->ring_depth ? r->n - (int64_t)c->cfg->ring_depth : 0;
    for (int64_t j = j0; j < r->n; ++j) {
      int64_t v = r->ents[j].value ^ ((r->corrupt && j == r->n - 1) ? 1 : 0);
      if (oracle_entry_crc(r->ents[j].term, v) != r->ents[j].crc) { res.match = r->prev_idx; return res; }
    }
  }
  if (r->prev_idx + r->n > I32MAX) { set_fault(G, RAFT_F_OVERFLOW); return res; }
  /* skip entries already present, truncate at the first conflict, append the rest */
  int64_t j = 0;
  for (; j < r->n; ++j) {
    int64_t idx = r->prev_idx + 1 + j;
    if (idx > n->last) break;
    int64_t t;
    if (!get_log_term(c, G, n, idx, &t)) return res;
    if (t != r->ents[j].term) { n->last = idx - 1; break; }
  }
  log_append(n, r->ents + j, r->n - j);
  int64_t last_new = r->prev_idx + r->n;
  if (r->lc > n->commit) n->commit = r->lc < last_new ? r->lc : last_new;
  res.term = n->term; res.match = last_new; res.ok = 1;
  return res;
}

static int r_candidate_round(o_ctx* c, o_group* G, int cand) {
  const int R = (int)c->cfg->replicas;
  o_node* n = &G->n[cand];
  int count = 1;                                   /* its own vote (votedFor = self since the timeout) */
  for (int p = 0; p < R; ++p) {
    if (p == cand) continue;
    if (n->role != RAFT_CANDIDATE) return 0;
    if (dropped(c, cand, p)) continue;
    int64_t rt;
    int grant = r_deliver_vr(c, G, p, n->term, cand, n->last, last_term_of(n), &rt);
    if (G->fault) return 0;
    if (rt > n->term) { r_observe_term(c, G, cand, rt); return 0; }
    if (grant) { count++; c->st[RAFT_STAT_VOTES_GRANTED]++; }
  }
  if (n->role == RAFT_CANDIDATE && 2 * count > R) {
    n->role = RAFT_LEADER;
    for (int p = 0; p < R; ++p) { n->match[p] = 0; n->next[p] = n->last + 1; }
    c->st[RAFT_STAT_ELECTIONS_WON]++;
    return 1;
  }
  return 0;
}

/* commitIndex = the largest N replicated on a majority (leader included),
 * only if log[N].term == currentTerm. */
static void r_leader_commit(o_ctx* c, o_group* G, int L) {
  const int R = (int)c->cfg->replicas;
  o_node* n = &G->n[L];
  int64_t v[RAFT_MAX_REPLICAS];
  for (int p = 0; p < R; ++p) v[p] = p == L ? n->last : n->match[p];
  for (int i = 1; i < R; ++i)                      /* insertion sort, descending */
    for (int k = i; k > 0 && v[k] > v[k - 1]; --k) { int64_t t = v[k]; v[k] = v[k - 1]; v[k - 1] = t; }
  int64_t N = v[R / 2];
  if (N > n->commit) {
    int64_t t;
    if (!get_log_term(c, G, n, N, &t)) return;
    if (t == n->term) {
      c->st[RAFT_STAT_COMMITTED] += N - n->commit;
      n->commit = N;
    }
  }
}

static void r_leader_round(o_ctx* c, o_group* G, int L) {
  const int R = (int)c->cfg->replicas;
  o_node* n = &G->n[L];
  for (int p = 0; p < R; ++p) {
    if (p == L) continue;
    if (n->role != RAFT_LEADER) return;
    if (dropped(c, L, p)) { c->st[RAFT_STAT_AE_FAIL]++; continue; }
    o_ae r;
    r.term = n->term; r.lc = n->commit;
    r.corrupt = oracle_corrupted(c->cfg, c->gid, (uint32_t)p, c->tick);
    int64_t nxt = n->next[p];
    if (nxt < 1 || nxt > n->last + 1) { set_fault(G, RAFT_F_PANIC_GETLOG); return; }
    if (nxt <= n->hwm - (int64_t)c->cfg->ring_depth) { set_fault(G, RAFT_F_RING_EVICTED); return; }
    r.prev_idx = nxt - 1;
    r.prev_term = 0;
    if (r.prev_idx > 0 && !get_log_term(c, G, n, r.prev_idx, &r.prev_term)) return;
    r.ents = n->log + (nxt - 1);
    r.n = n->last - nxt + 1;
    o_aer res = r_deliver_ae(c, G, p, &r);
    if (G->fault) return;
    if (res.term > n->term) { r_observe_term(c, G, L, res.term); c->st[RAFT_STAT_AE_FAIL]++; return; }
    if (res.ok) {
      n->match[p] = res.match;
      n->next[p] = res.match + 1;
      c->st[RAFT_STAT_AE_OK]++;
    } else {
      int64_t nn = n->next[p] - 1 < res.match + 1 ? n->next[p] - 1 : res.match + 1;
      n->next[p] = nn < 1 ? 1 : nn;
      c->st[RAFT_STAT_AE_FAIL]++;
    }
  }
  r_leader_commit(c, G, L);
}

static void r_timeout_fire(o_ctx* c, o_group* G, int x) {
  o_node* n = &G->n[x];
  if (n->term >= I32MAX) { set_fault(G, RAFT_F_OVERFLOW); return; }
  n->term++;
  n->voted = x;                                    /* votes for itself */
  c->st[RAFT_STAT_TERM_BUMPS]++;
  enter_candidate(c, n, x);
  memset(n->match, 0, sizeof n->match);
  memset(n->next, 0, sizeof n->next);
}

static int is_raft(const o_ctx* c) { return c->cfg->semantics == RAFT_SEM_RAFT; }

/* One tick of one group. */
static void tick_group(o_ctx* c, o_group* G) {
  const int R = (int)c->cfg->replicas;
  if (G->fault) return;
  /* 0. EXT isolation of this tick (leader mode: a window starting now takes the current leader) */
  c->iso = group_iso_mask(c->cfg, c->gid, G, c->tick, 1);
  /* 1. client (main.go:87-93): every replica whose State is Leader */
  if (c->cfg->client_period && c->tick % c->cfg->client_period == 0) {
    for (int r = 0; r < R && !G->fault; ++r) {
      if (G->n[r].role != RAFT_LEADER) continue;
      for (uint32_t e = 0; e < c->cfg->entries_per_tick && !G->fault; ++e)
        /* rand.Int() (main.go:92), or the request the caller staged for the group
         * (RAFT_CLIENT_STAGED: the same value to every leader, main.go:90-93) */
        client_append(c, G, r, c->cv ? c->cv[(uint64_t)e * c->cv_stride]
                                     : (int64_t)oracle_client_value(c->cfg->seed, c->gid, (uint32_t)r, (uint64_t)c->tick, e));
    }
  }
  /* 2. rounds, ascending replica id */
  for (int r = 0; r < R && !G->fault; ++r) {
    if (G->n[r].role == RAFT_LEADER) { if (is_raft(c)) r_leader_round(c, G, r); else leader_round(c, G, r); }
    else if (G->n[r].role == RAFT_CANDIDATE) { if (is_raft(c)) r_candidate_round(c, G, r); else candidate_round(c, G, r); }
  }
  /* 3. expired timers in (deadline, id) order; a new candidate runs its
   *    vote round at once (CandidateRun's default branch). */
  for (int it = 0; it < R && !G->fault; ++it) {
    int best = -1;
    for (int r = 0; r < R; ++r) {
      const o_node* n = &G->n[r];
      if (n->role == RAFT_LEADER || n->deadline > c->now) continue;
      if (best < 0 || n->deadline < G->n[best].deadline) best = r;
    }
    if (best < 0) break;
    if (is_raft(c)) r_timeout_fire(c, G, best); else timeout_fire(c, G, best);
    if (G->fault) break;
    if (is_raft(c)) r_candidate_round(c, G, best); else candidate_round(c, G, best);
  }
  if (G->fault) { c->st[RAFT_STAT_FAULTS]++; return; }
  for (int r = 0; r < R; ++r)
    if (G->n[r].role == RAFT_LEADER) { c->st[RAFT_STAT_LEADER_GROUPS]++; break; }
}

/* ------------------------------------------------------------- API ----- */
oracle* oracle_create(const raft_config* cfg) {
  if (!cfg || cfg->replicas < 1 || cfg->replicas > RAFT_MAX_REPLICAS || cfg->semantics > RAFT_SEM_RAFT) return NULL;
  oracle* o = (oracle*)calloc(1, sizeof *o);
  o->cfg = *cfg;
  o->g = (o_group*)calloc(cfg->groups ? cfg->groups : 1, sizeof(o_group));
  return o;
}

static void free_logs(oracle* o) {
  for (uint64_t g = 0; g < o->cfg.groups; ++g)
    for (uint32_t r = 0; r < o->cfg.replicas; ++r) {
      free(o->g[g].n[r].log);
      o->g[g].n[r].log = NULL; o->g[g].n[r].cap = 0;
    }
}

void oracle_destroy(oracle* o) {
  if (!o) return;
  free_logs(o);
  free(o->g);
  free(o->cv);
  free(o);
}

static o_ctx make_ctx(const oracle* o, uint64_t g, int64_t tick) {
  o_ctx c;
  memset(&c, 0, sizeof c);
  c.cfg = &o->cfg;
  c.gid = o->cfg.group_base + g;
  if (o->cfg.client_source == RAFT_CLIENT_STAGED && o->cv && tick >= o->cv_t0 && tick < o->cv_t0 + (int64_t)o->cv_n) {
    c.cv = o->cv + ((uint64_t)(tick - o->cv_t0) * o->cfg.entries_per_tick) * o->cfg.groups + g;
    c.cv_stride = o->cfg.groups;
  }
  c.tick = tick;
  c.now = tick * o->cfg.tick_seconds;
  /* message-level handlers see the windows as they stand (no leader-mode decision) */
  c.iso = group_iso_mask(&o->cfg, c.gid, &((oracle*)o)->g[g], tick, 0);
  return c;
}

/* NewNode (main.go:59-76) + FollowerRun entry (main.go:113-115). */
void oracle_init_new_nodes(oracle* o, int64_t tick0) {
  free_logs(o);
  for (uint64_t g = 0; g < o->cfg.groups; ++g) {
    o_ctx c = make_ctx(o, g, tick0);
    memset(&o->g[g], 0, sizeof(o_group));
    for (uint32_t r = 0; r < o->cfg.replicas; ++r) {
      enter_follower(&c, &o->g[g].n[r], (int)r);
      o->g[g].n[r].voted = o->cfg.semantics == RAFT_SEM_RAFT ? -1 : 0;
    }
  }
}

uint32_t oracle_steady_leader(const raft_config* cfg, uint64_t gid, int32_t leader) {
  if (leader >= 0) return (uint32_t)leader % cfg->replicas;
  return (uint32_t)(sm64(cfg->seed ^ 0x1EADE5ULL ^ sm64(gid)) >> 33) % cfg->replicas;
}

/* KAT-1 generalised: the state right after the first election. */
void oracle_init_steady(oracle* o, int32_t leader, int64_t tick0) {
  free_logs(o);
  for (uint64_t g = 0; g < o->cfg.groups; ++g) {
    o_ctx c = make_ctx(o, g, tick0);
    o_group* G = &o->g[g];
    memset(G, 0, sizeof(o_group));
    uint32_t L = oracle_steady_leader(&o->cfg, c.gid, leader);
    for (uint32_t r = 0; r < o->cfg.replicas; ++r) {
      o_node* n = &G->n[r];
      n->term = 1;
      n->voted = o->cfg.semantics == RAFT_SEM_RAFT ? (int)L : 1;   /* RAFT: everyone voted for L */
      if (r == L) {
        enter_candidate(&c, n, (int)r);
        n->role = RAFT_LEADER;
        for (uint32_t p = 0; p < o->cfg.replicas; ++p) n->next[p] = 1;
      } else {
        enter_follower(&c, n, (int)r);
      }
    }
  }
}

int oracle_load_state(oracle* o, const raft_state_view* v) {
  const uint32_t R = o->cfg.replicas, K = o->cfg.ring_depth;
  free_logs(o);
  for (uint64_t g = 0; g < o->cfg.groups; ++g) {
    o_group* G = &o->g[g];
    memset(G, 0, sizeof(o_group));
    G->fault = v->fault[g];
    G->iso = v->iso_victim ? v->iso_victim[g] : 0;
    for (uint32_t r = 0; r < R; ++r) {
      uint64_t i = g * R + r;
      o_node* n = &G->n[r];
      n->role = v->role[i];
      n->voted = o->cfg.semantics == RAFT_SEM_RAFT ? (int)v->voted[i] - 1 : v->voted[i];
      n->term = v->term[i]; n->commit = v->commit[i];
      n->deadline = v->deadline[i]; n->timeout = v->timeout[i];
      for (uint32_t p = 0; p < R; ++p) {
        n->match[p] = v->match[i * R + p];
        /* RAFT: a zero (or absent) NextIndex derives match+1, as REF always does */
        int32_t nx = (o->cfg.semantics == RAFT_SEM_RAFT && v->next) ? v->next[i * R + p] : 0;
        n->next[p] = nx > 0 ? nx : n->match[p] + 1;
      }
      int64_t last = v->last[i];
      if (last < 0) return RAFT_EINVAL;
      /* hwm below last (e.g. an all-zero plane) means "= last"; REF never truncates so hwm == last */
      int64_t hwm = (o->cfg.semantics == RAFT_SEM_RAFT && v->hwm && v->hwm[i] > last) ? v->hwm[i] : last;
      if (last > 0 && last <= hwm - (int64_t)K) return RAFT_EINVAL;   /* last entry outside the ring window */
      n->last = 0;
      if (last > 0) {
        o_ent* tmp = (o_ent*)calloc((size_t)last, sizeof(o_ent));
        for (int64_t idx = hwm > K ? hwm - K + 1 : 1; idx <= last; ++idx) {
          uint64_t s = i * K + (uint64_t)((idx - 1) & (K - 1));
          tmp[idx - 1].term = v->log_term[s];
          tmp[idx - 1].value = v->log_value[s];
          tmp[idx - 1].crc = v->log_crc ? v->log_crc[s]
                           : (o->cfg.payload_crc ? oracle_entry_crc(v->log_term[s], v->log_value[s]) : 0u);
        }
        log_append(n, tmp, last);
        free(tmp);
      }
      n->hwm = hwm;
    }
  }
  return RAFT_OK;
}

void oracle_store_state(const oracle* o, raft_state_view* v) {
  const uint32_t R = o->cfg.replicas, K = o->cfg.ring_depth;
  for (uint64_t g = 0; g < o->cfg.groups; ++g) {
    const o_group* G = &o->g[g];
    if (v->fault) v->fault[g] = (uint8_t)G->fault;
    if (v->iso_victim) v->iso_victim[g] = G->iso;
    for (uint32_t r = 0; r < R; ++r) {
      uint64_t i = g * R + r;
      const o_node* n = &G->n[r];
      if (v->role) v->role[i] = (uint8_t)n->role;
      if (v->voted) v->voted[i] = (uint8_t)(o->cfg.semantics == RAFT_SEM_RAFT ? n->voted + 1 : n->voted);
      if (v->hwm) v->hwm[i] = (int32_t)n->hwm;
      if (v->term) v->term[i] = (int32_t)n->term;
      if (v->last) v->last[i] = (int32_t)n->last;
      if (v->commit) v->commit[i] = (int32_t)n->commit;
      if (v->deadline) v->deadline[i] = (int32_t)n->deadline;
      if (v->timeout) v->timeout[i] = (int32_t)n->timeout;
      if (v->match)
        for (uint32_t p = 0; p < R; ++p)
          v->match[i * R + p] = (n->role == RAFT_LEADER && p != r) ? (int32_t)n->match[p] : 0;
      if (v->next)
        for (uint32_t p = 0; p < R; ++p)
          v->next[i * R + p] = (n->role == RAFT_LEADER && p != r)
                                   ? (int32_t)(o->cfg.semantics == RAFT_SEM_RAFT ? n->next[p] : n->match[p] + 1)
                                   : 0;
      for (uint32_t s = 0; s < K; ++s) {
        if (v->log_term) v->log_term[i * K + s] = 0;
        if (v->log_value) v->log_value[i * K + s] = 0;
        if (v->log_crc) v->log_crc[i * K + s] = 0;
      }
      int64_t lo = n->hwm > K ? n->hwm - K + 1 : 1;
      for (int64_t idx = lo; idx <= n->last; ++idx) {
        uint64_t s = i * K + (uint64_t)((idx - 1) & (K - 1));
        if (v->log_term) v->log_term[s] = (int32_t)n->log[idx - 1].term;
        if (v->log_value) v->log_value[s] = n->log[idx - 1].value;
        if (v->log_crc) v->log_crc[s] = n->log[idx - 1].crc;
      }
    }
  }
}

typedef struct {
  oracle* o;
  uint64_t g0, g1;
  int64_t first;
  uint32_t nticks;
  int64_t st[RAFT_NSTATS];
} o_job;

static void* run_job(void* arg) {
  o_job* j = (o_job*)arg;
  for (uint64_t g = j->g0; g < j->g1; ++g) {
    for (uint32_t t = 0; t < j->nticks; ++t) {
      o_ctx c = make_ctx(j->o, g, j->first + (int64_t)t);
      tick_group(&c, &j->o->g[g]);
      for (int s = 0; s < RAFT_NSTATS; ++s) j->st[s] += c.st[s];
    }
  }
  return NULL;
}

int oracle_stage_values(oracle* o, int64_t first_tick, uint32_t nticks, const int64_t* values) {
  if (o->cfg.client_source != RAFT_CLIENT_STAGED || (nticks && !values)) return -22;
  const size_t n = (size_t)nticks * o->cfg.entries_per_tick * o->cfg.groups;
  free(o->cv);
  o->cv = n ? (int64_t*)malloc(n * sizeof(int64_t)) : NULL;
  if (n) memcpy(o->cv, values, n * sizeof(int64_t));
  o->cv_t0 = first_tick;
  o->cv_n = nticks;
  return 0;
}

void oracle_tick(oracle* o, int64_t first_tick, uint32_t nticks, int nthreads, raft_tick_stats* out) {
  if (o->cfg.client_source == RAFT_CLIENT_STAGED &&
      (nticks && (!o->cv || first_tick < o->cv_t0 || first_tick + (int64_t)nticks > o->cv_t0 + (int64_t)o->cv_n))) {
    fprintf(stderr, "oracle_tick: ticks [%lld, %lld) are not staged\n", (long long)first_tick,
            (long long)(first_tick + nticks));
    abort();   /* (test infrastructure: oracle.py checks the range first) */
  }
  if (nthreads < 1) nthreads = 1;
  if ((uint64_t)nthreads > o->cfg.groups) nthreads = o->cfg.groups ? (int)o->cfg.groups : 1;
  o_job* jobs = (o_job*)calloc((size_t)nthreads, sizeof(o_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int i = 0; i < nthreads; ++i) {
    jobs[i].o = o;
    jobs[i].g0 = o->cfg.groups * (uint64_t)i / (uint64_t)nthreads;
    jobs[i].g1 = o->cfg.groups * (uint64_t)(i + 1) / (uint64_t)nthreads;
    jobs[i].first = first_tick;
    jobs[i].nticks = nticks;
    if (nthreads > 1) pthread_create(&th[i], NULL, run_job, &jobs[i]);
  }
  if (nthreads == 1) run_job(&jobs[0]);
  else for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  if (out) {
    memset(out, 0, sizeof *out);
    for (int i = 0; i < nthreads; ++i)
      for (int s = 0; s < RAFT_NSTATS; ++s) out->v[s] += jobs[i].st[s];
  }
  free(jobs);
  free(th);
}

static int check_distinct(const oracle* o, const uint64_t* gs, size_t stride, size_t n) {
  unsigned char* seen = (unsigned char*)calloc(o->cfg.groups ? o->cfg.groups : 1, 1);
  int rc = RAFT_OK;
  for (size_t i = 0; i < n; ++i) {
    uint64_t g = *(const uint64_t*)((const char*)gs + i * stride);
    if (g >= o->cfg.groups || seen[g]) { rc = RAFT_EINVAL; break; }
    seen[g] = 1;
  }
  free(seen);
  return rc;
}

static int fits32(int64_t v) { return v >= -I32MAX - 1 && v <= I32MAX; }

int oracle_append_entries(oracle* o, int64_t now_tick, const raft_ae_req* reqs, size_t n,
                          const raft_log_entry* entries, raft_ae_resp* out) {
  int rc = check_distinct(o, &reqs[0].group, sizeof(raft_ae_req), n);
  if (rc) return rc;
  for (size_t i = 0; i < n; ++i) {
    const raft_ae_req* q = &reqs[i];
    if (q->to >= o->cfg.replicas || !fits32(q->term) || !fits32(q->prev_log_index) ||
        !fits32(q->prev_log_term) || !fits32(q->leader_commit))
      return RAFT_EINVAL;
    for (uint64_t k = 0; k < q->n_entries; ++k)
      if (!fits32(entries[q->entries_offset + k].term)) return RAFT_EINVAL;
  }
  for (size_t i = 0; i < n; ++i) {
    const raft_ae_req* q = &reqs[i];
    o_group* G = &o->g[q->group];
    o_ctx c = make_ctx(o, q->group, now_tick);
    raft_ae_resp* rs = &out[i];
    memset(rs, 0, sizeof *rs);
    if (G->fault) { rs->fault = G->fault; continue; }
    o_ent* ents = (o_ent*)calloc(q->n_entries ? q->n_entries : 1, sizeof(o_ent));
    for (uint64_t k = 0; k < q->n_entries; ++k) {   /* host payloads are stamped on ingest */
      const raft_log_entry* le = &entries[q->entries_offset + k];
      ents[k].term = le->term; ents[k].value = le->value;
      ents[k].crc = o->cfg.payload_crc ? oracle_entry_crc(le->term, le->value) : 0u;
    }
    o_ae r;
    r.term = q->term; r.prev_idx = q->prev_log_index; r.prev_term = q->prev_log_term;
    r.lc = q->leader_commit; r.n = (int64_t)q->n_entries;
    r.ents = ents;
    r.corrupt = 0;
    o_aer a = is_raft(&c) ? r_deliver_ae(&c, G, (int)q->to, &r) : deliver_ae(&c, G, (int)q->to, &r);
    free(ents);
    rs->term = a.term; rs->match_index = a.match; rs->success = G->fault ? 0 : a.ok;
    rs->fault = G->fault;
  }
  return RAFT_OK;
}

int oracle_request_vote(oracle* o, int64_t now_tick, const raft_vote_req* reqs, size_t n,
                        raft_vote_resp* out) {
  int rc = check_distinct(o, &reqs[0].group, sizeof(raft_vote_req), n);
  if (rc) return rc;
  for (size_t i = 0; i < n; ++i)
    if (reqs[i].to >= o->cfg.replicas || reqs[i].candidate_id >= o->cfg.replicas || !fits32(reqs[i].term) ||
        !fits32(reqs[i].last_log_index) || !fits32(reqs[i].last_log_term))
      return RAFT_EINVAL;
  for (size_t i = 0; i < n; ++i) {
    const raft_vote_req* q = &reqs[i];
    o_group* G = &o->g[q->group];
    o_ctx c = make_ctx(o, q->group, now_tick);
    raft_vote_resp* rs = &out[i];
    memset(rs, 0, sizeof *rs);
    if (G->fault) { rs->fault = G->fault; continue; }
    int64_t rt;
    int grant = is_raft(&c) ? r_deliver_vr(&c, G, (int)q->to, q->term, (int)q->candidate_id, q->last_log_index,
                                           q->last_log_term, &rt)
                            : deliver_vr(&c, G, (int)q->to, q->term, &rt);
    rs->term = rt; rs->vote_granted = grant; rs->fault = G->fault;
  }
  return RAFT_OK;
}

int oracle_group_ops(oracle* o, int64_t now_tick, const raft_group_op* ops, size_t n,
                     raft_op_result* out) {
  int rc = check_distinct(o, &ops[0].group, sizeof(raft_group_op), n);
  if (rc) return rc;
  for (size_t i = 0; i < n; ++i)
    if (ops[i].replica >= o->cfg.replicas || ops[i].kind < RAFT_OP_CLIENT_APPEND ||
        ops[i].kind > RAFT_OP_LEADER_COMMIT)
      return RAFT_EINVAL;
  for (size_t i = 0; i < n; ++i) {
    const raft_group_op* q = &ops[i];
    o_group* G = &o->g[q->group];
    o_ctx c = make_ctx(o, q->group, now_tick);
    raft_op_result* rs = &out[i];
    memset(rs, 0, sizeof *rs);
    int x = (int)q->replica;
    o_node* nd = &G->n[x];
    if (G->fault) { rs->fault = G->fault; continue; }
    switch (q->kind) {
      case RAFT_OP_CLIENT_APPEND:  /* arg = Value */
        if (nd->role != RAFT_LEADER) { rs->status = RAFT_EINVAL; break; }
        client_append(&c, G, x, q->arg);
        rs->value = nd->last;
        break;
      case RAFT_OP_LEADER_ROUND:
        if (nd->role != RAFT_LEADER) { rs->status = RAFT_EINVAL; break; }
        if (is_raft(&c)) r_leader_round(&c, G, x); else leader_round(&c, G, x);
        rs->value = nd->commit;
        break;
      case RAFT_OP_CANDIDATE_ROUND:
        if (nd->role != RAFT_CANDIDATE) { rs->status = RAFT_EINVAL; break; }
        rs->value = is_raft(&c) ? r_candidate_round(&c, G, x) : candidate_round(&c, G, x);
        break;
      case RAFT_OP_TIMEOUT:
        if (nd->role == RAFT_LEADER) { rs->status = RAFT_EINVAL; break; }
        if (is_raft(&c)) r_timeout_fire(&c, G, x); else timeout_fire(&c, G, x);
        rs->value = nd->term;
        break;
      case RAFT_OP_LEADER_COMMIT:
        if (nd->role != RAFT_LEADER) { rs->status = RAFT_EINVAL; break; }
        if (is_raft(&c)) r_leader_commit(&c, G, x); else leader_commit(&c, G, x);
        rs->value = nd->commit;
        break;
    }
    rs->fault = G->fault;
  }
  return RAFT_OK;
}

/* nodelog (main.go:399-401): "[Id:Term:CommitIndex:LastApplied][State]". */
int oracle_nodelog(const oracle* o, uint64_t group, char* buf, size_t cap) {
  static const char* names[] = {"follower", "candidate", "leader"};
  size_t off = 0;
  if (group >= o->cfg.groups) return RAFT_EINVAL;
  for (uint32_t r = 0; r < o->cfg.replicas; ++r) {
    const o_node* n = &o->g[group].n[r];
    int w = snprintf(buf + off, cap > off ? cap - off : 0, "[Server%u:%lld:%lld:%lld][%s]\n", r,
                     (long long)n->term, (long long)n->commit, (long long)n->last, names[n->role]);
    if (w < 0) return RAFT_EINVAL;
    off += (size_t)w;
  }
  return (int)off;
}

/* State digest (the engine's raft_state_digest, include/raftstep.h): per group
 * a splitmix64 chain over the canonical host view of raft_store_state, keyed
 * by the global group id; *total is the wrapping sum over groups (order- and
 * shard-independent). Words, per replica r in order: role | voted<<8 | r<<16;
 * term | last<<32; commit | deadline<<32; timeout | hwm<<32; for each peer p:
 * match | next<<32; for each live log index i (max(1, hwm-K+1)..last):
 * term | i<<32, value, crc; then the group's fault code, then (only when
 * nonzero) 0x1500 | the leader-isolation victim byte. */
static uint64_t dg_mix(uint64_t h, uint64_t w) { return sm64(h ^ w); }
static uint64_t lo32(int64_t v) { return (uint64_t)(uint32_t)(int32_t)v; }
void oracle_state_digest(const oracle* o, uint64_t* per_group, uint64_t* total) {
  const uint32_t R = o->cfg.replicas, K = o->cfg.ring_depth;
  const int raft = o->cfg.semantics == RAFT_SEM_RAFT;
  uint64_t sum = 0;
  for (uint64_t g = 0; g < o->cfg.groups; ++g) {
    const o_group* G = &o->g[g];
    uint64_t h = sm64(0x5241465444494721ULL ^ (o->cfg.group_base + g));
    for (uint32_t r = 0; r < R; ++r) {
      const o_node* n = &G->n[r];
      const uint64_t voted = (uint64_t)(raft ? n->voted + 1 : n->voted);
      h = dg_mix(h, (uint64_t)n->role | (voted << 8) | ((uint64_t)r << 16));
      h = dg_mix(h, lo32(n->term) | (lo32(n->last) << 32));
      h = dg_mix(h, lo32(n->commit) | (lo32(n->deadline) << 32));
      h = dg_mix(h, lo32(n->timeout) | (lo32(n->hwm) << 32));
      for (uint32_t p = 0; p < R; ++p) {
        const int lead = n->role == RAFT_LEADER && p != r;
        const int64_t m = lead ? n->match[p] : 0;
        const int64_t nx = lead ? (raft ? n->next[p] : n->match[p] + 1) : 0;
        h = dg_mix(h, lo32(m) | (lo32(nx) << 32));
      }
      for (int64_t idx = n->hwm > K ? n->hwm - K + 1 : 1; idx <= n->last; ++idx) {
        h = dg_mix(h, lo32(n->log[idx - 1].term) | (lo32(idx) << 32));
        h = dg_mix(h, (uint64_t)n->log[idx - 1].value);
        h = dg_mix(h, (uint64_t)n->log[idx - 1].crc);
      }
    }
    h = dg_mix(h, (uint64_t)G->fault);
    if (G->iso) h = dg_mix(h, 0x1500u | G->iso);   /* EXT leader-isolation victims (absent: digest unchanged) */
    if (per_group) per_group[g] = h;
    sum += h;
  }
  if (total) *total = sum;
}
