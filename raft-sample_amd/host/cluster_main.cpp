// raft_cluster — config 1 of BASELINE.json through the engine: main.go's
// 3-node in-process cluster (main.go:78-96) electing a leader and
// replicating N client entries, on the virtual clock.
//
//   --mode handlers : a host loop shaped like main.go's goroutines, calling
//                     the per-node handlers (raftnode.hpp -> C-ABI) in the
//                     engine's canonical tick order
//   --mode tick     : the fused raft_tick launch
// Both must end in the identical state (tests/test_gpu_cluster.py).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "raftnode.hpp"
#include "trace_rng.hpp"

using raft::Engine;
using raft::Node;
using raft::State;

static uint64_t digest(const Engine::Snapshot& s) {
  uint64_t h = 1469598103934665603ULL;
  auto mix = [&](const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ULL;
  };
  mix(s.role.data(), s.role.size()); mix(s.voted.data(), s.voted.size()); mix(s.fault.data(), s.fault.size());
  mix(s.term.data(), s.term.size() * 4); mix(s.last.data(), s.last.size() * 4);
  mix(s.commit.data(), s.commit.size() * 4); mix(s.deadline.data(), s.deadline.size() * 4);
  mix(s.timeout.data(), s.timeout.size() * 4); mix(s.match.data(), s.match.size() * 4);
  mix(s.log_term.data(), s.log_term.size() * 4); mix(s.log_value.data(), s.log_value.size() * 8);
  mix(s.log_crc.data(), s.log_crc.size() * 4);
  return h;
}

int main(int argc, char** argv) {
  std::string mode = "handlers";
  int64_t entries = 10000;
  bool log = false;
  raft_config cfg;
  raft_config_default(&cfg);
  cfg.replicas = 3;                 // main.go:81
  cfg.groups = 1;
  cfg.client_period = 1;
  cfg.ring_depth = 64;
  for (int i = 1; i < argc; ++i) {
    auto arg = [&](const char* k) { return std::strcmp(argv[i], k) == 0 && i + 1 < argc; };
    if (arg("--mode")) mode = argv[++i];
    else if (arg("--entries")) entries = std::atoll(argv[++i]);
    else if (arg("--seed")) cfg.seed = std::strtoull(argv[++i], nullptr, 0);
    else if (arg("--client-period")) cfg.client_period = uint32_t(std::atoi(argv[++i]));
    else if (arg("--device")) cfg.device = std::atoi(argv[++i]);
    else if (std::strcmp(argv[i], "--log") == 0) log = true;
    else { std::fprintf(stderr, "usage: raft_cluster [--mode handlers|tick] [--entries N] [--seed S] [--log]\n"); return 2; }
  }
  try {
    Engine eng(cfg);
    eng.NewNodes(0);                                 // NewNode x3 (main.go:81-85)
    std::vector<Node> nodes;
    for (uint32_t r = 0; r < cfg.replicas; ++r) nodes.emplace_back(eng, 0, r, "Server" + std::to_string(r));
    const int R = int(cfg.replicas);
    Engine::Snapshot prev = eng.Store();
    int64_t t = 0;
    const int64_t max_ticks = entries * std::max<int64_t>(1, cfg.client_period) + 100000;
    int64_t commit = 0;
    for (; t < max_ticks; ++t) {
      if (mode == "tick") {
        eng.Tick(t, 1);
      } else {
        const int64_t now = t * cfg.tick_seconds;
        // 1. client: every leader gets the tick's NewLogRequests (main.go:87-93)
        if (cfg.client_period && t % cfg.client_period == 0) {
          Engine::Snapshot s = eng.Store();
          for (int r = 0; r < R; ++r)
            if (State(s.role[r]) == State::Leader)
              for (uint32_t e = 0; e < cfg.entries_per_tick; ++e)
                nodes[r].OnNewLog(t, raft::NewLogRequest{raft::client_value(cfg.seed, 0, uint32_t(r), uint64_t(t), e)});
        }
        // 2. each node's role loop, ascending id (LeaderRun / CandidateRun default branches)
        for (int r = 0; r < R; ++r) {
          Engine::Snapshot s = eng.Store();
          if (s.fault[0]) break;
          if (State(s.role[r]) == State::Leader) nodes[r].LeaderRound(t);
          else if (State(s.role[r]) == State::Candidate) nodes[r].CandidateRound(t);
        }
        // 3. expired timers in (deadline, id) order, each candidate voting at once
        for (int it = 0; it < R; ++it) {
          Engine::Snapshot s = eng.Store();
          if (s.fault[0]) break;
          int best = -1;
          for (int r = 0; r < R; ++r)
            if (State(s.role[r]) != State::Leader && s.deadline[r] <= now &&
                (best < 0 || s.deadline[r] < s.deadline[best]))
              best = r;
          if (best < 0) break;
          nodes[best].OnTimeout(t);
          if (eng.Store().fault[0]) break;
          nodes[best].CandidateRound(t);
        }
      }
      Engine::Snapshot s = eng.Store();
      if (log)
        for (int r = 0; r < R; ++r)
          if (s.role[r] != prev.role[r] || s.term[r] != prev.term[r])
            std::printf("%s\n", nodes[r].nodelog(s, s.role[r] == prev.role[r] ? "term change" :
                                                 std::string("I am ") + raft::to_string(State(s.role[r]))).c_str());
      commit = *std::max_element(s.commit.begin(), s.commit.end());
      prev = s;
      if (s.fault[0] || commit >= entries) { ++t; break; }
    }
    const Engine::Snapshot s = eng.Store();
    int leader = -1;
    for (int r = 0; r < R; ++r) if (State(s.role[r]) == State::Leader) leader = r;
    std::printf("{\"mode\": \"%s\", \"ticks\": %lld, \"leader\": \"%s\", \"term\": %d, \"commit\": [%d, %d, %d], "
                "\"last\": [%d, %d, %d], \"fault\": %d, \"digest\": \"%016llx\"}\n",
                mode.c_str(), (long long)t, leader >= 0 ? nodes[leader].Id.c_str() : "none", s.term[0],
                s.commit[0], s.commit[1 % R], s.commit[2 % R], s.last[0], s.last[1 % R], s.last[2 % R],
                int(s.fault[0]), (unsigned long long)digest(s));
    return (s.fault[0] == 0 && commit >= entries) ? 0 : 1;
  } catch (const raft::Error& e) {
    std::fprintf(stderr, "raft_cluster: %s\n", e.what());
    return 3;
  }
}
