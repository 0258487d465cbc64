// avalanche_gpu_tests.cpp — the reference's Processor tests
// (avalanche_test.go) restated against the C++ mirror on the MI355X engine.
// Run by tests/test_cpp_mirror.py (-m gpu). Exit code = number of failures.
#include <cstdio>
#include <functional>
#include <tuple>
#include <memory>
#include <string>
#include <vector>

#include "avalanche.hpp"

using namespace avalanche::gpu;

namespace {

int g_failures = 0;
std::string g_test;

#define EXPECT(cond)                                                                   \
  do {                                                                                 \
    if (!(cond)) {                                                                     \
      std::fprintf(stderr, "%s:%d [%s] expectation failed: %s\n", __FILE__, __LINE__, \
                   g_test.c_str(), #cond);                                             \
      ++g_failures;                                                                    \
      return;                                                                          \
    }                                                                                  \
  } while (0)

// avalanche.go:110-160 Block stub (hash, work, valid, isInActiveChain)
class Block : public Target {
 public:
  Block(Hash h, int64_t work, bool valid, bool in_chain) : h_(h), work_(work), valid_(valid), chain_(in_chain) {}
  Hash GetHash() const override { return h_; }
  std::string Type() const override { return "block"; }
  bool IsAccepted() const override { return chain_; }
  int64_t Score() const override { return work_; }
  bool IsValid() const override { return valid_; }
  void SetValid(bool v) { valid_ = v; }
  void SetInActiveChain(bool v) { chain_ = v; }

 private:
  Hash h_;
  int64_t work_;
  bool valid_, chain_;
};

constexpr uint32_t kNeutral = 0xFFFFFFFFu;  // uint32(-1), avalanche_test.go:8-11

std::shared_ptr<Engine> small_engine(int64_t nodes = 2, int64_t targets = 64) {
  EngineOptions o;
  o.n_nodes = nodes;
  o.n_targets = targets;
  o.k = 1;
  return std::make_shared<Engine>(o);
}

size_t poll_count(const Processor& p) { return p.GetInvsForNextPoll().size(); }

bool poll_has(const Processor& p, const Block& b) {
  for (const auto& inv : p.GetInvsForNextPoll())
    if (inv.target_hash == b.GetHash()) return inv.target_type == "block";
  return false;
}

// TestBlockRegister (avalanche_test.go:93-252)
void block_register() {
  Connman connman;
  auto engine = small_engine();
  Processor p(engine, 0, &connman);
  Block block(65, 99, true, true);
  connman.AddNode(0);
  std::vector<StatusUpdate> updates;
  const Response yes(0, 0, {NewVote(0, 65)}), no(0, 0, {NewVote(1, 65)}), neutral(0, 0, {NewVote(kNeutral, 65)});

  EXPECT(!p.IsAccepted(block));
  EXPECT(p.AddTargetToReconcile(block));
  EXPECT(poll_count(p) == 1 && poll_has(p, block));
  EXPECT(p.IsAccepted(block));
  for (int i = 0; i < 6; ++i) {  // not conclusive before 7 considered votes
    EXPECT(p.RegisterVotes(0, yes, &updates));
    EXPECT(p.IsAccepted(block) && p.GetConfidence(block) == 0 && updates.empty());
  }
  EXPECT(p.RegisterVotes(0, neutral, &updates));
  EXPECT(p.IsAccepted(block) && p.GetConfidence(block) == 0 && updates.empty());
  for (uint16_t c = 1; c < 7; ++c) {
    EXPECT(p.RegisterVotes(0, yes, &updates));
    EXPECT(p.GetConfidence(block) == c && updates.empty());
  }
  for (int i = 0; i < 2; ++i) {  // two neutral votes stall progress
    EXPECT(p.RegisterVotes(0, neutral, &updates));
    EXPECT(p.GetConfidence(block) == 6 && updates.empty());
  }
  for (int i = 2; i < 8; ++i) {
    EXPECT(p.RegisterVotes(0, yes, &updates));
    EXPECT(p.GetConfidence(block) == 6 && updates.empty());
  }
  for (uint16_t c = 7; c < kFinalizationScore; ++c) {
    EXPECT(p.RegisterVotes(0, yes, &updates));
    EXPECT(p.IsAccepted(block) && p.GetConfidence(block) == c && updates.empty());
  }
  EXPECT(poll_count(p) == 1 && poll_has(p, block));
  EXPECT(p.RegisterVotes(0, yes, &updates));
  EXPECT(updates.size() == 1 && updates[0] == (StatusUpdate{65, Status::Finalized}));
  updates.clear();
  EXPECT(poll_count(p) == 0);
  bool threw = false;
  try {
    p.GetConfidence(block);
  } catch (const VoteRecordNotFound&) {
    threw = true;  // the reference panics here (processor.go:136)
  }
  EXPECT(threw);

  EXPECT(p.AddTargetToReconcile(block));  // re-add after deletion, then finalize rejection
  EXPECT(poll_count(p) == 1);
  for (int i = 0; i < 6; ++i) {
    EXPECT(p.RegisterVotes(0, no, &updates));
    EXPECT(p.IsAccepted(block) && updates.empty());
  }
  EXPECT(p.RegisterVotes(0, no, &updates));
  EXPECT(!p.IsAccepted(block));
  EXPECT(updates.size() == 1 && updates[0] == (StatusUpdate{65, Status::Rejected}));
  updates.clear();
  for (int i = 1; i < kFinalizationScore; ++i) {
    EXPECT(p.RegisterVotes(0, no, &updates));
    EXPECT(!p.IsAccepted(block) && updates.empty());
  }
  EXPECT(poll_count(p) == 1 && poll_has(p, block));
  EXPECT(p.RegisterVotes(0, yes, &updates));
  EXPECT(!p.IsAccepted(block));
  EXPECT(updates.size() == 1 && updates[0] == (StatusUpdate{65, Status::Invalid}));
  updates.clear();
  EXPECT(poll_count(p) == 0);
  EXPECT(p.AddTargetToReconcile(block));
  EXPECT(!p.AddTargetToReconcile(block));
  EXPECT(p.IsAccepted(block));
}

// TestMultiBlockRegister (avalanche_test.go:254-363, without the flaky
// map-order assertion at :307-313)
void multi_block_register() {
  Connman connman;
  auto engine = small_engine();
  Processor p(engine, 0, &connman);
  Block a(65, 99, true, true), b(66, 100, true, false);
  connman.AddNode(0);
  connman.AddNode(1);
  b.SetInActiveChain(true);  // :281
  std::vector<StatusUpdate> updates;
  const Response yes_a(0, 0, {NewVote(0, 65)}), yes_b(1, 0, {NewVote(0, 66)}),
      yes_both(1, 0, {NewVote(0, 66), NewVote(0, 65)});

  EXPECT(!p.IsAccepted(a) && !p.IsAccepted(b));
  EXPECT(p.AddTargetToReconcile(a));
  EXPECT(poll_count(p) == 1 && poll_has(p, a));
  EXPECT(p.RegisterVotes(0, yes_a, &updates) && updates.empty());
  EXPECT(p.AddTargetToReconcile(b));
  EXPECT(poll_count(p) == 2);
  for (int i = 0; i < 4 + kFinalizationScore; ++i) {
    EXPECT(p.RegisterVotes(0, yes_both, &updates));
    EXPECT(updates.empty());
  }
  EXPECT(p.RegisterVotes(0, yes_both, &updates));  // A's 134th vote
  EXPECT(updates.size() == 1 && updates[0] == (StatusUpdate{65, Status::Finalized}));
  updates.clear();
  EXPECT(poll_count(p) == 1 && poll_has(p, b));
  EXPECT(p.RegisterVotes(0, yes_b, &updates));  // B's 134th vote
  EXPECT(updates.size() == 1 && updates[0] == (StatusUpdate{66, Status::Finalized}));
  EXPECT(poll_count(p) == 0);
}

// From TestPollAndResponse (avalanche_test.go:442-443, 533-539): the lowest
// connected node is the one to query; an invalid target is no longer polled
// and its votes are ignored.
void suitable_node_and_invalid_target() {
  Connman connman;
  auto engine = small_engine();
  Processor p(engine, 0, &connman);
  EXPECT(p.getSuitableNodeToQuery() == NoNode);
  connman.AddNode(7);
  connman.AddNode(3);
  EXPECT(p.getSuitableNodeToQuery() == 3);
  Block a(65, 99, true, true), b(66, 100, true, false);
  EXPECT(p.AddTargetToReconcile(a) && p.AddTargetToReconcile(b));
  std::vector<StatusUpdate> updates;
  const Response both(0, 0, {NewVote(0, 66), NewVote(0, 65)});
  EXPECT(p.RegisterVotes(3, both, &updates) && updates.empty());
  b.SetValid(false);
  EXPECT(poll_count(p) == 1 && poll_has(p, a));
  for (int i = 0; i < 10; ++i) EXPECT(p.RegisterVotes(3, both, &updates));
  EXPECT(p.GetConfidence(b) == 0);   // skipped while invalid (processor.go:101-103)
  EXPECT(p.GetConfidence(a) == 5);   // 11 yes votes: count 11 - 6
  EXPECT(updates.empty());
  Block c(67, 1, false, true);
  EXPECT(!p.AddTargetToReconcile(c));  // not worth polling (processor.go:46-48)
}

// The example's network (examples/basic-preconcensus): every node tracks
// every tx as accepted; batched rounds finalize every record exactly once.
void network_rounds() {
  EngineOptions o;
  o.n_nodes = 100;
  o.n_targets = 100;
  o.k = 8;
  auto engine = std::make_shared<Engine>(o);
  struct Tx : Target {
    explicit Tx(Hash h) : h(h) {}
    Hash GetHash() const override { return h; }
    std::string Type() const override { return "tx"; }
    bool IsAccepted() const override { return true; }
    int64_t Score() const override { return 1; }
    bool IsValid() const override { return true; }
    Hash h;
  };
  std::vector<std::unique_ptr<Tx>> txs;
  for (int t = 0; t < 100; ++t) txs.push_back(std::make_unique<Tx>(1000 + t));
  for (NodeID n = 0; n < 100; ++n) {
    Processor p(engine, n);
    for (auto& tx : txs) EXPECT(p.AddTargetToReconcile(*tx));
  }
  engine->RunRounds(20);
  auto ups = engine->FetchUpdates();
  EXPECT(ups.size() == 100u * 100u);
  for (uint64_t u : ups) EXPECT(av_update_status(u) == AV_STATUS_FINALIZED);
  Processor p0(engine, 0);
  EXPECT(p0.GetInvsForNextPoll().empty());
  // GetRound is the Processor's own field (processor.go:40-42), not the
  // engine's batched-round counter: rounds leave it alone, its owner sets it
  EXPECT(p0.GetRound() == 0);
  p0.SetRound(p0.GetRound() + 1);  // avalanche_test.go:302 `p.round++`
  EXPECT(p0.GetRound() == 1);
  EXPECT(Processor(engine, 1).GetRound() == 0);
  EXPECT(engine->Round() == 20);
}

// Pipelined delivery through the mirror (Engine::Rounds over the compact stream) hands every node
// exactly the StatusUpdates a plain round + FetchUpdates gives, in the same order.
void pipelined_rounds() {
  EngineOptions o;
  o.n_nodes = 3000;
  o.n_targets = 700;
  o.k = 8;
  o.byz_threshold = (uint32_t)(0.2 * 4294967296.0);
  auto a = std::make_shared<Engine>(o), b = std::make_shared<Engine>(o);
  EXPECT(av_init_records(a->handle(), AV_INIT_PAIRS, 0) == AV_OK);
  EXPECT(av_init_records(b->handle(), AV_INIT_PAIRS, 0) == AV_OK);
  std::vector<std::tuple<int64_t, NodeID, Hash, int>> got, want;
  b->Rounds(6, [&](int64_t r, NodeID n, const std::vector<StatusUpdate>& ups) {
    for (const auto& u : ups) got.emplace_back(r, n, u.hash, (int)u.status);
  });
  for (int r = 0; r < 6; ++r) {
    a->RunRounds(1);
    for (uint64_t u : a->FetchUpdates())
      want.emplace_back(r, (NodeID)av_update_node(u), (Hash)av_update_target(u), av_update_status(u));
  }
  EXPECT(!want.empty());
  EXPECT(got == want);
}

}  // namespace

int main() {
  const std::vector<std::pair<const char*, std::function<void()>>> tests = {
      {"TestBlockRegister", block_register},
      {"TestMultiBlockRegister", multi_block_register},
      {"SuitableNodeAndInvalidTarget", suitable_node_and_invalid_target},
      {"NetworkRounds", network_rounds},
      {"PipelinedRounds", pipelined_rounds},
  };
  for (const auto& t : tests) {
    g_test = t.first;
    const int before = g_failures;
    try {
      t.second();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "[%s] exception: %s\n", t.first, e.what());
      ++g_failures;
    }
    std::printf("%s %s\n", g_failures == before ? "PASS" : "FAIL", t.first);
  }
  return g_failures;
}
