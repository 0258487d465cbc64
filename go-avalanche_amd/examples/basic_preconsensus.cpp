// basic_preconsensus — go-avalanche's examples/basic-preconcensus/main.go
// (100 nodes x 100 txs, every node IsAccepted()=true, round-robin polling
// skipping self, main.go:110-116) re-expressed on the batched MI355X engine.
//
// Each node polls one peer per round (k = 1, AV_PEERS_ROUND_ROBIN reproduces
// the example's `i % N, skip self` peer sequence); the round is synchronous
//  instead of goroutine-interleaved. By default a finalized
// record publishes its decision (R2); -literal runs the example's own
// semantics: the responder re-adds a queried target it does not hold as
// accepted (main.go:175-177, engine option "responder" 2), and a node stops
// polling once it counted txCount Finalized updates (main.go:143-162,
// av_set_polling) while still answering. Prints the example's log lines and
// final count.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "avalanche.hpp"

using namespace avalanche::gpu;

namespace {

struct Tx : Target {  // main.go:196-209
  explicit Tx(Hash h) : h(h) {}
  Hash GetHash() const override { return h; }
  std::string Type() const override { return "tx"; }
  bool IsAccepted() const override { return true; }
  int64_t Score() const override { return 1; }
  bool IsValid() const override { return true; }
  Hash h;
};

}  // namespace

int main(int argc, char** argv) {
  bool logging = false;  // main.go:24 -logging
  bool literal = false;
  int64_t node_count = 100, tx_count = 100;  // main.go:13-16
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "-logging")) logging = true;
    if (!std::strcmp(argv[i], "-literal")) literal = true;
    if (!std::strcmp(argv[i], "-nodes") && i + 1 < argc) node_count = std::atoll(argv[++i]);
    if (!std::strcmp(argv[i], "-txs") && i + 1 < argc) tx_count = std::atoll(argv[++i]);
  }
  EngineOptions opt;
  opt.n_nodes = node_count;
  opt.n_targets = tx_count;
  opt.k = 1;
  opt.peer_mode = AV_PEERS_ROUND_ROBIN;
  auto engine = std::make_shared<Engine>(opt);

  std::vector<std::unique_ptr<Tx>> txs;
  for (int64_t t = 0; t < tx_count; ++t) txs.push_back(std::make_unique<Tx>(t));
  const auto t0 = std::chrono::steady_clock::now();
  for (int64_t n = 0; n < node_count; ++n) {  // every node ingests every tx (main.go:49-54, 99-106)
    Processor p(engine, n);
    for (auto& tx : txs) p.AddTargetToReconcile(*tx);
  }

  if (literal && av_set_option(engine->handle(), "responder", 2) != AV_OK) {
    std::fprintf(stderr, "responder option: %s\n", av_last_error());
    return 2;
  }
  std::vector<int64_t> finalized(node_count, 0);
  int64_t nodes_fully_finalized = 0, round = 0;
  while (nodes_fully_finalized < node_count && round < 100000) {
    engine->RunRounds(1);
    ++round;
    for (uint64_t u : engine->FetchUpdates()) {
      const int64_t node = av_update_node(u);
      const int32_t st = av_update_status(u);
      const char* what = st == AV_STATUS_FINALIZED ? "Finalized"
                         : st == AV_STATUS_ACCEPTED ? "Accepted"
                         : st == AV_STATUS_REJECTED ? "Rejected" : "Invalidated";
      if (logging)
        std::printf("%s tx %lld on node %lld after %lld queries\n", what, (long long)av_update_target(u),
                    (long long)node, (long long)round);
      if (st == AV_STATUS_FINALIZED && ++finalized[node] == tx_count) {
        ++nodes_fully_finalized;  // main.go:159-162: the node's run loop returns
        if (literal) av_set_polling(engine->handle(), node, 0);
      }
    }
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("Finished in %fs\n", secs);  // main.go:63
  std::printf("Nodes fully finalized: %lld\n", (long long)nodes_fully_finalized);  // main.go:64
  return nodes_fully_finalized == node_count ? 0 : 1;
}
