// Exercises the header-only C++ client against live servers:
//   client_test <classifier_port> <stat_port>
// Every generated header is included so all of them are compile-checked.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "jubatus_amd/anomaly_client.hpp"
#include "jubatus_amd/bandit_client.hpp"
#include "jubatus_amd/burst_client.hpp"
#include "jubatus_amd/classifier_client.hpp"
#include "jubatus_amd/clustering_client.hpp"
#include "jubatus_amd/graph_client.hpp"
#include "jubatus_amd/nearest_neighbor_client.hpp"
#include "jubatus_amd/recommender_client.hpp"
#include "jubatus_amd/regression_client.hpp"
#include "jubatus_amd/stat_client.hpp"
#include "jubatus_amd/weight_client.hpp"

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  namespace jc = jubatus_amd::classifier;
  jc::client::classifier c("127.0.0.1", std::atoi(argv[1]), "", 10.0);
  std::vector<jc::labeled_datum> data;
  for (int i = 0; i < 20; ++i) {
    jc::labeled_datum ld;
    ld.label = i % 2 ? "pos" : "neg";
    ld.data.add_number("x", i % 2 ? 1.0 + 0.1 * i : -1.0 - 0.1 * i).add_string("t", ld.label + "w");
    data.push_back(ld);
  }
  CHECK(c.train(data) == 20);
  jubatus_amd::datum q;
  q.add_number("x", 2.0).add_string("t", "posw");
  auto res = c.classify({q});
  CHECK(res.size() == 1 && res[0].size() == 2);
  const auto& best = res[0][0].score > res[0][1].score ? res[0][0] : res[0][1];
  CHECK(best.label == "pos");
  auto labels = c.get_labels();
  CHECK(labels["pos"] == 10 && labels["neg"] == 10);
  CHECK(!c.get_config().empty());
  auto st = c.get_status();
  CHECK(st.size() == 1 && st.begin()->second.at("type") == "classifier");
  CHECK(c.save("cpp").size() == 1);
  CHECK(c.clear());
  CHECK(c.get_labels().empty());
  CHECK(c.load("cpp"));
  CHECK(c.get_labels().size() == 2);
  bool threw = false;
  try {
    c.get_client().call("no_such_method", std::string(""));
  } catch (const jubatus_amd::rpc_no_method&) {
    threw = true;
  }
  CHECK(threw);

  jubatus_amd::stat::client::stat s("127.0.0.1", std::atoi(argv[2]), "", 10.0);
  for (double v : {1.0, 2.0, 6.0}) CHECK(s.push("k", v));
  CHECK(std::fabs(s.sum("k") - 9.0) < 1e-9);
  CHECK(std::fabs(s.max("k") - 6.0) < 1e-9 && std::fabs(s.min("k") - 1.0) < 1e-9);
  threw = false;
  try {
    s.sum("missing");
  } catch (const jubatus_amd::rpc_call_error& e) {
    threw = std::string(e.what()).find("missing") != std::string::npos;
  }
  CHECK(threw);
  std::cout << "cpp client ok" << std::endl;
  return 0;
}
