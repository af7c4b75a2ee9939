// jubarecommender, native: the recommender server without Python
// (csrc/server/jb_row_server.hpp over jb_row_engine.hpp; reference
// jubatus/server/server/recommender_serv.cpp:126-224, recommender_impl.cpp).
#include "jb_row_server.hpp"

int main(int argc, char** argv) {
  return jb::rowsrv::row_main(argc, argv, jb::rowsrv::Kind::kRecommender);
}
