// jubanearest_neighbor, native: the nearest_neighbor server without Python
// (csrc/server/jb_row_server.hpp over jb_row_engine.hpp; reference
// jubatus/server/server/nearest_neighbor_serv.cpp:121-178,
// nearest_neighbor_impl.cpp).
#include "jb_row_server.hpp"

int main(int argc, char** argv) {
  return jb::rowsrv::row_main(argc, argv, jb::rowsrv::Kind::kNearestNeighbor);
}
