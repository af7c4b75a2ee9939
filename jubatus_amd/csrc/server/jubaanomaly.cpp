// jubaanomaly, native: the LOF / light_lof anomaly server without Python
// (csrc/server/jb_row_server.hpp over jb_row_engine.hpp and the HBM LOF
// state of jb_lof_state.hpp; reference jubatus/server/server/
// anomaly_serv.cpp:149-320, anomaly_impl.cpp).
#include "jb_row_server.hpp"

int main(int argc, char** argv) {
  return jb::rowsrv::row_main(argc, argv, jb::rowsrv::Kind::kAnomaly);
}
