"""jubatus_amd - an MI355X-native distributed online machine-learning framework
with the capabilities and wire protocol of Jubatus 0.9.2.

Layers (see SURVEY.md and docs/ARCHITECTURE.md):
  utils/       L0  logger, signals, argv, system status, crc32
  common/      L1-L2 msgpack-RPC (native core), coordinator (lock_service), membership, CHT
  parallel/    L3  MIX: linear_mixer (RCCL all-reduce), push mixers (send/recv), dummy
  framework/   L4  server_base/helper, model file save/load, proxy, aggregators
  server/      L5  the 11 engine servers (juba<engine>) and their proxies
  models/      engine drivers (GPU kernels + host oracles)
  fv_converter/ datum -> feature vector (GPU fast path + host path, plugins)
  ops/         HIP kernel bindings (csrc/hip) and the host->HBM feature pipeline
  client/      msgpack-RPC client library
  cmd/         jubactl, jubaconfig, jubaconv, jubavisor
"""

__version__ = "0.9.2"
JUBATUS_VERSION = (0, 9, 2)
