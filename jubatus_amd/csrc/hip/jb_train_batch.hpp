// Argument block of jb_train_batch_submit (csrc/hip/train_batch.hip): one
// GPU-scan train batch. Shared by the HIP library, the ctypes mirror
// (ops/hip.py TrainBatchArgs) and the native server (csrc/server).
#ifndef JUBATUS_AMD_CSRC_HIP_JB_TRAIN_BATCH_HPP_
#define JUBATUS_AMD_CSRC_HIP_JB_TRAIN_BATCH_HPP_
#include <hip/hip_runtime_api.h>
#include <stdint.h>

// Every field is 8 bytes (ops/hip.py TrainBatchArgs mirrors the order).
struct JbTrainBatch {
  // streams; events recorded by the call (hot_free / hot_seen may be null)
  hipStream_t copy_stream, prep_stream, compute_stream;
  hipEvent_t copy_done;   // copy stream, after the H2D copies (pinned meta reusable)
  hipEvent_t check_done;  // prep stream, after the scan (host_out valid)
  hipEvent_t ready;       // prep stream, after hashing / hot detection
  hipEvent_t set_free;    // compute stream, after the train launch (device set reusable)
  hipEvent_t hot_free;    // compute stream, after the train launch that read the hot set;
                          // the prep stream waits on its previous record first
  hipEvent_t hot_seen;    // prep stream, after the copy of the hot-row count
  // request bytes (pinned host) and the per-request table [off R | len R | base R+1]
  const uint8_t* arena;
  int64_t used;
  const int64_t* meta_host;
  int64_t R, n;
  // device buffers of the set
  uint8_t* d_buf;
  int64_t buf_cap, empty_off;
  int64_t* d_meta;
  int64_t* d_off;
  int32_t* d_len;
  int32_t* d_lab;
  int64_t* d_row;
  int64_t* d_slots;
  uint32_t* d_hist;
  int64_t nhist;
  int32_t* d_err;
  int32_t* host_out;
  // label table
  const uint64_t* lt_hash;
  const int32_t* lt_meta;
  int64_t lt_cap;
  const uint8_t* lt_blob;
  int64_t lt_blob_len, sps, spn;
  // feature hashing
  const void* srules;
  const void* nrules;
  int64_t n_srules, n_nrules;
  const uint8_t* blob;
  int64_t blob_len, H;
  int32_t* d_idx;
  float* d_val;
  int64_t slot_cap;
  int32_t* hash_err;
  // hot rows (hot_rows null: no detection)
  int32_t* hot_rows;
  int32_t* hot_n;
  float* hot_rep;
  int32_t* gkey;
  int32_t* gcnt;
  int64_t gcap, block_min, min_count, max_rows, hot_free_valid;
  int32_t* hot_count_host;  // nullable: receives the hot-row count
  // train (W null: prepare only)
  float* W;
  float* S;
  const int32_t* active;
  int64_t LC, method;
  double C;
  int64_t mode, merge_every, hot_waves;
  unsigned long long* stats;
  uint8_t* touched;
  // mode kSerial: scratch of jb_serial_scratch_bytes_lc(n, LC) bytes (serial.hip)
  void* serial_scratch;
  int64_t serial_bytes;
  // 1: W is a bf16 table (uint16 bit patterns; jb_linear_train_bf16)
  int64_t w_bf16;
};

extern "C" int64_t jb_train_batch_args_bytes();
// 0 ok, 1 a launch helper refused its arguments, 2 a HIP runtime error
extern "C" int jb_train_batch_submit(const JbTrainBatch* a);

#endif  // JUBATUS_AMD_CSRC_HIP_JB_TRAIN_BATCH_HPP_
