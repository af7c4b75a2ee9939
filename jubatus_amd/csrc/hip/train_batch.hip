// One host call per GPU-scan train batch: H2D of the request bytes, request
// scan, feature hashing, hot-row detection and the train launch, with the
// stream / event choreography of ops/feature_pipeline.py (copy stream ->
// prep stream -> compute stream). The served train path (models/
// classifier.py train_arena_sync) and the arena path (train_arena) submit
// here, so a batch costs one ctypes call instead of ~20 Python-level
// launches, slices, copies and event records (measured ~420 us of host time
// per batch under the model lock, the bound of the served rate).
//
// Reference context: the per-request train of jubatus/server/server/
// classifier_serv.cpp:128-147 (a sample loop under the model's write lock);
// here one call covers every request the transport batched into a slot.
//
// Also: a small event API (create / record / wait / query / sync / destroy)
// so that the Python side can hold the batch's events without torch.
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" int jb_scan_train(const uint8_t* buf, const int64_t* req_off, const int64_t* req_len,
                             const int64_t* sample_base, int R, const uint64_t* lt_hash,
                             const int32_t* lt_meta, int lt_cap, const uint8_t* lt_blob,
                             int lt_blob_len, int sps, int spn, int64_t* datum_off,
                             int32_t* datum_len, int32_t* labels, int64_t* row_ptr,
                             int64_t* req_slots, uint32_t* hist, int nhist, int32_t* err,
                             uint8_t* empty_at, int64_t empty_off, int32_t* host_out,
                             hipStream_t stream);
extern "C" int jb_fv_hash(const uint8_t* buf, int64_t buf_len, int64_t buf_cap,
                          const int64_t* datum_off, const int32_t* datum_len,
                          const int64_t* row_ptr, int n, const void* srules, int n_srules,
                          const void* nrules, int n_nrules, const uint8_t* blob, int blob_len,
                          uint64_t H, int32_t* out_idx, float* out_val, int32_t* err,
                          hipStream_t stream);
extern "C" int jb_hot_detect(const int64_t* row_ptr, int n, const int32_t* fidx, int64_t max_slots,
                             int block_min, int min_count, int max_rows, int32_t* gkey,
                             int32_t* gcnt, int gcap, int32_t* hot_rows, int32_t* hot_n,
                             hipStream_t stream);
extern "C" int jb_linear_train(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                               const int32_t* labels, const int64_t* stream_ptr, int nstreams,
                               float* W, float* S, const int32_t* active, int LC, int method,
                               float C, int mode, const int32_t* hot_rows, const int32_t* hot_n,
                               float* hot_rep, int merge_every, int hot_waves,
                               unsigned long long* stats, uint8_t* touched, int64_t n_max,
                               void* scratch, int64_t scratch_bytes, hipStream_t stream);
extern "C" int jb_linear_train_bf16(const int64_t* row_ptr, const int32_t* fidx,
                                    const float* fval, const int32_t* labels,
                                    const int64_t* stream_ptr, int nstreams, uint16_t* W,
                                    float* S, const int32_t* active, int LC, int method, float C,
                                    int mode, unsigned long long* stats, uint8_t* touched,
                                    void* scratch, int64_t scratch_bytes, hipStream_t stream);

#include "jb_train_batch.hpp"

#define JB_TRY(x) do { if ((x) != hipSuccess) return 2; } while (0)

extern "C" int64_t jb_train_batch_args_bytes() { return (int64_t)sizeof(JbTrainBatch); }

// 0 ok, 1 a launch helper refused its arguments, 2 a HIP runtime error
extern "C" int jb_train_batch_submit(const JbTrainBatch* a) {
  const int R = (int)a->R;
  const int n = (int)a->n;
  if (R <= 0 || a->R > INT32_MAX || a->n > INT32_MAX) return 1;
  if (a->used) JB_TRY(hipMemcpyAsync(a->d_buf, a->arena, (size_t)a->used, hipMemcpyHostToDevice,
                                     a->copy_stream));
  JB_TRY(hipMemcpyAsync(a->d_meta, a->meta_host, sizeof(int64_t) * (size_t)(3 * a->R + 1),
                        hipMemcpyHostToDevice, a->copy_stream));
  JB_TRY(hipEventRecord(a->copy_done, a->copy_stream));
  JB_TRY(hipStreamWaitEvent(a->prep_stream, a->copy_done, 0));
  ((volatile int32_t*)a->host_out)[0] = -1;          // not yet written by the fixup kernel
  const int64_t* sbase = a->d_meta + 2 * a->R;
  if (jb_scan_train(a->d_buf, a->d_meta, a->d_meta + a->R, sbase, R, a->lt_hash, a->lt_meta,
                    (int)a->lt_cap, a->lt_blob, (int)a->lt_blob_len, (int)a->sps, (int)a->spn,
                    a->d_off, a->d_len, a->d_lab, a->d_row, a->d_slots, a->d_hist, (int)a->nhist,
                    a->d_err, a->d_buf + a->empty_off, a->empty_off, a->host_out,
                    a->prep_stream) != 0)
    return 1;
  JB_TRY(hipEventRecord(a->check_done, a->prep_stream));
  const bool hot = a->hot_rows != nullptr && n > 0;
  if (n > 0) {
    if (jb_fv_hash(a->d_buf, a->empty_off + 3, a->buf_cap, a->d_off, a->d_len, a->d_row, n,
                   a->srules, (int)a->n_srules, a->nrules, (int)a->n_nrules, a->blob,
                   (int)a->blob_len, (uint64_t)a->H, a->d_idx, a->d_val, a->hash_err,
                   a->prep_stream) != 0)
      return 1;
    if (hot) {
      if (a->hot_free_valid) JB_TRY(hipStreamWaitEvent(a->prep_stream, a->hot_free, 0));
      if (jb_hot_detect(a->d_row, n, a->d_idx, a->slot_cap, (int)a->block_min, (int)a->min_count,
                        (int)a->max_rows, a->gkey, a->gcnt, (int)a->gcap, a->hot_rows, a->hot_n,
                        a->prep_stream) != 0)
        return 1;
      if (a->hot_count_host) {
        JB_TRY(hipMemcpyAsync(a->hot_count_host, a->hot_n, sizeof(int32_t), hipMemcpyDeviceToHost,
                              a->prep_stream));
        JB_TRY(hipEventRecord(a->hot_seen, a->prep_stream));
      }
    }
  }
  JB_TRY(hipEventRecord(a->ready, a->prep_stream));
  JB_TRY(hipStreamWaitEvent(a->compute_stream, a->ready, 0));
  if (a->W != nullptr && n > 0 && a->w_bf16) {
    if (jb_linear_train_bf16(a->d_row, a->d_idx, a->d_val, a->d_lab, sbase, R, (uint16_t*)a->W,
                             a->S, a->active, (int)a->LC, (int)a->method, (float)a->C,
                             (int)a->mode, a->stats, a->touched, a->serial_scratch,
                             a->serial_bytes, a->compute_stream) != 0)
      return 1;
  } else if (a->W != nullptr && n > 0) {
    if (jb_linear_train(a->d_row, a->d_idx, a->d_val, a->d_lab, sbase, R, a->W, a->S, a->active,
                        (int)a->LC, (int)a->method, (float)a->C, (int)a->mode,
                        hot ? a->hot_rows : nullptr, hot ? a->hot_n : nullptr,
                        hot ? a->hot_rep : nullptr, (int)a->merge_every, (int)a->hot_waves,
                        a->stats, a->touched, a->n, a->serial_scratch, a->serial_bytes,
                        a->compute_stream) != 0)
      return 1;
    if (hot) JB_TRY(hipEventRecord(a->hot_free, a->compute_stream));
  }
  JB_TRY(hipEventRecord(a->set_free, a->compute_stream));
  return 0;
}

// ------------------------------------------------------------------ events
extern "C" int64_t jb_event_create() {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return 0;
  return (int64_t)(intptr_t)e;
}

extern "C" int jb_event_destroy(int64_t e) {
  return e ? (int)hipEventDestroy((hipEvent_t)(intptr_t)e) : 0;
}

extern "C" int jb_event_record(int64_t e, hipStream_t stream) {
  return (int)hipEventRecord((hipEvent_t)(intptr_t)e, stream);
}

extern "C" int jb_stream_wait_event(hipStream_t stream, int64_t e) {
  return (int)hipStreamWaitEvent(stream, (hipEvent_t)(intptr_t)e, 0);
}

// 0 complete, 1 not yet, other: the HIP error
extern "C" int jb_event_query(int64_t e) {
  const hipError_t r = hipEventQuery((hipEvent_t)(intptr_t)e);
  if (r == hipSuccess) return 0;
  return r == hipErrorNotReady ? 1 : (int)r;
}

extern "C" int jb_event_sync(int64_t e) {
  return (int)hipEventSynchronize((hipEvent_t)(intptr_t)e);
}
