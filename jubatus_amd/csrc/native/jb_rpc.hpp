// msgpack-RPC transport (server side), native C++17.
//
// Reference: jubatus/server/common/mprpc/rpc_server.{hpp,cpp} (dispatcher
// over msgpack-rpc/mpio). Wire protocol (msgpack-RPC):
//   request      [0, msgid, method, params]
//   response     [1, msgid, error, result]
//   notification [2, method, params]
//
// Design: one epoll IO thread owns every socket (accept, non-blocking reads,
// message framing by a validating skip-walk, deferred writes); complete
// requests go to a queue served by `nworkers` threads that call the
// dispatcher callback (Python, with the GIL) and hand back the encoded
// response. Request parameter bytes are copied once out of the socket buffer
// into an owned string (or, for the train fast path, into a pinned arena by
// the callback) - never decoded in C++ unless the callback asks for it.
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace jb {

struct RpcRequest {
  uint64_t conn_id;
  uint32_t msgid;
  bool notify;
  std::string method;
  std::string params;  // msgpack array bytes
  std::shared_ptr<void> prep;   // the prep hook's result (set_prep), or null
};

// A request of the arena-batched method: its body (params[1]) sits at
// [off, off + len) of an arena slot.
struct ArenaReq {
  uint64_t conn_id;
  uint32_t msgid;
  uint64_t off;
  uint64_t len;
};

// Resumable framing state of one connection's partial message: the walk
// continues where the previous read stopped (no re-parse per read).
struct FrameState {
  uint64_t pos = 0;                 // next token, relative to the message start (may
                                    // lie past the bytes received: a payload in flight)
  uint64_t rem = 0;                 // objects still to skip
  bool started = false;
  void reset() { pos = 0; rem = 0; started = false; }
};

// 1 complete (st.pos = length), 0 need more bytes, -1 malformed
int frame_resume(const uint8_t* b, size_t n, FrameState& st);

// Every complete message in [b, b + n), the first one continuing the state
// st: appends their end offsets (from b) to *ends and leaves st describing
// the incomplete message after the last end (positions relative to it).
// 0, or -1 at a malformed byte (the ends before it stand). speculative:
// frame large buffers by parallel walks (jb_rpc.cpp; measured slower than
// the single walk on train requests, kept for the tests and experiments).
int frame_all(const uint8_t* b, size_t n, FrameState& st, std::vector<uint64_t>* ends,
              bool speculative = false);

// Receive buffer of one connection: reads land at the tail, framed messages
// leave at the head (no per-message erase; the live bytes move to the front
// only when the free tail runs short).
class RecvBuf {
 public:
  const uint8_t* data() const { return d_.get() + head_; }
  size_t size() const { return tail_ - head_; }
  // writable space of at least `want` bytes at the tail
  uint8_t* space(size_t want, size_t* got);
  void produced(size_t n) { tail_ += n; }
  void consume(size_t n) {
    head_ += n;
    if (head_ == tail_) {
      head_ = tail_ = 0;
      // one large request must not pin its buffer for the connection's
      // lifetime: drop back to the steady-state size once drained
      if (cap_ > kShrinkAbove) {
        d_.reset();
        cap_ = 0;
      }
    }
  }
  static constexpr size_t kShrinkAbove = (size_t)4 << 20;

 private:
  std::unique_ptr<uint8_t[]> d_;
  size_t cap_ = 0, head_ = 0, tail_ = 0;
};

class RpcServer {
 public:
  // handler(request) -> encoded response bytes (empty for notifications)
  using Handler = std::function<std::string(const RpcRequest&)>;

  // batch handler(method, requests) -> one encoded response per request
  // (empty string: no response, e.g. a notification)
  using BatchHandler =
      std::function<std::vector<std::string>(const std::string&, std::vector<RpcRequest>&)>;

  RpcServer(Handler h, int nworkers, double idle_timeout_sec);
  // Requests of `methods` bypass the per-request workers: one batch thread
  // drains everything queued for a method and calls `h` once for all of it
  // (concurrent train / classify RPCs become one GPU launch). Call before start().
  void set_batch(const std::vector<std::string>& methods, BatchHandler h, size_t max_batch);
  // Batched methods that write: a batch keeps arrival order around them
  // (it never takes a request past one of another method when either is
  // an ordered method), so pipelined writes of different methods - an
  // update_row, then a clear_row of the row - apply in the order sent.
  // Reads of different methods still batch past each other.
  void set_ordered(const std::vector<std::string>& methods) { ordered_ = methods; }
  // Called on the IO thread for every request of a batched method before it
  // is queued (e.g. decode and hash a write's datum there, so the batch
  // thread - the serial part - only applies it). Call before start().
  void set_prep(std::function<void(RpcRequest&)> h) { prep_ = std::move(h); }

  // arena handler(slot, requests) -> one encoded response per request
  using ArenaHandler = std::function<std::vector<std::string>(int, const std::vector<ArenaReq>&)>;
  // Arena batching for `method` (params [name, body], e.g. train): the IO
  // thread that frames a request copies its body straight into the open slot
  // of caller-owned (pinned) memory - no intermediate string, no Python;
  // the batch thread seals the slot and calls `h` once for every request in
  // it. A slot is reused after release_slot(); when no slot has room the
  // request takes the ordinary batch path (the handler of set_batch).
  void set_arena_batch(const std::string& method, const std::vector<uint8_t*>& slots,
                       size_t slot_bytes, ArenaHandler h);
  void release_slot(int slot);
  // largest accepted request (bytes); a connection sending more is closed
  void set_max_message(uint64_t n) { max_message_ = n; }
  uint64_t batches() const { return batches_.load(); }
  // arena batches: nanoseconds in the handler / in sending the responses
  uint64_t arena_handler_ns() const { return arena_handler_ns_.load(); }
  uint64_t arena_send_ns() const { return arena_send_ns_.load(); }
  ~RpcServer();
  // returns the bound port (useful with port 0)
  int listen(const std::string& addr, int port);
  void start();
  void stop();
  // number of epoll IO threads (connections are spread round-robin); call
  // before start(). One thread frames ~1 GB/s of request bytes.
  void set_io_threads(int n) { nio_ = n < 1 ? 1 : n; }
  // batch threads (>1: a batch is served while the next one is collected
  // and submitted; the arena handler waits on the GPU without the GIL)
  void set_batch_threads(int n) { nbatch_ = n < 1 ? 1 : n; }
  bool running() const { return running_.load(); }
  uint64_t requests_served() const { return served_.load(); }
  uint64_t connections() const { return nconn_.load(); }

 private:
  struct Conn {
    int fd;
    uint64_t id;
    int loop = 0;
    RecvBuf rbuf;
    FrameState fs;     // framing progress of the message at the head of rbuf
    std::mutex wmu;
    std::string wbuf;  // pending output
    bool want_write = false;
    bool closed = false;
    double last_active = 0;
  };
  struct Loop {
    int epfd = -1;
    int wake_fd = -1;
    std::thread th;
    std::mutex wq_mu;
    std::vector<uint64_t> want_write;  // conns this loop must arm for EPOLLOUT
  };
  void io_loop(int li);
  void worker_loop();
  void on_readable(const std::shared_ptr<Conn>& c);
  void flush(const std::shared_ptr<Conn>& c);
  void close_conn(uint64_t id);
  void send_response(uint64_t conn_id, const std::string& bytes);
  void send_responses(const std::vector<uint64_t>& conn_ids, const std::vector<std::string>& resp);
  // idx 0 also serves the generic batch queue (one thread, so batched
  // requests are handled in arrival order); the others take arena slots only
  void batch_loop(int idx);
  void enqueue(RpcRequest&& req);
  bool arena_take(uint64_t conn_id, uint32_t msgid, const uint8_t* body, size_t len);
  bool arena_batch_once();

  Handler handler_;
  int nworkers_;
  double idle_timeout_;
  int listen_fd_ = -1;
  int nio_ = 1;
  std::vector<std::unique_ptr<Loop>> loops_;
  std::atomic<uint64_t> next_loop_{0};
  std::atomic<bool> running_{false};
  std::atomic<uint64_t> served_{0};
  std::atomic<uint64_t> nconn_{0};
  std::vector<std::thread> workers_;
  std::mutex cmu_;
  std::unordered_map<uint64_t, std::shared_ptr<Conn>> conns_;
  uint64_t next_id_ = 1;
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<RpcRequest> queue_;
  std::atomic<size_t> qlen_{0};   // queue_.size(), readable without qmu_
  // batched methods
  std::vector<std::string> batch_methods_;
  std::vector<std::string> ordered_;
  std::function<void(RpcRequest&)> prep_;
  BatchHandler batch_handler_;
  size_t max_batch_ = 4096;
  std::mutex bmu_;
  std::condition_variable bcv_;
  std::deque<RpcRequest> bqueue_;
  std::vector<std::thread> batchers_;
  int nbatch_ = 1;
  std::atomic<uint64_t> batches_{0};
  std::atomic<uint64_t> arena_handler_ns_{0}, arena_send_ns_{0};
  uint64_t max_message_ = (uint64_t)1 << 31;
  // arena batching
  struct Slot {
    uint8_t* base = nullptr;
    uint64_t used = 0;
    int writers = 0;          // IO threads still copying into this slot
    bool busy = false;        // handed to the handler, not released yet
    std::vector<ArenaReq> reqs;
  };
  std::string arena_method_;
  ArenaHandler arena_handler_;
  uint64_t slot_bytes_ = 0;
  std::vector<Slot> slots_;
  int open_ = -1;             // slot receiving bodies (-1: none)
  std::mutex amu_;            // guards slots_ / open_; waits on bcv_ use bmu_
  std::condition_variable acv_;   // writers drained / slot released
};

// Frame one complete msgpack object at the head of [p, p+n): returns its
// length, 0 if incomplete, -1 if malformed.
int64_t msgpack_frame(const uint8_t* p, size_t n);

}  // namespace jb
