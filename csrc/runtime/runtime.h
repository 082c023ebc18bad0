// Host-side native runtime of paddle2_amd (no GPU code): rendezvous store, comm watchdog,
// host event tracer, and the bounded blocking queue used by the data loader.
#pragma once

#include <array>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace pdrt {

// ------------------------------------------------------------------ TCPStore (tcp_store.cpp)
class TCPStoreServer {
 public:
  TCPStoreServer(const std::string& host, int port);
  ~TCPStoreServer();
  int port() const;
  void shutdown();

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

class TCPStoreClient {
 public:
  TCPStoreClient(const std::string& host, int port, double timeout_s);
  ~TCPStoreClient();
  void set(const std::string& k, const std::string& v);
  std::string get(const std::string& k);  // blocks until the key exists (or timeout)
  int64_t add(const std::string& k, int64_t inc);
  bool check(const std::vector<std::string>& keys);
  void wait(const std::vector<std::string>& keys);
  bool remove(const std::string& k);
  int64_t num_keys();
  std::string compare_set(const std::string& k, const std::string& expected, const std::string& desired);
  int64_t append(const std::string& k, const std::string& v);  // server-side atomic append -> new length
  void set_timeout(double s);
  double timeout() const { return timeout_s_; }

 private:
  void send_all(const std::string& b);
  void recv_all(char* p, size_t n);
  std::string recv_str();
  int fd_ = -1;
  double timeout_s_;
  std::mutex mu_;
};

// ------------------------------------------------------------------ host tracer (tracer.cpp)
struct HostEvent {
  uint32_t name_id;
  uint32_t type;  // 0 = user range (RecordEvent), 1 = op, 2 = comm, 3 = dataloader, 4 = optimizer
  uint64_t tid;
  uint64_t start_ns, end_ns;
};

void tracer_enable(bool on);
bool tracer_enabled();
void tracer_push(const std::string& name, uint32_t type);
void tracer_pop();
void tracer_instant(const std::string& name, uint32_t type, uint64_t start_ns, uint64_t end_ns);
uint64_t tracer_now_ns();
void tracer_clear();
std::vector<HostEvent> tracer_events();
std::string tracer_name(uint32_t id);
std::string tracer_chrome_json(int pid);

// ------------------------------------------------------------------ comm watchdog (watchdog.cpp)
void watchdog_start(double poll_s, bool abort_on_timeout);
void watchdog_stop();
int64_t watchdog_begin(const std::string& desc, double timeout_s, uintptr_t hip_event = 0);
std::vector<int64_t> watchdog_take_finished();
void watchdog_end(int64_t id);
std::vector<std::string> watchdog_timed_out();
int64_t watchdog_inflight();

// ------------------------------------------------------------------ FleetExecutor (fleet_executor.cpp)
struct FleetTask {
  enum Role : int { kCompute = 0, kAmplifier = 1, kSource = 2, kSink = 3 };
  int64_t id = 0;
  int rank = 0;
  int role = kCompute;
  int64_t max_run_times = 1;
  int64_t run_per_steps = 1;
  int64_t run_at_offset = 0;
  std::vector<std::pair<int64_t, int64_t>> upstream;    // (task id, buffer size)
  std::vector<std::pair<int64_t, int64_t>> downstream;  // (task id, buffer size)
};

class FleetCarrier {
 public:
  using ComputeFn = std::function<void(int64_t task, int64_t step)>;
  FleetCarrier(int rank, int num_threads);
  ~FleetCarrier();
  void add_task(const FleetTask& t);           // every task of the job; only this rank's get interceptors
  void add_remote_task(int64_t id, int rank);
  void set_compute(ComputeFn fn);
  int listen(const std::string& host);          // message-bus listener; returns the port
  void set_peer(int rank, const std::string& host, int port);
  void start();
  bool wait(double timeout_s);                  // true when every local task finished; throws on error
  std::vector<std::array<int64_t, 3>> trace();  // (task, step, sequence) of compute callbacks
  void clear_trace();
  void shutdown();

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

// ------------------------------------------------------------------ static-graph interpreter (interpreter.cpp)
struct InterpPlan {
  int n = 0;
  int64_t num_edges_raw = 0;                       // RAW + WAR + WAW + barrier edges before the reduction
  std::vector<std::vector<int>> downstream;        // transitively reduced successors
  std::vector<int> dep_count;                      // predecessors per instruction
  std::vector<int> order;                          // issue order (topological; side streams first when ready)
  std::vector<std::vector<int>> waits;             // producers on another stream (wait on their events)
  std::vector<char> record;                        // record an event after this instruction
  std::vector<std::vector<int64_t>> free_after;    // sequential issue: variables dead after this instruction
  std::unordered_map<int64_t, int> reader_count;   // async queue: readers per (non-kept) variable
  std::vector<std::vector<int64_t>> reads;         // per instruction, de-duplicated
};

InterpPlan build_interp_plan(const std::vector<std::vector<int64_t>>& reads,
                             const std::vector<std::vector<int64_t>>& writes, const std::vector<int>& stream,
                             const std::vector<int>& barrier, const std::vector<int64_t>& keep);

// Dependency-counting ready queue over a plan: worker threads pop() ready instructions, run them, and report
// done(i), which releases successors and returns the variables whose last reader just finished.
class ReadyQueue {
 public:
  explicit ReadyQueue(const InterpPlan& plan);
  ~ReadyQueue();
  void start();
  int pop(double timeout_s);          // instruction id; -1 = finished or aborted; -2 = timed out
  std::vector<int64_t> done(int i);
  void fail();                        // abort: every waiting pop() returns -1
  bool finished();

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

}  // namespace pdrt
