// Worker inference engine: weights resident in HBM, N1 warm-start, N2
// forward captured as a hipGraph (one graph launch per pass).
#pragma once

#include <hip/hip_runtime.h>

#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace kiosk {

void check_hip(hipError_t err, const char* what);
long long monotonic_ns();

// Standby pre-initialisation on the (already pinned) device: create the
// HIP context and load every kernel code object by launching each kernel
// once on a tiny scratch buffer, then free it.  Leaves no HBM allocated
// and nothing running; the later Engine ctor then skips ~150 ms of
// runtime init + code-object loading.  Returns stage timestamps.
// Destroys the stream preinit_device kept for the next Engine (if no Engine
// took it): the standby's exit path, so teardown does not depend on process
// exit.
void release_kept_stream();
// The kept stream for a caller outside Engine (the PyTorch engine wraps it
// in torch.cuda.ExternalStream): 0 if none is kept for `device`.  The
// caller owns it until it hands it back with return_stream.
unsigned long long take_stream(int device);
void return_stream(unsigned long long handle, int device);
std::vector<std::pair<std::string, long long>> preinit_device(int device);
// Pays the HIP runtime's one-time graph set-up (the first instantiation of
// a non-empty graph) on a one-memset graph; preinit_device runs it.
hipError_t graph_prewarm(int device);
// `context` standby: HIP context + every kernel's code object, no launch (so
// no hardware queue and no HBM beyond the code objects).
std::vector<std::pair<std::string, long long>> preload_modules(int device);

struct WarmStartResult {
  int blocks = 0;
  int distinct_cus = 0;
  int distinct_xccs = 0;
  int iters = 0;
  int lds_bytes = 0;
  double kernel_us = 0;     // hipEvent-timed
  double span_us = 0;       // first start -> last end, s_memrealtime
  double wall_us = 0;       // host wall incl. launch + sync
  double checksum = 0;
  std::vector<unsigned> cu_keys;   // (xcc << 16) | (se << 8) | (sh << 4) | cu
};

struct ForwardResult {
  double ms = 0;        // host wall of the key (incl. sync)
  double gpu_ms = 0;    // hipEvent-timed device span
  double checksum = 0;
  int rows = 0;
  int passes = 0;
  bool graph = false;
};

class Engine {
 public:
  Engine(int device, int dim, int hidden, int layers, int max_rows,
         unsigned long long seed);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  WarmStartResult warmstart(int iters, int lds_bytes);
  void prepare(int rows);                      // capture + instantiate graph
  ForwardResult forward(int rows, int passes, unsigned long long seed);
  // fault injection: stall the engine's stream for `ms` (bounded kernel)
  double spin(double ms);
  void close();

  const std::vector<std::pair<std::string, long long>>& stages() const {
    return stages_;
  }
  std::map<std::string, double> info() const;

  // copy the last forward's [rows, dim] bf16 output to device memory `dst`
  // (numerics tests: elementwise comparison against the fp32 reference)
  void copy_output(unsigned long long dst, int rows);
  // raw pointers for numerics tests
  unsigned long long weight_ptr(int layer, int which) const;
  unsigned long long act_ptr(int which) const;
  unsigned long long stream_handle() const {
    return reinterpret_cast<unsigned long long>(stream_);
  }
  int dim() const { return dim_; }
  int hidden() const { return hidden_; }
  int layers() const { return layers_; }
  int max_rows() const { return max_rows_; }

 private:
  void stage(const char* name);
  void init(int device, unsigned long long seed);   // constructor body
  void enqueue_forward(int rows);              // one pass on stream_
  void launch_or_throw(hipError_t err, const char* what);
  void build_warm_graph(int iters, int lds_bytes);

  int device_ = 0;
  int dim_, hidden_, layers_, max_rows_;
  int cu_count_ = 0;
  bool closed_ = false;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
  char* arena_ = nullptr;
  size_t arena_bytes_ = 0;
  std::vector<uint16_t*> w1_, w2_;
  std::vector<float*> b1_, b2_;
  uint16_t* x_ = nullptr;      // layer input / ping
  uint16_t* y_ = nullptr;      // layer output / pong
  uint16_t* h_ = nullptr;      // hidden activation
  float* partials_ = nullptr;
  float* workspace_ = nullptr;     // split-K fp32 partials (may be null)
  size_t workspace_bytes_ = 0;
  unsigned long long* seed_dev_ = nullptr;
  // N1 as one instantiated graph (memset record -> warm-start kernel ->
  // record to pinned host): a READY after the first is a hipGraphLaunch,
  // which -- unlike a kernel launch -- never waits on the HIP runtime lock
  // RCCL holds while it loads (profiles/r4_collision)
  hipGraph_t warm_graph_ = nullptr;
  hipGraphExec_t warm_exec_ = nullptr;
  int warm_iters_ = -1, warm_lds_ = -1;
  uint32_t* warm_rec_ = nullptr;       // device record, blocks x words
  uint32_t* warm_host_ = nullptr;      // pinned copy
  unsigned long long* seed_host_ = nullptr;   // pinned staging
  float* partials_host_ = nullptr;            // pinned
  std::map<int, std::pair<hipGraph_t, hipGraphExec_t>> graphs_;
  std::vector<std::pair<std::string, long long>> stages_;
};

}  // namespace kiosk
