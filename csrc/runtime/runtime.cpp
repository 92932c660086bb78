// Native host runtime: the data path the reference runs serially in Python
// (DataLoader with num_workers=0, main.py:102; GetData.__getitem__, data_loader.py:29-37).
//
// BatchRing: a bounded ring of pinned (hipHostMalloc) batch slots filled by C++ producer
// threads, consumed by the training loop, which issues one async H2D copy per batch on a
// dedicated copy stream and hands the slot back once that copy's event has completed.
// Producers never hold the GIL.  Two producer modes:
//   * synthetic: deterministic pseudo-random uint8 HWC images + uniform labels
//     (BASELINE.json: synthetic data, no Herbarium images offline);
//   * external: Python (PIL decode threads) writes decoded images into a slot obtained
//     with acquire_empty()/commit() - the same ring feeds the GPU preprocess kernel.
//
// Markers: roctx ranges so rocprofv3 --marker-trace shows step phases.
#include "runtime.h"

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace mpa_runtime {

namespace {

inline uint64_t splitmix(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Slot {
  uint8_t* img = nullptr;    // pinned [B,H,W,3]
  int64_t* labels = nullptr; // pinned [B]
  int64_t batch_index = -1;
};

class BatchRing {
 public:
  BatchRing(int batch, int H, int W, int64_t num_classes, int depth, int threads, uint64_t seed,
            int64_t start_index, int64_t stride, bool synthetic)
      : B_(batch), H_(H), W_(W), nc_(num_classes), seed_(seed), next_index_(start_index),
        stride_(stride), synthetic_(synthetic) {
    TORCH_CHECK(depth >= 2, "BatchRing depth must be >= 2");
    slots_.resize(depth);
    const size_t img_bytes = (size_t)B_ * H_ * W_ * 3;
    for (auto& s : slots_) {
      void* p = nullptr;
      TORCH_CHECK(hipHostMalloc(&p, img_bytes, hipHostMallocDefault) == hipSuccess,
                  "hipHostMalloc failed");
      s.img = (uint8_t*)p;
      TORCH_CHECK(hipHostMalloc(&p, sizeof(int64_t) * B_, hipHostMallocDefault) == hipSuccess,
                  "hipHostMalloc failed");
      s.labels = (int64_t*)p;
    }
    for (int i = 0; i < depth; ++i) empty_.push_back(i);
    if (synthetic_) {
      for (int t = 0; t < std::max(1, threads); ++t) workers_.emplace_back([this] { produce(); });
    }
  }

  ~BatchRing() { stop(); free_all(); }

  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stopping_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_)
      if (t.joinable()) t.join();
    workers_.clear();
  }

  // consumer: block until a filled slot is available (releases the GIL while waiting)
  std::tuple<int, torch::Tensor, torch::Tensor, int64_t> acquire() {
    int id;
    {
      pybind11::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return !ready_.empty() || stopping_; });
      TORCH_CHECK(!ready_.empty(), "BatchRing stopped");
      id = ready_.front();
      ready_.pop_front();
    }
    return {id, view_img(id), view_labels(id), slots_[id].batch_index};
  }

  void release(int id) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      empty_.push_back(id);
    }
    cv_.notify_all();
  }

  // external producer API (real-data mode): grab an empty slot, fill it, commit
  std::tuple<int, torch::Tensor, torch::Tensor> acquire_empty() {
    int id;
    {
      pybind11::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return !empty_.empty() || stopping_; });
      TORCH_CHECK(!empty_.empty(), "BatchRing stopped");
      id = empty_.front();
      empty_.pop_front();
    }
    return {id, view_img(id), view_labels(id)};
  }

  void commit(int id, int64_t batch_index) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      slots_[id].batch_index = batch_index;
      ready_.push_back(id);
    }
    cv_.notify_all();
  }

  int depth() const { return (int)slots_.size(); }

 private:
  torch::Tensor view_img(int id) {
    auto opt = torch::TensorOptions().dtype(torch::kUInt8).pinned_memory(true);
    return torch::from_blob(slots_[id].img, {B_, H_, W_, 3}, opt);
  }
  torch::Tensor view_labels(int id) {
    auto opt = torch::TensorOptions().dtype(torch::kInt64).pinned_memory(true);
    return torch::from_blob(slots_[id].labels, {B_}, opt);
  }

  void fill_synthetic(Slot& s, int64_t bidx) {
    const size_t per_img = (size_t)H_ * W_ * 3;
    for (int b = 0; b < B_; ++b) {
      uint64_t st = seed_ * 0x100000001B3ull ^ ((uint64_t)bidx * B_ + b);
      s.labels[b] = (int64_t)(splitmix(st) % (uint64_t)nc_);
      uint64_t* dst = (uint64_t*)(s.img + per_img * b);
      const size_t n64 = per_img / 8;
      uint64_t x = splitmix(st);
      for (size_t i = 0; i < n64; ++i) {  // xorshift64*: ~1 ns / 8 bytes
        x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
        dst[i] = x * 0x2545F4914F6CDD1Dull;
      }
      for (size_t i = n64 * 8; i < per_img; ++i) s.img[per_img * b + i] = (uint8_t)(x >> (i & 7));
    }
    s.batch_index = bidx;
  }

  void produce() {
    while (true) {
      int id;
      int64_t bidx;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !empty_.empty() || stopping_; });
        if (stopping_) return;
        id = empty_.front();
        empty_.pop_front();
        bidx = next_index_;
        next_index_ += stride_;
      }
      fill_synthetic(slots_[id], bidx);
      {
        std::lock_guard<std::mutex> lk(mu_);
        // keep batches in order: insert sorted by batch index
        auto it = ready_.begin();
        while (it != ready_.end() && slots_[*it].batch_index < bidx) ++it;
        ready_.insert(it, id);
      }
      cv_.notify_all();
    }
  }

  void free_all() {
    for (auto& s : slots_) {
      if (s.img) (void)hipHostFree(s.img);
      if (s.labels) (void)hipHostFree(s.labels);
      s.img = nullptr;
      s.labels = nullptr;
    }
  }

  int B_, H_, W_;
  int64_t nc_;
  uint64_t seed_;
  int64_t next_index_, stride_;
  bool synthetic_;
  std::vector<Slot> slots_;
  std::deque<int> empty_, ready_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stopping_ = false;
  std::vector<std::thread> workers_;
};

}  // namespace

void register_bindings(pybind11::module_& m) {
  pybind11::class_<BatchRing>(m, "BatchRing")
      .def(pybind11::init<int, int, int, int64_t, int, int, uint64_t, int64_t, int64_t, bool>(),
           pybind11::arg("batch"), pybind11::arg("height"), pybind11::arg("width"),
           pybind11::arg("num_classes"), pybind11::arg("depth") = 4, pybind11::arg("threads") = 2,
           pybind11::arg("seed") = 0, pybind11::arg("start_index") = 0,
           pybind11::arg("stride") = 1, pybind11::arg("synthetic") = true)
      .def("acquire", &BatchRing::acquire)
      .def("release", &BatchRing::release)
      .def("acquire_empty", &BatchRing::acquire_empty)
      .def("commit", &BatchRing::commit)
      .def("stop", &BatchRing::stop)
      .def("depth", &BatchRing::depth);
  m.def("range_push", [](const std::string& s) { return roctxRangePushA(s.c_str()); });
  m.def("range_pop", []() { return roctxRangePop(); });
  m.def("mark", [](const std::string& s) { roctxMarkA(s.c_str()); });
}

}  // namespace mpa_runtime
