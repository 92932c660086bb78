// Native host runtime: the data path the reference runs serially in Python
// (DataLoader with num_workers=0, main.py:102; GetData.__getitem__, data_loader.py:29-37;
// the eval pipeline's read stage, evaluation_pipeline.py:53-71).
//
// BatchRing: a bounded ring of pinned (hipHostMalloc) batch slots filled by producers,
// consumed by the training loop / eval pipeline, which issue one async H2D copy per batch on
// a dedicated copy stream and hand the slot back once that copy's event has completed.
// Every slot carries uint8 images [B][H][W][3] (H x W is the PITCH: an image may occupy only
// its top-left extent, ext[b] = (h, w), so real JPEGs of different sizes share one slot and
// one preprocess launch), int64 labels [B], the batch index and the valid image count.
// Consumers receive batches in batch-index order (start_index, start_index + stride, ...),
// whatever order the producers finish them in, so data order is deterministic.
// Producer modes (native ones never hold the GIL):
//   * synthetic: deterministic pseudo-random uint8 images + uniform labels per batch index
//     (BASELINE.json: synthetic data, no Herbarium images offline);
//   * window: image i of a manifest is the window of a shared uint8 texture at offs[i]
//     (data/manifest.SyntheticImages, bitwise), label labels[i]; batches 0..ceil(N/B)-1;
//   * external: Python (PIL decode threads) writes decoded images into a slot obtained
//     with acquire_empty() and hands it over with commit(id, batch_index, count).
//
// Markers: roctx ranges so rocprofv3 --marker-trace shows step phases.
#include "runtime.h"
#include "ring_core.h"

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
  int32_t* ext = nullptr;    // pinned [B,2] (h, w) of each image inside the pitch
};

static int checked_depth(int depth) {
  TORCH_CHECK(depth >= 2, "BatchRing depth must be >= 2");
  return depth;
}

// Torch-facing ring: pinned slot payloads + the producers' fill functions around the
// scheduling core (ring_core.h: slot states, batch-order hand-off, stop).
class BatchRing {
 public:
  BatchRing(int batch, int H, int W, int64_t num_classes, int depth, int threads, uint64_t seed,
            int64_t start_index, int64_t stride, bool synthetic)
      : B_(batch), H_(H), W_(W), nc_(num_classes), seed_(seed), synthetic_(synthetic),
        threads_(std::max(1, threads)),
        core_(checked_depth(depth), start_index, stride) {
    TORCH_CHECK(batch >= 1 && H >= 1 && W >= 1 && stride >= 1, "BatchRing: bad geometry");
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
      TORCH_CHECK(hipHostMalloc(&p, sizeof(int32_t) * 2 * B_, hipHostMallocDefault) == hipSuccess,
                  "hipHostMalloc failed");
      s.ext = (int32_t*)p;
    }
    if (synthetic_)
      core_.run_producers(threads_, [this](int id, int64_t b) { return fill_synthetic(id, b); });
  }

  ~BatchRing() { stop(); free_all(); }

  void stop() { core_.stop(); }

  // window mode: image i = tex[offs[i,0] : +H, offs[i,1] : +W], label labels[i]
  void set_window_source(torch::Tensor tex, torch::Tensor offs, torch::Tensor labels) {
    TORCH_CHECK(!synthetic_ && !core_.producing() && !window_, "BatchRing: source already set");
    TORCH_CHECK(tex.device().is_cpu() && tex.scalar_type() == torch::kUInt8 && tex.dim() == 3 &&
                    tex.size(2) == 3 && tex.is_contiguous(),
                "set_window_source: tex must be a contiguous CPU uint8 [TH, TW, 3]");
    TORCH_CHECK(offs.device().is_cpu() && offs.scalar_type() == torch::kInt64 && offs.dim() == 2 &&
                    offs.size(1) == 2 && offs.is_contiguous(),
                "set_window_source: offs must be CPU int64 [N, 2]");
    TORCH_CHECK(labels.device().is_cpu() && labels.scalar_type() == torch::kInt64 &&
                    labels.numel() == offs.size(0) && labels.is_contiguous(),
                "set_window_source: labels must be CPU int64 [N]");
    const int64_t TH = tex.size(0), TW = tex.size(1);
    auto o = offs.accessor<int64_t, 2>();
    for (int64_t i = 0; i < offs.size(0); ++i)  // every window inside the texture
      TORCH_CHECK(o[i][0] >= 0 && o[i][1] >= 0 && o[i][0] + H_ <= TH && o[i][1] + W_ <= TW,
                  "set_window_source: window ", i, " outside the texture");
    tex_ = tex;
    offs_ = offs;
    wlabels_ = labels;
    n_items_ = offs.size(0);
    window_ = true;
    core_.run_producers(threads_, [this](int id, int64_t b) { return fill_window(id, b); },
                        num_batches());
  }

  int64_t num_batches() const { return window_ ? (n_items_ + B_ - 1) / B_ : -1; }

  // consumer: block until the NEXT batch (in batch-index order) is filled; releases the GIL
  std::tuple<int, torch::Tensor, torch::Tensor, int64_t> acquire() {
    int id;
    {
      pybind11::gil_scoped_release nogil;
      id = core_.acquire();
    }
    TORCH_CHECK(id >= 0, "BatchRing stopped");
    return {id, view_img(id), view_labels(id), core_.batch_index(id)};
  }

  // (valid image count, pinned int32 [B,2] extents) of an acquired slot
  std::tuple<int, torch::Tensor> info(int id) {
    TORCH_CHECK(id >= 0 && id < (int)slots_.size(), "BatchRing: bad slot");
    auto opt = torch::TensorOptions().dtype(torch::kInt32).pinned_memory(true);
    return {core_.count(id), torch::from_blob(slots_[id].ext, {B_, 2}, opt)};
  }

  void release(int id) {
    TORCH_CHECK(id >= 0 && id < (int)slots_.size(), "BatchRing: bad slot");
    core_.release(id);
  }

  // external producer API (real-data mode): grab an empty slot, fill it, commit
  std::tuple<int, torch::Tensor, torch::Tensor, torch::Tensor> acquire_empty() {
    int id;
    {
      pybind11::gil_scoped_release nogil;
      id = core_.acquire_empty();
    }
    TORCH_CHECK(id >= 0, "BatchRing stopped");
    auto opt = torch::TensorOptions().dtype(torch::kInt32).pinned_memory(true);
    return {id, view_img(id), view_labels(id), torch::from_blob(slots_[id].ext, {B_, 2}, opt)};
  }

  void commit(int id, int64_t batch_index, int count) {
    TORCH_CHECK(id >= 0 && id < (int)slots_.size(), "BatchRing: bad slot");
    TORCH_CHECK(count >= 0 && count <= B_, "BatchRing: count outside [0, batch]");
    for (int b = 0; b < count; ++b)
      TORCH_CHECK(slots_[id].ext[2 * b] >= 1 && slots_[id].ext[2 * b] <= H_ &&
                      slots_[id].ext[2 * b + 1] >= 1 && slots_[id].ext[2 * b + 1] <= W_,
                  "BatchRing.commit: image ", b, " extent outside the slot pitch");
    core_.commit(id, batch_index, count);
  }

  int depth() const { return core_.depth(); }

  // consumer starvation counters (acquires, waits, blocked ms) since the last reset
  std::tuple<int64_t, int64_t, double> stats(bool reset) {
    int64_t v[3];
    core_.stats(v, reset);
    return {v[0], v[1], v[2] * 1e-6};
  }

 private:
  torch::Tensor view_img(int id) {
    auto opt = torch::TensorOptions().dtype(torch::kUInt8).pinned_memory(true);
    return torch::from_blob(slots_[id].img, {B_, H_, W_, 3}, opt);
  }
  torch::Tensor view_labels(int id) {
    auto opt = torch::TensorOptions().dtype(torch::kInt64).pinned_memory(true);
    return torch::from_blob(slots_[id].labels, {B_}, opt);
  }

  void full_extents(Slot& s) {
    for (int b = 0; b < B_; ++b) {
      s.ext[2 * b] = H_;
      s.ext[2 * b + 1] = W_;
    }
  }

  int fill_synthetic(int id, int64_t bidx) {
    Slot& s = slots_[id];
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
    full_extents(s);
    return B_;
  }

  int fill_window(int id, int64_t bidx) {
    Slot& s = slots_[id];
    const int64_t i0 = bidx * B_;
    const int n = (int)std::min<int64_t>(B_, n_items_ - i0);
    const uint8_t* tex = tex_.data_ptr<uint8_t>();
    const int64_t TW = tex_.size(1);
    const int64_t* off = offs_.data_ptr<int64_t>();
    const int64_t* lab = wlabels_.data_ptr<int64_t>();
    const size_t row = (size_t)W_ * 3;
    for (int b = 0; b < n; ++b) {
      const int64_t r0 = off[2 * (i0 + b)], c0 = off[2 * (i0 + b) + 1];
      uint8_t* dst = s.img + (size_t)b * H_ * row;
      for (int y = 0; y < H_; ++y)
        std::memcpy(dst + (size_t)y * row, tex + ((r0 + y) * TW + c0) * 3, row);
      s.labels[b] = lab[i0 + b];
    }
    full_extents(s);
    return n;
  }

  void free_all() {
    for (auto& s : slots_) {
      if (s.img) (void)hipHostFree(s.img);
      if (s.labels) (void)hipHostFree(s.labels);
      if (s.ext) (void)hipHostFree(s.ext);
      s.img = nullptr;
      s.labels = nullptr;
      s.ext = nullptr;
    }
  }

  int B_, H_, W_;
  int64_t nc_;
  uint64_t seed_;
  bool synthetic_;
  int threads_;
  bool window_ = false;
  torch::Tensor tex_, offs_, wlabels_;
  int64_t n_items_ = 0;
  std::vector<Slot> slots_;
  RingCore core_;  // last: its producer threads stop (destructor) before the slots go
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
      .def("commit", &BatchRing::commit, pybind11::arg("id"), pybind11::arg("batch_index"),
           pybind11::arg("count"))
      .def("info", &BatchRing::info)
      .def("set_window_source", &BatchRing::set_window_source)
      .def("num_batches", &BatchRing::num_batches)
      .def("stop", &BatchRing::stop)
      .def("depth", &BatchRing::depth)
      .def("stats", &BatchRing::stats, pybind11::arg("reset") = true);
  m.def("range_push", [](const std::string& s) { return roctxRangePushA(s.c_str()); });
  m.def("range_pop", []() { return roctxRangePop(); });
  m.def("mark", [](const std::string& s) { roctxMarkA(s.c_str()); });
}

}  // namespace mpa_runtime
