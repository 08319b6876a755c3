// _gshook: the per-parameter gradient hook of the libgsync DDP in C++.
//
// torch's Reducer registers a C++ post-hook on every parameter's
// AccumulateGrad node (T:include/torch/csrc/distributed/c10d/reducer.hpp:73,
// reducer.cpp autograd_hook); the libgsync DDP did the same from Python
// (register_post_accumulate_grad_hook -> closure -> ctypes
// gs_bucketer_mark_ready), which costs a GIL acquisition and a Python frame per
// gradient on the autograd thread.  Here the hook is a FunctionPostHook on the
// AccumulateGrad node that calls gs_bucketer_mark_ready directly (the bucket's
// pack + RCCL collective are enqueued inside that call, GS_BKT_AUTO_COLLECTIVE),
// and the end-of-backward callback calls gs_bucketer_finalize, then hands back
// to Python once per backward for the bookkeeping the Python DDP keeps.
//
// Used only on the fast path (device buckets, library collective, no comm hook,
// no find_unused_parameters, no overlapped optimizer, no parity capture); the
// Python hooks serve every other configuration (ddp.py decides per forward).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/function_hook.h>
#include <torch/csrc/autograd/variable.h>
#include <torch/csrc/utils/pybind.h>

#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/hip/HIPStream.h>

#include <algorithm>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/gsync.h"

namespace py = pybind11;
using torch::autograd::Node;
using torch::autograd::variable_list;

namespace {

// grad's memory is one dense block in param's element order
// (multi_tensor.dense_like_param)
bool dense_like(const at::Tensor& g, const at::Tensor& p) {
  if (!g.sizes().equals(p.sizes()) || !g.strides().equals(p.strides())) return false;
  if (g.is_contiguous()) return true;
  std::vector<std::pair<int64_t, int64_t>> dims;
  for (int64_t d = 0; d < g.dim(); ++d)
    if (g.size(d) != 1) dims.emplace_back(g.stride(d), g.size(d));
  std::sort(dims.begin(), dims.end());
  int64_t expected = 1;
  for (auto& [st, sz] : dims) {
    if (st != expected) return false;
    expected *= sz;
  }
  return true;
}

class Hooks;

struct MarkReady : torch::autograd::FunctionPostHook {
  Hooks* owner;
  int index;
  MarkReady(Hooks* o, int i) : owner(o), index(i) {}
  variable_list operator()(const variable_list& outputs, const variable_list& inputs) override;
};

class Hooks : public std::enable_shared_from_this<Hooks> {
 public:
  // constructed from Python (GIL held): the callable is kept as a plain
  // reference, so the destructor never needs pybind11's GIL machinery
  // release: the ZeRO engine's mode — a grad is released from its parameter
  // once marked ready (DeepSpeed frees it too) and held until its bucket's
  // pack is enqueued, then recorded on the comm stream for the allocator
  Hooks(std::vector<at::Tensor> params, int device, py::function on_finalize, bool release)
      : params_(std::move(params)), device_(device), on_finalize_(on_finalize.release().ptr()), release_(release) {
    dense_strides_.resize(params_.size());
    dense_seen_.assign(params_.size(), 0);
    accs_.resize(params_.size());
    keys_.assign(params_.size(), 0);
  }
  ~Hooks() {
    detach();
    // the last reference may go on the autograd thread (the queued callback's
    // copy) or during interpreter teardown: drop the callable only when this
    // thread holds the GIL, else leave it (one small object)
    if (on_finalize_ && Py_IsInitialized() && PyGILState_Check()) Py_DECREF(on_finalize_);
  }

  // The hooks are armed per synchronising step (arm(), from prepare()), never
  // on nodes pinned at wrap time: an AccumulateGrad runs on the stream that was
  // current when it was created, so a node pinned at wrap time would
  // accumulate on that stream even inside a later hipGraph capture on another
  // one.  attach() / detach() switch the arming on and off.
  void attach() { active_ = true; }

  void detach() {
    active_ = false;
    pinned_.clear();
    for (size_t i = 0; i < accs_.size(); ++i) {
      if (auto a = accs_[i].lock()) a->del_post_hook(keys_[i]);
      accs_[i].reset();
    }
  }

  bool attached() const { return active_; }

  // bucket_of: each parameter's bucket (release mode); comm_stream: where the
  // library runs the packs (release mode: held grads are recorded on it)
  void set_bucketer(uintptr_t handle, int n_buckets, std::vector<int> bucket_of, uintptr_t comm_stream) {
    b_ = reinterpret_cast<gs_bucketer*>(handle);
    ready_.assign(static_cast<size_t>(std::max(1, n_buckets)), 0);  // mark_ready's ready-bucket list
    bucket_of_ = std::move(bucket_of);
    held_.assign(static_cast<size_t>(std::max(1, n_buckets)), {});
    comm_stream_ = reinterpret_cast<void*>(comm_stream);
    if (release_ && b_ != nullptr && bucket_of_.size() != params_.size())
      throw std::runtime_error("_gshook: release mode needs every parameter's bucket");
  }

  // forward of a synchronising step (ddp._prepare_for_backward): arms the hooks
  void prepare(bool record_order) {
    in_backward_ = true;
    finalize_queued_ = false;
    record_order_ = record_order;
    if (record_order) order_.clear();
    for (auto& h : held_) h.clear();  // nothing held past a backward that did not finish
    if (active_) arm();
  }

  // one post-hook on each parameter's AccumulateGrad: the node of the graph just
  // built (DDP arms after its forward), or — armed before the forward, as the
  // ZeRO engine's prepare_backward is — a node created now, on the current
  // stream, that the coming forward adopts (the variable holds its node weakly:
  // it is pinned here until finalize).  A node that outlived its graph
  // (retain_graph) keeps its one hook.
  void arm() {
    pinned_.clear();
    for (size_t i = 0; i < params_.size(); ++i) {
      auto a = torch::autograd::impl::grad_accumulator(params_[i]);
      if (!a) continue;
      pinned_.push_back(a);
      if (accs_[i].lock() == a) continue;
      keys_[i] = a->add_post_hook(std::make_unique<MarkReady>(this, static_cast<int>(i)));
      accs_[i] = a;
    }
  }

  void on_grad(int i) {
    if (!in_backward_) return;  // no_sync: accumulate only
    if (b_ == nullptr) throw std::runtime_error("_gshook: the DDP's bucketer is closed");
    if (!finalize_queued_) {
      finalize_queued_ = true;
      // device < 0: host buckets (the CPU test of this hook), no stream
      stream_ = device_ < 0 ? nullptr
                            : c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(device_)).stream();
      auto self = shared_from_this();
      torch::autograd::Engine::get_default_engine().queue_callback([self] { self->finalize(); });
    }
    if (record_order_) order_.push_back(i);
    const at::Tensor& p = params_[i];
    if (release_) return on_grad_release(i, p);
    at::Tensor& g = p.mutable_grad();
    if (!g.defined()) throw std::runtime_error("_gshook: gradient hook fired without a gradient");
    // fast path: strides of a parameter already seen dense (grads in that layout are too)
    if (!dense_seen_[i] || !g.strides().equals(dense_strides_[i])) {
      if (!dense_like(g, p)) {
        at::Tensor dense = at::empty_like(p);
        dense.copy_(g);
        g = dense;
      } else if (dense_like(p, p)) {
        dense_seen_[i] = 1;
        dense_strides_[i] = p.strides().vec();
      }
    }
    int32_t n_ready = 0;
    const int rc = gs_bucketer_mark_ready(b_, i, g.data_ptr(), stream_, ready_.data(), &n_ready);
    if (rc < 0) throw std::runtime_error(std::string("gs_bucketer_mark_ready: ") + gs_last_error());
  }

  void on_grad_release(int i, const at::Tensor& p) {
    at::Tensor g = p.grad();
    if (!g.defined()) throw std::runtime_error("_gshook: gradient hook fired without a gradient");
    if (!dense_like(g, p)) {
      at::Tensor dense = at::empty_like(p);
      dense.copy_(g);
      g = dense;
    }
    const int bk = bucket_of_[i];
    held_[bk].push_back(g);
    p.mutable_grad() = at::Tensor();  // released: the bucket holds the data from here on
    int32_t n_ready = 0;
    const int rc = gs_bucketer_mark_ready(b_, i, g.data_ptr(), stream_, ready_.data(), &n_ready);
    if (rc < 0) throw std::runtime_error(std::string("gs_bucketer_mark_ready: ") + gs_last_error());
    for (int k = 0; k < n_ready; ++k) {
      auto& hs = held_[ready_[k]];
      if (comm_stream_ != nullptr) {
        // the pack on the comm stream is enqueued: the allocator may reuse these
        // grads' memory only after it has run
        // torch-ROCm's device type for GPU tensors is "cuda": the stream must say so too
        const c10::Stream cs = c10::hip::getStreamFromExternalMasqueradingAsCUDA(
            static_cast<hipStream_t>(comm_stream_), static_cast<c10::DeviceIndex>(device_));
        for (auto& t : hs) t.record_stream(cs);
      }
      hs.clear();
    }
  }

  // static_graph DDP: a parameter the (fixed) graph never uses is marked ready at
  // the end of backward, as torch's static-graph Reducer does (ddp.py
  // _finalize_backward's static_graph branch); its slot reduces as zeros
  void set_mark_unused(bool on) { mark_unused_ = on; }

  void finalize() {
    if (mark_unused_) {
      int32_t n_ready = 0;
      const int ru = gs_bucketer_mark_unused(b_, stream_, ready_.data(), &n_ready);
      if (ru < 0) {
        in_backward_ = false;
        finalize_queued_ = false;
        pinned_.clear();
        throw std::runtime_error(std::string("gs_bucketer_mark_unused: ") + gs_last_error());
      }
    }
    const int rc = gs_bucketer_finalize(b_, stream_);
    in_backward_ = false;
    finalize_queued_ = false;
    pinned_.clear();
    if (rc < 0) throw std::runtime_error(std::string("gs_bucketer_finalize: ") + gs_last_error());
    // the Python DDP's bookkeeping (ddp._native_finalized), once per backward
    std::string err;
    const PyGILState_STATE st = PyGILState_Ensure();
    PyObject* r = PyObject_CallObject(on_finalize_, nullptr);
    if (r == nullptr) {
      PyObject *t, *v, *tb;
      PyErr_Fetch(&t, &v, &tb);
      PyObject* sv = v ? PyObject_Str(v) : nullptr;
      const char* msg = sv ? PyUnicode_AsUTF8(sv) : nullptr;
      err = msg ? msg : "error in the DDP finalize callback";
      Py_XDECREF(sv);
      Py_XDECREF(t);
      Py_XDECREF(v);
      Py_XDECREF(tb);
      PyErr_Clear();
    }
    Py_XDECREF(r);
    PyGILState_Release(st);
    if (!err.empty()) throw std::runtime_error(err);
  }

  std::vector<int> order() const { return order_; }
  bool in_backward() const { return in_backward_; }
  bool finalize_queued() const { return finalize_queued_; }
  uintptr_t stream() const { return reinterpret_cast<uintptr_t>(stream_); }

 private:
  std::vector<at::Tensor> params_;
  int device_;
  PyObject* on_finalize_;  // strong reference (see the constructor)
  std::vector<std::weak_ptr<Node>> accs_;  // the node each hook is on (owned by its graph)
  std::vector<std::shared_ptr<Node>> pinned_;  // armed nodes, held from arm() to finalize
  std::vector<uintptr_t> keys_;
  bool active_ = false;
  std::vector<std::vector<int64_t>> dense_strides_;
  std::vector<char> dense_seen_;
  gs_bucketer* b_ = nullptr;
  std::vector<int32_t> ready_;
  void* stream_ = nullptr;
  bool in_backward_ = false, finalize_queued_ = false, record_order_ = false;
  bool release_ = false;
  bool mark_unused_ = false;
  std::vector<int> bucket_of_;
  std::vector<std::vector<at::Tensor>> held_;
  void* comm_stream_ = nullptr;
  std::vector<int> order_;
};

variable_list MarkReady::operator()(const variable_list& outputs, const variable_list& /*inputs*/) {
  owner->on_grad(index);
  return outputs;
}

}  // namespace

PYBIND11_MODULE(_gshook, m) {
  m.doc() = "libgsync DDP gradient hooks in C++ (AccumulateGrad post-hooks -> gs_bucketer_mark_ready)";
  py::class_<Hooks, std::shared_ptr<Hooks>>(m, "Hooks")
      .def(py::init<std::vector<at::Tensor>, int, py::function, bool>(), py::arg("params"), py::arg("device"),
           py::arg("on_finalize"), py::arg("release") = false)
      .def("attach", &Hooks::attach)
      .def("detach", &Hooks::detach)
      .def("attached", &Hooks::attached)
      .def("set_bucketer", &Hooks::set_bucketer, py::arg("handle"), py::arg("n_buckets"),
           py::arg("bucket_of") = std::vector<int>(), py::arg("comm_stream") = 0)
      .def("set_mark_unused", &Hooks::set_mark_unused)
      .def("prepare", &Hooks::prepare)
      .def("order", &Hooks::order)
      .def("in_backward", &Hooks::in_backward)
      .def("finalize_queued", &Hooks::finalize_queued)
      .def("stream", &Hooks::stream);
}
