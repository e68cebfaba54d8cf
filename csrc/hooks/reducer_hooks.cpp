// Native gradient-readiness hooks for the bucketed reducers (parallel/ddp.py, parallel/zero.py).
//
// torch's DDP runs a C++ Reducer -- a post hook on every parameter's AccumulateGrad node
// (torch/csrc/distributed/c10d/reducer.cpp: grad_accumulator->add_post_hook) -- so a backward makes no
// Python call per parameter.  This module does the same for our engines: one C++ post hook per parameter
// counts readiness per bucket and releases buckets strictly in plan order (identical collective order on
// every rank even when autograd finishes parameters in a different order); Python is entered only when
// a bucket becomes ready (and once per backward to queue the end-of-backward callback).  SwinIR-S has 330
// parameters in ~10 buckets: 330 Python hook calls per backward become ~11.
//
// The AccumulateGrad nodes are held by shared_ptr here: a leaf keeps only a weak reference to its
// accumulator, so an accumulator nobody holds is rebuilt on the next forward and would lose the hook.
#include <torch/extension.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/utils/lambda_post_hook.h>
#include <torch/csrc/autograd/variable.h>

#include <memory>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace py = pybind11;
using torch::autograd::Node;
using torch::autograd::variable_list;

namespace {

class BucketReadiness : public std::enable_shared_from_this<BucketReadiness> {
 public:
  BucketReadiness(const std::vector<std::vector<int>>& buckets, int nparams, py::object on_first, py::object on_ready)
      : param_bucket_(nparams, -1), pending_init_(buckets.size()), on_first_(std::move(on_first)),
        on_ready_(std::move(on_ready)) {
    for (size_t b = 0; b < buckets.size(); ++b) {
      for (int p : buckets[b]) {
        if (p < 0 || p >= nparams) throw std::out_of_range("BucketReadiness: parameter index out of range");
        if (param_bucket_[p] >= 0) throw std::invalid_argument("BucketReadiness: parameter in two buckets");
        param_bucket_[p] = (int)b;
      }
      pending_init_[b] = (int)buckets[b].size();
    }
    reset();
  }

  // The last owner can be a hook lambda's temporary on the autograd thread (Python dropped the engine while a
  // backward was in flight): release the Python callables under the GIL, never without it.
  ~BucketReadiness() {
    if (!Py_IsInitialized()) {
      on_first_.release();   // interpreter gone: leak rather than touch its heap
      on_ready_.release();
      return;
    }
    py::gil_scoped_acquire gil;
    on_first_ = py::object();
    on_ready_ = py::object();
  }

  // attach to parameter i's gradient accumulator (params that do not require grad get none)
  void attach(const std::vector<at::Tensor>& params) {
    if ((int)params.size() != (int)param_bucket_.size())
      throw std::invalid_argument("BucketReadiness.attach: parameter count differs from the plan");
    std::weak_ptr<BucketReadiness> self = shared_from_this();
    for (size_t i = 0; i < params.size(); ++i) {
      if (!params[i].requires_grad()) continue;
      auto acc = torch::autograd::impl::grad_accumulator(params[i]);
      if (!acc) continue;
      const int idx = (int)i;
      const uintptr_t key = acc->add_post_hook(std::make_unique<torch::autograd::utils::LambdaPostHook>(
          [self, idx](const variable_list& outputs, const variable_list& /*inputs*/) {
            if (auto s = self.lock()) s->mark(idx);
            return outputs;
          }));
      accumulators_.push_back(std::move(acc));
      keys_.push_back(key);
    }
  }

  // remove every hook this object attached (an engine re-planning its buckets attaches a new object)
  void detach() {
    for (size_t i = 0; i < accumulators_.size(); ++i) accumulators_[i]->del_post_hook(keys_[i]);
    accumulators_.clear();
    keys_.clear();
  }

  void set_enabled(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    enabled_ = on;
  }
  bool enabled() const {
    std::lock_guard<std::mutex> g(mu_);
    return enabled_;
  }

  // buckets not yet released (parameters that got no gradient), in plan order; marks them released
  std::vector<int> flush() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int> out;
    while (next_ < (int)pending_.size()) out.push_back(next_++);
    return out;
  }

  void reset() {
    std::lock_guard<std::mutex> g(mu_);
    pending_ = pending_init_;
    seen_.assign(param_bucket_.size(), 0);
    next_ = 0;
    ready_ = 0;
  }

  int ready_count() const {
    std::lock_guard<std::mutex> g(mu_);
    return ready_;
  }
  bool all_released() const {
    std::lock_guard<std::mutex> g(mu_);
    return next_ == (int)pending_.size();
  }
  int hooks() const { return (int)accumulators_.size(); }

 private:
  void mark(int i) {
    std::vector<int> launch;
    bool first = false;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!enabled_) return;
      const int b = param_bucket_[i];
      if (b < 0) return;
      if (seen_[i]) throw std::runtime_error("BucketReadiness: parameter ready twice in one backward (reentrant "
                                             "backward or a parameter used by two engines)");
      seen_[i] = 1;
      first = ready_++ == 0;
      if (--pending_[b] == 0)
        while (next_ < (int)pending_.size() && pending_[next_] == 0) launch.push_back(next_++);
    }
    if (!first && launch.empty()) return;
    py::gil_scoped_acquire gil;
    if (first) on_first_();
    for (int b : launch) on_ready_(b);
  }

  mutable std::mutex mu_;
  std::vector<int> param_bucket_, pending_init_, pending_, seen_;
  int next_ = 0, ready_ = 0;
  bool enabled_ = true;
  py::object on_first_, on_ready_;
  std::vector<std::shared_ptr<Node>> accumulators_;
  std::vector<uintptr_t> keys_;
};

}  // namespace

PYBIND11_MODULE(_pdt_hooks, m) {
  m.doc() = "C++ AccumulateGrad post hooks with bucket-granular readiness for the reducers";
  py::class_<BucketReadiness, std::shared_ptr<BucketReadiness>>(m, "BucketReadiness")
      .def(py::init<const std::vector<std::vector<int>>&, int, py::object, py::object>(), py::arg("buckets"),
           py::arg("nparams"), py::arg("on_first"), py::arg("on_ready"))
      .def("attach", &BucketReadiness::attach)
      .def("detach", &BucketReadiness::detach)
      .def("set_enabled", &BucketReadiness::set_enabled)
      .def_property_readonly("enabled", &BucketReadiness::enabled)
      .def("flush", &BucketReadiness::flush)
      .def("reset", &BucketReadiness::reset)
      .def_property_readonly("ready_count", &BucketReadiness::ready_count)
      .def("all_released", &BucketReadiness::all_released)
      .def_property_readonly("hooks", &BucketReadiness::hooks);
}
