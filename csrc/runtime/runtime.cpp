// Host-side runtime of pytorch_distributedtraining_amd (pybind11 module `_pdt_runtime`).
//
// These are the planning / bookkeeping engines that sit on the hot path of every step but do not
// touch device memory themselves:
//
//  * BucketPlanner / ReadyTracker -- the DDP gradient bucketer (replaces torch's C++ Reducer used by
//    the reference's DDP path, Stoke-DDP.py:248 `distributed=ddp`; semantics of
//    torch/csrc/distributed/c10d/reducer.hpp:30-31 (first bucket / cap) and
//    torch/nn/parallel/distributed.py:1198-1229 (reverse-order assignment, rebuild from the observed
//    backward order)).  Bucket sizes are tuned for 7 xGMI links (bigger default cap than NCCL's 25 MiB).
//  * greedy_partition -- Fairscale OSS / ZeRO-1 parameter->rank assignment (Fairscale-DDP.py:86,
//    semantics of torch/distributed/optim/zero_redundancy_optimizer.py:680-700).
//  * FlatLayout -- FSDP / ZeRO-2/3 flat-parameter layout: aligned offsets, padding to a multiple of
//    world_size, per-rank shard ranges and per-parameter shard intersections
//    (torch/distributed/fsdp/_flat_param.py:1091-1160 semantics, re-derived for 288 GB HBM3E shards).
//  * CollectiveTracer -- per-rank collective sequence numbers + rolling shape hash used by the
//    debug-mode cross-rank consistency check.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

namespace py = pybind11;

namespace {

int64_t align_up(int64_t x, int64_t a) { return a <= 1 ? x : (x + a - 1) / a * a; }

// ------------------------------------------------------------------------------------------------
// Bucket planning
// ------------------------------------------------------------------------------------------------
struct Bucket {
  std::vector<int> params;        // parameter indices in bucket order
  std::vector<int64_t> offsets;   // element offsets of each param inside the flat bucket
  int64_t numel = 0;              // padded element count
  int64_t bytes = 0;
};

class BucketPlanner {
 public:
  // numels/elem_sizes/dtypes indexed by parameter index; params in different dtypes never share a
  // bucket.  align_elems pads every param start (16-B alignment for vector kernels).
  BucketPlanner(std::vector<int64_t> numels, std::vector<int> elem_sizes, std::vector<int> dtypes,
                int64_t first_bucket_bytes, int64_t bucket_cap_bytes, int64_t align_elems)
      : numels_(std::move(numels)),
        elem_sizes_(std::move(elem_sizes)),
        dtypes_(std::move(dtypes)),
        first_(first_bucket_bytes),
        cap_(bucket_cap_bytes),
        align_(align_elems) {
    if (numels_.size() != elem_sizes_.size() || numels_.size() != dtypes_.size())
      throw std::invalid_argument("BucketPlanner: size mismatch");
  }

  // Plan in the given order (the order gradients are expected to become ready).
  std::vector<Bucket> plan(const std::vector<int>& order) const {
    std::vector<Bucket> out;
    // one open bucket per dtype
    std::vector<std::pair<int, Bucket>> open;
    bool first_done = false;
    auto limit = [&]() { return first_done ? cap_ : first_; };
    for (int idx : order) {
      if (idx < 0 || idx >= (int)numels_.size()) throw std::out_of_range("BucketPlanner: bad index");
      const int dt = dtypes_[idx];
      auto it = std::find_if(open.begin(), open.end(), [&](const std::pair<int, Bucket>& p) { return p.first == dt; });
      if (it == open.end()) {
        open.emplace_back(dt, Bucket{});
        it = open.end() - 1;
      }
      Bucket& b = it->second;
      const int64_t off = align_up(b.numel, align_);
      b.params.push_back(idx);
      b.offsets.push_back(off);
      b.numel = off + numels_[idx];
      b.bytes = b.numel * elem_sizes_[idx];
      if (b.bytes >= limit()) {
        b.numel = align_up(b.numel, align_);
        out.push_back(std::move(b));
        open.erase(it);
        first_done = true;
      }
    }
    for (auto& p : open) {
      p.second.numel = align_up(p.second.numel, align_);
      out.push_back(std::move(p.second));
    }
    return out;
  }

  // DDP default: reverse registration order (gradients of the last layers arrive first)
  std::vector<Bucket> plan_default() const {
    std::vector<int> order(numels_.size());
    std::iota(order.begin(), order.end(), 0);
    std::reverse(order.begin(), order.end());
    return plan(order);
  }

 private:
  std::vector<int64_t> numels_;
  std::vector<int> elem_sizes_;
  std::vector<int> dtypes_;
  int64_t first_, cap_, align_;
};

// Tracks readiness of parameters inside buckets during one backward pass.  mark_ready returns the
// list of buckets that became complete *in launch order*: a bucket is released only once every
// earlier bucket has been released (keeps the collective order identical on every rank even if
// autograd fires hooks in a different order on different ranks).
class ReadyTracker {
 public:
  explicit ReadyTracker(const std::vector<std::vector<int>>& bucket_params, int nparams)
      : param_bucket_(nparams, -1), pending_init_(bucket_params.size()) {
    for (size_t b = 0; b < bucket_params.size(); ++b) {
      for (int p : bucket_params[b]) {
        if (p < 0 || p >= nparams) throw std::out_of_range("ReadyTracker: bad param");
        param_bucket_[p] = (int)b;
      }
      pending_init_[b] = (int)bucket_params[b].size();
    }
    reset();
  }
  void reset() {
    pending_ = pending_init_;
    seen_.assign(param_bucket_.size(), 0);
    next_launch_ = 0;
    ready_count_ = 0;
  }
  std::vector<int> mark_ready(int p) {
    std::vector<int> launch;
    if (p < 0 || p >= (int)param_bucket_.size()) throw std::out_of_range("ReadyTracker: bad param");
    const int b = param_bucket_[p];
    if (b < 0) return launch;
    if (seen_[p]) throw std::runtime_error("ReadyTracker: parameter marked ready twice in one backward "
                                           "(reentrant backward or shared parameter without find_unused)");
    seen_[p] = 1;
    ++ready_count_;
    if (--pending_[b] == 0) {
      while (next_launch_ < (int)pending_.size() && pending_[next_launch_] == 0) launch.push_back(next_launch_++);
    }
    return launch;
  }
  // buckets not yet launched (unused parameters): force-release in order
  std::vector<int> flush() {
    std::vector<int> launch;
    while (next_launch_ < (int)pending_.size()) launch.push_back(next_launch_++);
    return launch;
  }
  std::vector<int> unready_params() const {
    std::vector<int> r;
    for (size_t i = 0; i < seen_.size(); ++i)
      if (!seen_[i] && param_bucket_[i] >= 0) r.push_back((int)i);
    return r;
  }
  int ready_count() const { return ready_count_; }
  bool all_launched() const { return next_launch_ == (int)pending_.size(); }

 private:
  std::vector<int> param_bucket_;
  std::vector<int> pending_init_, pending_;
  std::vector<char> seen_;
  int next_launch_ = 0;
  int ready_count_ = 0;
};

// ------------------------------------------------------------------------------------------------
// ZeRO-1 greedy partition: sort by numel descending (stable), give each to the least-loaded rank.
// Returns rank id per parameter.
// ------------------------------------------------------------------------------------------------
std::vector<int> greedy_partition(const std::vector<int64_t>& numels, int world) {
  if (world <= 0) throw std::invalid_argument("world must be > 0");
  std::vector<int> order(numels.size());
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return numels[a] > numels[b]; });
  std::vector<int64_t> load(world, 0);
  std::vector<int> owner(numels.size(), 0);
  for (int idx : order) {
    int best = 0;
    for (int r = 1; r < world; ++r)
      if (load[r] < load[best]) best = r;
    owner[idx] = best;
    load[best] += numels[idx];
  }
  return owner;
}

// ------------------------------------------------------------------------------------------------
// Flat-parameter layout for sharded engines.
// ------------------------------------------------------------------------------------------------
struct ShardPiece {     // intersection of one parameter with this rank's shard
  int param;
  int64_t param_offset;  // offset inside the parameter (elements)
  int64_t shard_offset;  // offset inside the local shard
  int64_t numel;
};

class FlatLayout {
 public:
  FlatLayout(std::vector<int64_t> numels, int world, int64_t align_elems)
      : numels_(std::move(numels)), world_(world), align_(align_elems) {
    if (world_ <= 0) throw std::invalid_argument("world must be > 0");
    int64_t off = 0;
    for (int64_t n : numels_) {
      off = align_up(off, align_);
      offsets_.push_back(off);
      off += n;
    }
    unpadded_ = off;
    // every shard is a multiple of align so each rank's shard start stays 16-B aligned
    total_ = align_up(std::max<int64_t>(off, 1), (int64_t)world_ * std::max<int64_t>(align_, 1));
    shard_ = total_ / world_;
  }
  int64_t total() const { return total_; }
  int64_t unpadded() const { return unpadded_; }
  int64_t shard_numel() const { return shard_; }
  const std::vector<int64_t>& offsets() const { return offsets_; }
  std::pair<int64_t, int64_t> shard_range(int rank) const { return {rank * shard_, (rank + 1) * shard_}; }
  std::vector<ShardPiece> pieces(int rank) const {
    std::vector<ShardPiece> r;
    const int64_t s0 = rank * shard_, s1 = s0 + shard_;
    for (size_t i = 0; i < numels_.size(); ++i) {
      const int64_t p0 = offsets_[i], p1 = p0 + numels_[i];
      const int64_t a = std::max(p0, s0), b = std::min(p1, s1);
      if (a < b) r.push_back(ShardPiece{(int)i, a - p0, a - s0, b - a});
    }
    return r;
  }

 private:
  std::vector<int64_t> numels_;
  std::vector<int64_t> offsets_;
  int world_;
  int64_t align_;
  int64_t unpadded_ = 0, total_ = 0, shard_ = 0;
};

// ------------------------------------------------------------------------------------------------
// ZeRO-1 / ZeRO-2 owner-contiguous layout (parallel/zero.py).  Each owner's parameters (greedy partition)
// are packed into ONE segment and every segment is padded to a common length, so
//   * the post-step parameter exchange is ONE all-gather of [seg_0 | seg_1 | ... ] (not world broadcasts),
//   * a rank's optimizer state, fp32 master and (ZeRO-2) gradient are one contiguous slice,
// and inside a segment parameters run in DESCENDING index order (~ the order backward produces their
// gradients), so the reduction buckets -- windows of <= cap elements of one segment -- fill in order.
// Buckets are returned in launch order: descending smallest parameter index (the bucket whose last
// gradient arrives first is released first).
// ------------------------------------------------------------------------------------------------
struct ZeroBucket {
  int owner;
  int64_t start;   // absolute element offset in the flat buffer
  int64_t numel;
  std::vector<int> params;
};

class ZeroLayout {
 public:
  ZeroLayout(std::vector<int64_t> numels, std::vector<int> owners, int world, int64_t align, int64_t cap)
      : offsets_(numels.size(), 0), world_(world) {
    if (world <= 0) throw std::invalid_argument("ZeroLayout: world must be > 0");
    if (owners.size() != numels.size()) throw std::invalid_argument("ZeroLayout: owners/numels size mismatch");
    if (align < 1) align = 1;
    if (cap < 1) cap = 1;
    std::vector<std::vector<int>> mine(world);
    for (int i = (int)numels.size() - 1; i >= 0; --i) {
      if (owners[i] < 0 || owners[i] >= world) throw std::out_of_range("ZeroLayout: bad owner");
      mine[owners[i]].push_back(i);
    }
    std::vector<int64_t> used(world, 0);
    std::vector<std::vector<int64_t>> local(world);
    for (int r = 0; r < world; ++r) {
      int64_t off = 0;
      for (int i : mine[r]) {
        off = align_up(off, align);
        local[r].push_back(off);
        off += numels[i];
      }
      used[r] = off;
    }
    seg_ = align_up(std::max<int64_t>(1, *std::max_element(used.begin(), used.end())), align);
    for (int r = 0; r < world; ++r) {
      ZeroBucket cur{r, -1, 0, {}};
      int64_t end = 0;
      for (size_t k = 0; k < mine[r].size(); ++k) {
        const int i = mine[r][k];
        const int64_t abs = (int64_t)r * seg_ + local[r][k];
        offsets_[i] = abs;
        if (cur.start >= 0 && abs + numels[i] - cur.start > cap) {
          cur.numel = align_up(end, align) - cur.start;   // whole 16-element granules (16-B collectives)
          buckets_.push_back(cur);
          cur = ZeroBucket{r, -1, 0, {}};
        }
        if (cur.start < 0) cur.start = abs;
        cur.params.push_back(i);
        end = abs + numels[i];
      }
      if (cur.start >= 0) {
        cur.numel = align_up(end, align) - cur.start;
        buckets_.push_back(cur);
      }
    }
    std::stable_sort(buckets_.begin(), buckets_.end(), [](const ZeroBucket& a, const ZeroBucket& b) {
      return *std::min_element(a.params.begin(), a.params.end()) > *std::min_element(b.params.begin(), b.params.end());
    });
  }
  int64_t seg() const { return seg_; }
  int64_t total() const { return seg_ * world_; }
  const std::vector<int64_t>& offsets() const { return offsets_; }
  const std::vector<ZeroBucket>& buckets() const { return buckets_; }

 private:
  std::vector<int64_t> offsets_;
  std::vector<ZeroBucket> buckets_;
  int world_;
  int64_t seg_ = 0;
};

// ------------------------------------------------------------------------------------------------
// Collective tracer (debug consistency checking across ranks).
// ------------------------------------------------------------------------------------------------
class CollectiveTracer {
 public:
  explicit CollectiveTracer(size_t capacity) : cap_(capacity ? capacity : 1) {}
  // returns the sequence number assigned to this collective
  uint64_t record(const std::string& op, const std::vector<int64_t>& shape, int dtype) {
    std::lock_guard<std::mutex> g(mu_);
    uint64_t h = 1469598103934665603ull;  // FNV-1a
    auto mix = [&](uint64_t v) {
      for (int i = 0; i < 8; ++i) {
        h ^= (v >> (8 * i)) & 0xff;
        h *= 1099511628211ull;
      }
    };
    for (char c : op) mix((uint64_t)(unsigned char)c);
    for (int64_t s : shape) mix((uint64_t)s);
    mix((uint64_t)dtype);
    rolling_ = rolling_ * 1099511628211ull ^ h;
    const uint64_t seq = seq_++;
    if (log_.size() < cap_) log_.emplace_back(seq, op, h);
    else log_[seq % cap_] = std::make_tuple(seq, op, h);
    return seq;
  }
  uint64_t seq() const { return seq_; }
  uint64_t rolling_hash() const { return rolling_; }
  std::vector<std::tuple<uint64_t, std::string, uint64_t>> recent() const {
    std::lock_guard<std::mutex> g(mu_);
    auto r = log_;
    std::sort(r.begin(), r.end());
    return r;
  }
  void reset() {
    std::lock_guard<std::mutex> g(mu_);
    seq_ = 0;
    rolling_ = 0;
    log_.clear();
  }

 private:
  size_t cap_;
  mutable std::mutex mu_;
  uint64_t seq_ = 0, rolling_ = 0;
  std::vector<std::tuple<uint64_t, std::string, uint64_t>> log_;
};

}  // namespace

PYBIND11_MODULE(_pdt_runtime, m) {
  m.doc() = "pytorch_distributedtraining_amd host runtime (bucket planner, shard planners, tracer)";

  py::class_<Bucket>(m, "Bucket")
      .def_readonly("params", &Bucket::params)
      .def_readonly("offsets", &Bucket::offsets)
      .def_readonly("numel", &Bucket::numel)
      .def_readonly("bytes", &Bucket::bytes);

  py::class_<BucketPlanner>(m, "BucketPlanner")
      .def(py::init<std::vector<int64_t>, std::vector<int>, std::vector<int>, int64_t, int64_t, int64_t>(),
           py::arg("numels"), py::arg("elem_sizes"), py::arg("dtypes"), py::arg("first_bucket_bytes"),
           py::arg("bucket_cap_bytes"), py::arg("align_elems") = 8)
      .def("plan", &BucketPlanner::plan, py::arg("order"))
      .def("plan_default", &BucketPlanner::plan_default);

  py::class_<ReadyTracker>(m, "ReadyTracker")
      .def(py::init<const std::vector<std::vector<int>>&, int>())
      .def("reset", &ReadyTracker::reset)
      .def("mark_ready", &ReadyTracker::mark_ready)
      .def("flush", &ReadyTracker::flush)
      .def("unready_params", &ReadyTracker::unready_params)
      .def("ready_count", &ReadyTracker::ready_count)
      .def("all_launched", &ReadyTracker::all_launched);

  m.def("greedy_partition", &greedy_partition, py::arg("numels"), py::arg("world"));

  py::class_<ShardPiece>(m, "ShardPiece")
      .def_readonly("param", &ShardPiece::param)
      .def_readonly("param_offset", &ShardPiece::param_offset)
      .def_readonly("shard_offset", &ShardPiece::shard_offset)
      .def_readonly("numel", &ShardPiece::numel);

  py::class_<FlatLayout>(m, "FlatLayout")
      .def(py::init<std::vector<int64_t>, int, int64_t>(), py::arg("numels"), py::arg("world"),
           py::arg("align_elems") = 8)
      .def_property_readonly("total", &FlatLayout::total)
      .def_property_readonly("unpadded", &FlatLayout::unpadded)
      .def_property_readonly("shard_numel", &FlatLayout::shard_numel)
      .def_property_readonly("offsets", &FlatLayout::offsets)
      .def("shard_range", &FlatLayout::shard_range)
      .def("pieces", &FlatLayout::pieces);

  py::class_<ZeroBucket>(m, "ZeroBucket")
      .def_readonly("owner", &ZeroBucket::owner)
      .def_readonly("start", &ZeroBucket::start)
      .def_readonly("numel", &ZeroBucket::numel)
      .def_readonly("params", &ZeroBucket::params);

  py::class_<ZeroLayout>(m, "ZeroLayout")
      .def(py::init<std::vector<int64_t>, std::vector<int>, int, int64_t, int64_t>(), py::arg("numels"),
           py::arg("owners"), py::arg("world"), py::arg("align"), py::arg("bucket_cap"))
      .def_property_readonly("seg", &ZeroLayout::seg)
      .def_property_readonly("total", &ZeroLayout::total)
      .def_property_readonly("offsets", &ZeroLayout::offsets)
      .def_property_readonly("buckets", &ZeroLayout::buckets);

  py::class_<CollectiveTracer>(m, "CollectiveTracer")
      .def(py::init<size_t>(), py::arg("capacity") = 4096)
      .def("record", &CollectiveTracer::record)
      .def_property_readonly("seq", &CollectiveTracer::seq)
      .def_property_readonly("rolling_hash", &CollectiveTracer::rolling_hash)
      .def("recent", &CollectiveTracer::recent)
      .def("reset", &CollectiveTracer::reset);
}
