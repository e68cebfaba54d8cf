// Peer-to-peer xGMI collectives for one node of MI355X: every rank owns one
// symmetric buffer in HBM that the other ranks map with hipIpcOpenMemHandle, and the collectives are
// plain HIP kernels that READ peers' buffers directly over the xGMI mesh (7 links per GPU, all used at
// once) instead of a ring that drives one link per step.
//
//   symmetric buffer = [signal block 4 KB][staging slot 0][staging slot 1]
//   signal block     = uint32 sig[NBAR][MAXW] (sig[b][p] = last epoch peer p reached barrier b at) + error word
//
// Protocol per call (epoch e = host call counter, identical on every rank, never 0):
//   K1 copy-in   : the local input is stored into this rank's staging slot (e & 1), write-through at
//                  system scope (sc0 sc1), so no peer can read a stale line from any L2.  Every block then
//                  counts itself in (system-scope acq_rel counter); the LAST block alone signals barrier 0 to
//                  every peer (system-scope atomic store into the PEER's signal block), waits until every peer
//                  signalled it for epoch e, and publishes stat[0] = e in its own signal block.
//   K2.. phases  : every block reads stat[b] once (no spinning), then reads peers' slots with system-scope
//                  (cache-bypassing) loads, reduces in fp32 (fp64 for fp64) and writes the result; a phase that
//                  produces slot data for a later phase (two-shot) ends with the same last-block barrier.  At
//                  most ONE wave per rank spins on the mesh, so the collectives never hold CUs that the
//                  compute stream's GEMMs (one 512-register wave per SIMD) need.  Waits are bounded: on
//                  timeout the waiter records an error word, stat[b] stays stale and the payload is poisoned.
//   Slot reuse   : slot (e & 1) is rewritten at call e+2, whose copy-in runs after this rank's payload kernels
//                  of call e+1, which ran after barrier 0 of e+1 completed -- signalled by every peer only
//                  after its own call-e kernels (the last readers of our slot e & 1) finished.
//
// one-shot all-reduce (latency class: scalars, grad-norm, SyncBN stats): 2 kernels, every rank reads W
// slots.  two-shot all-reduce (bandwidth class): reduce-scatter phase (rank r reduces chunk r from all
// peers into its own slot) + all-gather phase (every rank reads chunk p from peer p): 2(W-1)/W of the
// payload crosses the fabric, spread over all 7 links.  all_gather / reduce_scatter: 2 kernels each.
//
// Every collective of a rank runs on that rank's dedicated communication stream (parallel/xgmi.py), so
// the per-rank kernel order -- which the slot-reuse argument above relies on -- is the issue order.
// Payloads larger than a slot are chunked by the host, one epoch per chunk; reduce-scatter inputs and
// all-gather outputs are addressed with a per-peer pitch so a chunk is a strided window of the tensor.
//
// A wait that exceeds the spin budget is an error, never a silent result: the block poisons its part
// of the output with NaN (all-ones bits, NaN in fp32 and bf16) instead of reading possibly stale peer
// slots, and sets the error word in device memory AND in a host-mapped word that the engines poll at
// their synchronisation points without a device sync (XGMIComm.raise_if_failed).
//
// The scalar data cache is never written: flags and payload use vector atomics / vector buffer stores.
#include "common.h"
#include <string.h>

using namespace pdt;

namespace {

constexpr int MAXW = 8;
constexpr int NBAR = 4;
constexpr int64_t SIG_BYTES = 4096;
constexpr int ERR_OFF = 1024;         // byte offset of the error word in the signal block
constexpr int CNT_OFF = 2048;         // uint32 [NBAR]: blocks of the current kernel that arrived (arrive())
constexpr int STAT_OFF = 3072;        // uint32 [NBAR]: epoch of the last call whose barrier b completed
constexpr int NT = 256;
constexpr int SYS = 1 | 16;           // buffer-op cache policy: sc0 | sc1 = system-scope coherent

struct XArgs {
  char* buf[MAXW];                    // symmetric buffer base of every rank (own + IPC-mapped peers)
  unsigned* host_err;                 // host-mapped error word (may be null)
  int rank, world;
  unsigned epoch;
  uint64_t timeout_ticks;             // wall-clock budget of one mesh wait, in s_memrealtime ticks
  int64_t slot_bytes;
};

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((address_space(1))) unsigned int gu32;

__device__ __forceinline__ char* slot_of(const XArgs& a, int p) {
  return a.buf[p] + SIG_BYTES + (int64_t)(a.epoch & 1u) * a.slot_bytes;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// Signal barrier `b` of epoch a.epoch to every peer, then wait for every peer's signal -- ONE workgroup (lanes
// t < world) per call: the last block of the kernel that produced this rank's slot data (arrive()), or the
// barrier kernel.  Success is published as stat[b] = epoch in the own signal block; the payload kernel that
// follows on the stream reads that word once per block (passed()) instead of spinning, so at most one wave
// per rank ever spins on the mesh and the rest of the GPU stays with the compute stream.
__device__ __forceinline__ void mesh_wait(const XArgs& a, int b) {
  __shared__ int timed_out;
  const int t = threadIdx.x;
  if (t == 0) timed_out = 0;
  __syncthreads();
  if (t < a.world) {
    gu32* remote = (gu32*)(a.buf[t]) + b * MAXW + a.rank;
    __hip_atomic_store(remote, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    gu32* mine = (gu32*)(a.buf[a.rank]) + b * MAXW + t;
    // wall-clock budget (s_memrealtime: 100 MHz): ranks that share a GPU time-slice its queues, and a rank
    // whose host is still in a first-call library load can arrive a second late -- an iteration count
    // mis-measures both
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t budget = a.timeout_ticks;
    unsigned spins = 0;
    unsigned seen;
    while ((int)((seen = __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) - a.epoch) < 0) {
      if ((++spins & 63) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > budget) {
        // give up: record the failure, never hang the queue
        __hip_atomic_fetch_or((gu32*)(a.buf[a.rank] + ERR_OFF), 1u << b, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_SYSTEM);
        if (a.host_err != nullptr) {  // plain system-scope stores (no PCIe atomics needed): any bit = failure
          // diagnosis words (last writer wins): the epoch waited for, barrier / late peer, the peer's last epoch
          __hip_atomic_store(a.host_err + 1, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(a.host_err + 2, (unsigned)(b << 8 | t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(a.host_err + 3, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(a.host_err, 0x100u | (1u << b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        atomicOr(&timed_out, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system-scope acquire (one lane per peer)
  }
  __syncthreads();
  if (t == 0)
    __hip_atomic_store((gu32*)(a.buf[a.rank] + STAT_OFF) + b, timed_out ? 0u : a.epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// End of a kernel whose blocks stored this rank's slot data: every block releases its stores and counts itself
// in; the last one to arrive runs the mesh wait for barrier `b` (and re-arms the counter for the next call).
__device__ __forceinline__ void arrive(const XArgs& a, int b) {
  __shared__ unsigned last;
  // every wave's slot stores acknowledged (a workgroup barrier alone does not wait for other waves' stores)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    gu32* cnt = (gu32*)(a.buf[a.rank] + CNT_OFF) + b;
    const unsigned n = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    last = n + 1 == gridDim.x;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (last) mesh_wait(a, b);
}

// did barrier `b` of this call complete (published by the previous kernel on this stream)?
__device__ __forceinline__ bool passed(const XArgs& a, int b) {
  __shared__ int ok;
  if (threadIdx.x == 0)
    ok = __hip_atomic_load((gu32*)(a.buf[a.rank] + STAT_OFF) + b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) ==
         a.epoch;
  __syncthreads();
  return ok != 0;
}

__device__ __forceinline__ u32x4 poison() { return u32x4{~0u, ~0u, ~0u, ~0u}; }

// 16-B vectors of T, accumulated in A (fp32 for fp32 / bf16, fp64 for fp64)
template <typename T> struct Acc;
template <> struct Acc<float> {   // 4 fp32
  static constexpr int N = 4;
  typedef float A;
  __device__ static void add(A* acc, const u32x4& v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] += __uint_as_float(v[i]);
  }
  __device__ static u32x4 pack(const A* acc, float s) {
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(acc[i] * s);
    return r;
  }
};
template <> struct Acc<bf16_t> {  // 8 bf16
  static constexpr int N = 8;
  typedef float A;
  __device__ static void add(A* acc, const u32x4& v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[2 * i] += __uint_as_float(v[i] << 16);
      acc[2 * i + 1] += __uint_as_float(v[i] & 0xffff0000u);
    }
  }
  __device__ static u32x4 pack(const A* acc, float s) {
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      r[i] = (uint32_t)f2bf(acc[2 * i] * s) | ((uint32_t)f2bf(acc[2 * i + 1] * s) << 16);
    return r;
  }
};
template <> struct Acc<double> {  // 2 fp64 (SyncBN statistics)
  static constexpr int N = 2;
  typedef double A;
  __device__ static void add(A* acc, const u32x4& v) {
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[i] += __hiloint2double((int)v[2 * i + 1], (int)v[2 * i]);
  }
  __device__ static u32x4 pack(const A* acc, float s) {
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const double d = acc[i] * (double)s;
      r[2 * i] = (uint32_t)__double2loint(d);
      r[2 * i + 1] = (uint32_t)__double2hiint(d);
    }
    return r;
  }
};

// 16-B vector i of a payload of `bytes` bytes (the last vector may be partial: latency-class scalars)
__device__ __forceinline__ u32x4 load_vec(const u32x4* src, int64_t i, int64_t bytes) {
  if ((i + 1) * 16 <= bytes) return src[i];
  u32x4 v = u32x4{0u, 0u, 0u, 0u};
  const unsigned char* b = (const unsigned char*)(src + i);
  for (int k = 0; k < (int)(bytes - i * 16); ++k) v[k >> 2] |= (unsigned)b[k] << (8 * (k & 3));
  return v;
}
__device__ __forceinline__ void store_vec(u32x4* dst, int64_t i, int64_t bytes, const u32x4& v) {
  if ((i + 1) * 16 <= bytes) {
    dst[i] = v;
    return;
  }
  unsigned char* b = (unsigned char*)(dst + i);
  for (int k = 0; k < (int)(bytes - i * 16); ++k) b[k] = (unsigned char)(v[k >> 2] >> (8 * (k & 3)));
}

// K1: local input -> own staging slot (write-through, system scope), then barrier 0.  `pieces` windows of
// `pbytes` bytes, window p read at src + p * pitch (reduce-scatter chunk), stored back to back in the slot
// (a partial last vector of a single piece is zero-padded).
__global__ __launch_bounds__(NT) void xgmi_copy_in_kernel(const u32x4* __restrict__ src, XArgs a, int64_t pbytes,
                                                          int pieces, int64_t pitch) {
  const int64_t pvec = (pbytes + 15) / 16;
  const __amdgpu_buffer_rsrc_t dst = rsrc_of(slot_of(a, a.rank), pvec * pieces * 16);
  for (int p = 0; p < pieces; ++p)
    for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < pvec; i += (int64_t)gridDim.x * NT)
      __builtin_amdgcn_raw_buffer_store_b128(load_vec(src + p * pitch, i, pbytes), dst, (int)((p * pvec + i) * 16),
                                             0, SYS);
  arrive(a, 0);
}

// sum over ranks of vector i of every peer slot, starting at byte offset `off`
template <typename T>
__device__ __forceinline__ u32x4 reduce_vec(const __amdgpu_buffer_rsrc_t* src, int world, int64_t byte, float s) {
  typename Acc<T>::A acc[Acc<T>::N];
#pragma unroll
  for (int k = 0; k < Acc<T>::N; ++k) acc[k] = 0;
  u32x4 v[MAXW];
#pragma unroll
  for (int p = 0; p < MAXW; ++p)   // all W loads in flight before the first add (one xGMI round trip)
    if (p < world) v[p] = __builtin_amdgcn_raw_buffer_load_b128(src[p], (int)byte, 0, SYS);
#pragma unroll
  for (int p = 0; p < MAXW; ++p)
    if (p < world) Acc<T>::add(acc, v[p]);
  return Acc<T>::pack(acc, s);
}

__device__ __forceinline__ void peer_rsrcs(const XArgs& a, int64_t bytes, __amdgpu_buffer_rsrc_t (&r)[MAXW]) {
#pragma unroll
  for (int p = 0; p < MAXW; ++p) r[p] = rsrc_of(slot_of(a, p < a.world ? p : 0), bytes);
}

// one-shot all-reduce: out = s * sum_p slot_p (payload of `bytes` bytes, any size)
// root >= 0: reduce to one rank (ZeRO-2 reduce-to-owner): the others only take part in the barrier.
template <typename T>
__global__ __launch_bounds__(NT) void xgmi_allreduce_kernel(XArgs a, u32x4* __restrict__ out, int64_t bytes, float s,
                                                            int root) {
  const bool ok = passed(a, 0);
  if (root >= 0 && a.rank != root) return;
  const int64_t nvec = (bytes + 15) / 16;
  __amdgpu_buffer_rsrc_t src[MAXW];
  peer_rsrcs(a, nvec * 16, src);
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * NT)
    store_vec(out, i, bytes, ok ? reduce_vec<T>(src, a.world, i * 16, s) : poison());
}

// two-shot phase 1 / reduce_scatter: chunk `rank` (cvec vectors) reduced from every peer.
//   to_slot: write into own staging chunk (phase 1 of two-shot, then barrier 1) instead of `out`.
template <typename T>
__global__ __launch_bounds__(NT) void xgmi_reduce_chunk_kernel(XArgs a, u32x4* __restrict__ out, int64_t cvec, float s,
                                                              int to_slot) {
  const bool ok = passed(a, 0);
  const int64_t total = cvec * a.world;
  __amdgpu_buffer_rsrc_t src[MAXW];
  peer_rsrcs(a, total * 16, src);
  const int64_t base = (int64_t)a.rank * cvec;
  const __amdgpu_buffer_rsrc_t mine = rsrc_of(slot_of(a, a.rank), total * 16);
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < cvec; i += (int64_t)gridDim.x * NT) {
    const u32x4 v = ok ? reduce_vec<T>(src, a.world, (base + i) * 16, s) : poison();
    if (to_slot) __builtin_amdgcn_raw_buffer_store_b128(v, mine, (int)((base + i) * 16), 0, SYS);
    else out[i] = v;
  }
  if (to_slot) arrive(a, 1);
}

// all-gather: out[p * pitch + i] = chunk p of peer p's slot (chunk_in_slot: peer p keeps its piece at
// chunk p of its slot (two-shot phase 2) or at offset 0 (all_gather of a shard)).  Block g starts at peer
// rank + g: concurrent blocks pull from different peers, so all links carry traffic at once.
__global__ __launch_bounds__(NT) void xgmi_gather_kernel(XArgs a, u32x4* __restrict__ out, int64_t cvec, int64_t pitch,
                                                         int bar, int chunk_in_slot) {
  const bool ok = passed(a, bar);
  for (int j = 0; j < a.world; ++j) {
    const int p = (a.rank + (int)blockIdx.x + j) % a.world;
    const int64_t off = chunk_in_slot ? (int64_t)p * cvec : 0;
    const __amdgpu_buffer_rsrc_t src = rsrc_of(slot_of(a, p), (off + cvec) * 16);
    for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < cvec; i += (int64_t)gridDim.x * NT)
      out[(int64_t)p * pitch + i] = ok ? __builtin_amdgcn_raw_buffer_load_b128(src, (int)((off + i) * 16), 0, SYS)
                                       : poison();
  }
}

__global__ void xgmi_barrier_kernel(XArgs a) { mesh_wait(a, 3); }

// Communication kernels share the GPU with the compute stream: a modest grid (<= 128 blocks of 256
// lanes, half a block per CU) keeps enough 16-B loads in flight to saturate the links while leaving most
// of every CU to the GEMMs it overlaps with.
// s_memrealtime rate of the current device (hipDeviceAttributeWallClockRate, kHz; 100 MHz on gfx950)
int wallclock_khz() {
  static int khz = 0;
  if (khz <= 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev) == hipSuccess &&
        v > 0)
      khz = v;
    else
      khz = 100000;
  }
  return khz;
}

int grid_of(int64_t nvec) {
  int64_t g = (nvec + NT - 1) / NT;
  if (g < 1) g = 1;
  if (g > 128) g = 128;
  return (int)g;
}

}  // namespace

// -------------------------------------------------------------------------------------------------
// host entry points
// -------------------------------------------------------------------------------------------------
PDT_API int pdt_xgmi_alloc(int64_t bytes, int uncached, void** out) {
  // uncached fine-grained HBM: every access to the staging / signal words is coherent across devices
  // (the kernels also use cache-bypassing sc0|sc1 accesses, so plain device memory works as well)
  hipError_t e = uncached ? hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocUncached)
                          : hipMalloc(out, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*out, 0, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  return (int)hipDeviceSynchronize();
}

PDT_API int pdt_xgmi_free(void* p) { return (int)hipFree(p); }

PDT_API int pdt_xgmi_ipc_get(void* p, void* handle_out /* 64 B */) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e == hipSuccess) memcpy(handle_out, &h, sizeof(h));
  return (int)e;
}

PDT_API int pdt_xgmi_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

PDT_API int pdt_xgmi_ipc_open(const void* handle_in, void** out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle_in, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

PDT_API int pdt_xgmi_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

// error word of this rank's buffer (bit b = a wait at barrier b timed out); cleared by the read
PDT_API int pdt_xgmi_error(void* own_buf, unsigned* out) {
  hipError_t e = hipMemcpy(out, (char*)own_buf + ERR_OFF, 4, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return (int)e;
  const unsigned z = 0;
  return (int)hipMemcpy((char*)own_buf + ERR_OFF, &z, 4, hipMemcpyHostToDevice);
}

// Host-mapped error word (pinned, coherent): the kernels OR timeout bits into it, the host reads it
// without synchronising the device.
PDT_API int pdt_xgmi_host_flag_alloc(void** host_ptr, void** dev_ptr) {
  hipError_t e = hipHostMalloc(host_ptr, 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return (int)e;
  memset(*host_ptr, 0, 64);
  return (int)hipHostGetDevicePointer(dev_ptr, *host_ptr, 0);
}

PDT_API int pdt_xgmi_host_flag_free(void* host_ptr) { return (int)hipHostFree(host_ptr); }

// the device's s_memrealtime rate in kHz (the mesh-wait budget's unit conversion)
PDT_API int pdt_xgmi_wallclock_khz() { return wallclock_khz(); }

// kind: 0 one-shot all-reduce, 1 two-shot all-reduce, 2 all-gather, 3 reduce-scatter, 4 barrier,
//       5 reduce to root (root rank passed as pitch_bytes / 16).
//   bytes: all-reduce: the whole payload (one-shot / reduce: any size; two-shot: multiple of 16 * world);
//          all-gather / reduce-scatter: ONE rank's piece (a multiple of 16).
//   pitch_bytes: all-gather: distance between consecutive peers' pieces in `out`; reduce-scatter: distance
//          between consecutive pieces in `in` (both = bytes for a contiguous tensor).
//   dtype: fp32 / bf16 (fp32 accumulation) or fp64 (one-shot / reduce only: SyncBN statistics).
//   scale multiplies reduced values (1/world = AVG).
PDT_API int pdt_xgmi_collective(int kind, const void* in, void* out, int64_t bytes, int64_t pitch_bytes, int dtype,
                                float scale, const void* const* bufs, int rank, int world, unsigned epoch,
                                int64_t slot_bytes, unsigned timeout_us, unsigned* host_err, hipStream_t s) {
  if (world < 1 || world > MAXW || rank < 0 || rank >= world || epoch == 0) return (int)hipErrorInvalidValue;
  const bool any_size = kind == 0 || kind == 5;
  if ((!any_size && bytes % 16 != 0) || pitch_bytes % 16 != 0 || bytes < 0) return (int)hipErrorInvalidValue;
  if (kind != 4 && dtype != kF32 && dtype != kBF16 && !(dtype == kF64 && any_size)) return (int)hipErrorInvalidValue;
  if (slot_bytes >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;   // 32-bit buffer offsets
  const int64_t padded = (bytes + 15) / 16 * 16;
  const int64_t staged = kind == 3 ? bytes * world : padded;
  if (staged > slot_bytes) return (int)hipErrorInvalidValue;
  XArgs a{};
  for (int p = 0; p < world; ++p) a.buf[p] = (char*)bufs[p];
  a.host_err = host_err;
  a.rank = rank;
  a.world = world;
  a.epoch = epoch;
  a.timeout_ticks = (uint64_t)timeout_us * (uint64_t)wallclock_khz() / 1000;
  a.slot_bytes = slot_bytes;
  if (kind == 4) {
    hipLaunchKernelGGL(xgmi_barrier_kernel, dim3(1), dim3(64), 0, s, a);
    return (int)hipGetLastError();
  }
  const int64_t nvec = padded / 16, pitch = pitch_bytes / 16;
  // copy-in; its last block runs barrier 0
  if (kind == 3)
    hipLaunchKernelGGL(xgmi_copy_in_kernel, dim3(grid_of(nvec * world)), dim3(NT), 0, s, (const u32x4*)in, a, bytes,
                       world, pitch);
  else
    hipLaunchKernelGGL(xgmi_copy_in_kernel, dim3(grid_of(nvec)), dim3(NT), 0, s, (const u32x4*)in, a, bytes, 1,
                       (int64_t)0);
  const bool bf = dtype == kBF16, f64 = dtype == kF64;
  switch (kind) {
    case 0:
    case 5: {
      const int root = kind == 5 ? (int)(pitch_bytes / 16) : -1;   // reduce: pitch carries the root rank
      if (bf) hipLaunchKernelGGL(xgmi_allreduce_kernel<bf16_t>, dim3(grid_of(nvec)), dim3(NT), 0, s, a, (u32x4*)out, bytes, scale, root);
      else if (f64) hipLaunchKernelGGL(xgmi_allreduce_kernel<double>, dim3(grid_of(nvec)), dim3(NT), 0, s, a, (u32x4*)out, bytes, scale, root);
      else hipLaunchKernelGGL(xgmi_allreduce_kernel<float>, dim3(grid_of(nvec)), dim3(NT), 0, s, a, (u32x4*)out, bytes, scale, root);
      break;
    }
    case 1: {
      if (nvec % world != 0) return (int)hipErrorInvalidValue;
      const int64_t cvec = nvec / world;
      if (bf) hipLaunchKernelGGL(xgmi_reduce_chunk_kernel<bf16_t>, dim3(grid_of(cvec)), dim3(NT), 0, s, a, (u32x4*)out, cvec, scale, 1);
      else hipLaunchKernelGGL(xgmi_reduce_chunk_kernel<float>, dim3(grid_of(cvec)), dim3(NT), 0, s, a, (u32x4*)out, cvec, scale, 1);
      hipLaunchKernelGGL(xgmi_gather_kernel, dim3(grid_of(cvec)), dim3(NT), 0, s, a, (u32x4*)out, cvec, cvec, 1, 1);
      break;
    }
    case 3:
      if (bf) hipLaunchKernelGGL(xgmi_reduce_chunk_kernel<bf16_t>, dim3(grid_of(nvec)), dim3(NT), 0, s, a, (u32x4*)out, nvec, scale, 0);
      else hipLaunchKernelGGL(xgmi_reduce_chunk_kernel<float>, dim3(grid_of(nvec)), dim3(NT), 0, s, a, (u32x4*)out, nvec, scale, 0);
      break;
    case 2:
      hipLaunchKernelGGL(xgmi_gather_kernel, dim3(grid_of(nvec)), dim3(NT), 0, s, a, (u32x4*)out, nvec, pitch, 0, 0);
      break;
    default:
      return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
