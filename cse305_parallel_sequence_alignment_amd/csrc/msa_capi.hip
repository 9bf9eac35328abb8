// msa_capi.hip -- host side of the C-ABI (include/msa.h): plans, launches,
// and the reference-compatible entry points.  All DP cells are computed by the
// kernels in msa_kernels.hip; the host only encodes inputs, de-skews outputs
// and walks traceback bits (O(m+n), like the reference's find_alignment).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <condition_variable>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <deque>
#include <map>
#include <tuple>
#include <vector>

#include "../../include/msa.h"
#include "msa_kernels.hip"
#include "msa_flow.hip"
#include "msa_cflow.hip"
#include "msa_band.hip"
#include "msa_rowsweep.hip"
#include "msa_traceback.hip"

using namespace msa;

namespace {

#define HIPCHK(x)                                         \
  do {                                                    \
    hipError_t e_ = (x);                                  \
    if (e_ != hipSuccess) {                               \
      std::fprintf(stderr, "msa: %s failed: %s\n", #x, hipGetErrorString(e_)); \
      return MSA_ERR_HIP;                                 \
    }                                                     \
  } while (0)

int g_dev_checked = 0;
int g_dev_ok = 0;
std::mutex g_dev_mu;

int ensure_device() {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  if (!g_dev_checked) {
    g_dev_checked = 1;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
      g_dev_ok = 0;
    } else {
      hipDeviceProp_t prop;
      int dev = 0;
      (void)hipGetDevice(&dev);
      g_dev_ok = (hipGetDeviceProperties(&prop, dev) == hipSuccess) &&
                 (std::strncmp(prop.gcnArchName, "gfx950", 6) == 0);
      if (!g_dev_ok) std::fprintf(stderr, "msa: device 0 is %s, need gfx950\n", prop.gcnArchName);
    }
  }
  return g_dev_ok ? MSA_OK : MSA_ERR_NODEV;
}

int current_device() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  return dev;
}

// Frees pooled blocks held by idle cached plans (msa_refapi.inc) when the device runs out.
void (*g_pool_reclaim)() = nullptr;

// Device memory pool.  The reference's harness calls main_alignment_function
// from hardware_concurrency threads at once (testing.cpp:145-158, 269-280,
// 352-358); with plain hipMalloc/hipFree every call would serialize on
// hipFree's implicit device synchronization.  Blocks are cached per (device,
// size class) (powers of two up to 1 MiB, then 2 MiB multiples) in one
// mutex-protected free list, so a block allocated while device d was current
// is only handed to a caller for which d is current.  A block is only returned
// by its owner after the stream work that used it has completed (run_one syncs
// its stream, msa_plan_destroy syncs every stream the plan queued work on), so
// a block never changes hands while a kernel uses it.
class DevPool {
 public:
  static size_t size_class(size_t b) {
    if (b < 256) b = 256;
    if (b <= (size_t(1) << 20)) {
      size_t c = 256;
      while (c < b) c <<= 1;
      return c;
    }
    const size_t mb2 = size_t(2) << 20;
    return (b + mb2 - 1) / mb2 * mb2;
  }
  void* get(size_t bytes) {
    const size_t c = size_class(bytes);
    const int dev = current_device();
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = free_.find(std::make_pair(dev, c));
      if (it != free_.end()) {
        void* p = it->second;
        free_.erase(it);
        cached_ -= c;
        return p;
      }
    }
    void* p = nullptr;
    if (hipMalloc(&p, c) != hipSuccess) {
      // cached blocks of other sizes (and those idle cached plans hold) may be what fills the
      // device: release them, retry once
      (void)hipGetLastError();
      if (g_pool_reclaim) g_pool_reclaim();
      release(dev);
      p = nullptr;
      if (hipMalloc(&p, c) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
      }
    }
    std::lock_guard<std::mutex> lk(mu_);
    owner_[p] = dev;
    return p;
  }
  void put(void* p, size_t bytes) {
    if (!p) return;
    const size_t c = size_class(bytes);
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto o = owner_.find(p);
      const int dev = (o != owner_.end()) ? o->second : current_device();
      if (cached_ + c <= kCap) {
        free_.emplace(std::make_pair(dev, c), p);
        cached_ += c;
        return;
      }
      owner_.erase(p);
    }
    (void)hipFree(p);
  }
  // free every cached block of device dev
  void release(int dev) {
    std::vector<void*> victims;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto it = free_.begin(); it != free_.end();) {
        if (it->first.first == dev) {
          victims.push_back(it->second);
          cached_ -= it->first.second;
          owner_.erase(it->second);
          it = free_.erase(it);
        } else {
          ++it;
        }
      }
    }
    for (void* v : victims) (void)hipFree(v);
  }
  size_t cached() {
    std::lock_guard<std::mutex> lk(mu_);
    return cached_;
  }
  size_t cached(int dev) {  // free blocks of device dev
    std::lock_guard<std::mutex> lk(mu_);
    size_t b = 0;
    for (const auto& e : free_)
      if (e.first.first == dev) b += e.first.second;
    return b;
  }

 private:
  static constexpr size_t kCap = size_t(8) << 30;  // bytes kept cached (HBM is 288 GB)
  std::mutex mu_;
  std::multimap<std::pair<int, size_t>, void*> free_;  // (device, size class) -> block
  std::map<void*, int> owner_;                         // block -> device it was allocated on
  size_t cached_ = 0;
};

DevPool& dev_pool() {
  static DevPool* p = new DevPool();  // never destroyed: no HIP calls during static teardown
  return *p;
}

// Admission control at the drop-in boundary.  The reference's callers run main_alignment_function
// from hardware_concurrency threads at once, each on whole sequences (testing.cpp:209-287, call at
// :261; :295-369, call at :345): on a 256-thread host, a 97k pair's ~13 GB footprint (1 B/cell
// direction bytes + pass-2 inputs) times the callers in flight exceeds any device.  Every host-pointer
// entry point therefore reserves its call's device footprint (estimated from m, n before anything
// is allocated: a call never holds part of its memory while it waits) against a per-device budget and
// waits -- FIFO, so no caller is overtaken -- until it fits.  A call larger than the whole budget
// runs alone (it waits until nothing else is admitted).  Budget: MSA_DEVICE_BUDGET_MB, else 90% of
// the device's memory; msa_set_device_budget overrides it at run time.
// Memory the library holds on a device outside the admitted calls: idle cached plans of the reference
// walk and free blocks of the device pool (msa_refapi.inc).  An admission that would put admitted +
// idle bytes over the budget first releases the idle ones, so cached memory never pushes admitted calls
// into the allocator's out-of-memory path.
size_t idle_device_bytes(int dev);
size_t idle_plan_bytes(int dev);
void reclaim_idle_device_bytes(int dev);

class Admission {
 public:
  void acquire(int dev, size_t bytes) {
    std::unique_lock<std::mutex> lk(mu_);
    Dev& d = get(dev);
    const uint64_t t = d.next++;
    bool waited = false;
    cv_.wait(lk, [&] {
      const bool ok = d.serving == t && (d.inuse == 0 || d.inuse + bytes <= d.budget);
      waited = waited || !ok;
      return ok;
    });
    d.inuse += bytes;
    d.peak = std::max(d.peak, d.inuse);
    d.admitted++;
    if (waited) d.waits++;
    d.serving++;
    const size_t inuse = d.inuse, budget = d.budget;
    cv_.notify_all();  // the next ticket may fit too
    lk.unlock();
    if (inuse + idle_device_bytes(dev) > budget) {
      reclaim_idle_device_bytes(dev);
      std::lock_guard<std::mutex> lk2(mu_);
      get(dev).reclaims++;
    }
  }
  void release(int dev, size_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    Dev& d = get(dev);
    d.inuse -= std::min(bytes, d.inuse);
    cv_.notify_all();
  }
  void set_budget(int dev, size_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    Dev& d = get(dev);
    d.budget = bytes ? bytes : default_budget(dev);
    d.peak = d.inuse;
    d.waits = d.admitted = d.reclaims = 0;
    cv_.notify_all();
  }
  void info(int dev, int64_t* out, int n = 5) {
    std::lock_guard<std::mutex> lk(mu_);
    Dev& d = get(dev);
    out[0] = (int64_t)d.budget;
    out[1] = (int64_t)d.inuse;
    out[2] = (int64_t)d.peak;
    out[3] = (int64_t)d.waits;
    out[4] = (int64_t)d.admitted;
    if (n > 5) out[5] = (int64_t)d.reclaims;
  }

 private:
  struct Dev {
    bool init = false;
    size_t budget = 0, inuse = 0, peak = 0;
    uint64_t next = 0, serving = 0, waits = 0, admitted = 0, reclaims = 0;
  };
  static size_t default_budget(int dev) {
    const char* e = std::getenv("MSA_DEVICE_BUDGET_MB");
    if (e && std::atoll(e) > 0) return (size_t)std::atoll(e) << 20;
    size_t fr = 0, tot = 0;
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (cur != dev) (void)hipSetDevice(dev);
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) { (void)hipGetLastError(); tot = size_t(16) << 30; }
    if (cur != dev) (void)hipSetDevice(cur);
    return tot / 10 * 9;
  }
  Dev& get(int dev) {  // (mu_ held)
    Dev& d = dev_[dev];
    if (!d.init) {
      d.init = true;
      d.budget = default_budget(dev);
    }
    return d;
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<int, Dev> dev_;
};

Admission& admission() {
  static Admission* a = new Admission();
  return *a;
}

// RAII reservation of one call's device footprint (declare it before the call's streams and blocks:
// destroyed last, after they have been synchronized and returned)
struct Admit {
  int dev = 0;
  size_t bytes = 0;
  explicit Admit(size_t b) : bytes(b) {
    (void)hipGetDevice(&dev);
    admission().acquire(dev, bytes);
  }
  ~Admit() { admission().release(dev, bytes); }
  Admit(const Admit&) = delete;
  Admit& operator=(const Admit&) = delete;
};

// Non-blocking streams reused across calls (creating one costs ~10s of us), one
// free list per device: a stream is only handed to a caller whose current device
// created it.
class StreamPool {
 public:
  hipStream_t get() {
    const int dev = current_device();
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto& fl = free_[dev];
      if (!fl.empty()) {
        hipStream_t s = fl.back();
        fl.pop_back();
        return s;
      }
    }
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu_);
    owner_[s] = dev;
    return s;
  }
  void put(hipStream_t s) {
    if (!s) return;
    std::lock_guard<std::mutex> lk(mu_);
    auto o = owner_.find(s);
    free_[o != owner_.end() ? o->second : current_device()].push_back(s);
  }

 private:
  std::mutex mu_;
  std::map<int, std::vector<hipStream_t>> free_;
  std::map<hipStream_t, int> owner_;
};

std::atomic<uint32_t> g_epoch{0};  // granule epoch of the next run (msa_plan_run)

StreamPool& stream_pool() {
  static StreamPool* p = new StreamPool();
  return *p;
}

int nc_of(int alg) {
  switch (alg) {
    case MSA_ALG_SWL: case MSA_ALG_SWL0: case MSA_ALG_SWLP: return 1;
    case MSA_ALG_SWA: case MSA_ALG_NWA: case MSA_ALG_REF1: return 2;
    default: return 3;
  }
}

typedef void (*kfn_t)(KArgs);

// Per-process caches of what plan creation asks the runtime: compute units per device
// (hipGetDeviceProperties is slow, and main_alignment_function creates a plan per call)
// and, per (device, kernel, block, LDS), the dynamic-LDS attribute and the occupancy.
std::mutex g_shape_mu;
int device_cus() {
  static std::map<int, int> cus;
  const int dev = current_device();
  std::lock_guard<std::mutex> lk(g_shape_mu);
  auto it = cus.find(dev);
  if (it != cus.end()) return it->second;
  hipDeviceProp_t prop;
  const int n = (hipGetDeviceProperties(&prop, dev) == hipSuccess) ? prop.multiProcessorCount : 1;
  cus[dev] = n;
  return n;
}
// LDS a workgroup may allocate on the current device: min(sharedMemPerBlockOptin, 160 KiB), read once
// per device (plans reject larger requests instead of failing the attribute call on a smaller part)
size_t device_lds_max() {
  static std::map<int, size_t> lds;
  const int dev = current_device();
  std::lock_guard<std::mutex> lk(g_shape_mu);
  auto it = lds.find(dev);
  if (it != lds.end()) return it->second;
  hipDeviceProp_t prop;
  size_t v = 64 * 1024;
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess)
    v = std::max<size_t>(prop.sharedMemPerBlockOptin, prop.sharedMemPerBlock);
  v = std::min<size_t>(v, 160 * 1024);
  lds[dev] = v;
  return v;
}
// raises the kernel's dynamic-LDS limit to the CU's whole LDS (once per device and kernel: plans of
// one kernel with different LDS sizes then never lower it under each other) and returns its
// occupancy at `lds` bytes (blocks per CU, >= 1), or -1
int kernel_shape(kfn_t fn, int threads, size_t lds) {
  static std::map<std::tuple<int, kfn_t, int, size_t>, int> occ_of;
  static std::map<std::pair<int, kfn_t>, bool> attr_set;
  const size_t lds_max = device_lds_max();
  const auto key = std::make_tuple(current_device(), fn, threads, lds);
  std::lock_guard<std::mutex> lk(g_shape_mu);
  auto it = occ_of.find(key);
  if (it != occ_of.end()) return it->second;
  if (lds > lds_max) return -1;
  const auto ak = std::make_pair(current_device(), fn);
  if (!attr_set[ak]) {
    if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max) != hipSuccess)
      return -1;
    attr_set[ak] = true;
  }
  int occ = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)fn, threads, lds) != hipSuccess || occ < 1)
    occ = 1;
  occ_of[key] = occ;
  return occ;
}

// single-pair phase length: 32 steps for one carried value (SW linear); 16 when
// two or three values per cell are carried (register pressure: no spills)
constexpr int ks_single(int alg) { return (alg == MSA_ALG_SWL || alg == MSA_ALG_SWL0) ? MSA_KS_SINGLE : 16; }
constexpr int ks_batch(int alg) { return (alg == MSA_ALG_SWLP) ? MSA_KS_BATCH_SWLP : MSA_KS_BATCH; }

template <int ALG, int OUT, int TP>
kfn_t kf(bool sgl) {
  // single pair: (MSA_WAVES_SINGLE waves, MSA_KS_SINGLE steps/phase); batch: (MSA_WAVES_BATCH, MSA_KS_BATCH)
  return sgl ? stripe_kernel<ALG, OUT, TP, MSA_WAVES_SINGLE, ks_single(ALG), true>
                               : stripe_kernel<ALG, OUT, TP, MSA_WAVES_BATCH, ks_batch(ALG), false>;
}

kfn_t pick_kernel(int alg, int out, int tp, bool sgl) {
#define K3(A, O) return tp == 2 ? kf<A, O, 2>(sgl) : (tp ? kf<A, O, 1>(sgl) : kf<A, O, 0>(sgl))
  switch (alg) {
    case MSA_ALG_SWL:
      if (out == MSA_OUT_NONE) K3(MSA_ALG_SWL, MSA_OUT_NONE);
      if (out == MSA_OUT_H) K3(MSA_ALG_SWL, MSA_OUT_H);
      break;
    case MSA_ALG_SWLP:
      if (out == MSA_OUT_NONE && !sgl && tp == 0) return kf<MSA_ALG_SWLP, MSA_OUT_NONE, 0>(false);
      break;
    case MSA_ALG_SWL0:
      if (out == MSA_OUT_NONE) K3(MSA_ALG_SWL0, MSA_OUT_NONE);
      if (out == MSA_OUT_H) K3(MSA_ALG_SWL0, MSA_OUT_H);
      break;
    case MSA_ALG_SWA:
      if (out == MSA_OUT_NONE) K3(MSA_ALG_SWA, MSA_OUT_NONE);
      if (out == MSA_OUT_H) K3(MSA_ALG_SWA, MSA_OUT_H);
      if (out == MSA_OUT_DIR) K3(MSA_ALG_SWA, MSA_OUT_DIR);
      break;
    case MSA_ALG_NWA:
      if (out == MSA_OUT_NONE) return kf<MSA_ALG_NWA, MSA_OUT_NONE, 0>(sgl);
      if (out == MSA_OUT_H) return kf<MSA_ALG_NWA, MSA_OUT_H, 0>(sgl);
      break;
    case MSA_ALG_REF:
      if (out == MSA_OUT_NONE) return kf<MSA_ALG_REF, MSA_OUT_NONE, 0>(sgl);
      if (out == MSA_OUT_TAB) return kf<MSA_ALG_REF, MSA_OUT_TAB, 0>(sgl);
      if (out == MSA_OUT_DIR) return kf<MSA_ALG_REF, MSA_OUT_DIR, 0>(sgl);
      if (out == MSA_OUT_H) return kf<MSA_ALG_REF, MSA_OUT_H, 0>(sgl);
      break;
    case MSA_ALG_REF1:
      if (out == MSA_OUT_NONE) return kf<MSA_ALG_REF1, MSA_OUT_NONE, 0>(sgl);
      if (out == MSA_OUT_DIR) return kf<MSA_ALG_REF1, MSA_OUT_DIR, 0>(sgl);
      break;
    case MSA_ALG_PART:
      if (out == MSA_OUT_TAB) return kf<MSA_ALG_PART, MSA_OUT_TAB, 0>(sgl);
      break;
  }
#undef K3
  return nullptr;
}

// single-pair SW linear (msa_flow.hip): pass 1 (chain), pass 2 (fill + H)
kfn_t pick_flow(int alg, bool best, bool save, int tp, int R, bool nneg) {
  // SW affine / the reference's Gotoh (direction bytes): pass 1 + in-launch pass 2, one row per lane;
  // SW affine with scores >= 0: pass 1 applies the zero floor in its head phases only
  if (alg == MSA_ALG_SWA) {
    if (!save) return nullptr;
    if (R == 2) return nneg ? flow_kernel<false, false, true, true, 2, 1> : flow_kernel<true, false, true, true, 2, 1>;
    return nneg ? flow_kernel<false, false, true, true, 1, 1> : flow_kernel<true, false, true, true, 1, 1>;
  }
  if (alg == MSA_ALG_REF1)
    return !save ? nullptr : (R == 2 ? flow_kernel<true, false, true, true, 2, 2> : flow_kernel<true, false, true, true, 1, 2>);
  // score-only plans: pass 1 alone, one row per lane, best cell tracked in the chain;
  // H plans: pass 1 + in-launch pass 2, two rows per lane
  const bool fl = (alg == MSA_ALG_SWL);
  if (best) return fl ? flow_kernel<true, true, false, false> : flow_kernel<false, true, false, false>;
  if (save && R == 2) {
    if (fl) return tp ? flow_kernel<true, false, true, true, 2> : flow_kernel<true, false, true, false, 2>;
    return tp ? flow_kernel<false, false, true, true, 2> : flow_kernel<false, false, true, false, 2>;
  }
  return nullptr;
}

// the separate pass-2 launch of a long pair (flow_fill_kernel), same instantiation parameters
kfn_t pick_fill(int alg, int tp, int R, bool nneg) {
  if (alg == MSA_ALG_SWA)
    return R == 2 ? (nneg ? flow_fill_kernel<false, false, 2, 1> : flow_fill_kernel<true, false, 2, 1>)
                  : (nneg ? flow_fill_kernel<false, false, 1, 1> : flow_fill_kernel<true, false, 1, 1>);
  if (alg == MSA_ALG_REF1) return R == 2 ? flow_fill_kernel<true, false, 2, 2> : flow_fill_kernel<true, false, 1, 2>;
  if (R != 2) return nullptr;
  if (alg == MSA_ALG_SWL) return tp ? flow_fill_kernel<true, true, 2, 0> : flow_fill_kernel<true, false, 2, 0>;
  return tp ? flow_fill_kernel<false, true, 2, 0> : flow_fill_kernel<false, false, 2, 0>;
}

}  // namespace

struct msa_plan {
  msa_plan_desc d;
  msa_kparams kp;
  int nc = 1;
  int W = MSA_WAVES_BATCH;  // compute waves per workgroup
  int KS = MSA_KS_BATCH;    // DP steps per phase
  std::vector<msa_pair_desc> pairs;
  int64_t total_stripes = 0;
  int64_t cells_elems = 0;
  size_t lds_bytes = 0;
  int grid = 1;
  int threads = 64;
  bool flow = false;   // flow_kernel (single-pair SW linear) instead of stripe_kernel
  bool band_k = false;  // band_kernel (banded single pair, msa_band.hip)
  int band_items = 0;   // band_kernel: items of the larger of its launches (granule slots)
  bool flow2 = false;  // + pass-2 blocks inside the same launch (O_H)
  bool fused_reduce = false;  // the pass-2 blocks write the pair result (fl_block_done): no reduce launch
  bool cflow = false;  // cflow_kernel: packed-couple score-only batch as flag-synchronised chains
  kfn_t fill_fn = nullptr;  // long pairs: pass 2 as a launch of its own behind pass 1
  int fill_grid = 0;
  size_t fill_lds = 0;
  unsigned long long* d_br = nullptr;
  unsigned long long* d_snap = nullptr;
  int4* d_blk = nullptr;
  int* d_order = nullptr;
  bool timing = true;  // record HIP events around the DP kernel (msa_plan_last_kernel_ms)
  bool timed = false;  // events of the last run exist
  int R = 1;      // flow kernel rows per lane
  int nflow = 0;  // two-pass: pass-1 workgroups (the rest of the grid runs pass-2 blocks)
  int brw = 0, nseg = 0, nblk = 0;
  int ps = FL_PS;  // phases per pass-2 segment (FL_PS_FILL when pass 2 is a launch of its own)
  int gbuf_stride = 0;
  kfn_t fn = nullptr;
  // device
  msa_pair_desc* d_pairs = nullptr;
  msa_stripe_meta* d_meta = nullptr;
  // [0] ticket, [4..11] per-XCD item chunks; flow kernels: [32] arrival, [64] pass-2 blocks, each
  // in a 128-byte line of its own (thousands of pass-2 waves claim blocks while pass-1 workgroups
  // claim their items: on one line the item claims queued ~16 us behind them).  Reset every run.
  int* d_ticket = nullptr;
  int* d_err = nullptr;     // sticky error word: set by a kernel wait that hit its spin limit; cleared
                            // only at plan creation and by msa_plan_clear_error
  unsigned long long* d_gbuf = nullptr;
  uint8_t* d_cod = nullptr;                // MSA_NCOPY byte-shifted padded column-code copies
  msa_pair_desc* d_segs = nullptr;         // distinct column sequences (b_off, n, cod_off)
  std::vector<msa_pair_desc> segs;
  int64_t cod_copy = 0;                    // bytes per copy
  PairResult* d_res = nullptr;
  unsigned long long* d_sum = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  uint32_t epoch = 0;
  unsigned long long* stamps = nullptr;  // diagnostic build
  std::vector<hipStream_t> streams;      // every stream work of this plan was queued on
                                         // (msa_plan_destroy waits on all of them)
  std::vector<std::pair<void*, size_t>> blocks;  // pooled device blocks owned by the plan
  // chunked banded single pair (kp.single == 2, rank convergence): the main launch runs the
  // chunks; the exact single-mode launch (fb_*) is queued behind it and exits at once
  // unless a chunk failed to converge
  bool chunked = false;
  int n_chunks = 0;
  msa_kparams fb_kp;
  kfn_t fb_fn = nullptr;
  int fb_grid = 1, fb_threads = 64;
  size_t fb_lds = 0;
  int* d_ck = nullptr;  // [chunk][2][2][ckw] band states (msa_kernels.hip)
  int ckw = 0;
  int* d_dk = nullptr;    // per-chunk constant d_k
  int* d_okk = nullptr;   // per-chunk converged flag
  int* d_skip = nullptr;  // 1: every chunk converged (the exact launch exits)
  bool h16 = false;       // band_kernel chunks >= 1 write int16 cells to d_h16 (chunk_add_kernel widens)
  int16_t* d_h16 = nullptr;

  void note_stream(hipStream_t s) {
    if (std::find(streams.begin(), streams.end(), s) == streams.end()) streams.push_back(s);
  }
  // a pooled device block of `bytes`, owned by the plan
  template <class T>
  bool alloc(T** p, size_t bytes) {
    void* q = dev_pool().get(bytes);
    if (!q) return false;
    blocks.emplace_back(q, bytes);
    *p = (T*)q;
    return true;
  }
};

extern "C" {

const char* msa_status_string(int s) {
  switch (s) {
    case MSA_OK: return "ok";
    case MSA_ERR_ARG: return "invalid argument";
    case MSA_ERR_ALPHABET: return "more than 8 distinct symbols";
    case MSA_ERR_HIP: return "HIP runtime error";
    case MSA_ERR_NODEV: return "no gfx950 device";
    case MSA_ERR_UNSUPPORTED: return "unsupported parameters (GPU path needs integral g,h)";
    case MSA_ERR_TIMEOUT: return "cross-workgroup wait timed out";
    case MSA_ERR_NOMEM: return "out of memory";
    case MSA_ERR_CAPACITY: return "output buffer too small";
    case MSA_ERR_NOMATCH: return "traceback found no predecessor";
  }
  return "unknown status";
}

int msa_version(void) { return 1; }

int msa_set_device_budget(int64_t bytes) {
  if (bytes < 0) return MSA_ERR_ARG;
  int rc = ensure_device();
  if (rc != MSA_OK) return rc;
  admission().set_budget(current_device(), (size_t)bytes);
  return MSA_OK;
}

int msa_device_budget_info(int64_t* out5) {
  if (!out5) return MSA_ERR_ARG;
  int rc = ensure_device();
  if (rc != MSA_OK) return rc;
  admission().info(current_device(), out5);
  return MSA_OK;
}

int msa_device_memory_info(int64_t* out4) {
  if (!out4) return MSA_ERR_ARG;
  int rc = ensure_device();
  if (rc != MSA_OK) return rc;
  const int dev = current_device();
  int64_t b[6];
  admission().info(dev, b, 6);
  out4[0] = b[1];
  out4[1] = (int64_t)idle_plan_bytes(dev);
  out4[2] = (int64_t)dev_pool().cached(dev);
  out4[3] = b[5];
  return MSA_OK;
}

int msa_device_count(int* count) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  if (count) *count = n;
  return n > 0 ? MSA_OK : MSA_ERR_NODEV;
}

int msa_encode_pair(const char* A0, size_t m, const char* B0, size_t n, uint8_t* ca, uint8_t* cb) {
  int map[256];
  for (int k = 0; k < 256; ++k) map[k] = -1;
  int next = 0;
  auto enc = [&](const char* s, size_t len, uint8_t* out) -> int {
    for (size_t k = 0; k < len; ++k) {
      const unsigned char c = (unsigned char)s[k];
      if (map[c] < 0) {
        if (next >= 8) return MSA_ERR_ALPHABET;
        map[c] = next++;
      }
      out[k] = (uint8_t)map[c];
    }
    return MSA_OK;
  };
  // DNA fast path: fixed codes so batches share one code map
  const char* dna = "ACGT";
  for (int k = 0; k < 4; ++k) map[(unsigned char)dna[k]] = k;
  next = 4;
  int rc = enc(A0, m, ca);
  if (rc != MSA_OK) return rc;
  return enc(B0, n, cb);
}

int msa_plan_create(const msa_plan_desc* desc, msa_plan** out) {
  if (!desc || !out || desc->n_pairs <= 0 || !desc->m || !desc->n || !desc->a_off || !desc->b_off) return MSA_ERR_ARG;
  int rc = ensure_device();
  if (rc != MSA_OK) return rc;
  msa_plan* P = new (std::nothrow) msa_plan();
  if (!P) return MSA_ERR_NOMEM;
  P->d = *desc;
  P->d.m = P->d.n = P->d.a_off = P->d.b_off = nullptr;
  const int alg = desc->alg;
  int out_mode = desc->cells;
  int kalg;
  switch (alg) {
    case MSA_SW_LINEAR:
      kalg = (desc->match >= 0 && desc->mismatch >= 0) ? MSA_ALG_SWL0 : MSA_ALG_SWL;
      if (kalg == MSA_ALG_SWL0 && !desc->single && out_mode == MSA_OUT_NONE && !desc->track_end &&
          desc->n_pairs >= 2) {
        // score-only batch: two pairs per lane as packed int16 (MSA_ALG_SWLP) when every pair
        // couple (2c, 2c+1) shares its row / column counts and column sequence (one stripe
        // geometry, one code stream) and G = H + g(i+j) stays inside int16
        bool pk = true;
        const int64_t g = desc->gap_extend, smax = std::max({0, desc->match, desc->mismatch});
        for (int64_t p = 0; p < desc->n_pairs && pk; ++p) {
          const int64_t q = (p & 1) ? p - 1 : p;
          pk = desc->m[p] == desc->m[q] && desc->n[p] == desc->n[q] && desc->b_off[p] == desc->b_off[q] &&
               g * (desc->m[p] + desc->n[p] + 2) + smax * std::min(desc->m[p], desc->n[p]) + 2 * g + 127 < 32000 &&
               desc->match + 2 * g <= 127;
        }
        if (pk) kalg = MSA_ALG_SWLP;
      }
      break;
    case MSA_SW_AFFINE: kalg = MSA_ALG_SWA; break;
    case MSA_NW_BANDED: kalg = MSA_ALG_NWA; break;
    case MSA_REF_GOTOH: {
      // start type -1 (main_alignment_function's single subproblem) with direction bytes or no
      // cells: the tagged-max form (every interior value is finite; values carried x4)
      int64_t span = 0;
      for (int64_t p = 0; p < desc->n_pairs; ++p) span = std::max(span, desc->m[p] + desc->n[p] + 2);
      const bool ref1 = desc->start_type == -1 && (out_mode == MSA_OUT_DIR || out_mode == MSA_OUT_NONE) &&
                        desc->gap_extend >= 0 && desc->gap_open >= desc->gap_extend &&
                        (int64_t)4 * (desc->gap_open + 1) * span < (int64_t(1) << 28);
      kalg = ref1 ? MSA_ALG_REF1 : MSA_ALG_REF;
      break;
    }
    case MSA_PARTIAL: kalg = MSA_ALG_PART; break;
    default: delete P; return MSA_ERR_ARG;
  }
  int tp = (kalg == MSA_ALG_SWL || kalg == MSA_ALG_SWL0 || kalg == MSA_ALG_SWA) ? (desc->track_end ? 1 : 0) : 0;
  if (tp) {
    // the first-maximum position packs with the value into one int (TRACKPOS 2) when every
    // local score is below 2^16 and a stripe has < 2^15 steps.  A local score gains at
    // most max(0, match, mismatch) per diagonal step (gaps only subtract), and a path
    // has at most min(m, n) diagonal steps.
    const int64_t smax = std::max({0, desc->match, desc->mismatch});
    bool pack = true;
    for (int64_t p = 0; p < desc->n_pairs && pack; ++p)
      pack = smax * std::min(desc->m[p], desc->n[p]) < 65536 && desc->n[p] + 512 < 32768;
    if (pack) tp = 2;
  }
  if (desc->single && desc->n_pairs != 1) { delete P; return MSA_ERR_ARG; }
  // A banded pair has only ~(2*band+64)/(64*lag) stripes in flight at once:
  // one workgroup cycling its waves over all stripes (the batch kernel, wrap
  // link through the LDS row buffer) beats a chain of cross-workgroup hand-offs.
  const bool single = desc->single != 0;
  P->d.single = single ? 1 : 0;
  // flow kernels: one SW-linear pair (8 byte-shifted LDS code rings), or one SW-affine /
  // reference-Gotoh (start type -1, tagged) pair with direction bytes (two values per link
  // column, 4 code rings); the column codes stream through fixed-size LDS rings, so any n fits
  const bool aff = kalg == MSA_ALG_SWA || kalg == MSA_ALG_REF1;
  // the code copies: whole rows when they fit (kp.code_whole: no ring bookkeeping), else rings
  const size_t flow_lds0 = (size_t)(FL_FLAGS + (FL_W + 1) * 256 * (aff ? 2 : 1)) * 4;
  const size_t flow_whole = flow_lds0 + (size_t)(aff ? 4 : FL_NCOPY) * (fl_code_bytes((int)desc->n[0]) + 16);
  const bool code_whole = flow_whole <= 96 * 1024;
  const size_t flow_lds = code_whole ? flow_whole : flow_lds0 + (size_t)(aff ? 4 : FL_NCOPY) * FL_CSTR;
  // affine: profile bytes score + 2e + (o - e) must be int8
  const bool aff_ok = kalg == MSA_ALG_SWA && out_mode == MSA_OUT_DIR && desc->gap_extend >= 0 &&
                      desc->gap_open >= desc->gap_extend &&
                      std::max(desc->match, desc->mismatch) + desc->gap_open + desc->gap_extend <= 127 &&
                      std::min(desc->match, desc->mismatch) + desc->gap_open + desc->gap_extend >= -128 &&
                      (int64_t)desc->gap_extend * (desc->m[0] + desc->n[0] + 2) < (int64_t(1) << 28);
  // Gotoh: profile bytes 4 (f + 2g) <= 127; the shifted tagged values 4 (T + g(i+j)) stay far
  // inside int32 (REF1's own bound covers the shift: |T| + g(i+j) <= (g+h+1) span)
  const bool got_ok = kalg == MSA_ALG_REF1 && out_mode == MSA_OUT_DIR && 4 * (1 + 2 * desc->gap_extend) <= 127;
  const bool flow = single && ((kalg == MSA_ALG_SWL || kalg == MSA_ALG_SWL0) ?
                               (out_mode == MSA_OUT_H || (out_mode == MSA_OUT_NONE && !tp)) : (aff_ok || got_ok)) &&
                    desc->m[0] > 0 && flow_lds <= device_lds_max();
  P->flow = flow;
  P->flow2 = flow && (out_mode == MSA_OUT_H || aff);
  {
    // SW two-pass plans reduce their pair result inside the launch when the cell index fits 32 bits
    // (MSA_FUSED_REDUCE=0: the reduce_blocks_kernel launch, for A/B)
    const char* fr = std::getenv("MSA_FUSED_REDUCE");
    const int64_t cells1 = (desc->m[0] + 1) * (desc->n[0] + 1);
    P->fused_reduce = P->flow2 && kalg != MSA_ALG_REF1 && cells1 < (int64_t(1) << 32) && !(fr && fr[0] == '0');
  }
  const int W = flow ? FL_W : (single ? MSA_WAVES_SINGLE : MSA_WAVES_BATCH);
  P->W = W;
  const int KS = flow ? 16 : (single ? ks_single(kalg) : ks_batch(kalg));
  P->KS = KS;
  P->threads = (flow ? W + 2 : W + 1 + (single ? 1 : 0)) * 64;
  // rows per lane of the flow kernel (two-pass plans): 2 halves the inter-wave hand-offs per row
  // (SW linear with H; the reference's Gotoh and SW affine with direction bytes; MSA_FLOW_GOT_R=1 /
  // MSA_FLOW_AFF_R=1 keep one row for those two)
  static const int got_r = [] {
    const char* e = std::getenv("MSA_FLOW_GOT_R");
    return (e && std::atoi(e) == 1) ? 1 : 2;
  }();
  static const int aff_r = [] {
    const char* e = std::getenv("MSA_FLOW_AFF_R");
    return (e && std::atoi(e) == 1) ? 1 : 2;
  }();
  P->R = !flow ? 1 : kalg == MSA_ALG_REF1 ? got_r : kalg == MSA_ALG_SWA ? aff_r : (out_mode == MSA_OUT_H ? 2 : 1);
  P->fn = flow ? pick_flow(kalg, out_mode == MSA_OUT_NONE, P->flow2, tp, P->R, desc->match >= 0 && desc->mismatch >= 0)
               : pick_kernel(kalg, out_mode, tp, single);
  if (!P->fn) { delete P; return MSA_ERR_UNSUPPORTED; }
  P->nc = nc_of(kalg);
  const int band = (kalg == MSA_ALG_NWA) ? desc->band : -1;
  msa_kparams& kp = P->kp;
  std::memset(&kp, 0, sizeof(kp));
  kp.alg = kalg;
  kp.out = out_mode;
  kp.match = desc->match;
  kp.mismatch = desc->mismatch;
  kp.gap_open = desc->gap_open;
  kp.gap_ext = desc->gap_extend;
  if (kalg == MSA_ALG_SWL || kalg == MSA_ALG_SWL0 || kalg == MSA_ALG_SWLP) kp.gap_open = kp.gap_ext = desc->gap_extend;
  kp.h = desc->gap_open - desc->gap_extend;
  kp.start_type = desc->start_type;
  kp.band = band;
  kp.code_whole = (flow && code_whole) ? 1 : 0;
  kp.single = single ? 1 : 0;
  kp.n_pairs = (int)desc->n_pairs;
  if (kalg == MSA_ALG_NWA && kp.h < 0) { delete P; return MSA_ERR_UNSUPPORTED; }
  // geometry
  int64_t stripe0 = 0, off = 0, cod_bytes = 0;
  std::map<std::pair<int64_t, int64_t>, int64_t> seg_of;
  int max_S = 0, max_P = 0;
  P->pairs.resize(desc->n_pairs);
  for (int64_t p = 0; p < desc->n_pairs; ++p) {
    const int64_t m = desc->m[p], n = desc->n[p];
    if (m <= 0 || n <= 0 || m > (1 << 26) || n > (1 << 26)) { delete P; return MSA_ERR_ARG; }
    if (kalg == MSA_ALG_SWL || kalg == MSA_ALG_SWL0 || kalg == MSA_ALG_SWLP) {
      // shifted recurrence G = H + g*(i+j): G must stay far from the -2^30 sentinel
      // and from int32 overflow; the profile byte holds score + 2g
      const int64_t g = kp.gap_open;
      const int64_t top = g * (m + n + 2) + (int64_t)std::max({0, kp.match, kp.mismatch}) * std::min(m, n);
      const int64_t sm = kp.match + 2 * g, sx = kp.mismatch + 2 * g;  // profile bytes (int8)
      if (g < 0 || top >= (int64_t(1) << 29) || sm > 127 || sm < -128 || sx > 127 || sx < -128) {
        delete P;
        return MSA_ERR_UNSUPPORTED;
      }
    }
    if (kalg == MSA_ALG_SWA) {
      // int8 profile bytes; H stays far from the -2^30 sentinel and from int32 overflow
      const int64_t top = (int64_t)std::max({0, kp.match, kp.mismatch}) * std::min(m, n);
      if (kp.match < -128 || kp.match > 127 || kp.mismatch < -128 || kp.mismatch > 127 || kp.gap_open < 0 ||
          kp.gap_ext < 0 || top >= (int64_t(1) << 29)) {
        delete P;
        return MSA_ERR_UNSUPPORTED;
      }
    }
    if (band >= 0 && std::llabs(m - n) > band) { delete P; return MSA_ERR_ARG; }
    const int S = (int)((m + 63) / 64);
    int pmax = 0;
    for (int k = 0; k < S; ++k) {
      StripeGeom g;
      stripe_geom(k, (int)m, (int)n, band, g, KS);
      pmax = std::max(pmax, g.P * (KS / MSA_K));  // in 16-step layout blocks
    }
    if (flow) {  // the flow kernels' own geometry (R rows per lane)
      const int SR = (int)((m + 64 * P->R - 1) / (64 * P->R));
      for (int k = 0; k < SR; ++k) pmax = std::max(pmax, fl_P(k, (int)m, (int)n, P->R));
    }
    msa_pair_desc& pd = P->pairs[p];
    pd.a_off = desc->a_off[p];
    pd.b_off = desc->b_off[p];
    pd.m = (int)m;
    pd.n = (int)n;
    pd.stripe0 = (int)stripe0;
    pd.pmax = pmax;
    pd.out_off = off;
    // padded column-code segment, shared by pairs with the same column sequence
    {
      const auto key = std::make_pair(pd.b_off, (int64_t)n);
      auto it = seg_of.find(key);
      if (it == seg_of.end()) {
        it = seg_of.emplace(key, cod_bytes).first;
        msa_pair_desc sd{};
        sd.b_off = pd.b_off;
        sd.n = (int)n;
        sd.cod_off = cod_bytes;
        P->segs.push_back(sd);
        cod_bytes += ((n + 2 * MSA_CPAD) + 63) & ~int64_t(63);
      }
      pd.cod_off = it->second;
    }
    // R = 2 layout: (m+127)/128 stripes of pmax * 2048 cells
    const int64_t cells = std::max((int64_t)S * pmax * MSA_K * 64,
                                   (int64_t)((m + 64 * P->R - 1) / (64 * P->R)) * pmax * MSA_K * 64 * P->R);
    off += (cells + 63) & ~int64_t(63);
    stripe0 += S;
    max_S = std::max(max_S, S);
    max_P = std::max(max_P, pmax);
  }
  P->total_stripes = stripe0;
  P->cells_elems = off;
  kp.sched_cap = single ? W : max_S;
  kp.lds_code_bytes = 0;  // column codes come from the staged global copies (stage_codes_kernel)
  P->cod_copy = cod_bytes;
  kp.lds_row_words = single ? 0 : (((max_P * MSA_K + MSA_ROWOFF + 32) + 15) & ~15);
  if (single) {
    const int S = (int)((desc->m[0] + 64 * P->R - 1) / (64 * P->R));
    kp.n_items = (S + W - 1) / W;
  } else {
    kp.n_items = (kalg == MSA_ALG_SWLP) ? (int)((desc->n_pairs + 1) / 2) : (int)desc->n_pairs;
    // A batch with fewer pairs (couples) than two workgroups per CU leaves CUs idle while each
    // workgroup walks its pair's whole stripe chain (C4 at 8 GPUs: 128 pairs per rank).  Then
    // every pair is split into items of W stripes, chained through granules (kp.single == 3):
    // a pair's stripes run on several CUs at once.  Measured (C4 shape, 4k x 4k, packed
    // couples, ms): 64 couples 1.72 -> 0.80, 128: 1.39, 256: 2.38.  Items of C > W stripes
    // (fewer items, the waves cycling inside one) were slower at every count -- 128 couples
    // with C = 16: 1.81, 256 with C = 32: 2.46 -- since an item's second round of stripes waits
    // for its first to finish, so a pair's chain grows to ~(S / W) stripe lengths; kp.chunk_c
    // stays general (the kernel runs any multiple of W) but the plan uses C = W.  Items of
    // four stripes (a 4-wave instantiation) were slower too: 128 pairs 0.81 -> 1.01 ms.
    bool eq_m = true;
    for (int64_t p = 1; p < desc->n_pairs; ++p) eq_m = eq_m && desc->m[p] == desc->m[0];
    const int S0 = (int)((desc->m[0] + 63) / 64);
    const int slots = 2 * device_cus();
    if (eq_m && kp.n_items < slots && S0 >= 2 * W && band < 0) {
      const int C = W;
      {
        kp.single = 3;
        kp.chunk_c = C;
        kp.groups = (S0 + C - 1) / C;
        kp.n_items *= kp.groups;
        kp.sched_cap = C;
        // the wave W-1 -> wave 0 wrap link inside an item goes through the LDS row buffer
        if (C <= W) kp.lds_row_words = 0;
      }
    }
  }
  // Packed score-only batches (C4): cflow_kernel (msa_cflow.hip) -- items of CF_W stripes of one couple,
  // chained through granules, claimed item-major -- for batches of fewer couples than two per CU whose code
  // rows fit LDS.  MSA_C4_KERNEL=lockstep / =cflow (diagnostics) force either kernel.
  if (kalg == MSA_ALG_SWLP && !single) {
    // (read per plan, not cached: a test forces either kernel in one process)
    const char* c4k = std::getenv("MSA_C4_KERNEL");
    const bool lockstep = c4k && std::strcmp(c4k, "lockstep") == 0;
    int64_t nmax = 0, mmax = 0;
    for (int64_t p = 0; p < desc->n_pairs; ++p) {
      nmax = std::max(nmax, desc->n[p]);
      mmax = std::max(mmax, desc->m[p]);
    }
    const int L8 = fl_code_bytes((int)nmax);
    const size_t clds = (size_t)(FL_FLAGS + (CF_W + 1) * 256) * 4 + (size_t)FL_NCOPY * (L8 + 16);
    // a batch with at least two couples per CU keeps the lock-step kernel's SIMDs busy (its 8 waves per
    // workgroup hide each other's step latency): measured on C4's shape, 1,024 pairs 2.39 ms lock-step vs
    // 2.73 cflow; 512 pairs 2.07 vs 1.58, 128 pairs 0.72 vs 0.55 (profiles/r05_c4_*_bench.json)
    const int ncpl = (int)((desc->n_pairs + 1) / 2);
    const bool force_cflow = c4k && std::strcmp(c4k, "cflow") == 0;
    if (!lockstep && clds <= 96 * 1024 && (force_cflow || ncpl < 2 * device_cus())) {
      P->cflow = true;
      P->fn = cflow_kernel<CF_W>;
      P->W = CF_W;
      P->KS = 16;
      P->threads = (CF_W + 1) * 64;
      kp.single = 0;
      kp.lds_code_bytes = L8;
      kp.code_whole = 1;
      const int G = (int)(((mmax + 63) / 64 + CF_W - 1) / CF_W);
      kp.n_items = ncpl * G;
      kp.sched_cap = 0;
      kp.lds_row_words = 0;
    }
  }
  const size_t lds_ints = 16 + (size_t)kp.sched_cap * 8 + (size_t)(2 * W + 1) * P->nc * MSA_RING +
                          (size_t)P->nc * kp.lds_row_words +
                          (single ? (size_t)4 * (MSA_CRING / 4 + 16) : 0);  // code ring
  P->lds_bytes = lds_ints * 4;
  if (P->cflow) P->lds_bytes = (size_t)(FL_FLAGS + (CF_W + 1) * 256) * 4 + (size_t)FL_NCOPY * (kp.lds_code_bytes + 16);
  if (flow) {
    kp.lds_code_bytes = fl_code_bytes((int)desc->n[0]);
    P->lds_bytes = flow_lds;
    // pass-2 blocks: FL_P2INTS ints per wave (inputs + column codes staged in LDS)
    if (P->flow2) P->lds_bytes = std::max(flow_lds, (size_t)(FL_W + 2) * fl_p2ints(FL_PS) * 4);
  }
  if (P->lds_bytes > device_lds_max()) {
    std::fprintf(stderr, "msa: problem needs %zu B of LDS per workgroup (> %zu B, the device's limit)\n",
                 P->lds_bytes, device_lds_max());
    delete P;
    return MSA_ERR_UNSUPPORTED;
  }
  const int occ = kernel_shape(P->fn, P->threads, P->lds_bytes);
  if (occ < 0) {
    delete P;
    return MSA_ERR_HIP;
  }
  const int ncu = device_cus();
  const int cap = ncu * (P->cflow ? occ : std::min(occ, 2));
  P->grid = std::max(1, std::min(kp.n_items, cap));
  if (flow) {
    // Items go to the 8 XCDs in runs of G consecutive items, round-robin (workgroup b takes
    // tickets of XCD b % 8 first, round-robin placement puts it there): a run hands off inside
    // one L2.  When an XCD's share fits its workgroups (chunk <= CUs per XCD) the runs are 8
    // contiguous chunks (7 seams).  A longer pair keeps more items in flight than an XCD has
    // workgroups (97k: ~240 of 381 items at once, 32 CUs per XCD): contiguous chunks would then
    // serialize -- chunk c + 1 waits for chunk c's last items, which wait for a free workgroup of
    // XCD c (measured 28 ms for 97k x 97k) -- so the runs shrink to G = CUs per XCD / 8 and every
    // XCD holds its share of the items in flight.  Speed only: an item only waits on an earlier
    // one and every workgroup is resident (one per CU, grid <= CUs), whatever the placement.
    const int per_xcd = std::max(1, ncu / 8);
    const int chunk = (kp.n_items + 7) / 8;
    kp.sched_cap = chunk <= per_xcd ? chunk : std::max(1, per_xcd / 8);  // G
    P->grid = 8 * std::max(1, std::min(chunk, per_xcd));
    // two-pass: the remaining CUs run pass-2 blocks inside the same launch, one flow workgroup per
    // CU (the LDS floor): a pass-2 workgroup sharing a CU with a pass-1 one takes issue slots from its
    // chain waves.  A long pair keeps ~n / (W lag) items in flight (97k: ~240), so pass 1 may hold
    // most CUs; then every CU also gets a pass-2 workgroup (two per CU), whose waves issue at the
    // lowest priority, behind the pass-1 waves (s_setprio, msa_flow.hip).  MSA_FLOW_LDS_MIN
    // (bytes, diagnostic) overrides the one-per-CU floor.
    P->nflow = P->grid;
    if (P->flow2) {
      static const long lds_min = [] {
        const char* e = std::getenv("MSA_FLOW_LDS_MIN");
        return e ? std::strtol(e, nullptr, 10) : 80 * 1024 + 1024;
      }();
      if (P->nflow > ncu / 2) {
        // pass 1 holds most CUs: pass 2 runs as a launch of its own behind it (flow_fill_kernel), whose
        // register budget is the pass-2 code's alone (97k x 97k: 23 -> ~16 ms)
        P->grid = P->nflow;
        P->fill_fn = pick_fill(kalg, tp, P->R, desc->match >= 0 && desc->mismatch >= 0);
        if (!P->fill_fn) { delete P; return MSA_ERR_UNSUPPORTED; }
        P->fill_lds = (size_t)FL_FILLW * fl_p2ints(FL_PS_FILL) * 4;
        P->ps = FL_PS_FILL;  // its blocks are segments of FL_PS_FILL phases (pass 1 saves state that often)
        const int focc = kernel_shape(P->fill_fn, FL_FILLW * 64, P->fill_lds);
        if (focc < 0) { delete P; return MSA_ERR_HIP; }
        P->fill_grid = ncu * std::max(1, std::min(focc, 8));
        P->lds_bytes = std::max(P->lds_bytes, (size_t)std::max(0L, lds_min));
      } else {
        P->grid = std::max(P->grid + 8, 8 * per_xcd);
        P->lds_bytes = std::max(P->lds_bytes, (size_t)std::max(0L, lds_min));
      }
      if (kernel_shape(P->fn, P->threads, P->lds_bytes) < 0) {
        delete P;
        return MSA_ERR_HIP;
      }
    }
  }
  // Banded single pair (C3-type): the band has only ~9 stripes in flight, so the exact
  // launch is one long chain of ~S x 8 phases.  Chunked mode runs it as n_chunks
  // independent chains of chunk_c (+ warm-up) stripes at once (rank convergence,
  // msa_kernels.hip header), with the exact launch kept behind it as the fallback.
// Measured on MI355X for C3 (profiles/r03_c3_*): (warm, chunk) = (24, 24) 0.925 ms, (24, 12)
// 0.768, (16, 16) 0.733, (20, 10) 0.678 -- and (16, 8) did not converge in every chunk (the
// exact fallback ran: 18.3 ms).  C3's pair converges within ~900 rows, its synthetic mutated
// copy within ~1,024; 20 stripes = 1,280 rows.  Chunk workgroups of 4 or 12 waves instead of 8:
// 0.90 and 0.72 ms (8: 0.67).  (20, 6) = 254 chunks, one per CU: not every chunk converged
// (17.4 ms with the fallback) -- more start rows, and the slowest needs more than 1,280 rows.
#ifndef MSA_CHUNK_WARM
#define MSA_CHUNK_WARM 20  // warm-up stripes
#endif
#ifndef MSA_CHUNK_MIN
#define MSA_CHUNK_MIN 10   // stripes per chunk, at least
#endif
  constexpr int kWarm = MSA_CHUNK_WARM;
  // Banded single pair (C3-type): band_kernel (msa_band.hip), flag-synchronised chains of 4-stripe
  // items.  The exact launch chains all of the pair's items; chunked (rank convergence, >= 4
  // chunks) runs chunks of C output stripes, each started W stripes early from a guessed row, with
  // the exact launch queued behind as the fallback.  MSA_BAND_WARM / MSA_BAND_CHUNK (diagnostic)
  // override the warm-up and chunk stripes (multiples of 4).
  if (single && kalg == MSA_ALG_NWA && band >= 0 && (out_mode == MSA_OUT_H || out_mode == MSA_OUT_NONE)) {
    const int m0 = (int)desc->m[0], n0 = (int)desc->n[0];
    const int S = (m0 + 63) / 64;
    const int L8 = bk_code_bytes(m0, n0, band);
    const size_t blds = bk_lds_bytes(L8);
    const int bocc = (blds <= device_lds_max()) ? kernel_shape(band_kernel, (BK_W + 1) * 64, blds) : -1;
    if (bocc > 0) {
      // diagnostic knobs, read once per process; a warm-up shorter than one item (BK_W stripes) gives
      // chunk_check nothing to compare (checkpoint slot 2c is never written): chunking is then off
      static const int warm = [] {
        const char* e = std::getenv("MSA_BAND_WARM");
        return std::max(0, (e ? std::atoi(e) : kWarm) / BK_W * BK_W);
      }();
      static const int cc = [] {
        const char* e = std::getenv("MSA_BAND_CHUNK");
        return std::max(BK_W, (e ? std::atoi(e) : 12) / BK_W * BK_W);
      }();
      const int nch = (S + cc - 1) / cc;
      msa_kparams ek = kp;  // the exact launch
      ek.single = 1;
      ek.groups = (S + BK_W - 1) / BK_W;
      ek.n_items = ek.groups;
      ek.chunk_c = S;
      ek.chunk_warm = 0;
      ek.lds_code_bytes = L8;
      ek.sched_cap = 0;
      P->band_k = true;
      P->fn = band_kernel;
      P->W = BK_W;
      P->KS = 16;
      P->threads = (BK_W + 1) * 64;
      P->lds_bytes = blds;
      P->grid = std::max(1, std::min(ek.n_items, ncu * bocc));
      kp = ek;
      P->band_items = ek.n_items;
      if (nch >= 4 && out_mode == MSA_OUT_H && warm >= BK_W) {
        P->chunked = true;
        P->n_chunks = nch;
        P->fb_kp = ek;
        P->fb_fn = band_kernel;
        P->fb_grid = P->grid;
        P->fb_threads = P->threads;
        P->fb_lds = blds;
        kp.single = 2;
        kp.chunk_c = cc;
        kp.chunk_warm = warm;
        // item slots per chunk: its warm-up + output stripes in items of BK_W (a chunk whose warm-up
        // would reach the matrix border starts at row 0 instead -- band_kernel -- and so has more)
        int ipc = 1;
        for (int c2 = 0; c2 < nch; ++c2) {
          const int ks0 = c2 * cc, ke = std::min(S, ks0 + cc);
          int kb = ks0 - warm;
          if (kb < 0 || kb * 64 <= band + 64) kb = 0;
          ipc = std::max(ipc, (ke - kb + BK_W - 1) / BK_W);
        }
        kp.groups = ipc;
        kp.n_items = nch * kp.groups;
        P->grid = std::max(1, std::min(kp.n_items, ncu * bocc));
        P->band_items = std::max(P->band_items, kp.n_items);
        P->ckw = (2 * band + 1 + 3) & ~3;
        // int16 chunk cells: a chunk >= 1 starts from its guessed row (H <= -h, inside the band >= -h - g band)
        // at row r0 > band + 64, so an in-band cell (i, j) is reached from (r0, j - i + r0), in the band, along
        // its diagonal: -h - g band <= H <= i - r0 - h.  Both bounds fit int16 with room when rows + h + g band
        // stays under 30,000 (C3: 2,112 + 2 + 512); the cells are then written as 2 B, and chunk_add_kernel
        // reads 2 B and writes 4 B per cell instead of reading and re-writing 4 B.  MSA_BAND_H16=0 (diagnostic)
        // keeps int32 cells.
        static const bool h16_on = [] {
          const char* e = std::getenv("MSA_BAND_H16");
          return !(e && std::atoi(e) == 0);
        }();
        const long long rows = (long long)(warm + cc) * 64 + 64;
        P->h16 = h16_on && kp.h >= 0 && kp.gap_ext >= 0 && rows + kp.h + (long long)kp.gap_ext * band <= 30000;
      }
    }
  }
  if (single && kalg == MSA_ALG_NWA && band >= 0 && (out_mode == MSA_OUT_H || out_mode == MSA_OUT_NONE) &&
      !P->band_k) {
    const int S = (int)((desc->m[0] + 63) / 64);
    const int cc = std::max(MSA_CHUNK_MIN, (S + ncu - 1) / ncu);
    const int nch = (S + cc - 1) / cc;
    kfn_t cfn = pick_kernel(kalg, out_mode, 0, false);
    if (nch >= 4 && cfn) {
      P->chunked = true;
      P->n_chunks = nch;
      P->fb_kp = kp;
      P->fb_fn = P->fn;
      P->fb_grid = P->grid;
      P->fb_threads = P->threads;
      P->fb_lds = P->lds_bytes;
      kp.single = 2;
      kp.chunk_c = cc;
      kp.chunk_warm = kWarm;
      kp.n_items = nch;
      kp.sched_cap = cc + kWarm;
      kp.lds_row_words = ((max_P * MSA_K + MSA_ROWOFF + 32) + 15) & ~15;
      P->fn = cfn;
      P->W = MSA_WAVES_BATCH;
      P->threads = (MSA_WAVES_BATCH + 1) * 64;
      P->lds_bytes = (16 + (size_t)kp.sched_cap * 8 + (size_t)(2 * MSA_WAVES_BATCH + 1) * P->nc * MSA_RING +
                      (size_t)P->nc * kp.lds_row_words) * 4;
      const int occ2 = (P->lds_bytes > device_lds_max()) ? -1 : kernel_shape(P->fn, P->threads, P->lds_bytes);
      if (occ2 < 0) {
        delete P;
        return MSA_ERR_UNSUPPORTED;
      }
      // every chunk at once (one workgroup each); more chunks than slots just queue
      P->grid = std::max(1, std::min(nch, ncu * std::min(occ2, 2)));
      P->ckw = (2 * band + 1 + 3) & ~3;
    }
  }
  // device buffers
  auto fail = [&](void) { msa_plan_destroy(P); return MSA_ERR_HIP; };
  if (!P->alloc(&P->d_pairs, sizeof(msa_pair_desc) * P->pairs.size())) return fail();
  if (hipMemcpy(P->d_pairs, P->pairs.data(), sizeof(msa_pair_desc) * P->pairs.size(), hipMemcpyHostToDevice) !=
      hipSuccess)
    return fail();
  if (!P->alloc(&P->d_meta, sizeof(msa_stripe_meta) * std::max<int64_t>(1, P->total_stripes)))
    return fail();
  if (hipMemset(P->d_meta, 0, sizeof(msa_stripe_meta) * std::max<int64_t>(1, P->total_stripes)) != hipSuccess)
    return fail();
  if (!P->alloc(&P->d_ticket, 4 * MSA_NTICKET)) return fail();
  if (!P->alloc(&P->d_err, 64) || hipMemset(P->d_err, 0, 64) != hipSuccess) return fail();
  if (!P->alloc(&P->d_cod, (size_t)MSA_NCOPY * P->cod_copy + 64)) return fail();
  if (!P->alloc(&P->d_segs, sizeof(msa_pair_desc) * P->segs.size())) return fail();
  if (hipMemcpy(P->d_segs, P->segs.data(), sizeof(msa_pair_desc) * P->segs.size(), hipMemcpyHostToDevice) !=
      hipSuccess)
    return fail();
  if (!P->alloc(&P->d_res, sizeof(PairResult) * desc->n_pairs)) return fail();
  if (!P->alloc(&P->d_sum, 64)) return fail();
  const int single_items = P->chunked ? P->fb_kp.n_items : kp.n_items;  // single-mode launch's items
  if (P->band_k && P->band_items > 1) {
    // band_kernel: item t publishes (Z, F~) of its last row into slot t (chunked and exact launches)
    P->gbuf_stride = (int)(((desc->n[0] + 2 * MSA_GOFF + 16) + 15) & ~15);
    const size_t gb = (size_t)P->band_items * 2 * P->gbuf_stride * sizeof(unsigned long long);
    if (!P->alloc(&P->d_gbuf, gb)) return fail();
    if (hipMemset(P->d_gbuf, 0, gb) != hipSuccess) return fail();
  } else if (P->cflow) {
    // cflow_kernel: item t publishes the last link of its stripes into slot t (read by item t + couples)
    int64_t nmax = 0;
    for (int64_t p = 0; p < desc->n_pairs; ++p) nmax = std::max(nmax, desc->n[p]);
    P->gbuf_stride = (int)(((nmax + 2 * MSA_GOFF + 16) + 15) & ~15);
    const size_t gb = (size_t)kp.n_items * P->gbuf_stride * sizeof(unsigned long long);
    if (!P->alloc(&P->d_gbuf, gb)) return fail();
    if (hipMemset(P->d_gbuf, 0, gb) != hipSuccess) return fail();
  } else if ((single || kp.single == 3) && single_items > 1) {
    int64_t nmax = 0;
    for (int64_t p = 0; p < desc->n_pairs; ++p) nmax = std::max(nmax, desc->n[p]);
    P->gbuf_stride = (int)(((nmax + 2 * MSA_GOFF + 16) + 15) & ~15);
    // (mode 3: item k publishes into slot k, so one slot per item)
    const size_t gb = (size_t)(kp.single == 3 ? single_items : single_items - 1) * P->nc * P->gbuf_stride *
                      sizeof(unsigned long long);
    if (!P->alloc(&P->d_gbuf, gb)) return fail();
    if (hipMemset(P->d_gbuf, 0, gb) != hipSuccess) return fail();
  }
  if (P->flow2) {
    const int S = (int)((desc->m[0] + 64 * P->R - 1) / (64 * P->R));
    P->brw = 16 * P->pairs[0].pmax + 16;
    P->nseg = (P->pairs[0].pmax + P->ps - 1) / P->ps;
    P->nblk = S * P->nseg;
    // pass-2 blocks in expected readiness order: stripe s starts ~6.5 phases after
    // stripe s-1, and segment seg is complete ps (seg + 1) phases after its start
    std::vector<int> order(P->nblk);
    std::vector<double> key(P->nblk);
    for (int b = 0; b < P->nblk; ++b) {
      order[b] = b;
      key[b] = (P->R == 2 ? 7.5 : 6.5) * (b / P->nseg) + (double)P->ps * (b % P->nseg + 1);
    }
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return key[x] < key[y]; });
    // (affine: the F~ bottom rows follow the Z rows; a snapshot is 4 values per lane)
    const bool two = P->kp.alg == MSA_ALG_SWA || P->kp.alg == MSA_ALG_REF1;
    const size_t brb = sizeof(unsigned long long) * (size_t)S * P->brw * (two ? 2 : 1);
    const size_t snb = sizeof(unsigned long long) * (size_t)P->nblk * (two ? 128 * (P->R + 1) : 128 * P->R);
    if (!P->alloc(&P->d_br, brb) || hipMemset(P->d_br, 0, brb) != hipSuccess) return fail();
    if (!P->alloc(&P->d_snap, snb) || hipMemset(P->d_snap, 0, snb) != hipSuccess) return fail();
    if (!P->alloc(&P->d_blk, sizeof(int4) * (size_t)P->nblk)) return fail();
    if (!P->alloc(&P->d_order, sizeof(int) * (size_t)P->nblk)) return fail();
    if (hipMemcpy(P->d_order, order.data(), sizeof(int) * (size_t)P->nblk, hipMemcpyHostToDevice) != hipSuccess)
      return fail();
  }
  if (P->chunked) {
    const size_t ckb = sizeof(int) * (size_t)P->n_chunks * 4 * P->ckw;
    // entries a chunk never writes (outside the band row / matrix) read as -inf
    if (!P->alloc(&P->d_ck, ckb) || hipMemset(P->d_ck, 0xC0, ckb) != hipSuccess) return fail();
    if (!P->alloc(&P->d_dk, sizeof(int) * P->n_chunks) || !P->alloc(&P->d_okk, sizeof(int) * P->n_chunks) ||
        !P->alloc(&P->d_skip, 64))
      return fail();
    if (P->h16 && out_mode == MSA_OUT_H) {
      const msa_pair_desc& pd = P->pairs[0];
      const int S = (int)((pd.m + 63) / 64);
      const size_t per = (size_t)pd.pmax * MSA_K * 64;
      if (S > P->kp.chunk_c && !P->alloc(&P->d_h16, sizeof(int16_t) * per * (size_t)(S - P->kp.chunk_c))) return fail();
    }
    if (!P->d_h16) P->h16 = false;
  }
  if (hipEventCreate(&P->ev0) != hipSuccess || hipEventCreate(&P->ev1) != hipSuccess) return fail();
  // the memsets above went to the null stream, which does not order the non-blocking
  // streams runs are launched on: finish them before the plan can run anywhere
  if (hipStreamSynchronize(nullptr) != hipSuccess) return fail();
  *out = P;
  return MSA_OK;
}

void msa_plan_destroy(msa_plan* P) {
  if (!P) return;
  // the plan's blocks go back to the pool: every run, traceback and score copy it
  // queued (on whichever streams) must be complete
  for (hipStream_t s : P->streams) (void)hipStreamSynchronize(s);
  for (auto& b : P->blocks) dev_pool().put(b.first, b.second);
  if (P->ev0) (void)hipEventDestroy(P->ev0);
  if (P->ev1) (void)hipEventDestroy(P->ev1);
  delete P;
}

int msa_plan_cells_size(const msa_plan* P, int64_t* elems) {
  if (!P || !elems) return MSA_ERR_ARG;
  *elems = (P->d.cells == MSA_CELLS_NONE) ? 0 : P->cells_elems;
  return MSA_OK;
}

int64_t msa_plan_stripes(const msa_plan* P) { return P ? P->total_stripes : 0; }

int msa_plan_pair_layout(const msa_plan* P, int64_t pair, int64_t* out4) {
  if (!P || !out4 || pair < 0 || pair >= (int64_t)P->pairs.size()) return MSA_ERR_ARG;
  const msa_pair_desc& pd = P->pairs[(size_t)pair];
  out4[0] = pd.stripe0;
  out4[1] = pd.pmax;
  out4[2] = pd.out_off;
  out4[3] = P->KS | ((int64_t)P->R << 16);  // bits 16+: rows per lane of the layout (0 = 1)
  return MSA_OK;
}

int msa_plan_run(msa_plan* P, const uint8_t* dA, const uint8_t* dB, void* c0, void* c1, void* c2, void* stream) {
  if (!P || !dA || !dB) return MSA_ERR_ARG;
  if (P->d.cells != MSA_CELLS_NONE && !c0) return MSA_ERR_ARG;
  if (P->d.cells == MSA_CELLS_TAB && (!c1 || !c2)) return MSA_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  P->note_stream(st);
  KArgs a;
  std::memset(&a, 0, sizeof(a));
  a.kp = P->kp;
  // epochs are process-wide, so granules left in a pooled block by an earlier plan
  // can never carry the epoch a new run polls for
  uint32_t ep = g_epoch.fetch_add(1) + 1;
  if (ep == 0) ep = g_epoch.fetch_add(1) + 1;
  P->epoch = ep;
  a.kp.epoch = ep;
  a.A = dA;
  a.B = dB;
  a.pairs = P->d_pairs;
  a.meta = P->d_meta;
  a.ticket = P->d_ticket;
  a.err = P->d_err;
  a.gbuf = P->d_gbuf;
  a.gbuf_stride = P->gbuf_stride;
  if (P->d.cells == MSA_CELLS_DIR) a.outDir = (uint8_t*)c0;
  else a.outH = (int32_t*)c0;
  a.outT2 = (int32_t*)c1;
  a.outT3 = (int32_t*)c2;
  a.stamps = P->stamps;
  a.cod = P->d_cod;
  a.cod_copy = P->cod_copy;
  a.br = P->d_br;
  a.snap = P->d_snap;
  a.blk = P->d_blk;
  a.border = P->d_order;
  a.nflow = P->nflow;
  a.best_key = P->fused_reduce ? reinterpret_cast<unsigned long long*>(P->d_ticket + MSA_TK_BEST) : nullptr;
  a.brw = P->brw;
  a.nseg = P->nseg;
  a.ps_shift = __builtin_ctz((unsigned)P->ps);
  a.nblk = P->nblk;
  {
    const unsigned virt = (P->kp.alg == MSA_ALG_SWL || P->kp.alg == MSA_ALG_SWL0 || P->kp.alg == MSA_ALG_SWLP ||
                           P->kp.alg == MSA_ALG_SWA) ? MSA_VIRT_CODE : 0u;
    // about two output words per thread for one long pair (64 x 256 threads took 22 us for
    // C3's 97k columns, 24 dependent rounds each), at least 64 workgroups per segment
    const int64_t words = MSA_NCOPY * (P->cod_copy / 4) / std::max<int64_t>(1, (int64_t)P->segs.size());
    const unsigned gx = (unsigned)std::min<int64_t>(1024, std::max<int64_t>(64, words / 512));
    hipLaunchKernelGGL(stage_codes_kernel, dim3(gx, (unsigned)P->segs.size()), dim3(256), 0, st, dB, P->d_segs,
                       (int)P->segs.size(), P->d_cod, (long long)P->cod_copy, virt, P->d_ticket);
    HIPCHK(hipGetLastError());
  }
  const bool ev = P->timing;  // timing events are instrumentation: msa_plan_set_timing
  if (ev) HIPCHK(hipEventRecord(P->ev0, st));
  P->timed = ev;
  if (P->chunked) {
    a.ck = P->d_ck;
    a.ckw = P->ckw;
    if (P->h16 && P->d.cells == MSA_CELLS_H) a.outH16 = P->d_h16;
  }
  hipLaunchKernelGGL(P->fn, dim3(P->grid), dim3(P->threads), P->lds_bytes, st, a);
  HIPCHK(hipGetLastError());
  if (P->chunked) {
    // verify every chunk's constant, add the prefix of the constants to its cells; then the
    // exact single-mode launch, which returns at once when *skip == 1
    // (a fused check + add launch, roles by arrival ticket, the adders' first loads in flight
    // across the checks, measured slower: C3 0.94 vs 0.67 ms)
    hipLaunchKernelGGL(chunk_check_kernel, dim3(P->n_chunks), dim3(256), 0, st, (const int*)P->d_ck, P->ckw, P->d_dk,
                       P->d_okk);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(chunk_add_kernel, dim3(32, P->n_chunks), dim3(256), 0, st,
                       P->d.cells == MSA_CELLS_H ? a.outH : (int32_t*)nullptr, (const int16_t*)a.outH16,
                       (const msa_pair_desc*)P->d_pairs,
                       P->d_meta, (const int*)P->d_dk, (const int*)P->d_okk, P->n_chunks, P->kp.chunk_c, P->d_skip,
                       P->d_ticket);
    HIPCHK(hipGetLastError());
    KArgs b = a;
    b.kp = P->fb_kp;
    // its own epoch: the band kernel's chunked launch leaves granules of this run's epoch in the
    // slots the exact launch reads
    uint32_t ep2 = g_epoch.fetch_add(1) + 1;
    if (ep2 == 0) ep2 = g_epoch.fetch_add(1) + 1;
    b.kp.epoch = ep2;
    b.ck = nullptr;
    b.outH16 = nullptr;  // the exact launch writes every cell as int32
    b.skip = P->d_skip;
    hipLaunchKernelGGL(P->fb_fn, dim3(P->fb_grid), dim3(P->fb_threads), P->fb_lds, st, b);
    HIPCHK(hipGetLastError());
  }
  if (P->fill_fn) {  // long pair: pass 2 behind pass 1
    hipLaunchKernelGGL(P->fill_fn, dim3(P->fill_grid), dim3(FL_FILLW * 64), P->fill_lds, st, a);
    HIPCHK(hipGetLastError());
  }
  if (ev) HIPCHK(hipEventRecord(P->ev1, st));
  if (P->flow2 && P->kp.alg != MSA_ALG_REF1) {  // (Gotoh: the final state is in the last stripe's meta)
    if (!P->fused_reduce) {  // (fused: the pass-2 blocks folded the result into the best-cell key)
      hipLaunchKernelGGL(reduce_blocks_kernel, dim3(1), dim3(1024), 0, st, (const int4*)P->d_blk, P->nblk, P->d_res);
      HIPCHK(hipGetLastError());
    }
    return MSA_OK;
  }
  const int sw = (P->kp.alg == MSA_ALG_SWL || P->kp.alg == MSA_ALG_SWL0 || P->kp.alg == MSA_ALG_SWLP ||
                  P->kp.alg == MSA_ALG_SWA) ? 1 : 0;
  const int np = (int)P->d.n_pairs;
  hipLaunchKernelGGL(reduce_pairs_kernel, dim3(np), dim3(64), 0, st, P->d_pairs, P->d_meta, np, sw,
                     P->d_res);
  HIPCHK(hipGetLastError());
  return MSA_OK;
}

#ifdef MSA_STAMPS
extern "C" int msa_debug_stamps(msa_plan* P, unsigned long long* d) { P->stamps = d; return 0; }
#endif

int msa_plan_set_timing(msa_plan* P, int on) {
  if (!P) return MSA_ERR_ARG;
  P->timing = on != 0;
  return MSA_OK;
}

int msa_plan_last_kernel_ms(msa_plan* P, float* ms) {
  if (!P || !ms) return MSA_ERR_ARG;
  if (!P->timed) return MSA_ERR_ARG;  // no run with timing on yet
  HIPCHK(hipEventSynchronize(P->ev1));
  HIPCHK(hipEventElapsedTime(ms, P->ev0, P->ev1));
  return MSA_OK;
}

int msa_plan_results(msa_plan* P, msa_pair_result* out, void* stream) {
  if (!P || !out) return MSA_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  int err = 0;
  HIPCHK(hipMemcpyAsync(&err, P->d_err, sizeof(err), hipMemcpyDeviceToHost, st));
  unsigned long long key = 0;
  if (P->fused_reduce)  // one pair: its result is the pass-2 blocks' best-cell key
    HIPCHK(hipMemcpyAsync(&key, P->d_ticket + MSA_TK_BEST, sizeof(key), hipMemcpyDeviceToHost, st));
  else
    HIPCHK(hipMemcpyAsync(out, P->d_res, sizeof(PairResult) * P->d.n_pairs, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  static_assert(sizeof(PairResult) == sizeof(msa_pair_result), "result layout");
  if (P->fused_reduce) {
    const PairResult r = best_key_decode(key, P->pairs[0].n);
    std::memcpy(out, &r, sizeof(r));
  }
  if (err) {
    std::fprintf(stderr, "msa: a kernel wait hit its spin limit (site %d) in a run since the plan was created "
                 "or last cleared\n", err);
    return MSA_ERR_TIMEOUT;
  }
  return MSA_OK;
}

int msa_plan_run_info(msa_plan* P, int32_t* out4, void* stream) {
  if (!P || !out4) return MSA_ERR_ARG;
  out4[0] = P->chunked ? 2 : (P->flow ? 1 : 0);
  out4[1] = P->n_chunks;
  out4[2] = -1;
  out4[3] = P->chunked ? (P->kp.chunk_warm | (P->h16 ? (1 << 16) : 0)) : 0;  // bit 16: int16 chunk cells
  if (P->chunked) {
    int v = 0;
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(&v, P->d_skip, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    out4[2] = v;
  }
  return MSA_OK;
}

int msa_plan_launch_info(const msa_plan* P, int32_t* out8) {
  if (!P || !out8) return MSA_ERR_ARG;
  const int mode = P->cflow ? 6 : P->band_k ? (P->chunked ? 5 : 4)
                             : (P->chunked ? 2 : (P->flow ? 1 : (P->kp.single == 3 ? 3 : 0)));
  out8[0] = mode;
  out8[1] = P->grid;
  out8[2] = P->threads;
  out8[3] = (int32_t)P->lds_bytes;
  out8[4] = P->nflow;
  out8[5] = P->fill_fn ? P->fill_grid : 0;
  out8[6] = P->R;
  out8[7] = P->kp.n_items;
  return MSA_OK;
}

int msa_plan_error(msa_plan* P, int* code, void* stream) {
  if (!P || !code) return MSA_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipMemcpyAsync(code, P->d_err, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return MSA_OK;
}

int msa_plan_clear_error(msa_plan* P, void* stream) {
  if (!P) return MSA_ERR_ARG;
  HIPCHK(hipMemsetAsync(P->d_err, 0, sizeof(int), (hipStream_t)stream));
  return MSA_OK;
}

int msa_plan_scores(msa_plan* P, int32_t* dst, void* stream) {
  if (!P || !dst) return MSA_ERR_ARG;
  // the score field of every PairResult, device to device (no host sync)
  P->note_stream((hipStream_t)stream);
  if (P->fused_reduce) {  // the pair result from the best-cell key first
    hipLaunchKernelGGL(best_key_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                       reinterpret_cast<const unsigned long long*>(P->d_ticket + MSA_TK_BEST), (long long)P->pairs[0].n,
                       P->d_res);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipMemcpy2DAsync(dst, sizeof(int32_t), P->d_res, sizeof(PairResult), sizeof(int32_t), (size_t)P->d.n_pairs,
                          hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return MSA_OK;
}

int msa_plan_stripe_meta(msa_plan* P, int32_t* out, int64_t cap, void* stream) {
  if (!P || !out || cap < P->total_stripes) return MSA_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  static_assert(sizeof(msa_stripe_meta) == 12 * 4, "meta layout");
  HIPCHK(hipMemcpyAsync(out, P->d_meta, sizeof(msa_stripe_meta) * P->total_stripes, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return MSA_OK;
}

int msa_plan_traceback(msa_plan* P, int64_t pair, const uint8_t* dDir, uint8_t* d_ops, int64_t ops_cap,
                       int64_t* d_info, void* stream) {
  if (!P || !dDir || !d_ops || !d_info || ops_cap < 0 || pair < 0 || pair >= P->d.n_pairs) return MSA_ERR_ARG;
  // the walk starts at the fill's end cell: plans without track_end have none
  if (P->kp.alg != MSA_ALG_SWA || P->d.cells != MSA_CELLS_DIR || !P->d.track_end) return MSA_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  P->note_stream(st);
  hipLaunchKernelGGL((P->R == 2 ? traceback_kernel<TB_SW, 2> : traceback_kernel<TB_SW>), dim3(1), dim3(384), 0, st, dDir, P->d_pairs, P->d_meta,
                     (const PairResult*)P->d_res, (int)pair, 0, 0, d_ops, (long long)ops_cap, (long long*)d_info,
                     P->flow ? 1 : 0,
                     P->fused_reduce ? reinterpret_cast<const unsigned long long*>(P->d_ticket + MSA_TK_BEST) : nullptr);
  HIPCHK(hipGetLastError());
  return MSA_OK;
}

int msa_plan_traceback_gotoh(msa_plan* P, int64_t pair, int end_type, const uint8_t* dDir, uint8_t* d_ops,
                             int64_t ops_cap, int64_t* d_info, void* stream) {
  if (!P || !dDir || !d_ops || !d_info || ops_cap < 0 || pair < 0 || pair >= P->d.n_pairs) return MSA_ERR_ARG;
  if (end_type < -3 || end_type > 3 || end_type == 0) return MSA_ERR_ARG;
  if ((P->kp.alg != MSA_ALG_REF && P->kp.alg != MSA_ALG_REF1) || P->d.cells != MSA_CELLS_DIR)
    return MSA_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  P->note_stream(st);
  // REF1 bytes hold tags (3 / 2 / 1 = T1 / T2 / T3), REF bytes the table numbers
  hipLaunchKernelGGL(P->kp.alg == MSA_ALG_REF1 ? (P->R == 2 ? traceback_kernel<TB_REF_TAG, 2> : traceback_kernel<TB_REF_TAG>)
                                               : traceback_kernel<TB_REF>, dim3(1),
                     dim3(384), 0, st, dDir, P->d_pairs, P->d_meta, (const PairResult*)P->d_res, (int)pair, end_type,
                     (int)P->kp.h, d_ops, (long long)ops_cap, (long long*)d_info, P->flow ? 1 : 0,
                     (const unsigned long long*)nullptr);
  HIPCHK(hipGetLastError());
  return MSA_OK;
}

int msa_plan_checksum(msa_plan* P, const int32_t* dH, int64_t pair, uint64_t* digest, void* stream) {
  if (!P || !dH || !digest || pair < 0 || pair >= P->d.n_pairs) return MSA_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipMemsetAsync(P->d_sum, 0, 8, st));
  hipLaunchKernelGGL(checksum_kernel, dim3(1024), dim3(256), 0, st, dH, P->d_pairs, P->d_meta, (int)pair,
                     P->kp.band, P->R, P->d_sum);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(digest, P->d_sum, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return MSA_OK;
}

}  // extern "C"
#include "msa_refapi.inc"
#include "msa_rowapi.inc"
