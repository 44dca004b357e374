// Native communication core: RCCL communicator + in-order gradient-bucket engine + chrome-trace
// timeline, driven from Python through ctypes (parallel/native_comm.py).
//
// Reference behaviour it replaces (SURVEY §2.2 E-HVD-core / §2.3 N1, §2.5): Horovod's C++ core
// (background negotiation, fusion buffer, MPI/NCCL collectives, HOROVOD_TIMELINE), entered from
// /root/reference/train.py:20-21 (hvd.init) and :103-104 (DistributedOptimizer).  MI355X design:
//
// * no negotiation: the gradient buckets are slices of one persistent flat fp32 buffer, registered
//   once; every rank launches them strictly in bucket order (bucket b+1 never before b), so the
//   collective order is identical on all ranks by construction;
// * a bucket becomes ready on the COMPUTE stream (hipEventRecord) when its last gradient has been
//   produced; the dedicated comm stream waits on that event and runs ncclAllReduce in place, so the
//   reduction overlaps the rest of the backward pass; `wait` makes the compute stream wait on the
//   per-bucket done events (no host synchronisation anywhere);
// * RCCL is not linked: the library the process already uses (PyTorch's bundled librccl) is
//   dlopen'ed by path, so there is exactly ONE RCCL instance per process;
// * timeline: READY instants (host clock) and ALLREDUCE spans measured with timing events on the
//   comm stream (GPU execution, not host enqueue), one chrome://tracing JSON file per rank
//   (Horovod's HOROVOD_TIMELINE format); per-step statistics (summed all-reduce time, exposed tail
//   after the backward) come from the same per-bucket events;
// * watchdog: an optional host thread polls every launched bucket's done event and
//   ncclCommGetAsyncError; a bucket still pending after the timeout (a dead or stalled peer) or an
//   async RCCL error aborts the communicator (ncclCommAbort) so the rank fails with an error that
//   names the bucket instead of hanging in the next wait.  The watchdog never waits on the enqueue
//   lock: an enqueuer blocked inside RCCL behind a stalled peer cannot keep it from aborting.
#include <dlfcn.h>
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#define MXR_API extern "C" __attribute__((visibility("default")))

namespace {

// ---- minimal RCCL ABI (rccl.h): opaque comm, 128-byte unique id, enums as int
typedef struct ncclComm* ncclComm_t;
typedef struct { char internal[128]; } ncclUniqueId;
typedef int ncclResult_t;
enum { ncclInt8 = 0, ncclUint8 = 1, ncclInt32 = 2, ncclUint32 = 3, ncclInt64 = 4, ncclUint64 = 5, ncclFloat16 = 6,
       ncclFloat32 = 7, ncclFloat64 = 8, ncclBfloat16 = 9 };
enum { ncclSum = 0, ncclProd = 1, ncclMax = 2, ncclMin = 3, ncclAvg = 4 };

struct Api {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*ReduceScatter)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;   // optional
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;                           // optional
  ncclResult_t (*CommCount)(ncclComm_t, int*) = nullptr;                     // optional (introspection)
  ncclResult_t (*CommCuDevice)(ncclComm_t, int*) = nullptr;                  // optional
  ncclResult_t (*CommUserRank)(ncclComm_t, int*) = nullptr;                  // optional
} api;

std::mutex g_mu;
std::string g_err;

void set_err(const std::string& e) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_err = e;
}

double now_us() {
  using namespace std::chrono;
  return (double)duration_cast<microseconds>(steady_clock::now().time_since_epoch()).count();
}

struct TimelineEv {
  std::string name, phase;
  char ph;
  double ts;
};

// one all-reduce bracketed by timing events on the comm stream, converted to timestamps at flush
struct GpuRec {
  int bucket;
  size_t bytes;
  hipEvent_t start, end;
};

struct Comm {
  std::atomic<ncclComm_t> comm{nullptr};
  int rank = 0, nranks = 1, device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = true;          // false: the stream was handed in (mxr_comm_set_stream)
  // Locking: `enq_mu` serialises the host enqueue paths (buckets and plain collectives) and is never
  // waited on by the watchdog; `book_mu` guards the short bookkeeping the watchdog reads (launch
  // times, the bucket event vectors while they are replaced, the abort reason).
  std::mutex enq_mu, book_mu;
  // bucket engine
  std::vector<void*> bptr;
  std::vector<size_t> bcount;
  int bdtype = ncclFloat32, bop = ncclSum, belem = 4;
  std::vector<hipEvent_t> ready_ev, start_ev, done_ev;   // timing-enabled: per-step comm statistics
  std::vector<char> ready;
  std::vector<char> launched;
  std::vector<double> launch_us;   // host time of the bucket's launch, 0 = not pending (watchdog)
  int next_launch = 0;
  bool have_stats = false;
  bool timing = true;              // bucket events carry timestamps (MXR_COMM_TIMING=0: disabled)
  // Events only order streams of THIS device (RCCL fences its own peer traffic), so they skip the
  // system-scope fence: with it every record/wait writes back and invalidates the caches, and the
  // compute stream's following kernels run cold (measured: memory-bound kernels 3-4x slower,
  // 41 -> 57 ms per training step, A/B of round 2).
  unsigned ev_flags = hipEventDisableSystemFence;
  hipStream_t cur_compute = nullptr;
  // the step being issued is captured into a HIP graph (the compute stream was capturing at readiness): the
  // bucket events are graph-internal dependencies, so no watchdog registration, no timeline spans, and no
  // per-step statistics until an eager step records them again
  bool capturing = false;
  // watchdog
  std::thread wd;
  std::atomic<bool> wd_stop{false}, aborted{false};
  double wd_timeout_us = 0;
  int wd_inject = -1;              // test hook: this bucket never reports completion
  std::string wd_err;
  // timeline: host instants (READY) + GPU-timed all-reduce spans
  bool tl_on = false;
  std::string tl_path;
  std::vector<TimelineEv> tl;
  std::vector<GpuRec> tl_gpu;
  hipEvent_t tl_base = nullptr;
  double tl_base_us = 0;
  // stream-ordering perturbation (tests): a spin before and a scale after every bucket
  // all-reduce on the comm stream -- a consumer that does not wait on the done events reads stale data
  long long dbg_delay_cycles = 0;
  float dbg_scale = 1.f;
};

// spin for `cycles` of the constant-rate wall clock (one wave; the stream is what it delays)
__global__ void spin_kernel(long long cycles) {
  long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
}

template <class T>
__global__ void scale_kernel(T* p, size_t n, float s) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (T)((float)p[i] * s);
}

int to_nccl_dtype(int d) {   // 0 f32, 1 bf16, 2 f16, 3 i32, 4 i64, 5 u8, 6 f64
  switch (d) {
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt32;
    case 4: return ncclInt64;
    case 5: return ncclUint8;
    case 6: return ncclFloat64;
    default: return ncclFloat32;
  }
}

int elem_size(int d) {
  switch (d) {
    case 1: case 2: return 2;
    case 4: case 6: return 8;
    case 5: return 1;
    default: return 4;
  }
}

int check(ncclResult_t r, const char* what) {
  if (r != 0) {
    set_err(std::string(what) + ": " + (api.GetErrorString ? api.GetErrorString(r) : "rccl error"));
    return -10 - r;
  }
  return 0;
}

int hcheck(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    set_err(std::string(what) + ": " + hipGetErrorString(e));
    return -100 - (int)e;
  }
  return 0;
}

int refuse_aborted(Comm* c) {
  std::lock_guard<std::mutex> lk(c->book_mu);
  set_err(c->wd_err.empty() ? std::string("communicator aborted") : c->wd_err);
  return -4;
}

void tl_add(Comm* c, const std::string& name, const char* phase, char ph) {
  if (c->tl_on) c->tl.push_back({name, phase, ph, now_us()});
}

// convert finished GPU spans to timeline records (blocking = wait for the unfinished ones too)
void tl_harvest(Comm* c, bool blocking) {
  size_t keep = 0;
  for (size_t i = 0; i < c->tl_gpu.size(); ++i) {
    GpuRec& r = c->tl_gpu[i];
    bool done = blocking ? hipEventSynchronize(r.end) == hipSuccess : hipEventQuery(r.end) == hipSuccess;
    if (!done) {
      c->tl_gpu[keep++] = r;
      continue;
    }
    float a = 0, b = 0;
    hipEventElapsedTime(&a, c->tl_base, r.start);
    hipEventElapsedTime(&b, c->tl_base, r.end);
    std::string n = "bucket" + std::to_string(r.bucket);
    c->tl.push_back({n, "ALLREDUCE", 'B', c->tl_base_us + 1000.0 * a});
    c->tl.push_back({n, "ALLREDUCE", 'E', c->tl_base_us + 1000.0 * b});
    hipEventDestroy(r.start);
    hipEventDestroy(r.end);
  }
  c->tl_gpu.resize(keep);
}

// abort the communicator from any thread.  The enqueue lock is taken if it frees up quickly (no
// enqueue can then be mid-flight on the comm); an enqueuer blocked INSIDE RCCL behind a stalled peer
// is exactly what the abort has to unblock, so after ~1 s the abort proceeds without it.
void do_abort(Comm* c, const std::string& why) {
  {
    std::lock_guard<std::mutex> lk(c->book_mu);
    if (c->aborted) return;
    c->wd_err = "rank " + std::to_string(c->rank) + ": " + why + "; communicator aborted";
    c->aborted = true;
    set_err(c->wd_err);
  }
  bool locked = false;
  for (int i = 0; i < 100 && !(locked = c->enq_mu.try_lock()); ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  ncclComm_t cm = c->comm.exchange(nullptr);
  if (cm && api.CommAbort) api.CommAbort(cm);
  if (locked) c->enq_mu.unlock();
}

// caller holds enq_mu
int launch_bucket(Comm* c, int b) {
  // the collective runs on the comm stream, ordered after the bucket's readiness event
  hipStream_t st = c->stream;
  int rc = 0;
  if ((rc = hcheck(hipStreamWaitEvent(st, c->ready_ev[b], 0), "hipStreamWaitEvent"))) return rc;
  GpuRec rec{b, c->bcount[b] * (size_t)c->belem, nullptr, nullptr};
  if (c->tl_on && !c->capturing) {
    hipEventCreateWithFlags(&rec.start, c->ev_flags);
    hipEventCreateWithFlags(&rec.end, c->ev_flags);
    hipEventRecord(rec.start, st);
  }
  if ((rc = hcheck(hipEventRecord(c->start_ev[b], st), "hipEventRecord"))) return rc;
  ncclComm_t cm = c->comm.load();
  if (!cm) return refuse_aborted(c);
  if (c->dbg_delay_cycles > 0) spin_kernel<<<1, 64, 0, st>>>(c->dbg_delay_cycles);
  rc = check(api.AllReduce(c->bptr[b], c->bptr[b], c->bcount[b], c->bdtype, c->bop, cm, st), "ncclAllReduce");
  if (rc) return rc;
  if (c->dbg_scale != 1.f) {
    size_t n = c->bcount[b];
    unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 1024);
    if (c->bdtype == ncclFloat32)
      scale_kernel<float><<<blocks, 256, 0, st>>>(static_cast<float*>(c->bptr[b]), n, c->dbg_scale);
    else if (c->bdtype == ncclBfloat16)
      scale_kernel<__hip_bfloat16><<<blocks, 256, 0, st>>>(static_cast<__hip_bfloat16*>(c->bptr[b]), n,
                                                            c->dbg_scale);
  }
  rc = hcheck(hipEventRecord(c->done_ev[b], st), "hipEventRecord");
  if (c->tl_on && !c->capturing) {
    hipEventRecord(rec.end, st);
    c->tl_gpu.push_back(rec);
  }
  c->launched[b] = 1;
  if (c->capturing) return rc;     // replays are checked through the eager steps around them, not per bucket
  std::lock_guard<std::mutex> lk(c->book_mu);
  c->launch_us[b] = now_us();
  return rc;
}

// one watchdog pass: 0 = healthy, 1 = aborted the communicator (reason in c->wd_err)
int watchdog_pass(Comm* c) {
  std::string why;
  if (api.CommGetAsyncError) {
    ncclComm_t cm = c->comm.load();
    ncclResult_t ar = 0;
    if (cm && api.CommGetAsyncError(cm, &ar) == 0 && ar != 0)
      why = std::string("async RCCL error: ") + (api.GetErrorString ? api.GetErrorString(ar) : "?");
  }
  {
    std::lock_guard<std::mutex> lk(c->book_mu);
    double t = now_us();
    for (size_t b = 0; why.empty() && b < c->launch_us.size(); ++b) {
      if (c->launch_us[b] == 0) continue;
      bool done = (int)b != c->wd_inject && hipEventQuery(c->done_ev[b]) == hipSuccess;
      if (done) {
        c->launch_us[b] = 0;
      } else if (t - c->launch_us[b] > c->wd_timeout_us) {
        why = "bucket " + std::to_string(b) + " (" + std::to_string(c->bcount[b]) + " elements) all-reduce not done after " +
              std::to_string((long long)((t - c->launch_us[b]) / 1000)) + " ms";
      }
    }
  }
  if (why.empty()) return 0;
  do_abort(c, why);
  return 1;
}

void watchdog_loop(Comm* c, int poll_ms) {
  hipSetDevice(c->device);
  while (!c->wd_stop.load()) {
    if (watchdog_pass(c)) return;
    std::this_thread::sleep_for(std::chrono::milliseconds(poll_ms));
  }
}

void watchdog_stop(Comm* c) {
  c->wd_stop = true;
  if (c->wd.joinable()) c->wd.join();
  c->wd_stop = false;
}

void destroy_bucket_events(Comm* c) {
  for (auto* v : {&c->ready_ev, &c->start_ev, &c->done_ev})
    for (auto e : *v)
      if (e) hipEventDestroy(e);
}

}  // namespace

// copied under the lock: the watchdog thread may be rewriting the message
MXR_API const char* mxr_comm_last_error() {
  static thread_local std::string copy;
  std::lock_guard<std::mutex> lk(g_mu);
  copy = g_err;
  return copy.c_str();
}

// dlopen the RCCL the process uses (path from Python: torch's bundled librccl.so)
MXR_API int mxr_comm_load(const char* path) {
  if (api.h) return 0;
  void* h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    set_err(std::string("dlopen: ") + dlerror());
    return -1;
  }
#define SYM(field, name)                                                   \
  api.field = reinterpret_cast<decltype(api.field)>(dlsym(h, name));       \
  if (!api.field) {                                                        \
    set_err(std::string("dlsym ") + name);                                 \
    return -2;                                                             \
  }
  SYM(GetUniqueId, "ncclGetUniqueId")
  SYM(CommInitRank, "ncclCommInitRank")
  SYM(CommDestroy, "ncclCommDestroy")
  SYM(AllReduce, "ncclAllReduce")
  SYM(Broadcast, "ncclBroadcast")
  SYM(AllGather, "ncclAllGather")
  SYM(ReduceScatter, "ncclReduceScatter")
  SYM(GetErrorString, "ncclGetErrorString")
#undef SYM
  api.CommGetAsyncError = reinterpret_cast<decltype(api.CommGetAsyncError)>(dlsym(h, "ncclCommGetAsyncError"));
  api.CommAbort = reinterpret_cast<decltype(api.CommAbort)>(dlsym(h, "ncclCommAbort"));
  api.CommCount = reinterpret_cast<decltype(api.CommCount)>(dlsym(h, "ncclCommCount"));
  api.CommCuDevice = reinterpret_cast<decltype(api.CommCuDevice)>(dlsym(h, "ncclCommCuDevice"));
  api.CommUserRank = reinterpret_cast<decltype(api.CommUserRank)>(dlsym(h, "ncclCommUserRank"));
  api.h = h;
  return 0;
}

MXR_API int mxr_comm_unique_id(char* out128) {
  if (!api.h) return -1;
  ncclUniqueId id;
  int rc = check(api.GetUniqueId(&id), "ncclGetUniqueId");
  if (rc) return rc;
  memcpy(out128, id.internal, 128);
  return 0;
}

// returns an opaque handle (0 on failure; see mxr_comm_last_error)
MXR_API void* mxr_comm_init(const char* id128, int nranks, int rank, int device) {
  if (!api.h) {
    set_err("RCCL not loaded");
    return nullptr;
  }
  if (hcheck(hipSetDevice(device), "hipSetDevice")) return nullptr;
  Comm* c = new Comm();
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  ncclUniqueId id;
  memcpy(id.internal, id128, 128);
  ncclComm_t cm = nullptr;
  if (check(api.CommInitRank(&cm, nranks, id, rank), "ncclCommInitRank")) {
    delete c;
    return nullptr;
  }
  c->comm = cm;
  int lo = 0, hi = 0;
  hipDeviceGetStreamPriorityRange(&lo, &hi);
  const int prio = hi;   // the highest stream priority (A/B: high beat normal, profiles/r2_stream_priority_ab.txt)
  const char* te = getenv("MXR_COMM_TIMING");             // "0": bucket events without timing
  c->timing = !(te && strcmp(te, "0") == 0);
  if (hcheck(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio), "hipStreamCreate")) {
    api.CommDestroy(cm);
    delete c;
    return nullptr;
  }
  return c;
}

// drain the comm stream with a bound (the watchdog timeout, else 60 s); a stream still busy after
// that means a stalled peer -> abort instead of hanging the caller's close()/__del__
MXR_API int mxr_comm_destroy(void* h) {
  Comm* c = static_cast<Comm*>(h);
  if (!c) return 0;
  watchdog_stop(c);
  if (!c->aborted) {
    double limit = c->wd_timeout_us > 0 ? c->wd_timeout_us : 60e6;
    double t0 = now_us();
    while (hipStreamQuery(c->stream) == hipErrorNotReady) {
      if (now_us() - t0 > limit) {
        do_abort(c, "comm stream still busy at destroy");
        break;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }
  if (c->tl_on) tl_harvest(c, !c->aborted);
  for (auto& r : c->tl_gpu) {
    hipEventDestroy(r.start);
    hipEventDestroy(r.end);
  }
  if (c->tl_base) hipEventDestroy(c->tl_base);
  destroy_bucket_events(c);
  ncclComm_t cm = c->comm.exchange(nullptr);
  int rc = cm ? check(api.CommDestroy(cm), "ncclCommDestroy") : 0;
  if (c->own_stream) hipStreamDestroy(c->stream);
  delete c;
  return rc;
}

// ---- plain collectives, ordered after the caller's stream and back (event handshake)
static int fence_in(Comm* c, hipStream_t s, hipEvent_t* ev) {
  int rc = hcheck(hipEventCreateWithFlags(ev, hipEventDisableTiming | c->ev_flags), "hipEventCreate");
  if (rc) return rc;
  rc = hcheck(hipEventRecord(*ev, s), "hipEventRecord");
  if (rc) return rc;
  return hcheck(hipStreamWaitEvent(c->stream, *ev, 0), "hipStreamWaitEvent");
}

static int fence_out(Comm* c, hipStream_t s, hipEvent_t ev) {
  int rc = hcheck(hipEventRecord(ev, c->stream), "hipEventRecord");
  if (rc) return rc;
  rc = hcheck(hipStreamWaitEvent(s, ev, 0), "hipStreamWaitEvent");
  hipEventDestroy(ev);
  return rc;
}

// run `op(comm)` on the comm stream between the two fences; refuses after an abort
template <class F>
static int fenced(Comm* c, hipStream_t s, const char* what, F op) {
  std::lock_guard<std::mutex> lk(c->enq_mu);
  if (c->aborted) return refuse_aborted(c);
  ncclComm_t cm = c->comm.load();
  if (!cm) return refuse_aborted(c);
  hipEvent_t ev;
  int rc = fence_in(c, s, &ev);
  if (rc) return rc;
  rc = check(op(cm), what);
  if (rc) {
    hipEventDestroy(ev);
    return rc;
  }
  return fence_out(c, s, ev);
}

MXR_API int mxr_comm_allreduce(void* h, const void* send, void* recv, long long count, int dtype, int avg,
                               hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  return fenced(c, s, "ncclAllReduce", [&](ncclComm_t cm) {
    return api.AllReduce(send, recv, (size_t)count, to_nccl_dtype(dtype), avg ? ncclAvg : ncclSum, cm, c->stream);
  });
}

MXR_API int mxr_comm_broadcast(void* h, void* buf, long long count, int dtype, int root, hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  return fenced(c, s, "ncclBroadcast", [&](ncclComm_t cm) {
    return api.Broadcast(buf, buf, (size_t)count, to_nccl_dtype(dtype), root, cm, c->stream);
  });
}

MXR_API int mxr_comm_allgather(void* h, const void* send, void* recv, long long count, int dtype, hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  return fenced(c, s, "ncclAllGather", [&](ncclComm_t cm) {
    return api.AllGather(send, recv, (size_t)count, to_nccl_dtype(dtype), cm, c->stream);
  });
}

MXR_API int mxr_comm_reduce_scatter(void* h, const void* send, void* recv, long long count, int dtype, int avg,
                                    hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  return fenced(c, s, "ncclReduceScatter", [&](ncclComm_t cm) {
    return api.ReduceScatter(send, recv, (size_t)count, to_nccl_dtype(dtype), avg ? ncclAvg : ncclSum, cm, c->stream);
  });
}

// ---- bucket engine
MXR_API int mxr_comm_set_buckets(void* h, int n, void** ptrs, const long long* counts, int dtype, int avg) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::mutex> lk(c->enq_mu);
  std::lock_guard<std::mutex> lk2(c->book_mu);
  destroy_bucket_events(c);
  c->ready_ev.assign(n, nullptr);
  c->start_ev.assign(n, nullptr);
  c->done_ev.assign(n, nullptr);
  c->bptr.assign(ptrs, ptrs + n);
  c->bcount.resize(n);
  for (int i = 0; i < n; ++i) {
    c->bcount[i] = (size_t)counts[i];
    const unsigned fl = (c->timing ? hipEventDefault : hipEventDisableTiming) | c->ev_flags;
    int rc = hcheck(hipEventCreateWithFlags(&c->ready_ev[i], fl), "hipEventCreate");
    if (!rc) rc = hcheck(hipEventCreateWithFlags(&c->start_ev[i], fl), "hipEventCreate");
    if (!rc) rc = hcheck(hipEventCreateWithFlags(&c->done_ev[i], fl), "hipEventCreate");
    if (rc) return rc;
  }
  c->bdtype = to_nccl_dtype(dtype);
  c->belem = elem_size(dtype);
  c->bop = avg ? ncclAvg : ncclSum;
  c->ready.assign(n, 0);
  c->launched.assign(n, 0);
  c->launch_us.assign(n, 0.0);
  c->next_launch = 0;
  c->have_stats = false;
  return 0;
}

static int bucket_ready_locked(Comm* c, int b, hipStream_t compute) {
  if (c->aborted) return refuse_aborted(c);
  if (b < 0 || b >= (int)c->bptr.size()) {
    set_err("bucket " + std::to_string(b) + " out of range (" + std::to_string(c->bptr.size()) + " buckets)");
    return -3;
  }
  if (c->ready[b]) {
    set_err("bucket " + std::to_string(b) + " marked ready twice in one step (missing reset after an aborted step?)");
    return -3;
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  int rc = hcheck(hipStreamIsCapturing(compute, &cs), "hipStreamIsCapturing");
  if (rc) return rc;
  const bool cap = cs == hipStreamCaptureStatusActive;
  if (std::find(c->ready.begin(), c->ready.end(), 1) == c->ready.end()) c->capturing = cap;   // first of the step
  else if (cap != c->capturing) {
    set_err("bucket " + std::to_string(b) + ": stream capture began or ended in the middle of a step");
    return -3;
  }
  rc = hcheck(hipEventRecord(c->ready_ev[b], compute), "hipEventRecord");
  if (rc) return rc;
  c->cur_compute = compute;
  c->ready[b] = 1;
  tl_add(c, "bucket" + std::to_string(b), "READY", 'i');
  while (c->next_launch < (int)c->bptr.size() && c->ready[c->next_launch]) {
    rc = launch_bucket(c, c->next_launch);
    if (rc) return rc;
    ++c->next_launch;
  }
  return 0;
}

// bucket b's gradients are complete on `compute`; launch every consecutive ready bucket in order
MXR_API int mxr_comm_bucket_ready(void* h, int b, hipStream_t compute) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::mutex> lk(c->enq_mu);
  return bucket_ready_locked(c, b, compute);
}

// launch whatever is left (recording readiness on `compute` now), then make `compute` wait for all
MXR_API int mxr_comm_wait(void* h, hipStream_t compute) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::mutex> lk(c->enq_mu);
  if (c->aborted) return refuse_aborted(c);
  int rc;
  for (int b = 0; b < (int)c->bptr.size(); ++b)
    if (!c->ready[b] && (rc = bucket_ready_locked(c, b, compute))) return rc;
  for (int b = 0; b < (int)c->bptr.size(); ++b)
    if ((rc = hcheck(hipStreamWaitEvent(compute, c->done_ev[b], 0), "hipStreamWaitEvent"))) return rc;
  std::fill(c->ready.begin(), c->ready.end(), 0);
  std::fill(c->launched.begin(), c->launched.end(), 0);
  c->next_launch = 0;
  c->have_stats = !c->bptr.empty() && !c->capturing;
  c->capturing = false;
  if (c->tl_on) tl_harvest(c, false);
  return 0;
}

// abandon the current step (exception / OOM mid-backward): `compute` waits for every bucket already
// launched (so the next step cannot zero a buffer RCCL is still reducing), then the flags clear
MXR_API int mxr_comm_reset(void* h, hipStream_t compute) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::mutex> lk(c->enq_mu);
  int rc = 0;
  if (!c->aborted)
    for (int b = 0; b < (int)c->bptr.size(); ++b)
      if (c->launched[b] && !rc) rc = hcheck(hipStreamWaitEvent(compute, c->done_ev[b], 0), "hipStreamWaitEvent");
  std::fill(c->ready.begin(), c->ready.end(), 0);
  std::fill(c->launched.begin(), c->launched.end(), 0);
  c->next_launch = 0;
  c->capturing = false;
  return rc;
}

// run the collectives on a caller-owned stream instead of the communicator's own one (must be idle)
MXR_API int mxr_comm_set_stream(void* h, hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::mutex> lk(c->enq_mu);
  hipStreamSynchronize(c->stream);
  if (c->own_stream) hipStreamDestroy(c->stream);
  c->stream = s;
  c->own_stream = false;
  return 0;
}

// what RCCL itself reports for the communicator (not what it was asked for): out = {nranks, device,
// rank}; -1 where the symbol is missing.  bench.py checks nranks == --gpus.
MXR_API int mxr_comm_info(void* h, int* out3) {
  Comm* c = static_cast<Comm*>(h);
  out3[0] = out3[1] = out3[2] = -1;
  ncclComm_t cm = c ? c->comm.load() : nullptr;
  if (!cm) return -1;
  int rc = 0;
  if (api.CommCount) rc |= check(api.CommCount(cm, &out3[0]), "ncclCommCount");
  if (api.CommCuDevice) rc |= check(api.CommCuDevice(cm, &out3[1]), "ncclCommCuDevice");
  if (api.CommUserRank) rc |= check(api.CommUserRank(cm, &out3[2]), "ncclCommUserRank");
  return rc;
}

MXR_API int mxr_comm_next_launch(void* h) { return static_cast<Comm*>(h)->next_launch; }

// statistics of the last completed step (blocks until its last bucket is done):
// out[0] = sum of the bucket all-reduce times (ms, GPU), out[1] = exposed tail (ms from the last bucket
// becoming ready on the compute stream to its all-reduce finishing), out[2 + b] = bucket b's time
MXR_API int mxr_comm_step_stats(void* h, float* out, int n) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::mutex> lk(c->enq_mu);
  if (!c->have_stats || c->aborted || !c->timing) return -1;
  int nb = (int)c->bptr.size();
  int rc = hcheck(hipEventSynchronize(c->done_ev[nb - 1]), "hipEventSynchronize");
  if (rc) return rc;
  float total = 0;
  for (int b = 0; b < nb; ++b) {
    float ms = 0;
    hipEventElapsedTime(&ms, c->start_ev[b], c->done_ev[b]);
    total += ms;
    if (2 + b < n) out[2 + b] = ms;
  }
  float tail = 0;
  hipEventElapsedTime(&tail, c->ready_ev[nb - 1], c->done_ev[nb - 1]);
  if (n > 0) out[0] = total;
  if (n > 1) out[1] = tail > 0 ? tail : 0;
  return nb;
}

// ---- watchdog: timeout_ms <= 0 stops it; inject_bucket >= 0 is the fault-injection test hook
MXR_API int mxr_comm_watchdog(void* h, int timeout_ms, int poll_ms, int inject_bucket) {
  Comm* c = static_cast<Comm*>(h);
  watchdog_stop(c);
  c->wd_inject = inject_bucket;
  if (timeout_ms <= 0 || c->aborted) return 0;
  c->wd_timeout_us = 1000.0 * timeout_ms;
  c->wd = std::thread(watchdog_loop, c, poll_ms > 0 ? poll_ms : 100);
  return 0;
}

// test hook: delay (µs of the 100 MHz wall clock) before, and scale after, every bucket all-reduce
MXR_API int mxr_comm_debug(void* h, int delay_us, float post_scale) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::mutex> lk(c->enq_mu);
  c->dbg_delay_cycles = 100LL * (delay_us > 0 ? delay_us : 0);
  c->dbg_scale = post_scale;
  return 0;
}

// 0 = healthy, 1 = aborted (message in mxr_comm_last_error)
MXR_API int mxr_comm_status(void* h) {
  Comm* c = static_cast<Comm*>(h);
  if (!c->aborted) return 0;
  refuse_aborted(c);
  return 1;
}

// ---- timeline: READY instants (host clock) + ALLREDUCE spans from GPU timing events on the comm
// stream, placed on the same clock through a base event synchronised when the timeline starts
MXR_API int mxr_comm_timeline(void* h, const char* path) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::mutex> lk(c->enq_mu);
  if (c->tl_on) tl_harvest(c, true);
  c->tl_on = path && path[0];
  c->tl_path = c->tl_on ? path : "";
  c->tl.clear();
  if (c->tl_on) {
    if (!c->tl_base && hcheck(hipEventCreateWithFlags(&c->tl_base, c->ev_flags), "hipEventCreate")) return -1;
    if (hcheck(hipEventRecord(c->tl_base, c->stream), "hipEventRecord")) return -1;
    if (hcheck(hipEventSynchronize(c->tl_base), "hipEventSynchronize")) return -1;
    c->tl_base_us = now_us();
  }
  return 0;
}

MXR_API int mxr_comm_timeline_flush(void* h) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::mutex> lk(c->enq_mu);
  if (!c->tl_on) return 0;
  tl_harvest(c, true);
  FILE* f = fopen(c->tl_path.c_str(), "w");
  if (!f) {
    set_err("cannot open timeline " + c->tl_path);
    return -1;
  }
  fprintf(f, "[\n");
  for (size_t i = 0; i < c->tl.size(); ++i) {
    const TimelineEv& e = c->tl[i];
    fprintf(f, "{\"name\": \"%s\", \"cat\": \"%s\", \"ph\": \"%c\", \"ts\": %.1f, \"pid\": %d, \"tid\": %d%s}%s\n",
            e.phase.c_str(), e.name.c_str(), e.ph, e.ts, c->rank, e.ph == 'i' ? 0 : 1,
            e.ph == 'i' ? ", \"s\": \"t\"" : "", i + 1 < c->tl.size() ? "," : "");
  }
  fprintf(f, "]\n");
  fclose(f);
  return 0;
}
