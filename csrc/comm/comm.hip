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
// * timeline: begin/end records with host timestamps (µs) for READY / ALLREDUCE phases, written
//   as a chrome://tracing JSON array (Horovod's HOROVOD_TIMELINE format, one file per rank);
// * watchdog: an optional host thread polls every launched bucket's done event and
//   ncclCommGetAsyncError; a bucket still pending after the timeout (a dead or stalled peer) or an
//   async RCCL error aborts the communicator (ncclCommAbort) so the rank fails with an error that
//   names the bucket instead of hanging in the next wait.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
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

struct Comm {
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1, device = 0;
  hipStream_t stream = nullptr;
  // bucket engine
  std::vector<void*> bptr;
  std::vector<size_t> bcount;
  int bdtype = ncclFloat32, bop = ncclSum;
  std::vector<hipEvent_t> ready_ev, done_ev;
  std::vector<char> ready;
  std::vector<char> launched;
  std::vector<double> launch_us;   // host time of the bucket's launch, 0 = not pending
  int next_launch = 0;
  // watchdog (guarded by wd_mu: the bucket vectors are shared with the watchdog thread)
  std::recursive_mutex wd_mu;
  std::thread wd;
  std::atomic<bool> wd_stop{false}, aborted{false};
  double wd_timeout_us = 0;
  int wd_inject = -1;              // test hook: this bucket never reports completion
  std::string wd_err;
  // timeline
  bool tl_on = false;
  std::string tl_path;
  std::vector<TimelineEv> tl;
};

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

void tl_add(Comm* c, const std::string& name, const char* phase, char ph) {
  if (c->tl_on) c->tl.push_back({name, phase, ph, now_us()});
}

int launch_bucket(Comm* c, int b) {
  int rc = hcheck(hipStreamWaitEvent(c->stream, c->ready_ev[b], 0), "hipStreamWaitEvent");
  if (rc) return rc;
  tl_add(c, "bucket" + std::to_string(b), "ALLREDUCE", 'B');
  rc = check(api.AllReduce(c->bptr[b], c->bptr[b], c->bcount[b], c->bdtype, c->bop, c->comm, c->stream),
             "ncclAllReduce");
  if (rc) return rc;
  rc = hcheck(hipEventRecord(c->done_ev[b], c->stream), "hipEventRecord");
  tl_add(c, "bucket" + std::to_string(b), "ALLREDUCE", 'E');
  c->launched[b] = 1;
  c->launch_us[b] = now_us();
  return rc;
}

// one watchdog pass: 0 = healthy, 1 = aborted the communicator (reason in c->wd_err)
int watchdog_pass(Comm* c) {
  std::lock_guard<std::recursive_mutex> lk(c->wd_mu);
  std::string why;
  if (api.CommGetAsyncError) {
    ncclResult_t ar = 0;
    if (api.CommGetAsyncError(c->comm, &ar) == 0 && ar != 0)
      why = std::string("async RCCL error: ") + (api.GetErrorString ? api.GetErrorString(ar) : "?");
  }
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
  if (why.empty()) return 0;
  c->wd_err = "rank " + std::to_string(c->rank) + ": " + why + "; communicator aborted";
  if (api.CommAbort && c->comm) api.CommAbort(c->comm);
  c->comm = nullptr;
  c->aborted = true;
  set_err(c->wd_err);
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

}  // namespace

MXR_API const char* mxr_comm_last_error() { return g_err.c_str(); }

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
  if (check(api.CommInitRank(&c->comm, nranks, id, rank), "ncclCommInitRank")) {
    delete c;
    return nullptr;
  }
  int lo = 0, hi = 0;
  hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (hcheck(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi), "hipStreamCreate")) {
    api.CommDestroy(c->comm);
    delete c;
    return nullptr;
  }
  return c;
}

MXR_API int mxr_comm_destroy(void* h) {
  Comm* c = static_cast<Comm*>(h);
  if (!c) return 0;
  watchdog_stop(c);
  if (!c->aborted) hipStreamSynchronize(c->stream);
  for (auto e : c->ready_ev) hipEventDestroy(e);
  for (auto e : c->done_ev) hipEventDestroy(e);
  int rc = c->comm ? check(api.CommDestroy(c->comm), "ncclCommDestroy") : 0;
  hipStreamDestroy(c->stream);
  delete c;
  return rc;
}

// ---- plain collectives, ordered after the caller's stream and back (event handshake)
static int fence_in(Comm* c, hipStream_t s, hipEvent_t* ev) {
  int rc = hcheck(hipEventCreateWithFlags(ev, hipEventDisableTiming), "hipEventCreate");
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

MXR_API int mxr_comm_allreduce(void* h, const void* send, void* recv, long long count, int dtype, int avg,
                               hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::recursive_mutex> lk(c->wd_mu);   // no abort between fence and enqueue
  if (c->aborted) {
    set_err(c->wd_err);
    return -4;
  }
  hipEvent_t ev;
  int rc = fence_in(c, s, &ev);
  if (rc) return rc;
  rc = check(api.AllReduce(send, recv, (size_t)count, to_nccl_dtype(dtype), avg ? ncclAvg : ncclSum, c->comm,
                           c->stream), "ncclAllReduce");
  if (rc) return rc;
  return fence_out(c, s, ev);
}

MXR_API int mxr_comm_broadcast(void* h, void* buf, long long count, int dtype, int root, hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::recursive_mutex> lk(c->wd_mu);   // no abort between fence and enqueue
  if (c->aborted) {
    set_err(c->wd_err);
    return -4;
  }
  hipEvent_t ev;
  int rc = fence_in(c, s, &ev);
  if (rc) return rc;
  rc = check(api.Broadcast(buf, buf, (size_t)count, to_nccl_dtype(dtype), root, c->comm, c->stream), "ncclBroadcast");
  if (rc) return rc;
  return fence_out(c, s, ev);
}

MXR_API int mxr_comm_allgather(void* h, const void* send, void* recv, long long count, int dtype, hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::recursive_mutex> lk(c->wd_mu);   // no abort between fence and enqueue
  if (c->aborted) {
    set_err(c->wd_err);
    return -4;
  }
  hipEvent_t ev;
  int rc = fence_in(c, s, &ev);
  if (rc) return rc;
  rc = check(api.AllGather(send, recv, (size_t)count, to_nccl_dtype(dtype), c->comm, c->stream), "ncclAllGather");
  if (rc) return rc;
  return fence_out(c, s, ev);
}

MXR_API int mxr_comm_reduce_scatter(void* h, const void* send, void* recv, long long count, int dtype, int avg,
                                    hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::recursive_mutex> lk(c->wd_mu);   // no abort between fence and enqueue
  if (c->aborted) {
    set_err(c->wd_err);
    return -4;
  }
  hipEvent_t ev;
  int rc = fence_in(c, s, &ev);
  if (rc) return rc;
  rc = check(api.ReduceScatter(send, recv, (size_t)count, to_nccl_dtype(dtype), avg ? ncclAvg : ncclSum, c->comm,
                               c->stream), "ncclReduceScatter");
  if (rc) return rc;
  return fence_out(c, s, ev);
}

// ---- bucket engine
MXR_API int mxr_comm_set_buckets(void* h, int n, void** ptrs, const long long* counts, int dtype, int avg) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::recursive_mutex> lk(c->wd_mu);
  for (auto e : c->ready_ev) hipEventDestroy(e);
  for (auto e : c->done_ev) hipEventDestroy(e);
  c->ready_ev.assign(n, nullptr);
  c->done_ev.assign(n, nullptr);
  c->bptr.assign(ptrs, ptrs + n);
  c->bcount.resize(n);
  for (int i = 0; i < n; ++i) {
    c->bcount[i] = (size_t)counts[i];
    int rc = hcheck(hipEventCreateWithFlags(&c->ready_ev[i], hipEventDisableTiming), "hipEventCreate");
    if (!rc) rc = hcheck(hipEventCreateWithFlags(&c->done_ev[i], hipEventDisableTiming), "hipEventCreate");
    if (rc) return rc;
  }
  c->bdtype = to_nccl_dtype(dtype);
  c->bop = avg ? ncclAvg : ncclSum;
  c->ready.assign(n, 0);
  c->launched.assign(n, 0);
  c->launch_us.assign(n, 0.0);
  c->next_launch = 0;
  return 0;
}

// bucket b's gradients are complete on `compute`; launch every consecutive ready bucket in order
MXR_API int mxr_comm_bucket_ready(void* h, int b, hipStream_t compute) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::recursive_mutex> lk(c->wd_mu);
  if (c->aborted) {
    set_err(c->wd_err);
    return -4;
  }
  if (b < 0 || b >= (int)c->bptr.size() || c->ready[b]) return -3;
  int rc = hcheck(hipEventRecord(c->ready_ev[b], compute), "hipEventRecord");
  if (rc) return rc;
  c->ready[b] = 1;
  tl_add(c, "bucket" + std::to_string(b), "READY", 'i');
  while (c->next_launch < (int)c->bptr.size() && c->ready[c->next_launch]) {
    rc = launch_bucket(c, c->next_launch);
    if (rc) return rc;
    ++c->next_launch;
  }
  return 0;
}

// launch whatever is left (recording readiness on `compute` now), then make `compute` wait for all
MXR_API int mxr_comm_wait(void* h, hipStream_t compute) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::recursive_mutex> lk(c->wd_mu);
  if (c->aborted) {
    set_err(c->wd_err);
    return -4;
  }
  int rc;
  for (int b = 0; b < (int)c->bptr.size(); ++b)
    if (!c->ready[b] && (rc = mxr_comm_bucket_ready(h, b, compute))) return rc;
  for (int b = 0; b < (int)c->bptr.size(); ++b)
    if ((rc = hcheck(hipStreamWaitEvent(compute, c->done_ev[b], 0), "hipStreamWaitEvent"))) return rc;
  std::fill(c->ready.begin(), c->ready.end(), 0);
  std::fill(c->launched.begin(), c->launched.end(), 0);
  c->next_launch = 0;
  return 0;
}

MXR_API int mxr_comm_next_launch(void* h) { return static_cast<Comm*>(h)->next_launch; }

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

// 0 = healthy, 1 = aborted (message in mxr_comm_last_error)
MXR_API int mxr_comm_status(void* h) {
  Comm* c = static_cast<Comm*>(h);
  if (c->aborted) set_err(c->wd_err);
  return c->aborted ? 1 : 0;
}

// ---- timeline
MXR_API int mxr_comm_timeline(void* h, const char* path) {
  Comm* c = static_cast<Comm*>(h);
  c->tl_on = path && path[0];
  c->tl_path = c->tl_on ? path : "";
  c->tl.clear();
  return 0;
}

MXR_API int mxr_comm_timeline_flush(void* h) {
  Comm* c = static_cast<Comm*>(h);
  if (!c->tl_on) return 0;
  FILE* f = fopen(c->tl_path.c_str(), "w");
  if (!f) {
    set_err("cannot open timeline " + c->tl_path);
    return -1;
  }
  fprintf(f, "[\n");
  for (size_t i = 0; i < c->tl.size(); ++i) {
    const TimelineEv& e = c->tl[i];
    fprintf(f, "{\"name\": \"%s\", \"cat\": \"%s\", \"ph\": \"%c\", \"ts\": %.1f, \"pid\": %d, \"tid\": 0%s}%s\n",
            e.phase.c_str(), e.name.c_str(), e.ph, e.ts, c->rank, e.ph == 'i' ? ", \"s\": \"t\"" : "",
            i + 1 < c->tl.size() ? "," : "");
  }
  fprintf(f, "]\n");
  fclose(f);
  return 0;
}
