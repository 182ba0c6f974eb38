// Python bindings for the rdp HIP kernels (built in-tree as robotic_discovery_platform_amd/_C.so).
//
// Activations are NHWC bf16 torch tensors ([N,H,W,C], channel stride 1, possibly a channel slice
// of a wider tensor: pixel pitch = stride(2)). Every launcher validates shapes/strides here so a
// kernel never sees an inconsistent view; the kernels themselves use buffer descriptors sized from
// these views (out-of-range = zero / dropped, never a fault).
#include <torch/extension.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <link.h>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <vector>
#include <array>

extern "C" {
int rdp_conv_igemm(const void*, const void*, long, long, int, int, int, int, const void*, long, int, void*, void*, long,
                   long, int, int, int, float*, int, int, int, int, int, int, int, const float*, const float*, int,
                   float*, long, void*, int, int*, void*, int, int, int, int, int, const void*, int, const float*,
                   float*, int*, hipStream_t);
int rdp_conv_rowband_ex(const void*, const void*, long, long, int, int, int, int, const void*, long, int, void*, long, int,
                        int, int, int, int, const float*, const float*, int, void*, long, int, int, hipStream_t);
int rdp_conv_rowband_frag_auto(int, int, int, int, int, int);
int rdp_conv_rowband_chain(int, const void*, long, int, int, const void* const*, const long*, const int*, void* const*,
                           const long*, const int*, const int*, const float* const*, const float* const*, int, int, int,
                           int*, int*, hipStream_t);
int rdp_conv_ring_ex(const void*, long, int, int, const void*, long, int, void*, long, int, void*, long, int, int, int,
                     float*, int, int, int, const float*, const float*, int, int, const void*, int, const float*,
                     const float*, const float*, void*, long, int, hipStream_t);
long rdp_conv_ws_elems(int, int, int, int, int, int, int, int, int);
int rdp_geo_nblocks(int);
long rdp_geo_work_ints(int, int);
int rdp_geo_edges(const void*, const void*, int, int, double, double, double, double, double, int*, double*, double*,
                  double*, int, int*, double*, int, int*, int, double, int, double*, int, int*, const void*, int, int,
                  int*, double*, int*, int, void*, hipStream_t);
int rdp_preprocess(const void*, int, int, const int*, const int*, const float*, const int*, const int*, const float*, int,
                   int, int, void*, hipStream_t);
int rdp_mask_upsample(const void*, int, int, void*, int, int, unsigned*, hipStream_t);
int rdp_conv_wgrad(const void*, const void*, long, long, int, int, int, int, const void*, long, int, float*, long,
                   float*, int, int, int, int, int, int, int, int, int, int, hipStream_t);
long rdp_conv_wgrad_slab_elems(int, int, int, int, int, int, int, int);
long rdp_conv_wgrad_halo_slab_elems(int, int, int, int, int);
int rdp_wgrad_first_bn(const void*, long, int, const void*, long, int, const void*, long, int, const float*, const float*,
                       float*, long, float*, int, int, int, int, int, int, hipStream_t);
int rdp_bn_finalize(const float*, int, int, long, const float*, const float*, float*, float*, long long*, float, float,
                    float*, float*, hipStream_t);
int rdp_bn_eval_coef(int, const float*, const float*, const float*, const float*, float, float*, hipStream_t);
int rdp_bn_relu_apply(const void*, int, void*, int, const float*, int, int, int, hipStream_t);
int rdp_bn_relu_bwd_reduce(const void*, int, const void*, int, const float*, int, int, int, float*, int, hipStream_t);
int rdp_bn_bwd_finalize(const float*, int, int, long, const float*, const float*, float*, float*, float*, float*,
                        hipStream_t);
int rdp_bn_relu_bwd_apply(const void*, int, const void*, int, const float*, const float*, void*, int, int, int, int,
                          hipStream_t);
int rdp_maxpool2_fwd(const void*, int, void*, int, int, int, int, int, hipStream_t);
int rdp_conv_ring_head(const void*, long, int, int, const void*, long, int, int, int, int, int, const float*,
                       const float*, const float*, const float*, float, void*, hipStream_t);
int rdp_maxpool2_bwd(const void*, int, const void*, int, const void*, int, void*, int, int, int, int, int, hipStream_t);
int rdp_bn_relu_apply_pool(const void*, int, void*, int, void*, int, const float*, int, int, int, int, hipStream_t);
int rdp_maxpool2_bwd_bn_reduce(const void*, int, const void*, int, const void*, int, void*, int, const void*, int,
                               const float*, int, int, int, int, float*, int, hipStream_t);
int rdp_upsample2_fwd(const void*, int, void*, int, int, int, int, int, int, int, int, int, const float*,
                      hipStream_t);
int rdp_upsample2_bwd(const void*, int, void*, int, int, int, int, int, int, int, int, int, const void*, int,
                      const float*, float*, int, hipStream_t);
int rdp_conv_upT_fwd(const void*, long, int, int, const void*, long, int, void*, long, int, const float*, int, int, int, int,
                     int, int, int, int, hipStream_t);
int rdp_conv_upT_dgrad(const void*, long, int, int, int, int, int, int, const void*, long, int, void*, long, int, int,
                       int, int, int, hipStream_t);
int rdp_conv_wgrad_upT(const void*, long, int, int, int, int, int, int, const void*, long, int, int, int, int, int,
                       float*, long, float*, int, int, hipStream_t);
int rdp_upT_shuffle(const void*, int, const float*, void*, int, int, int, int, int, int, int, int, int, hipStream_t);
int rdp_upT_unshuffle(const void*, int, void*, int, int, int, int, int, int, int, int, int, hipStream_t);
int rdp_colsum_bf16(const void*, int, long, int, int, float*, float*, int, hipStream_t);
int rdp_head_partial_blocks(long);
int rdp_head_fwd(const void*, int, const float*, const float*, const float*, float*, float*, float*, float*, int, float,
                 float, const float*, float*, float*, float, hipStream_t);
int rdp_head_grad_finalize(const float*, int, float*, float*, hipStream_t);
int rdp_head_bwd(const void*, int, const float*, const float*, const float*, const float*, void*, int, float*, float*,
                 float*, int, float, float, float, const float*, float*, hipStream_t);
int rdp_head_bn_bwd_apply(const void*, int, const float*, const float*, const float*, const float*, const float*,
                          const float*, void*, int, int, float, float, float, hipStream_t);
int rdp_head_mask(const void*, int, const float*, const float*, float, void*, int, hipStream_t);
int rdp_adam(float*, const void*, int, float*, float*, void*, long, float, float, float, float, float, float, int*, int,
             int, hipStream_t);
int rdp_cast_bf16(const float*, void*, long, hipStream_t);
int rdp_comm_emulate(double, int, hipStream_t);
int rdp_comm_emulate_traffic(double, int, void*, long, long, hipStream_t);
int rdp_rows_fold(const float*, int, int, double*, hipStream_t);
int rdp_rows_hilo(const double*, float*, int, hipStream_t);
int rdp_wprep(const float*, void*, const void*, int, int*, int, int, hipStream_t);
int rdp_wseg_size();
int rdp_h2d_copy(const void*, void*, long, hipStream_t);
int rdp_parcur(int, int, const double*, const double*, double, int, int, double*, double*, int*, double*);
double rdp_splev1(const double*, int, const double*, int, double, int);
int rdp_fit_curvature(const double*, int, double, int, int, double, double*, double*);
int rdp_geo_spline_res_len(int);
int rdp_preprocess_batch(int, const void* const*, int, int, const int*, const int*, const float*, const int*,
                         const int*, const float*, int, int, int, void* const*, hipStream_t);
int rdp_jpeg_gpu_batch(int, const void* const*, const int* const*, const int* const*, void* const*, int, int, int,
                       void* const*, hipStream_t);
int rdp_geo_edges_batch(int, const void* const*, const void* const*, int, int, double, double, double, double, double,
                        int* const*, double* const*, double* const*, double* const*, int, int* const*, double* const*,
                        int, int* const*, int, double, int, const void* const*, int, int, int* const*, double* const*,
                        int* const*, int, void* const*, hipStream_t);
int rdp_geo_spline_batch(int, int, int, const int* const*, const int* const*, double* const*, double* const*, int,
                         double, int, int, double, int, int, const int* const*, int, double* const*, const void* const*,
                         void* const*, long, hipStream_t);
int rdp_png_info(const uint8_t*, long, int*, int*, int*);
long rdp_jpeg_info(const uint8_t*, long, int*);
void rdp_jpeg_meta(const int*, int*);
int rdp_jpeg_decode(const uint8_t*, long, int16_t*, long, uint16_t*, int);
int rdp_jpeg_gpu(const void*, const int*, const int*, void*, int, int, int, void*, hipStream_t);
long rdp_jpeg_plane_bytes(int, int);
long rdp_jpeg_max_coefs(int, int);
int rdp_png_decode(const uint8_t*, long, uint8_t*, long, int);
long rdp_png_encode_gray(const uint8_t*, int, int, int, int, int, uint8_t*, long);
long rdp_png_encode_bound(int, int, int, int);
int rdp_area_maxtap();
int rdp_resize_area_u8(const void*, int, int, int, const int*, const int*, const double*, const int*, const int*,
                       const double*, int, int, int, void*, hipStream_t);
int rdp_geo_spline(const double*, int, int, const int*, const int*, double*, int*, double*, int, double, int, int,
                   double, int, int, const int*, int, double*, double*, int, const void*, void*, long, hipStream_t);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// ---- device placement: every binding runs on the GPU that holds its tensors -------------------------
// `on_device(fn)` wraps a binding: it checks that every GPU tensor argument (plain or optional) lives
// on ONE device and makes that device current for the call (HIPGuard), so the launches below go to
// that device's current stream -- a per-GPU serving replica (serve/engine.py EnginePool) launches on
// its own GPU whatever device the calling thread had current. Mixed devices raise.
void note_device(int& dev, const torch::Tensor& t) {
  if (!t.defined() || !t.is_cuda()) return;
  const int d = t.get_device();
  TORCH_CHECK(dev < 0 || d == dev, "tensor arguments on different GPUs (cuda:", dev, " and cuda:", d, ")");
  dev = d;
}
void note_device(int& dev, const c10::optional<torch::Tensor>& t) {
  if (t) note_device(dev, *t);
}
void note_device(int& dev, const std::vector<torch::Tensor>& ts) {
  for (const auto& t : ts) note_device(dev, t);
}
template <class T>
void note_device(int&, const T&) {}

template <class R, class... A>
auto on_device(R (*fn)(A...)) {
  return [fn](A... args) -> R {
    int dev = -1;
    (note_device(dev, args), ...);
    c10::hip::OptionalHIPGuard guard;
    if (dev >= 0) guard.set_index((c10::DeviceIndex)dev);
    return fn(std::move(args)...);
  };
}

// ---- launch plans: the training step recorded once and replayed from C++ --------------------------
// A plan is the step's launch sequence: every kernel launch of the bindings below (RDP_PLAN) and every
// cross-stream dependency (stream_wait), in issue order, each with the HIP stream it was issued on.
// Recording runs the step normally and keeps, per launch, a closure over the already-validated raw
// arguments (pointers into the executor's static buffers, ints); replay re-issues the closures on
// the recorded streams -- about 1-2 us of host time per launch instead of the Python executor's
// ~8 us, so at small batch the host stays ahead of the GPU (bs 4: 1.55 ms of host enqueue per 2.5 ms
// step, with idle gaps wherever a run of short kernels outpaced it). Unlike a hipGraph, replay keeps
// the eager launch order on the same two streams / hardware queues (graph replay spread the side
// branch over extra queues and measured slower, train/engine.py).
//
// A plan may also hold host call points (kind 2, ``plan_mark``): work the runtime cannot replay itself
// (the DDP bucket all-reduces, issued through torch.distributed). Recording marks the point, then runs
// that work with recording paused (``plan_pause`` / ``plan_resume``); replay calls back into Python with
// the mark's tag at the same position in the launch sequence, so the collectives keep their place
// between the recorded kernels.
struct PlanOp {
  int kind;        // 0: launch, 1: waiter waits for everything issued so far on waitee, 2: host call,
                   // 3: record a runtime-owned event on s, 4: s waits for that event's last record
  hipStream_t s;   // launch stream / waiter
  hipStream_t s2;  // waitee
  hipEvent_t ev;
  std::function<long(hipStream_t)> fn;
  int tag = -1;    // kind 2: the caller's call-point id
};
struct Plan {
  std::vector<PlanOp> ops;
};
std::vector<std::unique_ptr<Plan>> g_plans;
Plan* g_rec = nullptr;
Plan* g_paused = nullptr;  // the plan being recorded while a host call point runs

template <class F>
long plan_launch(F&& f) {
  const hipStream_t s = cur_stream();
  if (g_rec) g_rec->ops.push_back(PlanOp{0, s, nullptr, nullptr, std::function<long(hipStream_t)>(f)});
  return f(s);
}
#define RDP_PLAN(...) plan_launch([=](hipStream_t st) -> long { return (long)(__VA_ARGS__); })

// launches that a plan cannot hold (serving / geometry bindings): refuse while recording
hipStream_t unplanned_stream() {
  TORCH_CHECK(g_rec == nullptr, "this kernel launch cannot be recorded into a plan");
  return cur_stream();
}

// One reusable timing-free event per device and host thread for the eager path: hipStreamWaitEvent
// captures the event's most recent record at the time of the call, so re-recording it for the next
// wait is safe (no create / destroy per call). A plan being recorded owns one event per wait.
// Cross-stream dependencies on one GPU only order kernels, and every kernel dispatch already carries its
// own acquire / release fences, so the events skip the system-scope fence (L2 writeback for host
// visibility) that a default event record inserts into the waitee's queue: bs 4 step 2.50-2.53 ->
// 2.48 ms (1,584-1,601 -> 1,615 img/s, 2 rounds, same box; a device-scope release instead: no change;
// bs 64 neutral).
static unsigned wait_event_flags() { return hipEventDisableTiming | hipEventDisableSystemFence; }

hipEvent_t wait_event(hipStream_t s) {
  int dev = 0;
  TORCH_CHECK(hipStreamGetDevice(s, &dev) == hipSuccess, "stream_wait: stream device");
  thread_local std::vector<hipEvent_t> evs;
  if ((int)evs.size() <= dev) evs.resize(dev + 1, nullptr);
  if (!evs[dev]) {
    c10::hip::HIPGuard g((c10::DeviceIndex)dev);
    TORCH_CHECK(hipEventCreateWithFlags(&evs[dev], wait_event_flags()) == hipSuccess, "stream_wait: event");
  }
  return evs[dev];
}

void stream_wait(long waiter, long waitee) {
  const hipStream_t w = (hipStream_t)waiter, e = (hipStream_t)waitee;
  hipEvent_t ev;
  if (g_rec) {
    int dev = 0;
    TORCH_CHECK(hipStreamGetDevice(e, &dev) == hipSuccess, "stream_wait: stream device");
    c10::hip::HIPGuard g((c10::DeviceIndex)dev);
    TORCH_CHECK(hipEventCreateWithFlags(&ev, wait_event_flags()) == hipSuccess, "stream_wait: event");
  } else {
    ev = wait_event(e);
  }
  TORCH_CHECK(hipEventRecord(ev, e) == hipSuccess && hipStreamWaitEvent(w, ev, 0) == hipSuccess, "stream_wait");
  if (g_rec) g_rec->ops.push_back(PlanOp{1, w, e, ev, nullptr});
}

// Named cross-stream points (runtime-owned events, recorded into plans): event_record marks "everything
// issued so far on this stream", stream_wait_event makes another stream wait for the LAST such mark --
// a dependency on a point in the middle of a stream's work (NativeAdam's overlapped update: the next
// forward waits for the update, not for the weight re-layouts queued behind it).
std::vector<hipEvent_t> g_events;

int event_create() {
  hipEvent_t e;
  TORCH_CHECK(hipEventCreateWithFlags(&e, wait_event_flags()) == hipSuccess, "event_create");
  g_events.push_back(e);
  return (int)g_events.size() - 1;
}

void event_record(int id, long stream) {
  TORCH_CHECK(id >= 0 && id < (int)g_events.size(), "event_record: bad event id");
  const hipStream_t s = (hipStream_t)stream;
  TORCH_CHECK(hipEventRecord(g_events[id], s) == hipSuccess, "event_record");
  if (g_rec) g_rec->ops.push_back(PlanOp{3, s, nullptr, g_events[id], nullptr});
}

void stream_wait_event(long stream, int id) {
  TORCH_CHECK(id >= 0 && id < (int)g_events.size(), "stream_wait_event: bad event id");
  const hipStream_t s = (hipStream_t)stream;
  TORCH_CHECK(hipStreamWaitEvent(s, g_events[id], 0) == hipSuccess, "stream_wait_event");
  if (g_rec) g_rec->ops.push_back(PlanOp{4, s, nullptr, g_events[id], nullptr});
}

void plan_begin() {
  TORCH_CHECK(g_rec == nullptr && g_paused == nullptr, "plan_begin: already recording");
  g_plans.emplace_back(new Plan());
  g_rec = g_plans.back().get();
}

int plan_end() {
  TORCH_CHECK(g_rec != nullptr, "plan_end: not recording");
  g_rec = nullptr;
  return (int)g_plans.size() - 1;
}

void plan_abort() {
  if (g_paused) {
    g_rec = g_paused;
    g_paused = nullptr;
  }
  if (g_rec) {
    for (auto& op : g_rec->ops) if (op.ev && op.kind == 1) hipEventDestroy(op.ev);
    g_rec->ops.clear();
    g_rec = nullptr;
  }
}

bool plan_recording() { return g_rec != nullptr; }

void plan_mark(int tag) {
  TORCH_CHECK(g_rec != nullptr, "plan_mark: not recording");
  PlanOp op{2, nullptr, nullptr, nullptr, nullptr};
  op.tag = tag;
  g_rec->ops.push_back(std::move(op));
}

void plan_pause() {
  TORCH_CHECK(g_rec != nullptr && g_paused == nullptr, "plan_pause: not recording");
  g_paused = g_rec;
  g_rec = nullptr;
}

void plan_resume() {
  TORCH_CHECK(g_paused != nullptr && g_rec == nullptr, "plan_resume: not paused");
  g_rec = g_paused;
  g_paused = nullptr;
}

void plan_replay(int id, py::object host_call) {
  TORCH_CHECK(id >= 0 && id < (int)g_plans.size() && g_plans[id], "plan_replay: bad plan id");
  TORCH_CHECK(g_rec == nullptr && g_paused == nullptr, "plan_replay while recording");
  for (auto& op : g_plans[id]->ops) {
    if (op.kind == 0) {
      op.fn(op.s);
    } else if (op.kind == 1) {
      hipEventRecord(op.ev, op.s2);
      hipStreamWaitEvent(op.s, op.ev, 0);
    } else if (op.kind == 3) {
      hipEventRecord(op.ev, op.s);
    } else if (op.kind == 4) {
      hipStreamWaitEvent(op.s, op.ev, 0);
    } else {
      TORCH_CHECK(!host_call.is_none(), "plan_replay: the plan has host call points, pass a callback");
      host_call(op.tag);
    }
  }
}

int plan_size(int id) {
  TORCH_CHECK(id >= 0 && id < (int)g_plans.size() && g_plans[id], "plan_size: bad plan id");
  return (int)g_plans[id]->ops.size();
}

// the op kinds of a recorded plan, in order (tests: which cross-stream waits a plan holds)
std::vector<int> plan_kinds(int id) {
  TORCH_CHECK(id >= 0 && id < (int)g_plans.size() && g_plans[id], "plan_kinds: bad plan id");
  std::vector<int> k;
  for (auto& op : g_plans[id]->ops) k.push_back(op.kind);
  return k;
}

void plan_free(int id) {
  if (id < 0 || id >= (int)g_plans.size() || !g_plans[id]) return;
  for (auto& op : g_plans[id]->ops) if (op.ev && op.kind == 1) hipEventDestroy(op.ev);
  g_plans[id].reset();
}

// ---- RCCL collectives enqueued straight onto HIP streams ---------------------------------------------
// The DDP gradient buckets are all-reduced with ncclAllReduce on the communicator of a dedicated
// torch.distributed (nccl = RCCL) process group (ProcessGroupNCCL._comm_ptr), issued on the executor's
// stream in stream order -- no ProcessGroupNCCL work objects, events or host waits per bucket -- and
// recorded into launch plans like a kernel launch, so a DDP step replays from C++ with its collectives
// in place. The entry points are resolved from the librccl instance torch itself loaded (the
// communicator belongs to it), never from another copy of the library.
typedef int (*NcclAllReduceFn)(const void*, void*, size_t, int, int, void*, hipStream_t);
typedef int (*NcclAsyncErrFn)(void*, int*);
typedef const char* (*NcclErrStrFn)(int);
typedef int (*NcclAbortFn)(void*);
typedef int (*NcclCommIntFn)(const void*, int*);
struct RcclApi {
  NcclAllReduceFn all_reduce = nullptr;
  NcclAsyncErrFn async_err = nullptr;
  NcclErrStrFn err_str = nullptr;
  NcclAbortFn abort = nullptr;
  NcclCommIntFn count = nullptr, user_rank = nullptr, device = nullptr;
  std::string path;
} g_rccl;

int find_loaded_rccl(struct dl_phdr_info* info, size_t, void* out) {
  if (info->dlpi_name && std::strstr(info->dlpi_name, "librccl")) {
    *(std::string*)out = info->dlpi_name;
    return 1;
  }
  return 0;
}

std::string comm_bind() {
  if (g_rccl.all_reduce) return g_rccl.path;
  std::string path;
  dl_iterate_phdr(find_loaded_rccl, &path);
  TORCH_CHECK(!path.empty(), "comm_bind: RCCL is not loaded in this process (create the nccl process group first)");
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);
  TORCH_CHECK(h != nullptr, "comm_bind: dlopen ", path);
  g_rccl.all_reduce = (NcclAllReduceFn)dlsym(h, "ncclAllReduce");
  g_rccl.async_err = (NcclAsyncErrFn)dlsym(h, "ncclCommGetAsyncError");
  g_rccl.err_str = (NcclErrStrFn)dlsym(h, "ncclGetErrorString");
  g_rccl.abort = (NcclAbortFn)dlsym(h, "ncclCommAbort");
  g_rccl.count = (NcclCommIntFn)dlsym(h, "ncclCommCount");
  g_rccl.user_rank = (NcclCommIntFn)dlsym(h, "ncclCommUserRank");
  g_rccl.device = (NcclCommIntFn)dlsym(h, "ncclCommCuDevice");
  TORCH_CHECK(g_rccl.count && g_rccl.user_rank && g_rccl.device &&
              g_rccl.all_reduce && g_rccl.async_err && g_rccl.err_str && g_rccl.abort, "comm_bind: RCCL symbols in ",
              path);
  g_rccl.path = path;
  return path;
}

long rccl_check(int r, void* comm) {
  constexpr int kInProgress = 7;  // ncclInProgress: a non-blocking communicator is still enqueuing
  // bounded: the communicators are created blocking (parallel/ddp.py), so this loop should never
  // spin; if one does, fail after RDP_DIST_TIMEOUT_S instead of hanging the issuing thread
  static const double limit_s = [] {
    const char* v = std::getenv("RDP_DIST_TIMEOUT_S");
    return v ? std::atof(v) : 600.0;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  while (r == kInProgress) {
    int e = 0;
    g_rccl.async_err(comm, &e);
    r = e;
    if (r == kInProgress &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) {
      g_rccl.abort(comm);
      TORCH_CHECK(false, "ncclAllReduce: still in progress after ", limit_s, " s; communicator aborted");
    }
  }
  TORCH_CHECK(r == 0, "ncclAllReduce: ", g_rccl.err_str(r));
  return 0;
}

// in-place SUM all-reduce of `buf` (fp32 or bf16) over `comm`, on the current stream
void comm_all_reduce(torch::Tensor buf, long comm) {
  TORCH_CHECK(g_rccl.all_reduce != nullptr, "comm_all_reduce: call comm_bind() first");
  TORCH_CHECK(buf.is_cuda() && buf.is_contiguous(), "comm_all_reduce: contiguous device tensor");
  const int dt = buf.scalar_type() == torch::kFloat      ? 7
                 : buf.scalar_type() == torch::kBFloat16 ? 9
                 : buf.scalar_type() == torch::kDouble   ? 8
                                                         : -1;
  TORCH_CHECK(dt >= 0 && comm != 0, "comm_all_reduce: fp32 / bf16 / fp64 buffer and a communicator");
  void* const p = buf.data_ptr();
  const size_t n = (size_t)buf.numel();
  void* const c = (void*)comm;
  const NcclAllReduceFn fn = g_rccl.all_reduce;
  RDP_PLAN(rccl_check(fn(p, p, n, dt, /*ncclSum*/ 0, c, st), c));
}

// SyncBN: fold buf's [rows][width] fp32 partial rows into `out` (width fp64 sums) / write fp64 sums back as
// hi + lo fp32 rows; both recorded in plans
void rows_fold(torch::Tensor buf, int rows, int width, torch::Tensor out) {
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == torch::kFloat && buf.is_contiguous() &&
              (long)rows * width <= buf.numel() && rows >= 1 && width >= 1, "rows_fold: fp32 buffer of rows x width");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kDouble && out.is_contiguous() && out.numel() >= width,
              "rows_fold: fp64 out");
  const float* p = buf.data_ptr<float>();
  double* o = out.data_ptr<double>();
  RDP_PLAN(rdp_rows_fold(p, rows, width, o, st));
}

void rows_hilo(torch::Tensor in, torch::Tensor buf, int width) {
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == torch::kDouble && in.is_contiguous() && in.numel() >= width,
              "rows_hilo: fp64 sums");
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == torch::kFloat && buf.is_contiguous() && buf.numel() >= 2l * width,
              "rows_hilo: fp32 buffer of 2 rows");
  const double* i = in.data_ptr<double>();
  float* b = buf.data_ptr<float>();
  RDP_PLAN(rdp_rows_hilo(i, b, width, st));
}

// ncclCommGetAsyncError of `comm` (0 = healthy) and its message: polled by the host watchdog
// (parallel/watchdog.py) while natively issued collectives are outstanding -- they have no
// ProcessGroupNCCL work objects, so c10d's own watchdog never sees them.
py::tuple comm_async_error(long comm) {
  TORCH_CHECK(g_rccl.async_err != nullptr && comm != 0, "comm_async_error: call comm_bind() first");
  int e = 0;
  const int r = g_rccl.async_err((void*)comm, &e);
  const int code = r != 0 ? r : e;
  return py::make_tuple(code, std::string(code ? g_rccl.err_str(code) : ""));
}

// (ranks, this rank, device) of `comm` as RCCL itself sees them (ncclCommCount / ncclCommUserRank /
// ncclCommCuDevice): bench.py's self-check that the gradient communicator spans WORLD_SIZE ranks
py::tuple comm_info(long comm) {
  TORCH_CHECK(g_rccl.count != nullptr && comm != 0, "comm_info: call comm_bind() first");
  int n = -1, r = -1, d = -1;
  TORCH_CHECK(g_rccl.count((void*)comm, &n) == 0, "ncclCommCount failed");
  TORCH_CHECK(g_rccl.user_rank((void*)comm, &r) == 0, "ncclCommUserRank failed");
  TORCH_CHECK(g_rccl.device((void*)comm, &d) == 0, "ncclCommCuDevice failed");
  return py::make_tuple(n, r, d);
}

// ncclCommAbort: unblocks every kernel of the communicator still waiting on a dead peer (the watchdog's
// last step before it exits the process)
int comm_abort(long comm) {
  TORCH_CHECK(g_rccl.abort != nullptr && comm != 0, "comm_abort: call comm_bind() first");
  py::gil_scoped_release nogil;
  return g_rccl.abort((void*)comm);
}

// RDP_DDP_EMULATE: the modelled all-reduce (`us` microseconds, `blocks` resident workgroups) on the current
// stream in place of ncclAllReduce (csrc/comm.hip), recorded into plans like the real call
// with `scratch` and traffic_bytes > 0: the modelled collective's HBM traffic too (traffic_bytes read from
// the scratch's first half and written to its second, paced over the duration)
void comm_emulate(double us, int blocks, c10::optional<torch::Tensor> scratch, long traffic_bytes) {
  TORCH_CHECK(us >= 0 && blocks >= 1 && blocks <= 4096, "comm_emulate: bad duration / block count");
  if (scratch && traffic_bytes > 0) {
    TORCH_CHECK(scratch->is_cuda() && scratch->is_contiguous() &&
                    scratch->numel() * scratch->element_size() >= 2 * traffic_bytes,
                "comm_emulate: scratch must hold 2 x traffic_bytes");
    void* const p = scratch->data_ptr();
    const long nb = scratch->numel() * scratch->element_size();
    TORCH_CHECK(RDP_PLAN(rdp_comm_emulate_traffic(us, blocks, p, nb, traffic_bytes, st)) == 0, "comm_emulate_traffic");
    return;
  }
  RDP_PLAN(rdp_comm_emulate(us, blocks, st));
}

struct Act {
  void* ptr = nullptr;
  int N = 0, H = 0, W = 0, C = 0, pitch = 0;
  long bytes = 0;
};

Act act(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, ": must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16, name, ": must be bf16");
  TORCH_CHECK(t.dim() == 4, name, ": must be NHWC 4-D");
  Act a;
  a.N = t.size(0); a.H = t.size(1); a.W = t.size(2); a.C = t.size(3);
  TORCH_CHECK(t.stride(3) == 1, name, ": channel stride must be 1");
  a.pitch = t.stride(2);
  TORCH_CHECK(a.pitch >= a.C, name, ": pixel pitch < C");
  TORCH_CHECK(t.stride(1) == (long)a.W * a.pitch && t.stride(0) == (long)a.H * a.W * a.pitch, name,
              ": pixels must be densely packed (only channel slicing allowed)");
  TORCH_CHECK(a.pitch % 8 == 0 && ((uintptr_t)t.data_ptr() % 16) == 0, name, ": pitch/base must be 16-B aligned");
  a.ptr = t.data_ptr();
  a.bytes = ((long)a.N * a.H * a.W - 1) * a.pitch * 2 + (long)a.C * 2;
  return a;
}

// Images per launch so that every tensor of the launch stays below 2 GiB (the conv kernels' 32-bit
// buffer offsets). RDP_CONV_CHUNK_BYTES (tests) lowers the bound to exercise the chunked path.
int chunk_images(long bytes_per_image, int N) {
  static const long lim = [] {
    const char* e = getenv("RDP_CONV_CHUNK_BYTES");
    const long v = e ? atol(e) : 0L;
    return v > 0 ? v : (1L << 31) - 1;
  }();
  if (bytes_per_image <= 0 || bytes_per_image * N <= lim) return N > 0 ? N : 1;
  return (int)std::max(1L, lim / bytes_per_image);
}

void check_f32(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous(), name,
              ": must be a contiguous fp32 GPU tensor");
}

// reduction workspace for the two-stage BN finalize (>= 64 rows x K floats), or nullptr
float* ws_ptr(const c10::optional<torch::Tensor>& ws, int K) {
  if (!ws) return nullptr;
  check_f32(*ws, "ws");
  TORCH_CHECK(ws->numel() >= 64l * K, "workspace too small");
  return ws->data_ptr<float>();
}

// stats slab rows written by conv_fwd: one per (M tile, wave row)
int conv_stats_rows(long M, int Cout, int bm_pref) {
  bm_pref %= 1000;
  // forced tiles: one row per (M tile, wave row), or up to 512 rows when split-K reduces them
  if (bm_pref == 128 && Cout % 128 == 0) return (int)std::max<long>((M + 127) / 128 * 2, 512);
  if (bm_pref == 256) return (int)std::max<long>((M + 255) / 256 * 4, 512);
  // auto / halo: upper bound over every tile choice (halo: up to 8 wave rows per 256-pixel tile)
  // split-K reduce: up to 512 rows
  const long a = (M + 127) / 128 * 2, b = (M + 255) / 256 * 8;
  const long ab = a > b ? a : b;
  // + room for batch-chunked launches (conv_fwd: tensors past 2 GiB run as image slices, each with
  // its own 512-row floor and tile rounding): one chunk per 2 GiB of a 1024-channel bf16 tensor
  const long chunks = 1 + M * 2048 / (1L << 31);
  return (int)((ab > 512 ? ab : 512) + 520 * chunks);
}

// y = conv(cat(x1, x2), w); returns #M-tiles (stats rows)
int conv_fwd(torch::Tensor x1, c10::optional<torch::Tensor> x2, torch::Tensor w, int taps, int packed,
             torch::Tensor y1, c10::optional<torch::Tensor> y2, c10::optional<torch::Tensor> stats, int bm_pref,
             c10::optional<torch::Tensor> affine, int relu, c10::optional<torch::Tensor> ws,
             c10::optional<torch::Tensor> pool, c10::optional<torch::Tensor> up, int up_oy, int up_ox,
             c10::optional<torch::Tensor> wfrag) {
  Act a1 = act(x1, "x1"), a2;
  if (x2) {
    a2 = act(*x2, "x2");
    TORCH_CHECK(a2.N == a1.N && a2.H == a1.H && a2.W == a1.W, "x2 spatial mismatch");
  }
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kBFloat16 && w.is_contiguous() && w.dim() == 2, "w: bf16 [Cout][K]");
  Act o1 = act(y1, "y1"), o2;
  int Cout = o1.C;
  if (y2) { o2 = act(*y2, "y2"); Cout += o2.C; }
  TORCH_CHECK(o1.N == a1.N && o1.H == a1.H && o1.W == a1.W, "y spatial mismatch");
  TORCH_CHECK(w.size(0) == Cout, "w rows != Cout");
  float* sp = nullptr;
  if (stats) {
    check_f32(*stats, "stats");
    const long M = (long)a1.N * a1.H * a1.W;
    const long rows = conv_stats_rows(M, Cout, bm_pref);
    TORCH_CHECK(stats->numel() >= rows * 2 * Cout, "stats slab too small");
    sp = stats->data_ptr<float>();
  }
  const float* esc = nullptr;
  const float* esh = nullptr;
  if (affine) {  // BN coefficient block [mean | invstd | scale | shift] (4*Cout floats)
    check_f32(*affine, "affine");
    TORCH_CHECK(affine->numel() >= 4l * Cout, "affine must hold 4*Cout floats");
    esc = affine->data_ptr<float>() + 2 * Cout;
    esh = affine->data_ptr<float>() + 3 * Cout;
  }
  if (ws) check_f32(*ws, "ws");
  // pool (eval): MaxPool2d(2) of y1 -> pool [N][H/2][W/2][Cout]; fused into the split-K reduce when
  // that path runs, else a maxpool2_fwd launch after the conv
  Act po;
  if (pool) {
    po = act(*pool, "pool");
    TORCH_CHECK(!y2 && !stats && po.N == o1.N && po.H == o1.H / 2 && po.W == o1.W / 2 && po.C == o1.C,
                "pool: eval conv with one destination, [N][H/2][W/2][Cout]");
  }
  // up (eval): bilinear x2 upsample of y1 into up at (up_oy, up_ox); fused into the split-K reduce
  // when that path runs, else an upsample2_fwd launch after the conv
  Act uo;
  if (up) {
    uo = act(*up, "up");
    TORCH_CHECK(!pool && !y2 && !stats && uo.N == o1.N && uo.C == o1.C && up_oy >= 0 && up_ox >= 0 &&
                2 * o1.H + up_oy <= uo.H && 2 * o1.W + up_ox <= uo.W, "up: eval conv, [N][>=2H][>=2W][Cout]");
  }
  // Batch chunks: the conv kernels address each tensor through ONE buffer descriptor with 32-bit
  // offsets (< 2 GiB), so a batch whose largest tensor passes that (256^2 x 64 ch bf16 at N >= 256)
  // runs as consecutive launches over image slices (convs never cross images); BN partial rows of
  // the slices are appended, fused pool / upsample outputs sliced alike.
  const long per_img = std::max(std::max((long)a1.H * a1.W * a1.pitch, x2 ? (long)a2.H * a2.W * a2.pitch : 0L),
                                std::max((long)o1.H * o1.W * o1.pitch, y2 ? (long)o2.H * o2.W * o2.pitch : 0L)) * 2;
  const int nc = chunk_images(per_img, a1.N);
  const long avail_rows = stats ? stats->numel() / (2l * Cout) : 0;
  int rows = 0;
  for (int n0 = 0; n0 < a1.N; n0 += nc) {
    const int nn = std::min(nc, a1.N - n0);
    // every launch argument is a value here: RDP_PLAN may keep the launch for replay (plan mode)
    auto img = [](const Act& t, int n) { return (void*)((char*)t.ptr + (long)n * t.H * t.W * t.pitch * 2); };
    auto nbytes = [nn](const Act& t) { return ((long)nn * t.H * t.W - 1) * t.pitch * 2 + (long)t.C * 2; };
    float* spc = sp ? sp + (long)rows * 2 * Cout : nullptr;
    if (sp) TORCH_CHECK(rows + conv_stats_rows((long)nn * a1.H * a1.W, Cout, bm_pref) <= avail_rows, "stats slab too small");
    void* const px1 = img(a1, n0);
    void* const px2 = x2 ? img(a2, n0) : nullptr;
    void* const py1 = img(o1, n0);
    void* const py2 = y2 ? img(o2, n0) : nullptr;
    void* const ppo = pool ? img(po, n0) : nullptr;
    void* const pup = up ? img(uo, n0) : nullptr;
    const long bx1 = nbytes(a1), bx2 = x2 ? nbytes(a2) : 0, by1 = nbytes(o1), by2 = y2 ? nbytes(o2) : 0;
    void* const wp = w.data_ptr();
    const long wb = w.numel() * 2, ldw = w.size(1);
    float* const wsp = ws ? ws->data_ptr<float>() : nullptr;
    const long wsn = ws ? (long)ws->numel() : 0L;
    const int C2 = x2 ? a2.C : 0, p2 = x2 ? a2.pitch : 0, yp2 = y2 ? o2.pitch : 0, ppit = pool ? po.pitch : 0;
    const int upit = up ? uo.pitch : 0, uH = up ? uo.H : 0, uW = up ? uo.W : 0;
    const bool want_fused = pool || up;
    // the fused pool / upsample result flag: a heap cell owned by the launch (kept alive in a plan)
    auto pooled = std::make_shared<int>(0);
    // eval with the fragment-major weight copy (wfrag): the row-band kernel wherever its traffic model picks it
    const int fmode = wfrag && esc && !sp && !y2 && taps == 9 && !packed && bm_pref == 0
                          ? rdp_conv_rowband_frag_auto(nn, a1.H, a1.W, a1.C, C2, Cout) : 0;
    int r = -1;
    if (fmode > 0) {
      void* const wfp = wfrag->data_ptr();
      const long wfb = wfrag->numel() * 2;
      const long pbytes = pool ? ((long)nn * po.H * po.W - 1) * ppit * 2 + (long)po.C * 2 : 0;
      const int rb = RDP_PLAN(rdp_conv_rowband_ex(px1, px2, bx1, bx2, a1.C, C2, a1.pitch, p2, wfp, wfb, 0, py1, by1,
                                                  o1.pitch, nn, a1.H, a1.W, Cout, esc, esh, relu, ppo, pbytes, ppit, fmode,
                                                  st));
      // the selector checks every predicate of the launch; should one still reject (rb < 0: nothing was
      // launched), the layer runs on the implicit GEMM below instead of failing the eval
      if (rb >= 0) {
        *pooled = rb == 1 ? 1 : 0;
        r = 0;
      }
    }
    if (r < 0) {
      r = RDP_PLAN(rdp_conv_igemm(px1, px2, bx1, bx2, a1.C, C2, a1.pitch, p2, wp, wb, (int)ldw, py1, py2, by1, by2, o1.C,
                                  o1.pitch, yp2, spc, nn, a1.H, a1.W, Cout, taps, packed, bm_pref, esc, esh, relu, wsp,
                                  wsn, ppo, ppit, want_fused ? pooled.get() : nullptr, pup, upit, uH, uW, up_oy, up_ox,
                                  nullptr, 0, nullptr, nullptr, nullptr, st));
    }
    TORCH_CHECK(r >= 0, "conv_fwd: unsupported shape (C1=", a1.C, ", C2=", C2, ", Cout=", Cout, ")");
    const int oN = nn, oH = o1.H, oW = o1.W, oC = o1.C, op1 = o1.pitch;
    if (pool && !*pooled)
      TORCH_CHECK(RDP_PLAN(rdp_maxpool2_fwd(py1, op1, ppo, ppit, oN, oH, oW, oC, st)) == 0, "conv_fwd: maxpool");
    if (up && !*pooled)
      TORCH_CHECK(RDP_PLAN(rdp_upsample2_fwd(py1, op1, pup, upit, oN, oH, oW, uH, uW, up_oy, up_ox, oC, nullptr, st)) == 0,
                  "conv_fwd: upsample");
    rows += r;
  }
  return rows;
}


int conv_wgrad(torch::Tensor x1, c10::optional<torch::Tensor> x2, torch::Tensor dy, int taps, int packed, int cin_real,
               torch::Tensor slab, torch::Tensor out, int accumulate, int splits, int variant) {
  Act a1 = act(x1, "x1"), a2;
  if (x2) a2 = act(*x2, "x2");
  Act d = act(dy, "dy");
  TORCH_CHECK(d.N == a1.N && d.H == a1.H && d.W == a1.W, "dy spatial mismatch");
  check_f32(slab, "slab");
  check_f32(out, "out");
  const int Cin = packed ? cin_real : a1.C + (x2 ? a2.C : 0);
  TORCH_CHECK(out.numel() == (long)d.C * taps * Cin, "wgrad out numel mismatch");
  // batch chunks below the 2 GiB buffer-offset reach (see conv_fwd), accumulated into out
  const long per_img = std::max(std::max((long)a1.H * a1.W * a1.pitch, x2 ? (long)a2.H * a2.W * a2.pitch : 0L),
                                (long)d.H * d.W * d.pitch) * 2;
  const int nc = chunk_images(per_img, a1.N);
  int r = 0;
  for (int n0 = 0; n0 < a1.N; n0 += nc) {
    const int nn = std::min(nc, a1.N - n0);
    auto img = [n0](const Act& t) { return (void*)((char*)t.ptr + (long)n0 * t.H * t.W * t.pitch * 2); };
    auto nbytes = [nn](const Act& t) { return ((long)nn * t.H * t.W - 1) * t.pitch * 2 + (long)t.C * 2; };
    void* const px1 = img(a1);
    void* const px2 = x2 ? img(a2) : nullptr;
    void* const pdy = img(d);
    const long bx1 = nbytes(a1), bx2 = x2 ? nbytes(a2) : 0, bdy = nbytes(d);
    const int C2 = x2 ? a2.C : 0, p2 = x2 ? a2.pitch : 0, acc = n0 > 0 ? 1 : accumulate;
    float* const slp = slab.data_ptr<float>();
    const long sln = slab.numel();
    float* const outp = out.data_ptr<float>();
    r = RDP_PLAN(rdp_conv_wgrad(px1, px2, bx1, bx2, a1.C, C2, a1.pitch, p2, pdy, bdy, d.pitch, slp, sln, outp, acc, nn,
                                a1.H, a1.W, d.C, taps, packed, cin_real, splits, variant, st));
    TORCH_CHECK(r >= 0, "conv_wgrad: unsupported shape or slab too small (code ", r, ")");
  }
  return r;
}

// First layer: BN-backward apply (+ ReLU mask) fused into the packed weight gradient (conv_wgrad.hip).
// x: the 8-channel packed input, da: dL/d(post-ReLU activation), y: pre-BN conv output, coef / coef2:
// the layer's BN coefficients (bn_finalize / bn_bwd_finalize). Returns the splits, or -1 when the
// shape does not fit the kernel (nothing launched: the caller runs bn_relu_bwd_apply + conv_wgrad).
int wgrad_first_bn(torch::Tensor x, torch::Tensor da, torch::Tensor y, torch::Tensor coef, torch::Tensor coef2,
                   torch::Tensor slab, torch::Tensor out, int cin_real, int accumulate, int splits) {
  Act a = act(x, "x"), d = act(da, "da"), b = act(y, "y");
  TORCH_CHECK(a.C == 8 && d.C == 64 && b.C == 64, "wgrad_first_bn: x must have 8 (packed) and da / y 64 channels");
  TORCH_CHECK(d.N == a.N && d.H == a.H && d.W == a.W && b.N == a.N && b.H == a.H && b.W == a.W,
              "wgrad_first_bn: spatial mismatch");
  check_f32(coef, "coef"); check_f32(coef2, "coef2"); check_f32(slab, "slab"); check_f32(out, "out");
  TORCH_CHECK(coef.numel() >= 4 * 64 && coef2.numel() >= 3 * 64, "wgrad_first_bn: coef / coef2 too small");
  TORCH_CHECK(out.numel() == 64l * 9 * cin_real, "wgrad_first_bn: out numel mismatch");
  if (a.bytes >= (1l << 31) || d.bytes >= (1l << 31) || b.bytes >= (1l << 31)) return -1;
  if (((long)a.N * a.H * a.W) % 64) return -1;
  const int r = RDP_PLAN(rdp_wgrad_first_bn(a.ptr, a.bytes, a.pitch, d.ptr, d.bytes, d.pitch, b.ptr, b.bytes, b.pitch,
                                            coef.data_ptr<float>(), coef2.data_ptr<float>(), slab.data_ptr<float>(),
                                            slab.numel(), out.data_ptr<float>(), accumulate, a.N, a.H, a.W, cin_real,
                                            splits, st));
  TORCH_CHECK(r > 0, "wgrad_first_bn: slab too small (code ", r, ")");
  return r;
}

long wgrad_slab_elems(int N, int H, int W, int Cin, int Cout, int taps, int packed, int splits) {
  return rdp_conv_wgrad_slab_elems(N, H, W, Cin, Cout, taps, packed, splits);
}

void bn_finalize(torch::Tensor stats, int T, long count, torch::Tensor gamma, torch::Tensor beta,
                 c10::optional<torch::Tensor> rmean, c10::optional<torch::Tensor> rvar,
                 c10::optional<torch::Tensor> nbt, double momentum, double eps, torch::Tensor coef,
                 c10::optional<torch::Tensor> ws) {
  const int C = gamma.numel();
  check_f32(stats, "stats"); check_f32(gamma, "gamma"); check_f32(beta, "beta"); check_f32(coef, "coef");
  TORCH_CHECK(stats.numel() >= (long)T * 2 * C && coef.numel() >= 4 * C, "bn_finalize sizes");
  float* rm = nullptr; float* rv = nullptr; long long* nb = nullptr;
  if (rmean) { check_f32(*rmean, "rmean"); rm = rmean->data_ptr<float>(); }
  if (rvar) { check_f32(*rvar, "rvar"); rv = rvar->data_ptr<float>(); }
  if (nbt) { TORCH_CHECK(nbt->scalar_type() == torch::kInt64 && nbt->is_cuda(), "nbt int64"); nb = (long long*)nbt->data_ptr(); }
  RDP_PLAN(rdp_bn_finalize(stats.data_ptr<float>(), T, C, count, gamma.data_ptr<float>(), beta.data_ptr<float>(), rm, rv, nb,
                  (float)momentum, (float)eps, coef.data_ptr<float>(), ws_ptr(ws, 2 * C), st));
}

void bn_eval_coef(torch::Tensor gamma, torch::Tensor beta, torch::Tensor rmean, torch::Tensor rvar, double eps,
                  torch::Tensor coef) {
  const int C = gamma.numel();
  check_f32(coef, "coef");
  RDP_PLAN(rdp_bn_eval_coef(C, gamma.data_ptr<float>(), beta.data_ptr<float>(), rmean.data_ptr<float>(), rvar.data_ptr<float>(),
                   (float)eps, coef.data_ptr<float>(), st));
}

void bn_relu_apply(torch::Tensor y, torch::Tensor out, torch::Tensor coef, int relu) {
  Act a = act(y, "y"), o = act(out, "out");
  TORCH_CHECK(a.N == o.N && a.H == o.H && a.W == o.W && a.C == o.C, "bn_relu_apply shape");
  TORCH_CHECK(coef.numel() >= 4 * a.C, "coef");
  TORCH_CHECK(RDP_PLAN(rdp_bn_relu_apply(a.ptr, a.pitch, o.ptr, o.pitch, coef.data_ptr<float>(), a.N * a.H * a.W, a.C, relu,
                                st)) == 0, "bn_relu_apply");
}

// 3x3 dgrad (row-ring kernel) whose epilogue also writes the BN-backward partial rows of the layer that
// owns dx (y_bn: its pre-BN output, coef: its [mean|invstd|scale|shift]; ReLU). Returns the partial
// rows for bn_bwd_finalize, or -1 if the ring kernel does not apply (caller falls back to
// conv_fwd + bn_relu_bwd_reduce; nothing was launched).
int conv_dgrad_bnred(torch::Tensor dy, torch::Tensor w, torch::Tensor dx, torch::Tensor y_bn, torch::Tensor coef,
                     torch::Tensor partial) {
  Act a = act(dy, "dy"), o = act(dx, "dx"), b = act(y_bn, "y_bn");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kBFloat16 && w.is_contiguous() && w.dim() == 2, "w: bf16 [Cout][K]");
  TORCH_CHECK(o.N == a.N && o.H == a.H && o.W == a.W && b.N == a.N && b.H == a.H && b.W == a.W && b.C == o.C,
              "conv_dgrad_bnred: shape mismatch");
  TORCH_CHECK(w.size(0) == o.C, "w rows != Cout");
  check_f32(coef, "coef");
  check_f32(partial, "partial");
  TORCH_CHECK(coef.numel() >= 4l * o.C, "coef must hold 4*C floats");
  // ring grid <= 256 blocks x 4 pixel groups (64 couts) or 2 (128): <= 1024 rows of 2*C
  TORCH_CHECK(partial.numel() >= 1024l * 2 * o.C, "partial too small");
  // batches past the 2 GiB buffer-offset reach: the caller's chunked conv_fwd + bn_relu_bwd_reduce
  const long per_img = std::max(std::max((long)a.H * a.W * a.pitch, (long)o.H * o.W * o.pitch), (long)b.H * b.W * b.pitch) * 2;
  if (chunk_images(per_img, a.N) < a.N) return -1;
  return RDP_PLAN(rdp_conv_ring_ex(a.ptr, a.bytes, a.C, a.pitch, w.data_ptr(), w.numel() * 2, w.size(1), o.ptr, o.bytes,
                          o.pitch, nullptr, 0, 0, o.C, o.C, partial.data_ptr<float>(), a.N, a.H, a.W, nullptr, nullptr,
                          0, 256, b.ptr, b.pitch, coef.data_ptr<float>(), nullptr, nullptr, nullptr, 0, 0, st));
}

// 3x3 dgrad into one BN + ReLU layer's activation gradient (dx, one destination) through the implicit-GEMM
// dispatch: where it runs split-K (small M x long K: the reference batch's deep layers), the split-K
// reduce also writes that layer's BN-backward partial rows (y_bn: its pre-BN output, coef: its
// [mean|invstd|scale|shift]) and this returns their count; 0 when the conv ran on another path (the
// caller runs bn_relu_bwd_reduce); -1 when nothing was launched (batches past the 2 GiB reach: the
// caller's chunked conv_fwd).
int conv_dgrad_splitk_bnred(torch::Tensor dy, torch::Tensor w, torch::Tensor dx, torch::Tensor y_bn,
                            torch::Tensor coef, torch::Tensor partial, c10::optional<torch::Tensor> ws) {
  Act a = act(dy, "dy"), o = act(dx, "dx"), b = act(y_bn, "y_bn");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kBFloat16 && w.is_contiguous() && w.dim() == 2, "w: bf16 [Cout][K]");
  TORCH_CHECK(o.N == a.N && o.H == a.H && o.W == a.W && b.N == a.N && b.H == a.H && b.W == a.W && b.C == o.C,
              "conv_dgrad_splitk_bnred: shape mismatch");
  TORCH_CHECK(w.size(0) == o.C && w.size(1) >= 9l * a.C, "conv_dgrad_splitk_bnred: w must be [Cout][9 * Cin]");
  check_f32(coef, "coef");
  check_f32(partial, "partial");
  TORCH_CHECK(coef.numel() >= 4l * o.C, "coef must hold 4*C floats");
  TORCH_CHECK(partial.numel() >= 512l * 2 * o.C, "partial too small");  // the split-K reduce: <= 512 rows
  if (ws) check_f32(*ws, "ws");
  const long per_img = std::max(std::max((long)a.H * a.W * a.pitch, (long)o.H * o.W * o.pitch), (long)b.H * b.W * b.pitch) * 2;
  if (chunk_images(per_img, a.N) < a.N) return -1;
  auto rows = std::make_shared<int>(0);
  void* const px = a.ptr;
  void* const py = o.ptr;
  void* const pyb = b.ptr;
  void* const wp = w.data_ptr();
  const long wb = w.numel() * 2, bx = a.bytes, by = o.bytes;
  const int ldw = (int)w.size(1), C1 = a.C, p1 = a.pitch, Co = o.C, op = o.pitch, ypb = b.pitch, N = a.N, H = a.H,
            W = a.W;
  const float* const cf = coef.data_ptr<float>();
  float* const pp = partial.data_ptr<float>();
  float* const wsp = ws ? ws->data_ptr<float>() : nullptr;
  const long wsn = ws ? (long)ws->numel() : 0L;
  const int r = RDP_PLAN(rdp_conv_igemm(px, nullptr, bx, 0, C1, 0, p1, 0, wp, wb, ldw, py, nullptr, by, 0, Co, op, 0,
                                        nullptr, N, H, W, Co, 9, 0, 0, nullptr, nullptr, 0, wsp, wsn, nullptr, 0,
                                        nullptr, nullptr, 0, 0, 0, 0, 0, pyb, ypb, cf, pp, rows.get(), st));
  TORCH_CHECK(r >= 0, "conv_dgrad_splitk_bnred: unsupported shape (Cin=", C1, ", Cout=", Co, ")");
  return *rows;
}

// Training forward of a 3x3 64 -> 64 conv whose input is the producer layer's PRE-BN output x_pre: the
// row-ring kernel applies the producer's BN + ReLU (in_coef: its [mean|invstd|scale|shift]) to the
// staged rows itself, so the activation is never written (conv_ring.hip BNIN). Writes y and this
// conv's BN statistic rows; returns the rows, or -1 when the ring kernel does not apply (nothing
// launched: the caller runs bn_relu_apply + conv_fwd). a_out (optional): the activation is also
// written there (bitwise what bn_relu_apply writes), for a plain weight-gradient pass.
int conv_fwd_bnin(torch::Tensor x_pre, torch::Tensor w, torch::Tensor y, torch::Tensor stats, torch::Tensor in_coef,
                  c10::optional<torch::Tensor> a_out) {
  Act a = act(x_pre, "x_pre"), o = act(y, "y");
  void* aptr = nullptr;
  long abytes = 0;
  int apitch = 0;
  if (a_out && a_out->defined()) {
    Act q = act(*a_out, "a_out");
    TORCH_CHECK(q.N == a.N && q.H == a.H && q.W == a.W && q.C == a.C, "conv_fwd_bnin: a_out shape");
    aptr = q.ptr; abytes = q.bytes; apitch = q.pitch;
  }
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kBFloat16 && w.is_contiguous() && w.dim() == 2, "w: bf16 [Cout][K]");
  TORCH_CHECK(o.N == a.N && o.H == a.H && o.W == a.W && w.size(0) == o.C, "conv_fwd_bnin: shape mismatch");
  check_f32(stats, "stats");
  check_f32(in_coef, "in_coef");
  TORCH_CHECK(in_coef.numel() >= 4l * a.C, "in_coef: [4 C] f32");
  // (the ring grid writes <= 256 blocks x 4 pixel-group rows of 2 * C)
  if (a.C != 64 || o.C != 64 || a.W % 64 || a.H % 2 || stats.numel() < 1024l * 2 * o.C) return -1;
  const long per_img = std::max((long)a.H * a.W * a.pitch, (long)o.H * o.W * o.pitch) * 2;
  if (chunk_images(per_img, a.N) < a.N) return -1;
  const float* c = in_coef.data_ptr<float>();
  return RDP_PLAN(rdp_conv_ring_ex(a.ptr, a.bytes, a.C, a.pitch, w.data_ptr(), w.numel() * 2, w.size(1), o.ptr, o.bytes,
                                   o.pitch, nullptr, 0, 0, o.C, o.C, stats.data_ptr<float>(), a.N, a.H, a.W, nullptr,
                                   nullptr, 0, 256, nullptr, 0, nullptr, c + 2 * a.C, c + 3 * a.C, aptr, abytes, apitch,
                                   st));
}

int bn_relu_bwd_reduce(torch::Tensor da, torch::Tensor y, torch::Tensor coef, int relu, torch::Tensor partial) {
  Act d = act(da, "da"), a = act(y, "y");
  TORCH_CHECK(d.N == a.N && d.H == a.H && d.W == a.W && d.C == a.C, "bn bwd shape");
  check_f32(partial, "partial");
  const int maxb = partial.numel() / (2 * a.C);
  const int T = RDP_PLAN(rdp_bn_relu_bwd_reduce(d.ptr, d.pitch, a.ptr, a.pitch, coef.data_ptr<float>(), a.N * a.H * a.W, a.C,
                                       relu, partial.data_ptr<float>(), maxb, st));
  TORCH_CHECK(T > 0, "bn_relu_bwd_reduce");
  return T;
}

void bn_bwd_finalize(torch::Tensor partial, int T, long count, torch::Tensor gamma, torch::Tensor coef,
                     c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta, torch::Tensor coef2,
                     c10::optional<torch::Tensor> ws) {
  const int C = gamma.numel();
  RDP_PLAN(rdp_bn_bwd_finalize(partial.data_ptr<float>(), T, C, count, gamma.data_ptr<float>(), coef.data_ptr<float>(),
                      dgamma ? dgamma->data_ptr<float>() : nullptr, dbeta ? dbeta->data_ptr<float>() : nullptr,
                      coef2.data_ptr<float>(), ws_ptr(ws, 2 * C), st));
}

void bn_relu_bwd_apply(torch::Tensor da, torch::Tensor y, torch::Tensor coef, torch::Tensor coef2, torch::Tensor dy,
                       int relu) {
  Act d = act(da, "da"), a = act(y, "y"), o = act(dy, "dy");
  TORCH_CHECK(o.N == a.N && o.H == a.H && o.W == a.W && o.C == a.C, "bn bwd apply shape");
  TORCH_CHECK(RDP_PLAN(rdp_bn_relu_bwd_apply(d.ptr, d.pitch, a.ptr, a.pitch, coef.data_ptr<float>(), coef2.data_ptr<float>(),
                                    o.ptr, o.pitch, a.N * a.H * a.W, a.C, relu, st)) == 0, "bn bwd apply");
}

void maxpool2_fwd(torch::Tensor x, torch::Tensor out) {
  Act a = act(x, "x"), o = act(out, "out");
  TORCH_CHECK(o.N == a.N && o.H == a.H / 2 && o.W == a.W / 2 && o.C == a.C, "maxpool shape");
  TORCH_CHECK(RDP_PLAN(rdp_maxpool2_fwd(a.ptr, a.pitch, o.ptr, o.pitch, a.N, a.H, a.W, a.C, st)) == 0, "maxpool");
}

void maxpool2_bwd(torch::Tensor dp, torch::Tensor x, c10::optional<torch::Tensor> dskip, torch::Tensor dx) {
  Act p = act(dp, "dp"), a = act(x, "x"), o = act(dx, "dx"), s;
  if (dskip) { s = act(*dskip, "dskip"); TORCH_CHECK(s.N == a.N && s.H == a.H && s.W == a.W && s.C == a.C, "dskip shape"); }
  TORCH_CHECK(p.N == a.N && p.H == a.H / 2 && p.W == a.W / 2 && p.C == a.C, "maxpool bwd shape");
  TORCH_CHECK(o.N == a.N && o.H == a.H && o.W == a.W && o.C == a.C, "maxpool bwd dx shape");
  TORCH_CHECK(RDP_PLAN(rdp_maxpool2_bwd(p.ptr, p.pitch, a.ptr, a.pitch, dskip ? s.ptr : nullptr, dskip ? s.pitch : 0, o.ptr,
                               o.pitch, a.N, a.H, a.W, a.C, st)) == 0, "maxpool bwd");
}

// training forward at a Down boundary: a = relu(bn(y)) (skip activation) and its 2x2 max pool, one pass
// out = None: only the pool is written (bf16-exact activation, as if a had been stored and re-read)
void bn_relu_apply_pool(torch::Tensor y, c10::optional<torch::Tensor> out, torch::Tensor pool, torch::Tensor coef) {
  Act a = act(y, "y"), o, p = act(pool, "pool");
  if (out) {
    o = act(*out, "out");
    TORCH_CHECK(a.N == o.N && a.H == o.H && a.W == o.W && a.C == o.C, "bn_relu_apply_pool shape");
  }
  TORCH_CHECK(p.N == a.N && p.H == a.H / 2 && p.W == a.W / 2 && p.C == a.C, "bn_relu_apply_pool pool shape");
  check_f32(coef, "coef");
  TORCH_CHECK(coef.numel() >= 4 * a.C, "coef");
  TORCH_CHECK(RDP_PLAN(rdp_bn_relu_apply_pool(a.ptr, a.pitch, out ? o.ptr : nullptr, out ? o.pitch : 0, p.ptr, p.pitch, coef.data_ptr<float>(), a.N, a.H,
                                     a.W, a.C, st)) == 0, "bn_relu_apply_pool: channels must be 2^k in [8, 2048]");
}

// maxpool backward (+ skip gradient) fused with the BN backward reduction of the pooled layer;
// returns the partial rows written (input T of bn_bwd_finalize)
int maxpool2_bwd_bn_reduce(torch::Tensor dp, torch::Tensor x, c10::optional<torch::Tensor> dskip, torch::Tensor dx,
                           torch::Tensor y, torch::Tensor coef, torch::Tensor partial) {
  Act p = act(dp, "dp"), a = act(x, "x"), o = act(dx, "dx"), yy = act(y, "y"), s;
  if (dskip) { s = act(*dskip, "dskip"); TORCH_CHECK(s.N == a.N && s.H == a.H && s.W == a.W && s.C == a.C, "dskip shape"); }
  TORCH_CHECK(p.N == a.N && p.H == a.H / 2 && p.W == a.W / 2 && p.C == a.C, "maxpool bwd shape");
  TORCH_CHECK(o.N == a.N && o.H == a.H && o.W == a.W && o.C == a.C, "maxpool bwd dx shape");
  TORCH_CHECK(yy.N == a.N && yy.H == a.H && yy.W == a.W && yy.C == a.C, "maxpool bwd y shape");
  check_f32(coef, "coef");
  check_f32(partial, "partial");
  TORCH_CHECK(coef.numel() >= 4 * a.C, "coef");
  const int maxb = partial.numel() / (2 * a.C);
  TORCH_CHECK(maxb >= 1, "partial too small");
  const int T = RDP_PLAN(rdp_maxpool2_bwd_bn_reduce(p.ptr, p.pitch, a.ptr, a.pitch, dskip ? s.ptr : nullptr, dskip ? s.pitch : 0,
                                           o.ptr, o.pitch, yy.ptr, yy.pitch, coef.data_ptr<float>(), a.N, a.H, a.W, a.C,
                                           partial.data_ptr<float>(), maxb, st));
  TORCH_CHECK(T > 0, "maxpool2_bwd_bn_reduce: channels must be 2^k in [8, 2048]");
  return T;
}

// coef (optional, fp32 [4C] = mean|invstd|scale|shift): x is pre-BN; BN + ReLU applied on the fly
void upsample2_fwd(torch::Tensor x, torch::Tensor out, int oy, int ox, c10::optional<torch::Tensor> coef) {
  Act a = act(x, "x"), o = act(out, "out");
  TORCH_CHECK(o.N == a.N && o.C == a.C, "upsample shape");
  TORCH_CHECK(2 * a.H + oy <= o.H && 2 * a.W + ox <= o.W && oy >= 0 && ox >= 0, "upsample fwd placement");
  const float* cp = nullptr;
  if (coef && coef->defined()) {
    TORCH_CHECK(coef->is_cuda() && coef->scalar_type() == torch::kFloat32 && coef->numel() >= 4 * a.C, "coef [4C] f32");
    cp = coef->data_ptr<float>();
  }
  TORCH_CHECK(RDP_PLAN(rdp_upsample2_fwd(a.ptr, a.pitch, o.ptr, o.pitch, a.N, a.H, a.W, o.H, o.W, oy, ox, a.C, cp,
                                st)) == 0,
              "upsample fwd: channels must be 2^k in [8, 2048], pitches multiples of 8");
}

// y/coef/partial (optional): also accumulate the training-BN backward reduction of dx's BN (dx = da of
// the layer whose pre-BN output is y); returns the partial row count (0 without the fusion)
int upsample2_bwd(torch::Tensor dout, torch::Tensor dx, int oy, int ox, c10::optional<torch::Tensor> y,
                  c10::optional<torch::Tensor> coef, c10::optional<torch::Tensor> partial) {
  Act d = act(dout, "dout"), o = act(dx, "dx"), yy;
  TORCH_CHECK(o.N == d.N && o.C == d.C, "upsample bwd shape");
  TORCH_CHECK(2 * o.H + oy <= d.H && 2 * o.W + ox <= d.W && oy >= 0 && ox >= 0, "upsample bwd placement");
  const float* cf = nullptr;
  float* pp = nullptr;
  int maxb = 0;
  if (y) {
    TORCH_CHECK(coef && partial, "upsample2_bwd: y needs coef and partial");
    yy = act(*y, "y");
    TORCH_CHECK(yy.N == o.N && yy.H == o.H && yy.W == o.W && yy.C == o.C, "upsample bwd y shape");
    check_f32(*coef, "coef");
    check_f32(*partial, "partial");
    TORCH_CHECK(coef->numel() >= 4 * o.C, "coef");
    maxb = std::min<long>(partial->numel() / (2 * o.C), 4096);
    TORCH_CHECK(maxb >= 1, "partial too small");
    cf = coef->data_ptr<float>();
    pp = partial->data_ptr<float>();
  }
  const int T = RDP_PLAN(rdp_upsample2_bwd(d.ptr, d.pitch, o.ptr, o.pitch, o.N, o.H, o.W, d.H, d.W, oy, ox, o.C,
                                  y ? yy.ptr : nullptr, y ? yy.pitch : 0, cf, pp, maxb, st));
  TORCH_CHECK(T >= 0, "upsample2_bwd: channels must be 2^k in [8, 2048], pitches multiples of 8");
  return T;
}

// ConvTranspose2d(2, s2): yT [N,h,w,4C] (+bias) -> u [N,H2,W2,C] at offset (oy, ox), zero elsewhere
void upT_shuffle(torch::Tensor yT, torch::Tensor bias, torch::Tensor u, int oy, int ox) {
  Act y = act(yT, "yT"), o = act(u, "u");
  check_f32(bias, "bias");
  TORCH_CHECK(y.N == o.N && y.C == 4 * o.C && bias.numel() == o.C, "upT_shuffle shapes");
  TORCH_CHECK(oy >= 0 && ox >= 0 && 2 * y.H + oy <= o.H && 2 * y.W + ox <= o.W, "upT_shuffle placement");
  TORCH_CHECK(RDP_PLAN(rdp_upT_shuffle(y.ptr, y.pitch, bias.data_ptr<float>(), o.ptr, o.pitch, y.N, y.H, y.W, o.H, o.W, oy, ox,
                              o.C, st)) == 0, "upT_shuffle");
}

// ConvTranspose2d(2, s2) + bias written straight into u at (oy, ox) by the ping-pong GEMM's epilogue
// (w = the [4C][Cin] forward weight). Returns 0, or -1 when that kernel does not take the shape: the
// caller then runs conv_fwd into yT + upT_shuffle. u's border outside the window is not written.
int conv_upT_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor bias, torch::Tensor u, int oy, int ox) {
  Act a = act(x, "x"), o = act(u, "u");
  check_f32(bias, "bias");
  TORCH_CHECK(w.scalar_type() == torch::kBFloat16 && w.is_contiguous() && w.dim() == 2 && w.size(0) == 4 * o.C &&
                  w.size(1) >= a.C, "conv_upT_fwd: w must be bf16 [4C][>= Cin]");
  TORCH_CHECK(a.N == o.N && bias.numel() == o.C, "conv_upT_fwd shapes");
  TORCH_CHECK(oy >= 0 && ox >= 0 && 2 * a.H + oy <= o.H && 2 * a.W + ox <= o.W, "conv_upT_fwd placement");
  const long xb = ((long)a.N * a.H * a.W - 1) * a.pitch * 2 + (long)a.C * 2;
  const long ub = ((long)o.N * o.H * o.W - 1) * o.pitch * 2 + (long)o.C * 2;
  return RDP_PLAN(rdp_conv_upT_fwd(a.ptr, xb, a.C, a.pitch, w.data_ptr(), w.numel() * 2, (int)w.size(1), o.ptr, ub,
                                   o.pitch, bias.data_ptr<float>(), a.N, a.H, a.W, o.H, o.W, oy, ox, o.C, st));
}

// ConvTranspose2d(2, s2) input gradient dx [N,h,w,Cin] read straight from du (its 4 sub-pixels per
// pixel; wd = the [Cin][4C] dgrad weight) on the ping-pong kernel. Returns 0, or -1 (nothing
// launched) where that kernel does not take the shape: the caller unshuffles and runs the GEMM.
int conv_upT_dgrad(torch::Tensor du, torch::Tensor wd, torch::Tensor dx, int oy, int ox) {
  Act d = act(du, "du"), o = act(dx, "dx");
  TORCH_CHECK(wd.scalar_type() == torch::kBFloat16 && wd.is_contiguous() && wd.dim() == 2 && wd.size(0) == o.C &&
                  wd.size(1) >= 4 * d.C, "conv_upT_dgrad: wd must be bf16 [Cin][>= 4C]");
  TORCH_CHECK(d.N == o.N && oy >= 0 && ox >= 0 && 2 * o.H + oy <= d.H && 2 * o.W + ox <= d.W, "conv_upT_dgrad placement");
  const long db = ((long)d.N * d.H * d.W - 1) * d.pitch * 2 + (long)d.C * 2;
  const long ob = ((long)o.N * o.H * o.W - 1) * o.pitch * 2 + (long)o.C * 2;
  return RDP_PLAN(rdp_conv_upT_dgrad(d.ptr, db, d.C, d.pitch, d.H, d.W, oy, ox, wd.data_ptr(), wd.numel() * 2,
                                     (int)wd.size(1), o.ptr, ob, o.C, o.pitch, o.N, o.H, o.W, st));
}

// ConvTranspose2d(2, s2) weight gradient out [Cin][4C] (+)= from du (4 sub-pixels per pixel of x) and
// its input x [N,h,w,Cin]. Returns the split count (< 0: shape not taken, nothing launched).
int conv_wgrad_upT(torch::Tensor du, torch::Tensor x, int oy, int ox, torch::Tensor slab, torch::Tensor out,
                   int accumulate, int splits) {
  Act d = act(du, "du"), a = act(x, "x");
  check_f32(slab, "slab");
  check_f32(out, "out");
  TORCH_CHECK(out.numel() == (long)a.C * 4 * d.C, "conv_wgrad_upT out numel");
  TORCH_CHECK(d.N == a.N && oy >= 0 && ox >= 0 && 2 * a.H + oy <= d.H && 2 * a.W + ox <= d.W, "conv_wgrad_upT placement");
  const long db = ((long)d.N * d.H * d.W - 1) * d.pitch * 2 + (long)d.C * 2;
  const long xb = ((long)a.N * a.H * a.W - 1) * a.pitch * 2 + (long)a.C * 2;
  return RDP_PLAN(rdp_conv_wgrad_upT(d.ptr, db, d.C, d.pitch, d.H, d.W, oy, ox, a.ptr, xb, a.C, a.pitch, a.N, a.H, a.W,
                                     slab.data_ptr<float>(), slab.numel(), out.data_ptr<float>(), accumulate, splits, st));
}

void upT_unshuffle(torch::Tensor du, torch::Tensor dyT, int oy, int ox) {
  Act d = act(du, "du"), y = act(dyT, "dyT");
  TORCH_CHECK(y.N == d.N && y.C == 4 * d.C, "upT_unshuffle shapes");
  TORCH_CHECK(oy >= 0 && ox >= 0 && 2 * y.H + oy <= d.H && 2 * y.W + ox <= d.W, "upT_unshuffle placement");
  TORCH_CHECK(RDP_PLAN(rdp_upT_unshuffle(d.ptr, d.pitch, y.ptr, y.pitch, y.N, y.H, y.W, d.H, d.W, oy, ox, d.C, st)) == 0,
              "upT_unshuffle");
}

// out[c] (+)= sum over pixels and the `groups` channel blocks of x [N,H,W,groups*C]
void colsum_bf16(torch::Tensor x, int groups, torch::Tensor partial, torch::Tensor out, int accumulate) {
  Act a = act(x, "x");
  check_f32(partial, "partial"); check_f32(out, "out");
  TORCH_CHECK(out.numel() * groups == a.C && partial.numel() >= 1024L * a.C + 64L * out.numel(), "colsum_bf16 sizes");
  TORCH_CHECK(RDP_PLAN(rdp_colsum_bf16(a.ptr, a.pitch, (long)a.N * a.H * a.W, a.C, groups, partial.data_ptr<float>(),
                              out.data_ptr<float>(), accumulate, st)) == 0,
              "colsum_bf16: channels must be a power of two in [8, 2048]");
}

int head_partial_blocks(long M) { return rdp_head_partial_blocks(M); }

// coef (training, optional): `a` is the last conv's pre-BN output y and coef its BN coefficients
// gpart + bnpart (with coef, dice_w == 0): the forward also emits the backward partials
// (gpart [nb][65] head grads, bnpart [nb][128] BN-backward rows; nb = head_partial_blocks(M))
void head_fwd(torch::Tensor a, torch::Tensor w, torch::Tensor b, torch::Tensor target, torch::Tensor logits,
              torch::Tensor partial, torch::Tensor sums, torch::Tensor loss, double dice_w, double dice_eps,
              c10::optional<torch::Tensor> coef, c10::optional<torch::Tensor> gpart,
              c10::optional<torch::Tensor> bnpart, double gscale) {
  Act x = act(a, "a");
  TORCH_CHECK(x.C == 64, "head expects 64 channels");
  const long M = (long)x.N * x.H * x.W;
  TORCH_CHECK(target.numel() == M && logits.numel() == M, "head target/logits numel");
  TORCH_CHECK(partial.numel() >= (long)rdp_head_partial_blocks(M) * 65, "head partial too small");
  const float* cf = nullptr;
  if (coef) {
    TORCH_CHECK(coef->numel() >= 4 * 64 && coef->scalar_type() == torch::kFloat, "head coef");
    cf = coef->data_ptr<float>();
  }
  float* gp = nullptr;
  float* bp = nullptr;
  if (gpart) {
    const long nb = rdp_head_partial_blocks(M);
    TORCH_CHECK(cf && bnpart && dice_w == 0.0, "head_fwd grad partials need coef, bnpart and dice_w == 0");
    check_f32(*gpart, "gpart");
    check_f32(*bnpart, "bnpart");
    TORCH_CHECK(gpart->numel() >= nb * 65 && bnpart->numel() >= nb * 128, "head_fwd grad partials too small");
    gp = gpart->data_ptr<float>();
    bp = bnpart->data_ptr<float>();
  }
  TORCH_CHECK(RDP_PLAN(rdp_head_fwd(x.ptr, x.pitch, w.data_ptr<float>(), b.data_ptr<float>(), target.data_ptr<float>(),
                           logits.data_ptr<float>(), partial.data_ptr<float>(), sums.data_ptr<float>(),
                           loss.data_ptr<float>(), M, (float)dice_w, (float)dice_eps, cf, gp, bp, (float)gscale,
                           st)) > 0, "head_fwd");
}

void head_grad_finalize(torch::Tensor gpart, long M, torch::Tensor gw, torch::Tensor gb) {
  check_f32(gpart, "gpart");
  TORCH_CHECK(gpart.numel() >= (long)rdp_head_partial_blocks(M) * 65 && gw.numel() == 64 && gb.numel() == 1,
              "head_grad_finalize sizes");
  RDP_PLAN(rdp_head_grad_finalize(gpart.data_ptr<float>(), (int)M, gw.data_ptr<float>(), gb.data_ptr<float>(), st));
}

// coef + bnpart given: BN-fused backward (da not written, returns the BN partial row count);
// otherwise da = d loss / d a is written. Returns the number of partial rows.
int head_bwd(torch::Tensor a, torch::Tensor w, torch::Tensor logits, torch::Tensor target, torch::Tensor sums,
             c10::optional<torch::Tensor> da, torch::Tensor partial, torch::Tensor gw, torch::Tensor gb, double dice_w,
             double dice_eps, double gscale, c10::optional<torch::Tensor> coef, c10::optional<torch::Tensor> bnpart) {
  Act x = act(a, "a");
  const long M = (long)x.N * x.H * x.W;
  TORCH_CHECK(x.C == 64, "head bwd channels");
  TORCH_CHECK(partial.numel() >= (long)rdp_head_partial_blocks(M) * 65, "head partial too small");
  void* dptr = nullptr;
  int dpitch = 0;
  const float* cf = nullptr;
  float* bp = nullptr;
  if (coef) {
    TORCH_CHECK(bnpart && bnpart->numel() >= (long)rdp_head_partial_blocks(M) * 128, "head bnpart too small");
    TORCH_CHECK(coef->numel() >= 4 * 64 && coef->scalar_type() == torch::kFloat, "head coef");
    cf = coef->data_ptr<float>();
    bp = bnpart->data_ptr<float>();
  } else {
    TORCH_CHECK(da.has_value(), "head_bwd: da required without coef");
    Act d = act(*da, "da");
    TORCH_CHECK(d.C == 64 && (long)d.N * d.H * d.W == M, "head bwd da shape");
    dptr = d.ptr;
    dpitch = d.pitch;
  }
  return RDP_PLAN(rdp_head_bwd(x.ptr, x.pitch, w.data_ptr<float>(), logits.data_ptr<float>(), target.data_ptr<float>(),
                      sums.data_ptr<float>(), dptr, dpitch, partial.data_ptr<float>(), gw.data_ptr<float>(),
                      gb.data_ptr<float>(), M, (float)dice_w, (float)dice_eps, (float)gscale, cf, bp, st));
}

// dy of the last conv from the logits (BN-fused head backward, second pass)
void head_bn_bwd_apply(torch::Tensor y, torch::Tensor w, torch::Tensor logits, torch::Tensor target,
                       torch::Tensor sums, torch::Tensor coef, torch::Tensor coef2, torch::Tensor dy, double dice_w,
                       double dice_eps, double gscale) {
  Act x = act(y, "y"), d = act(dy, "dy");
  const long M = (long)x.N * x.H * x.W;
  TORCH_CHECK(x.C == 64 && d.C == 64 && (long)d.N * d.H * d.W == M, "head_bn_bwd_apply shapes");
  TORCH_CHECK(logits.numel() == M && target.numel() == M, "head_bn_bwd_apply logits/target numel");
  TORCH_CHECK(coef.numel() >= 4 * 64 && coef2.numel() >= 3 * 64, "head_bn_bwd_apply coef sizes");
  TORCH_CHECK(RDP_PLAN(rdp_head_bn_bwd_apply(x.ptr, x.pitch, w.data_ptr<float>(), logits.data_ptr<float>(),
                                    target.data_ptr<float>(), sums.data_ptr<float>(), coef.data_ptr<float>(),
                                    coef2.data_ptr<float>(), d.ptr, d.pitch, M, (float)dice_w, (float)dice_eps,
                                    (float)gscale, st)) == 0,
              "head_bn_bwd_apply: pitches must be multiples of 8");
}

// eval conv (64 -> 64, BN fold + ReLU) + serving 1x1 head + (logit > thr) in one kernel (row ring);
// returns false (nothing launched) where that kernel does not apply
bool conv_head_mask(torch::Tensor x, torch::Tensor w, torch::Tensor coef, torch::Tensor hw, torch::Tensor hb,
                    double thr, torch::Tensor mask) {
  Act a = act(x, "x");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kBFloat16 && w.is_contiguous() && w.dim() == 2, "w: bf16 [Cout][K]");
  check_f32(coef, "coef");
  check_f32(hw, "head_w");
  check_f32(hb, "head_b");
  TORCH_CHECK(coef.numel() >= 4l * w.size(0) && hw.numel() == w.size(0) && hb.numel() >= 1, "coef / head sizes");
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == torch::kUInt8 && mask.is_contiguous() &&
              mask.numel() >= (long)a.N * a.H * a.W, "mask: u8 [N*H*W]");
  const int Co = (int)w.size(0);
  const int r = RDP_PLAN(rdp_conv_ring_head(a.ptr, a.bytes, a.C, a.pitch, w.data_ptr(), w.numel() * 2, w.size(1), Co, a.N, a.H,
                                   a.W, coef.data_ptr<float>() + 2 * Co, coef.data_ptr<float>() + 3 * Co,
                                   hw.data_ptr<float>(), hb.data_ptr<float>(), (float)thr, mask.data_ptr(),
                                   st));
  return r == 0;
}

// Row-band eval conv called directly (csrc/conv_rowband.hip), with OHWI weights (wfrag = 0) or their
// fragment-major copy (wfrag = 1: [Cout/16][9 Cin/32][64 lanes][8], rowband_frag_weights in Python).
// Returns 1 when the pool was written, 0 when not, < 0 when the kernel does not take the shape.
int conv_rowband(torch::Tensor x1, c10::optional<torch::Tensor> x2, torch::Tensor w, torch::Tensor y,
                 torch::Tensor coef, c10::optional<torch::Tensor> pool, int wfrag) {
  Act a1 = act(x1, "x1"), a2;
  if (x2) a2 = act(*x2, "x2");
  Act o = act(y, "y");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kBFloat16 && w.is_contiguous(), "w: bf16 contiguous");
  check_f32(coef, "coef");
  TORCH_CHECK(coef.numel() >= 4l * o.C, "coef size");
  Act po;
  if (pool) po = act(*pool, "pool");
  const int ldw = wfrag ? 0 : (int)w.size(1);
  void* const px2 = x2 ? a2.ptr : nullptr;
  const long bx2 = x2 ? a2.bytes : 0;
  const int C2 = x2 ? a2.C : 0, p2 = x2 ? a2.pitch : 0;
  void* const pp = pool ? po.ptr : nullptr;
  const long pb = pool ? po.bytes : 0;
  const int ppit = pool ? po.pitch : 0;
  const float* sc = coef.data_ptr<float>() + 2 * o.C;
  const float* sh = coef.data_ptr<float>() + 3 * o.C;
  void* const wp = w.data_ptr();
  const long wb = w.numel() * 2;
  return (int)RDP_PLAN(rdp_conv_rowband_ex(a1.ptr, px2, a1.bytes, bx2, a1.C, C2, a1.pitch, p2, wp, wb, ldw, o.ptr, o.bytes,
                                           o.pitch, a1.N, a1.H, a1.W, o.C, sc, sh, 1, pp, pb, ppit, wfrag, st));
}

// Persistent row-band chain (csrc/conv_rowband.hip): layer 0 reads x, layer l > 0 layer l - 1's output;
// eval BN fold + ReLU per layer (coef = [mean|invstd|scale|shift]). cnt: int32 >= 1 + nl * N * H, err: int32.
bool conv_rowband_chain(torch::Tensor x, std::vector<torch::Tensor> ws, std::vector<torch::Tensor> ys,
                        std::vector<torch::Tensor> coefs, torch::Tensor cnt, torch::Tensor err) {
  const int nl = (int)ws.size();
  TORCH_CHECK(nl >= 1 && nl <= 4 && (int)ys.size() == nl && (int)coefs.size() == nl, "1..4 layers");
  Act a = act(x, "x");
  TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == torch::kInt32 && cnt.numel() >= 1 + (long)nl * a.N * a.H, "cnt");
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == torch::kInt32 && err.numel() >= 1, "err");
  std::array<const void*, 4> wp{};
  std::array<void*, 4> yp{};
  std::array<long, 4> wb{}, yb{};
  std::array<int, 4> ldw{}, ypit{}, co{};
  std::array<const float*, 4> sc{}, sh{};
  for (int l = 0; l < nl; ++l) {
    TORCH_CHECK(ws[l].is_cuda() && ws[l].scalar_type() == torch::kBFloat16 && ws[l].is_contiguous() && ws[l].dim() == 2,
                "w: bf16 [Cout][K]");
    Act o = act(ys[l], "y");
    TORCH_CHECK(o.N == a.N && o.H == a.H && o.W == a.W && o.C == ws[l].size(0), "y shape");
    check_f32(coefs[l], "coef");
    TORCH_CHECK(coefs[l].numel() >= 4l * o.C, "coef size");
    wp[l] = ws[l].data_ptr(); wb[l] = ws[l].numel() * 2; ldw[l] = (int)ws[l].size(1);
    yp[l] = o.ptr; yb[l] = o.bytes; ypit[l] = o.pitch; co[l] = o.C;
    sc[l] = coefs[l].data_ptr<float>() + 2 * o.C; sh[l] = coefs[l].data_ptr<float>() + 3 * o.C;
  }
  int* const cp = cnt.data_ptr<int>();
  int* const ep = err.data_ptr<int>();
  const int r = RDP_PLAN(rdp_conv_rowband_chain(nl, a.ptr, a.bytes, a.C, a.pitch, wp.data(), wb.data(), ldw.data(),
                                                yp.data(), yb.data(), ypit.data(), co.data(), sc.data(), sh.data(),
                                                a.N, a.H, a.W, cp, ep, st));
  return r == 0;
}

void head_mask(torch::Tensor a, torch::Tensor w, torch::Tensor b, double logit_thr, torch::Tensor mask) {
  Act x = act(a, "a");
  TORCH_CHECK(mask.scalar_type() == torch::kUInt8 && mask.numel() == (long)x.N * x.H * x.W, "mask u8 numel");
  RDP_PLAN(rdp_head_mask(x.ptr, x.pitch, w.data_ptr<float>(), b.data_ptr<float>(), (float)logit_thr, mask.data_ptr(),
                x.N * x.H * x.W, st));
}

void adam(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> shadow,
          double lr, double b1, double b2, double eps, double wd, double gscale, torch::Tensor step, bool inc,
          int max_blocks) {
  check_f32(p, "p"); check_f32(m, "m"); check_f32(v, "v");
  const bool gbf = g.scalar_type() == torch::kBFloat16;  // bf16 gradients (the DDP bf16 all-reduce buffer)
  if (!gbf) check_f32(g, "g");
  TORCH_CHECK(g.is_cuda() && g.is_contiguous(), "g: contiguous device tensor");
  TORCH_CHECK(g.numel() == p.numel() && m.numel() == p.numel() && v.numel() == p.numel(), "adam numel");
  TORCH_CHECK(step.scalar_type() == torch::kInt32 && step.is_cuda(), "step int32");
  void* sh = nullptr;
  if (shadow) {
    TORCH_CHECK(shadow->scalar_type() == torch::kBFloat16 && shadow->numel() == p.numel(), "shadow");
    sh = shadow->data_ptr();
  }
  const void* gp = g.data_ptr();
  TORCH_CHECK(RDP_PLAN(rdp_adam(p.data_ptr<float>(), gp, gbf ? 1 : 0, m.data_ptr<float>(), v.data_ptr<float>(), sh, p.numel(),
                       (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)gscale,
                       (int*)step.data_ptr(), inc ? 1 : 0, max_blocks, st)) == 0, "adam: numel must be a multiple of 4");
}

void cast_bf16(torch::Tensor p, torch::Tensor out) {
  check_f32(p, "p");
  TORCH_CHECK(out.scalar_type() == torch::kBFloat16 && out.numel() == p.numel(), "cast out");
  RDP_PLAN(rdp_cast_bf16(p.data_ptr<float>(), out.data_ptr(), p.numel(), st));
}

// The serving runtime's frame upload kernel (csrc/serve_kernels.hip), for tests: a pinned CPU tensor ->
// a device tensor of the same byte size through the host buffer's device mapping. Returns 0, or -1 when
// the kernel does not take the pair (unaligned) or the buffer has no mapping.
int h2d_copy(torch::Tensor src, torch::Tensor dst) {
  TORCH_CHECK(!src.is_cuda() && src.is_pinned() && src.is_contiguous(), "h2d_copy: src must be a pinned CPU tensor");
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "h2d_copy: dst must be a contiguous device tensor");
  const long bytes = (long)(src.numel() * src.element_size());
  TORCH_CHECK(bytes == (long)(dst.numel() * dst.element_size()), "h2d_copy: byte sizes differ");
  void* dp = nullptr;
  if (hipHostGetDevicePointer(&dp, src.data_ptr(), 0) != hipSuccess || !dp) {
    (void)hipGetLastError();
    return -1;
  }
  return rdp_h2d_copy(dp, dst.data_ptr(), bytes, c10::hip::getCurrentHIPStream().stream());
}

void wprep(torch::Tensor master, torch::Tensor out, torch::Tensor segs, int nseg, c10::optional<torch::Tensor> step,
           int blocks) {
  check_f32(master, "master");
  TORCH_CHECK(out.scalar_type() == torch::kBFloat16, "wprep out bf16");
  TORCH_CHECK(segs.is_cuda() && segs.numel() * segs.element_size() >= (long)nseg * rdp_wseg_size(), "segs");
  int* sp = nullptr;
  if (step) {
    TORCH_CHECK(step->scalar_type() == torch::kInt32 && step->is_cuda(), "step int32");
    sp = (int*)step->data_ptr();
  }
  RDP_PLAN(rdp_wprep(master.data_ptr<float>(), out.data_ptr(), segs.data_ptr(), nseg, sp, blocks, 0, st));
}

void check_cpu_f64(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.device().is_cpu() && t.scalar_type() == torch::kFloat64 && t.is_contiguous(), name,
              ": must be a contiguous float64 CPU tensor");
}

// FITPACK parcur: returns (ier, t[n], c[idim][n-k-1], fp)
py::tuple parcur(torch::Tensor u, torch::Tensor x, double s, int k) {
  check_cpu_f64(u, "u"); check_cpu_f64(x, "x");
  const int m = u.numel(), idim = x.size(1);
  TORCH_CHECK(x.size(0) == m, "x rows != len(u)");
  const int nest = m + 2 * k;
  auto t = torch::zeros({nest}, torch::kFloat64), c = torch::zeros({idim, nest}, torch::kFloat64);
  int n = 0;
  double fp = 0;
  int ier;
  {
    py::gil_scoped_release nogil;
    ier = rdp_parcur(idim, m, u.data_ptr<double>(), x.data_ptr<double>(), s, k, nest, t.data_ptr<double>(),
                     c.data_ptr<double>(), &n, &fp);
  }
  if (ier == 10) return py::make_tuple(ier, torch::Tensor(), torch::Tensor(), fp);
  return py::make_tuple(ier, t.narrow(0, 0, n).clone(), c.narrow(1, 0, n - k - 1).clone(), fp);
}

torch::Tensor splev(torch::Tensor t, torch::Tensor c, int k, torch::Tensor x, int der) {
  check_cpu_f64(t, "t"); check_cpu_f64(x, "x");
  auto cc = c.contiguous().to(torch::kFloat64);
  auto out = torch::empty_like(x);
  for (long i = 0; i < x.numel(); ++i)
    out.data_ptr<double>()[i] = rdp_splev1(t.data_ptr<double>(), t.numel(), cc.data_ptr<double>(), k,
                                           x.data_ptr<double>()[i], der);
  return out;
}

// sorted edge points [m,3] -> (ier, mean_k, max_k, spline points [nsamp,3], fp, n)
py::tuple fit_curvature(torch::Tensor pts, double s, int k, int nsamp, double eps) {
  check_cpu_f64(pts, "pts");
  auto out_pts = torch::zeros({nsamp, 3}, torch::kFloat64);
  double out[4] = {0, 0, 0, 0};
  int ier;
  {
    py::gil_scoped_release nogil;
    ier = rdp_fit_curvature(pts.data_ptr<double>(), pts.size(0), s, k, nsamp, eps, out_pts.data_ptr<double>(), out);
  }
  return py::make_tuple(ier, out[0], out[1], out_pts, out[2], (int)out[3]);
}

// geometry: mask u8 [H,W], depth u16-as-int16 [H,W] (GPU) -> packed edge points; returns E via hdr (device)
// m256 (serving form): mask is an OUTPUT (nearest upsample of the model mask) and cov[nblk] gets the
// per-row-block coverage counts; edges None: no packed edge list (hdr untouched)
void geo_edges(torch::Tensor mask, torch::Tensor depth, double fx, double fy, double cx, double cy, double scale,
               torch::Tensor work_i, torch::Tensor work_d, torch::Tensor pts, torch::Tensor npts, torch::Tensor out,
               torch::Tensor kout, int nbins, double top, int min_points, c10::optional<torch::Tensor> edges,
               c10::optional<torch::Tensor> hdr, c10::optional<torch::Tensor> m256, c10::optional<torch::Tensor> cov,
               c10::optional<torch::Tensor> sorted, c10::optional<torch::Tensor> gperm,
               c10::optional<torch::Tensor> mask_host) {
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == torch::kUInt8 && mask.dim() == 2 && mask.is_contiguous(), "mask");
  void* mhost = nullptr;
  if (mask_host && mask_host->defined()) {  // pinned / mapped host memory the kernel writes directly
    TORCH_CHECK(!mask_host->is_cuda() && mask_host->scalar_type() == torch::kUInt8 && mask_host->is_contiguous() &&
                    mask_host->numel() == mask.numel(), "mask_host: host u8 tensor of the mask's size");
    TORCH_CHECK(m256 && m256->defined(), "mask_host needs the serving form (m256)");
    mhost = mask_host->data_ptr();
  }
  TORCH_CHECK(depth.is_cuda() && depth.element_size() == 2 && depth.sizes() == mask.sizes() && depth.is_contiguous(),
              "depth u16");
  const int H = mask.size(0), W = mask.size(1);
  const int nblk = rdp_geo_nblocks(H);
  TORCH_CHECK(work_i.numel() >= rdp_geo_work_ints(H, W) && work_i.scalar_type() == torch::kInt32 &&
              work_i.is_contiguous(), "work_i: needs geo_work_ints(H, W) int32");
  TORCH_CHECK(work_d.numel() >= 2 * nblk && work_d.scalar_type() == torch::kFloat64, "work_d");
  TORCH_CHECK(pts.scalar_type() == torch::kFloat64 && pts.numel() >= (long)H * W * 4, "pts cap");
  TORCH_CHECK(out.scalar_type() == torch::kFloat64 && out.dim() == 3 && out.size(0) >= nbins && out.size(2) == 4, "out");
  const bool pack = edges && edges->defined();
  if (pack) {
    TORCH_CHECK(edges->scalar_type() == torch::kFloat64 && edges->dim() == 2 && edges->size(1) == 4, "edges");
    TORCH_CHECK(hdr && hdr->defined() && hdr->scalar_type() == torch::kInt32, "hdr int32");
  }
  const void* mp = nullptr;
  int mh = 0, mw = 0;
  int* covp = nullptr;
  if (m256 && m256->defined()) {
    TORCH_CHECK(m256->is_cuda() && m256->scalar_type() == torch::kUInt8 && m256->dim() == 2 && m256->is_contiguous(),
                "m256 u8 2-D");
    TORCH_CHECK(cov && cov->defined() && cov->scalar_type() == torch::kInt32 && cov->numel() >= nblk,
                "cov: geo_nblocks(H) int32");
    mp = m256->data_ptr();
    mh = m256->size(0);
    mw = m256->size(1);
    covp = cov->data_ptr<int>();
  }
  // sorted (+ gperm): the x-sorted edge points for geo_spline(presorted=True), fused into the select
  double* sp = nullptr;
  int* gp = nullptr;
  int secap = 0;
  if (sorted && sorted->defined()) {
    TORCH_CHECK(sorted->is_cuda() && sorted->scalar_type() == torch::kFloat64 && sorted->dim() == 2 &&
                sorted->size(1) == 3 && sorted->is_contiguous(), "sorted [ecap][3] f64");
    secap = sorted->size(0);
    TORCH_CHECK(gperm && gperm->defined() && gperm->scalar_type() == torch::kInt32 && gperm->numel() >= 2L * secap,
                "gperm: 2*ecap int32");
    sp = sorted->data_ptr<double>();
    gp = gperm->data_ptr<int>();
  }
  const int r = rdp_geo_edges(mask.data_ptr(), depth.data_ptr(), H, W, fx, fy, cx, cy, scale, work_i.data_ptr<int>(),
                              work_d.data_ptr<double>(), work_d.data_ptr<double>() + nblk, pts.data_ptr<double>(), H * W,
                              npts.data_ptr<int>(), out.data_ptr<double>(), out.size(1), kout.data_ptr<int>(), nbins,
                              top, min_points, pack ? edges->data_ptr<double>() : nullptr, pack ? edges->size(0) : 0,
                              pack ? hdr->data_ptr<int>() : nullptr, mp, mh, mw, covp, sp, gp, secap, mhost,
                              unplanned_stream());
  TORCH_CHECK(r >= 0, "geo_edges: nbins must be in [1, 128]");
}

int geo_nblocks(int H) { return rdp_geo_nblocks(H); }
long geo_work_ints(int H, int W) { return rdp_geo_work_ints(H, W); }

// The serving geometry of n <= 4 frames of one camera (BatchEngine): the edge stage (mask upsample +
// coverage, deprojection, bins, per-bin top-k + x-sort) and the spline fit, each ONE launch over the frames
// (csrc/geometry.hip rdp_geo_edges_batch, csrc/geo_spline.hip rdp_geo_spline_batch). Per-frame lists of
// the buffers GeometryEngine.launch_frame / launch_spline pass; the results (and the mask copies) go to
// host memory (res / mask_host).
void geo_frames_batch(std::vector<torch::Tensor> mask, std::vector<torch::Tensor> depth,
                      std::vector<torch::Tensor> m256, std::vector<torch::Tensor> work_i,
                      std::vector<torch::Tensor> work_d, std::vector<torch::Tensor> pts,
                      std::vector<torch::Tensor> npts, std::vector<torch::Tensor> out, std::vector<torch::Tensor> kout,
                      std::vector<torch::Tensor> cov, std::vector<torch::Tensor> sorted,
                      std::vector<torch::Tensor> gperm, std::vector<torch::Tensor> u, std::vector<torch::Tensor> res,
                      std::vector<torch::Tensor> mask_host, double fx, double fy, double cx, double cy, double scale,
                      int nbins, double top, int min_points, double smooth, int k, int nsamp, double eps,
                      int min_edge) {
  const int n = (int)mask.size();
  TORCH_CHECK(n >= 1 && n <= 4, "geo_frames_batch: 1..4 frames");
  for (auto* v : {&depth, &m256, &work_i, &work_d, &pts, &npts, &out, &kout, &cov, &sorted, &gperm, &u, &res})
    TORCH_CHECK((int)v->size() == n, "geo_frames_batch: every list needs one tensor per frame");
  TORCH_CHECK(mask_host.empty() || (int)mask_host.size() == n, "geo_frames_batch: mask_host: none or one per frame");
  const int H = mask[0].size(0), W = mask[0].size(1);
  const int nblk = rdp_geo_nblocks(H);
  const int mh = m256[0].size(0), mw = m256[0].size(1);
  const int cap = H * W, kcap = out[0].size(1), secap = sorted[0].size(0);
  std::vector<const void*> pm(n), pd(n), pm256(n);
  std::vector<int*> pcnt(n), pnpts(n), pkout(n), pcov(n), pgp(n);
  std::vector<double*> pxmin(n), pxmax(n), ppts(n), pout(n), psort(n), pu(n), pres(n);
  std::vector<void*> pmh(n);
  std::vector<const int*> ckout(n), cnpts(n), ccov(n);
  std::vector<const void*> cmask(n);
  for (int i = 0; i < n; ++i) {
    TORCH_CHECK(mask[i].is_cuda() && mask[i].scalar_type() == torch::kUInt8 && mask[i].dim() == 2 &&
                    mask[i].is_contiguous() && mask[i].size(0) == H && mask[i].size(1) == W, "mask: u8 HxW, one camera");
    TORCH_CHECK(depth[i].is_cuda() && depth[i].element_size() == 2 && depth[i].sizes() == mask[i].sizes() &&
                    depth[i].is_contiguous(), "depth u16 HxW");
    TORCH_CHECK(m256[i].is_cuda() && m256[i].scalar_type() == torch::kUInt8 && m256[i].dim() == 2 &&
                    m256[i].is_contiguous() && m256[i].size(0) == mh && m256[i].size(1) == mw, "m256 u8 2-D");
    TORCH_CHECK(work_i[i].numel() >= rdp_geo_work_ints(H, W) && work_i[i].scalar_type() == torch::kInt32, "work_i");
    TORCH_CHECK(work_d[i].numel() >= 2 * nblk && work_d[i].scalar_type() == torch::kFloat64, "work_d");
    TORCH_CHECK(pts[i].scalar_type() == torch::kFloat64 && pts[i].numel() >= (long)H * W * 4, "pts cap");
    TORCH_CHECK(out[i].scalar_type() == torch::kFloat64 && out[i].dim() == 3 && out[i].size(0) >= nbins &&
                    out[i].size(1) == kcap && out[i].size(2) == 4 && out[i].is_contiguous(), "out");
    TORCH_CHECK(kout[i].scalar_type() == torch::kInt32 && kout[i].numel() >= nbins, "kout");
    TORCH_CHECK(npts[i].scalar_type() == torch::kInt32, "npts");
    TORCH_CHECK(cov[i].scalar_type() == torch::kInt32 && cov[i].numel() >= nblk, "cov");
    TORCH_CHECK(sorted[i].scalar_type() == torch::kFloat64 && sorted[i].dim() == 2 && sorted[i].size(1) == 3 &&
                    sorted[i].size(0) == secap, "sorted");
    TORCH_CHECK(gperm[i].scalar_type() == torch::kInt32 && gperm[i].numel() >= 2L * secap, "gperm");
    TORCH_CHECK(u[i].scalar_type() == torch::kFloat64 && u[i].numel() >= secap, "u");
    TORCH_CHECK(res[i].scalar_type() == torch::kFloat64 && res[i].numel() >= rdp_geo_spline_res_len(nsamp) &&
                    res[i].is_contiguous(), "res");
    pm[i] = mask[i].data_ptr(); pd[i] = depth[i].data_ptr(); pm256[i] = m256[i].data_ptr();
    pcnt[i] = work_i[i].data_ptr<int>();
    pxmin[i] = work_d[i].data_ptr<double>(); pxmax[i] = pxmin[i] + nblk;
    ppts[i] = pts[i].data_ptr<double>(); pnpts[i] = npts[i].data_ptr<int>(); pout[i] = out[i].data_ptr<double>();
    pkout[i] = kout[i].data_ptr<int>(); pcov[i] = cov[i].data_ptr<int>(); psort[i] = sorted[i].data_ptr<double>();
    pgp[i] = gperm[i].data_ptr<int>(); pu[i] = u[i].data_ptr<double>(); pres[i] = res[i].data_ptr<double>();
    ckout[i] = pkout[i]; cnpts[i] = pnpts[i]; ccov[i] = pcov[i]; cmask[i] = pm[i];
    if (!mask_host.empty()) {
      TORCH_CHECK(!mask_host[i].is_cuda() && mask_host[i].scalar_type() == torch::kUInt8 &&
                      mask_host[i].is_contiguous() && mask_host[i].numel() == mask[i].numel(), "mask_host");
      pmh[i] = mask_host[i].data_ptr();
    }
  }
  const hipStream_t st = unplanned_stream();
  TORCH_CHECK(rdp_geo_edges_batch(n, pm.data(), pd.data(), H, W, fx, fy, cx, cy, scale, pcnt.data(), pxmin.data(),
                                  pxmax.data(), ppts.data(), cap, pnpts.data(), pout.data(), kcap, pkout.data(), nbins,
                                  top, min_points, pm256.data(), mh, mw, pcov.data(), psort.data(), pgp.data(), secap,
                                  nullptr, st) >= 0, "geo_frames_batch: nbins must be in [1, 128]");
  const int r = rdp_geo_spline_batch(n, nbins, kcap, ckout.data(), cnpts.data(), psort.data(), pu.data(), secap,
                                     smooth, k, nsamp, eps, min_points, min_edge, ccov.data(), nblk, pres.data(),
                                     cmask.data(), mask_host.empty() ? nullptr : pmh.data(),
                                     (long)H * W, st);
  TORCH_CHECK(r != -2, "geo_frames_batch: mask copy needs 4-byte aligned buffers and a size multiple of 4");
  TORCH_CHECK(r == 0, "geo_frames_batch: k must be in [1, 5], nsamp in [1, 256]");
}

// on-device spline stage: per-bin sort of the edge points (out/kout from geo_edges) + FITPACK-equivalent
// fit + nsamp-point evaluation and curvature into res (rdp_geo_spline_res_len(nsamp) doubles)
void geo_spline(torch::Tensor out, torch::Tensor kout, torch::Tensor npts, torch::Tensor sorted, torch::Tensor gperm,
                torch::Tensor u, torch::Tensor res, double s, int k, int nsamp, double eps, int min_points,
                int min_edge, c10::optional<torch::Tensor> cov, c10::optional<torch::Tensor> dbg, bool presorted,
                c10::optional<torch::Tensor> mask, c10::optional<torch::Tensor> mask_host) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kFloat64 && out.dim() == 3 && out.size(2) == 4 &&
              out.is_contiguous(), "out [nbins][kcap][4] f64");
  TORCH_CHECK(kout.scalar_type() == torch::kInt32 && kout.numel() >= out.size(0), "kout");
  TORCH_CHECK(npts.scalar_type() == torch::kInt32, "npts int32");
  TORCH_CHECK(sorted.scalar_type() == torch::kFloat64 && sorted.dim() == 2 && sorted.size(1) == 3 &&
              sorted.is_contiguous(), "sorted [ecap][3] f64");
  const int ecap = sorted.size(0);
  TORCH_CHECK(gperm.scalar_type() == torch::kInt32 && gperm.numel() >= 2L * ecap, "gperm: 2*ecap int32");
  TORCH_CHECK(u.scalar_type() == torch::kFloat64 && u.numel() >= ecap, "u: ecap f64");
  TORCH_CHECK(res.scalar_type() == torch::kFloat64 && res.numel() >= rdp_geo_spline_res_len(nsamp), "res");
  const int* covp = nullptr;
  int ncov = 0;
  if (cov && cov->defined()) {
    TORCH_CHECK(cov->scalar_type() == torch::kInt32, "cov int32");
    covp = cov->data_ptr<int>();
    ncov = cov->numel();
  }
  double* dbgp = nullptr;  // optional phase profile (20 doubles, see geo_fit_kernel)
  if (dbg && dbg->defined()) {
    TORCH_CHECK(dbg->is_cuda() && dbg->scalar_type() == torch::kFloat64 && dbg->numel() >= 20, "dbg: >= 20 f64");
    dbgp = dbg->data_ptr<double>();
  }
  // mask + mask_host (serving): the frame mask's host copy, written by blocks beside the fit block
  const void* mp = nullptr;
  void* mh = nullptr;
  long mbytes = 0;
  if (mask_host && mask_host->defined()) {
    TORCH_CHECK(mask && mask->defined() && mask->is_cuda() && mask->scalar_type() == torch::kUInt8 &&
                    mask->is_contiguous(), "geo_spline: mask_host needs the device mask (u8, contiguous)");
    TORCH_CHECK(!mask_host->is_cuda() && mask_host->scalar_type() == torch::kUInt8 && mask_host->is_contiguous() &&
                    mask_host->numel() == mask->numel(), "geo_spline: mask_host: host u8 tensor of the mask's size");
    mp = mask->data_ptr();
    mh = mask_host->data_ptr();
    mbytes = mask->numel();
  }
  const int r = rdp_geo_spline(out.data_ptr<double>(), out.size(0), out.size(1), kout.data_ptr<int>(),
                               npts.data_ptr<int>(), sorted.data_ptr<double>(), gperm.data_ptr<int>(),
                               u.data_ptr<double>(), ecap, s, k, nsamp, eps, min_points, min_edge, covp, ncov,
                               res.data_ptr<double>(), dbgp, presorted ? 1 : 0, mp, mh, mbytes, unplanned_stream());
  TORCH_CHECK(r != -2, "geo_spline: mask copy needs 4-byte aligned buffers and a size multiple of 4");
  TORCH_CHECK(r == 0, "geo_spline: k must be in [1, 5], nsamp in [1, 256]");
}

// INTER_AREA resize of one u8 HxWxC image on the device (tables from data/device_data.py)
void resize_area_u8(torch::Tensor in, torch::Tensor ys, torch::Tensor yn, torch::Tensor yw, torch::Tensor xs,
                    torch::Tensor xn, torch::Tensor xw, int swap_rb, torch::Tensor out) {
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == torch::kUInt8 && in.dim() == 3 && in.is_contiguous(), "in u8 HxWxC");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kUInt8 && out.dim() == 3 && out.is_contiguous() &&
              out.size(2) == in.size(2), "out u8 HxWxC");
  const int H = out.size(0), W = out.size(1), T = rdp_area_maxtap();
  TORCH_CHECK(ys.numel() == H && yn.numel() == H && yw.numel() == (long)H * T && xs.numel() == W &&
              xn.numel() == W && xw.numel() == (long)W * T, "area tables");
  TORCH_CHECK(ys.scalar_type() == torch::kInt32 && yw.scalar_type() == torch::kFloat64, "table dtypes");
  const int r = rdp_resize_area_u8(in.data_ptr(), in.size(0), in.size(1), in.size(2), ys.data_ptr<int>(),
                                   yn.data_ptr<int>(), yw.data_ptr<double>(), xs.data_ptr<int>(), xn.data_ptr<int>(),
                                   xw.data_ptr<double>(), H, W, swap_rb, out.data_ptr(), unplanned_stream());
  TORCH_CHECK(r == 0, "resize_area_u8: C must be 1..4");
}

// grayscale 8/16-bit PNG -> u8 / int16 (u16 bits) CPU tensor, decoded without the GIL; None when the
// PNG is not one this reader handles (or is corrupt): the caller falls back to PIL. `parallel`: inflate
// the bands of a banded stream (codecs.cpp) concurrently (2: only that way, else None -- tests).
py::object png_decode(py::bytes data, int parallel) {
  char* buf = nullptr;
  Py_ssize_t n = 0;
  if (PyBytes_AsStringAndSize(data.ptr(), &buf, &n) != 0) throw py::error_already_set();
  int w = 0, h = 0, bd = 0;
  if (rdp_png_info((const uint8_t*)buf, n, &w, &h, &bd) != 0) return py::none();
  auto t = torch::empty({h, w}, torch::TensorOptions().dtype(bd == 16 ? torch::kInt16 : torch::kUInt8));
  int r;
  {
    py::gil_scoped_release nogil;
    r = rdp_png_decode((const uint8_t*)buf, n, (uint8_t*)t.data_ptr(), (long)t.numel() * t.element_size(),
                       parallel);
  }
  if (r != 0) return py::none();
  return py::cast(t);
}

// Baseline JPEG -> (meta int32[32 + 3*64] = geometry + quant tables, quantized coefficient planes int16) on
// the CPU, entropy-decoded without the GIL (restart segments in parallel); None when the stream is not
// one this decoder handles (progressive, arithmetic, 12-bit, ...): the caller falls back to PIL.
// geometry: [0] W, [1] H, [2] ncomp, [3] hmax, [4] vmax, [5] total blocks; per component c at 8 + 8c:
// h, v, blocks per line, block rows, first block, plane byte offset, downsampled width, height.
py::object jpeg_decode(py::bytes data, bool parallel, bool pin) {
  char* buf = nullptr;
  Py_ssize_t n = 0;
  if (PyBytes_AsStringAndSize(data.ptr(), &buf, &n) != 0) throw py::error_already_set();
  int hi[24];
  const long nco = rdp_jpeg_info((const uint8_t*)buf, n, hi);
  if (nco <= 0) return py::none();
  // geometry and quant tables share one int32[32 + 192] tensor (one H2D copy per frame); with `pin`
  // both outputs come from the caching pinned-host allocator so the pipeline's copies are async DMA
  auto opt = torch::TensorOptions().pinned_memory(pin);
  auto meta = torch::zeros({32 + 192}, opt.dtype(torch::kInt32));
  int* g = meta.data_ptr<int>();
  rdp_jpeg_meta(hi, g);
  auto coefs = torch::empty({nco}, opt.dtype(torch::kInt16));
  uint16_t qt16[3 * 64];
  int r;
  {
    py::gil_scoped_release nogil;
    r = rdp_jpeg_decode((const uint8_t*)buf, n, coefs.data_ptr<int16_t>(), nco, qt16, parallel ? 1 : 0);
  }
  if (r != 0) return py::none();
  for (int i = 0; i < 3 * 64; ++i) g[32 + i] = qt16[i];
  return py::make_tuple(meta, coefs);
}

// Dequantisation + ISLOW 8x8 IDCT of every block into the component planes (`planes`, u8 scratch of
// jpeg_plane_bytes(H, W)), then fancy chroma upsampling + YCbCr -> RGB into rgb [H][W][3] u8 (GPU).
// geo / coefs / qt: jpeg_decode's outputs, on the device. Launch sizes come from the pipeline's
// frame size (H, W) so one captured graph serves every JPEG of that size; the kernels read the
// actual geometry from `geo`.
// the pixel stage + preprocess of n <= 4 frames of a serving batch in 2 + 1 launches (BatchEngine): per-frame
// lists; coefs / meta / planes empty for array sources (rgb: HxWx3 u8 colour frames, the preprocess input)
void batch_preprocess(std::vector<torch::Tensor> coefs, std::vector<torch::Tensor> meta,
                      std::vector<torch::Tensor> planes, std::vector<torch::Tensor> rgb, torch::Tensor ystart,
                      torch::Tensor ysize, torch::Tensor yw, torch::Tensor xstart, torch::Tensor xsize,
                      torch::Tensor xw, torch::Tensor out, int rgb_order) {
  const int n = (int)rgb.size();
  TORCH_CHECK(n >= 1 && n <= 4, "batch_preprocess: 1..4 frames");
  const int H = rgb[0].size(0), W = rgb[0].size(1);
  Act o = act(out, "out");
  TORCH_CHECK(o.N >= n && o.C == 8 && o.pitch == 8, "out must be [>= n, OH, OW, 8] contiguous");
  TORCH_CHECK(ystart.numel() == o.H && xstart.numel() == o.W && yw.numel() == (long)o.H * 16 &&
              xw.numel() == (long)o.W * 16, "aa tables");
  const bool jpeg = !coefs.empty();
  TORCH_CHECK(!jpeg || ((int)coefs.size() == n && (int)meta.size() == n && (int)planes.size() == n),
              "batch_preprocess: coefs / meta / planes: one per frame or none");
  std::vector<const void*> pc(n), pr(n);
  std::vector<const int*> pg(n), pq(n);
  std::vector<void*> pp(n), prw(n), po(n);
  for (int i = 0; i < n; ++i) {
    TORCH_CHECK(rgb[i].is_cuda() && rgb[i].scalar_type() == torch::kUInt8 && rgb[i].dim() == 3 && rgb[i].size(2) == 3 &&
                    rgb[i].is_contiguous() && rgb[i].size(0) == H && rgb[i].size(1) == W, "rgb u8 HxWx3, one size");
    pr[i] = rgb[i].data_ptr();
    prw[i] = rgb[i].data_ptr();
    po[i] = (char*)o.ptr + (long)i * o.H * o.W * 8 * 2;
    if (jpeg) {
      TORCH_CHECK(coefs[i].is_cuda() && coefs[i].scalar_type() == torch::kInt16 &&
                      coefs[i].numel() >= rdp_jpeg_max_coefs(H, W), "coefs");
      TORCH_CHECK(meta[i].is_cuda() && meta[i].scalar_type() == torch::kInt32 && meta[i].numel() >= 224, "meta");
      TORCH_CHECK(planes[i].is_cuda() && planes[i].numel() >= rdp_jpeg_plane_bytes(H, W), "planes");
      pc[i] = coefs[i].data_ptr();
      pg[i] = meta[i].data_ptr<int>();
      pq[i] = meta[i].data_ptr<int>() + 32;
      pp[i] = planes[i].data_ptr();
    }
  }
  const hipStream_t st = unplanned_stream();
  if (jpeg)
    TORCH_CHECK(rdp_jpeg_gpu_batch(n, pc.data(), pg.data(), pq.data(), pp.data(), H, W,
                                   (int)(coefs[0].numel() / 64), prw.data(), st) == 0, "jpeg batch");
  TORCH_CHECK(rdp_preprocess_batch(n, pr.data(), H, W, ystart.data_ptr<int>(), ysize.data_ptr<int>(),
                                   yw.data_ptr<float>(), xstart.data_ptr<int>(), xsize.data_ptr<int>(),
                                   xw.data_ptr<float>(), o.H, o.W, rgb_order, po.data(), st) == 0, "preprocess batch");
}

void jpeg_to_rgb(torch::Tensor coefs, torch::Tensor geo, torch::Tensor qt, torch::Tensor planes, torch::Tensor rgb) {
  TORCH_CHECK(coefs.is_cuda() && coefs.scalar_type() == torch::kInt16 && coefs.is_contiguous(), "coefs int16");
  TORCH_CHECK(geo.is_cuda() && geo.scalar_type() == torch::kInt32 && geo.numel() >= 32, "geo int32[32]");
  TORCH_CHECK(qt.is_cuda() && qt.scalar_type() == torch::kInt32 && qt.numel() >= 192, "qt int32[192]");
  TORCH_CHECK(rgb.is_cuda() && rgb.scalar_type() == torch::kUInt8 && rgb.dim() == 3 && rgb.size(2) == 3 &&
              rgb.is_contiguous(), "rgb u8 HxWx3");
  const int H = rgb.size(0), W = rgb.size(1);
  TORCH_CHECK(planes.is_cuda() && planes.scalar_type() == torch::kUInt8 && planes.numel() >= rdp_jpeg_plane_bytes(H, W),
              "planes: jpeg_plane_bytes(H, W) u8");
  TORCH_CHECK(coefs.numel() >= rdp_jpeg_max_coefs(H, W), "coefs: jpeg_max_coefs(H, W) int16");
  rdp_jpeg_gpu(coefs.data_ptr(), geo.data_ptr<int>(), qt.data_ptr<int>(), planes.data_ptr(), H, W,
               (int)(coefs.numel() / 64), rgb.data_ptr(), unplanned_stream());
}

// u8 [H, W] CPU tensor -> 8-bit grayscale PNG bytes (deflate level), encoded without the GIL
// u8 or int16 (u16 bits) [H, W] CPU tensor -> 8 / 16-bit grayscale PNG bytes, encoded without the GIL;
// bands > 1: a banded stream with its rdPs index (codecs.cpp), bands deflated in parallel
py::bytes png_encode(torch::Tensor img, int level, int bands) {
  TORCH_CHECK(!img.is_cuda() && (img.scalar_type() == torch::kUInt8 || img.scalar_type() == torch::kInt16) &&
                  img.dim() == 2 && img.is_contiguous(),
              "u8 / int16 HxW contiguous CPU tensor");
  const int h = img.size(0), w = img.size(1), bpp = (int)img.element_size();
  TORCH_CHECK(h > 0 && w > 0 && level >= 0 && level <= 9 && bands >= 1, "png_encode: bad size / level / bands");
  std::string out((size_t)rdp_png_encode_bound(w, h, bpp, bands), '\0');
  long len;
  {
    py::gil_scoped_release nogil;
    len = rdp_png_encode_gray((const uint8_t*)img.data_ptr(), w, h, bpp, level, bands, (uint8_t*)&out[0],
                              (long)out.size());
  }
  TORCH_CHECK(len > 0, "png encode failed");
  out.resize((size_t)len);
  return py::bytes(out);
}


void preprocess(torch::Tensor bgr, torch::Tensor ystart, torch::Tensor ysize, torch::Tensor yw, torch::Tensor xstart,
                torch::Tensor xsize, torch::Tensor xw, torch::Tensor out, int rgb) {
  TORCH_CHECK(bgr.is_cuda() && bgr.scalar_type() == torch::kUInt8 && bgr.dim() == 3 && bgr.size(2) == 3 &&
              bgr.is_contiguous(), "bgr u8 HxWx3");
  Act o = act(out, "out");
  TORCH_CHECK(o.N == 1 && o.C == 8 && o.pitch == 8, "out must be [1,OH,OW,8] contiguous");
  TORCH_CHECK(ystart.numel() == o.H && xstart.numel() == o.W && yw.numel() == (long)o.H * 16 &&
              xw.numel() == (long)o.W * 16, "aa tables");
  rdp_preprocess(bgr.data_ptr(), bgr.size(0), bgr.size(1), ystart.data_ptr<int>(), ysize.data_ptr<int>(),
                 yw.data_ptr<float>(), xstart.data_ptr<int>(), xsize.data_ptr<int>(), xw.data_ptr<float>(), o.H, o.W,
                 rgb, o.ptr, unplanned_stream());
}

void mask_upsample(torch::Tensor m, torch::Tensor out, torch::Tensor count) {
  TORCH_CHECK(m.is_cuda() && m.scalar_type() == torch::kUInt8 && m.dim() == 2 && m.is_contiguous(), "m");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kUInt8 && out.dim() == 2 && out.is_contiguous(), "out");
  TORCH_CHECK(count.is_cuda() && count.scalar_type() == torch::kInt32, "count int32");
  rdp_mask_upsample(m.data_ptr(), m.size(0), m.size(1), out.data_ptr(), out.size(0), out.size(1),
                    (unsigned*)count.data_ptr(), unplanned_stream());
}

}  // namespace

void register_serve_runtime(py::module_& m);  // serve_runtime.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  register_serve_runtime(m);
  m.doc() = "rdp MI355X (gfx950) HIP kernels";
  m.def("stream_wait", &stream_wait, "waiter stream waits for the work issued so far on waitee (recorded in plans)");
  m.def("event_create", &event_create, "runtime-owned cross-stream event (id)");
  m.def("event_record", &event_record, py::arg("id"), py::arg("stream"), "record event id on stream (recorded in plans)");
  m.def("stream_wait_event", &stream_wait_event, py::arg("stream"), py::arg("id"),
        "stream waits for the last record of event id (recorded in plans)");
  m.def("plan_begin", &plan_begin);
  m.def("plan_end", &plan_end);
  m.def("plan_abort", &plan_abort);
  m.def("plan_replay", &plan_replay, py::arg("id"), py::arg("host_call") = py::none());
  m.def("plan_kinds", &plan_kinds);
  m.def("plan_recording", &plan_recording);
  m.def("comm_bind", &comm_bind, "resolve RCCL from the library torch loaded; returns its path");
  m.def("comm_all_reduce", on_device(&comm_all_reduce), py::arg("buf"), py::arg("comm"),
        "in-place SUM all-reduce over an RCCL communicator on the current stream (recorded in plans)");
  m.def("rows_fold", on_device(&rows_fold), py::arg("buf"), py::arg("rows"), py::arg("width"), py::arg("out"));
  m.def("rows_hilo", on_device(&rows_hilo), py::arg("sums"), py::arg("buf"), py::arg("width"));
  m.def("comm_async_error", &comm_async_error, py::arg("comm"), "(code, message) of ncclCommGetAsyncError");
  m.def("comm_abort", &comm_abort, py::arg("comm"), "ncclCommAbort");
  m.def("comm_info", &comm_info, py::arg("comm"), "(ncclCommCount, ncclCommUserRank, ncclCommCuDevice)");
  m.def("comm_emulate", &comm_emulate, py::arg("us"), py::arg("blocks"), py::arg("scratch") = py::none(),
        py::arg("traffic_bytes") = 0, "RDP_DDP_EMULATE: the modelled all-reduce on the current stream (recorded in plans)");
  m.def("plan_mark", &plan_mark, "record a host call point (replay calls host_call(tag) there)");
  m.def("plan_pause", &plan_pause);
  m.def("plan_resume", &plan_resume);
  m.def("plan_size", &plan_size);
  m.def("plan_free", &plan_free);
  m.def("conv_fwd", on_device(&conv_fwd), py::arg("x1"), py::arg("x2"), py::arg("w"), py::arg("taps"), py::arg("packed"),
        py::arg("y1"), py::arg("y2"), py::arg("stats"), py::arg("bm_pref"), py::arg("affine"), py::arg("relu"),
        py::arg("ws") = py::none(), py::arg("pool") = py::none(), py::arg("up") = py::none(),
        py::arg("up_oy") = 0, py::arg("up_ox") = 0, py::arg("wfrag") = py::none());
  m.def("conv_ws_elems", [](int N, int H, int W, int C1, int C2, int Cout, int taps, int packed, int bm_pref) {
    return rdp_conv_ws_elems(N, H, W, C1, C2, Cout, taps, packed, bm_pref);
  });
  m.def("conv_stats_rows", &conv_stats_rows);
  m.def("conv_wgrad", on_device(&conv_wgrad), py::arg("x1"), py::arg("x2"), py::arg("dy"), py::arg("taps"),
        py::arg("packed"), py::arg("cin_real"), py::arg("slab"), py::arg("out"), py::arg("accumulate"),
        py::arg("splits"), py::arg("variant"));
  m.def("conv_fwd_bnin", on_device(&conv_fwd_bnin), py::arg("x_pre"), py::arg("w"), py::arg("y"), py::arg("stats"),
        py::arg("in_coef"), py::arg("a_out") = py::none());
  m.def("wgrad_first_bn", on_device(&wgrad_first_bn));
  m.def("wgrad_slab_elems", &wgrad_slab_elems);
  m.def("wgrad_halo_slab_elems", &rdp_conv_wgrad_halo_slab_elems);
  m.def("bn_finalize", on_device(&bn_finalize));
  m.def("bn_eval_coef", on_device(&bn_eval_coef));
  m.def("bn_relu_apply", on_device(&bn_relu_apply));
  m.def("bn_relu_bwd_reduce", on_device(&bn_relu_bwd_reduce));
  m.def("conv_dgrad_bnred", on_device(&conv_dgrad_bnred));
  m.def("conv_dgrad_splitk_bnred", on_device(&conv_dgrad_splitk_bnred), py::arg("dy"), py::arg("w"), py::arg("dx"),
        py::arg("y_bn"), py::arg("coef"), py::arg("partial"), py::arg("ws") = py::none());
  m.def("bn_bwd_finalize", on_device(&bn_bwd_finalize));
  m.def("bn_relu_bwd_apply", on_device(&bn_relu_bwd_apply));
  m.def("maxpool2_fwd", on_device(&maxpool2_fwd));
  m.def("maxpool2_bwd", on_device(&maxpool2_bwd));
  m.def("bn_relu_apply_pool", on_device(&bn_relu_apply_pool));
  m.def("maxpool2_bwd_bn_reduce", on_device(&maxpool2_bwd_bn_reduce));
  m.def("upsample2_fwd", on_device(&upsample2_fwd), py::arg("x"), py::arg("out"), py::arg("oy"), py::arg("ox"),
        py::arg("coef") = py::none());
  m.def("upT_shuffle", on_device(&upT_shuffle));
  m.def("conv_upT_fwd", on_device(&conv_upT_fwd));
  m.def("conv_upT_dgrad", on_device(&conv_upT_dgrad));
  m.def("conv_wgrad_upT", on_device(&conv_wgrad_upT));
  m.def("upT_unshuffle", on_device(&upT_unshuffle));
  m.def("colsum_bf16", on_device(&colsum_bf16));
  m.def("upsample2_bwd", on_device(&upsample2_bwd), py::arg("dout"), py::arg("dx"), py::arg("oy"), py::arg("ox"),
        py::arg("y") = py::none(), py::arg("coef") = py::none(), py::arg("partial") = py::none());
  m.def("head_partial_blocks", &head_partial_blocks);
  m.def("head_fwd", on_device(&head_fwd), py::arg("a"), py::arg("w"), py::arg("b"), py::arg("target"), py::arg("logits"),
        py::arg("partial"), py::arg("sums"), py::arg("loss"), py::arg("dice_w"), py::arg("dice_eps"),
        py::arg("coef") = py::none(), py::arg("gpart") = py::none(), py::arg("bnpart") = py::none(),
        py::arg("gscale") = 1.0);
  m.def("head_grad_finalize", on_device(&head_grad_finalize));
  m.def("head_bwd", on_device(&head_bwd), py::arg("a"), py::arg("w"), py::arg("logits"), py::arg("target"), py::arg("sums"),
        py::arg("da"), py::arg("partial"), py::arg("gw"), py::arg("gb"), py::arg("dice_w"), py::arg("dice_eps"),
        py::arg("gscale"), py::arg("coef") = py::none(), py::arg("bnpart") = py::none());
  m.def("head_bn_bwd_apply", on_device(&head_bn_bwd_apply));
  m.def("head_mask", on_device(&head_mask));
  m.def("conv_head_mask", on_device(&conv_head_mask));
  m.def("conv_rowband_chain", on_device(&conv_rowband_chain));
  m.def("conv_rowband", on_device(&conv_rowband));
  // host-only: the eval conv's row-band mode for a shape (0 = implicit GEMM), the same decision conv_fwd takes
  m.def("rowband_frag_mode", &rdp_conv_rowband_frag_auto, py::arg("n"), py::arg("h"), py::arg("w"), py::arg("c1"),
        py::arg("c2"), py::arg("cout"));
  m.def("adam", on_device(&adam), py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("shadow"), py::arg("lr"),
        py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("gscale"), py::arg("step"),
        py::arg("inc") = true, py::arg("max_blocks") = 0);
  m.def("cast_bf16", on_device(&cast_bf16));
  m.def("h2d_copy", &h2d_copy, py::arg("src"), py::arg("dst"));
  m.def("wprep", on_device(&wprep), py::arg("master"), py::arg("out"), py::arg("segs"), py::arg("nseg"),
        py::arg("step") = py::none(), py::arg("blocks") = 0);
  m.def("wseg_size", &rdp_wseg_size);
  m.def("parcur", &parcur);
  m.def("batch_preprocess", on_device(&batch_preprocess));
  m.def("geo_frames_batch", on_device(&geo_frames_batch));
  m.def("geo_edges", on_device(&geo_edges), py::arg("mask"), py::arg("depth"), py::arg("fx"), py::arg("fy"), py::arg("cx"),
        py::arg("cy"), py::arg("scale"), py::arg("work_i"), py::arg("work_d"), py::arg("pts"), py::arg("npts"),
        py::arg("out"), py::arg("kout"), py::arg("nbins"), py::arg("top"), py::arg("min_points"),
        py::arg("edges") = py::none(), py::arg("hdr") = py::none(), py::arg("m256") = py::none(),
        py::arg("cov") = py::none(), py::arg("sorted") = py::none(), py::arg("gperm") = py::none(),
        py::arg("mask_host") = py::none());
  m.def("geo_nblocks", &geo_nblocks);
  m.def("geo_spline", on_device(&geo_spline), py::arg("out"), py::arg("kout"), py::arg("npts"), py::arg("sorted"),
        py::arg("gperm"), py::arg("u"), py::arg("res"), py::arg("s"), py::arg("k"), py::arg("nsamp"), py::arg("eps"),
        py::arg("min_points"), py::arg("min_edge"), py::arg("cov") = py::none(), py::arg("dbg") = py::none(),
        py::arg("presorted") = false, py::arg("mask") = py::none(), py::arg("mask_host") = py::none());
  m.def("png_decode", &png_decode, py::arg("data"), py::arg("parallel") = 1,
        "parallel: 0 serial inflate, 1 banded (rdPs index) with serial fallback, 2 banded only (tests)");
  m.def("jpeg_decode", &jpeg_decode, py::arg("data"), py::arg("parallel") = true, py::arg("pin") = false);
  m.def("jpeg_to_rgb", on_device(&jpeg_to_rgb));
  m.def("jpeg_plane_bytes", &rdp_jpeg_plane_bytes);
  m.def("jpeg_max_coefs", &rdp_jpeg_max_coefs);
  m.def("png_encode", &png_encode, py::arg("img"), py::arg("level") = 1, py::arg("bands") = 1);
  m.def("resize_area_u8", on_device(&resize_area_u8));
  m.def("area_maxtap", &rdp_area_maxtap);
  m.def("geo_spline_res_len", &rdp_geo_spline_res_len);
  m.def("geo_work_ints", &geo_work_ints);
  m.def("preprocess", on_device(&preprocess), py::arg("bgr"), py::arg("ystart"), py::arg("ysize"), py::arg("yw"),
        py::arg("xstart"), py::arg("xsize"), py::arg("xw"), py::arg("out"), py::arg("rgb") = 0);
  m.def("mask_upsample", on_device(&mask_upsample));
  m.def("splev", &splev);
  m.def("fit_curvature", &fit_curvature);
}
