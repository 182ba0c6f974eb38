// Native per-frame serving runtime: the host side of one served frame, off the Python GIL.
//
// Reference per-frame path (/root/reference/services/vision_analysis/server.py:116-152): decode, model,
// mask resize, geometry, then build the AnalysisResponse in Python. Here the device work is one
// captured hipGraph per pipeline (serve/engine.py FramePipeline); what remained in Python per frame --
// ~15 torch calls for staging copies, event records and the graph replay, then the response message
// built field by field -- held the interpreter lock ~0.5 ms per frame, which capped a server process
// at ~1,000 frames/s however many streams it served (profiles/serve_e2e.md). Two pieces move here:
//
//   FrameRunner      stage a frame into the pipeline's pinned buffers, enqueue H2D copies, launch the
//                    graph execs, enqueue the D2H copies and the timing events, with the GIL released.
//                    A frame goes in two calls on the pipeline's stream: the colour half (H2D + the
//                    network graph) as soon as the colour frame is decoded, the depth half (H2D + the
//                    geometry graph + D2H) when the depth frame is -- so the network runs while the
//                    depth PNG is still inflating. wait() blocks on the frame's end event.
//   encode_response  mask PNG (banded, codecs.cpp) + the evofab.vision.AnalysisResponse wire encoding
//                    (/root/reference/protos/vision.proto:29-37), byte-identical to protobuf's own
//                    serializer (fields in number order, proto3 defaults omitted); the gRPC handler
//                    yields the bytes (proto/vision.py passes them through).
#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "host_pool.h"
#include "wire_parse.h"

namespace py = pybind11;

extern "C" int rdp_h2d_copy(const void*, void*, long, hipStream_t);
extern "C" int rdp_h2d_copy_multi(const void* const*, void* const*, const long*, int, hipStream_t);
extern "C" long rdp_png_encode_gray(const uint8_t*, int, int, int, int, int, uint8_t*, long);
extern "C" long rdp_png_encode_bound(int, int, int, int);
extern "C" long rdp_jpeg_info(const uint8_t*, long, int*);
extern "C" void rdp_jpeg_meta(const int*, int*);
extern "C" int rdp_jpeg_decode(const uint8_t*, long, int16_t*, long, uint16_t*, int);
extern "C" int rdp_png_info(const uint8_t*, long, int*, int*, int*);
extern "C" int rdp_png_decode(const uint8_t*, long, uint8_t*, long, int);

namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceScope {  // make `dev` current for this thread, restore on exit
  int prev = -1;
  explicit DeviceScope(int dev) {
    hip_check(hipGetDevice(&prev), "hipGetDevice");
    if (prev != dev) hip_check(hipSetDevice(dev), "hipSetDevice");
  }
  ~DeviceScope() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

inline void* P(uintptr_t v) { return reinterpret_cast<void*>(v); }

std::string encode_wire(double mean, double maxc, const double* pts, size_t npts, const std::string& status,
                        const uint8_t* mask01, int h, int w, float coverage, float proc_ms, int level, int bands);

using rdp_wire::parse_request;  // wire_parse.h: the request's two payloads, read in place

class FrameRunner {
 public:
  FrameRunner(int device, uintptr_t stream) : dev_(device), s_((hipStream_t)stream) {
    DeviceScope g(dev_);
    hip_check(hipEventCreate(&ev0_), "hipEventCreate");
    hip_check(hipEventCreate(&ev1_), "hipEventCreate");
    // the depth frame's H2D runs on its own stream, under the network graph; the geometry graph waits
    // for it (a GPU-side dependency only: no system-scope fence)
    hip_check(hipStreamCreateWithFlags(&cs_, hipStreamNonBlocking), "hipStreamCreate");
    hip_check(hipEventCreateWithFlags(&evd_, hipEventDisableTiming | hipEventDisableSystemFence), "hipEventCreate");
  }
  ~FrameRunner() {
    (void)hipEventDestroy(ev0_);
    (void)hipEventDestroy(ev1_);
    (void)hipEventDestroy(evd_);
    (void)hipStreamDestroy(cs_);
    for (void* p : host_) (void)hipHostFree(p);
  }
  // graph execs, owned by the pipeline's torch CUDAGraphs (kept alive there): slots 0..2 = the network
  // graph of colour source 0 BGR / 1 RGB / 2 JPEG coefficients, slot 3 = the geometry graph
  void set_graph(int slot, uintptr_t exec) {
    if (slot < 0 || slot > 3) throw std::invalid_argument("slot");
    exec_[slot] = (hipGraphExec_t)exec;
  }
  // Measured (same box, 2 rounds): the copy stream vs the depth H2D in order on the frame stream --
  // engine GPU p50 0.515-0.524 vs 0.536 ms, pipelined 3,025-3,105 vs 2,837-2,926 FPS, e2e 4 streams in
  // one process 1,886-2,582 vs 1,506-1,562 FPS, 2 processes x 2 streams 3,353-3,420 vs 3,177-3,433.
  void depth_stream(bool on) { depth_stream_ = on; }

  // fine-grained (coherent) host memory that kernels write directly -- the frame's mask and result
  // vector, so no read-back copies follow the geometry graph (freed with the runner)
  uintptr_t alloc_host(size_t bytes) {
    DeviceScope g(dev_);
    void* p = nullptr;
    hip_check(hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped), "hipHostMalloc");
    std::memset(p, 0, bytes);
    host_.push_back(p);
    return (uintptr_t)p;
  }

  // pinned host staging / device buffers of the pipeline (sizes in bytes; mask / result sizes 0: the
  // geometry kernels write them to host memory themselves)
  void set_buffers(uintptr_t d_color, uintptr_t h_color, size_t color_bytes, uintptr_t d_depth, uintptr_t h_depth,
                   size_t depth_bytes, uintptr_t d_meta, size_t meta_bytes, uintptr_t d_coef, size_t coef_cap,
                   uintptr_t d_mask, uintptr_t h_mask, size_t mask_bytes, uintptr_t d_res, uintptr_t h_res,
                   size_t res_bytes) {
    d_color_ = P(d_color); h_color_ = P(h_color); color_bytes_ = color_bytes;
    kernel_copy_ = !(getenv("RDP_COLOR_COPY") && std::string(getenv("RDP_COLOR_COPY")) == "dma");
    d_depth_ = P(d_depth); h_depth_ = P(h_depth); depth_bytes_ = depth_bytes;
    d_meta_ = P(d_meta); meta_bytes_ = meta_bytes; d_coef_ = P(d_coef); coef_cap_ = coef_cap;
    d_mask_ = P(d_mask); h_mask_ = P(h_mask); mask_bytes_ = mask_bytes;
    d_res_ = P(d_res); h_res_ = P(h_res); res_bytes_ = res_bytes;
  }

  // colour half, from an HxWx3 u8 array (src 0 BGR / 1 RGB)
  void submit_array(int src, py::buffer color) {
    py::buffer_info c = color.request();
    check_contig(c, color_bytes_, "colour");
    if (src != 0 && src != 1) throw std::invalid_argument("src must be 0 (BGR) or 1 (RGB)");
    need(src);
    const void* cp = c.ptr;
    py::gil_scoped_release nogil;
    DeviceScope g(dev_);
    std::memcpy(h_color_, cp, color_bytes_);  // host staging: the caller's "submit" stage, not device time
    hip_check(hipEventRecord(ev0_, s_), "hipEventRecord");
    upload(d_color_, h_color_, color_bytes_, "H2D colour");
    hip_check(hipGraphLaunch(exec_[src], s_), "hipGraphLaunch");
  }

  // colour half, from an entropy-decoded JPEG (data/jpeg.py JpegCoefs: pinned meta + coefficient
  // buffers; the caller keeps them alive until wait() returns)
  void submit_jpeg(uintptr_t meta, size_t meta_bytes, uintptr_t coefs, size_t coef_bytes) {
    if (meta_bytes != meta_bytes_ || coef_bytes > coef_cap_) throw std::invalid_argument("JPEG buffers exceed the pipeline");
    need(2);
    py::gil_scoped_release nogil;
    DeviceScope g(dev_);
    hip_check(hipEventRecord(ev0_, s_), "hipEventRecord");
    upload(d_meta_, P(meta), meta_bytes, "H2D meta", false);
    upload(d_coef_, P(coefs), coef_bytes, "H2D coefs", false);
    hip_check(hipGraphLaunch(exec_[2], s_), "hipGraphLaunch");
  }

  // depth half (HxW 16-bit): H2D, the geometry graph, the result read-back and the frame's end event
  void submit_depth(py::buffer depth) {
    py::buffer_info d = depth.request();
    check_contig(d, depth_bytes_, "depth");
    need(3);
    const void* dp = d.ptr;
    py::gil_scoped_release nogil;
    DeviceScope g(dev_);
    std::memcpy(h_depth_, dp, depth_bytes_);
    launch_depth_half();
  }

 private:
  // Host -> device upload on the frame stream: a copy kernel reading the pinned source through its device
  // mapping (rdp_h2d_copy) where it has one and RDP_COLOR_COPY != dma -- the DMA-engine copy costs an
  // engine -> compute hand-off (~10 us) before the next kernel (profiles/serve_experiments.md) -- else
  // hipMemcpyAsync. Device mappings of the (few, long-lived) staging buffers are cached.
  void upload(void* dst, const void* src, size_t bytes, const char* what, bool cache = true) {
    const hipStream_t st = s_;
    if (kernel_copy_ && bytes && !((uintptr_t)dst & 15)) {
      void* dp = nullptr;
      bool known = false;
      if (cache)
        for (auto& m : hmap_)
          if (m.first == src) { dp = m.second; known = true; }
      if (!known) {  // (with unified addressing the mapping is often the host address itself)
        if (hipHostGetDevicePointer(&dp, const_cast<void*>(src), 0) != hipSuccess) {
          (void)hipGetLastError();
          dp = nullptr;
        }
        if (cache) {  // runner-owned staging only: a caller's buffer may be freed and its address reused
          if (hmap_.size() >= 16) hmap_.erase(hmap_.begin());
          hmap_.emplace_back(src, dp);  // nullptr: no mapping, the DMA copy below
        }
      }
      if (dp && !((uintptr_t)dp & 15) && rdp_h2d_copy(dp, dst, (long)bytes, st) == 0) return;
      (void)hipGetLastError();
    }
    hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st), what);
  }

  void launch_depth_half() {  // h_depth_ staged; the device is current
    if (depth_stream_) {
      hip_check(hipMemcpyAsync(d_depth_, h_depth_, depth_bytes_, hipMemcpyHostToDevice, cs_), "H2D depth");
      hip_check(hipEventRecord(evd_, cs_), "hipEventRecord");
      hip_check(hipStreamWaitEvent(s_, evd_, 0), "hipStreamWaitEvent");
    } else {
      hip_check(hipMemcpyAsync(d_depth_, h_depth_, depth_bytes_, hipMemcpyHostToDevice, s_), "H2D depth");
    }
    hip_check(hipGraphLaunch(exec_[3], s_), "hipGraphLaunch");
    if (mask_bytes_) hip_check(hipMemcpyAsync(h_mask_, d_mask_, mask_bytes_, hipMemcpyDeviceToHost, s_), "D2H mask");
    if (res_bytes_) hip_check(hipMemcpyAsync(h_res_, d_res_, res_bytes_, hipMemcpyDeviceToHost, s_), "D2H result");
    hip_check(hipEventRecord(ev1_, s_), "hipEventRecord");
    recorded_ = true;
  }

 public:
  // ---- whole requests natively (the gRPC fast path) ---------------------------------------------------
  // The colour JPEG and depth PNG bytes of an AnalysisRequest: the JPEG is entropy-decoded into this
  // runner's pinned coefficient buffers and its network graph launched while the depth PNG inflates in
  // parallel (host pool), then the geometry half -- one call, no interpreter lock. collect_encoded()
  // waits for the frame and builds the AnalysisResponse wire bytes from the result the geometry kernels
  // wrote to host memory. Frames this path does not take (JPEG the native decoder declines, other frame
  // sizes, non-16-bit depth) return a code and nothing is launched: the caller decodes them itself.
  enum { kOk = 0, kNotNative = 1, kSize = 2, kCorrupt = 3 };
  void configure_encoded(int H, int W, int num_samples) {
    DeviceScope g(dev_);
    H_ = H; W_ = W; ns_ = num_samples;
    if (!h_meta_) {
      hip_check(hipHostMalloc(&h_meta_, meta_bytes_ ? meta_bytes_ : 224 * 4, hipHostMallocDefault), "hipHostMalloc");
      hip_check(hipHostMalloc(&h_coef_, coef_cap_ ? coef_cap_ : 2, hipHostMallocDefault), "hipHostMalloc");
      host_.push_back(h_meta_);
      host_.push_back(h_coef_);
    }
  }

  int submit_encoded(py::bytes color, py::bytes depth) {
    char *cp = nullptr, *dp = nullptr;
    Py_ssize_t cn = 0, dn = 0;
    if (PyBytes_AsStringAndSize(color.ptr(), &cp, &cn) != 0 || PyBytes_AsStringAndSize(depth.ptr(), &dp, &dn) != 0)
      throw py::error_already_set();
    if (!h_meta_ || !h_coef_ || !exec_[2] || !exec_[3]) throw std::runtime_error("FrameRunner: configure_encoded first");
    py::gil_scoped_release nogil;
    return submit_encoded_ptr((const uint8_t*)cp, (long)cn, (const uint8_t*)dp, (long)dn);
  }

  // the whole serialized AnalysisRequest (the server's raw-bytes handler): parsed here, without the GIL;
  // 1 (and nothing launched) when it is not a message this parser takes
  int submit_request(py::bytes raw) {
    char* rp = nullptr;
    Py_ssize_t rn = 0;
    if (PyBytes_AsStringAndSize(raw.ptr(), &rp, &rn) != 0) throw py::error_already_set();
    if (!h_meta_ || !h_coef_ || !exec_[2] || !exec_[3]) throw std::runtime_error("FrameRunner: configure_encoded first");
    py::gil_scoped_release nogil;
    const uint8_t *c, *d;
    size_t cn, dn;
    if (!parse_request((const uint8_t*)rp, (size_t)rn, c, cn, d, dn)) return kNotNative;
    return submit_encoded_ptr(c, (long)cn, d, (long)dn);
  }

  int submit_encoded_ptr(const uint8_t* c, long cn, const uint8_t* d, long dn) {  // GIL released
    t0_ = std::chrono::steady_clock::now();
    // headers first: nothing is launched unless both halves are native frames of this pipeline's size
    int hi[24];
    const long nco = rdp_jpeg_info(c, (long)cn, hi);
    if (nco == -1) return kCorrupt;
    if (nco <= 0) return kNotNative;
    int pw = 0, ph = 0, bd = 0;
    if (rdp_png_info(d, (long)dn, &pw, &ph, &bd) != 0 || bd != 16) return kNotNative;
    if (hi[0] != W_ || hi[1] != H_ || pw != W_ || ph != H_) return kSize;
    if ((size_t)nco * 2 > coef_cap_ || meta_bytes_ < 224 * 4) return kNotNative;
    int rc[2] = {0, 0};
    std::string err[2];  // one per half: both halves may throw concurrently
    DeviceScope g(dev_);
    rdp::host_pool().parallel_for(2, [&](int k) {
      try {
        work_half(k, c, (long)cn, d, (long)dn, hi, nco, rc);
      } catch (const std::exception& e) {  // never out of a pool thread
        rc[k] = -1;
        err[k] = e.what();
      }
    });
    if (rc[0] < 0 || rc[1] < 0) {
      (void)hipStreamSynchronize(s_);
      throw std::runtime_error("submit_encoded: " + (rc[0] < 0 ? err[0] : err[1]));
    }
    if (rc[0]) {  // nothing of the frame was launched
      return rc[0];
    }
    if (rc[1]) {  // the colour half is in flight: drain it, report the frame
      hip_check(hipStreamSynchronize(s_), "hipStreamSynchronize");
      return rc[1];
    }
    launch_depth_half();
    return kOk;
  }

  void work_half(int k, const uint8_t* c, long cn, const uint8_t* d, long dn, const int* hi, long nco, int* rc) {
    {
      if (k == 0) {  // colour: entropy decode, then the network half on the frame stream
        int* meta = (int*)h_meta_;
        rdp_jpeg_meta(hi, meta);
        uint16_t qt[3 * 64];
        if (rdp_jpeg_decode(c, cn, (int16_t*)h_coef_, nco, qt, 1) != 0) { rc[0] = kCorrupt; return; }
        for (int i = 0; i < 3 * 64; ++i) meta[32 + i] = qt[i];
        DeviceScope gk(dev_);
        hip_check(hipEventRecord(ev0_, s_), "hipEventRecord");
        upload(d_meta_, h_meta_, meta_bytes_, "H2D meta");
        upload(d_coef_, h_coef_, (size_t)nco * 2, "H2D coefs");
        hip_check(hipGraphLaunch(exec_[2], s_), "hipGraphLaunch");
      } else {  // depth: 16-bit PNG straight into the pinned staging buffer
        if (rdp_png_decode(d, dn, (uint8_t*)h_depth_, (long)depth_bytes_, 1) != 0) rc[1] = kCorrupt;
      }
    }
  }

  // (payload bytes, mean, max, coverage %, status code, gpu ms); status code 4 = the fit needs the host
  // (the caller finishes that frame from the device edge buffers)
  py::tuple collect_encoded(int level, int bands) {
    float gpu_ms = 0.f;
    double mean = 0, maxc = 0, cov = 0;
    int st = 0;
    std::string out;
    {
      py::gil_scoped_release nogil;
      DeviceScope g(dev_);
      sync_end();
      hip_check(hipEventElapsedTime(&gpu_ms, ev0_, ev1_), "hipEventElapsedTime");
      const double* r = (const double*)h_res_;
      st = (int)r[0];
      const double count = r[8 + 3 * ns_];
      cov = 100.0 * count / ((double)H_ * W_);
      if (st != 4) {
        static const char* names[4] = {"ok", "too_few_points", "too_few_edge_points", "fit_failed"};
        const std::string status = (st >= 0 && st < 4) ? names[st] : "fit_failed";
        if (st == 0) { mean = r[4]; maxc = r[5]; }
        const float proc =
            std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0_).count();
        out = encode_wire(mean, maxc, st == 0 ? r + 8 : nullptr, st == 0 ? (size_t)ns_ : 0, status,
                          (const uint8_t*)h_mask_, H_, W_, (float)cov, proc, level, bands);
      }
    }
    return py::make_tuple(py::bytes(out), mean, maxc, cov, st, gpu_ms);
  }

  // a frame whose depth half never came (its decode failed): drain the colour half
  void abort() {
    py::gil_scoped_release nogil;
    DeviceScope g(dev_);
    hip_check(hipStreamSynchronize(cs_), "hipStreamSynchronize");
    hip_check(hipStreamSynchronize(s_), "hipStreamSynchronize");
  }

  // block until the frame's results are on the host; returns its device time (ms, event to event)
  float wait() {
    if (!recorded_) return 0.f;  // nothing submitted yet
    py::gil_scoped_release nogil;
    DeviceScope g(dev_);
    sync_end();
    float ms = 0.f;
    hip_check(hipEventElapsedTime(&ms, ev0_, ev1_), "hipEventElapsedTime");
    return ms;
  }

  // Wait for the frame's end event: poll it for up to spin_us_ microseconds (a frame is ~0.4 ms of GPU
  // time, so a waiter that polls sees the result as soon as it lands instead of paying a blocking
  // wait's wake-up), then block. RDP_SERVE_SPIN_US (default 0: block at once) / set_spin_us.
  void sync_end() {
    if (spin_us_ > 0) {
      const auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        const hipError_t q = hipEventQuery(ev1_);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) hip_check(q, "hipEventQuery");
        if (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > spin_us_)
          break;
      }
    }
    hip_check(hipEventSynchronize(ev1_), "hipEventSynchronize");
  }
  void set_spin_us(double us) { spin_us_ = us; }

 private:
  static void check_contig(const py::buffer_info& b, size_t bytes, const char* what) {
    size_t n = (size_t)b.itemsize;
    for (auto s : b.shape) n *= (size_t)s;
    ssize_t expect = b.itemsize;
    for (ssize_t i = b.ndim - 1; i >= 0; --i) {
      if (b.shape[i] > 1 && b.strides[i] != expect) throw std::invalid_argument(std::string(what) + ": not C-contiguous");
      expect *= b.shape[i];
    }
    if (n != bytes) throw std::invalid_argument(std::string(what) + ": size does not match the pipeline");
  }
  void need(int slot) const {
    if (!exec_[slot]) throw std::runtime_error("FrameRunner: graph slot " + std::to_string(slot) + " not set");
  }

  double spin_us_ = [] {
    const char* e = getenv("RDP_SERVE_SPIN_US");
    return e ? atof(e) : 0.0;
  }();
  bool recorded_ = false;
  bool depth_stream_ = true;
  int H_ = 0, W_ = 0, ns_ = 0;
  void *h_meta_ = nullptr, *h_coef_ = nullptr;
  std::chrono::steady_clock::time_point t0_;
  int dev_;
  hipStream_t s_;
  hipEvent_t ev0_ = nullptr, ev1_ = nullptr, evd_ = nullptr;
  hipStream_t cs_ = nullptr;
  std::vector<void*> host_;
  hipGraphExec_t exec_[4] = {nullptr, nullptr, nullptr, nullptr};
  void *d_color_ = nullptr, *h_color_ = nullptr, *d_depth_ = nullptr, *h_depth_ = nullptr;
  bool kernel_copy_ = true;  // uploads by copy kernel (upload())
  std::vector<std::pair<const void*, void*>> hmap_;  // host staging pointer -> device mapping
  void *d_meta_ = nullptr, *d_coef_ = nullptr, *d_mask_ = nullptr, *h_mask_ = nullptr;
  void *d_res_ = nullptr, *h_res_ = nullptr;
  size_t color_bytes_ = 0, depth_bytes_ = 0, meta_bytes_ = 0, coef_cap_ = 0, mask_bytes_ = 0, res_bytes_ = 0;
};

// ---- batched frames across streams ----------------------------------------------------------------------
// BatchRunner: the host side of serve/engine.py BatchEngine. Frames of several client streams are gathered
// into a batch of n <= P positions and run as ONE captured graph -- the U-Net at batch n (the network costs
// 0.379 / 0.476 / 0.700 ms at n = 1 / 2 / 4, so four frames need 46 % of the GPU time of four n = 1
// frames) plus every frame's geometry -- instead of n graphs that time-slice the GPU. K batch frames
// rotate (one open for new frames, the others in flight or being collected); each (frame k, position j)
// owns its pinned staging and the host memory its results land in, the device inputs belong to position
// j (uploads are stream-ordered after the previous batch's graph). Everything here runs without the GIL:
// decoding a request into its position, the batch's uploads (one multi-segment copy kernel) and graph
// launch, the wait and the response encoding.
class BatchRunner {
 public:
  BatchRunner(int device, uintptr_t stream, int frames, int positions, int H, int W, int num_samples, int src,
              size_t coef_cap, size_t res_doubles)
      : dev_(device), s_((hipStream_t)stream), K_(frames), P_(positions), H_(H), W_(W), ns_(num_samples), src_(src),
        coef_cap_(coef_cap), res_len_(res_doubles) {
    if (K_ < 1 || P_ < 1 || P_ > 4 || src_ < 0 || src_ > 2) throw std::invalid_argument("BatchRunner: frames / positions / src");
    DeviceScope g(dev_);
    ev0_.resize(K_);
    ev1_.resize(K_);
    evup_.resize(K_);
    for (int k = 0; k < K_; ++k) {
      hip_check(hipEventCreate(&ev0_[k]), "hipEventCreate");
      hip_check(hipEventCreate(&ev1_[k]), "hipEventCreate");
      hip_check(hipEventCreateWithFlags(&evup_[k], hipEventDisableTiming | hipEventDisableSystemFence), "hipEventCreate");
    }
    // uploads run on the copy engine, on a stream of their own: batch k + 1's frames cross PCIe while batch
    // k computes (131 us of a 4-frame batch as a copy kernel in front of its graph; profiles/serve_batch.md)
    hip_check(hipStreamCreateWithFlags(&cs_, hipStreamNonBlocking), "hipStreamCreate");
    const size_t npos = (size_t)K_ * P_;
    slots_.resize(npos);
    for (auto& sl : slots_) {
      if (src_ == 2) {
        sl.color = pinned(coef_cap_ ? coef_cap_ : 16);
        sl.meta = pinned(224 * 4);
      } else {
        sl.color = pinned((size_t)H_ * W_ * 3);
      }
      sl.depth = pinned((size_t)H_ * W_ * 2);
      sl.mask = coherent((size_t)H_ * W_);
      sl.res = coherent(res_len_ * 8);
    }
    dcol_.assign(npos, nullptr);
    dmeta_.assign(npos, nullptr);
    ddep_.assign(npos, nullptr);
    exec_.assign((size_t)K_ * (P_ + 1), nullptr);
    fs_.assign(K_, s_);  // every batch frame on the engine's stream unless set_frame_stream says otherwise
    spin_us_ = getenv("RDP_SERVE_SPIN_US") ? atof(getenv("RDP_SERVE_SPIN_US")) : 1000.0;
  }
  ~BatchRunner() {
    for (auto e : ev0_) (void)hipEventDestroy(e);
    for (auto e : ev1_) (void)hipEventDestroy(e);
    for (auto e : evup_) (void)hipEventDestroy(e);
    if (cs_) (void)hipStreamDestroy(cs_);
    for (void* p : pinned_) (void)hipHostFree(p);
  }
  // host buffers of (k, j): 0 colour (arrays) / JPEG coefficients, 1 JPEG meta, 2 depth, 3 mask, 4 result
  uintptr_t host_ptr(int kind, int k, int j) {
    Slot& sl = slot(k, j);
    void* p = kind == 0 ? sl.color : kind == 1 ? sl.meta : kind == 2 ? sl.depth : kind == 3 ? sl.mask : kind == 4 ? sl.res
                                                                                                        : nullptr;
    if (!p) throw std::invalid_argument("BatchRunner.host_ptr: kind");
    return (uintptr_t)p;
  }
  // device inputs of (k, j) (the captured graphs of frame k read them): per batch frame, so that frame
  // k + 1's uploads never wait for frame k's graph
  void set_device(int k, int j, uintptr_t color, uintptr_t meta, uintptr_t depth) {
    slot(k, j);
    const size_t i = (size_t)k * P_ + j;
    dcol_[i] = P(color);
    dmeta_[i] = P(meta);
    ddep_[i] = P(depth);
  }
  void set_upload_kernel(bool on) { upload_kernel_ = on; }
  // the stream batch frame k runs on (BatchEngine lanes: frames of different lanes run concurrently)
  void set_frame_stream(int k, uintptr_t stream) {
    if (k < 0 || k >= K_) throw std::invalid_argument("BatchRunner.set_frame_stream");
    fs_[k] = (hipStream_t)stream;
  }
  void set_graph(int k, int n, uintptr_t exec) {
    if (k < 0 || k >= K_ || n < 1 || n > P_) throw std::invalid_argument("BatchRunner.set_graph");
    exec_[(size_t)k * (P_ + 1) + n] = (hipGraphExec_t)exec;
  }
  void set_spin_us(double us) { spin_us_ = us; }

  // a request's colour JPEG + 16-bit depth PNG decoded into (k, j): 0 ok, 1 not a frame this path takes,
  // 2 other frame size, 3 corrupt
  int decode(int k, int j, py::bytes color, py::bytes depth) {
    if (src_ != 2) throw std::runtime_error("BatchRunner.decode: not a JPEG batch runner");
    char *cp = nullptr, *dp = nullptr;
    Py_ssize_t cn = 0, dn = 0;
    if (PyBytes_AsStringAndSize(color.ptr(), &cp, &cn) != 0 || PyBytes_AsStringAndSize(depth.ptr(), &dp, &dn) != 0)
      throw py::error_already_set();
    slot(k, j);
    py::gil_scoped_release nogil;
    return decode_ptr(k, j, (const uint8_t*)cp, (long)cn, (const uint8_t*)dp, (long)dn);
  }

  // the whole serialized AnalysisRequest, parsed here (FrameRunner.submit_request)
  int decode_request(int k, int j, py::bytes raw) {
    if (src_ != 2) throw std::runtime_error("BatchRunner.decode_request: not a JPEG batch runner");
    char* rp = nullptr;
    Py_ssize_t rn = 0;
    if (PyBytes_AsStringAndSize(raw.ptr(), &rp, &rn) != 0) throw py::error_already_set();
    slot(k, j);
    py::gil_scoped_release nogil;
    const uint8_t *c, *d;
    size_t cn, dn;
    if (!parse_request((const uint8_t*)rp, (size_t)rn, c, cn, d, dn)) return 1;
    return decode_ptr(k, j, c, (long)cn, d, (long)dn);
  }

  int decode_ptr(int k, int j, const uint8_t* c, long cn, const uint8_t* d, long dn) {  // GIL released
    Slot& sl = slot(k, j);
    sl.t0 = std::chrono::steady_clock::now();
    int hi[24];
    const long nco = rdp_jpeg_info(c, (long)cn, hi);
    if (nco == -1) return 3;
    if (nco <= 0) return 1;
    int pw = 0, ph = 0, bd = 0;
    if (rdp_png_info(d, (long)dn, &pw, &ph, &bd) != 0 || bd != 16) return 1;
    if (hi[0] != W_ || hi[1] != H_ || pw != W_ || ph != H_) return 2;
    if ((size_t)nco * 2 > coef_cap_) return 1;
    int rc[2] = {0, 0};
    rdp::host_pool().parallel_for(2, [&](int h) {
      if (h == 0) {
        int* meta = (int*)sl.meta;
        rdp_jpeg_meta(hi, meta);
        uint16_t qt[3 * 64];
        if (rdp_jpeg_decode(c, (long)cn, (int16_t*)sl.color, nco, qt, 1) != 0) {
          rc[0] = 3;
          return;
        }
        for (int i = 0; i < 3 * 64; ++i) meta[32 + i] = qt[i];
      } else if (rdp_png_decode(d, (long)dn, (uint8_t*)sl.depth, (long)H_ * W_ * 2, 1) != 0) {
        rc[1] = 3;
      }
    });
    if (rc[0] || rc[1]) return 3;
    sl.bytes = (size_t)nco * 2;
    return 0;
  }

  // (arrays source) an HxWx3 u8 colour frame and HxW 16-bit depth frame staged into (k, j)
  void stage(int k, int j, py::buffer color, py::buffer depth) {
    if (src_ == 2) throw std::runtime_error("BatchRunner.stage: a JPEG batch runner");
    py::buffer_info c = color.request(), d = depth.request();
    contig(c, (size_t)H_ * W_ * 3, "colour");
    contig(d, (size_t)H_ * W_ * 2, "depth");
    Slot& sl = slot(k, j);
    const void *cp = c.ptr, *dp = d.ptr;
    py::gil_scoped_release nogil;
    sl.t0 = std::chrono::steady_clock::now();
    std::memcpy(sl.color, cp, (size_t)H_ * W_ * 3);
    std::memcpy(sl.depth, dp, (size_t)H_ * W_ * 2);
    sl.bytes = (size_t)H_ * W_ * 3;
  }

  // batch frame k with its first n positions: every upload in one copy kernel, the graph, the end event
  void launch(int k, int n) {
    if (k < 0 || k >= K_ || n < 1 || n > P_) throw std::invalid_argument("BatchRunner.launch");
    hipGraphExec_t ex = exec_[(size_t)k * (P_ + 1) + n];
    if (!ex) throw std::runtime_error("BatchRunner: graph (" + std::to_string(k) + ", " + std::to_string(n) + ") not set");
    py::gil_scoped_release nogil;
    DeviceScope g(dev_);
    const void* src[16];
    void* dst[16];
    long bytes[16];
    int m = 0;
    for (int j = 0; j < n; ++j) {
      Slot& sl = slot(k, j);
      const size_t i = (size_t)k * P_ + j;
      src[m] = sl.color; dst[m] = dcol_[i]; bytes[m++] = (long)sl.bytes;
      if (src_ == 2) { src[m] = sl.meta; dst[m] = dmeta_[i]; bytes[m++] = 224 * 4; }
      src[m] = sl.depth; dst[m] = ddep_[i]; bytes[m++] = (long)H_ * W_ * 2;
    }
    const hipStream_t fs = fs_[k];
    if (upload_kernel_) {  // one copy kernel on the frame's stream, in front of the graph
      hip_check(hipEventRecord(ev0_[k], fs), "hipEventRecord");
      for (int i = 0; i < m; ++i) src[i] = devptr(const_cast<void*>(src[i]));
      if (rdp_h2d_copy_multi(src, dst, bytes, m, fs) != 0) {
        (void)hipGetLastError();
        throw std::runtime_error("BatchRunner: upload kernel rejected the segments");
      }
    } else {  // DMA on the copy stream; the frame stream waits for it (GPU-side)
      hip_check(hipEventRecord(ev0_[k], cs_), "hipEventRecord");
      for (int i = 0; i < m; ++i)
        hip_check(hipMemcpyAsync(dst[i], src[i], (size_t)bytes[i], hipMemcpyHostToDevice, cs_), "H2D batch");
      hip_check(hipEventRecord(evup_[k], cs_), "hipEventRecord");
      hip_check(hipStreamWaitEvent(fs, evup_[k], 0), "hipStreamWaitEvent");
    }
    hip_check(hipGraphLaunch(ex, fs), "hipGraphLaunch");
    hip_check(hipEventRecord(ev1_[k], fs), "hipEventRecord");
  }

  // block until batch k's results are on the host; its device time (ms)
  float wait(int k) {
    py::gil_scoped_release nogil;
    DeviceScope g(dev_);
    return sync(k);
  }

  // (payload, mean, max, coverage %, status, gpu ms) of (k, j) after its batch ran (status 4: host fit needed)
  py::tuple collect_encoded(int k, int j, int level, int bands) {
    float gpu_ms = 0.f;
    double mean = 0, maxc = 0, cov = 0;
    int st = 0;
    std::string out;
    {
      py::gil_scoped_release nogil;
      DeviceScope g(dev_);
      gpu_ms = sync(k);
      Slot& sl = slot(k, j);
      const double* r = (const double*)sl.res;
      st = (int)r[0];
      cov = 100.0 * r[8 + 3 * ns_] / ((double)H_ * W_);
      if (st != 4) {
        static const char* names[4] = {"ok", "too_few_points", "too_few_edge_points", "fit_failed"};
        const std::string status = (st >= 0 && st < 4) ? names[st] : "fit_failed";
        if (st == 0) { mean = r[4]; maxc = r[5]; }
        const float proc = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - sl.t0).count();
        out = encode_wire(mean, maxc, st == 0 ? r + 8 : nullptr, st == 0 ? (size_t)ns_ : 0, status,
                          (const uint8_t*)sl.mask, H_, W_, (float)cov, proc, level, bands);
      }
    }
    return py::make_tuple(py::bytes(out), mean, maxc, cov, st, gpu_ms);
  }

  void drain() {
    py::gil_scoped_release nogil;
    DeviceScope g(dev_);
    hip_check(hipStreamSynchronize(cs_), "hipStreamSynchronize");
    for (auto fs : fs_) hip_check(hipStreamSynchronize(fs), "hipStreamSynchronize");
  }

 private:
  struct Slot {
    void *color = nullptr, *meta = nullptr, *depth = nullptr, *mask = nullptr, *res = nullptr;
    size_t bytes = 0;
    std::chrono::steady_clock::time_point t0;
  };
  Slot& slot(int k, int j) {
    if (k < 0 || k >= K_ || j < 0 || j >= P_) throw std::invalid_argument("BatchRunner: (frame, position)");
    return slots_[(size_t)k * P_ + j];
  }
  float sync(int k) {
    if (k < 0 || k >= K_) throw std::invalid_argument("BatchRunner: frame");
    if (spin_us_ > 0) {
      const auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        const hipError_t q = hipEventQuery(ev1_[k]);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) hip_check(q, "hipEventQuery");
        if (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > spin_us_) {
          hip_check(hipEventSynchronize(ev1_[k]), "hipEventSynchronize");
          break;
        }
      }
    } else {
      hip_check(hipEventSynchronize(ev1_[k]), "hipEventSynchronize");
    }
    float ms = 0.f;
    hip_check(hipEventElapsedTime(&ms, ev0_[k], ev1_[k]), "hipEventElapsedTime");
    return ms;
  }
  void* pinned(size_t bytes) {
    DeviceScope g(dev_);
    void* p = nullptr;
    hip_check(hipHostMalloc(&p, (bytes + 15) / 16 * 16, hipHostMallocDefault), "hipHostMalloc");
    std::memset(p, 0, bytes);
    pinned_.push_back(p);
    return p;
  }
  void* coherent(size_t bytes) {
    DeviceScope g(dev_);
    void* p = nullptr;
    hip_check(hipHostMalloc(&p, (bytes + 15) / 16 * 16, hipHostMallocCoherent | hipHostMallocMapped), "hipHostMalloc");
    std::memset(p, 0, bytes);
    pinned_.push_back(p);
    return p;
  }
  void* devptr(void* host) {  // the device mapping of a pinned buffer (the copy kernel reads through it)
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, host, 0) != hipSuccess) {
      (void)hipGetLastError();
      return host;
    }
    return dp;
  }
  static void contig(const py::buffer_info& b, size_t bytes, const char* what) {
    size_t n = (size_t)b.itemsize;
    for (auto sh : b.shape) n *= (size_t)sh;
    ssize_t expect = b.itemsize;
    for (ssize_t i = b.ndim - 1; i >= 0; --i) {
      if (b.shape[i] > 1 && b.strides[i] != expect) throw std::invalid_argument(std::string(what) + ": not C-contiguous");
      expect *= b.shape[i];
    }
    if (n != bytes) throw std::invalid_argument(std::string(what) + ": size does not match the batch runner");
  }

  int dev_;
  hipStream_t s_;
  int K_, P_, H_, W_, ns_, src_;
  size_t coef_cap_, res_len_;
  double spin_us_ = 1000.0;
  std::vector<hipEvent_t> ev0_, ev1_, evup_;
  hipStream_t cs_ = nullptr;
  std::vector<hipStream_t> fs_;
  bool upload_kernel_ = getenv("RDP_BATCH_UPLOAD") && std::string(getenv("RDP_BATCH_UPLOAD")) == "kernel";
  std::vector<Slot> slots_;
  std::vector<void*> dcol_, dmeta_, ddep_;
  std::vector<hipGraphExec_t> exec_;
  std::vector<void*> pinned_;
};

// ---- protobuf wire format (proto3)
void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}
void put_fixed64(std::string& o, int field, double v) {  // omitted when the bit pattern is zero (proto3)
  uint64_t b;
  std::memcpy(&b, &v, 8);
  if (!b) return;
  put_varint(o, (uint64_t)field << 3 | 1);
  for (int i = 0; i < 8; ++i) o.push_back((char)(b >> (8 * i)));
}
void put_fixed32(std::string& o, int field, float v) {
  uint32_t b;
  std::memcpy(&b, &v, 4);
  if (!b) return;
  put_varint(o, (uint64_t)field << 3 | 5);
  for (int i = 0; i < 4; ++i) o.push_back((char)(b >> (8 * i)));
}
void put_bytes(std::string& o, int field, const char* p, size_t n) {
  if (!n) return;
  put_varint(o, (uint64_t)field << 3 | 2);
  put_varint(o, n);
  o.append(p, n);
}

// AnalysisResponse bytes. mask: HxW u8 {0,1} (PNG-encoded as 0/255, `bands` deflate bands) or None;
// points: [n, 3] float64 or None.
py::bytes encode_response(double mean, double maxc, py::object points, const std::string& status, py::object mask,
                          float coverage, float proc_ms, int level, int bands) {
  std::vector<double> pts;
  if (!points.is_none()) {
    auto a = py::array_t<double, py::array::c_style | py::array::forcecast>::ensure(points);
    if (!a || (a.size() && (a.ndim() != 2 || a.shape(1) != 3))) throw std::invalid_argument("points: [n, 3]");
    pts.assign(a.data(), a.data() + a.size());
  }
  std::vector<uint8_t> img;
  int h = 0, w = 0;
  if (!mask.is_none()) {
    auto m = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>::ensure(mask);
    if (!m || m.ndim() != 2) throw std::invalid_argument("mask: HxW u8");
    h = (int)m.shape(0);
    w = (int)m.shape(1);
    img.assign(m.data(), m.data() + m.size());
  }
  std::string out;
  {
    py::gil_scoped_release nogil;
    out = encode_wire(mean, maxc, pts.data(), pts.size() / 3, status, h > 0 && w > 0 ? img.data() : nullptr, h, w,
                      coverage, proc_ms, level, bands);
  }
  return py::bytes(out);
}

// AnalysisResponse wire bytes (no Python objects: callable without the GIL). mask01: HxW u8 {0, 1}
// (PNG-encoded as 0 / 255) or nullptr; pts: npts x 3 doubles.
std::string encode_wire(double mean, double maxc, const double* pts, size_t npts, const std::string& status,
                        const uint8_t* mask01, int h, int w, float coverage, float proc_ms, int level, int bands) {
  std::string png;
  if (mask01 && h > 0 && w > 0) {
    std::vector<uint8_t> img((size_t)h * w);
    for (size_t i = 0; i < img.size(); ++i) img[i] = mask01[i] ? 255 : 0;
    png.resize((size_t)rdp_png_encode_bound(w, h, 1, bands));
    const long n = rdp_png_encode_gray(img.data(), w, h, 1, level, bands, (uint8_t*)&png[0], (long)png.size());
    if (n < 0) throw std::runtime_error("mask PNG encode failed");
    png.resize((size_t)n);
  }
  std::string out;
  out.reserve(png.size() + status.size() + npts * 30 + 64);
  put_fixed64(out, 1, mean);
  put_fixed64(out, 2, maxc);
  std::string sub;
  for (size_t i = 0; i < npts; ++i) {
    sub.clear();
    put_fixed64(sub, 1, pts[3 * i]);
    put_fixed64(sub, 2, pts[3 * i + 1]);
    put_fixed64(sub, 3, pts[3 * i + 2]);
    put_varint(out, 3 << 3 | 2);  // repeated Point3D: always present, even when empty
    put_varint(out, sub.size());
    out += sub;
  }
  put_bytes(out, 4, status.data(), status.size());
  put_bytes(out, 5, png.data(), png.size());
  put_fixed32(out, 6, coverage);
  put_fixed32(out, 7, proc_ms);
  return out;
}

}  // namespace

void register_serve_runtime(py::module_& m) {
  py::class_<FrameRunner>(m, "FrameRunner")
      .def(py::init<int, uintptr_t>(), py::arg("device"), py::arg("stream"))
      .def("set_graph", &FrameRunner::set_graph)
      .def("set_buffers", &FrameRunner::set_buffers)
      .def("alloc_host", &FrameRunner::alloc_host)
      .def("set_depth_stream", [](FrameRunner& r, bool on) { r.depth_stream(on); },
           "depth H2D on the copy stream (default) or in order on the frame stream")
      .def("submit_array", &FrameRunner::submit_array)
      .def("submit_jpeg", &FrameRunner::submit_jpeg)
      .def("submit_depth", &FrameRunner::submit_depth)
      .def("configure_encoded", &FrameRunner::configure_encoded, py::arg("H"), py::arg("W"), py::arg("num_samples"))
      .def("submit_encoded", &FrameRunner::submit_encoded, py::arg("color"), py::arg("depth"),
           "0 launched, 1 not a native frame, 2 other frame size, 3 corrupt (nothing in flight)")
      .def("submit_request", &FrameRunner::submit_request, py::arg("raw"),
           "a serialized AnalysisRequest: codes as submit_encoded")
      .def("collect_encoded", &FrameRunner::collect_encoded, py::arg("level") = 1, py::arg("bands") = 4)
      .def("abort", &FrameRunner::abort)
      .def("set_spin_us", &FrameRunner::set_spin_us, py::arg("us"),
           "poll the frame's end event for up to `us` microseconds before blocking")
      .def("wait", &FrameRunner::wait);
  py::class_<BatchRunner>(m, "BatchRunner")
      .def(py::init<int, uintptr_t, int, int, int, int, int, int, size_t, size_t>(), py::arg("device"),
           py::arg("stream"), py::arg("frames"), py::arg("positions"), py::arg("H"), py::arg("W"),
           py::arg("num_samples"), py::arg("src"), py::arg("coef_cap"), py::arg("res_doubles"))
      .def("host_ptr", &BatchRunner::host_ptr)
      .def("set_device", &BatchRunner::set_device)
      .def("set_graph", &BatchRunner::set_graph)
      .def("set_spin_us", &BatchRunner::set_spin_us)
      .def("set_upload_kernel", &BatchRunner::set_upload_kernel)
      .def("set_frame_stream", &BatchRunner::set_frame_stream)
      .def("decode", &BatchRunner::decode, "0 ok, 1 not a native frame, 2 other frame size, 3 corrupt")
      .def("decode_request", &BatchRunner::decode_request)
      .def("stage", &BatchRunner::stage)
      .def("launch", &BatchRunner::launch)
      .def("wait", &BatchRunner::wait)
      .def("collect_encoded", &BatchRunner::collect_encoded, py::arg("k"), py::arg("j"), py::arg("level") = 1,
           py::arg("bands") = 4)
      .def("drain", &BatchRunner::drain);
  m.def("parse_request", [](py::bytes raw) -> py::object {  // (colour bytes, depth bytes) or None (tests)
    char* rp = nullptr;
    Py_ssize_t rn = 0;
    if (PyBytes_AsStringAndSize(raw.ptr(), &rp, &rn) != 0) throw py::error_already_set();
    const uint8_t *c, *d;
    size_t cn, dn;
    if (!parse_request((const uint8_t*)rp, (size_t)rn, c, cn, d, dn)) return py::none();
    return py::make_tuple(py::bytes((const char*)c, cn), py::bytes((const char*)d, dn));
  });
  m.def("encode_response", &encode_response, py::arg("mean"), py::arg("max"), py::arg("points"), py::arg("status"),
        py::arg("mask"), py::arg("coverage"), py::arg("proc_ms"), py::arg("level") = 1, py::arg("bands") = 4);
}
