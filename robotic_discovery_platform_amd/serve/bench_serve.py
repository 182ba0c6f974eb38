"""Serving benchmark: e2e frames/s + p50/p99 latency (second half of the BASELINE.json metric).

Two measurements on 640x480 synthetic RGB-D frames (the reference camera format, pkg/camera.py:35):
  * engine:  ``FramePipeline.process`` per frame (H2D, hipGraph replay of preprocess + U-Net +
             mask + geometry kernels, D2H, host spline fit) -- the per-frame work of
             server.py:117-133 without codecs/transport.
  * e2e:     the full gRPC service over loopback (client-encoded JPEG colour + 16-bit PNG depth,
             server decode, engine, PNG mask encode, metrics CSV, response) -- one stream, streamed
             (throughput FPS) and lock-step (round-trip p50/p99); the load generator runs in its own
             process like the reference's client.py.

Weights: the reference U-Net architecture, briefly trained on synthetic scenes (so masks look like
an actuator and the geometry stage sees realistic point counts), unless ``train_steps=0``.
"""
from __future__ import annotations

import os
import sys
import queue
import tempfile
import threading
import time
from typing import Optional

import numpy as np
import torch


def _pct(v, q):
    return float(np.percentile(np.asarray(v), q)) if len(v) else float("nan")


def _freeze():
    """gc.freeze() once the long-lived objects exist, as the server does (server.freeze_heap)."""
    import gc
    gc.collect()
    gc.freeze()


def slow_frames(lat, parts: dict) -> dict:
    """Frames slower than 2x the median and, per frame, the part (of ``parts``: name -> per-frame ms) that
    exceeded its own median by the most: {"count": n, "<part>": frames, ...}."""
    lat = np.asarray(lat)
    med = {k: float(np.median(v)) for k, v in parts.items()}
    out = {"count": 0}
    for i in np.nonzero(lat > 2 * np.median(lat))[0]:
        k = max(parts, key=lambda k: parts[k][i] - med[k])
        out[k] = out.get(k, 0) + 1
        out["count"] += 1
    return out


def prepare_model(dev, train_steps: int = 200, batch: int = 16, n_scenes: int = 48, seed: int = 0):
    from ..data.image_io import bgr2rgb, resize_area, resize_nearest
    from ..data.synthetic import make_scene
    from ..models.unet import UNetNative
    from ..train.engine import NativeTrainer
    torch.manual_seed(seed)
    scenes = [make_scene(seed + i) for i in range(n_scenes)]
    model = UNetNative(3, 1, device=dev)
    if train_steps > 0:
        x = np.stack([resize_area(bgr2rgb(s.color), (256, 256)) for s in scenes]).astype(np.float32) / 255
        y = np.stack([resize_nearest(s.mask, (256, 256)) for s in scenes]).astype(np.float32) / 255
        X = torch.from_numpy(x).permute(0, 3, 1, 2).contiguous().to(dev)
        Y = torch.from_numpy(y)[:, None].contiguous().to(dev)
        tr = NativeTrainer(model, batch, 256, 256, lr=1e-3, graph=True)
        g = torch.Generator(device="cpu").manual_seed(seed)
        for _ in range(train_steps):
            idx = torch.randint(0, n_scenes, (batch,), generator=g).to(dev)
            tr.set_batch(X[idx], Y[idx])
            tr.step()
        torch.cuda.synchronize(dev)
    return model.eval(), scenes


def measure_engine(model, scenes, frames: int = 200, warmup: int = 20):
    from ..data.synthetic import DEFAULT_K
    from .engine import FramePipeline
    p = FramePipeline(model, DEFAULT_K, 0.001, graph=True)
    lat, gpu, fit = [], [], []
    ok = 0
    for i in range(warmup + frames):
        s = scenes[i % len(scenes)]
        if i == warmup:
            _freeze()
        t0 = time.perf_counter()
        r = p.process(s.color, s.depth)
        dt = (time.perf_counter() - t0) * 1e3
        if i >= warmup:
            lat.append(dt)
            gpu.append(r.timings["gpu_ms"])
            fit.append(r.timings["fit_ms"])
            ok += r.curvature.status == "ok"
    host = [a - b - c for a, b, c in zip(lat, gpu, fit)]
    out = {"engine_fps": round(1e3 * len(lat) / sum(lat), 1), "engine_p50_ms": round(_pct(lat, 50), 3),
           "engine_p99_ms": round(_pct(lat, 99), 3), "engine_gpu_p50_ms": round(_pct(gpu, 50), 3),
           "engine_gpu_p99_ms": round(_pct(gpu, 99), 3), "engine_frames": len(lat),
           "engine_fit_p50_ms": round(_pct(fit, 50), 3), "engine_ok_frac": ok / max(1, len(lat)),
           "engine_slow_frames": slow_frames(lat, {"gpu": gpu, "fit": fit, "host": host})}
    out.update(measure_engine_pipelined(model, scenes, frames, warmup))
    return out


def measure_engine_pipelined(model, scenes, frames: int = 200, warmup: int = 20, streams: int = 1):
    """Frames back to back through double-buffered stream sessions (EnginePool.session): frame i+1's
    H2D + graph overlap frame i's tail. ``streams`` concurrent sessions share the GPU."""
    from ..data.synthetic import DEFAULT_K
    from .engine import EnginePool
    pool = EnginePool(model, DEFAULT_K, 0.001, n=2 * streams, graph=True)
    res = {}

    def run(k):
        s = pool.session()
        for i in range(warmup):
            sc = scenes[i % len(scenes)]
            s.submit(sc.color, sc.depth, tag=i)
        s.drain()
        t0 = time.perf_counter()
        for i in range(frames):
            sc = scenes[i % len(scenes)]
            s.submit(sc.color, sc.depth, tag=i)
        s.drain()
        res[k] = time.perf_counter() - t0

    ths = [threading.Thread(target=run, args=(k,)) for k in range(streams)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    sfx = '' if streams == 1 else f'_{streams}streams'
    out = {f"engine_pipelined_fps{sfx}": round(frames * streams / max(res.values()), 1)}
    if streams > 1 and getattr(pool, "batchers", None):  # batched serving: how the frames were grouped
        out[f"engine_batch_sizes{sfx}"] = {str(k): v for k, v in sorted(pool.batchers[0].batch_sizes.items())}
        for b in pool.batchers:
            b.close()
    return out


def run_client_load(port: int, frames: int, warmup: int, n_scenes: int = 8, lockstep: bool = True,
                    go=None) -> dict:
    """The load generator: one client stream (the reference client's encodings: JPEG colour, 16-bit
    PNG depth), streamed throughput then (``lockstep``) lock-step round trips. Runs in its own
    process; ``go()`` (if given) blocks until every stream of a multi-stream run is ready."""
    import grpc
    from ..data.synthetic import make_scene
    from ..proto import vision as pb
    from .client import make_request
    reqs = [make_request(sc.color, sc.depth) for sc in (make_scene(i) for i in range(n_scenes))]
    _freeze()
    if go is not None:
        go()
    out = {}
    with grpc.insecure_channel(f"127.0.0.1:{port}", options=[("grpc.max_receive_message_length", 64 << 20),
                                                               ("grpc.max_send_message_length", 64 << 20)]) as ch:
        stub = pb.VisionAnalysisServiceStub(ch)
        n = warmup + frames

        def gen():
            for i in range(n):
                yield reqs[i % len(reqs)]

        t_start = None
        proc = []
        for i, resp in enumerate(stub.AnalyzeActuatorPerformance(gen())):
            if i == warmup - 1:
                t_start = time.perf_counter()
            if i >= warmup:
                proc.append(resp.proc_time_ms)
        t_end = time.perf_counter()
        out["e2e_fps"] = round(frames / (t_end - t_start), 1)
        out["e2e_server_proc_p50_ms"] = round(_pct(proc, 50), 3)  # processing only (proc_time_ms)
        if not lockstep:
            return out
        q: "queue.Queue" = queue.Queue()
        sent = []

        def gen_ls():
            for i in range(n):
                sent.append(time.perf_counter())
                yield reqs[i % len(reqs)]
                q.get()

        rtt, sproc = [], []
        for i, resp in enumerate(stub.AnalyzeActuatorPerformance(gen_ls())):
            now = time.perf_counter()
            if i >= warmup:
                rtt.append((now - sent[i]) * 1e3)
                sproc.append(resp.proc_time_ms)
            q.put(1)
        out["e2e_p50_ms"] = round(_pct(rtt, 50), 3)
        out["e2e_p99_ms"] = round(_pct(rtt, 99), 3)
        out["e2e_p999_ms"] = round(_pct(rtt, 99.9), 3)
        out["e2e_lockstep_frames"] = len(rtt)
        # each slow round trip: the server's processing (the response's proc_time_ms) or everything
        # around it (transport, gRPC threads, the client)
        out["e2e_slow_frames"] = slow_frames(rtt, {"server_proc": sproc,
                                                   "transport": [a - b for a, b in zip(rtt, sproc)]})
    return out


class NullPipeline:
    """Host-path stand-in for a frame pipeline: accepts a frame, returns a fixed result (a 640x480
    mask with an actuator-sized blob and a 50-point spline). With it the e2e bench measures the server's
    host machinery alone -- gRPC, codecs, threads, GIL -- on any machine (``measure_e2e(model=None)``)."""

    def __init__(self, H=480, W=640):
        from ..geometry.curvature import CurvatureResult, Point
        from .engine import FrameResult
        m = np.zeros((H, W), np.uint8)
        m[H // 4: 3 * H // 4, W // 3: 2 * W // 3] = 1
        pts = [Point(float(i), float(i) * 0.5, 0.4) for i in range(50)]
        self._res = FrameResult(m, 100.0 * m.mean(), CurvatureResult(0.01, 0.02, pts, "ok", 1000, 100))
        self._n = 0

    def submit(self, color, depth, rgb=False):
        self._n += 1

    def submit_color(self, color, rgb=False):
        pass

    def submit_depth(self, depth):
        self._n += 1

    def abort(self):
        pass

    def collect(self):
        return self._res

    def wait_idle(self):
        pass

    def refresh_weights(self):
        pass


class NullEngine:
    """EnginePool interface over NullPipelines (see NullPipeline)."""

    def __init__(self, n: int = 2, jpeg: bool = True):
        from . import engine as E
        self._E = E
        self.jpeg, self.gpu, self.n = jpeg, False, n
        self._pools = {}
        self._lock = threading.Lock()

    def _get(self, r, H, W):
        with self._lock:
            q = self._pools.get((H, W))
            if q is None:
                q = queue.Queue()
                for _ in range(self.n):
                    q.put(NullPipeline(H, W))
                self._pools[(H, W)] = q
            return q

    def session(self):
        return self._E.EngineSession(self, 0)

    def process(self, color, depth):
        return NullPipeline(*depth.shape[:2]).collect()


def _client_env():
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    return dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""),
                HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")  # the client never touches the GPU


def _run_clients(ports, frames, warmup, lockstep, env=None) -> list:
    """One load-generator process per entry of ``ports`` (stream k -> ports[k]), started together."""
    import json
    import subprocess
    env = env or _client_env()
    procs = [subprocess.Popen([sys.executable, "-m", "robotic_discovery_platform_amd.serve.bench_serve",
                               "--client-port", str(pt), "--frames", str(frames), "--warmup", str(warmup),
                               "--lockstep", str(int(lockstep))],
                              env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for pt in ports]
    try:
        for p in procs:  # every client has built its requests: start them together
            if p.stdout.readline().strip() != "ready":
                raise RuntimeError(f"client process failed: {p.stderr.read()[-1500:]}")
        for p in procs:
            p.stdin.write("go\n")
            p.stdin.flush()
        res = []
        for p in procs:
            so, se = p.communicate(timeout=600)
            if p.returncode != 0:
                raise RuntimeError(f"client process failed: {se[-1500:]}")
            res.append(json.loads(so.strip().splitlines()[-1]))
        return res
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()


def measure_e2e_procs(model, frames: int = 200, warmup: int = 20, procs: int = 2, streams: int = 4,
                      hw_queues: int = 0) -> dict:
    """``ServeConfig.workers`` topology: ``procs`` server processes on one GPU (each its own engine replica
    and interpreter lock), ``streams`` client streams spread round-robin over them. Aggregate frames/s
    = the sum of the streams' rates."""
    import json
    import subprocess
    tmp = tempfile.mkdtemp(prefix="rdp_serve_procs_")
    wpath = os.path.join(tmp, "weights.pt")
    torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()}, wpath)
    env = dict(_client_env(), HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""),
               CUDA_VISIBLE_DEVICES=os.environ.get("CUDA_VISIBLE_DEVICES", ""))
    for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if not env[k]:
            env.pop(k)
    if hw_queues > 0:  # hardware queues per server process (HIP default 4)
        env["GPU_MAX_HW_QUEUES"] = str(hw_queues)
    env.setdefault("RDP_SERVE_READER_SUBMIT", "0")  # as ServeConfig.workers > 1 sets it (serve/server.py)
    per = max(1, -(-streams // procs))
    servers = [subprocess.Popen([sys.executable, "-m", "robotic_discovery_platform_amd.serve.bench_serve",
                                 "--server-child", wpath, "--pool", str(2 * per)],
                                env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                text=True) for _ in range(procs)]
    out = {}
    try:
        ports = []
        for p in servers:
            line = p.stdout.readline().strip()
            if not line.startswith("port "):
                raise RuntimeError(f"server process failed: {p.stderr.read()[-1500:]}")
            ports.append(int(line.split()[1]))
        res = _run_clients([ports[k % procs] for k in range(streams)], frames, warmup, lockstep=False)
        sfx = f"_{streams}streams_{procs}procs" + (f"_{hw_queues}hwq" if hw_queues else "")
        out["e2e_fps" + sfx] = round(sum(r["e2e_fps"] for r in res), 1)
        out["e2e_server_proc_p50_ms" + sfx] = round(float(np.median([r["e2e_server_proc_p50_ms"] for r in res])), 3)
        stats = []
        for p in servers:
            so, _ = p.communicate("", timeout=120)
            stats.append(json.loads(so.strip().splitlines()[-1]))
        for k in ("submit", "decode_color", "decode_depth", "gpu", "respond"):
            v = float(np.median([st[f"{k}_p50_ms"] for st in stats]))
            if v == v:  # stages a path does not have (native frames: no separate decode / respond) stay out
                out[f"e2e_stage_{k}_p50_ms" + sfx] = round(v, 3)
        _progress(f"e2e procs: {out}")
    finally:
        for p in servers:
            if p.poll() is None:
                p.kill()
    return out


def _server_child(wpath: str, pool: int) -> None:
    """``--server-child``: one server process of ``measure_e2e_procs``; prints its port, serves until
    stdin closes, then prints its latency stats."""
    import json
    import grpc
    from concurrent import futures
    from ..data.synthetic import DEFAULT_K
    from ..models.unet import UNetNative
    from ..proto import vision as pb
    from .engine import EnginePool
    from .server import VisionAnalysisService
    dev = torch.device("cuda")
    model = UNetNative(3, 1, device=dev)
    model.load_state_dict(torch.load(wpath, map_location="cpu", weights_only=True))
    model.eval()
    engine = EnginePool(model, DEFAULT_K, 0.001, n=pool, graph=True, rgb=True, jpeg=True)
    svc = VisionAnalysisService(engine, None)
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=10))
    pb.add_VisionAnalysisServiceServicer_to_server(svc, server)
    port = server.add_insecure_port("127.0.0.1:0")
    server.start()
    _freeze()
    print(f"port {port}", flush=True)
    sys.stdin.read()
    server.stop(0).wait()
    svc.close()
    print(json.dumps(svc.latency_stats()), flush=True)


def measure_e2e(model, scenes, frames: int = 200, warmup: int = 20, pool: int = 2, gpu_jpeg: bool = True,
                streams: int = 1, switch_ms: float = 0.0):
    """Server in this process, load generator(s) in separate client processes (the reference's
    topology: client.py and server.py are different processes), over loopback gRPC. ``gpu_jpeg``:
    the server's JPEG path (native entropy decode + GPU pixel stage, as ``build_server``) or the host
    PIL decode. ``streams`` > 1: that many concurrent client streams (processes started together),
    aggregate frames/s = the sum of the streams' rates."""
    import grpc
    import json
    import subprocess
    import sys
    from ..data.synthetic import DEFAULT_K
    from ..proto import vision as pb
    from .engine import EnginePool
    from .server import MetricsLog, VisionAnalysisService
    from concurrent import futures
    tmp = tempfile.mkdtemp(prefix="rdp_serve_")
    old_switch = sys.getswitchinterval()
    if switch_ms > 0:
        sys.setswitchinterval(switch_ms * 1e-3)
    if model is None:  # host path only
        engine = NullEngine(n=max(pool, 2 * streams), jpeg=gpu_jpeg)
    else:
        engine = EnginePool(model, DEFAULT_K, 0.001, n=max(pool, 2 * streams), graph=True, rgb=True, jpeg=gpu_jpeg)
    svc = VisionAnalysisService(engine, MetricsLog(os.path.join(tmp, "metrics.csv")))
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max(10, 2 * streams)))
    pb.add_VisionAnalysisServiceServicer_to_server(svc, server)
    port = server.add_insecure_port("127.0.0.1:0")
    server.start()
    _freeze()  # as build_server does
    out = {}
    sfx = "" if streams == 1 else f"_{streams}streams"
    try:
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""),
                   HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")  # the client never touches the GPU
        res = _run_clients([port] * streams, frames, warmup, lockstep=streams == 1, env=env)
        if streams == 1:
            out.update(res[0])
        else:
            out["e2e_fps" + sfx] = round(sum(r["e2e_fps"] for r in res), 1)
            out["e2e_server_proc_p50_ms" + sfx] = round(float(np.median([r["e2e_server_proc_p50_ms"] for r in res])), 3)
        st = svc.latency_stats()
        out["e2e_server_queue_p50_ms" + sfx] = round(st["queue_p50_ms"], 3)  # request read -> processing start
        for k in ("decode_color", "decode_depth", "submit", "gpu", "respond", "hold"):  # server stages
            for q in ("p50", "p99"):
                v = st[f"{k}_{q}_ms"]
                if v == v:
                    out[f"e2e_stage_{k}_{q}_ms" + sfx] = round(v, 3)
        if streams == 1:
            out["e2e_client"] = "separate process"
        if not gpu_jpeg:
            out = {k.replace("e2e_", "e2e_hostjpeg_"): v for k, v in out.items() if k != "e2e_client"}
        _progress(f"e2e: {out}")
    finally:
        # wait for the gRPC core to finish shutting down before its objects are collected: a
        # server torn down at interpreter exit aborts the process ("terminate called without an
        # active exception") after the results were printed
        server.stop(0).wait()
        svc.close()
        del server
        sys.setswitchinterval(old_switch)
    return out


def _progress(msg):
    import sys
    print(f"[bench_serve] {msg}", file=sys.stderr, flush=True)


def measure_serving(dev: Optional[torch.device] = None, frames: int = 2000, warmup: int = 50,
                    train_steps: int = 200, e2e: bool = True, multi: bool = True) -> dict:
    dev = dev or torch.device("cuda")
    model, scenes = prepare_model(dev, train_steps)
    _progress("model ready")
    res = {"serve_frame": "640x480 RGB-D -> 256x256 U-Net", "serve_weights": f"trained {train_steps} steps on synthetic"}
    res.update({"serve_" + k: v for k, v in measure_engine(model, scenes, frames, warmup).items()})
    _progress(f"engine done: {res}")
    if multi:  # (rocprofv3 kernel tracing crashes on frames submitted from several threads: --multi 0)
        res.update({"serve_" + k: v for k, v in measure_engine_pipelined(model, scenes, frames, warmup,
                                                                          streams=4).items()})
    if e2e:
        res.update({"serve_" + k: v for k, v in measure_e2e(model, scenes, frames, warmup).items()})
        res.update({"serve_" + k: v for k, v in measure_e2e(model, scenes, frames, warmup, gpu_jpeg=False).items()})
        res.update({"serve_" + k: v for k, v in measure_e2e(model, scenes, frames, warmup, streams=4).items()})
        res.update({"serve_" + k: v for k, v in measure_e2e_procs(model, frames, warmup, procs=2, streams=4).items()})
        _progress("e2e done")
    return res


if __name__ == "__main__":
    import argparse
    import json
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--train-steps", type=int, default=200)
    ap.add_argument("--e2e", type=int, default=1)
    ap.add_argument("--multi", type=int, default=1, help="also the 4-thread engine rate")
    ap.add_argument("--client-port", type=int, default=0, help="internal: run as the e2e load-generator process")
    ap.add_argument("--lockstep", type=int, default=1, help="internal: client also measures lock-step round trips")
    ap.add_argument("--server-child", default=None, help="internal: run as a measure_e2e_procs server process")
    ap.add_argument("--pool", type=int, default=4)
    a = ap.parse_args()
    if a.server_child:
        _server_child(a.server_child, a.pool)
        raise SystemExit(0)
    if a.client_port:
        import sys

        def go():
            print("ready", flush=True)
            sys.stdin.readline()
        print(json.dumps(run_client_load(a.client_port, a.frames, a.warmup, lockstep=bool(a.lockstep), go=go)),
              flush=True)
        raise SystemExit(0)
    print(json.dumps(measure_serving(torch.device("cuda"), a.frames, a.warmup, a.train_steps, bool(a.e2e),
                                     bool(a.multi))),
          flush=True)
