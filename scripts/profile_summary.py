#!/usr/bin/env python3
"""Summarise rocprofv3 kernel stats/traces under gpurun_out/ into markdown tables in profiles/.

Writes profiles/train_step_kernels.md (per-kernel totals for 5 native training steps at bs32, plus
the per-layer conv table for the last step) and profiles/serve_frame_kernels.md (per-kernel totals
of the serving benchmark), and copies the raw *_kernel_stats.csv next to them.
"""
import csv
import glob
import io
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def stats_table(path, top=25):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = ["| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for r in rows[:top]:
        name = r["Name"].split("(")[0][:80]
        out.append(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                   f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    out.append(f"| **all kernels** | | **{tot / 1e6:.3f}** | | 100 |")
    return "\n".join(out)


def find(pattern):
    m = glob.glob(os.path.join(ROOT, "gpurun_out", pattern), recursive=True)
    return sorted(m)[-1] if m else None


def run_tool(script, *args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", script), *args], capture_output=True, text=True,
                       cwd=ROOT)
    return r.stdout.strip()


def main():
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    tr = find("prof_train/**/train_kernel_stats.csv")
    if tr:
        shutil.copy(tr, os.path.join(ROOT, "profiles", "train_kernel_stats.csv"))
        md = ["# Native training step at bs 64: kernel time (rocprofv3)", "",
              "Default schedule (eager launches, weight gradients on a side stream): "
              "`rocprofv3 --kernel-trace --stats -- python3 bench.py --batch 64 --steps 4 --warmup 3 --serve 0` "
              "on one MI355X (7 steps in the totals).", "", stats_table(tr)]
        trace = find("prof_train/**/train_kernel_trace.csv")
        serial = find("prof_serial/**/serial_kernel_trace.csv")
        if trace:
            md += ["", "## Wall / busy / idle per step (default schedule; sum > busy = stream overlap)", "", "```",
                   run_tool("graph_gaps.py", trace), "```"]
        if serial:
            md += ["", "## Same step with every kernel serialised on one stream (`RDP_WGRAD_OVERLAP=0`)", "",
                   "Clean per-kernel cost (no contention); compare the wall time with the default schedule above",
                   "for what the side-stream overlap buys.", "", "```",
                   run_tool("graph_gaps.py", serial), "```", "", "One step, per kernel (serialised | default):", "",
                   "```", run_tool("trace_breakdown.py", serial, "4", trace) if trace else "", "```", "",
                   "## Per-layer conv kernels (serialised step; TF/s = 2*N*H*W*9*Cin*Cout / time)", "", "```",
                   run_tool("analyze_trace.py", serial, "64"), "```"]
        open(os.path.join(ROOT, "profiles", "train_step_kernels.md"), "w").write("\n".join(md) + "\n")
        print("wrote profiles/train_step_kernels.md")
    tt = find("prof_tr/**/tr_kernel_stats.csv")
    if tt:
        md = ["# Native training step, transposed-conv decoder (fixed), bs 64: kernel time (rocprofv3)", "",
              "`rocprofv3 --kernel-trace --stats -- python3 bench.py --decoder transposed --batch 64 --steps 4 "
              "--warmup 3 --serve 0` on one MI355X (7 steps in the totals). 31.04M params, 96.3 GFLOP/img "
              "forward (1.2x the bilinear model).", "", stats_table(tt)]
        trace = find("prof_tr/**/tr_kernel_trace.csv")
        if trace:
            md += ["", "## Wall / busy / idle per step", "", "```", run_tool("graph_gaps.py", trace), "```", "",
                   "## One step, per kernel", "", "```", run_tool("trace_breakdown.py", trace, "4"), "```"]
        open(os.path.join(ROOT, "profiles", "train_step_transposed.md"), "w").write("\n".join(md) + "\n")
        print("wrote profiles/train_step_transposed.md")
    b4 = find("prof_bs4/**/bs4_kernel_trace.csv")
    if b4:
        md = ["# Native training step at the reference batch (bs 4, 256², bf16, Adam): kernel time (rocprofv3)", "",
              "Default schedule (eager launches, wgrads on the side stream): `rocprofv3 --kernel-trace --stats -- "
              "python3 bench.py --batch 4 --steps 20 --warmup 5 --serve 0` on one MI355X (the profiler adds "
              "per-launch overhead; the unprofiled rate is `ref_batch_imgs_per_s` in the bench line).", "",
              "## Wall / busy / idle per step (µs; sum > busy = the side-stream wgrads overlap the main stream)", "",
              "```", run_tool("graph_gaps.py", b4), "```", "", "## Per-kernel totals for one step", "", "```",
              run_tool("trace_breakdown.py", b4, "4"), "```"]
        open(os.path.join(ROOT, "profiles", "train_step_bs4.md"), "w").write("\n".join(md) + "\n")
        print("wrote profiles/train_step_bs4.md")
    sv = find("prof_serve/**/serve_kernel_stats.csv")
    if sv:
        shutil.copy(sv, os.path.join(ROOT, "profiles", "serve_kernel_stats.csv"))
        md = ["# Serving benchmark: kernel time (rocprofv3 --kernel-trace --stats)", "",
              "`python -m robotic_discovery_platform_amd.serve.bench_serve --frames 200 --warmup 20 --train-steps 200 --e2e 0` "
              "(includes the 200 training steps that produce realistic masks, then per-frame graph replays "
              "of the engine).", "", stats_table(sv, 40)]
        st = find("prof_serve/**/serve_kernel_trace.csv")
        if st:
            md += ["", "## One engine frame (graph replay), kernel timeline", "", "```",
                   run_tool("serve_frame.py", st), "```"]
        open(os.path.join(ROOT, "profiles", "serve_frame_kernels.md"), "w").write("\n".join(md) + "\n")
        print("wrote profiles/serve_frame_kernels.md")


def micro_table(paths):
    rows = []
    for p in paths:
        for line in open(p):
            line = line.strip()
            if line.startswith("{") and '"shape"' in line:
                import json
                rows.append(json.loads(line))
    if not rows:
        return None
    keys = sorted({k for r in rows for k in r if k.endswith("_tflops")})
    out = ["| layer shape | kind | " + " | ".join(k.replace("_tflops", " TF/s") for k in keys) + " |",
           "|---|---|" + "---:|" * len(keys)]
    for r in rows:
        out.append(f"| {r['shape']} | {r['kind']} | " + " | ".join(str(r.get(k, "")) for k in keys) + " |")
    return "\n".join(out)


def micro_main():
    # profiles/conv_microbench.md is written by scripts/micro_report.py (one labelled column per run);
    # this legacy path merged every micro_*.log into duplicate unlabelled rows, so it only prints now
    paths = sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "micro_*.log")))
    t = micro_table(paths)
    if t and os.environ.get("RDP_LEGACY_MICRO_MD"):
        md = ["# Conv kernels per U-Net layer shape (scripts/conv_microbench.py, bs 32, median of rounds)", "",
              "fwd variants: v0 = auto dispatch, v1 = halo-tile kernel, v128/v256 = implicit-GEMM tiles; "
              "wgrad: v0 = default (BK=64, 2 stages). TF/s counts 2*N*H*W*9*Cin*Cout.", "", t]
        open(os.path.join(ROOT, "profiles", "conv_microbench.md"), "w").write("\n".join(md) + "\n")
        print("wrote profiles/conv_microbench.md")
    pmc = os.path.join(ROOT, "gpurun_out", "pmc")
    if glob.glob(os.path.join(pmc, "set*", "pmc_counter_collection.csv")):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), pmc], capture_output=True,
                           text=True)
        open(os.path.join(ROOT, "profiles", "conv_pmc.md"), "w").write(
            "# PMC counters of the conv kernels (rocprofv3 --pmc, kernel-trace only)\n\n```\n" + r.stdout + "```\n")
        print("wrote profiles/conv_pmc.md")


if __name__ == "__main__":
    main()
