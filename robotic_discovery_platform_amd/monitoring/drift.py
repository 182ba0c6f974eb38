"""Data-drift detector over the serving metrics log.

Reference: ``/root/reference/scripts/monitoring/drift_detector.py:24-86``. Reads
``logs/vision_service_metrics.csv`` (header ``timestamp,mean_curvature,max_curvature,
mask_coverage_percent``), needs >= 50 rows, baseline = first 50 % of rows, recent = the rest, metric =
mean ``mask_coverage_percent``, relative change = (recent - base) / base, drift if |change| > 0.25;
prints the retraining recommendation; plots raw values + 20-sample rolling mean + the two spans to
``reports/drift_report.png`` at 150 dpi.

Fixes vs the reference: a zero baseline mean no longer divides by zero (change is +inf when the
recent mean is positive, 0 otherwise), and the result is returned as a dict for the workflow.
"""
from __future__ import annotations

import logging
import math
import os
from typing import Optional

import numpy as np

from ..config import DriftConfig

log = logging.getLogger("rdp.drift")


def analyze_drift(log_file: Optional[str] = None, cfg: Optional[DriftConfig] = None, make_plot: bool = True,
                  report_path: Optional[str] = None) -> dict:
    cfg = cfg or DriftConfig()
    log_file = log_file or cfg.log_file
    if not os.path.exists(log_file):
        log.error("Log file not found at '%s'. Please run the vision service first.", log_file)
        return {"status": "missing_log", "drift_detected": False}
    import pandas as pd
    df = pd.read_csv(log_file)
    if len(df) < cfg.min_rows:
        log.warning("Not enough data to perform drift analysis (need at least %d records).", cfg.min_rows)
        return {"status": "insufficient_data", "rows": len(df), "drift_detected": False}
    split = int(len(df) * cfg.baseline_frac)
    col = df[cfg.metric].astype(float)
    base, recent = float(col.iloc[:split].mean()), float(col.iloc[split:].mean())
    if base != 0:
        change = (recent - base) / base
    else:
        change = math.inf if recent > 0 else 0.0
    drift = abs(change) > cfg.threshold
    log.info("Baseline %s mean: %.2f%%", cfg.metric, base)
    log.info("Recent %s mean:   %.2f%%", cfg.metric, recent)
    log.info("Percentage change: %+.2f%%", change * 100 if math.isfinite(change) else change)
    if drift:
        log.warning("DRIFT DETECTED! Change exceeds threshold of %.2f%%.", cfg.threshold * 100)
        print("\nRECOMMENDATION: Trigger the retraining pipeline to adapt the model to the new data distribution.")
        print("-> python workflows/retraining_pipeline.py")
    else:
        log.info("No significant drift detected.")
    out = {"status": "ok", "rows": len(df), "baseline_mean": base, "recent_mean": recent,
           "percentage_change": change, "drift_detected": bool(drift), "split_index": split}
    if make_plot:
        out["report"] = _plot(df, col, split, base, recent, drift, cfg, report_path)
    return out


def _plot(df, col, split, base, recent, drift, cfg: DriftConfig, report_path: Optional[str]) -> Optional[str]:
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception as e:  # pragma: no cover
        log.warning("matplotlib unavailable (%s): no report", e)
        return None
    os.makedirs(cfg.reports_dir, exist_ok=True)
    path = report_path or os.path.join(cfg.reports_dir, "drift_report.png")
    try:
        plt.style.use("seaborn-v0_8-whitegrid")
    except Exception:
        pass
    fig, ax = plt.subplots(figsize=(12, 6))
    ax.plot(df.index, col, label="Mask Coverage", color="gray", alpha=0.5, zorder=1)
    ax.plot(df.index, col.rolling(window=cfg.rolling_window).mean(),
            label=f"Rolling Mean ({cfg.rolling_window} samples)", color="cornflowerblue", zorder=2)
    ax.axvspan(0, split, color="green", alpha=0.1, label=f"Baseline (Mean: {base:.2f}%)")
    ax.axvspan(split, len(df), color="orange", alpha=0.1, label=f"Recent (Mean: {recent:.2f}%)")
    ax.set_title(f"Drift Analysis: Mask Coverage\nDrift Detected: {drift}", fontsize=16, weight="bold")
    ax.set_xlabel("Log Entry Index")
    ax.set_ylabel("Mask Coverage (%)")
    ax.legend()
    ax.grid(True, which="both", linestyle="--", linewidth=0.5)
    fig.savefig(path, dpi=cfg.dpi, bbox_inches="tight")
    plt.close(fig)
    log.info("Drift analysis report saved to '%s'", path)
    return path
