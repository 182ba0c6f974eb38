#!/usr/bin/env python3
"""RDP_DDP_EMULATE fidelity: the modelled collective kernel (csrc/comm.hip) must occupy the GPU for its
modelled time -- no less (it would under-model the collective) and no more (a kernel that cannot move its
HBM traffic in time outlasts the model, and the A/B then measures the emulator). Times the kernel alone for
the bucket sizes of the bilinear U-Net at n = 8, 150 GB/s, with and without traffic (3x the bucket)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robotic_discovery_platform_amd.ops import native  # noqa: E402
from robotic_discovery_platform_amd.parallel.ddp import ring_allreduce_us  # noqa: E402


def main():
    blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    C = native()
    dev = torch.device("cuda")
    rows = []
    scratch = torch.zeros(2 * 3 * 19 * (1 << 20) + 64, dtype=torch.uint8, device=dev)
    for mb in (1.0, 9.4, 12.5, 18.9):
        nbytes = int(mb * 1e6)
        us = ring_allreduce_us(nbytes, 8, 150.0, 15.0)
        for traffic in (0, 3):
            tb = int(traffic * nbytes) // 16 * 16
            ts = []
            for _ in range(12):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                C.comm_emulate(us, blocks, scratch if tb else None, tb)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            t = sorted(ts[2:])[len(ts[2:]) // 2]
            rows.append({"blocks": blocks, "bucket_mb": mb, "traffic_x": traffic, "modelled_us": round(us, 1), "measured_us": round(t, 1),
                         "hbm_gbps": round(2 * tb / (t * 1e3), 1) if tb else 0.0})
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
