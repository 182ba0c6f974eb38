#!/usr/bin/env python3
"""Entry point at the reference's path (/root/reference/scripts/01_calibrate_camera.py): `rdp calibrate` with the same defaults.

All options: `python scripts/01_calibrate_camera.py --help`. Equivalent: `python -m robotic_discovery_platform_amd calibrate`.
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from robotic_discovery_platform_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["calibrate", *sys.argv[1:]]))
