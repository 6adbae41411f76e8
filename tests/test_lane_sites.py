"""The cross-lane read table stays complete: every readlane / DPP site of mrts_kernels.hip sits in
a function that tools/lane_sites.py gives a reason for (DESIGN.md §4 reproduces the table).  CPU only."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_cross_lane_site_has_a_reason():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lane_sites.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert len(r.stdout.strip().splitlines()) > 40  # (the scan found the sites)
