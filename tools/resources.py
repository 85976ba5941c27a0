#!/usr/bin/env python3
"""Per-kernel VGPR / SGPR spill / occupancy / LDS table of the product
library (hipcc -Rpass-analysis=kernel-resource-usage over its sources).

    python tools/resources.py [extra hipcc flags...]

Exits 1 if any kernel spills (VGPR or SGPR), so it doubles as a check."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ntt-gpu-qtesla_amd")
SRCS = ["csrc/ntt_kernels.hip", "csrc/nussbaumer.hip"]


def main():
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Wall", "--cuda-device-only",
           "-c", "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
    rows, cur = [], None
    for src in SRCS:
        out = subprocess.run(cmd + [src], cwd=PKG, capture_output=True, text=True).stderr
        for line in out.splitlines():
            m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
            if not m:
                continue
            key, val = m.group(1).strip(), m.group(2).strip()
            if key == "Function Name":
                cur = {"name": val}
                rows.append(cur)
            elif cur is not None:
                cur[key] = val
    bad = 0
    print(f"{'kernel':64s} {'VGPR':>5s} {'occ':>4s} {'vspill':>6s} {'sspill':>6s} {'LDS B':>7s}")
    for r in rows:
        dem = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        dem = dem.replace("(anonymous namespace)::", "").replace("qntt::", "")
        dem = re.sub(r"\(.*\)$", "", dem).replace("void ", "")
        vs, ss = int(r.get("VGPRs Spill", 0)), int(r.get("SGPRs Spill", 0))
        bad += vs + ss
        print(f"{dem[:64]:64s} {r.get('VGPRs', '?'):>5s} {r.get('Occupancy [waves/SIMD]', '?'):>4s} {vs:6d} {ss:6d} "
              f"{r.get('LDS Size [bytes/block]', '?'):>7s}")
    print("spills:", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
