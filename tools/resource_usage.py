"""Per-kernel register / LDS / occupancy report of one HIP source file (hipcc
-Rpass-analysis=kernel-resource-usage remarks; no GPU needed).
usage: python tools/resource_usage.py pgi_raytracing_amd/csrc/trace.hip"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-fhip-fp32-correctly-rounded-divide-sqrt", f"-I{ROOT}/include", f"-I{ROOT}/pgi_raytracing_amd/csrc", "-c",
           src, "-o", "/tmp/resource_usage.o", "-Rpass-analysis=kernel-resource-usage"]
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        n = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip().split("(")[0]
        g = r.get
        print(f"{n:58s} VGPR {g('VGPRs', '?'):>4} AGPR {g('AGPRs', '?'):>3} SGPR {g('TotalSGPRs', '?'):>4} "
              f"spillS {g('SGPRs Spill', '?'):>3} spillV {g('VGPRs Spill', '?'):>3} "
              f"LDS {g('LDS Size [bytes/block]', '?'):>6} occ {g('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    for s in sys.argv[1:]:
        main(s)
