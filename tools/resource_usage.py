"""Per-kernel VGPR / AGPR / spill / LDS / occupancy table of one HIP source (hipcc remarks).

    python tools/resource_usage.py spotter_amd/csrc/conv_mfma16.hip [name-filter]
"""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=fast",
           f"-I{ROOT}/include", "-c", src, "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith("Function Name:"):
            cur = {"name": txt.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        if filt not in r["name"]:
            continue
        dem = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        dem = re.sub(r"sp::\(anonymous namespace\)::", "", dem).replace("(sp::ConvArgs)", "")
        print(f"{dem[:60]:60s} vgpr={r.get('VGPRs'):>4} agpr={r.get('AGPRs'):>4} "
              f"vspill={r.get('VGPRs Spill')} sspill={r.get('SGPRs Spill')} "
              f"lds={r.get('LDS Size [bytes/block]')} occ={r.get('Occupancy [waves/SIMD]')}")


if __name__ == "__main__":
    main()
