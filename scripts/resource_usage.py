"""Compiler resource usage of every product kernel (VGPRs, AGPRs, SGPRs, spills, scratch, LDS, occupancy), from
hipcc -Rpass-analysis=kernel-resource-usage with the product flags (hello-raytracing_amd/Makefile).

usage: python scripts/resource_usage.py [extra hipcc flags ...] > profiles/rNN/resource_usage.txt
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize", "--cuda-device-only", "-c"]
KEYS = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("TotalSGPRs", "sgpr"), ("VGPRs Spill", "vgpr_spill"),
        ("SGPRs Spill", "sgpr_spill"), (r"ScratchSize \[bytes/lane\]", "scratch"), (r"LDS Size \[bytes/block\]", "lds"),
        (r"Occupancy \[waves/SIMD\]", "waves")]


def main() -> int:
    src = ROOT / "hello-raytracing_amd" / "csrc" / "rt_kernels.hip"
    cmd = ["/opt/rocm/bin/hipcc", *FLAGS, *sys.argv[1:], str(src), "-o", "/tmp/hrt_ru.o",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            sym = m.group(1)
            dem = subprocess.run(["c++filt", sym], capture_output=True, text=True).stdout.strip()
            cur = {"kernel": dem.split("(")[0].replace("void ", "")}
            rows.append(cur)
            continue
        for key, short in KEYS:
            m = re.search(r"\b" + key + r": (\d+)", line)
            if m and cur is not None and short not in cur:
                cur[short] = int(m.group(1))
    cols = ["kernel"] + [s for _, s in KEYS]
    print("# " + " ".join(cmd[:-1]))
    print("\t".join(cols))
    for r in rows:
        print("\t".join(str(r.get(c, "")) for c in cols))
    return 0


if __name__ == "__main__":
    sys.exit(main())
