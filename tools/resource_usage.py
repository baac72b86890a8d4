"""Per-instance register / scratch / occupancy / LDS summary of one trial-kernel object.

Compiles csrc/trial_inst.hip for one FFT size with -Rpass-analysis=kernel-resource-usage
(nothing is written to the build tree) and prints one line per kernel instance.

    python tools/resource_usage.py --F 2048 --f64 [-D MIMO_WAVE_FFT64=0 ...]
"""
import argparse
import os
import re
import subprocess
import tempfile

CSRC = os.environ.get("MIMO_CSRC") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "m-mimo-ofdm-with-nonlinear-pa-sim_amd", "csrc")
ARGS = re.compile(r"trial_kernelI([df])Li(\d+)ELi(\d+)ELi(\d+)ELb(\d)ELi(\d)ELb(\d)ELi(\d)ELi(\d)ELb(\d)")
CH = {"1": "rayleigh", "2": "los", "3": "twopath", "4": "table"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--F", type=int, default=2048)
    ap.add_argument("--f64", action="store_true")
    ap.add_argument("-D", action="append", default=[], help="extra macro definitions")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-fno-slp-vectorize",
               "-DINST_F=%d" % a.F, "-DINST_F64=%d" % int(a.f64), "-Rpass-analysis=kernel-resource-usage",
               "-c", "trial_inst.hip", "-o", os.path.join(tmp, "x.o")] + ["-D" + d for d in a.D]
        out = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        if "Function Name:" in line:
            m = ARGS.search(line)
            cur = dict(inst=("%s F=%s T=%s slots=%s %s %s csi=%s" % (
                "f64" if m.group(1) == "d" else "f32", m.group(2), m.group(3), m.group(4),
                "aligned" if m.group(5) == "1" else "generic", CH.get(m.group(6), m.group(6)), m.group(7)))
                       if m else line.split("Function Name:")[1].strip())
            rows.append(cur)
        elif cur is not None:
            for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                             ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
                m = re.search(pat, line)
                if m:
                    cur[key] = int(m.group(1))
    for r in rows:
        print("%-48s vgpr %3s agpr %3s scratch %4s occ %s lds %6s" % (
            r["inst"], r.get("vgpr"), r.get("agpr"), r.get("scratch"), r.get("occ"), r.get("lds")))


if __name__ == "__main__":
    main()
