"""Per-instance VGPRs / spills / occupancy / LDS of the fused trial kernels for one FFT size.

    python tools/resource_report.py 2048 [extra hipcc flags...]
"""
import re
import subprocess
import sys

REPO = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
F = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-fno-slp-vectorize",
       f"-DINST_F={F}", "-c", f"{REPO}/m-mimo-ofdm-with-nonlinear-pa-sim_amd/csrc/trial_inst.hip", "-o", "/tmp/rr.o",
       "-Rpass-analysis=kernel-resource-usage"] + (["-mllvm", "-amdgpu-sched-strategy=max-ilp"] if F == "2048" else []) \
    + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    s = m.group(1).strip()
    if s.startswith("Function Name:"):
        name = s.split(":", 1)[1].strip()
        t = re.search(r"trial_kernelI(.*)EEvNS", name)
        args = re.findall(r"L([ib])(\d+)E", t.group(1)) if t else []
        cur = {"inst": ("f64," if "trial_kernelId" in name else "f32,") + ",".join(v for _, v in args)}
        rows.append(cur)
    elif cur is not None and ":" in s:
        k, v = s.split(":", 1)
        cur[k.strip()] = v.strip()
print("R,F,T,NSLOT,aligned,CH,CSI,MINW,NBUF,SYMW_LDS  VGPRs spill occ LDS")
for r in rows:
    print(f'{r["inst"]:34s} {r.get("VGPRs","?"):>4} {r.get("VGPRs Spill","?"):>4} {r.get("Occupancy [waves/SIMD]","?"):>3} '
          f'{r.get("LDS Size [bytes/block]","?")}')
