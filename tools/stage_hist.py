"""Per-stage VALU opcode classes of the fused kernel's loops, from the ISA.

Compiles one trial_kernel instance (tools/one_inst.hip, -S, soft limiter only) once as is
and once per stage compiled out (-DMIMO_STATIC_ABLATE=<ABL_* bit>, trial_kernel.h), takes
the static instruction mix of the array-pass loop (the loop with the most Philox products)
and of pass 1, and attributes the differences to the stages:

  RNG   -- the channel draws of the array pass (Philox + Box-Muller; ABL_RNG = 1)
  FFT   -- both transforms incl. their LDS exchanges (ABL_FFT = 2)
  PA    -- the soft limiter (ABL_PA = 8)
  rest  -- what remains: precode, combine, alpha, vk, loop control

Static counts of the executed path (the antenna loop has no data-dependent branches at the
bench configuration besides the alpha fallback, which is out of line).

    python tools/stage_hist.py [--F 2048 --T 256 --NS 4 --MW 3 --R double] [--json out.json]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.environ.get("MIMO_CSRC") or os.path.join(REPO, "m-mimo-ofdm-with-nonlinear-pa-sim_amd", "csrc")
STAGES = {"RNG": 1, "FFT": 2, "PA": 8}


def classify(op):
    if op.startswith("s_") or op.startswith("ds_") or op.startswith(("global_", "scratch_", "buffer_", "flat_")):
        return None
    if re.match(r"v_(add|sub)_f64", op):
        return "f64_add"
    if re.match(r"v_mul_f64", op):
        return "f64_mul"
    if re.match(r"v_(fma|fmac)_f64", op):
        return "f64_fma"
    if op.endswith("_f64") or "_f64_" in op or op.startswith("v_cvt_f64") or "f64" in op:
        return "f64_other"  # rsq, min/max, ldexp, floor, fract, cvt, div_scale, cmp
    if op.startswith(("v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32")):
        return "int_mul"
    if op.startswith(("v_mov_b32_dpp", "v_mov_b64", "v_mov_b32", "v_readfirstlane", "v_writelane", "v_readlane")):
        return "mov"
    if op.startswith(("v_cndmask", "v_cmp")):
        return "cmp_cnd"
    if re.match(r"v_\w*(_f32|_f16)", op) or op.startswith(("v_log", "v_exp", "v_sin", "v_cos", "v_rcp")):
        return "f32"
    if op.startswith(("v_lshl_add_u64", "v_add_co", "v_addc_co", "v_sub_co", "v_subb_co")):
        return "addr64"
    return "int_other"  # xor / bitop3 / and / or / shifts / bfe / add_u32 / bcnt


def loops(asm_text):
    """{loop header: opcode counts of its blocks}, {marker name: loop header} (MIMO_ISA_MARK)."""
    lines = asm_text.split("\n")
    blocks, marks, cur, hdr_name = collections.OrderedDict(), {}, None, None
    for line in lines:
        m = re.match(r"^\.L(BB\d+_\d+):(.*)", line)
        if m:
            hdr = re.search(r"Header=(BB\d+_\d+) Depth=1", m.group(2))
            if "Loop Header: Depth=1" in m.group(2):
                hdr_name = m.group(1)
            elif hdr:
                hdr_name = hdr.group(1)
            else:
                hdr_name = None
            cur = blocks.setdefault(hdr_name, collections.Counter()) if hdr_name else None
            continue
        s = line.strip()
        mk = re.search(r"MIMO_MARK (\w+)", s)
        if mk and hdr_name:
            marks[mk.group(1)] = hdr_name
        if cur is not None and s and s[0] not in ";.":
            cur[s.split()[0]] += 1
    return blocks, marks


def compile_variant(a, extra):
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "x.s")
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
               "-fno-slp-vectorize", "-I" + CSRC, "-DXR=" + a.R, "-DXF=%d" % a.F, "-DXT=%d" % a.T, "-DXNS=%d" % a.NS,
               "-DXMW=%d" % a.MW, "-DXNB=1", "-DXSYM=false", "-DMIMO_DIAG_PA_SOFTLIM_ONLY", "-DMIMO_ISA_MARKERS", "-S",
               os.path.join(REPO, "tools", "one_inst.hip"), "-o", out] + extra
        subprocess.run(cmd, check=True, capture_output=True)
        return open(out).read()


def main_loop(parsed):
    """(array-pass loop, pass-1 loop) opcode counts, found by their MIMO_ISA_MARK comments."""
    blocks, marks = parsed
    return blocks[marks["array_pass"]], blocks.get(marks.get("pass1"), collections.Counter())


def classes(c):
    out = collections.Counter()
    for op, n in c.items():
        k = classify(op)
        if k:
            out[k] += n
    out["VALU"] = sum(v for k, v in out.items())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--F", type=int, default=2048)
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--NS", type=int, default=4)
    ap.add_argument("--MW", type=int, default=3)
    ap.add_argument("--R", default="double")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    base_arr, base_p1 = main_loop(loops(compile_variant(a, [])))
    full = classes(base_arr)
    res = {"instance": vars(a), "array_pass": dict(full), "pass1": dict(classes(base_p1)), "stages": {}}
    rest = collections.Counter(full)
    for name, bit in STAGES.items():
        arr, _ = main_loop(loops(compile_variant(a, ["-DMIMO_STATIC_ABLATE=%d" % bit])))
        diff = full.copy()
        diff.subtract(classes(arr))
        res["stages"][name] = {k: v for k, v in diff.items() if v}
        rest.subtract(diff)
    res["stages"]["rest"] = {k: v for k, v in rest.items() if v}
    keys = ["VALU", "f64_add", "f64_mul", "f64_fma", "f64_other", "int_mul", "int_other", "addr64", "mov", "cmp_cnd",
            "f32"]
    print("%-12s" % "" + "".join("%10s" % k for k in keys))
    for name, d in [("array pass", full), ("pass 1", res["pass1"])] + list(res["stages"].items()):
        print("%-12s" % name + "".join("%10d" % d.get(k, 0) for k in keys))
    for name, d in [("array pass", full)] + list(res["stages"].items()):
        f = d.get("f64_add", 0) + d.get("f64_mul", 0) + d.get("f64_fma", 0)
        if f:
            print("%-12s FMA share of f64 add/mul/fma: %.2f" % (name, d.get("f64_fma", 0) / f))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
