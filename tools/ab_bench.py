"""Interleaved A/B timing of engine variants in ONE process (guide §5.4 rule 24).

    python tools/ab_bench.py --var MIMO_TEAM=128 --var MIMO_TEAM=256 --rounds 5

Each --var is a set of environment overrides read by the engine at launch time
(comma-separated KEY=VAL).  Prints median / min kernel ms per 65536-trial launch and
the error totals of each variant (they must agree to fp32-rounding level).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "m-mimo-ofdm-with-nonlinear-pa-sim_amd")]

import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--var", action="append", default=[])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1 << 16)
    ap.add_argument("--iters", default="0")
    ap.add_argument("--workload", default="2")
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"])
    args = ap.parse_args()
    variants = [dict(kv.split("=", 1) for kv in v.split(",") if kv) for v in (args.var or [""])]
    eng = bench.make_engine(0, args.workload, args.precision)
    iters = [int(x) for x in args.iters.split(",")]
    res = {i: [] for i in range(len(variants))}
    errs = {}
    base_env = dict(os.environ)
    for r in range(args.rounds + 1):
        for i, v in enumerate(variants):
            os.environ.clear()
            os.environ.update(base_env)
            os.environ.update(v)
            e, b, _ = eng.run(2137, 0, args.batch, iters, False)
            if r:  # round 0 = warm-up
                res[i].append(eng.kernel_ms)
            errs[i] = (e.tolist(), eng.describe())
    out = []
    for i, v in enumerate(variants):
        ms = np.asarray(res[i])
        out.append(dict(variant=v, desc=errs[i][1], median_ms=float(np.median(ms)), min_ms=float(ms.min()),
                        trials_per_s=args.batch / (np.median(ms) / 1e3), errors=errs[i][0]))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
