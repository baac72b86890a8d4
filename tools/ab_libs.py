"""Interleaved A/B timing of several builds of libmimo_engine.so in ONE process.

    python tools/ab_libs.py abl/lib_base.so m-mimo-ofdm-with-nonlinear-pa-sim_amd/libmimo_engine.so

Each library gets its own engine (BASELINE config 2 via bench.make_engine); launches
alternate between them round by round.  Prints median / min kernel ms per launch and the
error totals (builds that differ only in fp32 rounding agree to a few errors in 1e7 bits).
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "m-mimo-ofdm-with-nonlinear-pa-sim_amd")]

import numpy as np  # noqa: E402

import _engine  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1 << 16)
    ap.add_argument("--iters", default="0")
    ap.add_argument("--workload", default="2")
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"])
    args = ap.parse_args()
    iters = [int(x) for x in args.iters.split(",")]
    handles, engines = [], []
    for path in args.libs:
        _engine._lib, _engine.LIB_PATH = None, os.path.abspath(path)
        # an older build may predate entry points the binding lists: bind what it exports
        probe = ctypes.CDLL(_engine.LIB_PATH)
        saved = dict(_engine.SYMBOLS)
        for name in [n for n in saved if not hasattr(probe, n)]:
            del _engine.SYMBOLS[name]
        handles.append(_engine.lib())
        _engine.SYMBOLS.clear()
        _engine.SYMBOLS.update(saved)
        engines.append(bench.make_engine(0, args.workload, args.precision))
    res = {i: [] for i in range(len(engines))}
    errs = {}
    for r in range(args.rounds + 1):
        for i, eng in enumerate(engines):
            e, b, _ = eng.run(2137, 0, args.batch, iters, False)
            if r:  # round 0 = warm-up
                res[i].append(eng.kernel_ms)
            errs[i] = (e.tolist(), eng.describe())
    out = []
    for i, path in enumerate(args.libs):
        ms = np.asarray(res[i])
        out.append(dict(lib=path, desc=errs[i][1], median_ms=float(np.median(ms)), min_ms=float(ms.min()),
                        trials_per_s=args.batch / (np.median(ms) / 1e3), errors=errs[i][0]))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
