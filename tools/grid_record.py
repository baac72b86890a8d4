"""Per-point work record of BASELINE config 4's 915-point grid on one GPU.

Runs ``sweep.run_grid`` over ``sweep.BASELINE_C4`` (Eb/N0 0..30 x IBO 0..7 dB, CNC 0..8, the
fixed-BER driver's stopping rule, paper geometry) exactly as bench.py's grid object does, and
writes, per grid point, the trials the stopping rule ran and the cost ``sweep.point_costs``
modelled, plus each stopping-rule round's open points, trials and kernel ms.  Every point of a
round shares one launch whose per-trial cost does not depend on the point (the same receiver
iterations run for all), so a point's kernel time is its trials x the round's ms per trial;
the record states that too.

tests/test_grid_balance.py checks the cost model against the committed record (rank
correlation, LPT makespan at N = 2, 4, 8 evaluated on the measured costs).

    python tools/grid_record.py [--channel rayleigh] [--out profiles/r05/grid/c4_points.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "m-mimo-ofdm-with-nonlinear-pa-sim_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--channel", default="rayleigh")
    ap.add_argument("--receiver", default="cnc")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import sweep
    c4 = sweep.BASELINE_C4
    link = sweep.paper_link(a.channel, a.receiver, "f64", device=0, n_err_min=c4["n_err_min"],
                            bits_sent_max=c4["bits_sent_max"])
    link.engine().run(0, 0, 1, [0])  # engine set-up outside the timed region
    st = {}
    t0 = time.perf_counter()
    err, bits = sweep.run_grid(link, c4["ibo"], c4["ebn0"], c4["iters"], incl_clean=False, seed=2137, stats=st)
    wall = time.perf_counter() - t0
    n_pts = len(c4["ibo"]) * len(c4["ebn0"])
    trials = np.zeros(n_pts, np.int64)
    trials[st["point_ids"]] = st["trials_per_point"]
    model = np.zeros(n_pts)
    model[st["point_ids"]] = st["cost_model"]
    ms_per_trial = [r["kernel_ms"] / max(1, r["trials"]) for r in st["round_log"]]
    ber = (err / np.maximum(bits, 1)).reshape(n_pts, -1)
    out = dict(channel=a.channel, receiver=a.receiver, grid="sweep.BASELINE_C4", axis="Eb/N0",
               ibo=c4["ibo"].tolist(), ebn0=c4["ebn0"].tolist(), iters=c4["iters"].tolist(),
               n_err_min=c4["n_err_min"], bits_sent_max=c4["bits_sent_max"], bits_per_symbol=2048 * 6,
               points=n_pts, trials_per_point=trials.tolist(), cost_model=model.round(3).tolist(),
               min_ber_per_point=[float(x) for x in ber.min(axis=1)],
               rounds=st["round_log"], kernel_ms=st["kernel_ms"], wall_s=round(wall, 4),
               kernel_ms_per_trial_by_round=[round(x, 6) for x in ms_per_trial],
               note="a point's kernel time = its trials x its round's ms per trial (one launch per round "
                    "covers every open point; the per-trial work does not depend on the point)")
    s = json.dumps(out)
    print(s[:400], flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
