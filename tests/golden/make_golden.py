"""Regenerate the golden fixtures in this directory (run in the build container, where
/root/reference exists; the GPU box only reads the committed JSON).

Sources, all independent of the oracle they pin:
  gripper_sequences.json  the reference's own luke::Gripper (src/gripper.cpp), compiled
                          from /root/reference by oracle/Makefile into oracle/_ref/ref_golden
  sliding_window.json     the reference's own luke::SlidingWindow (src/slidingwindow.h),
                          same binary, `window` mode
  rng.json                libstdc++'s default_random_engine + uniform_real_distribution
                          (the reference's RNG stack, mjclass.cpp:4,219-224,1415,1567),
                          oracle/_ref/rng_golden
  polyfit.json            numpy.polyfit (least squares, as arma::polyfit) on gauge point
                          sets (myfunctions.cpp:2699-2795)
  change_sample.json      the known answer printed by test.cpp:293-311
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_BIN = os.path.join(REPO, "oracle", "_ref")


def gripper_sequences():
    rng = np.random.default_rng(20240606)
    cmds = []
    for _ in range(400):
        u = rng.random()
        if u < 0.35:
            cmds.append([0, rng.uniform(-0.03, 0.03), rng.uniform(-0.4, 0.4), rng.uniform(-0.02, 0.02)])
        elif u < 0.6:
            cmds.append([1, rng.uniform(-0.03, 0.03), rng.uniform(-0.03, 0.03), rng.uniform(-0.02, 0.02)])
        elif u < 0.97:
            cmds.append([2, float(rng.integers(1, 25)), 0, 0])
        else:
            cmds.append([3, 0, 0, 0])
    # clamp edge cases: far outside every limit, then step all the way there
    cmds += [[1, 1.0, 1.0, 1.0], [2, 100000, 0, 0], [1, -1.0, -1.0, -1.0], [2, 100000, 0, 0],
             [0, 0.0, 3.0, 0.0], [2, 100000, 0, 0], [0, 0.0, -3.0, 0.0], [2, 100000, 0, 0]]

    def run(cmds):
        txt = "".join(f"{int(c[0])} {c[1]!r} {c[2]!r} {c[3]!r}\n" for c in cmds)
        out = subprocess.run([os.path.join(REF_BIN, "ref_golden"), "gripper"], input=txt, capture_output=True,
                             text=True, check=True).stdout
        return [[float(x) for x in line.split()] for line in out.strip().splitlines()]

    # set_xyz_m with |y - x| > leadscrew makes asin() NaN (gripper.cpp:50); a later
    # step_to on that NaN target converts NaN to int (undefined behaviour, hardware
    # dependent), so every NaN state is followed by a reset: the NaN state itself is
    # pinned, the undefined step after it is not.
    while True:
        rows = run(cmds)
        bad = [i for i, r in enumerate(rows) if any(np.isnan(r)) and i + 1 < len(cmds) and cmds[i + 1][0] != 3]
        if not bad:
            break
        cmds.insert(bad[0] + 1, [3, 0, 0, 0])
    return {"cmds": cmds, "out": rows,
            "columns": "ret end.x end.y end.z end.th end.step.x end.step.y end.step.z "
                       "next.x next.y next.z next.th next.step.x next.step.y next.step.z"}


def sliding_window():
    out = subprocess.run([os.path.join(REF_BIN, "ref_golden"), "window"], capture_output=True, text=True,
                         check=True).stdout
    rows = [[float(x) for x in line.split()] for line in out.strip().splitlines()]
    return {"adds": [k * 0.5 for k in range(1, 21)], "rows": rows,
            "columns": "k read_element(0..9) read(7)"}


def rng():
    out = subprocess.run([os.path.join(REF_BIN, "rng_golden")], capture_output=True, text=True,
                         check=True).stdout
    res = {}
    for line in out.strip().splitlines():
        p = line.split()
        res.setdefault(p[0], {})[p[1]] = [float(x) for x in p[2:]]
    return res


def polyfit():
    rng_ = np.random.default_rng(7)
    cases = []
    for N in (6, 8, 10):
        for _ in range(20):
            L = 0.235
            seg = L / N
            q = rng_.uniform(-0.06, 0.06, size=N) * rng_.choice([0.0, 0.01, 0.1, 1.0])
            X = [seg]; Y = [0.0]
            cum = 0.0
            for i in range(N):
                cum = q[0] if i == 0 else cum + q[i]
                X.append(X[-1] + seg * np.cos(cum)); Y.append(Y[-1] + seg * np.sin(cum))
            c = np.polyfit(np.array(X), np.array(Y), 3)
            y = float(np.polyval(c, 0.05)) * 1000
            cases.append({"X": X, "Y": Y, "order": 3, "x": 0.05, "reading_mm": y})
    return {"cases": cases}


def main():
    if not os.path.exists(os.path.join(REF_BIN, "ref_golden")):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    fixtures = {
        "gripper_sequences.json": gripper_sequences(),
        "sliding_window.json": sliding_window(),
        "rng.json": rng(),
        "polyfit.json": polyfit(),
        "change_sample.json": {"window_adds": [1, 2, 3, 4, 5, 6], "prev_steps": 3, "readings_per_step": 1,
                               "expected": [3, 1, 4, 1, 5, 1, 6], "source": "src/test.cpp:293-311"},
    }
    for name, data in fixtures.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f)
        print("wrote", name)


if __name__ == "__main__":
    sys.exit(main())
