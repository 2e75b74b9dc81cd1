"""Regenerate tests/golden/force_curves.json from the reference's thesis data files
rl/juypter/thesis_plots/sim_vs_real_forces.csv, sim_vs_real_forces_constrict.csv and
sim_vs_real_forces_tilt.csv (data only: the MuJoCo finger-gauge forces the reference's
"measure constrict" / "measure tilt" programs printed, mysimulate.cpp:2720-2811, next to the
real gripper's).  usage: python tests/golden/make_force_curves.py /root/reference"""
import csv
import json
import math
import os
import sys

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
D = os.path.join(ref, "rl/juypter/thesis_plots")


def columns(fn):
    rows = list(csv.reader(open(os.path.join(D, fn))))
    hdr = [h.strip() for h in rows[0]]
    out = {}
    for j, h in enumerate(hdr):
        vals = [float(r[j]) if j < len(r) and r[j].strip() else None for r in rows[1:]]
        out[h] = vals
    return out


out = {"source": "rl/juypter/thesis_plots/sim_vs_real_forces*.csv (reference repository). 'XY pos' is the "
                 "x (= y for constrict) motor target in mm; 'Sim D EIk' the MuJoCo finger-gauge SI force (N, "
                 "sim_sensors_SI_) for a sphere of diameter D mm with finger variant k; 'Real ...' the real "
                 "gripper's.  The notebook design_modelling_chapters.ipynb (cells 3-4) labels the three "
                 "finger variants of mujoco_timesteps.csv -- (t, w) = (0.9, 28), (1.0, 24), (1.0, 28) mm -- "
                 "EI = 0.29, 0.34, 0.40 N m^2, and plots the Sim 80/100/120 columns",
       "constrict_A": columns("sim_vs_real_forces.csv"),
       "constrict_B": columns("sim_vs_real_forces_constrict.csv"),
       "tilt": columns("sim_vs_real_forces_tilt.csv")}
for k, v in out.items():
    if isinstance(v, dict):
        for h, col in v.items():
            assert all(x is None or math.isfinite(x) for x in col), (k, h)
json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "force_curves.json"), "w"), indent=0)
