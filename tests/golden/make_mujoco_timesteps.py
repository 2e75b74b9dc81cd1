"""Regenerate tests/golden/mujoco_timesteps.json from the reference's thesis data file
rl/juypter/thesis_plots/mujoco_timesteps.csv (rows N = 5..10; data only).
usage: python tests/golden/make_mujoco_timesteps.py /root/reference"""
import csv
import json
import os
import sys

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
rows = list(csv.reader(open(os.path.join(ref, "rl/juypter/thesis_plots/mujoco_timesteps.csv"))))
hdr = [h.strip() for h in rows[0]]
cols = {h: {r[0].strip(): float(r[j]) for r in rows[1:] if 5 <= int(r[0]) <= 10} for j, h in enumerate(hdr[1:], 1)}
out = {"source": "rl/juypter/thesis_plots/mujoco_timesteps.csv (reference repository): highest stable MuJoCo "
                 "timestep in milliseconds found by MjClass::find_highest_stable_timestep (mjclass.cpp:4745-4816, "
                 "before the safety factor) per finger segment count N, for finger thickness t [mm], width w [mm] "
                 "and segment inertia scaling; rows N = 5..10 (the build's segment range)",
       "columns": cols}
json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "mujoco_timesteps.json"), "w"), indent=1)
