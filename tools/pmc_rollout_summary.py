"""Per-launch HBM traffic of the headline's rollout launches from tools/pmc_rollout.sh.

The step kernel's dispatches whose duration is over 5x the per-step launches' median are
the gm_rollout launches (R env-steps each).  FETCH_SIZE is scaled x2 (gfx950 correction,
/opt/skills/guides/MI355X_MICROARCH.md HBM section), WRITE_SIZE as read; KiB -> bytes.
usage: python tools/pmc_rollout_summary.py <dir with FETCH_SIZE/ WRITE_SIZE/> <R> <n_envs> [out.json]
"""
import csv
import json
import os
import sys


def launches(path, ctr):
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != ctr or not r["Kernel_Name"].startswith("void gm_step_kernel"):
            continue
        rows.append(((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6, float(r["Counter_Value"]),
                     int(r["Dispatch_Id"])))
    ms = sorted(x[0] for x in rows)
    med = ms[len(ms) // 2]
    roll = [x for x in rows if x[0] > 5 * med]
    return roll, med


def main(d, R, n, out=None):
    R, n = int(R), int(n)
    res = {"kernel": "gm_step_kernel", "n_envs": n, "env_steps_per_launch": R}
    for ctr, scale in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
        roll, med = launches(os.path.join(d, ctr, "run_counter_collection.csv"), ctr)
        assert roll, ctr
        b = sum(v for _, v, _ in roll) / len(roll) * 1024 * scale
        res[ctr.lower().replace("_size", "") + "_bytes_per_launch"] = b
        res[ctr.lower().replace("_size", "") + "_launches"] = len(roll)
        res[ctr.lower().replace("_size", "") + "_launch_ms"] = sum(x for x, _, _ in roll) / len(roll)
        res["per_step_launch_ms_median"] = med
    res["bytes_per_launch"] = res["fetch_bytes_per_launch"] + res["write_bytes_per_launch"]
    res["bytes_per_env_step"] = res["bytes_per_launch"] / (R * n)
    res["source"] = (f"tools/pmc_rollout.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over "
                     f"bench.py --steps 10 --warmup 10 (headline only), the {R}-env-step gm_rollout launches; "
                     f"FETCH_SIZE KiB x1024 x2 (gfx950 correction), WRITE_SIZE KiB x1024")
    s = json.dumps(res, indent=1)
    print(s)
    if out:
        open(out, "w").write(s + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
