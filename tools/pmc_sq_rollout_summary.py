"""SQ counters of the headline's rollout launches from tools/pmc_r06.sh (passes sq1, sq2):
the step kernel's dispatches over 5x the per-step launches' median duration are the
gm_rollout launches (R env-steps of every env); counters per launch, per env-substep
(R x n_envs x S) and as wave-cycle fractions, the VALU lane utilisation.
usage: python tools/pmc_sq_rollout_summary.py <dir> <R> <n_envs> [out.json]"""
import csv
import json
import os
import sys

S = 63


def rollout_rows(path):
    per = {}
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith("void gm_step_kernel"):
            continue
        d = per.setdefault(int(r["Dispatch_Id"]), {"_ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ms = sorted(v["_ms"] for v in per.values())
    med = ms[len(ms) // 2]
    return [v for v in per.values() if v["_ms"] > 5 * med]


def main(d, R, n, out=None):
    R, n = int(R), int(n)
    acc = {}
    launches = {}
    for name in ("sq1", "sq2"):
        rows = rollout_rows(os.path.join(d, name, "run_counter_collection.csv"))
        launches[name] = len(rows)
        for k in sorted({k for r in rows for k in r if not k.startswith("_")}):
            acc[k] = sum(r.get(k, 0.0) for r in rows) / len(rows)
    subs = R * n * S
    res = {"envs": n, "env_steps_per_launch": R, "substeps_per_env_step": S, "launches_per_pass": launches,
           "per_launch": acc}
    w = acc.get("SQ_WAVE_CYCLES")
    if w:
        res["wave_cycle_fractions"] = {k: round(acc[k] / w, 4) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                         "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                                                         "SQ_ACTIVE_INST_LDS") if k in acc}
    res["per_env_substep"] = {k: round(acc[k] / subs, 1) for k in (
        "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VALU_FMA_F64",
        "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64") if k in acc}
    if "SQ_THREAD_CYCLES_VALU" in acc and "SQ_ACTIVE_INST_VALU" in acc:
        res["valu_lane_utilisation"] = round(acc["SQ_THREAD_CYCLES_VALU"] / (64 * acc["SQ_ACTIVE_INST_VALU"]), 4)
    if "SQ_LDS_BANK_CONFLICT" in acc and "SQ_ACTIVE_INST_LDS" in acc:
        res["lds_bank_conflict_fraction_of_lds_active"] = round(acc["SQ_LDS_BANK_CONFLICT"] / acc["SQ_ACTIVE_INST_LDS"], 4)
    res["source"] = (f"tools/pmc_r06.sh: rocprofv3 --pmc SQ passes (sq1, sq2; each its own run) over bench.py "
                     f"--steps 10 --warmup 10 (headline only), the {R}-env-step gm_rollout launches of the C3 benchmark mix")
    s = json.dumps(res, indent=1)
    print(s)
    if out:
        open(out, "w").write(s + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
