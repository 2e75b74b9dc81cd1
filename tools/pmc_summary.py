"""Summarise a tools/pmc_r04.sh run: per gm_step_kernel dispatch (the last `last` of each
pass, the C3 steady state) the SQ / SQC / TCP counters, normalised per env-step and per
env-substep, plus FETCH_SIZE / WRITE_SIZE per 4096-env launch (gfx950: FETCH_SIZE x 2).
usage: python tools/pmc_summary.py <pmc dir> [envs] [last]"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
envs = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
last = int(sys.argv[3]) if len(sys.argv) > 3 else 3
S = 63


def step_rows(path):
    rows = list(csv.DictReader(open(path)))
    per = {}
    for r in rows:
        if "gm_step_kernel" not in r["Kernel_Name"]:
            continue
        per.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
        per[int(r["Dispatch_Id"])]["_grid"] = int(r["Grid_Size"])
    ids = sorted(per)
    return [per[i] for i in ids]


out = {}
for name in ("sq1", "sq2", "sq3", "sqc", "tcp"):
    f = glob.glob(os.path.join(d, name, "*counter_collection.csv"))
    if not f:
        continue
    rows = step_rows(f[0])[-last:]
    keys = sorted({k for r in rows for k in r if not k.startswith("_")})
    for k in keys:
        out[k] = sum(r.get(k, 0.0) for r in rows) / len(rows)
res = {"envs": envs, "substeps_per_env_step": S, "per_launch": out}
w = out.get("SQ_WAVE_CYCLES")
if w:
    res["wave_cycle_fractions"] = {k: round(out[k] / w, 4) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                                     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM")
                                   if k in out}
per_sub = {}
for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
          "SQ_INSTS_BRANCH", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64"):
    if k in out:
        per_sub[k] = round(out[k] / (envs * S), 1)
res["per_env_substep"] = per_sub
if "SQ_THREAD_CYCLES_VALU" in out and "SQ_ACTIVE_INST_VALU" in out:
    res["valu_lane_utilisation"] = round(out["SQ_THREAD_CYCLES_VALU"] / (64 * out["SQ_ACTIVE_INST_VALU"]), 4)
if "SQC_ICACHE_HITS" in out:
    h, m = out["SQC_ICACHE_HITS"], out.get("SQC_ICACHE_MISSES", 0.0)
    res["icache_hit_rate"] = round(h / (h + m), 4)
if "SQ_INSTS_VMEM_RD" in out and "SQ_INST_LEVEL_VMEM" in out:
    res["vmem_mean_latency_cycles"] = round(out["SQ_INST_LEVEL_VMEM"] / max(out["SQ_INSTS_VMEM_RD"] + out.get("SQ_INSTS_VMEM_WR", 0), 1), 1)
if "SQ_INSTS_LDS" in out and "SQ_INST_LEVEL_LDS" in out:
    res["lds_mean_latency_cycles"] = round(out["SQ_INST_LEVEL_LDS"] / max(out["SQ_INSTS_LDS"], 1), 1)
if "SQ_INSTS_SMEM" in out and "SQ_INST_LEVEL_SMEM" in out:
    res["smem_mean_latency_cycles"] = round(out["SQ_INST_LEVEL_SMEM"] / max(out["SQ_INSTS_SMEM"], 1), 1)
tr = {}
for name, key in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    f = glob.glob(os.path.join(d, name, "*counter_collection.csv"))
    if f:
        rows = [r for r in step_rows(f[0]) if r.get("_grid", 0) > 0]
        vals = [r[key] for r in rows if key in r]
        if vals:
            tr[key + "_KiB_mean"] = sum(vals) / len(vals)
if tr:
    fb = tr.get("FETCH_SIZE_KiB_mean", 0) * 1024 * 2
    wb = tr.get("WRITE_SIZE_KiB_mean", 0) * 1024
    tr.update({"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb})
    res["traffic"] = tr
print(json.dumps(res, indent=1))
