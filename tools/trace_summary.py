"""Summarise a rocprofv3 --kernel-trace CSV for the bench's timed launches.

The bench's headline drives gm_rollout launches of R env-steps each (R in the JSON's
roofline.env_steps_per_launch); the same process also runs per-step launches (the untimed
pre-roll, the parity step, side lines), so rocprofv3's per-kernel average mixes the two.
This picks the step kernel's dispatches by workgroup count and duration class and reports
the rollout launches' mean duration, to set beside roofline.kernel_launch_ms.

usage: python tools/trace_summary.py <run_kernel_trace.csv> <bench.json> [out.json]
"""
import csv
import json
import sys


def main(trace, bench, out=None):
    b = json.loads(open(bench).read().strip().split("\n")[-1])
    rf = b["roofline"]
    per_launch = rf.get("env_steps_per_launch", 1)
    rows = []
    for r in csv.DictReader(open(trace)):
        if not r["Kernel_Name"].startswith("void gm_step_kernel"):
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6   # ms
        rows.append(dict(name=r["Kernel_Name"].split("(")[0], ms=d, wg=int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]),
                         wgsize=int(r["Workgroup_Size_X"]), vgpr=int(r["VGPR_Count"]), lds=int(r["LDS_Block_Size"]),
                         scratch=int(r["Scratch_Size"])))
    # rollout launches: duration above (per_launch - 0.5) x the per-step launches' median
    steps = sorted(x["ms"] for x in rows if x["ms"] > 1.0)
    med = steps[len(steps) // 2] if steps else 0.0
    roll = [x for x in rows if per_launch > 1 and x["ms"] > (per_launch - 0.5) * med / 1.3]
    one = [x for x in rows if x not in roll and x["ms"] > 1.0]
    res = dict(
        trace=trace, dispatches=len(rows),
        rollout_launches=len(roll),
        rollout_launch_ms_mean=sum(x["ms"] for x in roll) / len(roll) if roll else None,
        rollout_ms_per_env_step=(sum(x["ms"] for x in roll) / len(roll) / per_launch) if roll else None,
        per_step_launches=len(one),
        per_step_launch_ms_median=sorted(x["ms"] for x in one)[len(one) // 2] if one else None,
        bench_kernel_launch_ms=rf.get("kernel_launch_ms"), bench_kernel_avg_ms=rf.get("kernel_avg_ms"),
        env_steps_per_launch=per_launch,
        kernels={x["name"] + f" wg{x['wgsize']}": dict(vgpr=x["vgpr"], lds=x["lds"], scratch=x["scratch"]) for x in rows},
    )
    if roll and rf.get("kernel_launch_ms"):
        res["trace_vs_bench_launch"] = res["rollout_launch_ms_mean"] / rf["kernel_launch_ms"]
    s = json.dumps(res, indent=1)
    print(s)
    if out:
        open(out, "w").write(s + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
