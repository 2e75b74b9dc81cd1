"""Copy a round's GPU profile outputs from gpurun_out/<tag>/ into profiles/ (tracked):
kernel stats, filtered PMC rows for the gm_* kernels, the HBM traffic summary bench.py
reads, SQ occupancy counters, the phase profile and the bench line."""
import csv, json, os, shutil, sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join("gpurun_out", tag)
tag = sys.argv[2] if len(sys.argv) > 2 else tag      # output prefix (the round name)
dst = "profiles"
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
shutil.copy(os.path.join(src, "phase_profile.txt"), os.path.join(dst, f"{tag}_phase_profile.txt"))
shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag}_bench.json"))
keep = ['Dispatch_Id', 'Grid_Size', 'Kernel_Name', 'Workgroup_Size', 'LDS_Block_Size', 'Scratch_Size', 'VGPR_Count',
        'Accum_VGPR_Count', 'SGPR_Count', 'Counter_Name', 'Counter_Value', 'Start_Timestamp', 'End_Timestamp']


def rows(name):
    f = os.path.join(src, name, "run_counter_collection.csv")
    return [r for r in csv.DictReader(open(f)) if r['Kernel_Name'].startswith('gm_') or 'gm_step_kernel' in r['Kernel_Name']]


for name in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_lanes"):
    if not os.path.exists(os.path.join(src, name)):
        continue
    rs = rows(name)
    with open(os.path.join(dst, f"{tag}_{name}.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=keep)
        w.writeheader()
        for r in rs:
            w.writerow({k: r[k] for k in keep})

n_envs = 4096
# the 4096-env launches: one workgroup per env (one-shot) or per resident wave slot
# (chunked dispatch, 2048 on MI355X); the bench's small launches (settle, C2) excluded
step = lambda r: 'gm_step_kernel' in r['Kernel_Name'] and int(r['Grid_Size']) >= 64 * 1024
fe = [float(r['Counter_Value']) for r in rows("pmc_fetch") if step(r)]
wr = [float(r['Counter_Value']) for r in rows("pmc_write") if step(r)]
fetch = sum(fe) / len(fe) * 1024 * 2
write = sum(wr) / len(wr) * 1024
json.dump({"kernel": "gm_step_kernel", "n_envs": n_envs, "bytes_per_launch": fetch + write,
           "fetch_bytes_corrected": fetch, "write_bytes": write, "launches": len(fe),
           "source": f"profiles/{tag}_pmc_fetch.csv + {tag}_pmc_write.csv (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in "
                     "separate passes over bench.py --steps 3): FETCH_SIZE KiB x1024 x2 (gfx950 correction), "
                     "WRITE_SIZE KiB x1024, averaged over the 4096-env step launches"},
          open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
print(open(os.path.join(dst, "pmc_traffic.json")).read())

# per-dispatch durations of the 4096-env step launches from the kernel trace (the stats
# summary's average also holds the one-env calibrate_reset settle launch at gm_create)
tr = [r for r in csv.DictReader(open(os.path.join(src, "stats", "run_kernel_trace.csv")))
      if 'gm_step_kernel' in r['Kernel_Name']]
grid = lambda r: int(r.get('Grid_Size_X') or r.get('Grid_Size') or 0)
durs = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in tr if grid(r) >= 64 * 1024]
summ = {"kernel": "gm_step_kernel", "grid_envs": n_envs, "launches": len(durs),
        "avg_ms_all": sum(durs) / len(durs), "avg_ms_after_first": sum(durs[1:]) / max(len(durs) - 1, 1),
        "min_ms": min(durs), "max_ms": max(durs), "durations_ms": durs,
        "source": f"gpurun_out/{sys.argv[1] if len(sys.argv) > 1 else tag}/stats/run_kernel_trace.csv "
                  "(rocprofv3 --kernel-trace --stats over bench.py --steps 5 --warmup 1)"}
json.dump(summ, open(os.path.join(dst, f"{tag}_step_kernel_trace.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in summ.items() if k != "durations_ms"}))
