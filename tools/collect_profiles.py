"""Copy a round's GPU profile outputs from gpurun_out/<tag>/ into profiles/ (tracked):
kernel stats, filtered PMC rows for the gm_* kernels, the HBM traffic summary bench.py
reads, SQ occupancy counters, the phase profile and the bench line."""
import csv, json, os, shutil, sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join("gpurun_out", tag)
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


for name in ("pmc_fetch", "pmc_write", "pmc_sq"):
    rs = rows(name)
    with open(os.path.join(dst, f"{tag}_{name}.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=keep)
        w.writeheader()
        for r in rs:
            w.writerow({k: r[k] for k in keep})

n_envs = 4096
step = lambda r: 'gm_step_kernel' in r['Kernel_Name'] and int(r['Grid_Size']) == 64 * n_envs
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
