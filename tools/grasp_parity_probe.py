"""Diagnostics for tests/test_grasp_parity.py without asserting: per snapshot, how many
envs exceed each bound and by how much (run on the GPU box)."""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "gripper-mujoco_amd"), os.path.join(REPO, "tests")]
import gmx as gm
import oracle_lib as ol
from test_grasp_parity import rollout, obs_err, SNAPS

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
SNAPS = tuple(int(x) for x in sys.argv[3].split(",")) if len(sys.argv) > 3 else SNAPS
oset = sys.argv[2] if len(sys.argv) > 2 else "set6_synthetic"
t0 = time.time()
env, snaps = rollout(gm, n, oset, 1234, steps=max(SNAPS) + 1, snaps=SNAPS)
print(f"rollout {time.time()-t0:.1f}s", flush=True)
for sn in snaps:
    t1 = time.time()
    obs_o, rew_o, done_o, after_o = ol.batch_step(env.model, env.cfg, env.objects, sn["rec"], actions=sn["a"])
    dv, ov = gm.env_state_view(sn["after"]), gm.env_state_view(after_o)
    rel, ab = obs_err(sn["obs"], obs_o)
    bad = (rel > 1e-4) | (ab > 1e-4)
    dq = np.abs(dv["qpos"] - ov["qpos"]).max(axis=1)
    exact = int((dv["qpos"] == ov["qpos"]).all(axis=1).sum())
    exact_obs = int((sn["obs"] == obs_o).all(axis=1).sum())
    mism = {f: int((dv[f] != ov[f]).reshape(n, -1).any(axis=1).sum()) for f in ("bev_row", "lev_row", "rng", "ring_i", "lock_active", "old_x", "old_z")}
    print(f"k={sn['k']} oracle {time.time()-t1:.1f}s bad_obs={bad.sum()} rel_max={rel.max():.2e} p99={np.percentile(rel,99):.2e} "
          f"abs_max={ab.max():.2e} done_dev={int(sn['done'].sum())} done_or={int(done_o.sum())} done_mism={int((sn['done'].astype(np.uint8)!=done_o).sum())} "
          f"rew_maxd={np.abs(sn['rew']-rew_o).max():.2e} qpos_max={dq.max():.2e} qpos_p50={np.median(dq):.2e} qpos_bitexact={exact}/{n} obs_bitexact={exact_obs}/{n} mism={mism}", flush=True)
    if sn is snaps[0] or sn is snaps[-1]:
        od = (sn["obs"] != obs_o)
        print("   obs mismatch count per index", od.sum(axis=0).tolist())
        for f in ("qpos", "qvel", "qacc_warm", "base", "last_read", "lock_q", "time"):
            a, b = dv[f].reshape(n, -1), ov[f].reshape(n, -1)
            print(f"   {f}: envs differing {int((a != b).any(axis=1).sum())}, per-column {(a != b).sum(axis=0).tolist()[:48]}")
        for g in ("end", "next"):
            for f in ("x", "y", "z", "th"):
                print(f"   {g}.{f}: envs differing {int((dv[g][f] != ov[g][f]).sum())}")
        rd, ro = dv["ring"], ov["ring"]
        print("   ring streams differing (envs):", [int((rd[:, st] != ro[:, st]).any(axis=1).sum()) for st in range(rd.shape[1])])
        # the same env-step from the device's states but with the input state == oracle's: isolate
    if bad.any():
        e = int(np.argmax(rel))
        print("   worst env", e, "obj", int(dv["obj_index"][e]), "obs dev", np.round(sn["obs"][e], 5).tolist())
        print("   worst env oracle", np.round(obs_o[e], 5).tolist())
for sn in snaps:
    env.set_env_states(sn["rec"])
    ncon, con, efc, qacc, nefc, w = env.debug_substep(full=True)
    ncon_o, nefc_o, con_o, efc_o, qacc_o, w_o, after_o = ol.batch_substep(env.model, env.cfg, env.objects, sn["rec"])
    fs = np.maximum(1.0, np.abs(efc_o).max(axis=1, keepdims=True))
    qs = np.maximum(1.0, np.abs(qacc_o).max(axis=1, keepdims=True))
    print(f"sub k={sn['k']} ncon_mism={int((ncon!=ncon_o).sum())} nefc>32={int((nefc>32).sum())} nefc_max={nefc.max()} "
          f"pair_mism={int((con[:,:,13:15]!=con_o[:,:,13:15]).any(axis=(1,2)).sum())} geo={np.abs(con[:,:,:13]-con_o[:,:,:13]).max():.2e} "
          f"efc={np.abs((efc-efc_o)/fs).max():.2e} qacc={np.abs((qacc-qacc_o)/qs).max():.2e} wr={np.abs(w-w_o).max():.2e}", flush=True)
last = gm.env_state_view(snaps[-1]["after"])
print({nm: int((last["bev_abs"][:, i] > 0).sum()) for i, nm in enumerate(gm.BINARY_EVENTS)})
