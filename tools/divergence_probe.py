"""Where do device and oracle separate inside one env-step?  Rolls the C3 grasp batch,
picks the envs whose qpos differs most after one env-step from identical states, and
replays those envs substep by substep on both sides, printing the first substeps where
the difference jumps (GPU box)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "gripper-mujoco_amd"), os.path.join(REPO, "tests")]
import gmx as gm
import oracle_lib as ol
from test_grasp_parity import rollout, obs_err

SNAP = int(sys.argv[1]) if len(sys.argv) > 1 else 52
env, snaps = rollout(gm, 4096, "set6_synthetic", 1234, steps=SNAP + 1, snaps=(SNAP,))
sn = snaps[0]
obs_o, rew_o, done_o, after_o = ol.batch_step(env.model, env.cfg, env.objects, sn["rec"], actions=sn["a"])
dv, ov = gm.env_state_view(sn["after"]), gm.env_state_view(after_o)
dq = np.abs(dv["qpos"] - ov["qpos"]).max(axis=1)
rel, ab = obs_err(sn["obs"], obs_o)
worst = np.argsort(-dq)[:16]
print("worst qpos diffs", dq[worst], "obs rel", rel[worst])
print("objects", dv["obj_index"][worst], "types", dv["obj_type"][worst])
s = gm.canonical_settings(noise=False, seed=1234)
sub = gm.BatchedGripperEnv(16, object_set="set6_synthetic", settings=s, seed=1234)
rec = sn["rec"][worst].copy()
# apply the step's actions on both sides first (set_action), then substep in lockstep
sub.set_env_states(rec)
sub.set_action(sn["a"][worst])
rec_a = sub.env_states()
rec_o = rec_a.copy()
prev = np.zeros(16)
for i in range(env.cfg.sim_steps_per_action):
    sub.set_env_states(rec_a)
    ncon, con, efc, qacc, nefc, w = sub.debug_substep(full=True)
    rec_a = sub.env_states()
    ncon_o, nefc_o, con_o, efc_o, qacc_o, w_o, rec_o = ol.batch_substep(env.model, env.cfg, env.objects, rec_o)
    va, vo = gm.env_state_view(rec_a), gm.env_state_view(rec_o)
    d = np.abs(va["qpos"] - vo["qpos"]).max(axis=1)
    for j in range(16):
        if d[j] > max(1e3 * prev[j], 1e-13) and d[j] > 1e-12:
            geo = np.abs(con[j, :, :13] - con_o[j, :, :13]).max()
            print(f"substep {i} env {worst[j]}: qpos diff {prev[j]:.2e} -> {d[j]:.2e}; ncon {ncon[j]}/{ncon_o[j]} "
                  f"nefc {nefc[j]}/{nefc_o[j]} geo {geo:.2e} efc {np.abs(efc[j]-efc_o[j]).max():.2e}")
            for c in range(max(ncon[j], ncon_o[j])):
                print("    dev", np.round(con[j, c, [0, 1, 2, 3, 4, 5, 6, 13, 14]], 7).tolist())
                print("    orc", np.round(con_o[j, c, [0, 1, 2, 3, 4, 5, 6, 13, 14]], 7).tolist())
    dv_ = np.abs(va["qvel"] - vo["qvel"]).max(axis=1)
    print(f"sub {i:2d} env0 dq {d[0]:.2e} dv {dv_[0]:.2e} ncon {ncon[0]} nefc {nefc[0]} geo {np.abs(con[0,:,:13]-con_o[0,:,:13]).max():.2e} "
          f"efc {np.abs(efc[0]-efc_o[0]).max():.2e} qacc {np.abs(qacc[0]-qacc_o[0]).max():.2e} | env1 dq {d[1]:.2e} ncon {ncon[1]}")
    prev = np.maximum(d, prev)
print("final", prev)
