"""Developer probe: per-step GPU vs oracle divergence for one scenario."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'),
                os.path.join(os.path.dirname(__file__), '..', 'tests')]
import numpy as np
import gmx, oracle_lib
x = float(sys.argv[1]) if len(sys.argv) > 1 else 0.3
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
s = gmx.canonical_settings(noise=False, seed=5)
env = gmx.BatchedGripperEnv(1, object_set="set1_synthetic", settings=s, seed=5)
sp = env.make_spawn(x=x, y=x, idx=0)
env.reset(spawn=sp)
o = oracle_lib.OracleEnv(env.model, env.cfg, env.objects, 0)
o.reset(sp[0])
rng = np.random.default_rng(1234)
m = env.model
seg = [d for f in range(3) for d in range(m.dof_seg[f], m.dof_seg[f] + m.n_seg)]
for t in range(steps):
    a = rng.uniform(-1, 1, size=(1, env.n_actions)).astype(np.float32)
    obs, rew, term, trunc = env.step(a)
    obs_o, r_o, d_o = o.step(a[0])
    q, v, _ = env.state()
    qo, vo, _ = o.state()
    big = np.abs(obs_o) >= 1e-3
    rel = (np.abs(obs[0] - obs_o)[big] / np.abs(obs_o[big])).max() if big.any() else 0
    dq = np.abs(q[0] - qo)
    segrel = (np.abs(q[0][seg] - qo[seg]) / np.maximum(np.abs(qo[seg]), 1e-9)).max()
    dd = np.abs(obs[0] - obs_o); k = int(np.argmax(dd / np.maximum(np.abs(obs_o), 1e-3)))
    print(f"   worst obs[{k}] gpu={obs[0][k]:.6f} ref={obs_o[k]:.6f} rew {rew[0]:.4f}/{r_o:.4f} done {term[0]}/{d_o}")
    print(f"t={t:2d} obs_rel={rel:.2e} obs_abs={np.abs(obs[0]-obs_o).max():.2e} seg_q_rel={segrel:.2e} "
          f"seg_q_abs={dq[seg].max():.2e} motor_q_abs={dq[[m.dof_base, m.dof_palm] + m.dof_pris + m.dof_rev].max():.2e} "
          f"obj_abs={dq[m.dof_obj:m.dof_obj+3].max():.2e} maxseg={np.abs(qo[seg]).max():.2e} v_abs={np.abs(v[0]-vo).max():.2e}", flush=True)
