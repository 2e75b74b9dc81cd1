"""Developer probe: substep-level GPU vs oracle comparison inside one env-step."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'),
                os.path.join(os.path.dirname(__file__), '..', 'tests')]
import numpy as np
import gmx, oracle_lib
x = float(sys.argv[1]); T0 = int(sys.argv[2])
s = gmx.canonical_settings(noise=False, seed=5)
env = gmx.BatchedGripperEnv(1, object_set="set1_synthetic", settings=s, seed=5)
sp = env.make_spawn(x=x, y=x, idx=0)
env.reset(spawn=sp)
o = oracle_lib.OracleEnv(env.model, env.cfg, env.objects, 0)
o.reset(sp[0])
rng = np.random.default_rng(1234)
for t in range(T0):
    a = rng.uniform(-1, 1, size=(1, env.n_actions)).astype(np.float32)
    env.step(a); o.step(a[0])
a = rng.uniform(-1, 1, size=(1, env.n_actions)).astype(np.float32)
env.set_action(a); o.set_action(a[0])
for k in range(env.cfg.sim_steps_per_action):
    n1, c1, f1, q1 = env.debug_substep()
    n2, c2, f2, q2 = o.debug_substep()
    qg, vg, _ = env.state(); qo, vo, _ = o.state()
    print(f"sub {k:2d} ncon {n1[0]}/{n2} dq {np.abs(qg[0]-qo).max():.2e} dv {np.abs(vg[0]-vo).max():.2e} "
          f"dqacc {np.abs(q1[0][:env.model.nv]-q2).max():.2e} |qacc| {np.abs(q2).max():.2e}")
    if (n1[0] or n2) and 35 <= k <= 38:
        for c in range(max(n1[0], n2)):
            print(f"     c{c}: gpu g{int(c1[0][c][13])}-{int(c1[0][c][14])} d={c1[0][c][0]:.3e} p={c1[0][c][1:4]}"
                  f" | ref g{int(c2[c][13])}-{int(c2[c][14])} d={c2[c][0]:.3e} p={c2[c][1:4]}")
        print(f"     efc gpu {f1[0][:24]}\n     efc ref {f2[:24]}")
        print(f"     qacc gpu {q1[0][:env.model.nv]}\n     qacc ref {q2}")
    if k > 40 and np.abs(vg[0]-vo).max() > 1e-2: break
