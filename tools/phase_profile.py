"""Developer probe: per-phase cycle breakdown of the fused env-step kernel."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd')]
import numpy as np
import gmx
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
s = gmx.canonical_settings(noise=True, seed=5)
env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=s, seed=5)
env.reset()
rng = np.random.default_rng(0)
for t in range(3):
    env.step(rng.uniform(-1, 1, size=(n, env.n_actions)).astype(np.float32))
tot = np.zeros(env.N_PHASE)
for t in range(3):
    env.set_action(rng.uniform(-1, 1, size=(n, env.n_actions)).astype(np.float32))
    ph = env.step_profiled().astype(np.float64)
    tot += ph.mean(axis=0)
tot /= 3
S = env.cfg.sim_steps_per_action if hasattr(env.cfg, 'sim_steps_per_action') else 63
TOP = [0, 1, 2, 5, 6, 8, 9, 10]
allc = tot[TOP].sum()
print(f"n={n} mean cycles per env-step (lane 0) total {allc:.3e}  per substep {allc/63:.3e}")
for k, name in enumerate(env.PHASES):
    if k in (22, 23, 25, 26, 27):
        continue
    if name == "-":
        continue
    if name.startswith("e:"):
        print(f"  {name:18s} {tot[k]:10.0f} cyc/env-step  (= {tot[k]/63:.0f} per substep)")
    else:
        print(f"  {name:18s} {tot[k]/63:10.0f} cyc/substep  {100*tot[k]/allc:5.1f}%")
print(f"  outlined-call overhead {(tot[22] - tot[[0, 1, 2, 5, 6, 8]].sum())/63:10.0f} cyc/substep (prologue/epilogue, CSR save/restore)")
print(f"  whole env-step on one wave {tot[23]:.3e} cyc (phases account for {100*(allc+tot[18:22].sum())/max(tot[23],1):.1f}%)")
print(f"  rows per substep {tot[env.PH_NEFC]/63:.1f}; Newton iterations per solve {tot[env.PH_NEWTON]/63:.3f}; line-search evals per solve {tot[env.PH_LS]/63:.3f}")
ncon, _, _, _ = env.debug_substep()
print("ncon per env: mean %.2f  max %d  histogram %s" % (ncon.mean(), ncon.max(), np.bincount(ncon, minlength=16).tolist()))
