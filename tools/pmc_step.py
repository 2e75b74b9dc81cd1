"""Developer probe: a few fused env-step launches for PMC counter collection."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd')]
import numpy as np
import gmx
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", seed=1)
env.reset()
rng = np.random.default_rng(0)
for t in range(3):
    env.step(rng.uniform(-1, 1, size=(n, env.n_actions)).astype(np.float32))
print("done")
