"""On-device DQN policy: VariableNetwork forward + select_action
(rl/networks.py:7-41, rl/agents/DQN.py:184-209) fused in gm_policy_kernel.

CPU tests pin the host-side parameter layout (gm_policy_pack) and the torch-facing
helpers; the GPU tests compare the kernel's softmax outputs and actions with a torch f32
forward of the same network on the env's own observations (tolerance below)."""
import math

import numpy as np
import pytest

import gmx
from gmx import policy as gp

Q_ATOL = 2e-6     # f32 softmax outputs: MFMA k-ordered fmaf chain vs torch's CPU GEMM order
CANON = [63, 150, 100, 50, 8]


def unpack_weights(sizes, packed):
    """Invert the documented B-fragment layout: lane l of (tile t, k step s) holds
    W[16 t + (l & 15)][4 s + (l >> 4)]."""
    out = []
    off = 0
    for l in range(len(sizes) - 1):
        n_in, n_out = sizes[l], sizes[l + 1]
        kpad = (n_in + 3) // 4 * 4
        tiles = (n_out + 15) // 16
        W = np.zeros((tiles * 16, kpad), dtype=np.float32)
        for t in range(tiles):
            for s in range(kpad // 4):
                blk = packed[off + (t * (kpad // 4) + s) * 64: off + (t * (kpad // 4) + s + 1) * 64]
                for lane in range(64):
                    W[16 * t + (lane & 15), 4 * s + (lane >> 4)] = blk[lane]
        off += tiles * (kpad // 4) * 64
        b = packed[off: off + tiles * 16]
        off += tiles * 16
        out.append((W, b))
    assert off == len(packed)
    return out


@pytest.mark.parametrize("sizes", [CANON, [5, 7, 3], [63, 64, 64, 8], [1, 256, 1]])
def test_pack_layout_round_trip(sizes):
    p = gp.init_params(sizes, seed=3)
    packed = gp.pack(sizes, p)
    off = 0
    for (W, b), l in zip(unpack_weights(sizes, packed), range(len(sizes) - 1)):
        n_in, n_out = sizes[l], sizes[l + 1]
        Wref = p[off: off + n_in * n_out].reshape(n_out, n_in); off += n_in * n_out
        bref = p[off: off + n_out]; off += n_out
        np.testing.assert_array_equal(W[:n_out, :n_in], Wref)
        assert not W[n_out:].any() and not W[:, n_in:].any()      # zero padding
        np.testing.assert_array_equal(b[:n_out], bref)
        assert not b[n_out:].any()


def test_pack_rejects_unsupported_sizes():
    with pytest.raises(ValueError):
        gp.pack([63, 300, 8], gp.init_params([63, 300, 8]))
    with pytest.raises(ValueError):
        gp.pack([4] * 11, gp.init_params([4] * 11))


def test_state_dict_round_trip_and_eps():
    torch = pytest.importorskip("torch")
    torch.manual_seed(0)
    layers = torch.nn.ModuleList([torch.nn.Linear(a, b) for a, b in zip(CANON[:-1], CANON[1:])])
    sd = {f"linear.{i}.{k}": v for i, m in enumerate(layers) for k, v in m.state_dict().items()}
    sizes, flat = gp.params_from_state_dict(sd)
    assert sizes == CANON
    assert flat[:150 * 63].reshape(150, 63).tolist() == layers[0].weight.detach().numpy().tolist()
    # DQN.py:195-198 with the agent defaults (eps_start 0.9, eps_end 0.05, eps_decay 1000)
    assert gp.eps_threshold(0) == pytest.approx(0.9)
    assert gp.eps_threshold(1000) == pytest.approx(0.05 + 0.85 * math.exp(-1))


def torch_forward(sizes, params, obs):
    """VariableNetwork.forward in torch f32 (rl/networks.py:26-38)."""
    import torch
    x = torch.from_numpy(np.asarray(obs, dtype=np.float32))
    off = 0
    n = len(sizes) - 1
    for l in range(n):
        W = torch.from_numpy(params[off: off + sizes[l] * sizes[l + 1]].reshape(sizes[l + 1], sizes[l])); off += W.numel()
        b = torch.from_numpy(params[off: off + sizes[l + 1]]); off += sizes[l + 1]
        x = torch.nn.functional.linear(x, W, b)
        if l < n - 1:
            x = torch.relu(x)
    return torch.softmax(x, dim=1).numpy()


def discrete_env(n, seed=11):
    s = gmx.canonical_settings(noise=False, seed=seed)
    s.continous_actions = 0
    env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=s, seed=seed)
    return env


@pytest.mark.gpu
def test_policy_matches_torch_forward():
    env = discrete_env(300)
    assert env.n_actions == 8 and env.n_obs == 63
    env.reset()
    rng = np.random.default_rng(0)
    for _ in range(3):      # move the observations away from the reset state
        env.step(rng.integers(0, 8, size=env.n_envs), discrete=True)
    obs = env.observation()
    pol = gmx.DevicePolicy(env, seed=5)
    pol.act(eps=0.0, seed=1, decision=0)
    acts, q = pol.read()
    qref = torch_forward(pol.sizes, pol.params, obs)
    np.testing.assert_allclose(q, qref, rtol=0, atol=Q_ATOL)
    top2 = np.sort(qref, axis=1)[:, -2:]
    clear = (top2[:, 1] - top2[:, 0]) > 4 * Q_ATOL
    assert clear.mean() > 0.9
    np.testing.assert_array_equal(acts[clear], np.argmax(qref, axis=1)[clear])
    pol.close()


@pytest.mark.gpu
def test_policy_epsilon_and_rollout():
    env = discrete_env(512, seed=4)
    env.reset()
    pol = gmx.DevicePolicy(env, seed=2)
    pol.act(eps=1.0, seed=9, decision=0)        # all random
    a_rand, _ = pol.read()
    assert a_rand.min() >= 0 and a_rand.max() < 8
    counts = np.bincount(a_rand, minlength=8)
    assert counts.min() > 30                      # 512 draws over 8 actions
    pol.act(eps=1.0, seed=9, decision=0)
    np.testing.assert_array_equal(pol.read()[0], a_rand)   # counter-based: reproducible
    pol.act(eps=0.0, seed=9, decision=1)
    a_greedy, q = pol.read()
    np.testing.assert_array_equal(a_greedy, np.argmax(q, axis=1))
    # a short fully on-device rollout: policy -> env step -> policy ...
    for t in range(5):
        pol.act(eps=gmx.eps_threshold(t), seed=9, decision=t)
        env.action_step()
    obs = env.observation()
    assert np.isfinite(obs).all()
    pol.close()
