"""The C-ABI library on the CPU: it loads, exports every entry point include/*.h
declares, and its host-side model / configuration builders reproduce the
reference's canonical configuration (no GPU needed)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for f in os.listdir(os.path.join(REPO, "include")):
        if not f.endswith(".h"):
            continue
        txt = open(os.path.join(REPO, "include", f)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(gm_\w+)\s*\(", txt, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def test_header_declares_the_boundary():
    names = declared_symbols()
    for required in ("gm_create", "gm_destroy", "gm_reset", "gm_set_action", "gm_set_discrete_action",
                     "gm_step", "gm_get_obs", "gm_get_reward_done", "gm_get_event_rows", "gm_n_obs",
                     "gm_n_actions", "gm_last_error", "gm_update_config", "gm_autoreset"):
        assert required in names


def test_library_exports_every_declared_symbol(gm):
    lib = C.CDLL(gm.LIB_PATH)
    missing = [n for n in declared_symbols() if not hasattr(lib, n)]
    assert not missing, f"libgm.so lacks {missing}"


def test_library_is_gfx950_code_object(gm):
    blob = open(gm.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"gm_step_kernel" in blob


def test_struct_sizes_match_ctypes(gm):
    lib = gm.load_library()
    assert lib.gm_struct_size(0) == C.sizeof(gm.Settings)
    assert lib.gm_struct_size(5) == C.sizeof(gm.ModelParams)
    assert lib.gm_struct_size(99) == -1
    # the raw per-env state record and its numpy view (checkpoint / oracle hand-off)
    assert lib.gm_env_state_size() == gm.env_state_dtype().itemsize
    import oracle_lib
    assert oracle_lib.lib().or_state_size() == lib.gm_env_state_size()


def test_spawn_draws_are_shard_independent(gm):
    """gm_spawn_int / spawn_draws: keyed on the global env id, not on the shard."""
    seed, n = 1234, 64
    full = gm.spawn_draws(seed, np.arange(2 * n), np.full(2 * n, 3), 20)
    second = gm.spawn_draws(seed, n + np.arange(n), np.full(n, 3), 20)
    for a, b in zip(full, second):
        np.testing.assert_array_equal(a[n:], b)
    idx, x, y, rot = gm.spawn_draws(seed, np.arange(4096), np.ones(4096), 20)
    assert idx.min() == 0 and idx.max() == 19
    assert np.abs(x).max() <= 10e-3 + 1e-12 and set(np.round(x * 1e3).astype(int)) <= set(range(-10, 11))
    deg = np.round(np.rad2deg(rot)).astype(int)
    assert set(np.unique(deg)) <= set(d + o for d in range(-5, 6) for o in (0, 60, 120))


def test_canonical_model_dimensions(model):
    """nq=39, nv=38, nbody=34, nM=219, 4 motor locks."""
    assert (model.nq, model.nv, model.nbody) == (39, 38, 34)
    assert model.nM == 219 and model.nlock == 4
    assert model.npair <= 64
    assert model.n_seg == 8


def test_canonical_configuration(gm, model):
    """baseline_06-09-24 yaml: 4 continuous actions, 9 sensor streams x 7 = 63 obs,
    time_for_action 0.2 s at dt 3.187e-3 -> S = 63 substeps."""
    cfg = gm.ConfigBlob(gm.canonical_settings(seed=1), model)
    assert cfg.n_actions == 4
    assert cfg.n_obs == 63
    assert cfg.sim_steps_per_action == 63
    assert cfg.sensor_fcn == 2 and cfg.state_fcn == 4     # average / sign samplers


def test_configure_derives_substeps(gm, model):
    s = gm.canonical_settings(seed=1)
    s.time_for_action = 0.25
    cfg = gm.ConfigBlob(s, model)
    assert cfg.sim_steps_per_action == int(np.ceil(0.25 / 3.187e-3))


def test_configure_rejects_windows_beyond_ring(gm, model):
    """Sensor windows hold the last GM_RING=64 readings (the reference keeps 1000 but the
    observation reads at most 1 + readings_per_step * prev_steps); longer histories than
    the canonical 3 steps run, larger requests are rejected loudly, never truncated."""
    s = gm.canonical_settings(seed=1)
    s.time_for_action = 0.5       # 5 readings per step x 3 prev steps + 1 = 16 <= 64
    gm.ConfigBlob(s, model)
    s = gm.canonical_settings(seed=1)
    s.sensor_n_prev_steps = s.state_n_prev_steps = 10
    cfg = gm.ConfigBlob(s, model)
    assert cfg.n_obs > gm.ConfigBlob(gm.canonical_settings(seed=1), model).n_obs
    s.sensor_n_prev_steps = 40    # 2 readings per step x 40 + 1 = 81 > 64
    with pytest.raises(RuntimeError):
        gm.ConfigBlob(s, model)


def test_state_sample_mode_quirk(gm, model):
    """mjclass.cpp:204-206: state_sample_mode=6 overwrites the *sensor* sampler."""
    s = gm.canonical_settings(seed=1)
    s.state_sample_mode = 6
    cfg = gm.ConfigBlob(s, model)
    assert cfg.sensor_fcn == 6


def test_object_sets(gm):
    for name, n in (("cylinder", 1), ("set1_synthetic", 3), ("set6_synthetic", 20)):
        objs = gm.make_object_set(name, 1234)
        assert len(objs) == n
        for o in objs:
            assert o.type in (2, 5, 6) and o.mass > 0
            assert 0 < o.size[0] < 0.1


def test_unknown_object_set_raises(gm):
    with pytest.raises(Exception):
        gm.make_object_set("set_that_does_not_exist", 1)


def test_create_without_gpu_fails_loudly(gm, model):
    """No CPU fallback: creating a context on a machine without the GPU is an error."""
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("a GPU is present")
    with pytest.raises(RuntimeError):
        gm.BatchedGripperEnv(2, object_set="cylinder")
